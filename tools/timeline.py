"""Per-step timeline from a rocprofv3 kernel_trace.csv of bench.py (graph replays).

Splits the trace at the untouched-Adam launches; for each step prints the main-queue busy
time, gaps, the Adam span and the kernels in order (with --verbose)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
verbose = "--verbose" in sys.argv
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows))
starts = [i for i, e in enumerate(ev) if "claim_rows" in e[2]]
# use the timed replay steps: skip the first few
for si in range(len(starts) - 1)[-14:-11]:
    lo = starts[si]
    hi = min(i for i in range(lo, len(ev)) if "step_end" in ev[i][2])
    ks = ev[lo:hi + 1]
    ad = [k for k in ks if "adam_table_untouched" in k[2]]
    a = ad[0] if ad else (ks[0][0], ks[0][0])
    t0 = ks[0][0]
    t1 = ks[-1][1]
    main = [k for k in ks if "adam_table_untouched" not in k[2]]
    busy = sum(k[1] - k[0] for k in main)
    gaps = 0
    last = main[0][1]
    for k in main[1:]:
        if k[0] > last:
            gaps += k[0] - last
        last = max(last, k[1])
    print(f"step span {(t1 - t0) / 1e3:8.1f} us | main busy {busy / 1e3:7.1f} gaps {gaps / 1e3:6.1f} | "
          f"adam {(a[1] - a[0]) / 1e3:6.1f} us starts at +{(a[0] - t0) / 1e3:6.1f} ends at +{(a[1] - t0) / 1e3:6.1f} | "
          f"kernels {len(main)} queues {sorted(set(k[3] for k in ks))}")
    if verbose:
        for k in ks:
            print(f"   +{(k[0] - t0) / 1e3:8.1f} {(k[1] - k[0]) / 1e3:7.1f}  q{k[3]}  {k[2][:90]}")
