"""Per-step timeline of bench.py's graph replays from a rocprofv3 kernel_trace.csv (lazy table Adam).

  python tools/step_timeline.py run_kernel_trace.csv [--steps N] [--verbose]

Steps are split at claim_rows_kernel (or, fused, the claimed-row adam_catchup).  The rolling-window Adam replay (adam_catchup on 256
workgroups) and the next-batch prefetch (adam_prefetch) run on the side stream ("window" below:
their span); every other kernel is on the main stream.  Prints, per step,
the span, the main stream's busy time and idle gaps, the window's span, and (--verbose) the
kernels in order with their durations and how much of each overlapped the window.
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 3
    verbose = "--verbose" in sys.argv
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                 int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)) for r in rows)
    starts = [i for i, e in enumerate(ev) if "claim_rows" in e[2] or "adam_claim2" in e[2]]
    if not starts:
        # fused claim + catch-up (lazy single GPU): steps start at the claimed-row catch-up, the
        # adam_catchup launch with the largest grid
        gmax = max((e[3] for e in ev if "adam_catchup" in e[2]), default=0)
        starts = [i for i, e in enumerate(ev) if "adam_catchup" in e[2] and e[3] == gmax]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else "gemm_dma16"
    # steps of the run being studied (bench.py also times an fp32 run: its GEMMs are gemm_kernel)
    starts = [s for j, s in enumerate(starts[:-1]) if any(match in e[2] for e in ev[s:starts[j + 1]])] + starts[-1:]

    def is_window(k, ks):
        # side stream: the rolling-window replay (the adam_catchup launch of the step with the
        # smaller grid) and the next batch's ahead-of-time catch-up (adam_prefetch)
        if any(s in k[2] for s in ("adam_prefetch", "adam_pretag", "adam_window2",
                                   "sparse_fixup_dup")):
            return True
        cs = [c[3] for c in ks if "adam_catchup" in c[2]]
        return "adam_catchup" in k[2] and len(cs) > 1 and k[3] == min(cs)
    agg = defaultdict(list)
    # graph replays are the steps with the fewest host gaps: take the nsteps with the smallest gap sum
    def gap_of(si):
        ks0 = ev[starts[si]:starts[si + 1]]
        ks = [k for k in ks0 if not is_window(k, ks0)]
        g, last = 0, ks[0][1]
        for k in ks[1:]:
            g += max(0, k[0] - last)
            last = max(last, k[1])
        return g
    picked = sorted(sorted(range(len(starts) - 1), key=gap_of)[:nsteps])
    for si in picked:
        ks = ev[starts[si]:starts[si + 1]]
        win = [k for k in ks if is_window(k, ks)]
        main_k = [k for k in ks if k not in win]
        t0, t1 = ks[0][0], max(k[1] for k in ks)
        busy = sum(k[1] - k[0] for k in main_k)
        gaps, last = 0, main_k[0][1]
        for k in main_k[1:]:
            gaps += max(0, k[0] - last)
            last = max(last, k[1])
        w = (min(k[0] for k in win), max(k[1] for k in win), "", 0) if win else (t0, t0, "", 0)
        print(f"step span {(t1 - t0) / 1e3:7.1f} us | main busy {busy / 1e3:6.1f} gaps {gaps / 1e3:5.1f} | window "
              f"{(w[1] - w[0]) / 1e3:6.1f} us [+{(w[0] - t0) / 1e3:.1f}, +{(w[1] - t0) / 1e3:.1f}]")
        for k in main_k:
            ov = max(0, min(k[1], w[1]) - max(k[0], w[0]))
            agg[(k[2][:60], k[3])].append(((k[1] - k[0]) / 1e3, ov / 1e3))
        if verbose and si == picked[-1]:
            for k in main_k:
                ov = max(0, min(k[1], w[1]) - max(k[0], w[0]))
                print(f"   +{(k[0] - t0) / 1e3:6.1f} {(k[1] - k[0]) / 1e3:6.1f} us  ov {ov / 1e3:5.1f}  {k[2][:70]} "
                      f"grid {k[3]}")
    print("\nper kernel (avg over steps): us, overlapped-with-window us")
    tot = 0.0
    for key, v in sorted(agg.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
        d = sum(x[0] for x in v) / len(picked)
        o = sum(x[1] for x in v) / len(picked)
        tot += d
        print(f"  {d:7.1f}  {o:6.1f}  x{len(v) // len(picked)}  {key[0]} grid {key[1]}")
    print(f"  total main {tot:.1f} us")


if __name__ == "__main__":
    main()
