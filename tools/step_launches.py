"""Every launch of one timed step from a rocprofv3 kernel trace, in start order: start offset (us,
from the previous step's adam_tail end), duration, idle time on its queue before it, queue, grid.
Shows per LAUNCH what the per-kernel-name averages of the stats CSV mix together (e.g. the three
gemm_dma16_kernel<64,128,...> launches of a step, or a launch slowed by side-stream work beside it).
    python tools/step_launches.py <run_kernel_trace.csv> [k]   (k: index among the fast steps, default -6)
"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    tails = [i for i, r in enumerate(rows) if "adam_tail" in r["Kernel_Name"]]
    end = lambda i: int(rows[i]["End_Timestamp"])
    spans = [(end(tails[j + 1]) - end(tails[j])) / 1e3 for j in range(len(tails) - 1)]
    fast = [j for j, s in enumerate(spans) if s < 800]          # timed steps (probe steps sleep first)
    j = fast[int(sys.argv[2]) if len(sys.argv) > 2 else -6]
    print(f"{len(tails)} steps in the trace; this step spans {spans[j]:.1f} us")
    print(f"{'start':>8} {'dur':>7} {'idle':>6}  queue {'grid':>8}  kernel")
    t0 = end(tails[j])
    last = {}
    for r in rows[tails[j] + 1:tails[j + 1] + 1]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        q = r["Queue_Id"][-3:]
        print(f"{s:8.1f} {d:7.1f} {s - last.get(q, 0.0):6.1f}  q{q:>4} {r['Grid_Size_X']:>8}  {r['Kernel_Name'][:70]}")
        last[q] = s + d


if __name__ == "__main__":
    main()
