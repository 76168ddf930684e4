"""Per-step kernel breakdown of a rocprofv3 kernel trace (any bench run): steps are split at the step
tail (adam_tail_kernel, one per step); the last --steps steps are averaged.

  python tools/shard_breakdown.py run_kernel_trace.csv [--steps 16]

Prints each kernel name's time per step (sum of its launches' durations), its queue, and per queue
the busy time per step, then the step span (tail to tail).
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    k = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 16
    rows = list(csv.DictReader(open(path)))
    qkey = "Queue_Id" if rows and "Queue_Id" in rows[0] else ("Stream_Id" if rows and "Stream_Id" in rows[0] else None)
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get(qkey, "?") if qkey else "?")
                for r in rows)
    tails = [i for i, e in enumerate(ev) if "adam_tail_kernel" in e[2]]
    if len(tails) < k + 1:
        k = len(tails) - 1
    a, b = tails[-k - 1], tails[-1]
    span = (ev[b][1] - ev[a][1]) / k / 1e3
    per = defaultdict(float)
    cnt = defaultdict(int)
    q = {}
    busy = defaultdict(float)
    for s, e, name, qq in ev[a + 1:b + 1]:
        short = name.split("(")[0][:90]
        per[short] += (e - s) / 1e3
        cnt[short] += 1
        q[short] = qq
        busy[qq] += (e - s) / 1e3
    print(f"{k} steps, span {span:.1f} us/step (tail to tail)")
    for name, t in sorted(per.items(), key=lambda x: -x[1]):
        print(f"{t / k:8.1f} us  x{cnt[name] / k:4.1f}  q{q[name]:>3}  {name}")
    for qq, t in sorted(busy.items()):
        print(f"queue {qq}: busy {t / k:.1f} us/step")


if __name__ == "__main__":
    main()
