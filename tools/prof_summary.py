"""Summarise a rocprofv3 kernel_stats.csv: per-kernel calls, average and share of total."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    per = f" per-step={float(r['TotalDurationNs']) / steps / 1e3:7.1f}us" if steps else ""
    print(f"{r['Name'][:80]:80s} n={r['Calls']:>5s} avg={float(r['AverageNs']) / 1e3:7.1f}us "
          f"{100 * float(r['TotalDurationNs']) / tot:5.1f}%{per}")
print(f"total kernel time {tot / 1e6:.2f} ms" + (f" = {tot / steps / 1e3:.1f} us/step" if steps else ""))
