"""Average PMC counter values per kernel from rocprofv3 counter_collection CSVs.
  python tools/pmc_summary.py DIR [DIR ...] [--filter substr]"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
flt = None
if "--filter" in sys.argv:
    flt = sys.argv[sys.argv.index("--filter") + 1]
    args = [a for a in args if a != flt]
acc = defaultdict(lambda: defaultdict(list))
for d in args:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        name = r["Kernel_Name"]
        if flt and flt not in name:
            continue
        acc[name[:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} avg {sum(v) / len(v):16.1f}  (n={len(v)})")
