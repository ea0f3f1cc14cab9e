"""Summarise rocprofv3 --pmc CSVs: per kernel name, counter sums over
dispatches (and dispatch count).  Usage: python scripts/pmc_summary.py DIR..."""
import csv
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((d, r["Dispatch_Id"]))
for k, c in tot.items():
    print(f"== {k}  dispatches={len(disp[k])}")
    for n, v in sorted(c.items()):
        print(f"   {n:28s} {v:.4g}")
