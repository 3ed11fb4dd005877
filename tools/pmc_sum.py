"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv: python tools/pmc_sum.py FILE [substr]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"].split("(")[0][-40:]
    if sub in k:
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
for k, v in agg.items():
    n = len(disp[k])
    print(f"{k:42s} x{n:3d} " + " ".join(f"{c}={x / n:.4g}" for c, x in sorted(v.items())))
