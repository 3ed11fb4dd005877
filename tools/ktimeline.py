#!/usr/bin/env python3
"""One FET scan's kernel timeline from a rocprofv3 --kernel-trace CSV: start/end (us from
the scan's first kernel), queue and grid per kernel.  usage: ktimeline.py TRACE.csv [scan#]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
first = ("k_fet_setup", "k_popsize")
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(first)]
i0, i1 = idx[k], idx[k + 1] if k + 1 < len(idx) else len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
print(f"{'kernel':30s} {'queue':>5s} {'start':>8s} {'end':>8s} {'us':>7s} {'grid':>8s} {'lds':>6s}")
for r in rows[i0:i1]:
    if "rocclr" in r["Kernel_Name"]:
        continue
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // int(r["Workgroup_Size_X"])
    print(f"{r['Kernel_Name'].split('(')[0][:30]:30s} {r['Queue_Id']:>5s} {s:8.1f} {e:8.1f} {e - s:7.1f} {g:8d} {r['LDS_Block_Size']:>6s}")
