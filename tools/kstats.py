#!/usr/bin/env python3
"""Print rocprofv3 --stats kernel rows (name prefix, calls, average and total µs) of one or more
*_kernel_stats.csv files:  python tools/kstats.py DIR_OR_CSV... [--grep SUBSTR] [--top N]"""
import argparse
import csv
import glob
import os

ap = argparse.ArgumentParser()
ap.add_argument("paths", nargs="+")
ap.add_argument("--grep", default="")
ap.add_argument("--top", type=int, default=12)
a = ap.parse_args()
for p in a.paths:
    files = sorted(glob.glob(os.path.join(p, "*kernel_stats.csv"))) if os.path.isdir(p) else [p]
    for f in files:
        rows = list(csv.DictReader(open(f)))
        rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        print(f"{f}  (all kernels {tot / 1e6:.2f} ms)")
        n = 0
        for r in rows:
            if a.grep and a.grep not in r["Name"]:
                continue
            name = r["Name"].replace("void ", "").replace("kan::", "")[:70]
            print(f"  {name:70s} calls={int(r['Calls']):6d} avg={float(r['AverageNs']) / 1e3:8.2f}us "
                  f"tot={float(r['TotalDurationNs']) / 1e6:8.2f}ms {float(r['Percentage']):5.1f}%")
            n += 1
            if n >= a.top:
                break
