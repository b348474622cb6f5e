#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean over dispatches)."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "kan::" not in name:
            continue
        short = name.split("(")[0].replace("void kan::", "")
        agg[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        line = f"{os.path.relpath(path, root)}  {k}: " + " ".join(f"{c}={v:.4g}" for c, v in sorted(m.items()))
        if "SQ_ACTIVE_INST_VALU" in m and "GRBM_GUI_ACTIVE" in m:
            simd = 1024
            busy = m["SQ_ACTIVE_INST_VALU"] * 4 / simd / (m["GRBM_GUI_ACTIVE"] / 8)
            line += f"  | VALU busy {busy:.2f}"
        print(line)
