#!/usr/bin/env python3
"""Effective shader clock per kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE pass with --kernel-trace
(MI355X_MICROARCH.md, DVFS give-back: clock ≈ GRBM_GUI_ACTIVE ÷ 8 XCDs ÷ kernel wall time; reads high on
dispatches shorter than ~0.3 ms):

    python3 tools/clock.py PASS_DIR [--grep SUBSTR]

PASS_DIR holds the pass's *counter_collection.csv and *kernel_trace.csv (joined on Dispatch_Id / Correlation_Id).
Prints per kernel: dispatches, median duration, median and interquartile clock in GHz."""
import argparse
import collections
import csv
import glob
import os
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--grep", default="")
a = ap.parse_args()
cc = sorted(glob.glob(os.path.join(a.root, "**", "*counter_collection.csv"), recursive=True))
kt = sorted(glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True))
if not cc:
    raise SystemExit(f"no counter_collection.csv under {a.root}")
dur = {}
for path in kt:
    for r in csv.DictReader(open(path)):
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
per = collections.defaultdict(list)
for path in cc:
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        name = r["Kernel_Name"]
        if a.grep and a.grep not in name:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        ns = None
        if "End_Timestamp" in r and r.get("End_Timestamp"):
            ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        elif key in dur:
            ns = dur[key]
        if not ns:
            continue
        short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("kan::", "")
        per[short].append((ns, float(r["Counter_Value"]) / 8.0 / ns))
for k, v in sorted(per.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
    ghz = sorted(x[1] for x in v)
    q = statistics.quantiles(ghz, n=4) if len(ghz) >= 4 else [ghz[0], statistics.median(ghz), ghz[-1]]
    print(f"{k[:80]:80s} n={len(v):6d} dur_med={statistics.median(x[0] for x in v) / 1e3:9.2f}us "
          f"clock_med={statistics.median(ghz):.3f}GHz iqr=[{q[0]:.3f},{q[2]:.3f}]")
