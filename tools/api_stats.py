#!/usr/bin/env python3
"""Host API time per call site from a rocprofv3 --hip-runtime-trace (--kernel-trace) directory: count and total
duration of every HIP runtime function, optionally divided by an iteration count, and the kernel busy time.
    python3 tools/api_stats.py TRACE_DIR [--per N] [--top 20]"""
import argparse
import collections
import csv
import glob
import os

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--per", type=float, default=1.0)
ap.add_argument("--top", type=int, default=20)
ap.add_argument("--window", default="", help="kernel-name substring: count only API calls between the start of its "
                "--skip-th launch and the end of its last launch (the timed iterations)")
ap.add_argument("--skip", type=int, default=1)
a = ap.parse_args()
lo, hi = None, None
if a.window:
    ks = []
    for path in glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if a.window in r["Kernel_Name"]:
                ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    ks.sort()
    lo, hi = ks[a.skip][0], ks[-1][1]
tot, cnt = collections.Counter(), collections.Counter()
span = [None, None]
for path in glob.glob(os.path.join(a.root, "**", "*hip_api_trace.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if lo is not None and not (lo <= s <= hi):
            continue
        tot[r["Function"]] += e - s
        cnt[r["Function"]] += 1
        span[0] = s if span[0] is None else min(span[0], s)
        span[1] = e if span[1] is None else max(span[1], e)
busy = 0
for path in glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        s = int(r["Start_Timestamp"])
        if lo is not None and not (lo <= s <= hi):
            continue
        busy += int(r["End_Timestamp"]) - s
print(f"api span {(span[1] - span[0]) / 1e6 if span[0] else 0:.2f} ms, kernel busy {busy / 1e6:.2f} ms "
      f"(per {a.per:g}: {busy / 1e3 / a.per:.1f} us)")
for f, t in tot.most_common(a.top):
    print(f"  {f:40s} calls={cnt[f] / a.per:8.1f}/it  total={t / 1e3 / a.per:9.1f} us/it  avg={t / cnt[f] / 1e3:7.2f} us")
