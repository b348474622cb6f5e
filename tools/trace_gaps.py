#!/usr/bin/env python3
"""GPU idle gaps in a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv): the last contiguous segment
(split at gaps > --split ms), busy vs span, and the gaps grouped by the (previous -> next) kernel pair.
    python3 tools/trace_gaps.py <dir with *kernel_trace.csv> [--split 2]"""
import argparse
import csv
import glob
import os
from collections import defaultdict

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--split", type=float, default=2.0)
ap.add_argument("--top", type=int, default=8)
a = ap.parse_args()
rows = []
for path in glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-48:]))
rows.sort()
st = np.array([r[0] for r in rows], dtype=np.int64)
en = np.array([r[1] for r in rows], dtype=np.int64)
gaps = st[1:] - en[:-1]
big = np.where(gaps > a.split * 1e6)[0]
s0 = int(big[-1]) + 1 if len(big) else 0
s, e = st[s0:], en[s0:]
names = [r[2] for r in rows[s0:]]
g = s[1:] - e[:-1]
print(f"segment: {len(s)} kernels, span {(e.max() - s.min()) / 1e6:.3f} ms, busy {(e - s).sum() / 1e6:.3f} ms, "
      f"idle {np.clip(g, 0, None).sum() / 1e6:.3f} ms; gap percentiles (us) 50/90/99: "
      f"{np.percentile(g, 50) / 1e3:.2f} {np.percentile(g, 90) / 1e3:.2f} {np.percentile(g, 99) / 1e3:.2f}")
d = defaultdict(list)
for i in range(len(g)):
    d[(names[i], names[i + 1])].append(g[i])
for (p, n), v in sorted(d.items(), key=lambda kv: -np.sum(kv[1]))[:a.top]:
    v = np.array(v)
    print(f"  {p:>48s} -> {n:<48s} n={len(v):6d} total {v.sum() / 1e6:8.3f} ms  median {np.median(v) / 1e3:6.2f} us")
