#!/usr/bin/env python3
"""GPU idle time in a rocprofv3 rocpd trace: kernels of the last contiguous segment (split at gaps
> --split ms), busy vs span, and the idle gaps grouped by the kernel that follows them.
    python3 tools/rocpd_gaps.py <run_results.db> [--split 2]"""
import argparse
import sqlite3
from collections import defaultdict

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--split", type=float, default=2.0)
    ap.add_argument("--top", type=int, default=10)
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute("select start, end, name from kernels order by start").fetchall()
    st = np.array([r[0] for r in rows], dtype=np.int64)
    en = np.array([r[1] for r in rows], dtype=np.int64)
    gaps = st[1:] - en[:-1]
    big = np.where(gaps > a.split * 1e6)[0]
    s0 = int(big[-1]) + 1 if len(big) else 0
    s, e = st[s0:], en[s0:]
    g = s[1:] - e[:-1]
    print(f"segment: {len(s)} kernels, span {(e.max() - s.min()) / 1e6:.3f} ms, busy {(e - s).sum() / 1e6:.3f} ms, "
          f"idle {g.sum() / 1e6:.3f} ms; gap percentiles (us) 50/90/99: "
          f"{np.percentile(g, 50) / 1e3:.2f} {np.percentile(g, 90) / 1e3:.2f} {np.percentile(g, 99) / 1e3:.2f}")
    d = defaultdict(list)
    for i in range(len(g)):
        d[rows[s0 + i + 1][2][:90]].append(g[i])
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
        print(f"{sum(v) / 1e6:9.3f} ms idle  {len(v):7d} x  median {np.median(v) / 1e3:7.2f} us  before {k}")
    busy = defaultdict(float)
    cnt = defaultdict(int)
    for i in range(s0, len(rows)):
        busy[rows[i][2][:90]] += (rows[i][1] - rows[i][0])
        cnt[rows[i][2][:90]] += 1
    for k, v in sorted(busy.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"{v / 1e6:9.3f} ms busy  {cnt[k]:7d} x  avg {v / cnt[k] / 1e3:7.2f} us  {k}")


if __name__ == "__main__":
    main()
