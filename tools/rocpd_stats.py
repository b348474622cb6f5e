#!/usr/bin/env python3
"""Kernel statistics (name, calls, total/avg/min/max ns, share) from a rocprofv3 rocpd SQLite database
(ROCm 7 default output), in the layout of rocprofv3's kernel_stats.csv:
    python3 tools/rocpd_stats.py <run_results.db> [--csv out.csv] [--top N]"""
import argparse
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                     "max(end - start) from kernels group by name order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [(n, k, s, a, 100.0 * s / tot, mn, mx) for n, k, s, a, mn, mx in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    st = stats(a.db)
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            w.writerows(st)
    for n, k, s, av, pc, mn, mx in st[:a.top]:
        print(f"{k:8d} {s / 1e6:10.3f} ms {av / 1e3:9.2f} us {pc:6.2f}%  {n[:150]}")
    sys.stdout.flush()


if __name__ == "__main__":
    main()
