#!/usr/bin/env python3
"""Per-kernel statistics of a rocprofv3 kernel trace split by grid size (one row per kernel name and
Grid_Size), so a kernel launched at several batch sizes in one run is not averaged across them:

    python3 tools/kstats_by_grid.py RUN_kernel_trace.csv [--grep SUBSTR] [--csv OUT.csv]

Columns: calls, average / min / max / median duration (µs) and total (ms) of the dispatches with that
grid size."""
import argparse
import collections
import csv
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--grep", default="")
ap.add_argument("--csv", default="")
a = ap.parse_args()
rows = collections.defaultdict(list)
for r in csv.DictReader(open(a.trace)):
    name = r["Kernel_Name"]
    if a.grep and a.grep not in name:
        continue
    short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("kan::", "")
    grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
    wg = int(r.get("Workgroup_Size") or r.get("Workgroup_Size_X") or 0)
    rows[(short, grid, wg)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = []
for (k, g, w), d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
    out.append(dict(kernel=k, grid_size=g, workgroup_size=w, calls=len(d), avg_us=sum(d) / len(d), min_us=min(d),
                    max_us=max(d), median_us=statistics.median(d), total_ms=sum(d) / 1e3))
for o in out:
    print(f"{o['kernel'][:78]:78s} grid={o['grid_size']:>10d} wg={o['workgroup_size']:>5d} calls={o['calls']:6d} "
          f"avg={o['avg_us']:9.2f}us med={o['median_us']:9.2f} min={o['min_us']:9.2f} max={o['max_us']:9.2f} "
          f"tot={o['total_ms']:9.3f}ms")
if a.csv:
    with open(a.csv, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(out[0].keys()) if out else ["kernel"])
        w.writeheader()
        w.writerows(out)
