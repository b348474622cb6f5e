#!/usr/bin/env python3
"""Count the host-blocking HIP calls of a rocprofv3 --hip-runtime-trace --memory-copy-trace CSV run
inside the driver's timed window (tools/tp_sync_trace.py writes it, CLOCK_MONOTONIC ns; when the
trace's clock does not bracket it the whole trace is counted and the report says so), and divide by
the solver steps of that window.
  python3 tools/hip_sync_count.py TRACE_DIR STATS_JSON"""
import collections
import csv
import glob
import json
import os
import sys

root, stats_path = sys.argv[1], sys.argv[2]
st = json.load(open(stats_path))
lo, hi = st["window_monotonic_ns"]
BLOCKING = ("hipStreamSynchronize", "hipDeviceSynchronize", "hipEventSynchronize", "hipMemcpy",
            "hipMemcpyWithStream", "hipMemcpyDtoH", "hipMemcpyHtoD", "hipMemcpy2D", "hipStreamQuery",
            "hipEventQuery")


def rows(pattern):
    for path in glob.glob(os.path.join(root, "**", pattern), recursive=True):
        yield from csv.DictReader(open(path))


api = list(rows("*hip_api_trace.csv"))
cps = list(rows("*memory_copy_trace.csv"))
inside = [r for r in api if lo <= int(r["Start_Timestamp"]) <= hi]
windowed = len(inside) > 0
if not windowed:
    inside = api
calls = collections.Counter(r["Function"] for r in inside)
cp_in = [r for r in cps if not windowed or lo <= int(r["Start_Timestamp"]) <= hi]
dirs = collections.Counter(r.get("Direction", "?") for r in cp_in)
steps = st["forward_steps"] + st["adjoint_steps"]
blocking = {k: v for k, v in calls.items() if k in BLOCKING}
d2h = sum(v for k, v in dirs.items() if "DEVICE_TO_HOST" in k)
out = dict(window="driver's timed window" if windowed else "whole trace (clock did not bracket the window)",
           iters=st["iters"], forward_steps=st["forward_steps"], adjoint_steps=st["adjoint_steps"],
           blocking_calls=blocking, blocking_total=sum(blocking.values()), device_to_host_copies=d2h,
           copies_by_direction=dict(dirs), d2h_per_solver_step=d2h / max(steps, 1),
           blocking_per_solver_step=sum(blocking.values()) / max(steps, 1),
           top_api=dict(calls.most_common(12)))
print(json.dumps(out, indent=1))
