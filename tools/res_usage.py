#!/usr/bin/env python3
"""Tabulate the kernels' resource usage from the build's remark files (kan-odes_amd/build/*.remarks,
written by the Makefile with -Rpass-analysis=kernel-resource-usage):
    python tools/res_usage.py [--grep SUBSTR] [files...]"""
import argparse
import glob
import os
import re
import subprocess

ap = argparse.ArgumentParser()
ap.add_argument("files", nargs="*")
ap.add_argument("--grep", default="")
a = ap.parse_args()
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
files = a.files or sorted(glob.glob(os.path.join(root, "kan-odes_amd/build/*.remarks")))
for f in files:
    cur = None
    rows = []
    for ln in open(f):
        m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", ln)
        if not m:
            continue
        t = m.group(1)
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    names = [r["name"] for r in rows]
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    for r, d in zip(rows, dem):
        if a.grep and a.grep not in d:
            continue
        d = d.replace("(anonymous namespace)::", "").replace("kan::", "").replace("void ", "")
        d = re.sub(r"\(.*", "", d)
        print(f"{d[:72]:72s} vgpr={r.get('VGPRs', '?'):>4s} agpr={r.get('AGPRs', '?'):>3s} "
              f"scratch={r.get('ScratchSize [bytes/lane]', '?'):>4s} occ={r.get('Occupancy [waves/SIMD]', '?'):>2s} "
              f"lds={r.get('LDS Size [bytes/block]', '?'):>6s}")
