#!/usr/bin/env python3
"""Run some of bench.py's training legs (GPU side only) and print their ms per iteration:
    python3 tools/legs.py lv4096_train lv1_train fk26_train [--reps N]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("legs", nargs="+")
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda:0")
out = {}
for leg in a.legs:
    out[leg] = round(getattr(bench, leg + "_bench")(dev, False, reps=a.reps)["gpu"], 4)
print(json.dumps(out), flush=True)
