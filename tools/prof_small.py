#!/usr/bin/env python3
"""The reference-size training iterations of bench.py (lv1_train: LV_driver_KANODE.jl one trajectory;
fk26_train: Fisher-KPP_Source.jl 26 points), GPU only, for rocprofv3 traces and A/B timing:
    python3 tools/prof_small.py [--reps 20] [--which lv1,fk26]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--which", default="lv1,fk26")
a = ap.parse_args()
dev = torch.device("cuda:0")
out = {}
if "lv1" in a.which:
    out["lv1_train"] = bench.lv1_train_bench(dev, False, reps=a.reps)
if "fk26" in a.which:
    out["fk26_train"] = bench.fk26_train_bench(dev, False, reps=a.reps)
print(json.dumps(out), flush=True)
