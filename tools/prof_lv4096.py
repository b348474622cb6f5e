#!/usr/bin/env python3
"""bench.py's lv4096_train leg (BASELINE configs[1] trained: 4096 ICs fp32, adaptive Tsit5 + InterpolatingAdjoint +
Adam) for rocprofv3 traces:  python3 tools/prof_lv4096.py [--reps 5]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
print(json.dumps(bench.lv4096_train_bench(torch.device("cuda:0"), False, reps=a.reps)), flush=True)
