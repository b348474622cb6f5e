#!/usr/bin/env python3
"""bench.py's adaptive reference-problem epoch (FK256, T = 5, saveat 0.5, default tolerances) for
rocprofv3 traces:  python3 tools/prof_epoch_adaptive.py [--batch 4096] [--reps 1] [--nx 256]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import kanode  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--reps", type=int, default=1)
ap.add_argument("--nx", type=int, default=256)
a = ap.parse_args()
p_np = bench.fk_trained_like_params()
out = bench.epoch_adaptive_bench(torch.device("cuda:0"), p_np, a.nx, 1 / (a.nx - 1), 0.01, a.batch, 0, reps=a.reps)
print(out, flush=True)
