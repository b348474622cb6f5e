#!/usr/bin/env python3
"""bench.py's Lotka-Volterra legs (configs[0], [1]) for library A/B runs (KANODE_LIB=...):
prints the LV 4096 fp32 device time per RHS and the single-trajectory training iteration."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kan-odes_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

dev = torch.device("cuda:0")
a = bench.lv4096_bench(dev)
b = bench.lv1_train_bench(dev, False, reps=20)
print(f"lv4096 us_per_rhs {a['us_per_rhs']:.3f}  lv1_train ms {b['gpu']:.3f}", flush=True)
