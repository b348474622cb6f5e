#!/usr/bin/env python3
"""Training iterations of bench.py's surrogate legs (BASELINE configs[3], [4]) for rocprofv3 kernel
traces:  python3 tools/prof_surrogate_train.py --case burgers512 --reps 2"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kan-odes_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="burgers512")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    t0 = time.perf_counter()
    out = bench.surrogate_bench(dev, False, only=a.case, reps=a.reps)
    print(out, f"{time.perf_counter() - t0:.2f} s")


if __name__ == "__main__":
    main()
