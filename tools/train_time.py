#!/usr/bin/env python3
"""Training-leg times for interleaved separate-process library A/B (KANODE_LIB): the adaptive FK256
reference-problem epoch (bench.epoch_adaptive_bench) and the surrogate training iterations
(bench.surrogate_bench).   python3 tools/train_time.py TAG [--batch 4096]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("tag")
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--no-epoch", action="store_true")
ap.add_argument("--no-surrogates", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")
if not a.no_epoch:
    import numpy as np
    import kanode
    p_np = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign")).setup(np.random.default_rng(0))[0].astype(np.float64)
    f = bench.epoch_bench(dev, p_np, 256, 1 / 255, 0.01, a.batch, 0, 50, 1e-3, 5)
    print(f"{a.tag:10s} epoch_fixed    {f['gpu'] * 1e3:8.3f} ms", flush=True)
    e = bench.epoch_adaptive_bench(dev, bench.fk_trained_like_params(), 256, 1 / 255, 0.01, a.batch, 0, reps=2)
    print(f"{a.tag:10s} epoch_adaptive {e['gpu'] * 1e3:8.2f} ms  steps {e['forward_steps']}/{e['adjoint_steps']}", flush=True)
s = {} if a.no_surrogates else bench.surrogate_bench(dev, False, reps=3)
for k, v in s.items():
    print(f"{a.tag:10s} {k:16s} train {v['train_iteration_ms']:7.2f} ms  rhs {v['rhs_us']:6.2f} us  vjp {v['vjp_us']:6.2f} us",
          flush=True)
