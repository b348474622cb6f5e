#!/usr/bin/env python3
"""Eager RHS / VJP calls of the surrogate chains for rocprofv3 --kernel-trace (per-kernel times).

    rocprofv3 --kernel-trace --stats -d gpurun_out/sprof -o run -- python3 tools/prof_surrogate.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kan-odes_amd"))
import kanode  # noqa: E402

dev = torch.device("cuda:0")
for name, N, G, B in (("burgers512", 512, 5, 1), ("schrodinger1024", 2048, 10, 1)):
    chain = kanode.Chain(kanode.KDense(N, 10, G, normalizer="softsign"), kanode.KDense(10, N, G, normalizer="softsign"))
    rhs = kanode.ChainRHS(chain, device=dev)
    p = torch.as_tensor(chain.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
    u = torch.rand(B, N, dtype=torch.float64, device=dev)
    lam = torch.randn_like(u)
    du, dp = torch.empty_like(u), torch.zeros_like(p)
    rhs.hd.reserve(B)
    for _ in range(int(os.environ.get("REPS", "30"))):
        rhs.hd.rhs(p, u, du)
        torch.cuda.synchronize()
        rhs.hd.vjp(p, u, lam, dp=dp)
        torch.cuda.synchronize()
print("done")
