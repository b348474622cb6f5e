#!/usr/bin/env python3
"""Interleaved A/B of the surrogate pullback: two launches (KANODE_OPT_PAIR_VJP = 1) vs four (0), per
VJP (hipGraph of back-to-back calls) and per training iteration (adaptive Tsit5 + InterpolatingAdjoint
+ Adam), BASELINE configs[3] (Burgers [512, 10, 512], 4 ICs) and [4] (Schrodinger [2048, 10, 2048], 8 ICs)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import kanode  # noqa: E402
from bench import _graph_us, _surrogate_problem  # noqa: E402

dev = torch.device("cuda:0")
cases = (("burgers512", 512, 5, 4, (0.0, 1.0), [0.005 * i for i in range(201)], 1e-2),
         ("schrodinger1024", 2048, 10, 8, (0.0, np.pi / 2), [0.1 + 0.2 * i for i in range(8)], 1e-3))
for name, N, G, B, tspan, saveat, eta in cases:
    chain = kanode.Chain(kanode.KDense(N, 10, G, normalizer="softsign"), kanode.KDense(10, N, G, normalizer="softsign"))
    rhs = kanode.ChainRHS(chain, device=dev)
    p = torch.as_tensor(chain.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
    u = torch.as_tensor(_surrogate_problem(name, B, 5), device=dev)
    lam = torch.randn_like(u)
    lamJ, dp = torch.empty_like(u), torch.zeros_like(p)
    rhs.hd.reserve(B)
    target = (0.9 * u).unsqueeze(0).expand(len(saveat), -1, -1).contiguous()
    res = {0: [], 1: []}
    for rnd in range(3):
        for pair in (1, 0):
            rhs.hd.set_option("pair_vjp", pair)
            v = _graph_us(lambda: rhs.hd.vjp(p, u, lam, dp=dp))
            tr = kanode.Trainer(rhs, u, tspan, saveat, target, p, eta=eta)
            tr.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(2):
                tr.step()
            torch.cuda.synchronize()
            it = (time.perf_counter() - t0) / 2 * 1e3
            res[pair].append((v, it))
            print(f"{name} round {rnd} pair_vjp={pair}: vjp {v:.1f} us, train iteration {it:.2f} ms", flush=True)
    for pair in (1, 0):
        a = np.array(res[pair])
        print(f"{name} pair_vjp={pair}: vjp median {np.median(a[:, 0]):.1f} us, iteration median {np.median(a[:, 1]):.2f} ms")
