#!/usr/bin/env python3
"""Device time of the surrogate pullback (standalone VJP and adjoint-stage VJP, hipGraph of back-to-back
calls) for BASELINE configs[3] (Burgers [512, 10, 512], 4 ICs) and [4] (Schrodinger [2048, 10, 2048],
8 ICs), with whatever libkanode.so KANODE_LIB names (tools/surr_ablate.sh runs it per variant)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import kanode  # noqa: E402
from bench import _graph_us, _surrogate_problem  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else os.path.basename(os.environ.get("KANODE_LIB", "base"))
dev = torch.device("cuda:0")
for name, N, G, B in (("burgers512", 512, 5, 4), ("schrodinger1024", 2048, 10, 8)):
    chain = kanode.Chain(kanode.KDense(N, 10, G, normalizer="softsign"), kanode.KDense(10, N, G, normalizer="softsign"))
    rhs = kanode.ChainRHS(chain, device=dev)
    p = torch.as_tensor(chain.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
    u = torch.as_tensor(_surrogate_problem(name, B, 5), device=dev)
    lam = torch.randn_like(u)
    dp = torch.zeros_like(p)
    du = torch.empty_like(u)
    rhs.hd.reserve(B)
    r = [_graph_us(lambda: rhs.hd.rhs(p, u, du)) for _ in range(3)]
    v = [_graph_us(lambda: rhs.hd.vjp(p, u, lam, dp=dp)) for _ in range(3)]
    print(f"{tag:12s} {name:16s} rhs {np.median(r):7.2f} us  vjp {np.median(v):7.2f} us", flush=True)
