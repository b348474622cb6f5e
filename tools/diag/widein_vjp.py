"""Diagnostic: wide-in layer pullback pbar / xbar vs the oracle for several column counts."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "kan-odes_amd"), os.path.join(ROOT, "tests"), ROOT]
import kanode  # noqa: E402
from gpu_util import cfgs_from_specs, t  # noqa: E402
from oracle import oracle as O  # noqa: E402

for N, G in ((512, 5), (2048, 10)):
    specs = [O.LayerSpec(N, 10, G, "softsign")]
    hd = kanode.KanodeHandle(cfgs_from_specs(specs), dtype=torch.float64, rhs_kind="chain", device="cuda:0")
    rng = np.random.default_rng(1)
    p = rng.uniform(-0.1, 0.1, hd.P)
    for K in (1, 8, 9, 16, 64, 200):
        x = rng.uniform(-1, 1, (K, N))
        yb = rng.normal(size=(K, 10))
        xb, pb = hd.layer_vjp(0, t(p), t(x), t(yb))
        rx, rp = O.chain_vjp(specs, p, x, yb)
        ep = np.abs(pb.cpu().numpy() - rp)
        ex = np.abs(xb.cpu().numpy() - rx)
        P0 = 10 * G * N
        print(f"N {N} G {G} K {K}: xbar err {ex.max():.2e}  pbar C err {ep[:P0].max():.2e} (at {ep[:P0].argmax()})  "
              f"W err {ep[P0:].max():.2e}  |p| {np.abs(rp).max():.2e}", flush=True)
