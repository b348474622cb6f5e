"""Diagnostic: several rows per wave (one-block grids) vs default grids, fused vs per-stage, fixed and
adaptive steps: max |Δu|, |Δdp|, |Δdu0| and step counts."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "kan-odes_amd"), os.path.join(ROOT, "tests"), ROOT]
import kanode  # noqa: E402
from test_gpu_native_solve import _fk_cfg, fk_u0  # noqa: E402
from gpu_util import t  # noqa: E402

one = dict(grid_rhs=1, grid_vjp=1, grid_adj_step=1)
for nx in (128, 256):
    for adaptive in (False, True):
        rhs = _fk_cfg(nx, 10, "softsign")
        u0 = t(fk_u0(nx, 12, 3))
        p0 = t(np.random.default_rng(8).uniform(-1.0, 1.0, 11))
        ts = [0.0, 0.2, 0.5] if adaptive else [0.0, 0.05, 0.1]
        tspan = (0.0, ts[-1])
        opt = kanode.Tsit5Options(adaptive=adaptive, dt=None if adaptive else 5e-4 * (256 / nx) ** 2,
                                  abstol=1e-11, reltol=1e-10)
        w = t(np.random.default_rng(12).normal(size=(len(ts),) + tuple(u0.shape)))
        res = {}
        for name, kw in (("fused", {}), ("staged", dict(fused_step=0)), ("fused1", one),
                         ("staged1", dict(fused_step=0, **one))):
            with rhs.hd.options(**kw):
                p = p0.clone().requires_grad_(True)
                x0 = u0.clone().requires_grad_(True)
                sol = kanode.solve(rhs, x0, tspan, p, ts, opt, sensealg="interpolating_adjoint")
                g, gu = torch.autograd.grad((sol.u * w).sum(), [p, x0])
                res[name] = (sol.u.detach(), g, gu, sol.stats["naccept"], sol.stats["adjoint"]["naccept"])
        for a, b in (("fused", "staged"), ("fused1", "staged1"), ("fused1", "fused"), ("staged1", "staged")):
            A, Bb = res[a], res[b]
            du = (A[0] - Bb[0]).abs()
            rows = du.amax(dim=(0, 2)).tolist()
            print(f"nx {nx} adaptive {adaptive} {a:7s} vs {b:7s}: steps {A[3]}/{Bb[3]} adj {A[4]}/{Bb[4]} "
                  f"u {du.max().item():.2e} dp {(A[1] - Bb[1]).abs().max().item():.2e} "
                  f"du0 {(A[2] - Bb[2]).abs().max().item():.2e} u rows " + " ".join(f"{r:.0e}" for r in rows),
                  flush=True)
