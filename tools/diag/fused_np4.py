"""Diagnostic: fused vs per-stage Fisher-KPP solve + adjoint, per-row du0 / dp differences and step
counts, for Nx = 128/256/512, adaptive and fixed (ADVICE r01 NP=4 case)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "kan-odes_amd"), os.path.join(ROOT, "tests"), ROOT]
import kanode  # noqa: E402
from test_gpu_native_solve import _fk_cfg, _fused_vs_staged, fk_u0  # noqa: E402
from gpu_util import t  # noqa: E402

for nx in (128, 256, 512):
    for adaptive in (True, False):
        for tol in (1e-7, 1e-10):
            rhs = _fk_cfg(nx, 10, "softsign")
            u0 = t(fk_u0(nx, 4))
            p0 = t(np.random.default_rng(7).uniform(-1.0, 1.0, 11))
            if adaptive:
                tspan, ts = (0.0, 1.0), [0.25 * i for i in range(5)]
            else:
                tspan, ts = (0.0, 0.1), [0.0, 0.05, 0.1]
            opt = kanode.Tsit5Options(adaptive=adaptive, dt=None if adaptive else 5e-4, abstol=tol * 0.1, reltol=tol)
            (sf, gf, guf), (ss, gs, gus) = _fused_vs_staged(rhs, u0, p0, tspan, ts, opt)
            rows = ((guf - gus).abs().amax(1) / gus.abs().amax(1)).tolist()
            print(f"nx {nx} adaptive {adaptive} reltol {tol:g}: fwd {sf.stats['naccept']}/{ss.stats['naccept']} "
                  f"adj {sf.stats['adjoint']['naccept']}/{ss.stats['adjoint']['naccept']} "
                  f"u {(sf.u - ss.u).abs().max().item():.2e} dp {((gf - gs).abs().max() / gs.abs().max()).item():.2e} "
                  f"du0 rows " + " ".join(f"{r:.1e}" for r in rows), flush=True)
