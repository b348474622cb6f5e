#!/usr/bin/env python3
"""Solve + InterpolatingAdjoint of the one-workgroup problems (LV [2,10,2] one trajectory; FK26 one IC) with
whatever library KANODE_LIB names, saved to an .npz, so two library builds can be compared bitwise:
    KANODE_LIB=... python tools/onewg_dump.py OUT.npz"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import kanode  # noqa: E402

dev = torch.device("cuda:0")
out = {}
chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
rhs = kanode.ChainRHS(chain, device=dev)
p0 = torch.as_tensor(chain.setup(np.random.default_rng(0))[0].astype(np.float64) / 10, device=dev)
ts = [0.1 * i for i in range(35)]
for name, r, u0, p_, tspan in (
        ("lv1", rhs, torch.tensor([[1.0, 1.0]], dtype=torch.float64, device=dev), p0, (0.0, 3.5)),):
    p = p_.clone().requires_grad_(True)
    x0 = u0.clone().requires_grad_(True)
    sol = kanode.solve(r, x0, tspan, p, ts, kanode.Tsit5Options(), sensealg="interpolating_adjoint")
    w = torch.as_tensor(np.random.default_rng(1).normal(size=tuple(sol.u.shape)), device=dev)
    g, gu = torch.autograd.grad((sol.u * w).sum(), [p, x0])
    out[name + "_u"], out[name + "_g"], out[name + "_gu"] = (a.detach().cpu().numpy() for a in (sol.u, g, gu))
    out[name + "_steps"] = np.array([sol.stats["naccept"], sol.stats["adjoint"]["naccept"]])
np.savez(sys.argv[1], **out)
print({k: v.shape for k, v in out.items()}, out["lv1_steps"])
