#!/usr/bin/env python3
"""The Fisher-KPP table path against the per-point direct kernels (KANODE_OPT_POINTWISE_TABLE = 0) on a field swept
over u in [-3.9, 3.9]: RHS, λᵀJ and dp differences per sign of u, at the trained-like and at random parameters."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import bench  # noqa: E402
import kanode  # noqa: E402

dev = torch.device("cuda:0")
out = {}
for name, pn in (("trained", bench.fk_trained_like_params()), ("random", np.random.default_rng(3).normal(0, 1, 11))):
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign", basis_func="rbf"))
    rhs = kanode.FisherKPPRHS(kan1, nx=256, dx=1 / 255, D=0.0, dtype=torch.float64, device=dev)
    p = torch.as_tensor(pn, device=dev)
    u = torch.linspace(-3.9, 3.9, 16 * 256, dtype=torch.float64, device=dev).reshape(16, 256)
    lam = torch.ones_like(u)
    r1 = rhs.hd.rhs(p, u, torch.empty_like(u)).clone()
    j1, d1 = [x.clone() for x in rhs.hd.vjp(p, u, lam)[:2]]
    rhs.hd.set_option("pointwise_table", 0)
    r0 = rhs.hd.rhs(p, u, torch.empty_like(u)).clone()
    j0, d0 = [x.clone() for x in rhs.hd.vjp(p, u, lam)[:2]]
    neg = u < 0
    out[name] = {"rhs_neg": float((r1 - r0)[neg].abs().max()), "rhs_pos": float((r1 - r0)[~neg].abs().max()),
                 "lamJ_neg": float((j1 - j0)[neg].abs().max()), "lamJ_pos": float((j1 - j0)[~neg].abs().max()),
                 "dp_rel": float((d1 - d0).abs().max() / d0.abs().max()), "rhs_scale": float(r0.abs().max())}
print(json.dumps(out), flush=True)
