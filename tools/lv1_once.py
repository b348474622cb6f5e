#!/usr/bin/env python3
"""One LV single-trajectory training iteration setup + 3 iterations (for PMC passes on the
one-workgroup forward / adjoint kernels); prints the step statistics."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kan-odes_amd"))
sys.path.insert(0, ROOT)

import kanode  # noqa: E402
from scipy.integrate import solve_ivp  # noqa: E402

dev = torch.device("cuda:0")
ts = [0.1 * i for i in range(35)]
f = lambda t, x: [1.5 * x[0] - x[0] * x[1], x[0] * x[1] - 3.0 * x[1]]   # noqa: E731
target = solve_ivp(f, (0.0, 3.5), [1.0, 1.0], t_eval=ts, method="DOP853", rtol=1e-10, atol=1e-12).y.T[:, None, :]
chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
p0 = chain.setup(np.random.default_rng(0))[0].astype(np.float64) / 1e5 * 1e4
tr = kanode.Trainer(kanode.ChainRHS(chain, device=dev), torch.tensor([[1.0, 1.0]], dtype=torch.float64, device=dev),
                    (0.0, 3.5), ts, torch.as_tensor(target, device=dev), torch.as_tensor(p0, device=dev), eta=1e-3,
                    sensealg="interpolating_adjoint")
for _ in range(3):
    tr.step()
_, _, sol = tr.loss_and_grad()
print("forward", {k: v for k, v in sol.stats.items() if k != "adjoint"}, "adjoint", sol.stats.get("adjoint"))
