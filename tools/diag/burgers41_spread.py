"""Rounding sensitivity of the Burgers-41 surrogate solve + InterpolatingAdjoint (the case of
tests/test_gpu_native_solve.py::test_native_surrogate_pair_solve_and_gradient_match_cpu_oracle):
GPU two-launch vs four-launch pullback vs the CPU oracle, and the GPU against itself with the
parameters perturbed by one ulp.  Diagnostic only (GPU)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch

import kanode
from oracle import oracle as O
from oracle.oracle_rhs import OracleChainRHS

dev = torch.device("cuda:0")
specs = [O.LayerSpec(41, 10, 5, "softsign"), O.LayerSpec(10, 41, 5, "softsign")]
chain = kanode.Chain(kanode.KDense(41, 10, 5, normalizer="softsign"), kanode.KDense(10, 41, 5, normalizer="softsign"))
rhs = kanode.ChainRHS(chain, device=dev)
x = np.linspace(-1.0, 1.0, 41)
a = np.random.default_rng(4).normal(0.0, 0.1, (2, 3))
u0 = -np.sin(np.pi * x)[None, :] + sum(a[:, k:k + 1] * np.sin((k + 1) * np.pi * x)[None, :] for k in range(3))
p0 = chain.setup(np.random.default_rng(0))[0].astype(np.float64)
ts = [0.0, 0.1, 0.3, 0.5]
w = np.random.default_rng(3).normal(size=(len(ts),) + u0.shape)
opt = kanode.Tsit5Options(abstol=1e-9, reltol=1e-9)


def run(f, d, pv):
    p = torch.as_tensor(pv, device=d).clone().requires_grad_(True)
    x0 = torch.as_tensor(u0, device=d).clone().requires_grad_(True)
    sol = kanode.solve(f, x0, (0.0, 0.5), p, ts, opt, sensealg="interpolating_adjoint")
    g, gu = torch.autograd.grad((sol.u * torch.as_tensor(w, device=d)).sum(), [p, x0])
    return g.cpu().numpy(), gu.cpu().numpy(), sol.stats


res = {}
for pair in (1, 0):
    rhs.hd.set_option("pair_vjp", pair)
    res[f"gpu pair={pair}"] = run(rhs, dev, p0)
rhs.hd.set_option("pair_vjp", 1)
res["gpu pair=1, p + 1 ulp"] = run(rhs, dev, np.nextafter(p0, np.inf))
res["cpu oracle"] = run(OracleChainRHS(specs), "cpu", p0)
ref = res["cpu oracle"]
for k, (g, gu, st) in res.items():
    print(f"{k:24s} steps {st['naccept']}/{st['adjoint']['naccept']}+{st['adjoint']['nreject']}  "
          f"|dp - cpu|/max {np.max(np.abs(g - ref[0])) / np.max(np.abs(ref[0])):.2e}  "
          f"|du0 - cpu|/max {np.max(np.abs(gu - ref[1])) / np.max(np.abs(ref[1])):.2e}", flush=True)
