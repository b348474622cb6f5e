"""Why test_gpu_fk_e2e.py::test_fk_default_path_negative_states[adaptive] does not compare adjoint step counts.

On the all-negative Fisher-KPP field (u in [-2.2, -1.2], D = 0) the KAN source is nearly linear and the adjoint's
embedded Tsit5 error estimate sits at the rounding level of the VJP itself, so the step sizes its PI controller picks
follow last-bit noise.  Shown here on the CPU oracle alone (the dense-Laplacian C restatement of
PDE examples/Fisher-KPP_Source.jl:55-59,95-98 behind the Python InterpolatingAdjoint): perturbing the oracle's VJP
by a relative 1e-14 (seeded, uniform) changes its adjoint step count from 10 to 8 while dL/dp stays put to 1e-12.
The GPU table path (8 steps) and the direct per-point kernels (10 steps) sit on either side of the same noise
(profiles/r06/negative/steps.json)."""
import numpy as np
import torch

from oracle import oracle as O
from oracle.oracle_rhs import OracleFKRHS

import kanode

NX, B, SEED = 256, 3, 31


def _u0():
    """test_gpu_fk_e2e._u0 (the reference IC family, Fisher-KPP_Source.jl:47-49), amplitude 1, shifted by -2.2"""
    rng = np.random.default_rng(SEED)
    x = np.arange(NX) / (NX - 1)
    c, d, a = rng.uniform(0.3, 0.7, (B, 1)), rng.uniform(0.1, 0.3, (B, 1)), rng.uniform(0.5, 1, (B, 1))
    return a * (np.tanh((x - (c - d / 2)) / (d / 10)) - np.tanh((x - (c + d / 2)) / (d / 10))) / 2 - 2.2


class _NoisyVJP(OracleFKRHS):
    def __init__(self, eps, *a, **k):
        super().__init__(*a, **k)
        self.eps, self.rng = eps, np.random.default_rng(7)

    def vjp(self, y, p, lam):
        lj, dp = super().vjp(y, p, lam)
        if self.eps:
            lj = lj * (1 + self.eps * torch.as_tensor(self.rng.uniform(-1, 1, lj.shape)))
            dp = dp * (1 + self.eps * torch.as_tensor(self.rng.uniform(-1, 1, dp.shape)))
        return lj, dp


def _run(eps):
    f = _NoisyVJP(eps, O.LayerSpec(1, 1, 10, "softsign"), 0.0, 1.0 / (NX - 1), dense=True)
    ts = [0.0, 0.15, 0.25, 0.5]
    w = torch.as_tensor(np.random.default_rng(SEED + 200).normal(size=(len(ts), B, NX)))
    p = torch.as_tensor(0.5 * np.random.default_rng(SEED + 100).uniform(-1.0, 1.0, 11)).requires_grad_(True)
    x0 = torch.as_tensor(_u0()).requires_grad_(True)
    sol = kanode.solve(f, x0, (0.0, 0.5), p, ts, kanode.Tsit5Options(abstol=1e-9, reltol=1e-9),
                       sensealg="interpolating_adjoint")
    gp, = torch.autograd.grad((sol.u * w).sum(), [p])
    return sol.stats["adjoint"], gp


def test_adjoint_steps_follow_rounding_noise_on_the_negative_field():
    st0, gp0 = _run(0.0)
    st1, gp1 = _run(1e-14)
    assert (st0["naccept"], st0["nreject"]) == (10, 0)
    assert (st1["naccept"], st1["nreject"]) == (8, 0)
    assert abs(st1["dts"][1] / st0["dts"][1] - 1.0) > 0.1
    assert (gp1 - gp0).abs().max().item() <= 1e-12 * gp0.abs().max().item()
