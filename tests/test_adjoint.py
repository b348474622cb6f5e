"""InterpolatingAdjoint driver (kanode.adjoint, SciMLSensitivity's default for NeuralODE) on CPU:
a pure-torch Lotka-Volterra RHS (lotka!, LV_driver_KANODE.jl:27-33) and the oracle KAN chain
(LV_driver_KANODE.jl:139-143), against central finite differences and the discrete adjoint.
The HIP adjoint stage is exercised by tests/test_gpu_adjoint.py."""
import numpy as np
import pytest
import torch

import kanode
from oracle import oracle as O
from oracle.oracle_rhs import OracleChainRHS


class TorchRHS:
    """Out-of-place RHS with a vjp_stage built from torch.autograd (same contract as kanode's)."""

    def __init__(self, f):
        self.f = f

    def __call__(self, u, p, t=None):
        return self.f(u, p)

    def vjp_stage(self, u, p, ks, c, lam, lks, lc, lam_out=None, error=None):
        y = u.clone()
        for cj, kj in zip(c, ks):
            y = y + cj * kj
        ls = lam.clone()
        for cj, kj in zip(lc, lks):
            ls = ls + cj * kj
        with torch.enable_grad():
            yy = y.detach().requires_grad_(True)
            pp = p.detach().requires_grad_(True)
            lamJ, dp = torch.autograd.grad(self.f(yy, pp), [yy, pp], ls)
        if lam_out is not None:
            lam_out.copy_(ls)
        if error is not None:
            ec, abstol, reltol, sumsq = error
            e = sum(ej * kj for ej, kj in zip(ec[:-1], lks)) + ec[-1] * lamJ
            sk = abstol + reltol * torch.maximum(lam.abs(), ls.abs())
            sumsq.fill_(float(((e / sk) ** 2).sum()))
        return lamJ, dp


def lotka(u, p):
    x, y = u[..., 0], u[..., 1]
    return torch.stack([p[0] * x - p[1] * x * y, p[2] * x * y - p[3] * y], dim=-1)


def loss_of(sol, w):
    return (sol.u * w).sum()


def grads(f, u0, p0, tspan, ts, w, opt, sensealg):
    p = p0.clone().requires_grad_(True)
    u = u0.clone().requires_grad_(True)
    sol = kanode.solve(f, u, tspan, p, ts, opt, sensealg=sensealg)
    gp, gu = torch.autograd.grad(loss_of(sol, w), [p, u])
    return gp, gu, sol


def fd(f, u0, p0, tspan, ts, w, opt, d, h=1e-6):
    with torch.no_grad():
        lp = loss_of(kanode.solve(f, u0, tspan, p0 + h * d, ts, opt), w)
        lm = loss_of(kanode.solve(f, u0, tspan, p0 - h * d, ts, opt), w)
    return float(lp - lm) / (2 * h)


@pytest.mark.parametrize("adaptive", [True, False])
def test_lotka_interpolating_adjoint_vs_fd_and_discrete(adaptive):
    f = TorchRHS(lotka)
    p0 = torch.tensor([1.5, 1.0, 1.0, 3.0], dtype=torch.float64)
    u0 = torch.tensor([[1.0, 1.0], [0.8, 1.4]], dtype=torch.float64)
    ts = [0.25 * i for i in range(13)]
    w = torch.as_tensor(np.random.default_rng(0).normal(size=(13, 2, 2)))
    opt = kanode.Tsit5Options(abstol=1e-11, reltol=1e-11) if adaptive else kanode.Tsit5Options(adaptive=False,
                                                                                                dt=1e-3)
    gi_p, gi_u, _ = grads(f, u0, p0, (0.0, 3.0), ts, w, opt, "interpolating_adjoint")
    gd_p, gd_u, _ = grads(f, u0, p0, (0.0, 3.0), ts, w, opt, "discrete")
    assert torch.allclose(gi_p, gd_p, rtol=1e-6, atol=1e-8 * gd_p.abs().max().item())
    assert torch.allclose(gi_u, gd_u, rtol=1e-6, atol=1e-8 * gd_u.abs().max().item())
    d = torch.as_tensor(np.random.default_rng(1).normal(size=4))
    assert abs(fd(f, u0, p0, (0.0, 3.0), ts, w, opt, d) - float(gi_p @ d)) <= 1e-5 * float(gi_p.abs().sum())


def test_lv_kan_interpolating_adjoint_default_tolerances():
    """The LV KAN (oracle chain) at the solver defaults (abstol 1e-6, reltol 1e-3): the continuous and
    discrete adjoints differ by the integration error only; the continuous one tracks FD."""
    specs = [O.LayerSpec(2, 10, 5, "tanh_fast"), O.LayerSpec(10, 2, 5, "tanh_fast")]
    f = OracleChainRHS(specs)
    p0 = torch.as_tensor(np.random.default_rng(2).uniform(-0.3, 0.3, 240))
    u0 = torch.tensor([[1.0, 1.0]], dtype=torch.float64)
    ts = [0.1 * i for i in range(35)]
    w = torch.as_tensor(np.random.default_rng(3).normal(size=(35, 1, 2)))
    opt = kanode.Tsit5Options()
    gi_p, _, sol = grads(f, u0, p0, (0.0, 3.5), ts, w, opt, "interpolating_adjoint")
    st = sol.stats.get("adjoint")
    assert st and st["naccept"] > 0
    gd_p, _, _ = grads(f, u0, p0, (0.0, 3.5), ts, w, opt, "discrete")
    rel = float((gi_p - gd_p).norm() / gd_p.norm())
    assert rel < 5e-2
    opt_t = kanode.Tsit5Options(abstol=1e-10, reltol=1e-10)
    gt_p, _, _ = grads(f, u0, p0, (0.0, 3.5), ts, w, opt_t, "interpolating_adjoint")
    d = torch.as_tensor(np.random.default_rng(4).normal(size=240))
    assert abs(fd(f, u0, p0, (0.0, 3.5), ts, w, opt_t, d) - float(gt_p @ d)) <= 1e-5 * float(gt_p.abs() @ d.abs())


def test_trainer_uses_interpolating_adjoint_by_default():
    specs = [O.LayerSpec(2, 10, 5, "tanh_fast"), O.LayerSpec(10, 2, 5, "tanh_fast")]
    f = OracleChainRHS(specs)
    tr = kanode.Trainer(f, torch.tensor([[1.0, 1.0]], dtype=torch.float64), (0.0, 1.0), [0.1 * i for i in range(11)],
                        torch.ones(11, 1, 2, dtype=torch.float64),
                        torch.as_tensor(np.random.default_rng(5).uniform(-0.1, 0.1, 240)), eta=1e-2)
    assert tr.sensealg == "interpolating_adjoint"
    l0 = tr.step()
    for _ in range(5):
        l1 = tr.step()
    assert l1 < l0


def test_replayed_step_sequences_reproduce_the_adaptive_run():
    """Tsit5Options.replay_dts / replay_adjoint_dts (the GPU surrogate test replays the GPU's accepted steps on
    the oracle): replaying an adaptive run's own forward and adjoint step sizes with adaptive=False takes the
    same steps and gives the same solution and gradients bitwise (the saveat stops land as before)."""
    specs = [O.LayerSpec(2, 10, 5, "tanh_fast"), O.LayerSpec(10, 2, 5, "tanh_fast")]
    f = OracleChainRHS(specs)
    p0 = torch.as_tensor(np.random.default_rng(2).uniform(-0.3, 0.3, 240))
    u0 = torch.tensor([[1.0, 1.0]], dtype=torch.float64)
    ts = [0.0, 0.35, 1.0, 1.7, 2.0]
    w = torch.as_tensor(np.random.default_rng(3).normal(size=(len(ts), 1, 2)))
    opt = kanode.Tsit5Options(abstol=1e-8, reltol=1e-8)
    ga, gua, sa = grads(f, u0, p0, (0.0, 2.0), ts, w, opt, "interpolating_adjoint")
    rep = kanode.Tsit5Options(abstol=1e-8, reltol=1e-8, adaptive=False, replay_dts=tuple(sa.stats["dts"]),
                              replay_adjoint_dts=tuple(sa.stats["adjoint"]["dts"]))
    gr, gur, sr = grads(f, u0, p0, (0.0, 2.0), ts, w, rep, "interpolating_adjoint")
    assert sr.stats["dts"] == sa.stats["dts"] and sr.stats["adjoint"]["dts"] == sa.stats["adjoint"]["dts"]
    assert len(sa.stats["adjoint"]["dts"]) == sa.stats["adjoint"]["naccept"] > 5
    assert torch.equal(sr.u, sa.u) and torch.equal(gr, ga) and torch.equal(gur, gua)
