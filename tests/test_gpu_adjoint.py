"""kanode_vjp_stage and the InterpolatingAdjoint on the GPU (SciMLSensitivity's default sensealg for
the reference's NeuralODE / Fisher-KPP problems) vs the same driver on the CPU oracle."""
import numpy as np
import pytest
import torch

from gpu_util import device, t
from oracle import oracle as O
from oracle.oracle_rhs import OracleChainRHS, OracleFKRHS

import kanode
from kanode.ode import A, BTILDE

pytestmark = pytest.mark.gpu


def fk(nx, table=None):
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
    return kanode.FisherKPPRHS(kan1, nx=nx, dx=1.0 / (nx - 1), D=0.01, device=device(), table=table)


def lv(dtype=torch.float64):
    return kanode.ChainRHS(kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5)), dtype=dtype,
                           device=device())


@pytest.mark.parametrize("name,make", [("fk256", lambda: fk(256)), ("fk256_rec", lambda: fk(256, False)),
                                       ("fk26", lambda: fk(26)), ("lv64", lv),
                                       ("lv32", lambda: lv(torch.float32))])
def test_vjp_stage_matches_composition(name, make):
    rhs = make()
    dtype = rhs.hd.dtype
    rng = np.random.default_rng(len(name))
    shape = (4, rhs.N)
    p = t(rng.uniform(-0.5, 0.5, rhs.P) * (1.0 if name.startswith("fk") else 0.3), dtype)
    u = t(rng.uniform(0, 1, shape), dtype)
    ks = [t(rng.normal(size=shape) * 0.3, dtype) for _ in range(7)]
    c = [0.01 * w for w in kanode.ode.interp_weights(0.37)]
    lam = t(rng.normal(size=shape), dtype)
    lks = [t(rng.normal(size=shape), dtype) for _ in range(6)]
    lc = [0.01 * a for a in A[5]]
    lam_out = torch.empty_like(lam)
    sumsq = torch.empty(1, dtype=torch.float64, device=device())
    ec = [0.01 * b for b in BTILDE]
    lamJ, dp = rhs.vjp_stage(u, p, ks, c, lam, lks, lc, lam_out, (ec, 1e-6, 1e-3, sumsq))
    y = u.clone()
    for cj, kj in zip(c, ks):
        y = torch.addcmul(y, kj, torch.full_like(kj, cj))
    ls = lam.clone()
    for cj, kj in zip(lc, lks):
        ls = torch.addcmul(ls, kj, torch.full_like(kj, cj))
    rJ, rdp = rhs.hd.vjp(p, y, ls)
    eps = 1e-12 if dtype == torch.float64 else 2e-5
    assert (lam_out - ls).abs().max().item() <= eps * ls.abs().max().item()
    assert (lamJ - rJ).abs().max().item() <= eps * max(1.0, rJ.abs().max().item())
    assert (dp - rdp).abs().max().item() <= eps * max(1.0, rdp.abs().max().item())
    e = sum(ej * kj.double() for ej, kj in zip(ec[:-1], lks)) + ec[-1] * lamJ.double()
    sk = 1e-6 + 1e-3 * torch.maximum(lam.double().abs(), ls.double().abs())
    ref = float(((e / sk) ** 2).sum())
    assert abs(sumsq.item() - ref) <= (1e-10 if dtype == torch.float64 else 1e-4) * ref


def _grad(f, u0, p0, tspan, ts, w, opt):
    p = p0.clone().requires_grad_(True)
    sol = kanode.solve(f, u0, tspan, p, ts, opt, sensealg="interpolating_adjoint")
    (g,) = torch.autograd.grad((sol.u * w).sum(), [p])
    return g, sol.stats


@pytest.mark.parametrize("case", ["lv", "fk26"])
def test_interpolating_adjoint_gpu_matches_cpu_oracle(case):
    rng = np.random.default_rng(9)
    if case == "lv":
        specs = [O.LayerSpec(2, 10, 5, "tanh_fast"), O.LayerSpec(10, 2, 5, "tanh_fast")]
        gpu, cpu = lv(), OracleChainRHS(specs)
        p0 = rng.uniform(-0.3, 0.3, 240)
        u0 = np.array([[1.0, 1.0], [0.6, 1.5]])
        tspan, ts = (0.0, 3.5), [0.1 * i for i in range(35)]
    else:
        gpu, cpu = fk(26), OracleFKRHS(O.LayerSpec(1, 1, 10, "softsign"), 0.01, 1.0 / 25)
        p0 = rng.uniform(-0.5, 0.5, 11)
        x = np.arange(26) / 25
        u0 = ((np.tanh((x - 0.4) / 0.02) - np.tanh((x - 0.6) / 0.02)) / 2)[None]
        tspan, ts = (0.0, 2.0), [0.5 * i for i in range(5)]
    w = rng.normal(size=(len(ts),) + u0.shape)
    opt = kanode.Tsit5Options(abstol=1e-8, reltol=1e-8)
    gg, sg = _grad(gpu, t(u0), t(p0), tspan, ts, t(w), opt)
    gc, sc = _grad(cpu, torch.as_tensor(u0), torch.as_tensor(p0), tspan, ts, torch.as_tensor(w), opt)
    assert sg["naccept"] == sc["naccept"]
    assert sg["adjoint"]["naccept"] == sc["adjoint"]["naccept"]
    assert (gg.cpu() - gc).abs().max().item() <= 1e-9 * gc.abs().max().item()


def test_fk256_interpolating_adjoint_vs_discrete():
    rhs = fk(256)
    x = np.arange(256) / 255
    u0 = np.stack([(np.tanh((x - c) / 0.03) - np.tanh((x - c - 0.2) / 0.03)) / 2 for c in (0.3, 0.5)])
    p0 = np.random.default_rng(4).uniform(-0.5, 0.5, 11)
    ts = [0.1 * i for i in range(6)]
    w = t(np.random.default_rng(5).normal(size=(6, 2, 256)))
    opt = kanode.Tsit5Options(abstol=1e-9, reltol=1e-9)
    gi, st = _grad(rhs, t(u0), t(p0), (0.0, 0.5), ts, w, opt)
    p = t(p0).requires_grad_(True)
    sol = kanode.solve(rhs, t(u0), (0.0, 0.5), p, ts, opt, sensealg="discrete")
    (gd,) = torch.autograd.grad((sol.u * w).sum(), [p])
    assert (gi - gd).norm().item() <= 1e-5 * gd.norm().item()
