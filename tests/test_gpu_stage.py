"""kanode_rhs_stage: the Tsit5 stage (OrdinaryDiffEqTsit5 perform_step!) fused into the RHS.

Checked against the unfused composition on the same device — y = u + Σ c_j k_j by torch,
then kanode_rhs — and the Tsit5 embedded error against its torch restatement; the
fused Fisher-KPP table kernel, the generic lincomb + RHS + error path (table off, odd
shapes, the LV chain in fp64 and fp32) and autograd through the stage.
"""
import numpy as np
import pytest
import torch

from gpu_util import RTOL, assert_close, device, fk_scale, t

import kanode
from kanode.ode import A, BTILDE

pytestmark = pytest.mark.gpu


def fk_rhs(nx, table=None, D=0.01):
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
    return kanode.FisherKPPRHS(kan1, nx=nx, dx=1.0 / (nx - 1), D=D, device=device(), table=table)


def lv_rhs(dtype):
    return kanode.ChainRHS(kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5)), dtype=dtype,
                           device=device())


def stage_inputs(rng, shape, n, dtype, scale=0.3):
    u = rng.uniform(0.0, 1.0, shape)
    ks = [rng.normal(size=shape) * scale for _ in range(n)]
    return t(u, dtype), [t(k, dtype) for k in ks]


CASES = [("fk256_table", lambda: fk_rhs(256)), ("fk256_rec", lambda: fk_rhs(256, table=False)),
         ("fk128_table", lambda: fk_rhs(128)), ("fk26", lambda: fk_rhs(26)),
         ("lv_f64", lambda: lv_rhs(torch.float64)), ("lv_f32", lambda: lv_rhs(torch.float32))]


@pytest.mark.parametrize("name,make", CASES)
@pytest.mark.parametrize("stage", [0, 1, 5])
def test_stage_matches_unfused(name, make, stage):
    rhs = make()
    dtype = rhs.hd.dtype
    rng = np.random.default_rng(stage * 7 + len(name))
    B = 5
    shape = (B, rhs.N)
    p = t(rng.uniform(-0.5, 0.5, rhs.P) * (1.0 if name.startswith("fk") else 0.3), dtype)
    u, ks = stage_inputs(rng, shape, stage + 1, dtype)
    dt = 0.01
    c = [dt * a for a in A[stage]]
    y_ref = u.clone()
    for cj, kj in zip(c, ks):
        y_ref = y_ref + cj * kj
    du_ref = rhs.rhs(y_ref, p)
    y = torch.empty_like(u)
    sumsq = torch.empty(1, dtype=torch.float64, device=device())
    ec = [dt * b for b in BTILDE[:len(ks)]] + [dt * BTILDE[-1]]
    du = rhs.hd.rhs_stage(p, u, ks, c, y_out=y, error=(ec, 1e-6, 1e-3, sumsq))
    yscale = u.abs() + sum(abs(cj) * kj.abs() for cj, kj in zip(c, ks))
    tol = RTOL[dtype]
    assert_close(y, y_ref.cpu().numpy(), yscale.cpu().numpy(), 4 * np.finfo(np.float64 if dtype == torch.float64
                                                                              else np.float32).eps, "y")
    if name.startswith("fk"):
        yn = y_ref.cpu().numpy()
        pn = p.cpu().numpy()
        dsc = fk_scale(pn, rhs.D, rhs.dx, yn) * (1 + 1e3 * np.abs(yn))   # + |f'|·|δy| from y's rounding
    else:
        dsc = du_ref.abs().cpu().numpy() + du_ref.abs().max().item() * 1e-3
    assert_close(du, du_ref.cpu().numpy(), dsc, 10 * tol, "du")
    e = sum(ecj * kj.double() for ecj, kj in zip(ec[:-1], ks)) + ec[-1] * du.double()
    sk = 1e-6 + 1e-3 * torch.maximum(u.double().abs(), y.double().abs())
    ref = float(((e / sk) ** 2).sum())
    assert abs(sumsq.item() - ref) <= 1e-10 * ref + 1e-300


def test_stage_n_prev_zero_is_rhs():
    rhs = fk_rhs(256)
    rng = np.random.default_rng(3)
    p = t(rng.uniform(-1, 1, 11))
    u = t(rng.uniform(0, 1, (4, 256)))
    assert torch.equal(rhs.hd.rhs_stage(p, u, [], []), rhs.rhs(u, p))


@pytest.mark.parametrize("name,make", [CASES[0], CASES[3], CASES[4]])
def test_stage_autograd_matches_unfused(name, make):
    rhs = make()
    rng = np.random.default_rng(11)
    shape = (3, rhs.N)
    p0 = rng.uniform(-0.5, 0.5, rhs.P) * (1.0 if name.startswith("fk") else 0.3)
    u0, ks0 = stage_inputs(rng, shape, 3, torch.float64)
    c = [0.02 * a for a in A[2]]
    w = t(rng.normal(size=shape))
    grads = []
    for fused in (True, False):
        p = t(p0).requires_grad_(True)
        u = u0.clone().requires_grad_(True)
        ks = [k.clone().requires_grad_(True) for k in ks0]
        if fused:
            du, y = rhs.stage(u, p, ks, c, want_y=True)
        else:
            y = u
            for cj, kj in zip(c, ks):
                y = y + cj * kj
            du = rhs(y, p)
        loss = (du * w).sum() + (y * w).sum() * 0.5
        grads.append(torch.autograd.grad(loss, [p, u] + ks))
    for gf, gu in zip(*grads):
        sc = gu.abs().max().item()
        assert (gf - gu).abs().max().item() <= 1e-11 * sc


@pytest.mark.parametrize("name,make", [CASES[0], CASES[3], CASES[4]])
def test_fused_solve_matches_unfused(name, make):
    rhs = make()
    rng = np.random.default_rng(5)
    if name.startswith("fk"):
        x = np.arange(rhs.N) / (rhs.N - 1)
        u0 = np.stack([(np.tanh((x - 0.4) / 0.02) - np.tanh((x - 0.6) / 0.02)) / 2 * a for a in (0.6, 0.9)])
        p = rng.uniform(-0.5, 0.5, rhs.P)
        tspan, ts = (0.0, 1.0), [0.25 * i for i in range(5)]
    else:
        u0 = np.array([[1.0, 1.0], [0.7, 1.3]])
        p = rng.uniform(-0.3, 0.3, rhs.P)
        tspan, ts = (0.0, 3.5), [0.1 * i for i in range(35)]
    sols = []
    for fused in (True, False):
        opt = kanode.Tsit5Options(fused=fused)
        sols.append(kanode.solve(rhs, t(u0), tspan, t(p), ts, opt))
    assert sols[0].stats["naccept"] == sols[1].stats["naccept"]
    # the fused stage combination rounds once per fma instead of per mul/add: 1-ulp
    # differences per stage accumulate over the run (738 steps of the stiff 256-point
    # Fisher-KPP, D/dx² = 650) to <= 1e-9 — the integrator's own tolerance is 1e-3
    tol = 1e-9 if name.startswith("fk") else 1e-11
    assert (sols[0].u - sols[1].u).abs().max().item() <= tol * max(1.0, sols[1].u.abs().max().item())
