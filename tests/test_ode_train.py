"""Host-side Tsit5 / Adam / checkpoint checks on CPU with pure-torch right-hand sides
(the integrator and optimiser are device-agnostic torch code; the HIP RHS is
exercised by tests/test_gpu_ode.py)."""
import os

import numpy as np
import pytest
import torch

import kanode
from kanode import ode


def lotka(u, p, t):
    """lotka! (LV_driver_KANODE.jl:27-33) out-of-place: p = [α, β, δ, γ]."""
    x, y = u[..., 0], u[..., 1]
    return torch.stack([p[0] * x - p[1] * x * y, p[2] * x * y - p[3] * y], dim=-1)


def test_tableau_consistency():
    for i, row in enumerate(ode.A[:5]):
        assert abs(sum(row) - ode.C[i]) < 1e-12
    assert abs(sum(ode.A[5]) - 1.0) < 1e-12
    assert abs(sum(ode.BTILDE)) < 1e-15
    w1 = ode.interp_weights(1.0)
    for a, b in zip(ode.A[5] + (0.0,), w1):
        assert abs(a - b) < 1e-12     # dense output at θ=1 is the step result
    assert all(abs(w) < 1e-15 for w in ode.interp_weights(0.0))


def test_lv_ground_truth(golden):
    """Tsit5 at 1e-12 reproduces the LV training data (LV_driver_KANODE.jl:119-126)."""
    d = golden("lv_truth")
    p = torch.tensor([1.5, 1.0, 1.0, 3.0], dtype=torch.float64)
    u0 = torch.tensor([1.0, 1.0], dtype=torch.float64)
    sol = kanode.solve(lotka, u0, (0.0, 14.0), p, saveat=0.1, opt=kanode.Tsit5Options(abstol=1e-12, reltol=1e-12))
    assert sol.u.shape == (141, 2)
    assert np.max(np.abs(sol.u.numpy().T - d["X"])) < 1e-8


def test_default_tolerances_and_saveat_interpolation(golden):
    d = golden("lv_truth")
    p = torch.tensor([1.5, 1.0, 1.0, 3.0], dtype=torch.float64)
    sol = kanode.solve(lotka, torch.tensor([1.0, 1.0], dtype=torch.float64), (0.0, 3.5), p,
                       saveat=[0.1 * i for i in range(35)])
    # default abstol 1e-6 / reltol 1e-3: interpolated saveat values within the tolerance band
    assert np.max(np.abs(sol.u.numpy().T - d["X"][:, :35])) < 2e-2
    assert sol.stats["naccept"] < 60


def test_fixed_step_fifth_order():
    f = lambda u, p, t: -u + torch.sin(torch.as_tensor(t, dtype=u.dtype))  # noqa: E731
    u0 = torch.tensor([1.0], dtype=torch.float64)
    exact = (1.5 * np.exp(-2.0) + 0.5 * (np.sin(2.0) - np.cos(2.0)))
    errs = []
    for dt in (0.1, 0.05):
        s = kanode.solve(f, u0, (0.0, 2.0), None, saveat=[2.0], opt=kanode.Tsit5Options(adaptive=False, dt=dt))
        errs.append(abs(s.u[-1, 0].item() - exact))
    assert 28 < errs[0] / errs[1] < 80    # >= 2^5 (this linear problem converges at ~2^5.9 here)


def test_adam_matches_flux_formula():
    x = torch.tensor([1.0, -2.0, 3.0], dtype=torch.float64)
    opt = kanode.Adam(0.01)
    xs = x.clone()
    m = np.zeros(3)
    v = np.zeros(3)
    b1, b2 = 0.9, 0.999
    xr = x.numpy().copy()
    for t in range(1, 6):
        g = np.array([0.5, -1.0, 2.0]) * t
        opt.update(xs, torch.as_tensor(g))
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        xr -= m / (1 - b1 ** t) / (np.sqrt(v / (1 - b2 ** t)) + 1e-8) * 0.01
    assert np.allclose(xs.numpy(), xr, rtol=0, atol=1e-15)


def test_adam_float32_promotes_like_flux():
    """Float32 parameters take Flux's Float64-promoted step (rounded on store), the statement
    kanode_adam_step runs on the GPU, so CPU and GPU trainers follow one optimiser trajectory."""
    rng = np.random.default_rng(3)
    x0 = rng.normal(size=240).astype(np.float32)
    grads = [rng.normal(size=240).astype(np.float32) for _ in range(5)]
    x = torch.as_tensor(x0.copy())
    opt = kanode.Adam(1e-3)
    m = np.zeros(240, np.float32)
    v = np.zeros(240, np.float32)
    xr = x0.copy()
    b1, b2, bp1, bp2 = 0.9, 0.999, 0.9, 0.999
    for g in grads:
        opt.update(x, torch.as_tensor(g))
        d = g.astype(np.float64)
        m = (b1 * m.astype(np.float64) + (1 - b1) * d).astype(np.float32)
        v = (b2 * v.astype(np.float64) + ((1 - b2) * d) * d).astype(np.float32)
        step = m.astype(np.float64) / (1 - bp1) / (np.sqrt(v.astype(np.float64) / (1 - bp2)) + 1e-8) * 1e-3
        xr = xr - step.astype(np.float32)   # Δ stored in the Float32 gradient array, x .-= Δ in Float32
        bp1 *= b1
        bp2 *= b2
    assert x.dtype == torch.float32
    assert np.array_equal(x.numpy(), xr)


def test_trainer_reduces_loss_on_lv():
    """Fit the LV parameters themselves with the Trainer (torch RHS on CPU)."""
    ptrue = torch.tensor([1.5, 1.0, 1.0, 3.0], dtype=torch.float64)
    u0 = torch.tensor([1.0, 1.0], dtype=torch.float64)
    ts = [0.1 * i for i in range(35)]
    target = kanode.solve(lotka, u0, (0.0, 3.5), ptrue, saveat=ts,
                          opt=kanode.Tsit5Options(abstol=1e-10, reltol=1e-10)).u
    tr = kanode.Trainer(lotka, u0, (0.0, 3.5), ts, target, ptrue * 1.1, eta=1e-2)
    l0 = tr.step()
    for _ in range(30):
        l1 = tr.step()
    assert l1 < 0.5 * l0


def test_checkpoint_roundtrip(tmp_path):
    P = [np.arange(240, dtype=np.float64) * k for k in range(3)]
    path = os.path.join(tmp_path, "LV_kanode_results.mat")
    kanode.checkpoint.save_lv(path, P, [3.0, 2.0, 1.0], [4.0, 3.0, 2.0], np.arange(5.0), np.ones((2, 5)),
                              [2, 10, 5])
    d = kanode.checkpoint.load(path)
    assert np.array_equal(d["p"], P[-1]) and len(d["p_list"]) == 3
    assert d["loss"].tolist() == [3.0, 2.0, 1.0] and d["size_KAN"].tolist() == [2.0, 10.0, 5.0]


def test_reg_loss_matches_driver_formula():
    """reg_loss (LV_driver_KANODE.jl:187-194): L1 activation loss + entropy of |p|/Σ|p|, and the
    driver's call shape reg_loss(p, 5e-4, 0) (:200, sparse_on = 1) that adds only the scaled L1 term."""
    rng = np.random.default_rng(0)
    p = rng.normal(size=240)
    l1 = np.abs(p)
    a = l1.sum()
    e = l1 / a
    ref = a * 0.7 + (-(e * np.log(e)).sum()) * 0.3
    assert abs(kanode.reg_loss(torch.as_tensor(p), 0.7, 0.3).item() - ref) <= 1e-13 * abs(ref)
    assert abs(kanode.reg_loss(torch.as_tensor(p)).item() - (a + -(e * np.log(e)).sum())) <= 1e-13 * a
    pt = torch.as_tensor(p).requires_grad_(True)
    r = kanode.reg_loss(pt, 5e-4, 0)
    assert abs(r.item() - 5e-4 * a) <= 1e-15 * a
    (g,) = torch.autograd.grad(r, [pt])
    assert torch.equal(g, 5e-4 * torch.sign(torch.as_tensor(p)))
    # an exact zero in p: 0·log(0) is NaN in Julia and in torch alike, and ·0 keeps it NaN
    p[3] = 0.0
    assert np.isnan(kanode.reg_loss(torch.as_tensor(p), 5e-4, 0).item())


def test_trainer_sparse_reg_adds_the_l1_term():
    """Trainer(sparse_reg = 5e-4) is the driver's loss(p) with sparse_on = 1 (:196-201): its gradient
    is the plain loss gradient plus 5e-4·sign(p)."""
    ptrue = torch.tensor([1.5, 1.0, 1.0, 3.0], dtype=torch.float64)
    u0 = torch.tensor([1.0, 1.0], dtype=torch.float64)
    ts = [0.1 * i for i in range(35)]
    target = kanode.solve(lotka, u0, (0.0, 3.5), ptrue, saveat=ts,
                          opt=kanode.Tsit5Options(abstol=1e-10, reltol=1e-10)).u
    plain = kanode.Trainer(lotka, u0, (0.0, 3.5), ts, target, ptrue * 1.1)
    reg = kanode.Trainer(lotka, u0, (0.0, 3.5), ts, target, ptrue * 1.1, sparse_reg=5e-4)
    l0, g0, _ = plain.loss_and_grad()
    l1, g1, _ = reg.loss_and_grad()
    assert abs((l1 - l0).item() - 5e-4 * (ptrue * 1.1).abs().sum().item()) <= 1e-15
    assert torch.allclose(g1 - g0, 5e-4 * torch.sign(ptrue), rtol=0, atol=1e-13)   # differences of O(1) gradients
