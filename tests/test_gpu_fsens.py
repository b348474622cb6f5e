"""Forward sensitivities: the gradient the reference computes for its small source-term problems.

`Zygote.gradient(x -> loss(x), p)` in PDE examples/Fisher-KPP_Source.jl:198 (and the Allen-Cahn source driver)
passes no sensealg; with length(u0) + length(p) = 26 + 11 <= 100 SciMLSensitivity 7.69 picks
ForwardDiffSensitivity: the solve over ForwardDiff.Dual numbers, one partial per parameter.  The
native kernel (kan_small.hip fk_small_fsens_kernel, kanode_forward_sensitivity_tsit5) is compared here with a torch
restatement of that Dual solve, written out below (third-party semantics, restated from the pinned
SciMLSensitivity 7.69 / DiffEqBase / OrdinaryDiffEq 6.89 — verify where Julia exists):

  * state [u; S_1..S_P], S_k = ∂u/∂p_k, S_k' = J S_k + ∂f/∂p_k (J = D lap + diag φ'(u): J S_k is the native VJP,
    J being symmetric; ∂φ/∂C_k = B_k(softsign(u)) by the reference formula, ∂φ/∂W = swish(u));
  * DiffEqBase's ODE_DEFAULT_NORM over Dual numbers counts the partials: per state entry i the residual scale is
    abstol + reltol·max(‖u_i‖, ‖unew_i‖), ‖x‖ = sqrt(value² + Σ partial²); EEst = RMS over all n·(1 + P) values;
    the Hairer-Wanner initial step uses the same norms; saveat from the same interpolant.

Bars: on the kernel's own step sequence (replayed) the values and sensitivities agree to rounding and the
restatement's controller proposes the kernel's step sizes; on its own steps the restatement takes the same
accepted / rejected counts (see the test's docstring for why its values are then held at 1e-6)."""
import math

import numpy as np
import pytest
import torch

import kanode
from kanode.ode import A, BTILDE, C as CNODE, interp_weights

pytestmark = pytest.mark.gpu

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def dual_tsit5(F, z0, t0, tf, saveat, opt, replay=None):
    """The Dual-number Tsit5 solve restated on the stacked state z = [u; S_1..S_P] (rows), entries in columns.
    replay: take these accepted step sizes in order (another solver's sequence) and return, with the usual
    results, the step size this controller would have proposed after each of them (and its initial step)."""
    numel = z0.numel()

    def nrm(z):   # per entry: sqrt(value² + Σ partials²)
        return torch.sqrt((z * z).sum(0))

    def rmsn(x):
        return math.sqrt(float((x * x).sum()) / numel)

    out, si = [], 0
    while si < len(saveat) and saveat[si] <= t0 + 1e-14 * max(1.0, abs(t0)):
        out.append(z0)
        si += 1
    z, t = z0, t0
    k1 = F(z)
    sk = opt.abstol + nrm(z0) * opt.reltol
    d0, d1 = rmsn(z0 / sk), rmsn(k1 / sk)
    dt0 = 1e-6 if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
    dt0 = min(dt0, tf - t0)
    f1 = F(z0 + dt0 * k1)
    d2 = rmsn((f1 - k1) / sk) / dt0
    mx = max(d1, d2)
    dt1 = max(1e-6, dt0 * 1e-3) if mx <= 1e-15 else (0.01 / mx) ** (1.0 / 5.0)
    dt = min(100 * dt0, dt1, tf - t0)
    proposed = [dt]
    qold, naccept, nreject = opt.qoldinit, 0, 0
    for _ in range(100000):
        if t >= tf - 1e-14 * max(1.0, abs(tf)):
            break
        if replay is not None:
            dt = float(replay[naccept])
        dt = min(dt, tf - t)
        ks = [k1]
        for i in range(6):
            y = z
            for j, a in enumerate(A[i]):
                y = y + (dt * a) * ks[j]
            ks.append(F(y))
        znew = y
        e = sum((dt * b) * k for b, k in zip(BTILDE, ks))
        skn = opt.abstol + torch.maximum(nrm(z), nrm(znew)) * opt.reltol
        EEst = rmsn(e / skn)
        q11 = EEst ** opt.beta1 if EEst > 0 else 0.0
        if EEst > 1.0 and replay is None:
            nreject += 1
            dt = dt / min(1.0 / opt.qmin, q11 / opt.gamma)
            continue
        q = q11 / (qold ** opt.beta2)
        q = max(1.0 / opt.qmax, min(1.0 / opt.qmin, q / opt.gamma))
        dtnew = dt / q
        qold = max(EEst, opt.qoldinit)
        proposed.append(dtnew)
        tn = t + dt
        while si < len(saveat) and saveat[si] <= tn + 1e-12 * max(1.0, abs(tn)):
            ts = saveat[si]
            if abs(ts - tn) <= 1e-12 * max(1.0, abs(tn)):
                out.append(znew)
            else:
                w = interp_weights((ts - t) / dt)
                out.append(z + dt * sum(wi * k for wi, k in zip(w, ks)))
            si += 1
        z, k1, t = znew, ks[6], tn
        naccept += 1
        dt = dtnew
    if replay is not None:
        return torch.stack(out), naccept, nreject, proposed
    return torch.stack(out), naccept, nreject


def sens_rhs(rhs, p, G, normalizer="softsign"):
    """F([u; S]) = [f(u); J S_k + ∂f/∂p_k] through the native RHS and VJP (J symmetric)."""
    nx = rhs.nx
    dev = p.device
    g = torch.as_tensor(kanode.linrange_f32(-1.0, 1.0, G).astype(np.float64), device=dev)
    invh = float(np.float32(1.0) / np.float32(2.0 / (G - 1)))

    def norm(u):
        return u / (1.0 + u.abs()) if normalizer == "softsign" else torch.tanh(u)

    def dfdp(u):   # ∂φ(u)/∂C_k = B_k(N(u)), ∂φ/∂W = swish(u): [P, nx]
        basis = torch.exp(-((norm(u)[None, :] - g[:, None]) * invh) ** 2)
        return torch.cat([basis, (u * torch.sigmoid(u))[None, :]], 0)

    def F(z):
        u, S = z[0:1], z[1:]
        du = rhs.rhs(u.contiguous(), p)
        jS, _ = rhs.vjp(u.expand(S.shape[0], nx).contiguous(), p, S.contiguous())
        return torch.cat([du, jS + dfdp(u[0])], 0)
    return F


def _problem(name):
    import anchors
    pr = anchors.source_problem(name)
    dev = torch.device("cuda:0")
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
    rhs = kanode.FisherKPPRHS(kan1, nx=pr["nx"], dx=pr["dx"], D=pr["D"], device=dev)
    return pr, rhs, dev


@pytest.mark.parametrize("name,tol", [("fk", 1e-3), ("fk", 1e-7), ("ac", 1e-3)])
def test_native_forward_sensitivities_match_dual_solve_restatement(name, tol):
    """Three checks.  (1) Replay: the restatement takes the kernel's accepted step sizes; values and sensitivities
    agree to rounding (values 1e-10 of their scale, measured 1.9e-12, the rounding of ~250 RHS evaluations carried
    near the stability limit; each sensitivity 1e-9 of its own scale, measured up to 1.4e-10 on the smallest, ∂u/∂p_9
    at 1.4e-3), and after every step the restatement's controller (its Dual error norm, PI control)
    proposes the kernel's next step size to 1e-5 (the first proposal carries the embedded error's cancellation at a
    tiny first step: measured 2.9e-7, the rest ~1e-11): this pins the norm semantics, since a per-value norm
    (without the partials) moves the proposals by ~10%.  (2) The restatement on its own step sequence takes the same
    accepted / rejected counts at the default tolerances; near Tsit5's stability limit (the Laplacian at dx = 0.04)
    the PI controller amplifies rounding-level step differences, so its results are held at 1e-6 of the scale
    (measured ~1e-9 on the CPU between two restatements), and at tol = 1e-7 (~100 steps) a decision can flip, so the
    counts are held within 2.  (3) The C port (oracle/cpu_epoch.c kref_fk_fsens_solve_f64, dense Laplacian) the
    same."""
    pr, rhs, dev = _problem(name)
    import bench
    rng = np.random.default_rng(3)
    p = torch.as_tensor(bench.fk_trained_like_params() + rng.normal(0.0, 0.05, 11), device=dev)
    if name == "ac":   # the Allen-Cahn source's scale: a random KAN of its size (Nx = 41: no table, odd Nx)
        p = torch.as_tensor(rng.normal(0.0, 0.5, 11), device=dev)
    u0 = torch.as_tensor(pr["u0"][None, :], device=dev)
    opt = kanode.Tsit5Options(abstol=tol * 1e-3, reltol=tol)
    assert rhs.hd.forward_sensitivity_supported(1)
    u_n, S_n, st = rhs.hd.forward_sensitivity_tsit5(p, u0, *pr["tspan"], pr["saveat"], opt.to_c())
    ts_n, dts_n = rhs.hd.forward_sensitivity_step_sizes()
    assert len(dts_n) == st["naccept"]
    z0 = torch.cat([u0, torch.zeros(11, pr["nx"], dtype=u0.dtype, device=dev)], 0)
    F = sens_rhs(rhs, p, 10)
    uscale = max(1.0, u_n.abs().max().item())
    # (1) replay
    with torch.no_grad():
        zr, na, _, proposed = dual_tsit5(F, z0, *pr["tspan"], pr["saveat"], opt, replay=dts_n)
    assert na == st["naccept"]
    assert (u_n - zr[:, 0:1]).abs().max().item() <= 1e-10 * uscale
    for k in range(11):
        sc = zr[:, 1 + k].abs().max().item()
        assert (S_n[:, k, 0] - zr[:, 1 + k]).abs().max().item() <= 1e-9 * max(sc, 1e-300), k
    if st["nreject"] == 0:   # the controller's proposals are the kernel's next steps (the last one is cut at tf)
        prop = np.asarray(proposed[:len(dts_n) - 1])
        assert np.max(np.abs(prop - dts_n[:-1]) / dts_n[:-1]) <= 1e-5
    # (2) the restatement on its own steps
    with torch.no_grad():
        zs, na, nr = dual_tsit5(F, z0, *pr["tspan"], pr["saveat"], opt)
    print(f"{name} tol {tol}: native {st} restatement naccept {na} nreject {nr}")
    if tol >= 1e-4:
        assert st["naccept"] == na and st["nreject"] == nr
        assert (u_n - zs[:, 0:1]).abs().max().item() <= 1e-6 * uscale
        for k in range(11):
            sc = zs[:, 1 + k].abs().max().item()
            assert (S_n[:, k, 0] - zs[:, 1 + k]).abs().max().item() <= 1e-6 * max(sc, 1e-300), k
    else:   # ~100 steps near the stability limit: an accept / reject can flip on rounding (measured 100 vs 99)
        assert abs(st["naccept"] - na) <= 2 and abs(st["nreject"] - nr) <= 2
    # (3) the C port of the same Dual solve
    from oracle import oracle as O
    uc, sc_, stc, _ = O.fk_fsens_solve(O.LayerSpec(1, 1, 10, "softsign"), p.cpu().numpy(), pr["D"], pr["dx"],
                                       pr["u0"][None, :], pr["tspan"][1], pr["saveat"], abstol=tol * 1e-3, reltol=tol)
    if tol >= 1e-4:
        assert stc["naccept"] == st["naccept"] and stc["nreject"] == st["nreject"]
        assert np.abs(uc - u_n.cpu().numpy()).max() <= 1e-6 * uscale
    else:
        assert abs(stc["naccept"] - st["naccept"]) <= 2


def test_trainer_picks_forward_mode_at_the_reference_size_and_adjoint_beyond():
    """SciMLSensitivity's automatic rule: forward mode where length(u0) + length(p) <= 100 (FK26: 37), the adjoint
    beyond it (FK256: 267); NeuralODE chains always take the InterpolatingAdjoint."""
    pr, rhs, dev = _problem("fk")
    import bench
    p = torch.as_tensor(bench.fk_trained_like_params(), device=dev)
    u0 = torch.as_tensor(pr["u0"][None, :], device=dev)
    X = torch.as_tensor(np.random.default_rng(4).uniform(0.0, 1.0, (len(pr["saveat"]), 1, pr["nx"])), device=dev)
    tr = kanode.Trainer(rhs, u0, pr["tspan"], pr["saveat"], X, p, eta=1e-2)
    assert tr.sensealg == "auto"
    loss, g, sol = tr.loss_and_grad()
    assert sol.stats.get("sensealg") == "forward"
    # the same gradient through solve(sensealg="forward") + autograd (the non-fast path)
    pg = p.clone().requires_grad_(True)
    s2 = kanode.solve(rhs, u0, pr["tspan"], pg, pr["saveat"], kanode.Tsit5Options(), sensealg="forward")
    (g2,) = torch.autograd.grad(((s2.u - X) ** 2).mean(), [pg])
    assert (g - g2).abs().max().item() <= 1e-13 * g.abs().max().item()
    # 256 points: the adjoint
    nx = 256
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
    big = kanode.FisherKPPRHS(kan1, nx=nx, dx=1.0 / (nx - 1), D=0.01, device=dev)
    ub = torch.as_tensor(np.sin(np.pi * np.arange(nx) / (nx - 1))[None, :] * 0.5, device=dev)
    Xb = torch.zeros((3, 1, nx), dtype=torch.float64, device=dev)
    trb = kanode.Trainer(big, ub, (0.0, 0.1), [0.0, 0.05, 0.1], Xb, p, eta=1e-2)
    _, _, solb = trb.loss_and_grad()
    assert "sensealg" not in solb.stats and "adjoint" in solb.stats
    # a NeuralODE chain stays on the adjoint
    chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
    assert kanode.Trainer(kanode.ChainRHS(chain, device=dev), torch.ones((1, 2), dtype=torch.float64, device=dev),
                          (0.0, 1.0), [0.0, 1.0], torch.zeros((2, 1, 2), dtype=torch.float64, device=dev),
                          torch.zeros(240, dtype=torch.float64, device=dev)).sensealg == "interpolating_adjoint"


def test_forward_sensitivity_rejects_uncovered_shapes():
    dev = torch.device("cuda:0")
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
    rhs = kanode.FisherKPPRHS(kan1, nx=256, dx=1.0 / 255, D=0.01, device=dev)
    assert not rhs.hd.forward_sensitivity_supported(1)
    p = torch.zeros(11, dtype=torch.float64, device=dev)
    u0 = torch.zeros((1, 256), dtype=torch.float64, device=dev)
    with pytest.raises(kanode.KanodeError, match="forward sensitivities"):
        rhs.hd.forward_sensitivity_tsit5(p, u0, 0.0, 1.0, [0.0, 1.0], kanode.Tsit5Options().to_c())
    small = kanode.FisherKPPRHS(kan1, nx=26, dx=0.04, D=0.01, device=dev)
    assert small.hd.forward_sensitivity_supported(2) and not small.hd.forward_sensitivity_supported(3)
