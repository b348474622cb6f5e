"""Continuous adjoint for `solve`: SciMLSensitivity 7.69 InterpolatingAdjoint (§8f next #2).

The reference's gradients come from SciMLSensitivity: DiffEqFlux's NeuralODE passes
`InterpolatingAdjoint(autojacvec = ZygoteVJP())` (LV_driver_KANODE.jl:180), and the
automatic choice for a Fisher-KPP 256-point problem (N + P > 100, out-of-place) is the same
(third-party, not under /root/reference; restated from the published package — verify where
Julia exists).  The algorithm:

  * the forward solve keeps its dense output (Tsit5 steps and their 7 stage vectors);
  * the adjoint ODE  dλ/dt = -(∂f/∂u)ᵀλ,  dμ/dt = -(∂f/∂p)ᵀλ  runs from t_f to t_0 with
    Tsit5 on the augmented state [λ; μ] (written here in τ = t_f - t, where both right-hand
    sides change sign), u(t) taken from the forward interpolant;
  * at every saveat time the loss gradient ∂L/∂u(t_j) is added to λ (a PresetTimeCallback,
    so the steps land on those times and FSAL is re-evaluated after each jump);
  * same abstol / reltol as the forward solve; error norm = RMS over all of [λ; μ];
  * result: dL/du0 = λ(t_0), dL/dp = μ(t_0).

Each adjoint RHS evaluation is one kanode_vjp_stage call: the kernel forms the interpolated
forward state u_n + dt_n Σ_i b_i(θ) k_i and the adjoint stage input λ + h Σ_j a_sj kλ_j in
place, returns λᵀ∂f/∂u and λᵀ∂f/∂p, and on the last stage the λ part of the error norm.
"""
from __future__ import annotations

import bisect
import math

import torch

from .ode import A, BTILDE, C as CNODE, Solution, Tsit5Options, interp_weights


class DenseRecord:
    """Accepted forward steps: t_n, dt_n, u_n and the 7 stage vectors of each."""

    def __init__(self):
        self.t, self.dt, self.u, self.k = [], [], [], []

    def add(self, t, dt, u, ks):
        self.t.append(t)
        self.dt.append(dt)
        self.u.append(u)
        self.k.append(ks)

    def locate(self, t: float):
        """(u_n, [k_1..k_7], [dt_n b_i(θ)]) with t = t_n + θ dt_n."""
        n = max(0, min(len(self.t) - 1, bisect.bisect_right(self.t, t) - 1))
        dt = self.dt[n]
        theta = min(1.0, max(0.0, (t - self.t[n]) / dt))
        return self.u[n], self.k[n], [dt * w for w in interp_weights(theta)]


def _adj_rhs(f, p, rec: DenseRecord, tf, tau, lam, lks, lc, lam_out=None, error=None):
    u, ks, c = rec.locate(tf - tau)
    return f.vjp_stage(u, p, ks, c, lam, lks, lc, lam_out, error)


def _rms2(x):
    return float((x.double() * x.double()).sum())


def _gsum(f, *vals: float) -> float:
    """Σ of the given local sums over the shards of a grid-sharded RHS (kanode.tp: f.reduce_sum,
    one scalar all-reduce), or their plain sum."""
    tot = float(sum(vals))
    red = getattr(f, "reduce_sum", None)
    return red(tot) if red is not None else tot


def interpolating_adjoint(f, p: torch.Tensor, rec: DenseRecord, tspan, saveat, grads, opt: Tsit5Options):
    """(dL/du0, dL/dp) for L with ∂L/∂u(saveat[j]) = grads[j] (tensors or None)."""
    t0, tf = float(tspan[0]), float(tspan[1])
    T = tf - t0
    eps = 1e-12 * max(1.0, abs(tf))
    jumps = {}
    for ts, g in zip(saveat, grads):
        if g is not None:
            jumps[ts] = g if ts not in jumps else jumps[ts] + g
    u_like = rec.u[0]
    lam = torch.zeros_like(u_like)
    mu = torch.zeros_like(p)
    if tf in jumps:
        lam = lam + jumps.pop(tf)
    # tstops in τ: the interior saveat times, then the end
    stops = sorted(tf - ts for ts in jumps if t0 + eps < ts < tf - eps) + [T]
    n_lam, n_mu = lam.numel(), mu.numel()
    ntot = _gsum(f, n_lam + n_mu)          # every shard's λ and μ entries (the norm is over all of them)

    def fz(tau, lam_):
        return _adj_rhs(f, p, rec, tf, tau, lam_, [], [])

    k1l, k1m = fz(0.0, lam)
    nf = 1
    # Hairer-Wanner initial step on the augmented state
    if opt.adaptive:
        sl = opt.abstol + lam.abs() * opt.reltol
        sm = opt.abstol + mu.abs() * opt.reltol
        d0 = math.sqrt(_gsum(f, _rms2(lam / sl), _rms2(mu / sm)) / ntot)
        d1 = math.sqrt(_gsum(f, _rms2(k1l / sl), _rms2(k1m / sm)) / ntot)
        h0 = 1e-6 if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
        h0 = min(h0, T)
        k2l, k2m = fz(h0, lam + h0 * k1l)
        nf += 1
        d2 = math.sqrt(_gsum(f, _rms2((k2l - k1l) / sl), _rms2((k2m - k1m) / sm)) / ntot) / h0
        mx = max(d1, d2)
        h1 = max(1e-6, h0 * 1e-3) if mx <= 1e-15 else (0.01 / mx) ** (1.0 / 5.0)
        h = min(100 * h0, h1, T)
    elif opt.replay_adjoint_dts is not None:
        h = float(opt.replay_adjoint_dts[0])
    else:
        h = opt.dt
    qold = opt.qoldinit
    tau = 0.0
    si = 0
    naccept = nreject = 0
    hs = []
    for _ in range(opt.maxiters):
        if tau >= T - 1e-14 * max(1.0, T):
            break
        if opt.replay_adjoint_dts is not None and not opt.adaptive:
            h = float(opt.replay_adjoint_dts[naccept])
        h = min(h, stops[si] - tau)
        kl, km = [k1l], [k1m]
        sumsq = None
        lam_new = None
        for i in range(6):
            lc = [h * a for a in A[i]]
            if i == 5:
                lam_new = torch.empty_like(lam)
                err = None
                if opt.adaptive:
                    sumsq = torch.empty(1, dtype=torch.float64, device=lam.device)
                    err = ([h * b for b in BTILDE], opt.abstol, opt.reltol, sumsq)
                l7, m7 = _adj_rhs(f, p, rec, tf, tau + h, lam, kl, lc, lam_new, err)
                kl.append(l7)
                km.append(m7)
            else:
                li, mi = _adj_rhs(f, p, rec, tf, tau + CNODE[i] * h, lam, kl, lc)
                kl.append(li)
                km.append(mi)
        nf += 6
        mu_new = mu + sum((h * a) * k for a, k in zip(A[5], km))
        if opt.adaptive:
            emu = sum((h * b) * k.double() for b, k in zip(BTILDE, km))        # norms in double
            skm = opt.abstol + torch.maximum(mu.abs(), mu_new.abs()).double() * opt.reltol
            red = getattr(f, "reduce_dev", None)
            if red is not None:     # grid shards: one device all-reduce of the step's error terms, one host read
                loc = sumsq.reshape(()) + ((emu / skm) ** 2).sum()
                EEst = math.sqrt(float(red(loc.reshape(1)).item()) / ntot)
            else:
                EEst = math.sqrt(_gsum(f, sumsq.item(), _rms2(emu / skm)) / ntot)
            q11 = EEst ** opt.beta1 if EEst > 0 else 0.0
            if EEst > 1.0 and h > opt.dtmin:
                nreject += 1
                h = h / min(1.0 / opt.qmin, q11 / opt.gamma)
                continue
            q = q11 / (qold ** opt.beta2)
            q = max(1.0 / opt.qmax, min(1.0 / opt.qmin, q / opt.gamma))
            hnew = h / q if q > 0 else h * opt.qmax
            qold = max(EEst, opt.qoldinit)
        else:
            hnew = h
        tau = tau + h
        lam, mu = lam_new, mu_new
        k1l, k1m = kl[6], km[6]
        hs.append(h)
        naccept += 1
        if abs(tau - stops[si]) <= 1e-12 * max(1.0, T):
            tau = stops[si]
            ts = tf - tau
            key = min(jumps, key=lambda s: abs(s - ts)) if jumps else None
            if key is not None and abs(key - ts) <= eps and si < len(stops) - 1:
                lam = lam + jumps.pop(key)                   # callback: λ += ∂L/∂u(t_j)
                k1l, k1m = fz(tau, lam)                      # u_modified!: FSAL re-evaluated
                nf += 1
            si = min(si + 1, len(stops) - 1)
        h = hnew
    else:
        raise RuntimeError("adjoint Tsit5: maxiters reached")
    for ts in list(jumps):                                   # a saveat at t0 adds to dL/du0 only
        if abs(ts - t0) <= eps:
            lam = lam + jumps.pop(ts)
    return lam, mu, dict(naccept=naccept, nreject=nreject, nf=nf, dts=hs)


class _InterpAdjointSolve(torch.autograd.Function):
    """solve(...) whose backward is the InterpolatingAdjoint (forward dense output kept)."""

    @staticmethod
    def forward(ctx, f, tspan, saveat, opt, stats, p, u0):
        from .ode import solve
        rec = DenseRecord()
        with torch.no_grad():
            sol = solve(f, u0, tspan, p, saveat, opt, dense_record=rec)
        ctx.f, ctx.rec, ctx.tspan, ctx.saveat, ctx.opt, ctx.stats = f, rec, tspan, sol.t, opt, stats
        ctx.save_for_backward(p)
        stats.update(sol.stats)
        stats["dts"] = [float(x) for x in rec.dt]
        return sol.u

    @staticmethod
    def backward(ctx, g):
        (p,) = ctx.saved_tensors
        grads = [g[j] if g is not None else None for j in range(len(ctx.saveat))]
        du0, dp, st = interpolating_adjoint(ctx.f, p.detach(), ctx.rec, ctx.tspan, ctx.saveat, grads, ctx.opt)
        ctx.stats["adjoint"] = st
        ctx.rec = None
        return None, None, None, None, None, dp, du0


def solve_interpolating_adjoint(f, u0, tspan, p, saveat, opt: Tsit5Options) -> Solution:
    stats = {}
    u = _InterpAdjointSolve.apply(f, tspan, saveat, opt, stats, p, u0)
    t0, tf = float(tspan[0]), float(tspan[1])
    ts = list(saveat) if saveat is not None else [t0, tf]
    return Solution(ts[:u.shape[0]], u, stats)


class _NativeAdjointSolve(torch.autograd.Function):
    """kanode_solve_tsit5 keeping its dense output; backward = kanode_adjoint_tsit5 (both native)."""

    @staticmethod
    def forward(ctx, hd, tspan, saveat, opt, stats, p, u0):
        oc = opt.to_c()
        u_save, st, dense = hd.solve_tsit5(p.detach().contiguous(), u0.detach().contiguous(), float(tspan[0]),
                                           float(tspan[1]), saveat, oc, keep_dense=True)
        ctx.hd, ctx.dense, ctx.oc, ctx.stats, ctx.u_shape = hd, dense, oc, stats, tuple(u0.shape)
        ctx.save_for_backward(p)
        stats.update(st)
        stats["dts"] = dense.step_sizes()[1].tolist()   # accepted step sizes (the solve's host copy)
        return u_save

    @staticmethod
    def backward(ctx, g):
        (p,) = ctx.saved_tensors
        du0, dp, st = ctx.hd.adjoint_tsit5(p.detach().contiguous(), ctx.dense, g.contiguous(), ctx.oc, ctx.u_shape)
        if ctx.hd.get_option("record_adjoint_steps"):
            st["dts"] = ctx.hd.adjoint_step_sizes().tolist()
        ctx.stats["adjoint"] = st
        ctx.hd.release_dense(ctx.dense)
        ctx.dense = None
        return None, None, None, None, None, dp, du0


def native_forward_dense(f, u0, tspan, p, saveat, opt: Tsit5Options):
    """The forward half of native_mse_gradient: (u_save, stats, DenseOutput) with the dense output kept."""
    return f.hd.solve_tsit5(p.detach().contiguous(), u0.detach().contiguous(), float(tspan[0]), float(tspan[1]),
                            saveat, opt.to_c(), keep_dense=True)


def native_mse_gradient(f, u0, tspan, p, saveat, opt: Tsit5Options, target, pre=None):
    """(loss, dL/dp, Solution) for L = mse_loss(solve(...).u, target) through the native solve and
    InterpolatingAdjoint, without the autograd engine: the same two C calls as backward() of
    solve_native_interpolating_adjoint, with ∂L/∂u formed as mse_loss's backward does ((u - X)·2/numel).
    For Trainer's plain-MSE step (a handful of launches per iteration, where the engine's own overhead showed).
    pre: an earlier native_forward_dense of the same problem at the same p (its dense output is consumed)."""
    hd = f.hd
    oc = opt.to_c()
    pc = p.detach().contiguous()
    if pre is None:
        pre = native_forward_dense(f, u0, tspan, p, saveat, opt)
    u_save, st, dense = pre
    try:
        stats = dict(st)
        stats["dts"] = dense.step_sizes()[1].tolist()
        loss = torch.nn.functional.mse_loss(u_save, target)
        dl = (u_save - target).mul_(2.0 / u_save.numel())
        _, dp, ast = hd.adjoint_tsit5(pc, dense, dl, oc, tuple(u0.shape))
        if hd.get_option("record_adjoint_steps"):
            ast["dts"] = hd.adjoint_step_sizes().tolist()
        stats["adjoint"] = ast
    finally:
        hd.release_dense(dense)
    return loss, dp, Solution(list(saveat), u_save, stats)


def solve_native_interpolating_adjoint(f, u0, tspan, p, saveat, opt: Tsit5Options) -> Solution:
    stats = {}
    u = _NativeAdjointSolve.apply(f.hd, tspan, list(saveat), opt, stats, p, u0)
    return Solution(list(saveat), u, stats)


# ---- forward mode: SciMLSensitivity ForwardDiffSensitivity (the reference's automatic choice for small problems) ----

def forward_ok(f, u0: torch.Tensor, p) -> bool:
    """The sensealg SciMLSensitivity 7.69 picks automatically for a hand-written ODEProblem (Fisher-KPP_Source.jl:198,
    the Allen-Cahn source driver: no sensealg given) is ForwardDiffSensitivity when length(u0) + length(p) <= 100
    (third-party rule, restated).  True when that applies and the native forward-sensitivity solve
    covers the shape."""
    hd = getattr(f, "hd", None)
    if hd is None or not getattr(f, "auto_sensealg", False) or not isinstance(p, torch.Tensor) or not u0.is_cuda:
        return False
    if u0.numel() + p.numel() > 100:
        return False
    B = u0.shape[0] if u0.dim() == 2 else 1
    return hd.forward_sensitivity_supported(B)


def _contract(S: torch.Tensor, dl: torch.Tensor) -> torch.Tensor:
    """dL/dp_k = Σ_j Σ_i ∂L/∂u_i(t_j) S[j, k, i] (ForwardDiffSensitivity's pullback)."""
    n_save, P = S.shape[0], S.shape[1]
    return torch.bmm(S.reshape(n_save, P, -1), dl.reshape(n_save, -1, 1)).sum(0).reshape(P)


class _ForwardSensSolve(torch.autograd.Function):
    """kanode_forward_sensitivity_tsit5: the solve keeps ∂u(saveat)/∂p; backward contracts it with the cotangent."""

    @staticmethod
    def forward(ctx, hd, tspan, saveat, opt, stats, p, u0):
        u_save, S, st = hd.forward_sensitivity_tsit5(p.detach().contiguous(), u0.detach().contiguous(),
                                                     float(tspan[0]), float(tspan[1]), saveat, opt.to_c())
        ctx.S = S
        stats.update(st)
        return u_save

    @staticmethod
    def backward(ctx, g):
        dp = _contract(ctx.S, g.contiguous())
        ctx.S = None
        return None, None, None, None, None, dp, None


def solve_forward_sensitivity(f, u0, tspan, p, saveat, opt: Tsit5Options) -> Solution:
    if u0.requires_grad:
        raise ValueError("sensealg='forward' differentiates with respect to p only (ForwardDiffSensitivity over p)")
    stats = {}
    u = _ForwardSensSolve.apply(f.hd, tspan, list(saveat), opt, stats, p, u0)
    return Solution(list(saveat), u, stats)


def native_forward_sens(f, u0, tspan, p, saveat, opt: Tsit5Options):
    """The solve of native_mse_gradient_forward: (u_save, S, stats)."""
    return f.hd.forward_sensitivity_tsit5(p.detach().contiguous(), u0.detach().contiguous(), float(tspan[0]),
                                          float(tspan[1]), saveat, opt.to_c())


def native_mse_gradient_forward(f, u0, tspan, p, saveat, opt: Tsit5Options, target, pre=None):
    """(loss, dL/dp, Solution) for L = mse_loss(solve(...).u, target) by ForwardDiffSensitivity: one native call
    (the solve with the sensitivities), then ∂L/∂u = (u - X)·2/numel contracted with them.  pre: an earlier
    native_forward_sens of the same problem at the same p."""
    u_save, S, st = pre if pre is not None else native_forward_sens(f, u0, tspan, p, saveat, opt)
    loss = torch.nn.functional.mse_loss(u_save, target)
    dl = (u_save - target).mul_(2.0 / u_save.numel())
    stats = dict(st)
    stats["sensealg"] = "forward"
    return loss, _contract(S, dl), Solution(list(saveat), u_save, stats)
