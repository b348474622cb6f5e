"""Device-resident Tsit5 integrator around the HIP RHS.

Restates OrdinaryDiffEqTsit5 1.1.0 / OrdinaryDiffEq 6.89 semantics (pinned at
Lotka-Volterra/Manifest.toml:1984,2162; third-party, not under /root/reference;
restated from the published package — verify where Julia exists):
  * Tsitouras 5(4) tableau, FSAL, 4th-order free dense output (Tsit5Interp);
  * error norm: RMS over ALL state entries of  utilde / (abstol + max(|u_prev|,|u|)·reltol)
    — a batched [N, B] state is ONE ODE with one step size, as in the reference
    (NeuralODE / ODEProblem on a matrix state);
  * PI step-size controller: beta1 = 7/(10·5), beta2 = 2/(5·5), gamma = 9/10,
    qmin = 1/5, qmax = 10, qoldinit = 1e-4, qsteady_min = qsteady_max = 1;
  * Hairer-Wanner initial step (ode_determine_initdt);
  * defaults abstol = 1e-6, reltol = 1e-3; saveat values from the dense interpolant.
Call sites the reference uses: LV_driver_KANODE.jl:122,180-184, Fisher-KPP_Source.jl:102-103.

Every RHS evaluation is one libkanode.so call (through the autograd Function),
so `solve(...)` is differentiable: backward runs the HIP VJP kernel once per
stage (discrete adjoint, ≡ reverse-mode AD through the solver steps).

RHS objects with a `stage` method (ChainRHS, FisherKPPRHS) take the fused path:
each stage is one kanode_rhs_stage call that forms u + dt·Σ a_sj k_j inside the
kernel, and the last stage also returns u_new and the embedded-error sum of
squares, so no stage broadcast or error pass runs as separate torch kernels.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from functools import lru_cache

import torch

# Tsitouras 5(4) coefficients (OrdinaryDiffEq tsit_tableaus.jl)
C = (0.161, 0.327, 0.9, 0.9800255409045097, 1.0, 1.0)
A = (
    (0.161,),
    (-0.008480655492356989, 0.335480655492357),
    (2.897153057105493, -6.359448489975075, 4.3622954328695815),
    (5.325864828439257, -11.748883564062828, 7.4955393428898365, -0.09249506636175525),
    (5.86145544294642, -12.92096931784711, 8.159367898576159, -0.071584973281401, -0.028269050394068383),
    (0.09646076681806523, 0.01, 0.4798896504144996, 1.379008574103742, -3.290069515436081, 2.324710524099774),
)
BTILDE = (-0.00178001105222577714, -0.0008164344596567469, 0.007880878010261995, -0.1447110071732629,
          0.5823571654525552, -0.45808210592918697, 0.015151515151515152)
# dense output b_i(θ) = Σ_m R[i][m] θ^(m+1)  (Tsit5Interp), i = 1..7
RI = (
    (1.0, -2.763706197274826, 2.9132554618219126, -1.0530884977290216),
    (0.0, 0.13169999999999998, -0.2234, 0.1017),
    (0.0, 3.9302962368947516, -5.941033872131505, 2.490627285651253),
    (0.0, -12.411077166933676, 30.33818863028232, -16.548102889244902),
    (0.0, 37.50931341651104, -88.1789048947664, 47.37952196281928),
    (0.0, -27.896526289197286, 65.09189467479366, -34.87065786149661),
    (0.0, 1.5, -4.0, 2.5),
)


def interp_weights(theta: float):
    return [sum(r * theta ** (m + 1) for m, r in enumerate(row)) for row in RI]


def rms(x: torch.Tensor) -> torch.Tensor:
    return torch.sqrt(torch.mean(x * x))


def _norm(f, x: torch.Tensor) -> float:
    """ODE_DEFAULT_NORM of x: RMS over every state entry.  A state sharded over ranks
    (kanode.tp) supplies f.reduce_dev / f.global_count, and the sum and count run over all shards
    (one device all-reduce, one host read)."""
    red = getattr(f, "reduce_dev", None)
    if red is None:
        return rms(x).item()
    x = x.detach().double()
    return math.sqrt(float(red((x * x).sum().reshape(1)).item()) / f.global_count(x.numel()))


_OPTS_C: dict = {}


@lru_cache(maxsize=64)
def _ascending(saveat: tuple) -> bool:
    return all(a <= b for a, b in zip(saveat, saveat[1:]))


@dataclass
class Tsit5Options:
    abstol: float = 1e-6
    reltol: float = 1e-3
    dt: float | None = None            # fixed step (adaptive=False) or initial step
    adaptive: bool = True
    maxiters: int = 100000
    dtmin: float = 0.0
    beta1: float = 7.0 / 50.0
    beta2: float = 2.0 / 25.0
    gamma: float = 0.9
    qmin: float = 0.2
    qmax: float = 10.0
    qoldinit: float = 1e-4
    fused: bool = True                 # use f.stage (kanode_rhs_stage) when the RHS has one
    native: bool = True                # run the loop in libkanode (kanode_solve_tsit5) when f is a kanode RHS
    control: str = "auto"              # native step control: "host", "device" (hipGraph replay) or "auto"
    graph_steps: int = 16              # step slots per graph replay (device control)
    # tests (Python driver, adaptive=False): take these accepted step sizes, in order, instead of a fixed dt --
    # another solver's step sequence replayed, so its arithmetic is compared on the same grid
    replay_dts: tuple | None = None
    replay_adjoint_dts: tuple | None = None

    def to_c(self):
        """A kanode_solver_options struct (a copy of one built per field values, which the caller may edit)."""
        key = (self.abstol, self.reltol, self.dt, self.adaptive, self.maxiters, self.dtmin, self.beta1, self.beta2,
               self.gamma, self.qmin, self.qmax, self.qoldinit, self.control, self.graph_steps)
        o = _OPTS_C.get(key)
        if o is None:
            if len(_OPTS_C) >= 64:
                _OPTS_C.clear()
            o = _OPTS_C[key] = self._to_c()
        return type(o).from_buffer_copy(o)

    def _to_c(self):
        from . import _lib as L
        o = L.SolverOptsC()
        L.lib().kanode_solver_options_default(ctypes.byref(o))
        o.abstol, o.reltol = float(self.abstol), float(self.reltol)
        o.dt = float(self.dt) if self.dt is not None else 0.0
        o.adaptive = 1 if self.adaptive else 0
        o.maxiters, o.dtmin = int(self.maxiters), float(self.dtmin)
        o.beta1, o.beta2, o.gamma = float(self.beta1), float(self.beta2), float(self.gamma)
        o.qmin, o.qmax, o.qoldinit = float(self.qmin), float(self.qmax), float(self.qoldinit)
        o.control = {"auto": 0, "host": 1, "device": 2}[self.control]
        o.graph_steps = int(self.graph_steps)
        return o


@dataclass
class Solution:
    t: list
    u: torch.Tensor                    # (len(saveat), *u0.shape)
    stats: dict = field(default_factory=dict)


def _initdt(f, u0, p, t0, tdist, opt: Tsit5Options, f0):
    """Hairer & Wanner initial step (OrdinaryDiffEq ode_determine_initdt, order 5)."""
    sk = opt.abstol + torch.abs(u0) * opt.reltol
    d0 = _norm(f, u0 / sk)
    d1 = _norm(f, f0 / sk)
    dt0 = 1e-6 if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
    dt0 = min(dt0, tdist)
    u1 = u0 + dt0 * f0
    f1 = f(u1, p, t0 + dt0)
    d2 = _norm(f, (f1 - f0) / sk) / dt0
    mx = max(d1, d2)
    dt1 = max(1e-6, dt0 * 1e-3) if mx <= 1e-15 else (0.01 / mx) ** (1.0 / 5.0)
    return min(100 * dt0, dt1, tdist)


def _step(f, u, p, t, dt, k1):
    ks = [k1]
    for i in range(6):
        acc = u
        for j, a in enumerate(A[i]):
            acc = acc + (dt * a) * ks[j]
        if i == 5:
            unew = acc
            ks.append(f(unew, p, t + dt))
        else:
            ks.append(f(acc, p, t + C[i] * dt))
    return unew, ks


def _step_fused(f, u, p, t, dt, k1, opt: Tsit5Options):
    """One Tsit5 step as six kanode_rhs_stage calls; returns (u_new, ks, EEst or None)."""
    ks = [k1]
    sumsq = None
    for i in range(6):
        c = [dt * a for a in A[i]]
        if i == 5:
            err = None
            if opt.adaptive:
                sumsq = torch.empty(1, dtype=torch.float64, device=u.device)
                err = ([dt * b for b in BTILDE], opt.abstol, opt.reltol, sumsq)
            k7, unew = f.stage(u, p, ks, c, want_y=True, error=err)
            ks.append(k7)
        else:
            ks.append(f.stage(u, p, ks, c)[0])
    eest = None
    if sumsq is not None:
        red = getattr(f, "reduce_dev", None)      # a grid-sharded RHS: Σ over the shards on the device
        eest = (math.sqrt(float(red(sumsq).item()) / f.global_count(u.numel())) if red is not None
                else math.sqrt(sumsq.item() / u.numel()))
    return unew, ks, eest


def _saveat_list(tspan, saveat) -> list:
    t0, tf = float(tspan[0]), float(tspan[1])
    if saveat is None:
        return [t0, tf]
    if isinstance(saveat, (int, float)):
        n = int(round((tf - t0) / saveat))
        return [t0 + i * saveat for i in range(n + 1)]
    return [float(s) for s in saveat]


def native_ok(f, u0: torch.Tensor, tspan, p, saveat: list, opt: Tsit5Options) -> bool:
    """solve() runs in libkanode (kanode_solve_tsit5 / kanode_adjoint_tsit5) for these arguments."""
    return (opt.native and hasattr(f, "hd") and isinstance(p, torch.Tensor) and u0.is_cuda and u0.dim() in (1, 2)
            and float(tspan[1]) > float(tspan[0]) and _ascending(tuple(saveat)))


def solve(f, u0: torch.Tensor, tspan, p: torch.Tensor, saveat=None, opt: Tsit5Options | None = None,
          sensealg: str = "discrete", dense_record=None) -> Solution:
    """solve(ODEProblem(f, u0, tspan, p), Tsit5(); saveat, abstol, reltol, sensealg) on device tensors.

    f(u, p, t) -> du (out-of-place, ODEFunction{false}); u0 any shape (e.g. (B, N)).
    Differentiable w.r.t. u0 and p when f is (kanode RHS objects are):
      sensealg="discrete"              reverse mode through every stage (discrete adjoint);
      sensealg="interpolating_adjoint" SciMLSensitivity's InterpolatingAdjoint, the reference's
                                       default (kanode.adjoint; f needs `vjp_stage`);
      sensealg="forward"               ForwardDiffSensitivity (gradient w.r.t. p; the native one-workgroup
                                       forward-sensitivity solve of a small Fisher-KPP field);
      sensealg="auto"                  SciMLSensitivity's automatic choice for a hand-written ODEProblem:
                                       "forward" where length(u0) + length(p) <= 100 and covered, else
                                       "interpolating_adjoint".
    dense_record: an adjoint.DenseRecord that receives every accepted step."""
    opt = opt or Tsit5Options()
    t0, tf = float(tspan[0]), float(tspan[1])
    saveat = _saveat_list(tspan, saveat)
    if sensealg not in ("discrete", "interpolating_adjoint", "forward", "auto"):
        raise ValueError(f"unknown sensealg {sensealg!r}")
    grad = torch.is_grad_enabled() and (getattr(p, "requires_grad", False) or u0.requires_grad)
    native = dense_record is None and native_ok(f, u0, tspan, p, saveat, opt)
    if native:
        tol = 1e-12 * max(1.0, abs(tf))
        saveat = [s for s in saveat if s <= tf + tol]
    if sensealg == "auto":   # SciMLSensitivity's automatic choice for a hand-written ODEProblem (adjoint.forward_ok)
        from .adjoint import forward_ok
        sensealg = "forward" if native and forward_ok(f, u0, p) else "interpolating_adjoint"
    if sensealg == "forward" and grad:
        from .adjoint import forward_ok, solve_forward_sensitivity
        hd = getattr(f, "hd", None)
        if not native or hd is None or not hd.forward_sensitivity_supported(u0.shape[0] if u0.dim() == 2 else 1):
            raise ValueError("sensealg='forward' needs the native forward-sensitivity solve (a small Fisher-KPP field, "
                             "kanode_forward_sensitivity_supported)")
        return solve_forward_sensitivity(f, u0, tspan, p, saveat, opt)
    if sensealg == "interpolating_adjoint" and grad:
        if native:
            from .adjoint import solve_native_interpolating_adjoint
            return solve_native_interpolating_adjoint(f, u0, tspan, p, saveat, opt)
        from .adjoint import solve_interpolating_adjoint
        return solve_interpolating_adjoint(f, u0, tspan, p, saveat, opt)
    if native and not grad:
        u_save, stats, _ = f.hd.solve_tsit5(p.detach().contiguous(), u0.detach().contiguous(), t0, tf, saveat,
                                            opt.to_c())
        return Solution(list(saveat), u_save, stats)
    out = []
    si = 0
    while si < len(saveat) and saveat[si] <= t0 + 1e-14 * max(1.0, abs(t0)):
        out.append(u0)
        si += 1
    t, u = t0, u0
    k1 = f(u, p, t)
    if opt.adaptive:
        dt = opt.dt if opt.dt is not None else _initdt(f, u0, p, t0, tf - t0, opt, k1)
    elif opt.replay_dts is not None:
        dt = float(opt.replay_dts[0])
    else:
        if opt.dt is None:
            raise ValueError("fixed-step Tsit5 needs opt.dt")
        dt = opt.dt
    qold = opt.qoldinit
    fused = opt.fused and hasattr(f, "stage") and u0.dim() == 2
    naccept = nreject = nf = 0
    for _ in range(opt.maxiters):
        if t >= tf - 1e-14 * max(1.0, abs(tf)):
            break
        if opt.replay_dts is not None and not opt.adaptive:
            dt = float(opt.replay_dts[naccept])
        dt = min(dt, tf - t)
        if fused:
            unew, ks, EEst = _step_fused(f, u, p, t, dt, k1, opt)
        else:
            unew, ks = _step(f, u, p, t, dt, k1)
        nf += 6
        if opt.adaptive:
            if not fused:
                utilde = dt * sum(b * k for b, k in zip(BTILDE, ks))
                sk = opt.abstol + torch.maximum(torch.abs(u), torch.abs(unew)) * opt.reltol
                EEst = _norm(f, utilde.detach() / sk.detach())
            q11 = EEst ** opt.beta1 if EEst > 0 else 0.0
            if EEst > 1.0 and dt > opt.dtmin:
                nreject += 1
                dt = dt / min(1.0 / opt.qmin, q11 / opt.gamma)
                continue
            q = q11 / (qold ** opt.beta2)
            q = max(1.0 / opt.qmax, min(1.0 / opt.qmin, q / opt.gamma))
            if 1.0 <= q <= 1.0:   # qsteady_min / qsteady_max
                q = 1.0
            dtnew = dt / q if q > 0 else dt * opt.qmax
            qold = max(EEst, opt.qoldinit)
        else:
            dtnew = dt
        # saveat points inside (t, t + dt] from the dense output
        tn = t + dt
        while si < len(saveat) and saveat[si] <= tn + 1e-12 * max(1.0, abs(tn)):
            ts = saveat[si]
            if abs(ts - tn) <= 1e-12 * max(1.0, abs(tn)):
                out.append(unew)
            else:
                w = interp_weights((ts - t) / dt)
                out.append(u + dt * sum(wi * k for wi, k in zip(w, ks)))
            si += 1
        if dense_record is not None:
            dense_record.add(t, dt, u, ks)
        t, u, k1 = tn, unew, ks[6]
        naccept += 1
        dt = dtnew
    else:
        raise RuntimeError("Tsit5: maxiters reached")
    return Solution(saveat[:len(out)], torch.stack(out), dict(naccept=naccept, nreject=nreject, nf=nf + 1))
