#!/usr/bin/env python3
"""The reference's recorded training outcomes, reproduced through the product path.

These are the only numbers /root/reference holds for the KAN-ODE path, so they are the end-to-end
anchors of this build:

  fk  Fisher-KPP source learning (PDE examples/Fisher-KPP_Source.jl:33-109,163-213): Nx = 26
      (dx = 0.04 on [0, 1]), D = 0.01, IC :47-49, ground truth rc_ode (:62-71) with the dense periodic
      Laplacian (:55-59) solved by Tsit5 at the default tolerances with saveat 0.5 over (0, 5);
      KAN [1, 1] G = 10 softsign rbf; loss mean(abs2, X - pred) (:107-109); ADAM(1e-2) (:167) for
      N_iter = 2e4 (:170).  Recorded outcome: the symbolic fit of the learned source
      x*(1.0024477071121443 - x)*0.9953110353893396 (:234) on u in 0:0.05:1 (:237).
  ac  Allen-Cahn source learning (PDE examples/Allen-Cahn_Source.jl:33-104,157-207): x = -1:0.05:1
      (41 points), u0 = x^2 cos(pi x), -1e-4*lap*u + (-5u^3 + 5u), tspan (0, 1), saveat 0.01, ADAM(1e-2),
      N_iter = 5e4 (:164).  Recorded: 5.675949973338312e-5 - (x^3 - x)*5.000357135982538 (:227) on
      u in -1:0.05:1 (:230).
  lv  Lotka-Volterra KAN-ODE (Lotka-Volterra/LV_driver_KANODE.jl:110-305): u0 = [1, 1], p_ = [1.5, 1, 1, 3],
      truth at abstol = reltol = 1e-12 with saveat 0.1 over (0, 14), the first 35 points for training;
      KAN [2, 10, 2] G = 5 tanh_fast (P = 240), p = Glorot / 1e5 (:175), Adam(5e-4) (:219), N_iter = 1e5
      (:221), loss_train / loss_test after every update (:290-291).  Recorded: converged loss 8.3e-7 at
      240 parameters (Lotka-Volterra/trend_plotter.py:7-8).

Every gradient is the product path: the native Tsit5 solve (kanode_solve_tsit5), the InterpolatingAdjoint
(kanode_adjoint_tsit5; the reference's default sensealg for NeuralODE, and what SciMLSensitivity picks for
the hand-written ODEProblem at larger sizes; at Nx = 26 it would pick ForwardDiffSensitivity, which gives
the same gradient up to the solver tolerance) and one FusedAdam launch per iteration (kanode.Trainer).
The ground-truth data is generated on the host with the same Tsit5 statement (kanode.ode, Python loop)
over the true right-hand side, as the reference generates it with Tsit5.

Not reproduced: Julia's RNG stream (the Glorot initial parameters differ), so converged outcomes are
compared, not trajectories; the reference keeps FK / AC parameters in Float32 (ComponentArray of the
Float32 Glorot init, Fisher-KPP_Source.jl:90,166), this run trains them in Float64.

Usage: python tools/anchors.py {fk,ac,lv} [--iters N] [--out DIR]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kan-odes_amd"))

import kanode  # noqa: E402


# ---------------------------------------------------------------- problem statements (host side)
def periodic_laplacian(nx: int, dx: float) -> np.ndarray:
    """Fisher-KPP_Source.jl:55-59 / Allen-Cahn_Source.jl:50-54."""
    return kanode.fisher_kpp_laplacian(nx, dx)


def source_problem(name: str) -> dict:
    """Grid, IC, coefficient, true source, training saveat and recorded symbolic fit of the two
    source-learning drivers."""
    if name == "fk":
        dx, X, T = 0.04, 1.0, 5.0
        nx = int(round(X / dx)) + 1                                   # Nx = Int64(X/dx+1) = 26
        x = np.arange(nx) * dx                                        # collect(0:dx:X)
        amp, delta = 1.0, 0.2
        u0 = amp * (np.tanh((x - (0.5 - delta / 2)) / (delta / 10)) - np.tanh((x - (0.5 + delta / 2)) / (delta / 10))) / 2
        return dict(name="fisher_kpp_source", ref="PDE examples/Fisher-KPP_Source.jl", nx=nx, dx=dx, D=0.01,
                    u0=u0, tspan=(0.0, T), saveat=[0.5 * i for i in range(11)], eta=1e-2, iters=20000,
                    reaction=lambda u: 1.0 * u * (1.0 - u),
                    fitted=lambda r: r * (1.0024477071121443 - r) * 0.9953110353893396,
                    fitted_text="x*(1.0024477071121443-x)*0.9953110353893396 (Fisher-KPP_Source.jl:234)",
                    rho=np.round(np.arange(21) * 0.05, 12))
    if name == "ac":
        dx = 0.05
        x = -1.0 + np.arange(41) * dx                                 # collect(-1:0.05:1)
        u0 = x ** 2 * np.cos(np.pi * x)
        return dict(name="allen_cahn_source", ref="PDE examples/Allen-Cahn_Source.jl", nx=41, dx=dx, D=-1e-4,
                    u0=u0, tspan=(0.0, 1.0), saveat=[0.01 * i for i in range(101)], eta=1e-2, iters=50000,
                    reaction=lambda u: -5.0 * u ** 3 + 5.0 * u,
                    fitted=lambda r: 5.675949973338312e-5 - (r * (r * r) - r) * 5.000357135982538,
                    fitted_text="5.675949973338312e-5 - (x^3 - x)*5.000357135982538 (Allen-Cahn_Source.jl:227)",
                    rho=np.round(-1.0 + np.arange(41) * 0.05, 12))
    raise ValueError(name)


def source_truth(pr: dict) -> np.ndarray:
    """X_n: solve(ODEProblem(rc_ode, u0, tspan, saveat = dt), Tsit5()) at the default tolerances
    (Fisher-KPP_Source.jl:62-71), on the host with kanode.ode's Tsit5 statement; (len(saveat), 1, Nx)."""
    lapT = torch.as_tensor(periodic_laplacian(pr["nx"], pr["dx"]).T.copy())
    D, reaction = pr["D"], pr["reaction"]

    def rc_ode(u, p, t):
        return D * (u @ lapT) + reaction(u)

    u0 = torch.as_tensor(pr["u0"], dtype=torch.float64).reshape(1, -1)
    sol = kanode.solve(rc_ode, u0, pr["tspan"], torch.zeros(1, dtype=torch.float64), pr["saveat"],
                       kanode.Tsit5Options(native=False))
    return sol.u.numpy()


def lv_truth() -> tuple[np.ndarray, list, list]:
    """LV_driver_KANODE.jl:110-127: the Lotka-Volterra truth at 1e-12 tolerances (scipy DOP853 here),
    saveat 0.1 over (0, 14); the first 35 samples are the training cut."""
    from scipy.integrate import solve_ivp
    t = [0.1 * i for i in range(141)]
    a, b, g, d = 1.5, 1.0, 1.0, 3.0
    f = lambda _t, x: [a * x[0] - b * x[1] * x[0], g * x[0] * x[1] - d * x[1]]   # noqa: E731
    X = solve_ivp(f, (0.0, 14.0), [1.0, 1.0], t_eval=t, method="DOP853", rtol=1e-12, atol=1e-12).y.T
    return X[:, None, :], t[:35], t


# ---------------------------------------------------------------- training runs (product path)
def _progress(msg: str) -> None:
    print(msg, flush=True)


def run_source(which: str, iters: int | None = None, seed: int = 0, log_every: int = 100, dev="cuda:0",
               loss_every: int = 0, out_path: str | None = None, max_seconds: float = 0.0,
               sensealg: str | None = None) -> dict:
    dev = torch.device(dev)
    pr = source_problem(which)
    iters = int(iters or pr["iters"])
    Xn = torch.as_tensor(source_truth(pr), device=dev)
    kan = kanode.KDense(1, 1, 10, normalizer="softsign", basis_func="rbf")
    chain = kanode.Chain(kan)
    rhs = kanode.FisherKPPRHS(chain, nx=pr["nx"], dx=pr["dx"], D=pr["D"], dtype=torch.float64, device=dev)
    p0 = torch.as_tensor(chain.setup(np.random.default_rng(seed))[0].astype(np.float64), device=dev)
    u0 = torch.as_tensor(pr["u0"], dtype=torch.float64, device=dev).reshape(1, -1)
    tr = kanode.Trainer(rhs, u0, pr["tspan"], pr["saveat"], Xn, p0, eta=pr["eta"], sensealg=sensealg)
    ev = kanode.ChainRHS(chain, device=dev)                       # kan1_.(ρgrid) through the C-ABI
    rho = torch.as_tensor(pr["rho"], dtype=torch.float64, device=dev).reshape(-1, 1)

    def learned(p):
        return ev.hd.layer_forward(0, p, rho).reshape(-1).cpu().numpy()

    def post_loss(p):
        with torch.no_grad():
            return float(kanode.mse_loss(kanode.solve(rhs, u0, pr["tspan"], p, pr["saveat"]).u, Xn))

    fit_rho = pr["fitted"](pr["rho"])
    curve = [(0, post_loss(tr.p))]
    dev_curve = [(0, float(np.max(np.abs(learned(tr.p) - fit_rho))))]   # max |kan1_(ρ) - recorded fit| per log point
    t0 = time.perf_counter()
    last = t0
    done = 0
    for i in range(1, iters + 1):
        tr.step()
        done = i
        if i % log_every == 0 or i == iters:
            curve.append((i, post_loss(tr.p)))           # l[end] = loss(p) after update! (:204)
            dev_curve.append((i, float(np.max(np.abs(learned(tr.p) - fit_rho)))))
            now = time.perf_counter()
            if now - last > 30 or i == iters:
                _progress(f"{pr['name']}: iteration {i}/{iters} loss {curve[-1][1]:.4e} ({now - t0:.0f} s)")
                last = now
            if max_seconds and now - t0 > max_seconds:    # time budget of the GPU call: stop at a log point
                _progress(f"{pr['name']}: stopping at iteration {i} (time budget {max_seconds:.0f} s)")
                break
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    lr = learned(tr.p)
    fit = pr["fitted"](pr["rho"])
    true = pr["reaction"](pr["rho"])
    scale = float(np.max(np.abs(fit)))
    _, _, sol = tr.loss_and_grad()
    out = {
        "anchor": pr["name"], "reference": pr["ref"], "iters": done, "iters_requested": iters, "eta": pr["eta"],
        "seed": seed,
        "nx": pr["nx"], "dx": pr["dx"], "D": pr["D"], "tspan": list(pr["tspan"]), "n_saveat": len(pr["saveat"]),
        "wall_s": wall, "ms_per_iteration": wall / max(done, 1) * 1e3,
        "what": "Trainer.step per iteration (native Tsit5 + the reference's automatic sensealg: ForwardDiffSensitivity "
                "at these sizes, else InterpolatingAdjoint; FusedAdam); wall_s includes the logged loss, a forward "
                "solve after the update every log_every iterations",
        "sensealg": sol.stats.get("sensealg", "interpolating_adjoint"),
        "log_every": log_every,
        "loss_initial": curve[0][1], "loss_final": curve[-1][1], "loss_min": min(l for _, l in curve),
        "loss_curve": curve,
        "dev_curve": dev_curve,
        "first_iter_within_0.01": next((i for i, d in dev_curve if d <= 0.01), None),
        "first_iter_within_0.005": next((i for i, d in dev_curve if d <= 0.005), None),
        "forward_steps": sol.stats["naccept"],
        "adjoint_steps": sol.stats["adjoint"]["naccept"] if "adjoint" in sol.stats else None,
        "rho": pr["rho"].tolist(), "learned_source": lr.tolist(),
        "recorded_fit": pr["fitted_text"], "recorded_fit_values": fit.tolist(),
        "max_abs_dev_from_recorded_fit": float(np.max(np.abs(lr - fit))),
        "max_rel_dev_from_recorded_fit": float(np.max(np.abs(lr - fit)) / scale),
        "max_abs_dev_from_true_source": float(np.max(np.abs(lr - true))),
        "recorded_fit_vs_true_source": float(np.max(np.abs(fit - true))),
        "p_final": tr.p.cpu().numpy().tolist(),
    }
    if out_path:
        with open(out_path, "w") as f:
            json.dump(out, f, indent=1)
    return out


def run_lv(iters: int | None = None, seed: int = 0, log_every: int = 100, dev="cuda:0",
           out_path: str | None = None) -> dict:
    dev = torch.device(dev)
    iters = int(iters or 100000)
    X, t_train, t_all = lv_truth()
    Xall = torch.as_tensor(X, device=dev)
    Xtr = Xall[:35].contiguous()
    chain = kanode.Chain(kanode.KDense(2, 10, 5, normalizer="tanh_fast"), kanode.KDense(10, 2, 5, normalizer="tanh_fast"))
    rhs = kanode.ChainRHS(chain, device=dev)
    p0 = torch.as_tensor(chain.setup(np.random.default_rng(seed))[0].astype(np.float64) / 1e5, device=dev)
    u0 = torch.tensor([[1.0, 1.0]], dtype=torch.float64, device=dev)
    tr = kanode.Trainer(rhs, u0, (0.0, 3.5), t_train, Xtr, p0, eta=5e-4, sensealg="interpolating_adjoint")

    def losses(p):
        with torch.no_grad():
            ltr = float(kanode.mse_loss(kanode.solve(rhs, u0, (0.0, 3.5), p, t_train).u, Xtr))
            lte = float(kanode.mse_loss(kanode.solve(rhs, u0, (0.0, 14.0), p, t_all).u, Xall))
        return ltr, lte

    curve = [(0,) + losses(tr.p)]
    t0 = time.perf_counter()
    last = t0
    for i in range(1, iters + 1):
        tr.step()
        if i % log_every == 0 or i == iters:
            curve.append((i,) + losses(tr.p))          # loss_train / loss_test after update! (:290-291)
            now = time.perf_counter()
            if now - last > 30 or i == iters:
                _progress(f"lv: iteration {i}/{iters} train {curve[-1][1]:.3e} test {curve[-1][2]:.3e} ({now - t0:.0f} s)")
                last = now
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    out = {
        "anchor": "lotka_volterra_kanode", "reference": "Lotka-Volterra/LV_driver_KANODE.jl", "iters": iters,
        "eta": 5e-4, "seed": seed, "P": int(p0.numel()), "wall_s": wall, "ms_per_iteration": wall / iters * 1e3,
        "log_every": log_every,
        "loss_train_initial": curve[0][1], "loss_train_final": curve[-1][1],
        "loss_train_min": min(c[1] for c in curve), "loss_test_final": curve[-1][2],
        "loss_test_min": min(c[2] for c in curve),
        "recorded_converged_loss": 8.3e-7,
        "recorded_source": "Lotka-Volterra/trend_plotter.py:7-8 (kan_err 8.3e-7 at kan_size 240)",
        "loss_curve": curve, "p_final": tr.p.cpu().numpy().tolist(),
    }
    if out_path:
        with open(out_path, "w") as f:
            json.dump(out, f, indent=1)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("problem", choices=["fk", "ac", "lv"])
    ap.add_argument("--iters", type=int, default=0, help="0: the reference driver's N_iter")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--log-every", type=int, default=100)
    ap.add_argument("--out", default="gpurun_out/anchors")
    ap.add_argument("--max-seconds", type=float, default=0.0, help="stop at the first log point past this")
    ap.add_argument("--sensealg", default=None, help="source problems: None = the reference's automatic choice")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    path = os.path.join(a.out, f"{a.problem}_seed{a.seed}.json")
    if a.problem == "lv":
        o = run_lv(a.iters or None, a.seed, a.log_every, out_path=path)
        print(json.dumps({k: o[k] for k in ("anchor", "iters", "ms_per_iteration", "loss_train_final",
                                            "loss_train_min", "loss_test_final", "recorded_converged_loss")}))
    else:
        o = run_source(a.problem, a.iters or None, a.seed, a.log_every, out_path=path, max_seconds=a.max_seconds,
                       sensealg=a.sensealg)
        print(json.dumps({k: o[k] for k in ("anchor", "iters", "ms_per_iteration", "loss_final",
                                            "max_abs_dev_from_recorded_fit", "max_abs_dev_from_true_source",
                                            "first_iter_within_0.01", "first_iter_within_0.005")}))


if __name__ == "__main__":
    main()
