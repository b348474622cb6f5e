"""The reference's recorded training outcomes, held as properties of three
initialisations rather than one trajectory's prefix.

The full runs are `tools/anchors.py` (`tools/gpu/r6_anchors.sh`), their JSONs under `profiles/r06/anchors/`.
Round 6, on the product path as it trains by default (Fisher-KPP: the reference's ForwardDiffSensitivity gradient;
Lotka-Volterra: the InterpolatingAdjoint):
  * Fisher-KPP source (Fisher-KPP_Source.jl:33-109,163-213; Nx = 26, KAN [1, 1] G = 10 softsign rbf, ADAM(1e-2),
    2e4 iterations): the learned kan1_(ρ) on ρ ∈ 0:0.05:1 (:237) against the recorded symbolic fit
    x*(1.0024477071121443-x)*0.9953110353893396 (:234): max deviation 0.050 (seed 0), 0.0048 (seed 1), 0.0067
    (seed 2); final loss 9.1e-5, 1.4e-7, 5.3e-7 from 2087, 10.1, 0.20.  Seed 0's initial W = 1.09 makes the first
    solve's source strongly positive (loss 2087); ADAM(1e-2) leaves that region with loss spikes (3.8e-2 at 10,000)
    and converges late: 0.087 at 18,000, 0.050 at 20,000.  After a rounding-level change of
    the forward-sensitivity kernel the same seed sat at 0.30 at 2e4 (loss 8.5e-3) and, run on, came within 0.01 of
    the fit from iteration 33,000 (0.0069 at 4e4, profiles/r06/anchors/fk_seed0_4e4.json): the seed's outcome at 2e4
    is a matter of when it leaves the plateau, so it is held to its loss drop only.
  * Lotka-Volterra (LV_driver_KANODE.jl:110-305; [2, 10, 2] G = 5, Adam(5e-4)): loss_train at 2e4 iterations
    4.9e-4, 3.3e-4, 4.4e-5 (seeds 0, 1, 2); at 1e5 the median over the last 2e4 iterations' log points is 1.3e-6,
    2.9e-6, 1.5e-6 against the recorded converged 8.3e-7 (trend_plotter.py:7-8).
The bars below hold every seed to a large drop of its loss, and the MEDIAN seed to the
recorded outcome, each with a margin of 1.5x or more over the recorded run: a rounding-level change of the path
moves these chaotic trajectories, so no single trajectory's prefix is pinned."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

_FK, _LV = {}, {}


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_fisher_kpp_source_training_seed(seed):
    import anchors
    out = anchors.run_source("fk", iters=20000, seed=seed, log_every=2000)
    _FK[seed] = out
    print(seed, {k: out[k] for k in ("loss_initial", "loss_final", "max_abs_dev_from_recorded_fit",
                                     "ms_per_iteration", "sensealg")})
    assert out["iters"] == 20000 and out["sensealg"] == "forward"
    assert np.all(np.isfinite(out["learned_source"]))
    assert out["loss_final"] <= 1e-4 * out["loss_initial"]
    assert out["max_abs_dev_from_recorded_fit"] <= 0.5       # (the source's peak is 0.25: a sanity bound)


def test_fisher_kpp_source_training_median_seed_follows_recorded_fit():
    if len(_FK) < 3:
        pytest.skip("needs the three seed runs above")
    devs = sorted(o["max_abs_dev_from_recorded_fit"] for o in _FK.values())
    losses = sorted(o["loss_final"] for o in _FK.values())
    print("deviations", devs, "final losses", losses)
    assert devs[1] <= 0.01          # the median seed: within 0.01 of the recorded fit everywhere on ρ ∈ 0:0.05:1
    assert losses[1] <= 1e-5


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_lotka_volterra_training_seed(seed):
    import anchors
    out = anchors.run_lv(iters=20000, seed=seed, log_every=5000)
    _LV[seed] = out
    print(seed, {k: out[k] for k in ("loss_train_initial", "loss_train_final", "ms_per_iteration")})
    assert out["loss_train_final"] <= 2e-3                      # recorded: <= 4.9e-4 at 2e4 (4x margin)
    assert out["loss_train_final"] <= 1e-3 * out["loss_train_initial"]


def test_lotka_volterra_training_best_seed():
    if len(_LV) < 3:
        pytest.skip("needs the three seed runs above")
    finals = sorted(o["loss_train_final"] for o in _LV.values())
    print("loss_train at 2e4", finals)
    assert finals[0] <= 1e-4                                   # recorded 4.4e-5 (seed 2)
    assert finals[1] <= 8e-4                                   # recorded median 3.3e-4


@pytest.mark.parametrize("tol", [1e-3, 1e-7])
def test_fisher_kpp_26_forward_sensitivity_gradient_matches_adjoint(tol):
    """at the reference's size (Nx = 26, one IC, Fisher-KPP_Source.jl:34-49,95-109) SciMLSensitivity
    7.69 picks forward-mode ForwardDiffSensitivity for `Zygote.gradient(loss, p)` (:198; 26 + 11 <= 100),
    which the Trainer now takes too (native kanode_forward_sensitivity_tsit5; tests/test_gpu_fsens.py pins it against
    the Dual-solve restatement).  The InterpolatingAdjoint is the other O(tol) approximation of the same derivative:
    at the default tolerances (abstol 1e-6, reltol 1e-3) the two agree to 10·reltol of the gradient's scale, and at
    tol = 1e-7 to 1e-5, i.e. the difference shrinks with the tolerance as a discretisation difference does, not a
    formula difference."""
    import torch
    import kanode
    import anchors
    pr = anchors.source_problem("fk")
    dev = torch.device("cuda:0")
    nx = pr["nx"]
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
    rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=pr["dx"], D=pr["D"], device=dev)
    import bench
    # a mid-training parameter set: the KAN fitted to the true source, perturbed
    p = torch.as_tensor(bench.fk_trained_like_params() + np.random.default_rng(3).normal(0.0, 0.05, 11), device=dev)
    u0 = torch.as_tensor(pr["u0"][None, :], device=dev)
    saveat = pr["saveat"]
    X = torch.as_tensor(np.random.default_rng(4).uniform(0.0, 1.0, (len(saveat), 1, nx)), device=dev)
    opt = kanode.Tsit5Options(abstol=tol * 1e-3, reltol=tol)
    grads = {}
    for sa in ("interpolating_adjoint", "forward"):
        pg = p.clone().requires_grad_(True)
        sol = kanode.solve(rhs, u0, pr["tspan"], pg, saveat, opt, sensealg=sa)
        (grads[sa],) = torch.autograd.grad(((sol.u - X) ** 2).mean(), [pg])
    g_adj, g_fwd = grads["interpolating_adjoint"], grads["forward"]
    scale = g_adj.abs().max().item()
    diff = (g_fwd - g_adj).abs().max().item()
    print(f"tol {tol}: max|g_fwd - g_adj| = {diff:.3e} of scale {scale:.3e} ({diff / scale:.2e})")
    assert diff <= (10 * tol if tol >= 1e-4 else 1e-5) * scale
