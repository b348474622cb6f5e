"""The reference's recorded Fisher-KPP training outcome, short form.

The full runs (2e4 iterations, three initialisations; Lotka-Volterra 1e5; Allen-Cahn) are
`tools/anchors.py`, their JSONs under `profiles/r04/anchors/`.  This test keeps the product training
path on that trajectory: Fisher-KPP_Source.jl:33-109,163-213 (Nx = 26, KAN [1, 1] G = 10 softsign rbf,
native Tsit5 + InterpolatingAdjoint + FusedAdam, ADAM(1e-2)) for 1,000 iterations from a fixed
initialisation.  The GPU path is deterministic (fixed-order reductions), so this is the first 1,000
iterations of profiles/r04/anchors/fk_seed1.json, whose loss there is 1.32e-4.

Bars: the loss falls from 10.1 below 1e-3 (recorded run: 1.3e-4 at this iteration, an 8x margin), and the
learned source kan1_(ρ) on ρ ∈ 0:0.05:1 (Fisher-KPP_Source.jl:237), compared with the reference's recorded
symbolic fit x*(1.0024477071121443-x)*0.9953110353893396 (:234), has its single maximum in the interior and
within 0.05 of the fit's 0.25, stays within 0.05 of the fit on ρ ∈ 0.1:0.05:0.7 (measured 0.03) and within
0.15 everywhere (measured 0.10, at ρ = 1: the ends converge later; the full run is within 0.004 at 2e4
iterations)"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_fisher_kpp_source_training_follows_recorded_fit():
    import anchors
    out = anchors.run_source("fk", iters=1000, seed=1, log_every=500)
    print({k: out[k] for k in ("loss_initial", "loss_final", "max_abs_dev_from_recorded_fit",
                               "ms_per_iteration", "forward_steps", "adjoint_steps")})
    print("learned", np.round(out["learned_source"], 4).tolist())
    print("recorded", np.round(out["recorded_fit_values"], 4).tolist())
    assert out["iters"] == 1000
    assert out["loss_initial"] > 1.0
    assert out["loss_final"] < 1e-3
    lr = np.asarray(out["learned_source"])
    fit = np.asarray(out["recorded_fit_values"])
    assert np.all(np.isfinite(lr))
    inner = slice(2, 15)                                   # ρ = 0.1 .. 0.7
    assert np.abs(lr[inner] - fit[inner]).max() < 0.05
    assert out["max_abs_dev_from_recorded_fit"] < 0.15
    assert abs(lr[0]) < 0.05
    assert 6 <= int(np.argmax(lr)) <= 14 and abs(lr.max() - fit.max()) < 0.05
