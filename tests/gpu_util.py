"""Helpers for the -m gpu parity tests (HIP path vs the CPU oracle)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

# Stated tolerances:
#   fp64: |gpu - oracle| <= 1e-13 * scale   (scale = Σ|terms| of that output, see below)
#   fp32: |gpu - oracle| <= 5e-6 * scale
RTOL = {torch.float64: 1e-13, torch.float32: 5e-6}


def device() -> torch.device:
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected (-m gpu) but no GPU is visible: the HIP path did not run")
    return torch.device("cuda:0")


def t(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device=device())


def specs_from_meta(meta):
    return [O.LayerSpec(l["in_dims"], l["out_dims"], l["grid_len"], l["normalizer"], l["basis"],
                        l["use_base_act"], tuple(l["grid_lims"]), None, l["iqf_reference_quirk"])
            for l in meta["layers"]]


def cfgs_from_specs(specs):
    from kanode import LayerCfg
    return [LayerCfg(s.in_dims, s.out_dims, s.grid_len, s.normalizer, s.basis, s.use_base_act,
                     tuple(s.grid_lims), None, s.iqf_reference_quirk) for s in specs]


def chain_scale(specs, p, u):
    """Per-output Σ|terms|: the chain evaluated with |C|, |W| and every basis value >= 0
    bounds the rounding-error scale of y (rbf/rswaf/iqf values are positive)."""
    ap = np.abs(p)
    y = O.chain_fwd(specs, ap, u)
    return np.abs(y) + np.max(np.abs(y)) * 1e-3


def assert_close(got, ref, scale, rtol, what=""):
    got = got.detach().cpu().numpy() if isinstance(got, torch.Tensor) else np.asarray(got)
    err = np.abs(got.astype(np.float64) - np.asarray(ref, np.float64))
    bound = rtol * np.broadcast_to(np.asarray(scale, np.float64), err.shape)
    worst = np.max(err / np.maximum(bound, 1e-300))
    assert worst <= 1.0, f"{what}: max err/bound = {worst:.3g} (max err {np.max(err):.3g})"


def fk_scale(p, D, dx, u):
    """Σ|terms| of du_i: |D lap| |u| + Σ_j |C_j| + |W||swish(u)|."""
    co = abs(D) / (dx * dx)
    lap = co * (np.abs(np.roll(u, 1, 1)) + 2 * np.abs(u) + np.abs(np.roll(u, -1, 1)))
    return lap + np.sum(np.abs(p[:-1])) + abs(p[-1]) * np.abs(u)
