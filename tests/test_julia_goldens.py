"""The C oracle against golden outputs produced by the REAL reference stack (tools/julia_regen.jl:
the reference's KolmogorovArnold.jl + Lux + Zygote), when such files exist under
tests/golden/julia_out/.  Julia is absent from this image, so none exist here and these tests skip;
on a machine with Julia this turns the oracle's pinning from 'partial' into a direct check
(VERDICT r2 #9)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as O

OUT = os.path.join(GOLDEN, "julia_out")
FILES = sorted(f for f in os.listdir(OUT) if f.endswith(".mat")) if os.path.isdir(OUT) else []


def test_regen_recipe_is_present():
    root = os.path.dirname(GOLDEN)
    assert os.path.exists(os.path.join(root, "..", "tools", "julia_regen.jl"))
    assert os.path.exists(os.path.join(root, "..", "tools", "export_golden_for_julia.py"))


@pytest.mark.skipif(not FILES, reason="no Julia-generated goldens (Julia is not in this image)")
@pytest.mark.parametrize("name", FILES or ["-"])
def test_oracle_matches_julia_reference(name, golden):
    import scipy.io
    jl = scipy.io.loadmat(os.path.join(OUT, name))
    d = golden(name[:-4])
    meta = d["meta"]
    specs = [O.LayerSpec(l["in_dims"], l["out_dims"], l["grid_len"], l["normalizer"], l["basis"], l["use_base_act"],
                         tuple(l["grid_lims"]), None, l["iqf_reference_quirk"]) for l in meta["layers"]]
    if meta["kind"] == "chain":
        y = O.chain_fwd(specs, d["p"], d["u"])
        xb, pb = O.chain_vjp(specs, d["p"], d["u"], d["ybar"])
        pairs = [(y, jl["y"].T), (xb, jl["xbar"].T), (pb, jl["pbar"].ravel())]
    else:
        du = O.fk_rhs(specs[0], d["p"], meta["D"], meta["dx"], d["u"], dense=True)
        lj, dp = O.fk_vjp(specs[0], d["p"], meta["D"], meta["dx"], d["u"], d["lam"])
        pairs = [(du, jl["du"].T), (lj, jl["lamJ"].T), (dp, jl["dp"].ravel())]
    for ours, ref in pairs:
        assert np.max(np.abs(ours - ref)) <= 1e-12 * max(1.0, np.max(np.abs(ref)))
