#!/usr/bin/env python3
"""Export the inputs of tests/golden/*.npz as MATLAB files for tools/julia_regen.jl (MAT.jl is in the
reference's Lotka-Volterra environment; NPZ.jl is not):  tests/golden/julia_in/<name>.mat with p, u,
ybar / lam, and the configuration (layers, nx, dx, D) as fields.  Arrays keep the Julia layout: a
numpy (K, I) array is written as the [I, K] matrix the reference's KDense takes."""
import json
import os
import sys

import numpy as np
import scipy.io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def main():
    out = os.path.join(GOLD, "julia_in")
    os.makedirs(out, exist_ok=True)
    n = 0
    for f in sorted(os.listdir(GOLD)):
        if not f.endswith(".npz"):
            continue
        with np.load(os.path.join(GOLD, f), allow_pickle=False) as z:
            d = {k: z[k] for k in z.files}
        if "meta" not in d:
            continue
        meta = json.loads(str(d["meta"]))
        if meta.get("kind") not in ("chain", "fisher_kpp") or meta.get("dtype") != "float64":
            continue
        if any(not l["iqf_reference_quirk"] and l["basis"] == "iqf" for l in meta["layers"]):
            continue   # the reference's IQF pullback is the quirk (utils.jl:59); the exact variant is ours
        rec = {"kind": meta["kind"], "p": d["p"],
               "u": d["u"].T.copy(),                               # [N, K] / [Nx, B]
               "nlayers": len(meta["layers"])}
        rec["ybar"] = (d["ybar"] if meta["kind"] == "chain" else d["lam"]).T.copy()
        for i, l in enumerate(meta["layers"]):
            for k in ("in_dims", "out_dims", "grid_len", "normalizer", "basis"):
                rec[f"l{i}_{k}"] = l[k]
            rec[f"l{i}_use_base_act"] = int(l["use_base_act"])
        if meta["kind"] == "fisher_kpp":
            rec.update(nx=meta["nx"], dx=meta["dx"], D=meta["D"])
        scipy.io.savemat(os.path.join(out, f[:-4] + ".mat"), rec)
        n += 1
    print(f"{n} input files in {out}")


if __name__ == "__main__":
    sys.exit(main())
