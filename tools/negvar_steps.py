#!/usr/bin/env python3
"""The all-negative adaptive case (tests/test_gpu_fk_e2e.py::test_fk_default_path_negative_states[adaptive]): the
adjoint's accepted step sizes on the table path and on the direct per-point kernels, side by side."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "kan-odes_amd")]
import kanode  # noqa: E402
import test_gpu_fk_e2e as T  # noqa: E402

dev = torch.device("cuda:0")
nx, B, seed = 256, 3, 31
u0 = 1.0 * T._u0(nx, B, seed) - 2.2
p0 = 0.5 * np.random.default_rng(seed + 100).uniform(-1.0, 1.0, 11)
tspan, ts = (0.0, 0.5), [0.0, 0.15, 0.25, 0.5]
w = np.random.default_rng(seed + 200).normal(size=(len(ts), B, nx))
opt = kanode.Tsit5Options(abstol=1e-9, reltol=1e-9)
out = {}
for name, opts in (("table", {}), ("direct", {"pointwise_table": 0})):
    f = kanode.FisherKPPRHS(kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign")), nx=nx, dx=1 / (nx - 1),
                            D=0.0, device=dev)
    f.hd.set_option("record_adjoint_steps", 1)
    with f.hd.options(**opts):
        u, gp, gu, st = T._run(f, dev, torch.as_tensor(u0, device=dev), p0, tspan, ts, w, opt)
    out[name] = {"fwd_dts": [round(x, 8) for x in st.get("dts", [])], "adj_dts": [round(float(x), 8) for x in st["adjoint"].get("dts", [])],
                 "adj": {k: st["adjoint"][k] for k in ("naccept", "nreject")}, "gp": gp.tolist()}
out["gp_rel_diff"] = float(np.abs(np.array(out["table"]["gp"]) - np.array(out["direct"]["gp"])).max() /
                           np.abs(np.array(out["direct"]["gp"])).max())
for k in ("table", "direct"):
    out[k].pop("gp")
print(json.dumps(out), flush=True)
