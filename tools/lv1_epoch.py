#!/usr/bin/env python3
"""BASELINE configs[0] shape: the LV_driver_KANODE.jl training iteration (KAN [2,10,2] G=5,
one trajectory u0 = [1, 1], tspan (0, 3.5), saveat 0:0.1:3.4, adaptive Tsit5 at the default
tolerances, InterpolatingAdjoint, Adam) — GPU native path vs the CPU oracle driven by the
same integrator.  Prints ms per iteration for each.

    python3 tools/lv1_epoch.py --reps 5 [--batch 1]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kan-odes_amd"))
sys.path.insert(0, ROOT)

import kanode  # noqa: E402


def lotka(u0, ts):
    from scipy.integrate import solve_ivp
    f = lambda t, x: [1.5 * x[0] - x[0] * x[1], x[0] * x[1] - 3.0 * x[1]]   # noqa: E731  (LV_driver_KANODE.jl:119-122)
    return solve_ivp(f, (0.0, 3.5), u0, t_eval=ts, method="DOP853", rtol=1e-10, atol=1e-12).y.T


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args()
    ts = [0.1 * i for i in range(35)]
    u0 = np.array([1.0, 1.0])
    target = np.stack([lotka(u0, ts)] * a.batch, axis=1)            # (35, B, 2)
    chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
    p0 = chain.setup(np.random.default_rng(0))[0].astype(np.float64) / 1e5 * 1e4   # a mid-training scale
    legs = [("gpu", torch.device("cuda:0"))] + ([("cpu", "cpu")] if a.cpu else [])
    for name, dev in legs:
        if name == "gpu":
            rhs = kanode.ChainRHS(chain, device=dev)
        else:
            from oracle import oracle as O
            from oracle.oracle_rhs import OracleChainRHS
            rhs = OracleChainRHS([O.LayerSpec(2, 10, 5, "tanh_fast"), O.LayerSpec(10, 2, 5, "tanh_fast")])
        U0 = torch.as_tensor(np.tile(u0, (a.batch, 1)), device=dev)
        tr = kanode.Trainer(rhs, U0, (0.0, 3.5), ts, torch.as_tensor(target, device=dev),
                            torch.as_tensor(p0, device=dev), eta=1e-3,
                            sensealg="interpolating_adjoint")
        tr.step()
        if name == "gpu":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            tr.step()
        if name == "gpu":
            torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        _, _, sol = tr.loss_and_grad()
        print(f"{name}: {ms:.2f} ms/iteration  (B={a.batch}, forward steps {sol.stats.get('naccept')}, "
              f"loss {tr.history[-1]:.4e})", flush=True)


if __name__ == "__main__":
    main()
