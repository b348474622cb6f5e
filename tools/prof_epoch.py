#!/usr/bin/env python3
"""One training epoch of bench.py's epoch leg (FK256 fp64, fixed-step Tsit5 forward +
InterpolatingAdjoint + Adam), repeated, for rocprofv3 kernel traces; prints the wall time
per epoch for the native integrator and (--python) the Python statement of it.

    python3 tools/prof_epoch.py --batch 4096 --reps 3 [--python]
"""
import argparse
import dataclasses
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kan-odes_amd"))
sys.path.insert(0, ROOT)

import kanode  # noqa: E402
from bench import fk_ics  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--python", action="store_true", help="also time the Python driver")
    ap.add_argument("--adaptive", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    nx, dx, D, dt = 256, 1 / 255, 0.01, 1e-3
    T = a.steps * dt
    saveat = [T * i / 5 for i in range(6)]
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
    rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=dx, D=D, device=dev)
    p0 = torch.as_tensor(kan1.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
    u0 = fk_ics(a.batch, nx, dx, 7, dev)
    target = (0.9 * u0).unsqueeze(0).expand(len(saveat), -1, -1).contiguous()
    solver = kanode.Tsit5Options(adaptive=a.adaptive, dt=None if a.adaptive else dt)
    variants = [("native", solver)] + ([("python", dataclasses.replace(solver, native=False))] if a.python else [])
    for name, opt in variants:
        tr = kanode.Trainer(rhs, u0, (0.0, T), saveat, target, p0, eta=1e-3, solver=opt)
        tr.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            tr.step()
        torch.cuda.synchronize()
        print(f"{name}: {(time.perf_counter() - t0) / a.reps * 1e3:.2f} ms/epoch (B={a.batch}, loss {tr.history[-1]:.6e})",
              flush=True)


if __name__ == "__main__":
    main()
