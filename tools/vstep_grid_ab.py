#!/usr/bin/env python3
"""Interleaved A/B of the adjoint-step kernel's grid (KANODE_OPT_GRID_ADJ_STEP)
on bench.py's epoch leg (FK256 fp64, fixed-step Tsit5 + InterpolatingAdjoint + Adam).

    python3 tools/vstep_grid_ab.py --batch 4096 --grids 0,512,640,1024 --rounds 5
(0 = the library's default grid)
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
from bench import fk_ics  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--grids", default="0,512,640,1024")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    grids = [int(g) for g in a.grids.split(",")]
    dev = torch.device("cuda:0")
    nx, dx, D, dt = 256, 1 / 255, 0.01, 1e-3
    T = a.steps * dt
    saveat = [T * i / 5 for i in range(6)]
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
    rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=dx, D=D, device=dev)
    p0 = torch.as_tensor(kan1.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
    u0 = fk_ics(a.batch, nx, dx, 7, dev)
    target = (0.9 * u0).unsqueeze(0).expand(len(saveat), -1, -1).contiguous()
    solver = kanode.Tsit5Options(adaptive=False, dt=dt)
    times = {g: [] for g in grids}
    first = {}
    for r in range(a.rounds):
        for g in grids:
            rhs.hd.set_option("grid_adj_step", g)
            tr = kanode.Trainer(rhs, u0, (0.0, T), saveat, target, p0, eta=1e-3, solver=solver)
            tr.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                tr.step()
            torch.cuda.synchronize()
            times[g].append((time.perf_counter() - t0) / a.reps * 1e3)
            if g not in first:
                first[g] = tr.loss_and_grad()[1].cpu().numpy()
        print(f"round {r}: " + "  ".join(f"grid {g}: {times[g][-1]:.3f} ms" for g in grids), flush=True)
    ref = first[grids[0]]
    for g in grids:
        print(f"grid {g:5d}: median {np.median(times[g]):.3f} ms/epoch  min {min(times[g]):.3f}  "
              f"gradient max rel diff vs grid {grids[0]}: {np.max(np.abs(first[g] - ref)) / np.max(np.abs(ref)):.2e}")


if __name__ == "__main__":
    main()
