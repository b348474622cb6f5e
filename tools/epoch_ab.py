#!/usr/bin/env python3
"""Interleaved A/B of handle options on bench.py's epoch leg (FK256 fp64, fixed-step Tsit5 +
InterpolatingAdjoint + Adam): each variant is a set of kanode_set_option values.

    python3 tools/epoch_ab.py --batch 4096 --variants "adj_step_rows=1;adj_step_rows=0" --rounds 5
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


def parse(v):
    return {k: int(x) for k, x in (kv.split("=") for kv in v.split(",") if kv)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--variants", default="adj_step_rows=1;adj_step_rows=0")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--adaptive", action="store_true")
    ap.add_argument("--dump-grad", default=None, help="save the first variant's gradient (.npy) for cross-library checks")
    a = ap.parse_args()
    variants = a.variants.split(";")
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
    times = {v: [] for v in variants}
    first = {}
    for r in range(a.rounds):
        for v in variants:
            with rhs.hd.options(**parse(v)):
                tr = kanode.Trainer(rhs, u0, (0.0, T), saveat, target, p0, eta=1e-3, solver=solver)
                tr.step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.reps):
                    tr.step()
                torch.cuda.synchronize()
                times[v].append((time.perf_counter() - t0) / a.reps * 1e3)
                if v not in first:
                    first[v] = tr.loss_and_grad()[1].cpu().numpy()
        print(f"round {r}: " + "  ".join(f"[{v}] {times[v][-1]:.3f} ms" for v in variants), flush=True)
    ref = first[variants[0]]
    if a.dump_grad:
        np.save(a.dump_grad, ref)
    for v in variants:
        d = np.max(np.abs(first[v] - ref)) / max(np.max(np.abs(ref)), 1e-300)
        print(f"[{v}]: median {np.median(times[v]):.3f} ms/epoch  min {np.min(times[v]):.3f}  "
              f"gradient max rel diff vs [{variants[0]}]: {d:.2e}")


if __name__ == "__main__":
    main()
