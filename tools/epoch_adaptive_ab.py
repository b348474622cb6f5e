#!/usr/bin/env python3
"""Interleaved A/B of handle options on bench.py's adaptive reference-problem epoch (FK256 fp64, T = 5,
saveat 0.5, default tolerances, 4,096 trajectories; native Tsit5 + InterpolatingAdjoint + Adam):
    python3 tools/epoch_adaptive_ab.py --variants "adj_step_rows=1;adj_step_rows=2" --rounds 3
Each round runs every variant once (a fresh Trainer, one warm-up epoch, `reps` timed epochs)."""
import argparse
import gc
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import bench  # noqa: E402


def parse(v):
    return {k: int(x) for k, x in (kv.split("=") for kv in v.split(",") if kv)}


ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="adj_step_rows=1;adj_step_rows=2")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--batch", type=int, default=4096)
a = ap.parse_args()
dev = torch.device("cuda:0")
p_np = bench.fk_trained_like_params()
variants = a.variants.split(";")
res = {v: [] for v in variants}
steps = {}
for r in range(a.rounds):
    for v in variants:
        out = bench.epoch_adaptive_bench(dev, p_np, 256, 1 / 255, 0.01, a.batch, 0, reps=a.reps, hd_opts=parse(v))
        res[v].append(out["gpu"] * 1e3)
        steps[v] = (out["forward_steps"], out["adjoint_steps"], out["adjoint_rejects"])
        print(f"round {r} {v}: {out['gpu'] * 1e3:.1f} ms/epoch  steps {steps[v]}", flush=True)
        gc.collect()               # the previous handle's dense output (~180 GB at 3,707 steps) goes first
        torch.cuda.empty_cache()
for v in variants:
    print(json.dumps({"variant": v, "median_ms": statistics.median(res[v]), "all_ms": res[v],
                      "forward_adjoint_rejects": steps[v]}))
