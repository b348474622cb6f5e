#!/usr/bin/env python3
"""Benchmark: KAN-ODE RHS evaluations/s on MI355X (BASELINE.json metric).

Workload (default `fisher_kpp_256`, BASELINE.json configs[2] — the north-star
target config): the Fisher-KPP source-term RHS
    du = D*lap*u + KDense(1,1,10; softsign).(u)      (PDE examples/Fisher-KPP_Source.jl:95-98)
on a 256-point periodic grid, fp64, B synthetic trajectories per GPU (the
reference's IC family, Fisher-KPP_Source.jl:47-49, randomised per trajectory),
random-init parameters.  One STEP = one RHS evaluation of the whole batch (one
kernel launch).  value = trajectories x steps x ranks / max-over-ranks wall time.

Multi-GPU: one process per GPU (torchrun); trajectories shard across ranks with
no collective on the data path (weak scaling: per-GPU batch fixed).

Extra JSON fields: `roofline` (dominant kernel, HIP-event timed on its stream),
`cpu_baseline` (the CPU restatement of the reference algorithm — dense Laplacian
matvec + per-point scalar KAN — timed on this host, rank 0 at N=1), `vjp` (the
adjoint kernel's rate, measured after the timed region).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kan-odes_amd"))
sys.path.insert(0, ROOT)

import kanode  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "RHS evals/sec (batched trajectories) at 1/8 GPU; wall-clock/epoch vs CPU ref"


def fk_ics(B: int, nx: int, dx: float, seed: int, device) -> torch.Tensor:
    g = torch.Generator(device="cpu").manual_seed(seed)
    c = 0.3 + 0.4 * torch.rand(B, 1, generator=g, dtype=torch.float64)
    dl = 0.1 + 0.2 * torch.rand(B, 1, generator=g, dtype=torch.float64)
    amp = 0.5 + 0.5 * torch.rand(B, 1, generator=g, dtype=torch.float64)
    c, dl, amp = c.to(device), dl.to(device), amp.to(device)
    x = torch.arange(nx, dtype=torch.float64, device=device) * dx
    return (amp * (torch.tanh((x - (c - dl / 2)) / (dl / 10)) - torch.tanh((x - (c + dl / 2)) / (dl / 10))) / 2).contiguous()


def load_traffic(workload: str, batch: int):
    """Per-launch HBM bytes of the dominant kernel from the committed PMC summary."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(workload)
        if e and int(e["batch"]) == batch:
            return float(e["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        pass
    return None


def cpu_baseline(nx, dx, D, p_np, target_s: float):
    """The faithful CPU restatement (oracle/cpu_bench.c) timed on this host."""
    from oracle import oracle as O
    spec = O.LayerSpec(1, 1, 10, "softsign")
    threads = max(1, min(16, os.cpu_count() or 1))
    rng = np.random.default_rng(123)
    B = 256
    x = np.arange(nx) * dx
    c, dl, amp = rng.uniform(0.3, 0.7, (B, 1)), rng.uniform(0.1, 0.3, (B, 1)), rng.uniform(0.5, 1.0, (B, 1))
    u = amp * (np.tanh((x - (c - dl / 2)) / (dl / 10)) - np.tanh((x - (c + dl / 2)) / (dl / 10))) / 2
    t1 = O.bench_fk_rhs(spec, p_np, D, dx, u, 1, threads)            # calibration
    reps = max(1, int(0.75 * target_s / max(t1, 1e-6)))
    tm = O.bench_fk_rhs(spec, p_np, D, dx, u, reps, threads)
    t1s = O.bench_fk_rhs(spec, p_np, D, dx, u[:32], 2, 1)          # single-core reference shape
    return {
        "value": B * reps / tm,
        "unit": "RHS-evals/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{B} trajectories x {reps} RHS evals, Nx={nx}, dense (D*lap)*u matvec + per-point "
                  f"KDense(1,1,10) (oracle/cpu_bench.c, OpenMP {threads} threads, {tm:.1f} s)",
        "single_core_value": 32 * 2 / t1s,
    }


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="fisher_kpp_256", choices=["fisher_kpp_256"])
    ap.add_argument("--batch", type=int, default=131072, help="trajectories per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-vjp", action="store_true")
    ap.add_argument("--no-table", action="store_true",
                    help="per-point basis recurrence instead of the piecewise-polynomial table (kan_pp.hip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if dist else 0)
    torch.cuda.set_device(dev)

    nx, D = 256, 0.01
    dx = 1.0 / (nx - 1)
    B = args.batch
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign", basis_func="rbf"))
    rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=dx, D=D, dtype=torch.float64, device=dev,
                              table=False if args.no_table else None)
    table = rhs.hd.pointwise_table
    p_np = kan1.setup(np.random.default_rng(0))[0].astype(np.float64)
    p = torch.as_tensor(p_np, device=dev)
    u = fk_ics(B, nx, dx, seed=1000 + rank, device=dev)
    du = torch.empty_like(u)
    rhs.hd.reserve(B)

    for _ in range(args.warmup):
        rhs.rhs(u, p, du)
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        rhs.rhs(u, p, du)
        ev[i][1].record(stream)
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        elapsed = float(tt.item())
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    total_evals = B * args.steps * world
    value = total_evals / elapsed
    alg_bytes = 8.0 * (rhs.P + B * (nx + nx))       # p + u in + du out, per launch
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = load_traffic(f"{args.workload}:{'table' if table else 'recurrence'}", B)

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "RHS-evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (reference IC family randomised per trajectory; random-init KAN params)",
        "config": {"workload": "fisher_kpp_256", "nx": nx, "batch_per_gpu": B, "kan": "KDense(1,1,10) softsign rbf",
                   "kan_eval": "piecewise-polynomial table" if table else "basis recurrence",
                   "parallelism": f"trajectory-sharded x{world} (no data-path collective)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": ("fk_pp_build_kernel + fk_rhs_pp_wave_kernel<SOFTSIGN,RBF,2>" if table
                                else "fk_rhs_kernel<double,SOFTSIGN,REC_CORR,10>"),
                     "kernel_ms": kern_ms,
                     "alg_bytes_per_launch": alg_bytes},
    }

    if not args.no_vjp:
        lam = torch.randn_like(u)
        lamJ = torch.empty_like(u)
        dp = torch.zeros_like(p)
        from kanode import _lib as L
        import ctypes as C
        hv = rhs.hd
        def vjp():
            L.check(L.lib().kanode_vjp(hv._h, C.c_void_p(p.data_ptr()), C.c_void_p(u.data_ptr()),
                                       C.c_void_p(lam.data_ptr()), C.c_void_p(lamJ.data_ptr()),
                                       C.c_void_p(dp.data_ptr()), B, C.c_void_p(stream.cuda_stream)), hv._h, "vjp")
        for _ in range(3):
            vjp()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        nv = max(5, args.steps // 2)
        e0.record(stream)
        for _ in range(nv):
            vjp()
        e1.record(stream)
        torch.cuda.synchronize()
        vms = e0.elapsed_time(e1) / nv
        vbytes = 8.0 * (2 * rhs.P + B * (2 * nx + nx))
        out["vjp"] = {"value": B * world / (vms * 1e-3), "unit": "VJP-evals/s", "ms_per_step": vms,
                      "achieved_GBps": vbytes / (vms * 1e-3) / 1e9}

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(nx, dx, D, p_np, args.cpu_seconds)
        out["cpu_baseline"] = cb
        out["gpu_vs_cpu"] = value / cb["value"]

    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
