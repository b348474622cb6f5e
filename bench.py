#!/usr/bin/env python3
"""Benchmark: KAN-ODE RHS evaluations/s on MI355X (BASELINE.json metric).

Workload (default `fisher_kpp_256`, BASELINE.json configs[2] — the north-star
target config, "≥6× strong scaling at 8 GPUs"): the Fisher-KPP source-term RHS
    du = D*lap*u + KDense(1,1,10; softsign).(u)      (PDE examples/Fisher-KPP_Source.jl:95-98)
on a 256-point periodic grid, fp64, synthetic trajectories (the reference's IC
family, Fisher-KPP_Source.jl:47-49, randomised per trajectory), random-init
parameters.  One STEP = one RHS evaluation of the whole batch (one `kanode_rhs`
call: table build + RHS kernel; the parameters alternate between two bitwise-different
vectors so that every step rebuilds the table).  value = total trajectories x steps /
max-over-ranks wall time.

Multi-GPU: one process per GPU; the fixed total batch (default 1,048,576
trajectories = 8 x 131,072) shards evenly across ranks with no collective on the
data path: strong scaling, total work fixed as N grows (`--batch-per-gpu`
switches to weak scaling).  Under an external launcher (torchrun: WORLD_SIZE set)
`--gpus` must equal WORLD_SIZE.  Without one, `--gpus N > 1` starts N child
processes of this script itself (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, before
anything in this process touches the GPU), forwards rank 0's JSON line and exits
non-zero if any rank fails.  The line carries `rccl_world` (the process group's
own world size after init) and every rank's timed-region seconds.

Extra JSON fields: `roofline` (dominant kernel, HIP-event timed on its stream),
`cpu_baseline` (the CPU restatement of the reference algorithm — dense Laplacian
matvec + per-point scalar KAN — timed on this host, rank 0 at N=1), `vjp` (the
adjoint kernel's rate, measured after the timed region).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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


def load_traffic(workload: str, alg_bytes: float):
    """Per-launch HBM bytes of the dominant kernel: the committed PMC measurement
    (profiles/traffic.json, FETCH_SIZE x2 + WRITE_SIZE) as a ratio to the algorithmic
    bytes of the launch it was measured on, applied to this launch's algorithmic bytes."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(workload)
        if e:
            return float(e["traffic_over_algorithmic"]) * alg_bytes
    except (OSError, ValueError, KeyError):
        pass
    return None


def host_cpu():
    """(model name, CPUs this process may run on, threads used).  The GPU box gives one GPU's job a
    16-core share and exports OMP_NUM_THREADS=16 (nproc shows the whole machine), so the OpenMP
    comparator uses OMP_NUM_THREADS when it is set and the affinity mask otherwise."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    visible = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    threads = int(omp) if omp.isdigit() and int(omp) > 0 else visible
    return model, visible, max(1, min(threads, visible))


def cpu_baseline(nx, dx, D, p_np, target_s: float):
    """The faithful CPU restatement (oracle/cpu_bench.c) timed on this host."""
    from oracle import oracle as O
    spec = O.LayerSpec(1, 1, 10, "softsign")
    model, visible, threads = host_cpu()
    rng = np.random.default_rng(123)
    B = 256
    x = np.arange(nx) * dx
    c, dl, amp = rng.uniform(0.3, 0.7, (B, 1)), rng.uniform(0.1, 0.3, (B, 1)), rng.uniform(0.5, 1.0, (B, 1))
    u = amp * (np.tanh((x - (c - dl / 2)) / (dl / 10)) - np.tanh((x - (c + dl / 2)) / (dl / 10))) / 2
    O.bench_fk_rhs(spec, p_np, D, dx, u, 1, threads)                 # (thread pool start-up, first touch)
    t1 = O.bench_fk_rhs(spec, p_np, D, dx, u, 4, threads) / 4        # calibration
    # the median of >= 20 timed repetitions after 3 warm-ups; one repetition is k
    # back-to-back RHS evaluations of the batch, sized so the 20 take ~3/4 of the budget
    n_rep, n_warm = 20, 3
    k = max(1, int(0.75 * target_s / n_rep / max(t1, 1e-6)))
    for _ in range(n_warm):
        O.bench_fk_rhs(spec, p_np, D, dx, u, k, threads)
    reps = [O.bench_fk_rhs(spec, p_np, D, dx, u, k, threads) for _ in range(n_rep)]
    tm = float(np.median(reps))
    t1s = O.bench_fk_rhs(spec, p_np, D, dx, u[:32], 2, 1)          # single-core reference shape
    return {
        "value": B * k / tm,
        "unit": "RHS-evals/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{B} trajectories x {k} RHS evals per repetition, median of {n_rep} repetitions after {n_warm} "
                  f"warm-ups, Nx={nx}, dense (D*lap)*u matvec + per-point KDense(1,1,10) (oracle/cpu_bench.c, "
                  f"OpenMP {threads} threads, {sum(reps):.1f} s timed)",
        "rep_spread": [B * k / max(reps), B * k / min(reps)],
        "single_core_value": 32 * 2 / t1s,
        "cpu_model": model,
        "cpus_visible": visible,
        "threads_from": "OMP_NUM_THREADS (the box's 16-core share per GPU)" if os.environ.get("OMP_NUM_THREADS")
                        else "sched_getaffinity",
    }


def cpu_epoch(p_np, nx, dx, D, B_cpu, T, saveat, seed, eta, adaptive, dt, gpu_s, B_gpu):
    """The epoch on the host, in C on one core (oracle/cpu_epoch.c): Tsit5 with dense output, MSE loss,
    InterpolatingAdjoint, Adam, with the reference's dense Laplacian matvec in the RHS and its
    transpose in the VJP.  No interpreter in the loop (tests/test_cpu_epoch.py pins it to the Python
    statement of the same epoch)."""
    from oracle import oracle as O
    u0 = fk_ics(B_cpu, nx, dx, seed=seed, device="cpu").numpy()
    target = 0.9 * np.broadcast_to(u0, (len(saveat), B_cpu, nx))
    _, _, _, st, secs = O.fk_epoch(O.LayerSpec(1, 1, 10, "softsign"), p_np, D, dx, u0, T, saveat, target,
                                   adaptive=adaptive, dt=dt, eta=eta)
    model, _, _ = host_cpu()
    return {"cpu": secs, "cpu_batch": B_cpu, "cpu_cores": 1, "cpu_model": model,
            "cpu_kind": "port (oracle/cpu_epoch.c: C Tsit5 + InterpolatingAdjoint + Adam, dense Laplacian matvec "
                        "+ scalar KAN, one core)",
            "cpu_steps": [st["naccept"], st["adjoint_naccept"]],
            "gpu_per_trajectory": gpu_s / B_gpu, "cpu_per_trajectory": secs / B_cpu,
            "speedup_per_trajectory": (secs / B_cpu) / (gpu_s / B_gpu)}


def epoch_bench(dev, p_np, nx, dx, D, B_gpu: int, B_cpu: int, steps: int, dt: float, reps: int, group=None,
                rank: int = 0, world: int = 1):
    """Wall-clock of one training epoch (BASELINE metric, second half): fixed-step Tsit5 forward
    solve with saveat (dense output kept), the InterpolatingAdjoint backward solve (the reference's
    SciMLSensitivity default), loss, Adam update (kanode.Trainer.step; Fisher-KPP_Source.jl:102-109,
    167-201).  With a process group every rank trains its own shard of B_gpu trajectories (data
    parallel, weak scaling) and Trainer.step all-reduces [dL/dp ; L] once per epoch (RCCL with the
    nccl backend); the epoch time is the max over ranks.  The CPU reference runs the same epoch
    through the oracle (dense Nx x Nx Laplacian matvec, as the reference does) on a bounded sample
    of B_cpu trajectories; per-trajectory times are reported for both."""
    T = steps * dt
    saveat = [T * i / 5 for i in range(6)]
    solver = kanode.Tsit5Options(adaptive=False, dt=dt)
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign", basis_func="rbf"))
    rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=dx, D=D, dtype=torch.float64, device=dev)
    u0 = fk_ics(B_gpu, nx, dx, seed=7 + rank, device=dev)
    target = (0.9 * u0).unsqueeze(0).expand(len(saveat), -1, -1).contiguous()
    tr = kanode.Trainer(rhs, u0, (0.0, T), saveat, target, torch.as_tensor(p_np, device=dev), eta=1e-3,
                        solver=solver, group=group)
    tr.step()                                   # warm-up (allocations, table builds, the collective)
    torch.cuda.synchronize()
    if group is not None:
        import torch.distributed as tdist
        tdist.barrier(group=group)
    t0 = time.perf_counter()
    for _ in range(reps):
        tr.step()
    torch.cuda.synchronize()
    gpu_s = (time.perf_counter() - t0) / reps
    if group is not None:
        tt = torch.tensor([gpu_s], dtype=torch.float64, device=dev if tdist.get_backend(group) == "nccl" else "cpu")
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX, group=group)
        gpu_s = float(tt.item())
    out = {"unit": "s/epoch", "gpu": gpu_s, "gpu_batch": B_gpu, "steps": steps, "dt": dt, "stages_per_step": 6,
           "what": "fixed-step Tsit5 solve + InterpolatingAdjoint + Adam, FK256 fp64 (native kanode_solve_tsit5 + kanode_adjoint_tsit5)"}
    if group is not None:
        out.update({"ranks": world, "trajectories_total": B_gpu * world, "scaling": "weak",
                    "trajectories_per_s": B_gpu * world / gpu_s,
                    "collective": "one all_reduce(SUM) of [dL/dp ; L] (12 doubles) per epoch"})
    if B_cpu > 0:
        out.update(cpu_epoch(p_np, nx, dx, D, B_cpu, T, saveat, 7, 1e-3, False, dt, gpu_s, B_gpu))
    return out


def fk_trained_like_params() -> np.ndarray:
    """A "trained" KDense(1,1,10; softsign) parameter set: the ridge least-squares fit (λ = 1e-4) of the
    layer to the Fisher-KPP reaction term r·u·(1 - u), r = 1, over u in [-0.25, 1.25]
    (Fisher-KPP_Source.jl:36,52: the source the reference's KAN is trained to recover).  Max fit error
    4e-3, |C| <= 2.  With Glorot-random parameters instead, the source is W·swish(u) + ... with
    W ~ 1: the T = 5 solution grows to |u| ~ 150, far outside the piecewise-polynomial table's
    [-4, 4) (every point then takes the direct-formula cold path), which no trained model does."""
    g = kanode.linrange_f32(-1.0, 1.0, 10).astype(np.float64)
    ih = float(np.float32(1.0) / np.float32(2.0 / 9.0))
    u = np.linspace(-0.25, 1.25, 301)
    n = u / (1.0 + np.abs(u))
    A = np.concatenate([np.exp(-((n[:, None] - g[None, :]) * ih) ** 2), (u / (1.0 + np.exp(-u)))[:, None]], 1)
    return np.linalg.solve(A.T @ A + 1e-4 * np.eye(11), A.T @ (u * (1.0 - u)))


def epoch_adaptive_bench(dev, p_np, nx, dx, D, B_gpu: int, B_cpu: int, reps: int = 1, hd_opts=None):
    """The reference's Fisher-KPP training epoch as written (Fisher-KPP_Source.jl:38-44,101-109,198-201):
    T = 5, saveat every 0.5 (11 points), solve(prob, Tsit5()) at the default tolerances (abstol 1e-6,
    reltol 1e-3, adaptive), the gradient by the InterpolatingAdjoint, one Adam step; here at Nx = 256
    (the configs[2] grid) over B_gpu trajectories on the GPU (native solve + adjoint: one launch per
    forward / adjoint step) and B_cpu on the CPU (cpu_epoch: C, one core)."""
    T = 5.0
    saveat = [0.5 * i for i in range(11)]
    solver = kanode.Tsit5Options()
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign", basis_func="rbf"))
    rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=dx, D=D, dtype=torch.float64, device=dev)
    u0 = fk_ics(B_gpu, nx, dx, seed=17, device=dev)
    target = (0.9 * u0).unsqueeze(0).expand(len(saveat), -1, -1).contiguous()
    tr = kanode.Trainer(rhs, u0, (0.0, T), saveat, target, torch.as_tensor(p_np, device=dev), eta=1e-2, solver=solver)
    for k, v in (hd_opts or {}).items():      # (A/B experiments: tools/epoch_adaptive_ab.py)
        rhs.hd.set_option(k, v)
    tr.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        tr.step()
    torch.cuda.synchronize()
    gpu_s = (time.perf_counter() - t0) / reps
    _, _, sol = tr.loss_and_grad()
    out = {"unit": "s/epoch", "gpu": gpu_s, "gpu_batch": B_gpu, "T": T, "saveat": 0.5, "abstol": 1e-6, "reltol": 1e-3,
           "params": "trained-like (fk_trained_like_params: the KAN fitted to u(1-u))",
           "forward_steps": sol.stats["naccept"], "forward_rejects": sol.stats["nreject"],
           "adjoint_steps": sol.stats["adjoint"]["naccept"], "adjoint_rejects": sol.stats["adjoint"]["nreject"],
           "what": "adaptive Tsit5 solve (T=5, saveat 0.5, default tolerances) + InterpolatingAdjoint + Adam, "
                   "FK256 fp64 (native kanode_solve_tsit5 + kanode_adjoint_tsit5)"}
    if B_cpu > 0:
        out.update(cpu_epoch(p_np, nx, dx, D, B_cpu, T, saveat, 17, 1e-2, True, 0.0, gpu_s, B_gpu))
    return out


def lv4096_bench(dev, steps: int = 200):
    """BASELINE configs[1]: Lotka-Volterra KAN [2,10,2] grid=5, 4096 batched ICs, fp32 — the
    NeuralODE dudt (LV_driver_KANODE.jl:139-143,180) over the batch, as RHS evals/s.  One RHS is
    one launch of the fused chain kernel (kd_chain_col_kernel); 32 KB of state makes a single
    call launch-bound, so the device rate is measured on a hipGraph of `steps` back-to-back RHS
    calls (captured through the C-ABI after kanode_reserve), next to the eager per-call time."""
    chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
    rhs = kanode.ChainRHS(chain, dtype=torch.float32, device=dev)
    p = torch.as_tensor(chain.setup(np.random.default_rng(0))[0] / 1e5, dtype=torch.float32, device=dev)
    g = torch.Generator(device="cpu").manual_seed(1)
    u = (0.5 + 1.5 * torch.rand(4096, 2, generator=g)).to(dev, torch.float32)
    du = torch.empty_like(u)
    rhs.hd.reserve(4096)
    for _ in range(10):
        rhs.rhs(u, p, du)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        rhs.rhs(u, p, du)
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / steps
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        rhs.rhs(u, p, du)
        torch.cuda.synchronize()
        with torch.cuda.graph(graph, stream=s):
            for _ in range(steps):
                rhs.rhs(u, p, du)
    graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        graph.replay()
    e1.record()
    torch.cuda.synchronize()
    dt = e0.elapsed_time(e1) * 1e-3 / (5 * steps)
    return {"value": 4096 / dt, "unit": "RHS-evals/s", "us_per_rhs": dt * 1e6, "batch": 4096, "dtype": "f32",
            "eager_us_per_call": eager * 1e6,
            "note": f"device time per RHS from a hipGraph of {steps} launches (one fused-chain kernel each)"}


def lv_targets(u0: np.ndarray, ts) -> np.ndarray:
    """The analytic Lotka-Volterra model (LV_driver_KANODE.jl:110-122: α = 1.5, β = 1, γ = 1, δ = 3) from every
    initial condition of u0 (B, 2), at the times ts: (len(ts), B, 2), one stacked DOP853 solve at 1e-10 / 1e-12."""
    from scipy.integrate import solve_ivp
    B = u0.shape[0]

    def f(t, x):
        a, b = x[:B], x[B:]
        return np.concatenate([1.5 * a - a * b, a * b - 3.0 * b])
    y = solve_ivp(f, (0.0, float(ts[-1])), np.concatenate([u0[:, 0], u0[:, 1]]), t_eval=ts, method="DOP853",
                  rtol=1e-10, atol=1e-12).y            # (2B, len(ts))
    return np.stack([y[:B].T, y[B:].T], axis=-1)


def lv4096_train_bench(dev, with_cpu: bool, reps: int = 10, B: int = 4096, B_cpu: int = 16):
    """BASELINE configs[1] trained: the LV KAN [2,10,2] G=5 NeuralODE over B = 4096 random initial conditions
    u0 ~ U[0.5, 2]² (seed 1) as ONE batched ODE (state [2, B], shared adaptive dt and RMS error
    norm, as a Lux chain on a matrix state in the reference), fp32, tspan (0, 3.5), saveat 0:0.1:3.4 against the
    analytic LV trajectories of every IC; one LV_driver_KANODE.jl:283-287 iteration = adaptive Tsit5 solve +
    InterpolatingAdjoint + Adam(5e-4) (Trainer.step).  CPU: the same iteration in C (oracle/cpu_epoch.c, fp64,
    one core) on the first B_cpu initial conditions (a bounded sample: the step count of a batched ODE depends on
    its batch), reported per trajectory beside the GPU's."""
    ts = [0.1 * i for i in range(35)]
    rng = np.random.default_rng(1)
    u0n = rng.uniform(0.5, 2.0, (B, 2))
    target = lv_targets(u0n, ts)
    chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
    # a trained network (the round-5 LV anchor run's final parameters, seed 1, 1e5 Adam iterations from [1, 1];
    # tests/golden/lv_trained_p_seed1.npy): the LV oscillation itself sets the step count, as late in training
    p0 = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden", "lv_trained_p_seed1.npy"))
    rhs = kanode.ChainRHS(chain, dtype=torch.float32, device=dev)
    u0 = torch.as_tensor(u0n, dtype=torch.float32, device=dev).contiguous()
    tgt = torch.as_tensor(target, dtype=torch.float32, device=dev).contiguous()
    tr = kanode.Trainer(rhs, u0, (0.0, 3.5), ts, tgt, torch.as_tensor(p0, dtype=torch.float32, device=dev),
                        eta=5e-4, sensealg="interpolating_adjoint")
    tr.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        tr.step()
    torch.cuda.synchronize()
    gpu_ms = (time.perf_counter() - t0) / reps * 1e3
    _, _, sol = tr.loss_and_grad()
    out = {"unit": "ms/iteration", "batch": B, "dtype": "f32", "gpu": gpu_ms,
           "gpu_per_trajectory_us": gpu_ms * 1e3 / B,
           "forward_steps": sol.stats["naccept"], "adjoint_steps": sol.stats["adjoint"]["naccept"],
           "adjoint_path": rhs.hd.get_option("last_adjoint"),
           "what": "configs[1] training iteration: adaptive Tsit5 + InterpolatingAdjoint + Adam(5e-4), LV KAN "
                   "[2,10,2] G=5, 4096 ICs as one batched ODE, fp32, saveat 0:0.1:3.4 vs the analytic LV model"}
    if with_cpu:
        from oracle import oracle as O
        specs = [O.LayerSpec(2, 10, 5, "tanh_fast"), O.LayerSpec(10, 2, 5, "tanh_fast")]
        pc = p0.copy()
        times, st = [], None
        for r in range(8):
            t1 = time.perf_counter()
            _, _, pc, st, _ = O.chain_epoch(specs, pc, u0n[:B_cpu], 3.5, ts, target[:, :B_cpu], eta=5e-4)
            if r >= 2:
                times.append(time.perf_counter() - t1)
        cpu_ms = float(np.median(times)) * 1e3
        out.update({"cpu": cpu_ms, "cpu_batch": B_cpu, "cpu_cores": 1, "cpu_forward_steps": st["naccept"],
                    "cpu_per_trajectory_us": cpu_ms * 1e3 / B_cpu,
                    "cpu_kind": "port (oracle/cpu_epoch.c, fp64, one core; the first 16 ICs as one batched ODE; "
                                "median of 6 after 2 warm-ups)",
                    "speedup_per_trajectory": (cpu_ms / B_cpu) / (gpu_ms / B)})
    return out


def lv1_train_bench(dev, with_cpu: bool, reps: int = 10):
    """BASELINE configs[0] shape: one LV_driver_KANODE.jl training iteration (KAN [2,10,2] G=5,
    u0 = [1, 1], tspan (0, 3.5), saveat 0:0.1:3.4, adaptive Tsit5 at the default tolerances,
    InterpolatingAdjoint, Adam; LV_driver_KANODE.jl:119-122,139-143,175-219).  On the GPU a
    single trajectory runs the forward solve and the adjoint as one workgroup each
    (kd_chain_tsit5_kernel, kd_chain_adjoint_kernel).  CPU: the same iteration in C on one core over the
    oracle chain (oracle/cpu_epoch.c, kind "port"); Julia is not available to time the reference."""
    from scipy.integrate import solve_ivp
    ts = [0.1 * i for i in range(35)]
    ts_test = [0.1 * i for i in range(141)]
    f = lambda t, x: [1.5 * x[0] - x[0] * x[1], x[0] * x[1] - 3.0 * x[1]]   # noqa: E731
    full = solve_ivp(f, (0.0, 14.0), [1.0, 1.0], t_eval=ts_test, method="DOP853", rtol=1e-10,
                     atol=1e-12).y.T[:, None, :]
    target = full[:35]
    chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
    p0 = chain.setup(np.random.default_rng(0))[0].astype(np.float64) / 1e5 * 1e4   # a mid-training scale
    out = {"unit": "ms/iteration", "batch": 1, "dtype": "f64",
           "what": "one LV_driver_KANODE.jl iteration (:283-291): adaptive Tsit5 solve + InterpolatingAdjoint "
                   "+ Adam, then the loss_train (tspan_train, 35 saveat) and loss_test (tspan (0, 14), 141 "
                   "saveat) forward solves, LV KAN [2,10,2] G=5, one trajectory"}
    rhs = kanode.ChainRHS(chain, device=dev)
    u0 = torch.tensor([[1.0, 1.0]], dtype=torch.float64, device=dev)
    tr = kanode.Trainer(rhs, u0, (0.0, 3.5), ts, torch.as_tensor(target, device=dev), torch.as_tensor(p0, device=dev),
                        eta=1e-3, sensealg="interpolating_adjoint")
    tgt_test = torch.as_tensor(full, device=dev)

    def iteration():
        tr.step()
        # loss_train(p) after update! (:289): Trainer.eval_loss keeps this forward solve (dense output) for the
        # next iteration's gradient -- the same problem at the same p -- instead of solving it twice
        l_tr = tr.eval_loss()
        with torch.no_grad():
            l_te = kanode.mse_loss(kanode.solve(rhs, u0, (0.0, 14.0), tr.p, ts_test).u, tgt_test)
        return l_tr, float(l_te)

    iteration()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        iteration()
    torch.cuda.synchronize()
    out["gpu"] = (time.perf_counter() - t0) / reps * 1e3
    if with_cpu:
        # the same iteration in C on one core (oracle/cpu_epoch.c: kref_chain_epoch_f64 + two kref_chain_solve_f64,
        # pinned to the Python statement by tests/test_cpu_epoch.py); median of 20 after 3 warm-ups
        from oracle import oracle as O
        specs = [O.LayerSpec(2, 10, 5, "tanh_fast"), O.LayerSpec(10, 2, 5, "tanh_fast")]
        u0c = np.array([[1.0, 1.0]])
        pc = p0.copy()
        times = []
        for r in range(23):
            t0 = time.perf_counter()
            _, _, pc, _, _ = O.chain_epoch(specs, pc, u0c, 3.5, ts, target, eta=1e-3)
            O.chain_solve(specs, pc, u0c, 3.5, ts)
            O.chain_solve(specs, pc, u0c, 14.0, ts_test)
            if r >= 3:
                times.append(time.perf_counter() - t0)
        out.update({"cpu": float(np.median(times)) * 1e3, "cpu_cores": 1,
                    "cpu_kind": "port (oracle/cpu_epoch.c: C Tsit5 + InterpolatingAdjoint + Adam over the oracle "
                                "chain, plus the two loss solves, one core; median of 20 after 3 warm-ups)",
                    "speedup": float(np.median(times)) * 1e3 / out["gpu"]})
    return out


def fk26_train_bench(dev, with_cpu: bool, reps: int = 20):
    """The reference's own Fisher-KPP training iteration (PDE examples/Fisher-KPP_Source.jl:34-49,95-109,194-213):
    26 points (dx = 0.04 on [0, 1], periodic Laplacian, D = 0.01), the one initial condition (Amp = 1, Delta = 0.2),
    T = 5, saveat every 0.5 (11 stops), adaptive Tsit5 at the default tolerances, the InterpolatingAdjoint gradient
    and one Adam(1e-2) step; the training data from the true reaction u(1 - u) (:52,60-66) and a trained-like
    KDense(1,1,10) (fk_trained_like_params: the state stays in the table's range as the reference's training does).
    GPU: the whole forward solve and the whole adjoint are one workgroup each (kan_small.hip).  CPU: the same
    iteration in C on one core (oracle/cpu_epoch.c over the dense-Laplacian oracle RHS, kind "port"; median of 20
    after 3 warm-ups).  The reference selects ForwardDiffSensitivity at this size; both sides here
    run the InterpolatingAdjoint (tests/test_gpu_anchors.py bounds the difference)."""
    from scipy.integrate import solve_ivp
    nx, dx, D, T = 26, 0.04, 0.01, 5.0
    x = np.arange(nx) * dx
    rho0 = (np.tanh((x - 0.4) / 0.02) - np.tanh((x - 0.6) / 0.02)) / 2
    lap = (np.diag(-2.0 * np.ones(nx)) + np.diag(np.ones(nx - 1), 1) + np.diag(np.ones(nx - 1), -1)) / dx ** 2
    lap[0, -1] = lap[-1, 0] = 1.0 / dx ** 2
    saveat = [0.5 * i for i in range(11)]
    truth = solve_ivp(lambda t, u: D * lap @ u + u * (1 - u), (0.0, T), rho0, t_eval=saveat, method="DOP853",
                      rtol=1e-10, atol=1e-12).y.T[:, None, :]
    p0 = fk_trained_like_params()
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign", basis_func="rbf"))
    rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=dx, D=D, dtype=torch.float64, device=dev)
    u0 = torch.as_tensor(rho0[None, :], device=dev)
    tr = kanode.Trainer(rhs, u0, (0.0, T), saveat, torch.as_tensor(truth, device=dev), torch.as_tensor(p0, device=dev),
                        eta=1e-2, solver=kanode.Tsit5Options())
    tr.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        tr.step()
    torch.cuda.synchronize()
    gpu = (time.perf_counter() - t0) / reps * 1e3
    _, _, sol = tr.loss_and_grad()
    sensealg = sol.stats.get("sensealg", "interpolating_adjoint")
    out = {"unit": "ms/iteration", "batch": 1, "nx": nx, "dtype": "f64", "gpu": gpu, "sensealg": sensealg,
           "forward_steps": sol.stats["naccept"],
           "adjoint_steps": sol.stats["adjoint"]["naccept"] if "adjoint" in sol.stats else None,
           "gpu_path": ("one-workgroup forward-sensitivity solve (kanode_forward_sensitivity_tsit5)"
                        if sensealg == "forward" else
                        "one-workgroup solve + one-workgroup adjoint" if rhs.hd.get_option("last_adjoint") == 2
                        else "host loop"),
           "what": "one Fisher-KPP_Source.jl training iteration: adaptive Tsit5 (T = 5, saveat 0.5, default "
                   "tolerances), the gradient the reference takes at this size (SciMLSensitivity's automatic choice: "
                   "ForwardDiffSensitivity), Adam(1e-2), 26 points, one IC"}
    # the InterpolatingAdjoint iteration beside it (the product's path for larger fields)
    tra = kanode.Trainer(rhs, u0, (0.0, T), saveat, torch.as_tensor(truth, device=dev), torch.as_tensor(p0, device=dev),
                         eta=1e-2, solver=kanode.Tsit5Options(), sensealg="interpolating_adjoint")
    tra.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        tra.step()
    torch.cuda.synchronize()
    out["gpu_interpolating_adjoint"] = (time.perf_counter() - t0) / reps * 1e3
    if with_cpu:
        from oracle import oracle as O
        spec = O.LayerSpec(1, 1, 10, "softsign")
        pc = p0.copy()
        times = []
        for r in range(23):
            t0 = time.perf_counter()
            _, _, pc, st, _ = O.fk_fsens_epoch(spec, pc, D, dx, rho0[None, :], T, saveat, truth, eta=1e-2)
            if r >= 3:
                times.append(time.perf_counter() - t0)
        pa = p0.copy()
        times_a = []
        for r in range(13):
            t0 = time.perf_counter()
            _, _, pa, _, _ = O.fk_epoch(spec, pa, D, dx, rho0[None, :], T, saveat, truth, eta=1e-2)
            if r >= 3:
                times_a.append(time.perf_counter() - t0)
        out.update({"cpu": float(np.median(times)) * 1e3, "cpu_cores": 1,
                    "cpu_steps": [st.get("naccept"), st.get("nreject")],
                    "cpu_kind": "port (oracle/cpu_epoch.c kref_fk_fsens_epoch_f64: the C Dual-number Tsit5 solve "
                                "(ForwardDiffSensitivity) + Adam over the dense-Laplacian oracle RHS, one core; median "
                                "of 20 after 3 warm-ups)",
                    "speedup": float(np.median(times)) * 1e3 / gpu,
                    "cpu_interpolating_adjoint": float(np.median(times_a)) * 1e3})
    return out


def shard_ceiling(rhs, u, du, ps, stream, steps: int, full_rate: float):
    """The compute side of strong scaling, measured on this one GPU: the same timed step (table build + RHS over
    one rank's shard, parameters alternating so every step rebuilds) at the per-rank batches of N = 2, 4, 8
    ranks (the first B/N trajectories).  projected_ratio = N x rate(B/N) / rate(B) is the speed-up N GPUs would
    reach with no cost of their own (the bench's ranks share nothing on the data path); a SCALE line can be
    checked against it."""
    B = u.shape[0]
    out = {}
    for n in (2, 4, 8):
        b = B // n
        us, dus = u[:b], du[:b]
        for i in range(5):
            rhs.rhs(us, ps[i & 1], dus)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(steps):
            rhs.rhs(us, ps[(5 + i) & 1], dus)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / steps
        rate = b / (ms * 1e-3)
        out[f"n{n}"] = {"batch_per_gpu": b, "ms_per_step": ms, "rate_per_gpu": rate,
                        "projected_ratio": n * rate / full_rate}
    return out


def _graph_us(fn, reps: int = 50) -> float:
    """Device time per call from a hipGraph of `reps` back-to-back calls (launch-bound sizes)."""
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=st):
            for _ in range(reps):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (3 * reps)


def surrogate_bench(dev, with_cpu: bool, only: str | None = None, reps: int = 3):
    """BASELINE configs[3] and [4]: the full-field KAN surrogates, per GPU.
    burgers512: KAN [512, 10, 512] G=5 softsign (Burgers_Surrogate.jl:85-97 at 512 points), 4 ICs
      u0 = -sin(pi x) + sum_k a_k sin(k pi x) on [-1, 1], tspan (0, 1), saveat every 0.005 (200 steps),
      ADAM(1e-2) (:160).
    schrodinger1024: KAN [2048, 10, 2048] G=10 softsign (Schrodinger_Surrogate.jl:93-104 at 1024 points,
      state [Re; Im]), 8 ICs u0 = A 2 sech(x) (cos th, sin th) on [-5, 5], tspan (0, pi/2), saveat
      0.1:0.2:1.5 (:73), ADAM(1e-3) (:170).
    Reported: device time per RHS and per VJP at the batch (hipGraph of back-to-back calls) and one
    training iteration (adaptive Tsit5 at the default tolerances, InterpolatingAdjoint, Adam;
    kanode.Trainer.step).  CPU: the oracle chain (C restatement of kdense.jl:109-130, one core) per RHS
    of the same batch."""
    out = {}
    cases = (("burgers512", 512, 5, 4, (-1.0, 1.0), (0.0, 1.0), [0.005 * i for i in range(201)], 1e-2),
             ("schrodinger1024", 1024, 10, 8, (-5.0, 5.0), (0.0, np.pi / 2), [0.1 + 0.2 * i for i in range(8)], 1e-3))
    for name, nx, G, B, xs, tspan, saveat, eta in cases:
        if only and name != only:
            continue
        N = nx if name.startswith("burgers") else 2 * nx
        chain = kanode.Chain(kanode.KDense(N, 10, G, normalizer="softsign"), kanode.KDense(10, N, G, normalizer="softsign"))
        rhs = kanode.ChainRHS(chain, device=dev)
        p_np = chain.setup(np.random.default_rng(0))[0].astype(np.float64)
        p = torch.as_tensor(p_np, device=dev)
        rng = np.random.default_rng(5)
        x = np.linspace(xs[0], xs[1], nx)
        if name.startswith("burgers"):
            a = rng.normal(0.0, 0.1, (B, 3))
            u0 = -np.sin(np.pi * x)[None, :] + sum(a[:, k:k + 1] * np.sin((k + 1) * np.pi * x)[None, :] for k in range(3))
        else:
            amp, th = rng.uniform(0.8, 1.2, (B, 1)), rng.uniform(0.0, 2 * np.pi, (B, 1))
            env = amp * 2.0 / np.cosh(x)[None, :]
            u0 = np.concatenate([env * np.cos(th), env * np.sin(th)], axis=1)
        u = torch.as_tensor(u0, device=dev)
        lam = torch.randn_like(u)
        du, dp = torch.empty_like(u), torch.zeros_like(p)
        rhs.hd.reserve(B)
        t_rhs = _graph_us(lambda: rhs.hd.rhs(p, u, du))
        t_vjp = _graph_us(lambda: rhs.hd.vjp(p, u, lam, dp=dp))
        target = (0.9 * u).unsqueeze(0).expand(len(saveat), -1, -1).contiguous()
        tr = kanode.Trainer(rhs, u, tspan, saveat, target, p, eta=eta)
        tr.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            tr.step()
        torch.cuda.synchronize()
        it_ms = (time.perf_counter() - t0) / reps * 1e3
        _, _, sol = tr.loss_and_grad()
        o = {"kan": f"[{N}, 10, {N}] G={G} softsign", "P": int(p.numel()), "batch": B, "dtype": "f64",
             "rhs_us": t_rhs, "vjp_us": t_vjp, "rhs_evals_per_s": B / (t_rhs * 1e-6),
             "param_GBps_rhs": 8.0 * p.numel() / (t_rhs * 1e-6) / 1e9,
             "train_iteration_ms": it_ms, "forward_steps": sol.stats["naccept"],
             "adjoint_steps": sol.stats["adjoint"]["naccept"] if "adjoint" in sol.stats else None}
        if with_cpu:
            from oracle import oracle as O
            specs = [O.LayerSpec(N, 10, G, "softsign"), O.LayerSpec(10, N, G, "softsign")]
            tc = O.bench_chain(specs, p_np, u0, 20, 1) / 20
            o.update({"cpu_rhs_us": tc * 1e6, "cpu_cores": 1, "cpu_kind": "port (oracle chain, C)",
                      "gpu_vs_cpu_rhs": tc * 1e6 / t_rhs})
            # one training iteration on the CPU: the C epoch port (oracle/cpu_epoch.c; Tsit5 + InterpolatingAdjoint
            # + Adam over the oracle chain, pinned to the Python driver by tests/test_cpu_epoch.py), one core, the
            # same problem; a bounded sample (about a second per repetition): median of 3
            tg = np.ascontiguousarray(np.broadcast_to(0.9 * u0, (len(saveat), B, N)))
            cs = []
            for _ in range(3):
                *_, cst, csec = O.chain_epoch(specs, p_np, u0, tspan[1], saveat, tg, eta=eta)
                cs.append(csec)
            o.update({"cpu_train_iteration_ms": float(np.median(cs)) * 1e3,
                      "cpu_train_steps": [cst["naccept"], cst["adjoint_naccept"]],
                      "cpu_train_sample": "median of 3 repetitions, one core",
                      "gpu_vs_cpu_train": float(np.median(cs)) * 1e3 / it_ms})
        out[name] = o
    return out


def _surrogate_problem(name: str, B: int, seed: int):
    """Synthetic ICs and random-init parameters of the BASELINE configs[3]/[4] surrogates:
    burgers512 u0 = -sin(pi x) + sum_k a_k sin(k pi x) on [-1, 1]; schrodinger1024 u0 = A 2 sech(x)
    (cos th, sin th) on [-5, 5] as the [Re; Im] state."""
    rng = np.random.default_rng(seed)
    if name == "burgers512":
        x = np.linspace(-1.0, 1.0, 512)
        a = rng.normal(0.0, 0.1, (B, 3))
        return -np.sin(np.pi * x)[None, :] + sum(a[:, k:k + 1] * np.sin((k + 1) * np.pi * x)[None, :] for k in range(3))
    x = np.linspace(-5.0, 5.0, 1024)
    amp, th = rng.uniform(0.8, 1.2, (B, 1)), rng.uniform(0.0, 2 * np.pi, (B, 1))
    env = amp * 2.0 / np.cosh(x)[None, :]
    return np.concatenate([env * np.cos(th), env * np.sin(th)], axis=1)


def _max_over_ranks(v: float, dev, backend: str, group=None) -> float:
    import torch.distributed as tdist
    t = torch.tensor([v], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX, group=group)
    return float(t.item())


def surrogate_dist_bench(dev, rank: int, world: int, backend: str, reps: int = 2):
    """BASELINE configs[3] and [4] on their multi-GPU layouts, one training iteration each (adaptive
    Tsit5 at the default tolerances, InterpolatingAdjoint, Adam), time = max over ranks.
    bu512_tp: KAN [512, 10, 512] G=5 with the 512-point grid sharded over groups of up to 4 ranks
      (Burgers_Surrogate.jl:85-97 "grid sharded 4x"; kanode.GridShardedChainRHS: per RHS one
      all_reduce of the [10, B] hidden partials, per adjoint stage two, shard-local gradients); with
      more than 4 ranks the groups train different ICs and all-reduce their gradients across groups.
      4 ICs per group, saveat every 0.005 over (0, 1), ADAM(1e-2).
    sc1024_dp: KAN [2048, 10, 2048] G=10, one IC per rank (Schrodinger_Surrogate.jl:93-104, 8 ICs over
      8 GPUs), native solve + adjoint per rank, one all_reduce(SUM) of [dL/dp ; L] (450,561 doubles)
      per iteration, ADAM(1e-3)."""
    import torch.distributed as tdist
    out = {}
    # ---- BU512: grid-sharded over tp ranks ------------------------------------------------------
    tp_size = max(d for d in (1, 2, 3, 4) if world % d == 0)
    n_groups = world // tp_size
    tp_groups = [tdist.new_group(list(range(g * tp_size, (g + 1) * tp_size))) for g in range(n_groups)]
    dp_groups = [tdist.new_group(list(range(j, world, tp_size))) for j in range(tp_size)]
    my_tp = tp_groups[rank // tp_size]
    my_dp = dp_groups[rank % tp_size] if n_groups > 1 else None
    c1 = kanode.LayerCfg(512, 10, 5, normalizer="softsign")
    c2 = kanode.LayerCfg(10, 512, 5, normalizer="softsign")
    tp = kanode.GridShardedChainRHS(c1, c2, group=my_tp, device=dev)
    chain = kanode.Chain(kanode.KDense(512, 10, 5, normalizer="softsign"), kanode.KDense(10, 512, 5, normalizer="softsign"))
    p_full = torch.as_tensor(chain.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
    u0 = torch.as_tensor(_surrogate_problem("burgers512", 4, 5 + rank // tp_size), device=dev)
    u_loc = u0[:, tp.a:tp.b].contiguous()
    saveat = [0.005 * i for i in range(201)]
    target = (0.9 * u_loc).unsqueeze(0).expand(len(saveat), -1, -1).contiguous()
    tr = kanode.Trainer(tp, u_loc, (0.0, 1.0), saveat, target, tp.shard_params(p_full), eta=1e-2, group=my_dp,
                        tp=True)
    tr.step()
    torch.cuda.synchronize()
    tdist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        tr.step()
    torch.cuda.synchronize()
    it = _max_over_ranks((time.perf_counter() - t0) / reps, dev, backend)
    _, _, sol = tr.loss_and_grad()
    out["bu512_tp"] = {"unit": "ms/iteration", "ms_per_iteration": it * 1e3, "ranks": world,
                       "host": "Python integrator (kanode.tp) over torch.distributed",
                       "grid_shards": tp_size, "data_parallel_groups": n_groups, "ics_per_group": 4,
                       "grid_points_per_rank": tp.n, "sensealg": tr.sensealg,
                       "forward_steps": sol.stats["naccept"],
                       "collectives": "per RHS: all_reduce of [10, 4] hidden partials; per adjoint stage: two; "
                                      "per step: error-norm scalar" + ("; per iteration: gradient all_reduce "
                                                                       "across groups" if n_groups > 1 else "")}
    # ---- BU512: trajectory-sharded (SURVEY §8e E1's recommended default) --------------------------
    # every rank trains its own 4 ICs with the whole [512, 10, 512] surrogate (native solve + adjoint,
    # no collective inside the solve), one all_reduce(SUM) of [dL/dp ; L] per iteration
    rhs_dp = kanode.ChainRHS(chain, device=dev)
    u_dp = torch.as_tensor(_surrogate_problem("burgers512", 4, 500 + rank), device=dev)
    target = (0.9 * u_dp).unsqueeze(0).expand(len(saveat), -1, -1).contiguous()
    tr = kanode.Trainer(rhs_dp, u_dp, (0.0, 1.0), saveat, target, p_full, eta=1e-2, group=tdist.group.WORLD)
    tr.step()
    torch.cuda.synchronize()
    tdist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        tr.step()
    torch.cuda.synchronize()
    it = _max_over_ranks((time.perf_counter() - t0) / reps, dev, backend)
    _, _, sol = tr.loss_and_grad()
    out["bu512_dp"] = {"unit": "ms/iteration", "ms_per_iteration": it * 1e3, "ranks": world, "ics_per_rank": 4,
                       "ics_total": 4 * world, "trajectories_per_s": 4 * world / it, "sensealg": tr.sensealg,
                       "forward_steps": sol.stats["naccept"], "adjoint_steps": sol.stats["adjoint"]["naccept"],
                       "collective": f"one all_reduce(SUM) of [dL/dp ; L] ({p_full.numel() + 1} doubles) per "
                                     "iteration"}
    out["bu512_tp"]["trajectories_per_s"] = 4 * n_groups / (out["bu512_tp"]["ms_per_iteration"] * 1e-3)
    # ---- SC1024: one IC per rank, data parallel --------------------------------------------------
    N = 2048
    chain = kanode.Chain(kanode.KDense(N, 10, 10, normalizer="softsign"), kanode.KDense(10, N, 10, normalizer="softsign"))
    rhs = kanode.ChainRHS(chain, device=dev)
    p = torch.as_tensor(chain.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
    u = torch.as_tensor(_surrogate_problem("schrodinger1024", 1, 100 + rank), device=dev)
    saveat = [0.1 + 0.2 * i for i in range(8)]
    target = (0.9 * u).unsqueeze(0).expand(len(saveat), -1, -1).contiguous()
    tr = kanode.Trainer(rhs, u, (0.0, np.pi / 2), saveat, target, p, eta=1e-3, group=tdist.group.WORLD)
    tr.step()
    torch.cuda.synchronize()
    tdist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        tr.step()
    torch.cuda.synchronize()
    it = _max_over_ranks((time.perf_counter() - t0) / reps, dev, backend)
    out["sc1024_dp"] = {"unit": "ms/iteration", "ms_per_iteration": it * 1e3, "ranks": world, "ics_per_rank": 1,
                        "P": int(p.numel()), "sensealg": tr.sensealg,
                        "collective": f"one all_reduce(SUM) of [dL/dp ; L] ({p.numel() + 1} doubles) per iteration"}
    return out


LAUNCH_ENV = "KANODE_BENCH_LAUNCH"      # set by launch_ranks in the children it starts


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def resolve_world(gpus: int, env) -> tuple[str, int]:
    """How this process runs: ("single", 1), ("rank", WORLD_SIZE) under a launcher, or ("spawn", N)
    when --gpus N > 1 and nothing launched us.  Raises SystemExit when an external launcher's
    WORLD_SIZE disagrees with --gpus (the driver's `torchrun --nproc-per-node N bench.py --gpus N`
    must time N ranks, never silently fewer)."""
    if gpus < 1:
        raise SystemExit(f"--gpus {gpus}: need at least one GPU")
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return ("spawn", gpus) if gpus > 1 else ("single", 1)
    world = int(ws)
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
    return ("rank", world) if world > 1 else ("single", 1)


def launch_ranks(n: int, cmd: list[str], env=None, poll_s: float = 0.2, grace_s: float = 20.0) -> int:
    """Start n fresh processes of `cmd` as the ranks of one job (127.0.0.1 rendezvous on a free port),
    each with RANK = LOCAL_RANK = r, WORLD_SIZE = n.  Children are started, never exec'd into: this
    process has not touched the GPU and does not.  The children inherit stdout (rank 0 prints the JSON
    line).  If a rank exits non-zero the others are terminated (exact PIDs; killed after `grace_s`) so a
    rank blocked in a collective cannot hang the job.  Returns 0 when every rank succeeded, otherwise
    the first failing rank's exit status (1 for a signal)."""
    base = dict(os.environ if env is None else env)
    port = _free_port()
    procs = []
    for r in range(n):
        e = dict(base)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                  "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), LAUNCH_ENV: "self"})
        procs.append(subprocess.Popen(cmd, env=e))
    rc, live = 0, set(range(n))
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                print(f"bench.py: rank {r} exited with status {c}; stopping the other ranks", file=sys.stderr,
                      flush=True)
                for q in live:
                    procs[q].terminate()
                t_end = time.time() + grace_s
                for q in live:
                    try:
                        procs[q].wait(timeout=max(0.1, t_end - time.time()))
                    except subprocess.TimeoutExpired:
                        procs[q].kill()
                        procs[q].wait()
                live.clear()
        if live:
            time.sleep(poll_s)
    return rc


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="fisher_kpp_256", choices=["fisher_kpp_256"])
    ap.add_argument("--batch-total", type=int, default=1048576,
                    help="trajectories over all ranks (strong scaling; must divide by the world size)")
    ap.add_argument("--batch-per-gpu", type=int, default=0, help="weak scaling: trajectories per rank")
    ap.add_argument("--cpu-seconds", type=float, default=40.0,
                    help="CPU-baseline budget; the calibrated sample lands near 1/3 of it (~10-15 s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-vjp", action="store_true")
    ap.add_argument("--no-epoch", action="store_true")
    ap.add_argument("--no-epoch-adaptive", action="store_true",
                    help="skip the adaptive reference-problem epoch (T = 5, default tolerances)")
    ap.add_argument("--no-dist-surrogates", action="store_true",
                    help="skip the multi-rank configs[3]/[4] training legs (N > 1 only)")
    ap.add_argument("--epoch-batch", type=int, default=4096, help="trajectories in the training-epoch leg")
    ap.add_argument("--epoch-steps", type=int, default=50, help="fixed Tsit5 steps per epoch (dt = 1e-3)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) for one rank per GPU; gloo only to rehearse the multi-rank path")
    ap.add_argument("--no-table", action="store_true",
                    help="per-point basis recurrence instead of the piecewise-polynomial table (kan_pp.hip)")
    ap.add_argument("--no-shard-ceiling", action="store_true",
                    help="skip the single-GPU shard_ceiling projection (its smaller-batch launches of the same kernel "
                         "would mix into a kernel-trace summary of the 1M-trajectory launch)")
    ap.add_argument("--grid-rhs", type=int, default=0,
                    help="tuning: persistent grid of the table RHS kernel (KANODE_OPT_GRID_RHS; 0 = default)")
    args = ap.parse_args()

    mode, world = resolve_world(args.gpus, os.environ)
    if mode == "spawn":
        # nothing in this process has touched the GPU: the ranks are fresh children of this script
        raise SystemExit(launch_ranks(world, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()) if dist else 0)
    torch.cuda.set_device(dev)
    rccl_world = None
    json_out = sys.stdout
    if dist:
        # the collective libraries print connection chatter to the process's stdout: route fd 1 to stderr and
        # keep a private handle on the real stdout for the one JSON line
        sys.stdout.flush()
        json_out = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
        import datetime
        import torch.distributed as tdist
        # a rank that dies inside a collective must not hang the others forever
        tmo = datetime.timedelta(minutes=10)
        if args.dist_backend == "nccl":
            tdist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            tdist.init_process_group("gloo", timeout=tmo)
        rccl_world = tdist.get_world_size()
        if rccl_world != world:
            raise SystemExit(f"bench.py: process group has {rccl_world} ranks, expected {world}")

    nx, D = 256, 0.01
    dx = 1.0 / (nx - 1)
    weak = args.batch_per_gpu > 0
    if weak:
        B = args.batch_per_gpu
    else:
        if args.batch_total % world:
            raise SystemExit(f"--batch-total {args.batch_total} does not divide by {world} ranks")
        B = args.batch_total // world
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign", basis_func="rbf"))
    rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=dx, D=D, dtype=torch.float64, device=dev,
                              table=False if args.no_table else None)
    table = rhs.hd.pointwise_table
    if args.grid_rhs:
        rhs.hd.set_option("grid_rhs", args.grid_rhs)
    p_np = kan1.setup(np.random.default_rng(0))[0].astype(np.float64)
    p = torch.as_tensor(p_np, device=dev)
    u = fk_ics(B, nx, dx, seed=1000 + rank, device=dev)
    du = torch.empty_like(u)
    rhs.hd.reserve(B)

    # The table build (fk_pp_build_kernel) skips its work when p equals the parameters of the last
    # build bit for bit (within a solve p is constant).  Each timed step here is a standalone RHS
    # evaluation, so it alternates between two parameter vectors that differ in the last bits and
    # every step rebuilds the table: the measured step is the full build + RHS.
    p_alt = p * (1.0 + 2.0 ** -40)
    ps = (p, p_alt)
    for i in range(args.warmup):
        rhs.rhs(u, ps[i & 1], du)
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)
    # one HIP-event pair on the launch stream brackets the timed steps: kernel_ms = its time / steps
    # (build + RHS kernel and the boundaries between them).  Timing events around every step put two
    # extra packets per step on the stream (measured: ~5 us/step of bubbles at 131,072 trajectories).
    e_beg, e_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e_beg.record(stream)
    for i in range(args.steps):
        rhs.rhs(u, ps[(args.warmup + i) & 1], du)
    e_end.record(stream)
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    rank_elapsed = [elapsed]
    if dist:
        cdev = dev if args.dist_backend == "nccl" else "cpu"
        mine = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        allt = [torch.zeros_like(mine) for _ in range(world)]
        tdist.all_gather(allt, mine)
        rank_elapsed = [float(t.item()) for t in allt]
        elapsed = max(rank_elapsed)
    kern_ms = e_beg.elapsed_time(e_end) / args.steps
    # this box's streaming reference: a device copy moving the same bytes (u -> du)
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    du.copy_(u)
    c0.record(stream)
    for _ in range(5):
        du.copy_(u)
    c1.record(stream)
    torch.cuda.synchronize()
    copy_gbps = 16.0 * B * nx / (c0.elapsed_time(c1) / 5 * 1e-3) / 1e9

    total_evals = B * args.steps * world
    value = total_evals / elapsed
    ceiling = None
    if world == 1 and not weak and not args.no_shard_ceiling:
        ceiling = shard_ceiling(rhs, u, du, ps, stream, args.steps, B / (kern_ms * 1e-3))
    alg_bytes = 8.0 * (rhs.P + B * (nx + nx))       # p + u in + du out, per launch
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = load_traffic(f"{args.workload}:{'table' if table else 'recurrence'}", alg_bytes)

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "RHS-evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (reference IC family randomised per trajectory; random-init KAN params)",
        "config": {"workload": "fisher_kpp_256", "nx": nx, "batch_total": B * world, "batch_per_gpu": B,
                   "kan": "KDense(1,1,10) softsign rbf",
                   "kan_eval": "piecewise-polynomial table" if table else "basis recurrence",
                   "parallelism": f"trajectory-sharded x{world} (no data-path collective)"},
        "rccl_world": rccl_world,
        "dist_backend": args.dist_backend if dist else None,
        "launch": ("self-spawned ranks (bench.py --gpus)" if os.environ.get(LAUNCH_ENV) == "self"
                   else "external launcher (WORLD_SIZE)") if dist else "single process",
        "rank_timed_s": rank_elapsed,
        "shard_ceiling": ceiling,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": ("fk_pp_build_kernel + fk_rhs_pp_wave_kernel<SOFTSIGN,RBF,2>" if table
                                else "fk_rhs_kernel<double,SOFTSIGN,REC_CORR,10>"),
                     "kernel_ms": kern_ms,
                     "alg_bytes_per_launch": alg_bytes,
                     "torch_copy_GBps": copy_gbps},
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

    if rank == 0 and not args.no_vjp:
        out["lv4096"] = lv4096_bench(dev)
        out["lv1_train"] = lv1_train_bench(dev, world == 1 and not args.no_cpu_baseline)
        out["lv4096_train"] = lv4096_train_bench(dev, world == 1 and not args.no_cpu_baseline)
        out["fk26_train"] = fk26_train_bench(dev, world == 1 and not args.no_cpu_baseline)
        out["surrogates"] = surrogate_bench(dev, world == 1 and not args.no_cpu_baseline)

    if not args.no_epoch:
        ep = epoch_bench(dev, p_np, nx, dx, D, args.epoch_batch, 0 if (args.no_cpu_baseline or world > 1) else 16,
                         args.epoch_steps, 1e-3, 3, group=tdist.group.WORLD if dist else None, rank=rank,
                         world=world)
        if rank == 0:
            out["epoch"] = ep
        if rank == 0 and not args.no_epoch_adaptive:
            out["epoch_adaptive"] = epoch_adaptive_bench(dev, fk_trained_like_params(), nx, dx, D, args.epoch_batch,
                                                         0 if (args.no_cpu_baseline or world > 1) else 2)

    if dist and not args.no_dist_surrogates:
        # a secondary leg: an exception here is recorded in the line instead of taking the metric above
        # down with it.  Every rank then all-reduces a failure flag before any further collective, so a
        # rank that failed alone (an allocation, a HIP error on one GPU) does not leave the others
        # waiting; a rank that dies inside one of the leg's collectives ends at the process-group timeout
        # and the launcher stops the job.
        err = None
        try:
            sd = surrogate_dist_bench(dev, rank, world, args.dist_backend)
        except Exception as e:  # noqa: BLE001
            err = f"rank {rank}: {type(e).__name__}: {e}"[:300]
            sd = {}
        flag = torch.tensor([1.0 if err else 0.0], dtype=torch.float64,
                            device=dev if args.dist_backend == "nccl" else "cpu")
        tdist.all_reduce(flag, op=tdist.ReduceOp.MAX)
        if float(flag.item()) > 0:
            sd = {"dist_surrogates_error": err or "failed on another rank"}
        if rank == 0:
            out.update(sd)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(nx, dx, D, p_np, args.cpu_seconds)
        out["cpu_baseline"] = cb
        out["gpu_vs_cpu"] = value / cb["value"]

    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
