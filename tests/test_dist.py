"""Multi-process (gloo, world_size 2) check of the distributed training step
(SURVEY §8e): trajectories shard across ranks, ONE all-reduce of [∂L/∂p ; L] per
step, identical Adam update on every rank.  CPU + pure-torch RHS (the collective
logic is what is under test; the HIP RHS plugs into the same Trainer)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import kanode


def lotka(u, p, t):
    x, y = u[..., 0], u[..., 1]
    return torch.stack([p[0] * x - p[1] * x * y, p[2] * x * y - p[3] * y], dim=-1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _shard(rank):
    ptrue = torch.tensor([1.5, 1.0, 1.0, 3.0], dtype=torch.float64)
    g = torch.Generator().manual_seed(100 + rank)
    u0 = (0.8 + 0.4 * torch.rand(4, 2, generator=g, dtype=torch.float64))
    ts = [0.1 * i for i in range(10)]
    target = kanode.solve(lotka, u0, (0.0, 1.0), ptrue, saveat=ts,
                          opt=kanode.Tsit5Options(abstol=1e-10, reltol=1e-10)).u
    return u0, ts, target, ptrue * 1.2


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    u0, ts, target, p0 = _shard(rank)
    tr = kanode.Trainer(lotka, u0, (0.0, 1.0), ts, target, p0, eta=1e-2, group=dist.group.WORLD)
    losses = [tr.step() for _ in range(3)]
    q.put((rank, tr.p.numpy(), losses))
    dist.destroy_process_group()


def test_gloo_two_ranks_identical_params_and_mean_gradient():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = dict((r, (p, l)) for r, p, l in (q.get(timeout=120) for _ in range(world)))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    # every rank holds the same parameters and the same (all-reduced) loss history
    assert np.array_equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1]
    # single-process reference: mean of the per-shard gradients and losses, same Adam
    trs = []
    for r in range(world):
        u0, ts, target, p0 = _shard(r)
        trs.append(kanode.Trainer(lotka, u0, (0.0, 1.0), ts, target, p0, eta=1e-2))
    p = trs[0].p.clone()
    opt = kanode.Adam(1e-2)
    ref_losses = []
    for _ in range(3):
        gl = []
        for tr in trs:
            tr.p = p.clone()
            gl.append(tr.loss_and_grad()[:2])
        g = sum(x[1] for x in gl) / world
        ref_losses.append(float(sum(x[0] for x in gl) / world))
        opt.update(p, g)
    assert np.allclose(res[0][0], p.numpy(), rtol=1e-12, atol=1e-14)
    assert np.allclose(res[0][1], ref_losses, rtol=1e-12)
