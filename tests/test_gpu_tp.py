"""Grid-sharded Burgers surrogate (BASELINE configs[3]: KAN [512, 10, 512], G = 5, softsign)
on the HIP layers: two or four ranks (BASELINE's "grid sharded 4x") share cuda:0 and exchange the hidden partials through gloo
(host-staged; backend "nccl" = RCCL is the same call on a multi-GPU node), against the
unsharded HIP chain and the CPU oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gpu_util import device, t
from oracle import oracle as O

import kanode
from kanode.tp import GridShardedChainRHS

pytestmark = pytest.mark.gpu

N, H, G, B = 512, 10, 5, 4
TS = [0.0, 0.05, 0.1]


def _cfgs():
    return (kanode.LayerCfg(N, H, G, normalizer="softsign"), kanode.LayerCfg(H, N, G, normalizer="softsign"))


def _problem():
    rng = np.random.default_rng(3)
    x = np.linspace(-1, 1, N)
    u0 = np.stack([-np.sin(np.pi * x) + sum(rng.normal(0, 0.1) * np.sin(k * np.pi * x) for k in (1, 2, 3))
                   for _ in range(B)])
    c1, c2 = _cfgs()
    lim1 = np.sqrt(6.0 / (H + G * N))
    lim2 = np.sqrt(6.0 / (N + G * H))
    p = np.concatenate([rng.uniform(-lim1, lim1, c1.param_length), rng.uniform(-lim2, lim2, c2.param_length)])
    w = rng.normal(size=(len(TS), B, N))
    return u0, p, w


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        c1, c2 = _cfgs()
        tp = GridShardedChainRHS(c1, c2, device=dev)
        u0, p, w = _problem()
        a, b = tp.a, tp.b
        u = torch.as_tensor(u0[:, a:b].copy(), device=dev)
        pl = tp.shard_params(torch.as_tensor(p, device=dev))
        out = {"rank": rank, "a": a, "b": b, "rhs": tp(u, pl).cpu().numpy()}
        plr = pl.clone().requires_grad_(True)
        sol = kanode.solve(tp, u, (0.0, 0.1), plr, TS, kanode.Tsit5Options(abstol=1e-8, reltol=1e-8))
        (g,) = torch.autograd.grad((sol.u * torch.as_tensor(w[:, :, a:b].copy(), device=dev)).sum(), [plr])
        out.update(sol=sol.u.detach().cpu().numpy(), naccept=sol.stats["naccept"],
                   grad=tp.gather_params(g).cpu().numpy())
        # InterpolatingAdjoint at fixed steps (vjp_stage: kanode_layer_forward_stage forming y and λs,
        # two hidden all-reduces, kanode_layer_vjp x 2 per adjoint stage)
        plf = pl.clone().requires_grad_(True)
        solf = kanode.solve(tp, u, (0.0, 0.1), plf, TS, kanode.Tsit5Options(adaptive=False, dt=0.005),
                            sensealg="interpolating_adjoint")
        (gf,) = torch.autograd.grad((solf.u * torch.as_tensor(w[:, :, a:b].copy(), device=dev)).sum(), [plf])
        out.update(grad_ia=tp.gather_params(gf).cpu().numpy(), stats_ia=dict(solf.stats))
        # adaptive InterpolatingAdjoint: the per-step error terms reduced on the device (reduce_dev)
        pla = pl.clone().requires_grad_(True)
        sola = kanode.solve(tp, u, (0.0, 0.1), pla, TS, kanode.Tsit5Options(abstol=1e-8, reltol=1e-8),
                            sensealg="interpolating_adjoint")
        (ga,) = torch.autograd.grad((sola.u * torch.as_tensor(w[:, :, a:b].copy(), device=dev)).sum(), [pla])
        out.update(sol_a=sola.u.detach().cpu().numpy(), grad_a=tp.gather_params(ga).cpu().numpy(),
                   stats_a=dict(sola.stats))
        q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_grid_sharded_burgers_on_hip_layers(world):
    dev = device()
    u0, p, w = _problem()
    c1, c2 = _cfgs()
    specs = [O.LayerSpec(N, H, G, "softsign"), O.LayerSpec(H, N, G, "softsign")]
    full = kanode.ChainRHS(kanode.Chain(kanode.KDense(N, H, G, normalizer="softsign"),
                                        kanode.KDense(H, N, G, normalizer="softsign")), device=dev)
    ref_rhs = O.chain_fwd(specs, p, u0)
    pr = t(p).requires_grad_(True)
    sol = kanode.solve(full, t(u0), (0.0, 0.1), pr, TS, kanode.Tsit5Options(abstol=1e-8, reltol=1e-8),
                       sensealg="discrete")
    (g,) = torch.autograd.grad((sol.u * t(w)).sum(), [pr])
    pf = t(p).requires_grad_(True)
    solf = kanode.solve(full, t(u0), (0.0, 0.1), pf, TS, kanode.Tsit5Options(adaptive=False, dt=0.005),
                        sensealg="interpolating_adjoint")
    (gf,) = torch.autograd.grad((solf.u * t(w)).sum(), [pf])
    pa = t(p).requires_grad_(True)
    sola = kanode.solve(full, t(u0), (0.0, 0.1), pa, TS, kanode.Tsit5Options(abstol=1e-8, reltol=1e-8),
                        sensealg="interpolating_adjoint")
    (ga,) = torch.autograd.grad((sola.u * t(w)).sum(), [pa])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr_ in procs:
        pr_.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for pr_ in procs:
        pr_.join(timeout=60)
        assert pr_.exitcode == 0
    scale = np.abs(O.chain_fwd(specs, np.abs(p), u0)).max()
    for r in res:
        a, b = r["a"], r["b"]
        assert np.max(np.abs(r["rhs"] - ref_rhs[:, a:b])) <= 1e-12 * scale
        assert r["naccept"] == sol.stats["naccept"]
        assert np.max(np.abs(r["sol"] - sol.u.detach().cpu().numpy()[:, :, a:b])) <= 1e-10
        gn = g.cpu().numpy()
        assert np.max(np.abs(r["grad"] - gn)) <= 1e-8 * np.abs(gn).max()
        # the sharded InterpolatingAdjoint (Python driver, HIP layer VJPs) against the native one of the
        # unsharded chain (kanode_adjoint_tsit5): same steps, the gradient to the sums' rounding
        assert r["stats_ia"]["adjoint"]["naccept"] == solf.stats["adjoint"]["naccept"]
        gfn = gf.cpu().numpy()
        assert np.max(np.abs(r["grad_ia"] - gfn)) <= 1e-10 * np.abs(gfn).max()
        # adaptive: the sharded forward (fused stages) and adjoint take the unsharded native solve's steps
        assert r["stats_a"]["naccept"] == sola.stats["naccept"]
        assert r["stats_a"]["adjoint"]["naccept"] == sola.stats["adjoint"]["naccept"]
        assert np.max(np.abs(r["sol_a"] - sola.u.detach().cpu().numpy()[:, :, a:b])) <= 1e-10
        gan = ga.cpu().numpy()
        assert np.max(np.abs(r["grad_a"] - gan)) <= 1e-8 * np.abs(gan).max()
