#!/usr/bin/env python3
"""A/B of the persistent surrogate-pair adjoint (KANODE_OPT_PAIR_PERSIST) on the bench's training iteration:
Burgers KAN [512, 10, 512] G=5, 4 ICs, saveat every 0.005 over (0, 1), ADAM(1e-2) (bench.py surrogate_bench),
interleaved rounds in one process; prints per-round ms per iteration, step counts and the gradient difference."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kan-odes_amd"))
sys.path.insert(0, ROOT)
import kanode  # noqa: E402
from bench import _surrogate_problem  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    name = sys.argv[1] if len(sys.argv) > 1 else "burgers512"
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    if name == "burgers512":
        N, G, B, tspan, saveat, eta = 512, 5, 4, (0.0, 1.0), [0.005 * i for i in range(201)], 1e-2
    else:
        N, G, B, tspan, saveat, eta = 2048, 10, 8, (0.0, np.pi / 2), [0.1 + 0.2 * i for i in range(8)], 1e-3
    chain = kanode.Chain(kanode.KDense(N, 10, G, normalizer="softsign"), kanode.KDense(10, N, G, normalizer="softsign"))
    rhs = kanode.ChainRHS(chain, device=dev)
    p = torch.as_tensor(chain.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
    u = torch.as_tensor(_surrogate_problem(name, B, 5), device=dev)
    target = (0.9 * u).unsqueeze(0).expand(len(saveat), -1, -1).contiguous()
    rhs.hd.set_option("pair_persist_s", S)
    grads = {}
    for mode in (0, 1):
        rhs.hd.set_option("pair_persist", mode)
        tr = kanode.Trainer(rhs, u, tspan, saveat, target, p, eta=eta)
        loss, g, sol = tr.loss_and_grad()
        grads[mode] = (g, sol.stats)
    g0, s0 = grads[0]
    g1, s1 = grads[1]
    print(f"{name} S={S}: steps fwd {s0['naccept']} adj {s0['adjoint']['naccept']}/{s1['adjoint']['naccept']} "
          f"rej {s0['adjoint']['nreject']}/{s1['adjoint']['nreject']}, max|dg|/max|g| = "
          f"{(g1 - g0).abs().max().item() / g0.abs().max().item():.3e}", flush=True)
    for r in range(rounds):
        for mode in (0, 1):
            rhs.hd.set_option("pair_persist", mode)
            tr = kanode.Trainer(rhs, u, tspan, saveat, target, p, eta=eta)
            tr.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                tr.step()
            torch.cuda.synchronize()
            print(f"round {r} persist={mode}: {(time.perf_counter() - t0) / 3 * 1e3:.2f} ms/iteration", flush=True)


if __name__ == "__main__":
    main()
