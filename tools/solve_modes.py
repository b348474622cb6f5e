#!/usr/bin/env python3
"""Forward-solve wall time per step control mode (kanode_solve_tsit5 control = host / device /
auto: auto runs a small chain of <= 16 trajectories as one workgroup),
with and without the dense output kept, for a few problem sizes.

    python3 tools/solve_modes.py
"""
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
    dev = torch.device("cuda:0")
    cases = []
    chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
    lv = kanode.ChainRHS(chain, device=dev)
    plv = torch.as_tensor(chain.setup(np.random.default_rng(0))[0].astype(np.float64) / 10, device=dev)
    for B in (1, 16, 4096):
        cases.append((f"lv B={B}", lv, torch.ones(B, 2, dtype=torch.float64, device=dev), plv, (0.0, 3.5),
                      [0.1 * i for i in range(35)], 0.01))
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
    fk = kanode.FisherKPPRHS(kan1, nx=256, dx=1 / 255, D=0.01, device=dev)
    pfk = torch.as_tensor(kan1.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
    for B in (256, 4096):
        cases.append((f"fk256 B={B}", fk, fk_ics(B, 256, 1 / 255, 7, dev), pfk, (0.0, 0.05),
                      [0.01 * i for i in range(6)], 1e-3))
    for name, rhs, u0, p, tspan, ts, dt in cases:
        for adaptive in (True, False):
            for keep in (False, True):
                row = []
                for control in ("host", "device", "auto"):
                    opt = kanode.Tsit5Options(adaptive=adaptive, dt=None if adaptive else dt, control=control).to_c()
                    dense = None
                    for it in range(4):
                        if it == 1:
                            torch.cuda.synchronize()
                            t0 = time.perf_counter()
                        _, st, dense_new = rhs.hd.solve_tsit5(p, u0, tspan[0], tspan[1], ts, opt, keep_dense=keep)
                        if keep:
                            rhs.hd.release_dense(dense_new)
                    torch.cuda.synchronize()
                    row.append((time.perf_counter() - t0) / 3 * 1e3)
                print(f"{name:14s} {'adaptive' if adaptive else 'fixed   '} {'dense' if keep else '     '} "
                      f"steps {st['naccept']:4d}  host {row[0]:7.2f} ms  device {row[1]:7.2f} ms  auto {row[2]:7.2f} ms",
                      flush=True)


if __name__ == "__main__":
    main()
