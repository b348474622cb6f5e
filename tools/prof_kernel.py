#!/usr/bin/env python3
"""Run one hot kernel repeatedly (for rocprofv3 --kernel-trace / --pmc passes).

    python3 tools/prof_kernel.py --what fk_rhs --batch 131072 --reps 20
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kan-odes_amd"))
sys.path.insert(0, ROOT)

import kanode  # noqa: E402
from bench import fk_ics  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="fk_rhs", choices=["fk_rhs", "fk_rhs_rec", "fk_vjp", "lv_rhs", "lv_vjp"])
    ap.add_argument("--batch", type=int, default=131072)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    if a.what.startswith("fk"):
        nx, dx = 256, 1 / 255
        kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
        rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=dx, D=0.01, device=dev,
                                  table=False if a.what == "fk_rhs_rec" else None)
        p = torch.as_tensor(kan1.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
        u = fk_ics(a.batch, nx, dx, 1, dev)
    else:
        chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
        rhs = kanode.ChainRHS(chain, dtype=torch.float32, device=dev)
        p = torch.as_tensor(chain.setup(np.random.default_rng(0))[0], device=dev)
        u = (0.5 + 1.5 * torch.rand(a.batch, 2, device=dev)).contiguous()
    out = torch.empty_like(u)
    lam = torch.randn_like(u)
    dp = torch.zeros_like(p)
    rhs.hd.reserve(a.batch)
    for _ in range(a.reps):
        if "rhs" in a.what:
            rhs.rhs(u, p, out)
        else:
            rhs.hd.vjp(p, u, lam, dp=dp)
    torch.cuda.synchronize()
    print("done", a.what, a.batch, a.reps)


if __name__ == "__main__":
    main()
