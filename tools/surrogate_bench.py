#!/usr/bin/env python3
"""Device time per RHS / VJP call of the full-field surrogate chains (BASELINE configs[3], [4]):
Burgers KAN [512, 10, 512] G=5 and Schrodinger KAN [2048, 10, 2048] G=10 (softsign, fp64), at
small batches, from hipGraphs of back-to-back calls (launch-bound sizes).

    python3 tools/surrogate_bench.py [--only burgers512:64]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kan-odes_amd"))

import kanode  # noqa: E402


def graph_time(fn, reps=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None, help="name:B, e.g. burgers512:64")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cases = (("burgers512", 512, 5, (1, 4, 64)), ("schrodinger1024", 2048, 10, (1, 8)))
    if args.only:
        nm, b = args.only.split(":")
        cases = tuple((n, N, G, (int(b),)) for n, N, G, _ in cases if n == nm)
    for name, N, G, Bs in cases:
        chain = kanode.Chain(kanode.KDense(N, 10, G, normalizer="softsign"), kanode.KDense(10, N, G, normalizer="softsign"))
        rhs = kanode.ChainRHS(chain, device=dev)
        p = torch.as_tensor(chain.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
        for B in Bs:
            u = torch.rand(B, N, dtype=torch.float64, device=dev)
            lam = torch.randn_like(u)
            du, lamJ, dp = torch.empty_like(u), torch.empty_like(u), torch.zeros_like(p)
            rhs.hd.reserve(B)
            t_rhs = graph_time(lambda: rhs.hd.rhs(p, u, du))
            t_vjp = graph_time(lambda: rhs.hd.vjp(p, u, lam, dp=dp))
            pbytes = 8 * p.numel()
            print(f"{name:16s} B={B:3d}  P={p.numel():7d}  rhs {t_rhs:7.2f} us  vjp {t_vjp:7.2f} us  "
                  f"(params {pbytes / 1e6:.2f} MB: {pbytes / t_rhs / 1e3:.0f} GB/s rhs)", flush=True)


if __name__ == "__main__":
    main()
