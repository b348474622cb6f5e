#!/usr/bin/env python3
"""Device time of one Fisher-KPP adjoint stage (kanode_vjp_stage: forward dense-output
interpolation + adjoint stage input + VJP + reductions) against the plain VJP, by batch,
number of interpolated arrays and grid (KANODE_OPT_GRID_VJP), from hipGraphs of back-to-back calls.

    python3 tools/stage_ab.py [--batch 4096]
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


def graph_time(fn, reps=40):
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
    ap.add_argument("--batch", type=int, nargs="+", default=[1024, 4096, 16384])
    ap.add_argument("--grids", type=int, nargs="+", default=[0])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
    fk = kanode.FisherKPPRHS(kan1, nx=256, dx=1 / 255, D=0.01, device=dev)
    p = torch.as_tensor(kan1.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
    for B in args.batch:
        u = fk_ics(B, 256, 1 / 255, 7, dev)
        ks = [torch.randn_like(u) * 1e-2 for _ in range(7)]
        lam = torch.randn_like(u)
        lks = [torch.randn_like(u) * 1e-2 for _ in range(6)]
        lam_out = torch.empty_like(u)
        sumsq = torch.zeros(1, dtype=torch.float64, device=dev)
        dp = torch.zeros_like(p)
        fk.hd.reserve(B)
        mb = B * 256 * 8 / 1e6
        for grid in args.grids:
            fk.hd.set_option("grid_vjp", grid or 0)
            t_vjp = graph_time(lambda: fk.hd.vjp(p, u, lam, dp=dp))
            row = [f"B={B:6d} grid={grid or 'auto':>5}  vjp {t_vjp:7.2f} us ({3 * mb / t_vjp:5.2f} TB/s)"]
            for nu, nl, err in ((0, 0, False), (7, 0, False), (7, 3, True), (7, 6, True)):
                c = [1e-3] * nu
                lc = [1e-3] * nl
                ec = [1e-4] * (nl + 1)
                t = graph_time(lambda: fk.hd.vjp_stage(p, u, ks[:nu], c, lam, lks[:nl], lc, lam_out=lam_out if nl else None,
                                                     error=(ec, 1e-6, 1e-3, sumsq) if err else None, dp=dp))
                arrays = 3 + nu + nl + (1 if nl else 0)
                row.append(f"stage u+{nu} l+{nl}{'e' if err else ' '} {t:7.2f} us ({arrays * mb / t:5.2f} TB/s)")
            y = torch.empty_like(u)
            for nk in (1, 6):
                ec = [1e-4] * (nk + 1)
                t = graph_time(lambda: fk.hd.rhs_stage(p, u, ks[:nk], [1e-3] * nk, y_out=y if nk == 6 else None,
                                                       error=(ec, 1e-6, 1e-3, sumsq) if nk == 6 else None))
                row.append(f"fwd stage nk={nk} {t:7.2f} us")
            print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
