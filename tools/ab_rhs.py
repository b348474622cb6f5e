#!/usr/bin/env python3
"""Interleaved A/B timing of Fisher-KPP RHS library variants in ONE process.

Each .so given is loaded through its own ctypes handle (separate copies of the
library), so box-to-box clock/thermal variance cancels: rounds alternate over
(variant, grid) and the median per cell is reported, next to a torch copy of the
same bytes (u -> du) as the streaming reference.

    python3 tools/ab_rhs.py --batch 1048576 --grids 0,1536,1792 tools/bin/var/*.so
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kan-odes_amd"))
sys.path.insert(0, ROOT)

from kanode import _lib as L  # noqa: E402  (structs only)
from bench import fk_ics  # noqa: E402


def load(path):
    lib = C.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL)
    for name, res, args in L.SIGNATURES:
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
    return lib


def fk_handle(lib, nx, dx, D):
    spec = L.SpecC()
    spec.n_layers = 1
    spec.layers[0] = L.LayerSpecC(1, 1, 10, L.NORM["softsign"], L.BASIS["rbf"], 1, -1.0, 1.0, 0.0, 1)
    spec.dtype = L.F64
    spec.rhs_kind = L.RHS_POINTWISE_PERIODIC_LAPLACIAN
    spec.nx, spec.diffusion, spec.dx, spec.device = nx, D, dx, 0
    h = C.c_void_p()
    assert lib.kanode_create(C.byref(spec), C.byref(h)) == 0
    return h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--batch", type=int, default=1048576)
    ap.add_argument("--grids", default="0")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--op", default="rhs", choices=["rhs", "vjp"], help="kanode_rhs or kanode_vjp")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    nx, dx, D = 256, 1 / 255, 0.01
    u = fk_ics(a.batch, nx, dx, 1, dev)
    du = torch.empty_like(u)
    lam = torch.randn_like(u) if a.op == "vjp" else None
    dp = torch.zeros(11, dtype=torch.float64, device=dev)
    p = torch.as_tensor(np.random.default_rng(0).uniform(-1, 1, 11), device=dev)
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    libs = [(os.path.basename(x).replace(".so", ""), load(x)) for x in a.libs]
    hs = {n: fk_handle(lib, nx, dx, D) for n, lib in libs}
    grids = [int(g) for g in a.grids.split(",")]
    cells = {}
    ref = None
    nbytes = 8.0 * (11 + 2 * a.batch * nx) if a.op == "rhs" else 8.0 * (22 + 3 * a.batch * nx)
    for r in range(a.rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(2):
            du.copy_(u)
        e0.record()
        for _ in range(a.reps):
            du.copy_(u)
        e1.record()
        torch.cuda.synchronize()
        cells.setdefault(("torch_copy", 0), []).append(e0.elapsed_time(e1) / a.reps)
        for n, lib in libs:
            for g in grids:
                assert lib.kanode_set_option(hs[n], 6 if a.op == "vjp" else 5, g) == 0   # KANODE_OPT_GRID_VJP / _RHS
                if a.op == "rhs":
                    call = lambda: lib.kanode_rhs(hs[n], C.c_void_p(p.data_ptr()), C.c_void_p(u.data_ptr()),  # noqa: E731
                                                  C.c_void_p(du.data_ptr()), a.batch, st)
                else:
                    call = lambda: lib.kanode_vjp(hs[n], C.c_void_p(p.data_ptr()), C.c_void_p(u.data_ptr()),  # noqa: E731
                                                  C.c_void_p(lam.data_ptr()), C.c_void_p(du.data_ptr()),
                                                  C.c_void_p(dp.data_ptr()), a.batch, st)
                for _ in range(2):
                    assert call() == 0
                e0.record()
                for _ in range(a.reps):
                    call()
                e1.record()
                torch.cuda.synchronize()
                cells.setdefault((n, g), []).append(e0.elapsed_time(e1) / a.reps)
                if ref is None:
                    ref = du.clone()
                else:
                    assert torch.equal(du, ref), f"{n} grid {g}: output differs"
    for (n, g), v in cells.items():
        ms = float(np.median(v))
        print(f"{n:14s} grid {g:5d}  {ms * 1e3:8.1f} us  {nbytes / ms / 1e6:7.0f} GB/s  frac {nbytes / ms / 1e6 / 8000:.3f}"
              f"  (min {min(v) * 1e3:.1f}, max {max(v) * 1e3:.1f})", flush=True)


if __name__ == "__main__":
    main()
