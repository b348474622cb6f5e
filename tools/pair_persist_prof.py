#!/usr/bin/env python3
"""Phase profile of the persistent pair adjoint (kd_pair_adjoint_kernel built with -DKAN_PA_PROF, e.g.
`tools/build_var.sh paprof -DKAN_PA_PROF kan_pair_adj.hip`, run with KANODE_LIB=tools/bin/var/paprof.so):
one Burgers [512, 10, 512] training-iteration adjoint; prints workgroup 0's wall time per phase."""
import ctypes
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

PHASES = ["controller (between stage evaluations)", "dense-output load", "y + layer-1 basis + partial A",
          "exchange A", "layer-2 basis", "partial B + dC2", "exchange B", "x̄ + dC1", "step tail (μ, error terms)",
          "error exchange", "final"]


def main():
    dev = torch.device("cuda", 0)
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    N, G, B, tspan, saveat, eta = 512, 5, 4, (0.0, 1.0), [0.005 * i for i in range(201)], 1e-2
    chain = kanode.Chain(kanode.KDense(N, 10, G, normalizer="softsign"), kanode.KDense(10, N, G, normalizer="softsign"))
    rhs = kanode.ChainRHS(chain, device=dev)
    rhs.hd.set_option("pair_persist", 1)
    rhs.hd.set_option("pair_persist_s", S)
    p = torch.as_tensor(chain.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
    u = torch.as_tensor(_surrogate_problem("burgers512", B, 5), device=dev)
    target = (0.9 * u).unsqueeze(0).expand(len(saveat), -1, -1).contiguous()
    tr = kanode.Trainer(rhs, u, tspan, saveat, target, p, eta=eta)
    _, _, sol = tr.loss_and_grad()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, _, sol = tr.loss_and_grad()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    out = (ctypes.c_double * 16)()
    rc = kanode.lib().kanode_debug_pair_profile(out)
    st = sol.stats["adjoint"]
    print(f"S={S}: loss_and_grad {wall * 1e3:.2f} ms; adjoint steps {st['naccept']} rejects {st['nreject']} "
          f"evaluations {st['nf']} (rc {rc})")
    tot = sum(out[i] for i in range(len(PHASES)))
    if tot <= 0:
        print("  (the persistent adjoint did not run for this shape: the launch path took it)")
        return
    for i, name in enumerate(PHASES):
        print(f"  {name:42s} {out[i] / 1e3:8.3f} ms  {out[i] / max(1, st['nf']):7.2f} us/eval  {100 * out[i] / tot:5.1f} %")


if __name__ == "__main__":
    main()
