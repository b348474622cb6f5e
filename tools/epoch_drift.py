#!/usr/bin/env python3
"""Wall time of consecutive adaptive reference epochs (bench.py epoch_adaptive's problem) with Adam(1e-2) and with
eta = 0 (p fixed): does the epoch slow down as the parameters move?   python3 tools/epoch_drift.py"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import bench  # noqa: E402
import kanode  # noqa: E402

dev = torch.device("cuda:0")
nx = 256
dx = 1 / (nx - 1)
etas = [float(x) for x in sys.argv[1:]] or [1e-2, 0.0]
for eta in etas:
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign", basis_func="rbf"))
    rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=dx, D=0.01, dtype=torch.float64, device=dev)
    u0 = bench.fk_ics(4096, nx, dx, seed=17, device=dev)
    saveat = [0.5 * i for i in range(11)]
    target = (0.9 * u0).unsqueeze(0).expand(len(saveat), -1, -1).contiguous()
    tr = kanode.Trainer(rhs, u0, (0.0, 5.0), saveat, target, torch.as_tensor(bench.fk_trained_like_params(), device=dev),
                        eta=eta, solver=kanode.Tsit5Options())
    times, losses = [], []
    for i in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        losses.append(tr.step())
        torch.cuda.synchronize()
        times.append(round((time.perf_counter() - t0) * 1e3, 1))
    _, _, sol = tr.loss_and_grad()
    u = sol.u
    print(json.dumps({"eta": eta, "epoch_ms": times, "loss": [round(x, 6) for x in losses],
                      "u_range": [float(u.min()), float(u.max())],
                      "p_drift": float((tr.p.cpu() - torch.as_tensor(bench.fk_trained_like_params())).abs().max())}),
          flush=True)
