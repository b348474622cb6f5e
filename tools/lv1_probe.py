#!/usr/bin/env python3
"""Where an LV1 training iteration's wall time goes (bench.py's lv1_train leg), and the same iteration with the
post-update loss_test solve on a second handle / stream / host thread, concurrent with loss_train's solve.
Interleaved rounds; prints one JSON line.   python3 tools/lv1_probe.py [--reps 50 --rounds 5]"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import kanode  # noqa: E402
from scipy.integrate import solve_ivp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--rounds", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda:0")
ts = [0.1 * i for i in range(35)]
ts_test = [0.1 * i for i in range(141)]
f = lambda t, x: [1.5 * x[0] - x[0] * x[1], x[0] * x[1] - 3.0 * x[1]]   # noqa: E731
full = solve_ivp(f, (0.0, 14.0), [1.0, 1.0], t_eval=ts_test, method="DOP853", rtol=1e-10, atol=1e-12).y.T[:, None, :]
chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
p0 = chain.setup(np.random.default_rng(0))[0].astype(np.float64) / 1e5 * 1e4
u0 = torch.tensor([[1.0, 1.0]], dtype=torch.float64, device=dev)
tgt_test = torch.as_tensor(full, device=dev)


def trainer():
    rhs = kanode.ChainRHS(chain, device=dev)
    tr = kanode.Trainer(rhs, u0, (0.0, 3.5), ts, torch.as_tensor(full[:35], device=dev),
                        torch.as_tensor(p0, device=dev), eta=1e-3, sensealg="interpolating_adjoint")
    return rhs, tr


rhs_a, tr_a = trainer()
rhs_b, tr_b = trainer()
rhs_t = kanode.ChainRHS(chain, device=dev)   # the loss_test solve's own handle (variant B)
side = torch.cuda.Stream(dev)
pool = ThreadPoolExecutor(1)


def it_a():
    tr_a.step()
    l_tr = tr_a.eval_loss()
    with torch.no_grad():
        l_te = kanode.mse_loss(kanode.solve(rhs_a, u0, (0.0, 14.0), tr_a.p, ts_test).u, tgt_test)
    return l_tr, float(l_te)


def test_loss(ev):
    with torch.cuda.stream(side):
        side.wait_event(ev)
        with torch.no_grad():
            return float(kanode.mse_loss(kanode.solve(rhs_t, u0, (0.0, 14.0), tr_b.p, ts_test).u, tgt_test))


def it_b():
    tr_b.step()
    ev = torch.cuda.Event()
    ev.record()
    fut = pool.submit(test_loss, ev)
    l_tr = tr_b.eval_loss()
    return l_tr, fut.result()


def timed(fn, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def parts(reps):
    out = {}
    tr = tr_a
    torch.cuda.synchronize()
    t = {"step": 0.0, "eval_loss": 0.0, "test_solve": 0.0}
    for _ in range(reps):
        t0 = time.perf_counter()
        tr.step()
        t1 = time.perf_counter()
        tr.eval_loss()
        t2 = time.perf_counter()
        with torch.no_grad():
            float(kanode.mse_loss(kanode.solve(rhs_a, u0, (0.0, 14.0), tr.p, ts_test).u, tgt_test))
        t3 = time.perf_counter()
        t["step"] += t1 - t0
        t["eval_loss"] += t2 - t1
        t["test_solve"] += t3 - t2
    for k, v in t.items():
        out[k] = v / reps * 1e3
    return out


for fn in (it_a, it_b):
    for _ in range(3):
        fn()
res = {"a_serial": [], "b_concurrent_test": []}
for r in range(a.rounds):
    res["a_serial"].append(timed(it_a, a.reps))
    res["b_concurrent_test"].append(timed(it_b, a.reps))
la = [it_a() for _ in range(3)]
lb = [it_b() for _ in range(3)]
out = {k: {"median_ms": float(np.median(v)), "all": v} for k, v in res.items()}
out["parts_ms"] = parts(a.reps)
out["losses_equal"] = la == lb
out["losses"] = [la[-1], lb[-1]]
print(json.dumps(out), flush=True)
