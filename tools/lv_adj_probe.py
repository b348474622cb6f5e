"""Per-attempt time of the one-trajectory Lotka-Volterra adjoint (bench.py lv1_train_bench's problem): the
adjoint kernel's time over one iteration's backward, divided by its attempts (accepted + rejected steps).
python tools/lv_adj_probe.py [--reps 20]   (KANODE_LIB selects a variant build)"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import kanode  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from scipy.integrate import solve_ivp
    ts = [0.1 * i for i in range(35)]
    f = lambda t, x: [1.5 * x[0] - x[0] * x[1], x[0] * x[1] - 3.0 * x[1]]   # noqa: E731
    target = solve_ivp(f, (0.0, 3.5), [1.0, 1.0], t_eval=ts, method="DOP853", rtol=1e-10, atol=1e-12).y.T[:, None, :]
    chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
    p0 = chain.setup(np.random.default_rng(0))[0].astype(np.float64) / 1e5 * 1e4
    rhs = kanode.ChainRHS(chain, device=dev)
    u0 = torch.tensor([[1.0, 1.0]], dtype=torch.float64, device=dev)
    tgt = torch.as_tensor(target, device=dev)
    p = torch.as_tensor(p0, device=dev)
    st = None
    times = []
    for r in range(a.reps + 2):
        pp = p.detach().requires_grad_(True)
        sol = kanode.solve(rhs, u0, (0.0, 3.5), pp, ts, sensealg="interpolating_adjoint")
        loss = kanode.mse_loss(sol.u, tgt)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        (g,) = torch.autograd.grad(loss, pp)
        torch.cuda.synchronize()
        if r >= 2:
            times.append(time.perf_counter() - t0)
        st = sol.stats["adjoint"]
    att = st["naccept"] + st["nreject"]
    med = float(np.median(times)) * 1e6
    print(json.dumps({"backward_us": med, "naccept": st["naccept"], "nreject": st["nreject"], "nf": st["nf"],
                      "us_per_attempt": med / att, "path": rhs.hd.get_option("last_adjoint"),
                      "lib": os.environ.get("KANODE_LIB", "default")}), flush=True)


if __name__ == "__main__":
    main()
