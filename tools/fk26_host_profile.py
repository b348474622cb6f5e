"""Where the FK26 training iteration's host time goes (bench.py fk26_train_bench's Trainer.step): per-phase
wall times with synchronisation (forward with dense output, loss, InterpolatingAdjoint backward, Adam + loss read).
python tools/fk26_host_profile.py [--reps 100]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import bench  # noqa: E402
import kanode  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from scipy.integrate import solve_ivp
    nx, dx, D, T = 26, 0.04, 0.01, 5.0
    x = np.arange(nx) * dx
    rho0 = (np.tanh((x - 0.4) / 0.02) - np.tanh((x - 0.6) / 0.02)) / 2
    lap = (np.diag(-2.0 * np.ones(nx)) + np.diag(np.ones(nx - 1), 1) + np.diag(np.ones(nx - 1), -1)) / dx ** 2
    lap[0, -1] = lap[-1, 0] = 1.0 / dx ** 2
    saveat = [0.5 * i for i in range(11)]
    truth = solve_ivp(lambda t, u: D * lap @ u + u * (1 - u), (0.0, T), rho0, t_eval=saveat, method="DOP853",
                      rtol=1e-10, atol=1e-12).y.T[:, None, :]
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign", basis_func="rbf"))
    rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=dx, D=D, dtype=torch.float64, device=dev)
    u0 = torch.as_tensor(rho0[None, :], device=dev)
    tr = kanode.Trainer(rhs, u0, (0.0, T), saveat, torch.as_tensor(truth, device=dev),
                        torch.as_tensor(bench.fk_trained_like_params(), device=dev), eta=1e-2,
                        solver=kanode.Tsit5Options())

    def phases():
        out = {}
        torch.cuda.synchronize(); t0 = time.perf_counter()
        p = tr.p.detach().requires_grad_(True)
        sol = tr.predict(p)
        torch.cuda.synchronize(); t1 = time.perf_counter(); out["forward_keep_dense"] = t1 - t0
        loss = kanode.mse_loss(sol.u, tr.target)
        torch.cuda.synchronize(); t2 = time.perf_counter(); out["loss"] = t2 - t1
        (g,) = torch.autograd.grad(loss, p)
        torch.cuda.synchronize(); t3 = time.perf_counter(); out["backward_adjoint"] = t3 - t2
        tr.opt.update(tr.p, g.contiguous(), 1.0)
        float(loss.detach())
        torch.cuda.synchronize(); t4 = time.perf_counter(); out["adam+float"] = t4 - t3
        out["total"] = t4 - t0
        return out

    for _ in range(5):
        phases()
    acc = {}
    for _ in range(a.reps):
        for k, v in phases().items():
            acc.setdefault(k, []).append(v)
    for k, v in acc.items():
        print(f"{k:22s} median {np.median(v) * 1e3:8.3f} ms")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        tr.step()
    torch.cuda.synchronize()
    print(f"Trainer.step          mean   {(time.perf_counter() - t0) / a.reps * 1e3:8.3f} ms")


if __name__ == "__main__":
    main()
