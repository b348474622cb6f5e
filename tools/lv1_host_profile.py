"""Where the LV1 training iteration's host time goes (bench.py lv1_train_bench's iteration):
per-phase wall times with synchronisation, and a cProfile of 50 iterations (top entries by own time).
python tools/lv1_host_profile.py [--reps 50]"""
import argparse, cProfile, io, os, pstats, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kan-odes_amd"))
import numpy as np
import torch
import bench
import kanode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    r = bench.lv1_train_bench(dev, False, reps=a.reps)
    print("bench iteration ms:", r["gpu"])
    from scipy.integrate import solve_ivp
    ts = [0.1 * i for i in range(35)]
    ts_test = [0.1 * i for i in range(141)]
    f = lambda t, x: [1.5 * x[0] - x[0] * x[1], x[0] * x[1] - 3.0 * x[1]]   # noqa: E731
    full = solve_ivp(f, (0.0, 14.0), [1.0, 1.0], t_eval=ts_test, method="DOP853", rtol=1e-10, atol=1e-12).y.T[:, None, :]
    chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
    p0 = chain.setup(np.random.default_rng(0))[0].astype(np.float64) / 1e5 * 1e4
    rhs = kanode.ChainRHS(chain, device=dev)
    u0 = torch.tensor([[1.0, 1.0]], dtype=torch.float64, device=dev)
    tr = kanode.Trainer(rhs, u0, (0.0, 3.5), ts, torch.as_tensor(full[:35], device=dev), torch.as_tensor(p0, device=dev),
                        eta=1e-3, sensealg="interpolating_adjoint")
    tgt = torch.as_tensor(full, device=dev)

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
        lv = float(loss)
        torch.cuda.synchronize(); t4 = time.perf_counter(); out["adam+float"] = t4 - t3
        with torch.no_grad():
            l1 = float(kanode.mse_loss(kanode.solve(rhs, u0, (0.0, 3.5), tr.p, ts).u, tr.target))
        torch.cuda.synchronize(); t5 = time.perf_counter(); out["solve_train+loss"] = t5 - t4
        with torch.no_grad():
            l2 = float(kanode.mse_loss(kanode.solve(rhs, u0, (0.0, 14.0), tr.p, ts_test).u, tgt))
        torch.cuda.synchronize(); t6 = time.perf_counter(); out["solve_test+loss"] = t6 - t5
        out["total"] = t6 - t0
        return out

    for _ in range(3):
        phases()
    acc = {}
    for _ in range(a.reps):
        for k, v in phases().items():
            acc.setdefault(k, []).append(v)
    for k, v in acc.items():
        print(f"{k:22s} median {np.median(v) * 1e3:8.3f} ms")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.reps):
        phases()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
