"""The fused optimiser step (kanode_adam_step, kan_optim.hip) against Flux's Adam formula
(LV_driver_KANODE.jl:219,287; Fisher-KPP_Source.jl:167,201; Flux 0.14 legacy Optimise.Adam, restated)
and against kanode.Adam (the torch statement), and the Trainer that uses it."""
import numpy as np
import pytest
import torch

from gpu_util import device, t

import kanode

pytestmark = pytest.mark.gpu


def flux_adam(x, grads, eta, scale, dtype=np.float64, b1=0.9, b2=0.999, eps=1e-8):
    """Flux's apply!/update! in float64 numpy (Float64 hyper-parameters promote a Float32 x; the
    results are rounded on store)."""
    x = x.astype(dtype).copy()
    flux_adam.abs_sum = np.abs(x).astype(np.float64)      # Σ|terms| of x after the steps (for the bound)
    m = np.zeros_like(x)
    v = np.zeros_like(x)
    bp1, bp2 = b1, b2
    for g in grads:
        d = g.astype(dtype).astype(np.float64) * scale
        m = (b1 * m.astype(np.float64) + (1 - b1) * d).astype(dtype)
        v = (b2 * v.astype(np.float64) + ((1 - b2) * d) * d).astype(dtype)
        step = m.astype(np.float64) / (1 - bp1) / (np.sqrt(v.astype(np.float64) / (1 - bp2)) + eps) * eta
        x = x - step.astype(dtype)      # apply! stores Δ in the gradient's eltype; x .-= Δ in that type
        flux_adam.abs_sum = flux_adam.abs_sum + np.abs(step)
        bp1 *= b1
        bp2 *= b2
    return x


@pytest.mark.parametrize("n", [11, 240, 450_561])      # FK, LV and the SC1024 parameter vector
def test_fused_adam_matches_flux_formula_fp64(n):
    rng = np.random.default_rng(n)
    x0 = rng.normal(size=n)
    grads = [rng.normal(size=n) * 10.0 ** rng.uniform(-6, 2, n) for _ in range(6)]
    ref = flux_adam(x0, grads, 1e-2, 0.5)
    x = t(x0)
    opt = kanode.FusedAdam(1e-2)
    for g in grads:
        opt.update(x, t(g), 0.5)
    got = x.cpu().numpy()
    # per entry against |x0| + Σ_t |Δ_t| (x - Δ cancels for some entries, so |x| itself is no scale)
    assert np.max(np.abs(got - ref) / flux_adam.abs_sum) <= 1e-15
    # the torch statement of the same step (8 elementwise launches) on the same device
    xs = t(x0)
    slow = kanode.Adam(1e-2)
    for g in grads:
        slow.update(xs, t(g) * 0.5)
    assert (x - xs).abs().max().item() <= 1e-15 * xs.abs().max().item()


def test_fused_adam_fp32_promotes_like_flux():
    """LV4k trains Float32 parameters: Flux's Float64 hyper-parameters promote each broadcast, which
    is rounded to Float32 on store; the kernel does the same."""
    rng = np.random.default_rng(3)
    x0 = rng.normal(size=240).astype(np.float32)
    grads = [rng.normal(size=240).astype(np.float32) for _ in range(4)]
    ref = flux_adam(x0, grads, 1e-3, 1.0, dtype=np.float32)
    x = t(x0, torch.float32)
    opt = kanode.FusedAdam(1e-3)
    for g in grads:
        opt.update(x, t(g, torch.float32))
    got = x.cpu().numpy()
    assert np.max(np.abs(got.astype(np.float64) - ref) / np.abs(ref)) <= 1.2e-7     # one float32 ulp
    # the CPU trainer's kanode.Adam promotes the same way: the same Float32 trajectory
    xc = torch.as_tensor(x0.copy())
    slow = kanode.Adam(1e-3)
    for g in grads:
        slow.update(xc, torch.as_tensor(g))
    assert np.max(np.abs(got.astype(np.float64) - xc.numpy().astype(np.float64)) / np.abs(ref)) <= 1.2e-7


def test_fused_adam_rejects_bad_arguments():
    opt = kanode.FusedAdam(1e-3)
    with pytest.raises(kanode.KanodeError):
        opt.update(torch.zeros(4, dtype=torch.float64), torch.zeros(4, dtype=torch.float64))   # CPU tensor
    with pytest.raises(kanode.KanodeError):
        opt.update(t(np.zeros(4)), t(np.zeros(4), torch.float32))
    lib = kanode.lib()
    x = t(np.zeros(4))
    p = x.data_ptr()
    assert lib.kanode_adam_step(p, p, p, p, -1, 1, 1.0, 1e-3, 0.9, 0.999, 1e-8, 0.9, 0.999, None) != 0
    assert lib.kanode_adam_step(p, p, p, p, 4, 1, 1.0, 1e-3, 1.0, 0.999, 1e-8, 1.0, 0.999, None) != 0
    assert lib.kanode_adam_step(p, p, p, p, 0, 1, 1.0, 1e-3, 0.9, 0.999, 1e-8, 0.9, 0.999, None) == 0


def test_trainer_uses_fused_adam_and_matches_torch_adam():
    """Trainer.step on the GPU (Fisher-KPP, native solve + InterpolatingAdjoint) takes the fused step;
    three steps give the parameters the torch Adam statement gives."""
    nx, B = 256, 4
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
    rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=1.0 / (nx - 1), D=0.01, device=device())
    x = np.arange(nx) / (nx - 1)
    u0 = t(np.stack([(np.tanh((x - c) / 0.02) - np.tanh((x - c - 0.2) / 0.02)) / 2 for c in (0.3, 0.35, 0.4, 0.45)]))
    ts = [0.0, 0.05, 0.1]
    opt = kanode.Tsit5Options(adaptive=False, dt=5e-4)
    ptrue = t(np.random.default_rng(1).uniform(-0.5, 0.5, 11))
    target = kanode.solve(rhs, u0, (0.0, 0.1), ptrue, ts, opt).u
    p0 = ptrue * 1.2
    fused = kanode.Trainer(rhs, u0, (0.0, 0.1), ts, target, p0, eta=1e-2, solver=opt)
    assert isinstance(fused.opt, kanode.FusedAdam)
    slow = kanode.Trainer(rhs, u0, (0.0, 0.1), ts, target, p0, eta=1e-2, solver=opt)
    slow.opt = kanode.Adam(1e-2)
    for _ in range(3):
        la, lb = fused.step(), slow.step()
        assert la == lb
    assert (fused.p - slow.p).abs().max().item() <= 1e-15 * slow.p.abs().max().item()
    assert fused.history[-1] < fused.history[0]


def test_trainer_fast_path_filters_saveat_past_tf():
    """a saveat point past tf is dropped as solve() drops it (not left as unwritten rows of the
    solution), and kanode_solve_tsit5 itself rejects such a stop."""
    nx, B = 256, 2
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
    rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=1.0 / (nx - 1), D=0.01, device=device())
    x = np.arange(nx) / (nx - 1)
    u0 = t(np.stack([(np.tanh((x - c) / 0.02) - np.tanh((x - c - 0.2) / 0.02)) / 2 for c in (0.3, 0.4)]))
    opt = kanode.Tsit5Options(adaptive=False, dt=5e-4)
    ptrue = t(np.random.default_rng(2).uniform(-0.5, 0.5, 11))
    ts = [0.0, 0.05, 0.1]
    target = kanode.solve(rhs, u0, (0.0, 0.1), ptrue, ts, opt).u
    p0 = ptrue * 1.1
    ref = kanode.Trainer(rhs, u0, (0.0, 0.1), ts, target, p0, eta=1e-2, solver=opt)
    past = kanode.Trainer(rhs, u0, (0.0, 0.1), ts + [0.3], target, p0, eta=1e-2, solver=opt)
    la, ga, _ = ref.loss_and_grad()
    lb, gb, _ = past.loss_and_grad()
    assert float(la) == float(lb)
    assert torch.equal(ga, gb)
    with pytest.raises(kanode.KanodeError, match="saveat"):
        rhs.hd.solve_tsit5(p0, u0, 0.0, 0.1, [0.0, 0.3], opt.to_c())


@pytest.mark.parametrize("case", ["lv1", "fk26"])
def test_eval_loss_forward_is_reused_by_the_next_step_bitwise(case):
    """the driver's loss_train(p) after update! (LV_driver_KANODE.jl:289) solves exactly the next
    iteration's InterpolatingAdjoint forward problem.  Trainer.eval_loss keeps that solve's dense output and the next
    step takes its gradient from it: the parameter trajectory and the logged losses are bitwise those of the trainer
    that solves again.  (FK26 takes forward mode, whose Dual solve is not the logged plain solve: nothing is kept,
    and the logged loss is the plain solve's.)"""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    dev = device()
    if case == "lv1":
        chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
        rhs = kanode.ChainRHS(chain, device=dev)
        p0 = t(chain.setup(np.random.default_rng(0))[0].astype(np.float64) / 1e4)
        u0 = t(np.array([[1.0, 1.0]]))
        ts = [0.1 * i for i in range(35)]
        X = t(np.random.default_rng(1).uniform(0.5, 2.0, (35, 1, 2)))
        tspan, eta = (0.0, 3.5), 5e-4
    else:
        import anchors
        pr = anchors.source_problem("fk")
        kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
        rhs = kanode.FisherKPPRHS(kan1, nx=pr["nx"], dx=pr["dx"], D=pr["D"], device=dev)
        p0 = t(kan1.setup(np.random.default_rng(1))[0].astype(np.float64))
        u0 = t(pr["u0"][None, :])
        ts, tspan, eta = pr["saveat"], pr["tspan"], 1e-2
        X = t(anchors.source_truth(pr))
    a = kanode.Trainer(rhs, u0, tspan, ts, X, p0, eta=eta)
    b = kanode.Trainer(rhs, u0, tspan, ts, X, p0, eta=eta)
    la, lb = [], []
    for _ in range(4):
        a.step()
        la.append(a.eval_loss())           # cached for a's next step
        b.step()
        with torch.no_grad():
            lb.append(float(kanode.mse_loss(kanode.solve(rhs, u0, tspan, b.p, ts,
                                                         sensealg="discrete").u, X)))
    assert torch.equal(a.p, b.p)
    assert a.history == b.history
    assert la == lb
