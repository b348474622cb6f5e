"""KAN-ODE solves on the GPU (HIP RHS + VJP inside Tsit5) vs the same integrator
driven by the CPU oracle RHS; discrete-adjoint gradients vs finite differences;
one training step.  (LV_driver_KANODE.jl:180-214, Fisher-KPP_Source.jl:95-109)"""
import numpy as np
import pytest
import torch

from gpu_util import device, t
from oracle import oracle as O
from oracle_rhs import OracleChainRHS, OracleFKRHS

import kanode

pytestmark = pytest.mark.gpu

LV_SPECS = [O.LayerSpec(2, 10, 5, "tanh_fast"), O.LayerSpec(10, 2, 5, "tanh_fast")]


def lv_chain():
    return kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))


def lv_params(scale=0.5):
    return np.random.default_rng(0).uniform(-scale, scale, 240)


@pytest.mark.parametrize("adaptive", [False, True])
def test_lv_kanode_solve_matches_oracle(adaptive):
    p = lv_params()
    u0 = np.array([[1.0, 1.0], [0.7, 1.3], [1.5, 0.6]])
    ts = [0.1 * i for i in range(35)]
    opt = kanode.Tsit5Options(adaptive=adaptive, dt=None if adaptive else 0.05, abstol=1e-9, reltol=1e-9)
    gpu = kanode.solve(kanode.ChainRHS(lv_chain(), device=device()), t(u0), (0.0, 3.5), t(p), ts, opt)
    ref = kanode.solve(OracleChainRHS(LV_SPECS), torch.as_tensor(u0), (0.0, 3.5), torch.as_tensor(p), ts, opt)
    assert gpu.stats["naccept"] == ref.stats["naccept"]
    err = np.max(np.abs(gpu.u.cpu().numpy() - ref.u.numpy()))
    assert err < 1e-11 * max(1.0, float(ref.u.abs().max()))


def test_lv_adjoint_gradient_matches_oracle_and_fd():
    p = lv_params(0.3)
    u0 = np.array([[1.0, 1.0]])
    ts = [0.1 * i for i in range(35)]
    target = np.random.default_rng(1).uniform(0.5, 2.0, (35, 1, 2))
    opt = kanode.Tsit5Options(adaptive=False, dt=0.05)
    rhs = kanode.ChainRHS(lv_chain(), device=device())

    def loss_gpu(pp):
        return kanode.mse_loss(kanode.solve(rhs, t(u0), (0.0, 3.5), pp, ts, opt).u, t(target))

    pt = t(p).requires_grad_(True)
    (g,) = torch.autograd.grad(loss_gpu(pt), pt)
    pr = torch.as_tensor(p).requires_grad_(True)
    lr = kanode.mse_loss(kanode.solve(OracleChainRHS(LV_SPECS), torch.as_tensor(u0), (0.0, 3.5), pr, ts, opt).u,
                         torch.as_tensor(target))
    (gr,) = torch.autograd.grad(lr, pr)
    assert np.max(np.abs(g.cpu().numpy() - gr.numpy())) < 1e-11 * np.max(np.abs(gr.numpy()))
    d = np.random.default_rng(2).normal(size=240)
    h = 1e-6
    with torch.no_grad():
        fd = (loss_gpu(t(p + h * d)) - loss_gpu(t(p - h * d))).item() / (2 * h)
    assert abs(fd - float(g.cpu().numpy() @ d)) < 1e-5 * max(1.0, abs(fd))


def test_fisher_kpp_solve_matches_oracle():
    nx, dx, D = 26, 0.04, 0.01
    x = np.arange(nx) * dx
    u0 = (np.tanh((x - 0.4) / 0.02) - np.tanh((x - 0.6) / 0.02)) / 2          # Fisher-KPP_Source.jl:49
    p = np.random.default_rng(3).uniform(-0.5, 0.5, 11)
    kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
    rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=dx, D=D, device=device())
    opt = kanode.Tsit5Options()
    ts = [0.5 * i for i in range(11)]
    gpu = kanode.solve(rhs, t(u0[None]), (0.0, 5.0), t(p), ts, opt)
    ref = kanode.solve(OracleFKRHS(O.LayerSpec(1, 1, 10, "softsign"), D, dx), torch.as_tensor(u0[None]), (0.0, 5.0),
                       torch.as_tensor(p), ts, opt)
    assert gpu.stats["naccept"] == ref.stats["naccept"]
    assert np.max(np.abs(gpu.u.cpu().numpy() - ref.u.numpy())) < 1e-10


def test_lv_training_step_reduces_loss(golden):
    d = golden("lv_truth")
    ts = list(d["t"][:35])
    target = t(d["X"][:, :35].T[:, None, :])
    p0 = t(lv_params(0.1))
    rhs = kanode.ChainRHS(lv_chain(), device=device())
    tr = kanode.Trainer(rhs, t(np.array([[1.0, 1.0]])), (0.0, 3.5), ts, target, p0, eta=5e-3)
    l0 = tr.step()
    for _ in range(15):
        l1 = tr.step()
    assert l1 < l0
