"""The C epoch comparator (oracle/cpu_epoch.c, bench.py's CPU epoch legs) against the Python statement
of the same epoch (kanode.solve + InterpolatingAdjoint + Adam on the oracle RHS, dense Laplacian):
Fisher-KPP_Source.jl:101-109,195-201.  Both are CPU restatements; this pins the comparator to the
driver the GPU path is checked against."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle.oracle_rhs import OracleFKRHS

import kanode


def _ics(B, nx, seed):
    rng = np.random.default_rng(seed)
    x = np.arange(nx) / (nx - 1)
    c, d, a = rng.uniform(0.3, 0.7, (B, 1)), rng.uniform(0.1, 0.3, (B, 1)), rng.uniform(0.5, 1, (B, 1))
    return a * (np.tanh((x - (c - d / 2)) / (d / 10)) - np.tanh((x - (c + d / 2)) / (d / 10))) / 2


@pytest.mark.parametrize("adaptive", [True, False])
def test_c_epoch_matches_python_driver(adaptive):
    nx, B, D = 32, 3, 0.01
    dx = 1.0 / (nx - 1)
    spec = O.LayerSpec(1, 1, 10, "softsign")
    u0 = _ics(B, nx, 1)
    p0 = np.random.default_rng(2).uniform(-1, 1, 11)
    T = 0.5
    saveat = [0.0, 0.1, 0.25, 0.25, 0.4, 0.5]
    target = 0.9 * np.broadcast_to(u0, (len(saveat), B, nx))
    dt = 2e-3
    opt = kanode.Tsit5Options(abstol=1e-8, reltol=1e-8) if adaptive else kanode.Tsit5Options(adaptive=False, dt=dt)
    loss, grad, p_new, st, secs = O.fk_epoch(spec, p0, D, dx, u0, T, saveat, target, abstol=1e-8, reltol=1e-8,
                                             adaptive=adaptive, dt=dt, eta=1e-2)
    tr = kanode.Trainer(OracleFKRHS(spec, D, dx, dense=True), torch.as_tensor(u0), (0.0, T), saveat,
                        torch.as_tensor(np.ascontiguousarray(target)), torch.as_tensor(p0), eta=1e-2, solver=opt,
                        sensealg="interpolating_adjoint")
    lt, gt, sol = tr.loss_and_grad()
    assert st["naccept"] == sol.stats["naccept"] and st["nreject"] == sol.stats["nreject"]
    assert st["adjoint_naccept"] == sol.stats["adjoint"]["naccept"]
    assert abs(loss - lt.item()) <= 1e-12 * abs(loss)
    assert np.max(np.abs(grad - gt.numpy())) <= 1e-10 * np.max(np.abs(gt.numpy()))
    tr.step()
    assert np.max(np.abs(p_new - tr.p.numpy())) <= 1e-12 * np.max(np.abs(p0))
    assert secs > 0


@pytest.mark.parametrize("adaptive", [True, False])
def test_c_chain_epoch_matches_python_driver(adaptive):
    """The LV comparator (bench.py lv1_train's CPU leg): the C NeuralODE epoch over the oracle chain
    (LV_driver_KANODE.jl:180-219,279-287) against Trainer + InterpolatingAdjoint over OracleChainRHS."""
    from oracle.oracle_rhs import OracleChainRHS
    specs = [O.LayerSpec(2, 10, 5, "tanh_fast"), O.LayerSpec(10, 2, 5, "tanh_fast")]
    rng = np.random.default_rng(4)
    P = 240                                    # LV [2, 10, 2] G = 5
    p0 = rng.uniform(-0.3, 0.3, P)
    u0 = np.array([[1.0, 1.0], [0.8, 1.3]])
    saveat = [0.1 * i for i in range(8)]
    T = 0.7
    target = np.ascontiguousarray(np.broadcast_to(u0 * 1.05, (len(saveat), 2, 2)))
    dt = 0.01
    opt = kanode.Tsit5Options(abstol=1e-8, reltol=1e-8) if adaptive else kanode.Tsit5Options(adaptive=False, dt=dt)
    loss, grad, p_new, st, secs = O.chain_epoch(specs, p0, u0, T, saveat, target, abstol=1e-8, reltol=1e-8,
                                                adaptive=adaptive, dt=dt, eta=5e-4)
    tr = kanode.Trainer(OracleChainRHS(specs), torch.as_tensor(u0), (0.0, T), saveat, torch.as_tensor(target),
                        torch.as_tensor(p0), eta=5e-4, solver=opt, sensealg="interpolating_adjoint")
    lt, gt, sol = tr.loss_and_grad()
    assert st["naccept"] == sol.stats["naccept"] and st["nreject"] == sol.stats["nreject"]
    assert st["adjoint_naccept"] == sol.stats["adjoint"]["naccept"]
    assert abs(loss - lt.item()) <= 1e-12 * abs(loss)
    assert np.max(np.abs(grad - gt.numpy())) <= 1e-10 * np.max(np.abs(gt.numpy()))
    tr.step()
    assert np.max(np.abs(p_new - tr.p.numpy())) <= 1e-12 * np.max(np.abs(p0))
    # the forward solve alone (the driver's loss_train / loss_test solves)
    pred, st2, _ = O.chain_solve(specs, p0, u0, T, saveat, abstol=1e-8, reltol=1e-8)
    ref = kanode.solve(OracleChainRHS(specs), torch.as_tensor(u0), (0.0, T), torch.as_tensor(p0), saveat,
                       kanode.Tsit5Options(abstol=1e-8, reltol=1e-8))
    assert st2["naccept"] == ref.stats["naccept"]
    assert np.max(np.abs(pred - ref.u.numpy())) <= 1e-12


def test_c_chain_epoch_wide_surrogate_shape():
    """The surrogate comparator (bench.py surrogates' CPU training iteration): a full-field chain
    KAN [N, H, N] (the Burgers/Schrödinger surrogate form, Burgers_Surrogate.jl:85-97) at a small N,
    several ICs and saveat stops: the C epoch against Trainer + InterpolatingAdjoint over OracleChainRHS."""
    from oracle.oracle_rhs import OracleChainRHS
    N, H, G, B = 24, 4, 5, 3
    specs = [O.LayerSpec(N, H, G, "softsign"), O.LayerSpec(H, N, G, "softsign")]
    chain = kanode.Chain(kanode.KDense(N, H, G, normalizer="softsign"), kanode.KDense(H, N, G, normalizer="softsign"))
    p0 = chain.setup(np.random.default_rng(6))[0].astype(np.float64)
    x = np.linspace(-1.0, 1.0, N)
    u0 = np.stack([-np.sin(np.pi * x) + 0.1 * k * np.sin(2 * np.pi * x) for k in range(B)])
    saveat = [0.05 * i for i in range(7)]
    T = 0.3
    target = np.ascontiguousarray(np.broadcast_to(0.9 * u0, (len(saveat), B, N)))
    loss, grad, p_new, st, secs = O.chain_epoch(specs, p0, u0, T, saveat, target, abstol=1e-8, reltol=1e-8,
                                                adaptive=True, eta=1e-2)
    tr = kanode.Trainer(OracleChainRHS(specs), torch.as_tensor(u0), (0.0, T), saveat, torch.as_tensor(target),
                        torch.as_tensor(p0), eta=1e-2, solver=kanode.Tsit5Options(abstol=1e-8, reltol=1e-8),
                        sensealg="interpolating_adjoint")
    lt, gt, sol = tr.loss_and_grad()
    assert st["naccept"] == sol.stats["naccept"] and st["adjoint_naccept"] == sol.stats["adjoint"]["naccept"]
    assert abs(loss - lt.item()) <= 1e-12 * abs(loss)
    assert np.max(np.abs(grad - gt.numpy())) <= 1e-10 * np.max(np.abs(gt.numpy()))
    tr.step()
    assert np.max(np.abs(p_new - tr.p.numpy())) <= 1e-12 * np.max(np.abs(p0))
