"""The DEFAULT Fisher-KPP training path end to end against the CPU oracle.

What runs on the GPU is exactly what `Trainer.step` / the bench's epoch leg runs for Fisher-KPP at
Nx = 128·k: the native `kanode_solve_tsit5` host loop issuing one `fk_step_pp_wave_kernel` launch per
Tsit5 step (Q-form dense output), then the native `kanode_adjoint_tsit5` InterpolatingAdjoint issuing
one `fk_vjp_step_rows_kernel` launch per adjoint step (Nx <= 256; `fk_vjp_step_pp_wave_kernel` at
Nx = 512) plus `vjp_finish_jobs_kernel` (the combined reductions and the μ update on fixed steps, the
per-stage reductions on adaptive steps).

What runs on the CPU is the Python statement of the same integrator and adjoint (kanode/ode.py,
kanode/adjoint.py with native=False, plain per-stage torch arithmetic) around the plain-C oracle of
`rc_kanode` with the reference's DENSE Laplacian matvec (PDE examples/Fisher-KPP_Source.jl:55-59,
95-98; problem set-up :38-44,102-109; oracle/kanode_ref_impl.inc).

Bar (VERDICT r2 "next round" #1): equal forward and adjoint step counts, saveat values within 1e-11,
dL/dp and dL/du0 within 1e-9 relative.  Fixed steps: dt = 5e-4 at Nx = 256, scaled by (256/Nx)² so
that every Nx sits at the same point of Tsit5's stability region (D·lap has eigenvalues down to
-4D/dx²: 5e-4 at Nx = 512 would be outside it and both sides would blow up identically), 40 steps.
Adaptive: abstol = reltol = 1e-9 over a short span, where accuracy rather than the stability limit
picks the steps (at the stability edge last-bit differences of the error norm can flip one
accept/reject, see test_gpu_native_solve.py)."""
import numpy as np
import pytest
import torch

from gpu_util import device, t
from oracle import oracle as O
from oracle.oracle_rhs import OracleFKRHS

import kanode

pytestmark = pytest.mark.gpu

D = 0.01


def _u0(nx, B, seed):
    """The reference IC family (Fisher-KPP_Source.jl:47-49) with random centre, width, amplitude."""
    rng = np.random.default_rng(seed)
    x = np.arange(nx) / (nx - 1)
    c, d, a = rng.uniform(0.3, 0.7, (B, 1)), rng.uniform(0.1, 0.3, (B, 1)), rng.uniform(0.5, 1, (B, 1))
    return a * (np.tanh((x - (c - d / 2)) / (d / 10)) - np.tanh((x - (c + d / 2)) / (d / 10))) / 2


def _run(f, dev, u0, p0, tspan, ts, w, opt):
    p = torch.as_tensor(p0, device=dev).clone().requires_grad_(True)
    x0 = torch.as_tensor(u0, device=dev).clone().requires_grad_(True)
    sol = kanode.solve(f, x0, tspan, p, ts, opt, sensealg="interpolating_adjoint")
    gp, gu = torch.autograd.grad((sol.u * torch.as_tensor(w, device=dev)).sum(), [p, x0])
    return sol.u.detach().cpu(), gp.cpu(), gu.cpu(), sol.stats


def _e2e(nx, B, mode, seed, diffusion=D, G=10, norm="softsign", amp=1.0, shift=0.0, pscale=1.0, adjoint_counts=True,
         **opts):
    dx = 1.0 / (nx - 1)
    gpu = kanode.FisherKPPRHS(kanode.Chain(kanode.KDense(1, 1, G, normalizer=norm)), nx=nx, dx=dx, D=diffusion,
                              device=device())
    assert gpu.hd.pointwise_table, "the default (table) path must be the one under test"
    cpu = OracleFKRHS(O.LayerSpec(1, 1, G, norm), diffusion, dx, dense=True)
    u0 = amp * _u0(nx, B, seed) + shift
    p0 = pscale * np.random.default_rng(seed + 100).uniform(-1.0, 1.0, G + 1)
    if mode == "fixed":
        dt = 5e-4 * (256 / nx) ** 2
        tspan, ts = (0.0, 40 * dt), [0.0, 10 * dt, 25 * dt, 40 * dt]
        opt = kanode.Tsit5Options(adaptive=False, dt=dt)
    else:
        T = 0.02 * (256 / nx) ** 2 if diffusion else 0.5
        tspan, ts = (0.0, T), [0.0, 0.3 * T, 0.5 * T, T]
        opt = kanode.Tsit5Options(abstol=1e-9, reltol=1e-9)
    w = np.random.default_rng(seed + 200).normal(size=(len(ts), B, nx))
    with gpu.hd.options(**opts):
        ug, gg, gug, sg = _run(gpu, device(), t(u0), p0, tspan, ts, w, opt)
    uc, gc, guc, sc = _run(cpu, "cpu", torch.as_tensor(u0), p0, tspan, ts, w, opt)
    assert (sg["naccept"], sg["nreject"]) == (sc["naccept"], sc["nreject"])
    if adjoint_counts:
        assert (sg["adjoint"]["naccept"], sg["adjoint"]["nreject"]) == (sc["adjoint"]["naccept"],
                                                                        sc["adjoint"]["nreject"])
    assert sg["naccept"] >= (40 if mode == "fixed" else 5)
    assert (ug - uc).abs().max().item() <= 1e-11
    assert (gg - gc).abs().max().item() <= 1e-9 * gc.abs().max().item()
    assert (gug - guc).abs().max().item() <= 1e-9 * guc.abs().max().item()
    return sg


@pytest.mark.parametrize("mode", ["fixed", "adaptive"])
@pytest.mark.parametrize("nx,B", [(128, 4), (256, 3), (512, 2)])
def test_fk_default_path_matches_cpu_oracle(nx, B, mode):
    _e2e(nx, B, mode, seed=nx + B)


@pytest.mark.parametrize("mode", ["fixed", "adaptive"])
def test_fk_default_path_several_rows_per_wave(mode):
    """Persistent grids of one block (4 waves) over 12 trajectories: the forward step kernel and the
    persistent-grid adjoint step run 3 rows per wave (GRID_ADJ_STEP set takes the adjoint off the
    one-row-per-wave kernel)."""
    _e2e(256, 12, mode, seed=5, grid_rhs=1, grid_vjp=1, grid_adj_step=1)


@pytest.mark.parametrize("mode", ["fixed", "adaptive"])
@pytest.mark.parametrize("G,norm", [(10, "softsign"), (10, "tanh_fast"), (5, "softsign"), (5, "tanh_fast")])
def test_fk_default_path_kan_only(G, norm, mode):
    """D = 0 (du/dt = kan1_(u) per point): the adjoint step kernels' λᵀJ is then the KAN part alone
    (φ' and swish' tables), so the whole native step / adjoint-step path is pinned on it.  u stays in
    [0.2, 2.2]: trajectories that cross softsign's kink at u = 0 (N'' jumps there) make the adjoint's
    controller reject about every other step (measured with the CPU driver: 115 rejects in 261 steps),
    and on such a sequence last-bit differences of the error norm flip decisions.  Here both sides
    take the same steps with no rejection."""
    _e2e(256, 3, mode, seed=G + len(norm), diffusion=0.0, G=G, norm=norm, amp=2.0, shift=0.2, pscale=0.5)


@pytest.mark.parametrize("mode", ["fixed", "adaptive"])
def test_fk_default_path_negative_states(mode):
    """Round 6: states below zero, where the swish table had been rejected (its acceptance scale formed with the
    |x| source modifier came out negative below u ≈ -0.2: every such point took the direct formula).  Fixed step:
    a field shifted below zero through the table path's forward and adjoint steps against the dense-Laplacian CPU
    oracle (values 1e-11, gradients 1e-9).  Adaptive: the whole field negative (u in [-2.2, -1.2], D = 0 so nothing
    crosses softsign's kink at 0): equal forward step counts, values and gradients at the file's bars, adjoint step
    counts NOT compared.  On this field the source is nearly linear and the adjoint's embedded error sits at the
    rounding level, so its step sizes follow last-bit noise: the oracle's own VJP perturbed by 1e-15 relative moves
    its second step 2%, by 1e-14 it takes 8 steps instead of 10 (tests/test_oracle_step_noise.py, on the CPU); the
    table path takes 8, the direct kernels 10, all with dL/dp equal to 3e-13 (profiles/r06/negative)."""
    if mode == "adaptive":
        _e2e(256, 3, mode, seed=31, diffusion=0.0, amp=1.0, shift=-2.2, pscale=0.5, adjoint_counts=False)
    else:
        _e2e(256, 3, mode, seed=33, shift=-0.6)
