"""ODE right-hand sides on the HIP kernels, differentiable through torch.autograd.

    ChainRHS     — DiffEqFlux NeuralODE's dudt(u, p, t) = Chain(u, p, st)[1]
                   (LV_driver_KANODE.jl:180, Burgers_Surrogate.jl:97, Schrodinger_Surrogate.jl:104)
    FisherKPPRHS — rc_kanode(u, p, t) = D*lap*u + kan1_.(u)  (PDE examples/Fisher-KPP_Source.jl:95-98)

Both expose `__call__(u, p, t)` (the out-of-place ODEFunction{false} form the
reference solves) and `vjp(u, p, lam)` — the pullback SciMLSensitivity requests
at every adjoint stage — each one C-ABI call into libkanode.so.
"""
from __future__ import annotations

import numpy as np
import torch

from .handle import KanodeHandle, LayerCfg


class _RHSFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hd: KanodeHandle, p, u):
        ctx.hd = hd
        ctx.save_for_backward(p, u)
        return hd.rhs(p, u)

    @staticmethod
    def backward(ctx, g):
        p, u = ctx.saved_tensors
        lamJ, dp = ctx.hd.vjp(p, u, g.contiguous(), want_lamJ=ctx.needs_input_grad[2],
                              accumulate_dp=ctx.needs_input_grad[1])
        return None, dp, lamJ


class _LayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hd: KanodeHandle, layer: int, p, x):
        ctx.hd, ctx.layer = hd, layer
        ctx.save_for_backward(p, x)
        return hd.layer_forward(layer, p, x)

    @staticmethod
    def backward(ctx, g):
        p, x = ctx.saved_tensors
        xbar, pbar = ctx.hd.layer_vjp(ctx.layer, p, x, g.contiguous())
        return None, None, pbar, xbar


class _StageFn(torch.autograd.Function):
    """du = f(y), y = u + Σ_j c_j k_j (one kanode_rhs_stage call); returns (du, y).

    Backward: (λᵀJ, dp) = VJP at the saved y; ∂/∂y = λᵀJ + ȳ, then ∂/∂u = ∂/∂y and
    ∂/∂k_j = c_j ∂/∂y (the stage broadcast's own pullback)."""

    @staticmethod
    def forward(ctx, hd: KanodeHandle, c, error, p, u, *ks):
        y = torch.empty_like(u)
        du = hd.rhs_stage(p, u, ks, c, y_out=y, error=error)
        ctx.hd, ctx.c = hd, c
        ctx.save_for_backward(p, y)
        return du, y

    @staticmethod
    def backward(ctx, gdu, gy):
        p, y = ctx.saved_tensors
        gy_total = gy
        dp = None
        if gdu is not None:
            lamJ, dp = ctx.hd.vjp(p, y, gdu.contiguous(), accumulate_dp=ctx.needs_input_grad[3])
            gy_total = lamJ if gy is None else lamJ + gy
        if gy_total is None:
            gy_total = torch.zeros_like(y)
        gks = [gy_total * cj for cj in ctx.c]
        return (None, None, None, dp, gy_total, *gks)


def stage_apply(hd: KanodeHandle, p: torch.Tensor, u: torch.Tensor, ks, c, want_y: bool = False, error=None):
    """Tsit5 stage through kanode_rhs_stage: (du, y or None).  Differentiable when autograd
    is recording (y is then written for the backward VJP); otherwise y is only written
    when asked for."""
    c = [float(x) for x in c]
    ks = [k.contiguous() for k in ks]
    if torch.is_grad_enabled() and (p.requires_grad or u.requires_grad or any(k.requires_grad for k in ks)):
        du, y = _StageFn.apply(hd, c, error, p.contiguous(), u.contiguous(), *ks)
        return du, y
    y = torch.empty_like(u) if want_y else None
    du = hd.rhs_stage(p, u.contiguous(), ks, c, y_out=y, error=error)
    return du, y


def rhs_apply(hd: KanodeHandle, p: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    return _RHSFn.apply(hd, p.contiguous(), u.contiguous())


def layer_apply(hd: KanodeHandle, layer: int, p: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    return _LayerFn.apply(hd, layer, p.contiguous(), x.contiguous())


class ChainRHS:
    """NeuralODE RHS f(u, p, t) = Chain(u; p) for a KDense chain with in == out."""

    def __init__(self, chain, dtype=torch.float64, device=None):
        self.chain = chain
        cfgs = chain.cfgs if hasattr(chain, "cfgs") else list(chain)
        if cfgs[0].in_dims != cfgs[-1].out_dims:
            raise ValueError("a NeuralODE RHS needs the chain's output size == input size")
        self.hd = KanodeHandle(cfgs, dtype=dtype, rhs_kind="chain", device=device)
        self.P, self.N = self.hd.P, self.hd.N

    def __call__(self, u: torch.Tensor, p: torch.Tensor, t=None) -> torch.Tensor:
        return rhs_apply(self.hd, p, u)

    def stage(self, u, p, ks, c, want_y=False, error=None):
        """Fused Runge-Kutta stage f(u + Σ c_j k_j) (see kanode_rhs_stage)."""
        return stage_apply(self.hd, p, u, ks, c, want_y, error)

    def vjp_stage(self, u, p, ks, c, lam, lks, lc, lam_out=None, error=None):
        """Adjoint stage (see kanode_vjp_stage): (λsᵀ∂f/∂u, λsᵀ∂f/∂p) at u + Σ c_j k_j."""
        return self.hd.vjp_stage(p, u, ks, c, lam, lks, lc, lam_out, error)

    def rhs(self, u, p, out=None):
        return self.hd.rhs(p, u, out)

    def vjp(self, u, p, lam, dp=None):
        return self.hd.vjp(p, u, lam, dp=dp)


def fisher_kpp_laplacian(nx: int, dx: float) -> np.ndarray:
    """The reference's dense periodic Laplacian (Fisher-KPP_Source.jl:55-59), for host-side checks."""
    lap = (np.diag(-2.0 * np.ones(nx)) + np.diag(np.ones(nx - 1), 1) + np.diag(np.ones(nx - 1), -1)) / dx ** 2
    lap[0, -1] = 1.0 / dx ** 2
    lap[-1, 0] = 1.0 / dx ** 2
    return lap


class FisherKPPRHS:
    """rc_kanode: du = D * lap * u + KDense(1,1,G).(u) pointwise, u (B, Nx) [Julia u[Nx, B]].

    A hand-written ODEProblem in the reference (no NeuralODE, no sensealg given: Fisher-KPP_Source.jl:102-103,198),
    so its gradient is SciMLSensitivity's automatic choice (auto_sensealg): ForwardDiffSensitivity for small
    problems, else the InterpolatingAdjoint."""

    auto_sensealg = True

    def __init__(self, kan1, nx: int, dx: float, D: float = 0.01, dtype=torch.float64, device=None,
                 table: bool | None = None):
        layer = kan1[0] if hasattr(kan1, "layers") else kan1
        cfg = layer.cfg if hasattr(layer, "cfg") else layer
        if not isinstance(cfg, LayerCfg) or cfg.in_dims != 1 or cfg.out_dims != 1:
            raise ValueError("Fisher-KPP source term needs one KDense(1, 1, G)")
        self.cfg, self.nx, self.dx, self.D = cfg, int(nx), float(dx), float(D)
        self.hd = KanodeHandle([cfg], dtype=dtype, rhs_kind="pointwise_periodic_laplacian", nx=nx,
                               diffusion=D, dx=dx, device=device)
        if table is not None:   # None: the library default (table where admissible)
            self.hd.pointwise_table = table
        self.P, self.N = self.hd.P, self.hd.N

    def __call__(self, u: torch.Tensor, p: torch.Tensor, t=None) -> torch.Tensor:
        return rhs_apply(self.hd, p, u)

    def stage(self, u, p, ks, c, want_y=False, error=None):
        """Fused Runge-Kutta stage f(u + Σ c_j k_j) (see kanode_rhs_stage)."""
        return stage_apply(self.hd, p, u, ks, c, want_y, error)

    def vjp_stage(self, u, p, ks, c, lam, lks, lc, lam_out=None, error=None):
        """Adjoint stage (see kanode_vjp_stage): (λsᵀ∂f/∂u, λsᵀ∂f/∂p) at u + Σ c_j k_j."""
        return self.hd.vjp_stage(p, u, ks, c, lam, lks, lc, lam_out, error)

    def rhs(self, u, p, out=None):
        return self.hd.rhs(p, u, out)

    def vjp(self, u, p, lam, dp=None):
        return self.hd.vjp(p, u, lam, dp=dp)
