"""Oracle-backed RHS objects (TEST / BASELINE INFRASTRUCTURE ONLY — never imported by the
product package): the CPU oracle's chain / Fisher-KPP forward and VJP wrapped as torch
autograd Functions, so the same Tsit5 driver integrates them on the CPU.  Used by the
ODE-level parity tests and by bench.py's CPU epoch baseline.

OracleFKRHS(dense=True) evaluates D*lap*u as the reference's dense Nx x Nx matvec
(PDE examples/Fisher-KPP_Source.jl:55-59,97) — the faithful CPU reference algorithm."""
import numpy as np
import torch

from oracle import oracle as O


class _OracleChainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, specs, p, u):
        ctx.specs = specs
        ctx.save_for_backward(p, u)
        y = O.chain_fwd(specs, p.detach().numpy(), u.detach().numpy().reshape(-1, specs[0].in_dims))
        return torch.as_tensor(y.reshape(u.shape[:-1] + (specs[-1].out_dims,)))

    @staticmethod
    def backward(ctx, g):
        p, u = ctx.saved_tensors
        s = ctx.specs
        xb, pb = O.chain_vjp(s, p.numpy(), u.numpy().reshape(-1, s[0].in_dims), g.numpy().reshape(-1, s[-1].out_dims))
        return None, torch.as_tensor(pb), torch.as_tensor(xb.reshape(u.shape))


class OracleChainRHS:
    def __init__(self, specs):
        self.specs = specs

    def __call__(self, u, p, t=None):
        return _OracleChainFn.apply(self.specs, p, u)


class _OracleFKFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec, D, dx, dense, p, u):
        ctx.cfg = (spec, D, dx)
        ctx.save_for_backward(p, u)
        return torch.as_tensor(O.fk_rhs(spec, p.detach().numpy(), D, dx, u.detach().numpy(), dense=dense))

    @staticmethod
    def backward(ctx, g):
        p, u = ctx.saved_tensors
        spec, D, dx = ctx.cfg
        lj, dp = O.fk_vjp(spec, p.numpy(), D, dx, u.numpy(), np.ascontiguousarray(g.numpy()))
        return None, None, None, None, torch.as_tensor(dp), torch.as_tensor(lj)


class OracleFKRHS:
    def __init__(self, spec, D, dx, dense=False):
        self.spec, self.D, self.dx, self.dense = spec, D, dx, bool(dense)

    def __call__(self, u, p, t=None):
        return _OracleFKFn.apply(self.spec, self.D, self.dx, self.dense, p, u)
