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


def _vjp_stage(vjp, u, ks, c, lam, lks, lc, lam_out, error):
    """CPU restatement of kanode_vjp_stage around an oracle VJP (same arithmetic order as the
    kernel's stage combination: fma over j ascending)."""
    y = u.clone()
    for cj, kj in zip(c, ks):
        y = torch.addcmul(y, kj, torch.full_like(kj, cj))
    ls = lam.clone()
    for cj, kj in zip(lc, lks):
        ls = torch.addcmul(ls, kj, torch.full_like(kj, cj))
    lamJ, dp = vjp(y, ls)
    if lam_out is not None:
        lam_out.copy_(ls)
    if error is not None:
        ec, abstol, reltol, sumsq = error
        e = torch.zeros_like(lam)
        for ej, kj in zip(ec[:-1], lks):
            e = e + ej * kj
        e = e + ec[-1] * lamJ
        sk = abstol + reltol * torch.maximum(lam.abs(), ls.abs())
        sumsq.fill_(float(((e / sk) ** 2).sum()))
    return lamJ, dp


class OracleChainRHS:
    def __init__(self, specs):
        self.specs = specs

    def __call__(self, u, p, t=None):
        return _OracleChainFn.apply(self.specs, p, u)

    def vjp(self, y, p, lam):
        s = self.specs
        xb, pb = O.chain_vjp(s, p.detach().numpy(), y.detach().numpy().reshape(-1, s[0].in_dims),
                             lam.detach().numpy().reshape(-1, s[-1].out_dims))
        return torch.as_tensor(xb.reshape(y.shape)), torch.as_tensor(pb)

    def vjp_stage(self, u, p, ks, c, lam, lks, lc, lam_out=None, error=None):
        return _vjp_stage(lambda y, ls: self.vjp(y, p, ls), u, ks, c, lam, lks, lc, lam_out, error)


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

    def vjp(self, y, p, lam):
        lj, dp = O.fk_vjp(self.spec, p.detach().numpy(), self.D, self.dx, y.detach().numpy(),
                          np.ascontiguousarray(lam.detach().numpy()))
        return torch.as_tensor(lj), torch.as_tensor(dp)

    def vjp_stage(self, u, p, ks, c, lam, lks, lc, lam_out=None, error=None):
        return _vjp_stage(lambda y, ls: self.vjp(y, p, ls), u, ks, c, lam, lks, lc, lam_out, error)
