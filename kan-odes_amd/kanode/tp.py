"""Grid-sharded (tensor-parallel) full-field KAN surrogate — BASELINE configs[3]
("Burgers_Surrogate.jl full-field KAN surrogate, 512 spatial x 200 steps, grid sharded
4xMI355X"), SURVEY §8e E1.

The surrogate RHS is du = KDense(H -> N)(KDense(N -> H)(u)) over the N-point field
(PDE examples/Burgers_Surrogate.jl:85-97: KAN [512, 10, 512]).  With the spatial grid
split over the R ranks of a process group, rank r owns the grid points [a_r, b_r):
  * its slice of the state u[a_r:b_r, B] (every Tsit5 stage combination is local);
  * layer 1's input columns C1[:, :, a_r:b_r], W1[:, a_r:b_r] -> the PARTIAL pre-activation
    h_r = Σ_{i in slice} (C1 φ(u_i) + W1 swish(u_i))  as a KDense(n_r -> H) launch;
  * one all_reduce(SUM) of the [H, B] partials per RHS (RCCL over xGMI with backend
    "nccl"; 10·B values — latency-bound, the only exchange of the forward);
  * layer 2's output rows C2[a_r:b_r, :, :], W2[a_r:b_r, :] -> du[a_r:b_r] as a
    KDense(H -> n_r) launch.
The pullback mirrors it: layer-2 VJP (local dC2/dW2 rows) -> all_reduce(SUM) of the [H, B]
hidden cotangent partials -> layer-1 VJP (local dC1/dW1 columns, local ū slice).  As an
InterpolatingAdjoint stage (`vjp_stage`, the reference's NeuralODE default sensealg,
Burgers_Surrogate.jl:97) that is: layer-1 forward at the interpolated state -> all_reduce of
the [H, B] partials -> layer-2 VJP -> all_reduce of the [H, B] hidden cotangents -> layer-1 VJP,
two 10·B-value collectives per adjoint stage and no layer-2 forward.  Every
parameter gradient is therefore shard-local: d(Σ_r L_r)/dp_r lands on the rank owning p_r,
and no gradient all-reduce is needed across the grid shards (a data-parallel group over
trajectories, if any, still all-reduces its gradients in Trainer).  The adaptive step
control's error norm is the one global reduction of the integrator: each shard's error terms stay on
the device and are all-reduced once per step (`reduce_dev`), read by the host once (the accept/reject
decision), so an adjoint step makes one host synchronisation.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .handle import KanodeHandle, LayerCfg
from .rhs import layer_apply


def shard_bounds(n: int, world: int, rank: int):
    """Contiguous, balanced split of n grid points: [a, b) of `rank`."""
    q, r = divmod(n, world)
    a = rank * q + min(rank, r)
    return a, a + q + (1 if rank < r else 0)


def shard_index(cfg1: LayerCfg, cfg2: LayerCfg, a: int, b: int) -> np.ndarray:
    """Positions in the full flat parameter vector (ComponentArray order, column-major:
    layer_1.C [H, G·N], layer_1.W [H, N], layer_2.C [N, G·H], layer_2.W [N, H];
    LV_driver_KANODE.jl:173-175) of the local vector [C1 cols, W1 cols, C2 rows, W2 rows] of the
    shard [a, b)."""
    N, H, G1, G2 = cfg1.in_dims, cfg1.out_dims, cfg1.grid_len, cfg2.grid_len
    if cfg2.in_dims != H or cfg2.out_dims != N:
        raise ValueError("a grid-sharded surrogate is KDense(N -> H) then KDense(H -> N)")
    parts = [np.arange(H * G1 * a, H * G1 * b)]                    # C1[o, g + G·i], i in [a, b): contiguous
    off = H * G1 * N
    if cfg1.use_base_act:
        parts.append(off + np.arange(H * a, H * b))                # W1[o, i]
        off += H * N
    rows = np.arange(a, b)
    parts.append(off + (rows[None, :] + N * np.arange(G2 * H)[:, None]).reshape(-1))   # C2[o, c], o in [a, b)
    off += N * G2 * H
    if cfg2.use_base_act:
        parts.append(off + (rows[None, :] + N * np.arange(H)[:, None]).reshape(-1))    # W2[o, i]
    return np.concatenate(parts)


class _AllReduceSum(torch.autograd.Function):
    """y = Σ_ranks x; backward: x̄ = Σ_ranks ȳ (the pullback of a sum over ranks)."""

    @staticmethod
    def forward(ctx, x, reduce):
        ctx.reduce = reduce
        return reduce(x.clone())

    @staticmethod
    def backward(ctx, g):
        return ctx.reduce(g.contiguous().clone()), None


class GridShardedChainRHS:
    """NeuralODE RHS of a KAN [N, H, N] surrogate with the grid sharded over `group`.

    u: (B, n_r) local slice of the Julia [N, B] state; p: the local parameter vector
    (`shard_params`).  `layer_fn(l, p_l, x)` overrides the HIP layer launches (tests run the
    CPU oracle through it); the default binds one kanode handle [KDense(n_r, H), KDense(H, n_r)]."""

    def __init__(self, cfg1: LayerCfg, cfg2: LayerCfg, group=None, dtype=torch.float64, device=None,
                 layer_fn=None):
        self.group = group if group is not None else (dist.group.WORLD if dist.is_initialized() else None)
        self.world = dist.get_world_size(self.group) if self.group is not None else 1
        self.rank = dist.get_rank(self.group) if self.group is not None else 0
        self.cfg1, self.cfg2 = cfg1, cfg2
        self.N, self.H = cfg1.in_dims, cfg1.out_dims
        self.a, self.b = shard_bounds(self.N, self.world, self.rank)
        self.n = self.b - self.a
        rep = dict(normalizer=cfg1.normalizer, basis=cfg1.basis, use_base_act=cfg1.use_base_act,
                   grid_lims=cfg1.grid_lims, denominator=cfg1.denominator, iqf_reference_quirk=cfg1.iqf_reference_quirk)
        self.local1 = LayerCfg(self.n, self.H, cfg1.grid_len, **rep)
        rep2 = dict(normalizer=cfg2.normalizer, basis=cfg2.basis, use_base_act=cfg2.use_base_act,
                    grid_lims=cfg2.grid_lims, denominator=cfg2.denominator, iqf_reference_quirk=cfg2.iqf_reference_quirk)
        self.local2 = LayerCfg(self.H, self.n, cfg2.grid_len, **rep2)
        self.P1 = self.local1.param_length
        self.P = self.P1 + self.local2.param_length
        self.index = shard_index(cfg1, cfg2, self.a, self.b)
        assert self.index.size == self.P
        self.P_full = cfg1.param_length + cfg2.param_length
        self.dtype = dtype
        if layer_fn is None:
            self._hd = KanodeHandle([self.local1, self.local2], dtype=dtype, rhs_kind="chain", device=device)
            layer_fn = lambda l, pl, x: layer_apply(self._hd, l, pl, x)   # noqa: E731
        self.layer_fn = layer_fn
        self.backend = dist.get_backend(self.group) if self.group is not None else None
        self._counts = {}

    # -- collectives ---------------------------------------------------------------
    def _allreduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return x
        if self.backend == "gloo" and x.is_cuda:      # gloo rehearsal on one GPU: stage through host
            h = x.cpu()
            dist.all_reduce(h, group=self.group)
            return h.to(x.device)
        dist.all_reduce(x, group=self.group)
        return x

    def reduce_sum(self, v: float) -> float:
        """Σ over the grid shards of a host scalar (once-per-solve quantities)."""
        if self.world == 1:
            return float(v)
        t = torch.tensor([float(v)], dtype=torch.float64)
        if self.backend == "nccl":
            t = t.cuda()
        dist.all_reduce(t, group=self.group)
        return float(t.item())

    def reduce_dev(self, t: torch.Tensor) -> torch.Tensor:
        """Σ over the grid shards of a small device tensor, without reading it on the host (the
        integrators' per-step error norms: the caller's one .item() is the step's only host sync)."""
        return self._allreduce(t.contiguous())

    def global_count(self, n: int) -> float:
        """Σ over the shards of a per-shard entry count (cached: the shard sizes are fixed)."""
        c = self._counts.get(n)
        if c is None:
            c = self._counts[n] = self.reduce_sum(float(n))
        return c

    # -- parameters -------------------------------------------------------------------
    def shard_params(self, p_full: torch.Tensor) -> torch.Tensor:
        return p_full[torch.as_tensor(self.index, device=p_full.device)].contiguous()

    def gather_params(self, p_local: torch.Tensor) -> torch.Tensor:
        """The full ComponentArray vector (for .mat checkpoints), assembled on every rank."""
        full = torch.zeros(self.P_full, dtype=p_local.dtype, device=p_local.device)
        full[torch.as_tensor(self.index, device=p_local.device)] = p_local
        return self._allreduce(full)

    # -- the RHS --------------------------------------------------------------------------
    def __call__(self, u: torch.Tensor, p: torch.Tensor, t=None) -> torch.Tensor:
        hpart = self.layer_fn(0, p[:self.P1], u)                  # (B, H) partial pre-activation
        h = _AllReduceSum.apply(hpart, self._allreduce)           # one [H, B] all-reduce per RHS
        return self.layer_fn(1, p[self.P1:], h)                   # (B, n_r): own rows of du

    @staticmethod
    def _error_sumsq(base, y, ks, out, error) -> None:
        """The embedded-error terms of kanode_stage on this shard, on the device:
        sumsq <- Σ (e / (abstol + reltol·max(|base|, |y|)))², e = Σ ec_j k_j + ec_n out."""
        ec, abstol, reltol, sumsq = error
        e = torch.zeros_like(out)
        for ej, kj in zip(ec[:-1], ks):
            e = e + ej * kj
        e = e + ec[-1] * out
        sk = abstol + reltol * torch.maximum(base.abs(), y.abs())
        sumsq.copy_(((e / sk).double() ** 2).sum().reshape(sumsq.shape))

    def stage(self, u, p, ks, c, want_y=False, error=None):
        """Fused Runge-Kutta stage (kanode/ode.py _step_fused; the statement of kanode_rhs_stage) on the
        grid shard: y = u + Σ c_j k_j formed inside the first layer's kernel (kanode_layer_forward_stage),
        one [H, B] all-reduce, the second layer on the own rows; `error` receives this shard's Σ (e/sk)²
        on the device (the integrator all-reduces it with reduce_dev).  Returns (du, y).  Under autograd
        (the discrete adjoint) the combination is composed of differentiable torch ops instead."""
        recording = torch.is_grad_enabled() and (p.requires_grad or u.requires_grad or any(k.requires_grad for k in ks))
        if recording or not hasattr(self, "_hd"):
            y = u
            for cj, kj in zip(c, ks):
                y = torch.addcmul(y, kj, torch.full_like(kj, cj))
            du = self(y, p)
        else:
            y = torch.empty_like(u)
            hpart = self._hd.layer_forward_stage(0, p[:self.P1].contiguous(), u.contiguous(),
                                                 [k.contiguous() for k in ks], c, y_out=y)
            du = self._hd.layer_forward(1, p[self.P1:].contiguous(), self._allreduce(hpart))
        if error is not None:
            with torch.no_grad():
                self._error_sumsq(u, y, ks, du, error)
        return du, y

    def _layer_vjp(self, l: int, pl: torch.Tensor, x: torch.Tensor, g: torch.Tensor):
        """(x̄, p̄_l) of one layer: kanode_layer_vjp on the default handle; through autograd on the
        layer_fn override otherwise."""
        if hasattr(self, "_hd"):
            return self._hd.layer_vjp(l, pl.contiguous(), x.contiguous(), g.contiguous())
        with torch.enable_grad():
            x_ = x.detach().requires_grad_(True)
            p_ = pl.detach().requires_grad_(True)
            xb, pb = torch.autograd.grad(self.layer_fn(l, p_, x_), [x_, p_], g)
        return xb, pb

    def vjp_stage(self, u, p, ks, c, lam, lks, lc, lam_out=None, error=None):
        """InterpolatingAdjoint stage on the grid shard (kanode/adjoint.py; the statement of
        kanode_vjp_stage): y = u + Σ c_j k_j, λs = lam + Σ lc_j lk_j (both local slices, formed inside
        the first layer's forward kernel, kanode_layer_forward_stage), returns this rank's λsᵀ∂f/∂u rows
        and its parameters' λsᵀ∂f/∂p.  `error` receives this shard's Σ (e/sk)² on the device; the
        adjoint driver adds the μ part and all-reduces once per step (reduce_dev).  No host sync here."""
        p1, p2 = p[:self.P1].contiguous(), p[self.P1:].contiguous()
        if hasattr(self, "_hd"):
            y = torch.empty_like(u)
            ls = lam_out if lam_out is not None else torch.empty_like(lam)
            hpart = self._hd.layer_forward_stage(0, p1, u.contiguous(), [k.contiguous() for k in ks], c, y_out=y,
                                                 lam=lam.contiguous(), lks=[k.contiguous() for k in lks], lc=lc,
                                                 ls_out=ls)
            h = self._allreduce(hpart)                                            # forward to the hidden layer
        else:
            y = u
            for cj, kj in zip(c, ks):
                y = torch.addcmul(y, kj, torch.full_like(kj, cj))
            ls = lam
            for cj, kj in zip(lc, lks):
                ls = torch.addcmul(ls, kj, torch.full_like(kj, cj))
            with torch.no_grad():
                h = self._allreduce(self.layer_fn(0, p1, y).contiguous())
            if lam_out is not None:
                lam_out.copy_(ls)
        hbar, dp2 = self._layer_vjp(1, p2, h, ls)
        hbar = self._allreduce(hbar.contiguous())                                 # Σ over the output shards
        lamJ, dp1 = self._layer_vjp(0, p1, y, hbar)
        if error is not None:
            with torch.no_grad():
                self._error_sumsq(lam, ls, lks, lamJ, error)
        return lamJ, torch.cat([dp1.reshape(-1), dp2.reshape(-1)])
