"""Training loop pieces around the HIP RHS/VJP.

    Adam        — Flux 0.14 legacy `Adam(η, β=(0.9,0.999), ϵ=1e-8)` + `update!`
                  (LV_driver_KANODE.jl:219,287; Fisher-KPP_Source.jl:167,201;
                  Flux pinned at Lotka-Volterra/Manifest.toml:841): the torch statement
    FusedAdam   — the same step as ONE HIP launch (kanode_adam_step) with the post-all-reduce
                  mean folded in; what Trainer uses on the GPU
    mse_loss    — `mean(abs2, X .- pred)` (LV_driver_KANODE.jl:197-203, Fisher-KPP_Source.jl:107-109)
    reg_loss    — L1 + entropy on the flat p (LV_driver_KANODE.jl:187-194)
    Trainer     — one iteration = forward Tsit5 solve, loss, the gradient by the
                  InterpolatingAdjoint (the reference's NeuralODE default sensealg; native
                  kanode_adjoint_tsit5 on the GPU) wherever the RHS provides the adjoint stage,
                  ForwardDiffSensitivity for a small hand-written ODEProblem (the Fisher-KPP /
                  Allen-Cahn source drivers at their own sizes: SciMLSensitivity's automatic
                  choice; native kanode_forward_sensitivity_tsit5),
                  else the discrete adjoint (reverse mode through the stages), ONE all-reduce
                  of [∂L/∂p ; L] across the trajectory shards (RCCL over xGMI with backend
                  "nccl"; gloo on CPU), then the identical Adam step on every rank.
"""
from __future__ import annotations

import torch

from .adjoint import forward_ok, native_forward_dense, native_mse_gradient, native_mse_gradient_forward
from .ode import Solution, Tsit5Options, _saveat_list, native_ok, solve


class Adam:
    """Flux.Optimise.Adam (legacy API):  mt = β1 mt + (1-β1) Δ;  vt = β2 vt + (1-β2) Δ²;
    Δ = mt / (1-β1^t) / (√(vt / (1-β2^t)) + ϵ) · η;  x .-= Δ.

    Flux evaluates these broadcasts with its Float64 hyper-parameters, so Float32 x, mt, vt are
    promoted, computed in Float64 and rounded on store; apply! stores the step into the gradient array
    (Float32 with Float32 parameters) and update! subtracts it in Float32.  This torch statement does the same, in the
    operation order of the fused kernel (kan_optim.hip: every product and sum rounded separately), so
    the CPU and GPU trainers take the same optimiser trajectory for either dtype."""

    def __init__(self, eta: float = 1e-3, beta=(0.9, 0.999), eps: float = 1e-8):
        self.eta, self.beta, self.eps = eta, beta, eps
        self.state = {}

    def apply(self, x: torch.Tensor, d: torch.Tensor) -> torch.Tensor:
        """Advances the moments; returns the Float64 step Δ (x is not changed)."""
        b1, b2 = self.beta
        st = self.state.get(id(x))
        if st is None:
            st = [torch.zeros_like(x), torch.zeros_like(x), [b1, b2]]
            self.state[id(x)] = st
        mt, vt, bp = st
        d64 = d.double()
        m64 = b1 * mt.double() + (1.0 - b1) * d64
        v64 = b2 * vt.double() + ((1.0 - b2) * d64) * d64
        mt.copy_(m64)                                   # the stored moments (rounded for Float32)
        vt.copy_(v64)
        den = torch.sqrt(vt.double() / (1.0 - bp[1])) + self.eps
        step = (mt.double() / (1.0 - bp[0])) / den * self.eta
        bp[0] *= b1
        bp[1] *= b2
        return step

    def update(self, x: torch.Tensor, d: torch.Tensor) -> None:
        """Flux.update!(opt, x, Δ): x .-= apply!(opt, x, Δ), the step rounded to x's dtype (apply! stores it
        into the gradient array) and subtracted in that dtype."""
        with torch.no_grad():
            x.sub_(self.apply(x, d).to(x.dtype))


class FusedAdam(Adam):
    """Adam whose step is one kanode_adam_step launch on x's device (m, v device-resident, Flux's
    running powers βp kept on the host).  update(x, g, scale) applies Δ = scale·g: Trainer passes the
    SUM all-reduced gradient with scale = 1/world_size, so the mean, both moments and x -= Δ are one
    pass over the parameters instead of ~8 torch launches."""

    def update(self, x: torch.Tensor, d: torch.Tensor, scale: float = 1.0) -> None:
        from . import _lib as L
        if not x.is_cuda:
            raise L.KanodeError("FusedAdam runs on the GPU (kanode_adam_step); use kanode.Adam on the CPU")
        if x.dtype not in (torch.float32, torch.float64) or d.dtype != x.dtype or d.numel() < x.numel():
            raise L.KanodeError("FusedAdam: x and the gradient must share a float dtype and size")
        if not (x.is_contiguous() and d.is_contiguous()):
            raise L.KanodeError("FusedAdam: x and the gradient must be contiguous")
        b1, b2 = self.beta
        st = self.state.get(id(x))
        if st is None:
            st = [torch.zeros_like(x), torch.zeros_like(x), [b1, b2]]
            self.state[id(x)] = st
        mt, vt, bp = st
        dt = L.F64 if x.dtype == torch.float64 else L.F32
        stream = torch.cuda.current_stream(x.device).cuda_stream
        L.check(L.lib().kanode_adam_step(x.data_ptr(), mt.data_ptr(), vt.data_ptr(), d.data_ptr(), x.numel(), dt,
                                         float(scale), float(self.eta), float(b1), float(b2), float(self.eps),
                                         float(bp[0]), float(bp[1]), stream), None, "kanode_adam_step")
        bp[0] *= b1
        bp[1] *= b2


def mse_loss(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """mean((target - pred)²) (the drivers' loss, Fisher-KPP_Source.jl:107-108 mean(abs2, X - pred)): torch's
    fused mse_loss, one launch forward and one backward instead of a sub / pow / mean chain."""
    return torch.nn.functional.mse_loss(pred, target)


def reg_loss(p: torch.Tensor, act_reg: float = 1.0, entropy_reg: float = 1.0) -> torch.Tensor:
    l1 = torch.abs(p)
    a = torch.sum(l1)
    e = l1 / a
    return a * act_reg + (-torch.sum(e * torch.log(e))) * entropy_reg


def _group_ranks(group) -> set[int]:
    import torch.distributed as dist
    if group is None or group is dist.group.WORLD:
        return set(range(dist.get_world_size()))
    return set(dist.get_process_group_ranks(group))


def _check_orthogonal(dp_group, tp_group) -> None:
    """The data-parallel gradient group of a grid-sharded trainer may share only this rank with the
    grid-shard group: every other member of dp_group must own the same parameter slice."""
    import torch.distributed as dist
    if tp_group is None or not dist.is_initialized():
        return
    shared = (_group_ranks(dp_group) & _group_ranks(tp_group)) - {dist.get_rank()}
    if dp_group is tp_group or shared:
        raise ValueError("Trainer(tp=True): `group` must be the data-parallel group orthogonal to the rhs's "
                         f"grid-shard group (it shares ranks {sorted(shared)}); all-reducing over it would add "
                         "gradients of different parameter slices")


class Trainer:
    """KAN-ODE training on a shard of trajectories.

    rhs(u, p, t) -> du must be differentiable (kanode.ChainRHS / FisherKPPRHS are:
    their backward is the HIP VJP).  `target` has the layout of the saved solution
    (len(saveat), *u0.shape).  `group` is a torch.distributed process group (or None)."""

    def __init__(self, rhs, u0, tspan, saveat, target, p0, eta: float = 5e-4, solver: Tsit5Options | None = None,
                 sparse_reg: float = 0.0, group=None, sensealg: str | None = None, tp: bool = False):
        """tp=True: `rhs` is grid-sharded (kanode.tp.GridShardedChainRHS); u0/target/p0 are this rank's
        slices, the loss is this shard's part of the global mean, gradients are shard-local.  `group`
        is then the ORTHOGONAL data-parallel group (ranks holding the same parameter slice for other
        trajectories); passing the grid-shard group would sum slices of different parameters, so a
        group sharing any rank with rhs.group other than this one is rejected."""
        if tp and group is not None:
            _check_orthogonal(group, getattr(rhs, "group", None))
        self.rhs, self.u0, self.tspan, self.saveat, self.target = rhs, u0, tspan, saveat, target
        self.tp = tp
        self.p = p0.detach().clone()
        self.opt = FusedAdam(eta) if self.p.is_cuda else Adam(eta)
        self.solver = solver or Tsit5Options()
        self.sparse_reg = sparse_reg
        self.group = group
        self.history = []
        # the reference's default: NeuralODE passes InterpolatingAdjoint(autojacvec = ZygoteVJP()); a hand-written
        # ODEProblem (rhs.auto_sensealg: Fisher-KPP / Allen-Cahn source) gets SciMLSensitivity's automatic choice,
        # ForwardDiffSensitivity where length(u0) + length(p) <= 100 (resolved per step: "auto"); reverse mode
        # through the solver steps for an RHS without an adjoint stage
        if sensealg is None:
            sensealg = ("auto" if getattr(rhs, "auto_sensealg", False) else "interpolating_adjoint") \
                if hasattr(rhs, "vjp_stage") else "discrete"
        self.sensealg = sensealg
        self._pver = 0        # bumped by every optimiser update (keys the cached forward of eval_loss)
        self._pre = None      # (pver, path, forward payload) from eval_loss, consumed by the next step

    def predict(self, p) -> Solution:
        return solve(self.rhs, self.u0, self.tspan, p, self.saveat, self.solver, sensealg=self.sensealg)

    def _fast_path(self):
        """(saveat list, path) with path "forward" / "interpolating_adjoint" for the native plain-MSE step, or None."""
        sv = _saveat_list(self.tspan, self.saveat)
        tf = float(self.tspan[1])
        sv = [s for s in sv if s <= tf + 1e-12 * max(1.0, abs(tf))]     # as solve() filters them
        sa = self.sensealg
        fast = (not self.tp and not self.sparse_reg and tuple(self.target.shape) == (len(sv),) + tuple(self.u0.shape)
                and native_ok(self.rhs, self.u0, self.tspan, self.p, sv, self.solver))
        if sa == "auto":
            sa = "forward" if fast and forward_ok(self.rhs, self.u0, self.p) else "interpolating_adjoint"
        return sv, (sa if fast and sa in ("forward", "interpolating_adjoint") else None)

    def _drop_pre(self):
        if self._pre is not None and self._pre[1] == "interpolating_adjoint":
            self.rhs.hd.release_dense(self._pre[2][2])
        self._pre = None

    def eval_loss(self) -> float:
        """loss(p) at the current parameters, as the drivers log it after update! (LV_driver_KANODE.jl:289-290
        loss_train(p); Fisher-KPP_Source.jl:204).  On the native plain-MSE path this forward solve is exactly the
        next iteration's InterpolatingAdjoint forward (same p, u0, tspan, saveat), so its dense output is kept and
        the next step() takes its gradient from it instead of solving again.  The cache is keyed
        on the Trainer's own updates: change self.p only through step() (or call eval_loss again)."""
        self._drop_pre()
        sv, path = self._fast_path()
        if path == "interpolating_adjoint":
            pre = native_forward_dense(self.rhs, self.u0, self.tspan, self.p, sv, self.solver)
        else:
            # (in forward mode the next gradient is a Dual solve, whose error norm counts the partials: its steps
            # and values are not the logged plain solve's, so nothing is kept)
            with torch.no_grad():
                return float(mse_loss(solve(self.rhs, self.u0, self.tspan, self.p.detach(), self.saveat,
                                            self.solver).u, self.target))
        self._pre = (self._pver, path, pre)
        return float(mse_loss(pre[0], self.target))

    def loss_and_grad(self):
        sv, path = self._fast_path()
        pre = None
        if self._pre is not None:
            if self._pre[0] == self._pver and self._pre[1] == path:
                pre = self._pre[2]
                self._pre = None
            else:
                self._drop_pre()
        if path == "forward":
            # ForwardDiffSensitivity: one native call carrying ∂u/∂p (adjoint.native_mse_gradient_forward)
            loss, g, sol = native_mse_gradient_forward(self.rhs, self.u0, self.tspan, self.p, sv, self.solver,
                                                       self.target, pre=pre)
            return loss.detach(), g, sol
        if path == "interpolating_adjoint":
            # the plain-MSE step through the two native calls directly (adjoint.native_mse_gradient)
            loss, g, sol = native_mse_gradient(self.rhs, self.u0, self.tspan, self.p, sv, self.solver, self.target,
                                               pre=pre)
            return loss.detach(), g, sol
        p = self.p.detach().requires_grad_(True)
        sol = self.predict(p)
        if self.tp:   # Σ over the grid shards of these partial sums = the global mean
            loss = torch.sum((self.target - sol.u) ** 2) / self.rhs.global_count(sol.u.numel())
        else:
            loss = mse_loss(sol.u, self.target)
        if self.sparse_reg:
            loss = loss + reg_loss(p, self.sparse_reg, 0.0)
        (g,) = torch.autograd.grad(loss, p)
        return loss.detach(), g.detach(), sol

    def step(self) -> float:
        loss, g, _ = self.loss_and_grad()
        if self.tp:
            loss = torch.as_tensor(self.rhs.reduce_sum(float(loss)), dtype=g.dtype)
        scale = 1.0
        if self.group is not None:
            import torch.distributed as dist
            ws = dist.get_world_size(self.group)
            buf = torch.cat([g.reshape(-1), loss.reshape(1).to(device=g.device, dtype=g.dtype)])   # one collective per step
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
            scale = 1.0 / ws
            g, loss = buf[:-1].reshape(g.shape), buf[-1] * scale
        if isinstance(self.opt, FusedAdam):
            self.opt.update(self.p, g.contiguous(), scale)      # the mean is formed inside the launch
        else:
            self.opt.update(self.p, g * scale if scale != 1.0 else g)
        self._pver += 1
        lv = float(loss)
        self.history.append(lv)
        return lv
