"""Owning wrapper of a `kanode_handle*` — device tensors in, device tensors out.

Array convention: a Julia column-major [N, B] array (one trajectory contiguous)
is a C-contiguous torch tensor of shape (B, N): identical memory, so no copies
cross the boundary.  The flat parameter vector is the ComponentArray order
(include/kanode.h).  Every call is asynchronous on torch's current stream.
"""
from __future__ import annotations

import contextlib
import ctypes as C
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib as L


@dataclass(frozen=True)
class LayerCfg:
    """One KDense layer's constructor arguments (kdense.jl:20-37)."""
    in_dims: int
    out_dims: int
    grid_len: int
    normalizer: str = "tanh_fast"
    basis: str = "rbf"
    use_base_act: bool = True
    grid_lims: tuple = (-1.0, 1.0)
    denominator: float | None = None
    iqf_reference_quirk: bool = True

    def to_c(self) -> L.LayerSpecC:
        if self.normalizer not in L.NORM:
            raise ValueError(f"normalizer {self.normalizer!r} not in {sorted(L.NORM)}")
        if self.basis not in L.BASIS:
            raise ValueError(f"basis_func {self.basis!r} not in {sorted(L.BASIS)}")
        den = 0.0 if self.denominator is None else float(np.float32(self.denominator))
        return L.LayerSpecC(self.in_dims, self.out_dims, self.grid_len, L.NORM[self.normalizer],
                            L.BASIS[self.basis], int(bool(self.use_base_act)),
                            float(np.float32(self.grid_lims[0])), float(np.float32(self.grid_lims[1])), den,
                            int(bool(self.iqf_reference_quirk)))

    @property
    def param_length(self) -> int:
        n = self.in_dims * self.grid_len * self.out_dims
        return n + (self.in_dims * self.out_dims if self.use_base_act else 0)


_DT = {torch.float32: L.F32, torch.float64: L.F64}


def _ptr(t: torch.Tensor | None):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(device: torch.device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class DenseOutput:
    """Owner of a kanode_solution* (the device-resident dense output of one solve)."""

    def __init__(self, hd):
        self.hd = hd
        self.ptr = C.c_void_p()

    @property
    def steps(self) -> int:
        return int(L.lib().kanode_solution_steps(self.ptr)) if self.ptr.value else 0

    def step_sizes(self):
        """(t_n, dt_n) of the accepted steps, float64 numpy arrays (kanode_solution_step_sizes)."""
        n = self.steps
        ts, dts = np.zeros(n), np.zeros(n)
        if n:
            L.lib().kanode_solution_step_sizes(self.ptr, ts.ctypes.data, dts.ctypes.data, n)
        return ts, dts

    def __del__(self):
        if getattr(self, "ptr", None) is not None and self.ptr.value:
            try:
                L.lib().kanode_solution_free(self.ptr)
            except Exception:
                pass
            self.ptr = C.c_void_p()


class KanodeHandle:
    """A configured RHS (chain or pointwise+periodic-Laplacian) bound to one device."""

    def __init__(self, layers, dtype=torch.float64, rhs_kind: str = "chain", nx: int = 0,
                 diffusion: float = 0.0, dx: float = 1.0, device=None):
        if dtype not in _DT:
            raise TypeError("dtype must be torch.float32 or torch.float64")
        layers = list(layers)
        if not 1 <= len(layers) <= L.MAX_LAYERS:
            raise ValueError(f"need 1..{L.MAX_LAYERS} layers")
        self.layers = layers
        self.dtype = dtype
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        spec = L.SpecC()
        spec.n_layers = len(layers)
        for i, lay in enumerate(layers):
            spec.layers[i] = lay.to_c()
        spec.dtype = _DT[dtype]
        spec.rhs_kind = {"chain": L.RHS_CHAIN, "pointwise_periodic_laplacian": L.RHS_POINTWISE_PERIODIC_LAPLACIAN}[rhs_kind]
        spec.nx = int(nx)
        spec.diffusion = float(diffusion)
        spec.dx = float(dx)
        spec.device = self.device.index or 0
        h = C.c_void_p()
        st = L.lib().kanode_create(C.byref(spec), C.byref(h))
        self._h = h
        if st != L.OK:
            msg = L.lib().kanode_last_error(h).decode() if h.value else ""
            L.lib().kanode_destroy(h)
            self._h = None
            raise L.KanodeError(f"kanode_create: {L.lib().kanode_status_string(st).decode()} ({msg})")
        self.rhs_kind = rhs_kind
        self.P = int(L.lib().kanode_param_length(h))
        self.N = int(L.lib().kanode_state_length(h))          # input state length
        self.N_out = self.N if rhs_kind != "chain" else layers[-1].out_dims
        self.layer_P = [int(L.lib().kanode_layer_param_length(h, i)) for i in range(len(layers))]
        self.layer_off = list(np.cumsum([0] + self.layer_P[:-1]))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                L.lib().kanode_destroy(h)
            except Exception:
                pass
            self._h = None

    # -- helpers -----------------------------------------------------------
    def _check_t(self, t: torch.Tensor, shape, name: str) -> None:
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"{name} must be a torch tensor")
        if t.device != self.device or t.dtype != self.dtype:
            raise TypeError(f"{name} must be {self.dtype} on {self.device}, got {t.dtype} on {t.device}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
        if shape is not None and tuple(t.shape) != tuple(shape):
            raise ValueError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")

    def knots(self, layer: int = 0) -> np.ndarray:
        g = np.zeros(self.layers[layer].grid_len, np.float32)
        L.check(L.lib().kanode_knots(self._h, layer, C.c_void_p(g.ctypes.data)), self._h, "kanode_knots")
        return g

    def reserve(self, max_batch: int) -> None:
        L.check(L.lib().kanode_reserve(self._h, int(max_batch)), self._h, "kanode_reserve")

    @property
    def pointwise_table(self) -> bool:
        """POINTWISE rhs: kan1_.(u) through the per-launch polynomial table (kan_pp.hip)."""
        return L.lib().kanode_get_option(self._h, L.OPT_POINTWISE_TABLE) == 1

    @pointwise_table.setter
    def pointwise_table(self, on: bool) -> None:
        L.check(L.lib().kanode_set_option(self._h, L.OPT_POINTWISE_TABLE, 1 if on else 0), self._h,
                "kanode_set_option")

    def set_option(self, name: str, value: int) -> None:
        """kanode_set_option by name (include/kanode.h; the names are _lib.OPTIONS: pointwise_table,
        fused_step, fused_solve, fused_solve_cap, grid_rhs, grid_vjp, grid_adj_step, adj_step_rows, pair_vjp,
        pair_fuse, pair_persist, pair_persist_s, adj_fused_finish, pair_persist_max_wg, pair_persist_abort;
        last_adjoint is read-only)."""
        if name not in L.OPTIONS:
            raise KeyError(f"unknown option {name!r}; known: {sorted(L.OPTIONS)}")
        L.check(L.lib().kanode_set_option(self._h, L.OPTIONS[name], int(value)), self._h, "kanode_set_option")

    def get_option(self, name: str) -> int:
        if name not in L.OPTIONS:
            raise KeyError(f"unknown option {name!r}; known: {sorted(L.OPTIONS)}")
        return int(L.lib().kanode_get_option(self._h, L.OPTIONS[name]))

    @contextlib.contextmanager
    def options(self, **kw):
        """Temporarily set options: `with hd.options(fused_step=0): ...`."""
        old = {k: self.get_option(k) for k in kw}
        try:
            for k, v in kw.items():
                self.set_option(k, v)
            yield self
        finally:
            for k, v in old.items():
                self.set_option(k, v)

    # -- RHS -----------------------------------------------------------------
    def rhs(self, p: torch.Tensor, u: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """du (B, N_out) = f(u (B, N); p)."""
        B = u.shape[0] if u.dim() == 2 else 1
        self._check_t(p, (self.P,), "p")
        self._check_t(u, None, "u")
        if u.numel() != B * self.N:
            raise ValueError(f"u must hold B x {self.N} values, got shape {tuple(u.shape)}")
        shape = (B, self.N_out) if u.dim() == 2 else (self.N_out,)
        du = torch.empty(shape, dtype=self.dtype, device=self.device) if out is None else out
        self._check_t(du, shape, "du")
        L.check(L.lib().kanode_rhs(self._h, _ptr(p), _ptr(u), _ptr(du), B, _stream(self.device)), self._h,
                "kanode_rhs")
        return du

    @staticmethod
    def _stage_struct(ks, c, y_out=None, error=None) -> "L.StageC":
        if len(ks) != len(c) or len(ks) > L.MAX_STAGES:
            raise ValueError("ks and c must have equal length <= KANODE_MAX_STAGES")
        sg = L.StageC()
        sg.n_prev = len(ks)
        for j, (k, cj) in enumerate(zip(ks, c)):
            sg.k[j] = k.data_ptr()
            sg.c[j] = float(cj)
        if y_out is not None:
            sg.y_out = y_out.data_ptr()
        if error is not None:
            ec, abstol, reltol, sumsq = error
            if len(ec) != len(ks) + 1:
                raise ValueError("error coefficients need len(ks) + 1 entries")
            if sumsq.dtype != torch.float64 or sumsq.numel() < 1:
                raise ValueError("sumsq must be a float64 device tensor")
            sg.want_error = 1
            for j, e in enumerate(ec):
                sg.ec[j] = float(e)
            sg.abstol, sg.reltol = float(abstol), float(reltol)
            sg.error_sumsq = sumsq.data_ptr()
        return sg

    def vjp_stage(self, p, u, ks, c, lam, lks, lc, lam_out=None, error=None, dp=None):
        """Adjoint stage (kanode_vjp_stage): with y = u + Σ c_j k_j (forward dense output) and
        λs = lam + Σ lc_j lk_j (adjoint stage input, written to lam_out if given), returns
        (λsᵀ∂f/∂u at y, dp) with dp accumulated (+=) — a fresh zero vector when dp is None."""
        B = u.shape[0] if u.dim() == 2 else 1
        self._check_t(p, (self.P,), "p")
        for x, nm in [(u, "u"), (lam, "lam")] + [(k, "k") for k in ks] + [(k, "lk") for k in lks]:
            self._check_t(x, tuple(u.shape), nm)
        if lam_out is not None:
            self._check_t(lam_out, tuple(u.shape), "lam_out")
        if error is not None and error[3].device != self.device:
            raise ValueError("sumsq must live on the handle's device")
        su = self._stage_struct(ks, c)
        sl = self._stage_struct(lks, lc, lam_out, error)
        lamJ = torch.empty_like(u)
        if dp is None:
            dp = torch.zeros_like(p)
        L.check(L.lib().kanode_vjp_stage(self._h, _ptr(p), _ptr(u), C.byref(su), _ptr(lam), C.byref(sl), _ptr(lamJ),
                                         _ptr(dp), B, _stream(self.device)), self._h, "kanode_vjp_stage")
        return lamJ, dp

    def rhs_stage(self, p: torch.Tensor, u: torch.Tensor, ks, c, y_out: torch.Tensor | None = None,
                  error=None, out: torch.Tensor | None = None):
        """Runge-Kutta stage: du = f(u + Σ_j c_j k_j; p) (kanode_rhs_stage).

        ks: sequence of (B, N) tensors; c: their coefficients; y_out: optional tensor
        receiving the stage input; error: optional (ec, abstol, reltol, sumsq) with ec of
        len(ks)+1 coefficients and sumsq a 1-element float64 device tensor that receives
        Σ (e / (abstol + reltol·max(|u|,|y|)))², e = Σ ec_j k_j + ec_last du."""
        B = u.shape[0] if u.dim() == 2 else 1
        if len(ks) != len(c) or len(ks) > L.MAX_STAGES:
            raise ValueError("ks and c must have equal length <= KANODE_MAX_STAGES")
        self._check_t(p, (self.P,), "p")
        self._check_t(u, None, "u")
        for k in ks:
            self._check_t(k, tuple(u.shape), "k")
        du = torch.empty_like(u) if out is None else out
        self._check_t(du, tuple(u.shape), "du")
        sg = L.StageC()
        sg.n_prev = len(ks)
        for j, (k, cj) in enumerate(zip(ks, c)):
            sg.k[j] = k.data_ptr()
            sg.c[j] = float(cj)
        if y_out is not None:
            self._check_t(y_out, tuple(u.shape), "y_out")
            sg.y_out = y_out.data_ptr()
        if error is not None:
            ec, abstol, reltol, sumsq = error
            if len(ec) != len(ks) + 1:
                raise ValueError("error coefficients need len(ks) + 1 entries")
            if sumsq.dtype != torch.float64 or sumsq.device != self.device or sumsq.numel() < 1:
                raise ValueError("sumsq must be a float64 tensor on the handle's device")
            sg.want_error = 1
            for j, e in enumerate(ec):
                sg.ec[j] = float(e)
            sg.abstol, sg.reltol = float(abstol), float(reltol)
            sg.error_sumsq = sumsq.data_ptr()
        L.check(L.lib().kanode_rhs_stage(self._h, _ptr(p), _ptr(u), C.byref(sg), _ptr(du), B,
                                         _stream(self.device)), self._h, "kanode_rhs_stage")
        return du

    def vjp(self, p: torch.Tensor, u: torch.Tensor, lam: torch.Tensor, want_lamJ: bool = True,
            dp: torch.Tensor | None = None, accumulate_dp: bool = True):
        """(λᵀ∂f/∂u, Σ_b λᵀ∂f/∂p).  dp (if given) is ACCUMULATED into."""
        B = u.shape[0] if u.dim() == 2 else 1
        self._check_t(p, (self.P,), "p")
        self._check_t(u, None, "u")
        self._check_t(lam, (B, self.N_out) if u.dim() == 2 else (self.N_out,), "lam")
        lamJ = torch.empty_like(u) if want_lamJ else None
        if dp is None and accumulate_dp:
            dp = torch.zeros_like(p)
        L.check(L.lib().kanode_vjp(self._h, _ptr(p), _ptr(u), _ptr(lam), _ptr(lamJ), _ptr(dp), B,
                                   _stream(self.device)), self._h, "kanode_vjp")
        return lamJ, dp

    # -- integrator (kanode_solve_tsit5 / kanode_adjoint_tsit5) --------------------
    def solve_tsit5(self, p: torch.Tensor, u0: torch.Tensor, t0: float, tf: float, saveat, opts: "L.SolverOptsC",
                    keep_dense: bool = False):
        """Native Tsit5 solve on the device: (u_save (len(saveat), *u0.shape), stats dict,
        DenseOutput or None).  saveat: ascending floats within [t0, tf]."""
        B = u0.shape[0] if u0.dim() == 2 else 1
        self._check_t(p, (self.P,), "p")
        self._check_t(u0, None, "u0")
        if u0.numel() != B * self.N or self.N_out != self.N:
            raise ValueError("solve needs u0 of B x N entries and an RHS with N_in == N_out")
        sv = self._saveat_c(saveat)
        u_save = torch.empty((len(saveat),) + tuple(u0.shape), dtype=self.dtype, device=self.device)
        st = L.SolveStatsC()
        dense = None
        dptr = None
        if keep_dense:
            dense = self._dense_pool.pop() if getattr(self, "_dense_pool", None) else DenseOutput(self)
            dptr = C.byref(dense.ptr)
        L.check(L.lib().kanode_solve_tsit5(self._h, _ptr(p), _ptr(u0), B, float(t0), float(tf), sv, len(saveat),
                                           _ptr(u_save), C.byref(opts), dptr, C.byref(st), _stream(self.device)),
                self._h, "kanode_solve_tsit5")
        return u_save, dict(naccept=st.naccept, nreject=st.nreject, nf=st.nf), dense

    def _saveat_c(self, saveat):
        key = tuple(saveat)
        cache = self.__dict__.setdefault("_saveat_cache", {})
        sv = cache.get(key)
        if sv is None:   # (the C array of a saveat list, kept: training solves pass the same list every step)
            if len(cache) >= 16:
                cache.clear()
            sv = cache[key] = (C.c_double * max(1, len(saveat)))(*[float(x) for x in saveat])
        return sv

    def forward_sensitivity_supported(self, batch: int) -> bool:
        """kanode_forward_sensitivity_supported: the one-workgroup forward-sensitivity solve covers this batch."""
        return bool(L.lib().kanode_forward_sensitivity_supported(self._h, int(batch)))

    def forward_sensitivity_step_sizes(self):
        """(t_n, dt_n) of the accepted steps of the last forward_sensitivity_tsit5 (float64 numpy arrays)."""
        n = int(L.lib().kanode_forward_sensitivity_step_sizes(self._h, None, None, 0))
        ts, dts = np.zeros(max(n, 0)), np.zeros(max(n, 0))
        if n > 0:
            L.lib().kanode_forward_sensitivity_step_sizes(self._h, ts.ctypes.data, dts.ctypes.data, n)
        return ts, dts

    def forward_sensitivity_tsit5(self, p: torch.Tensor, u0: torch.Tensor, t0: float, tf: float, saveat,
                                  opts: "L.SolverOptsC"):
        """ForwardDiffSensitivity's solve (kanode_forward_sensitivity_tsit5): (u_save (n_save, *u0.shape),
        s_save (n_save, P, *u0.shape) = ∂u(saveat)/∂p, stats dict)."""
        B = u0.shape[0] if u0.dim() == 2 else 1
        self._check_t(p, (self.P,), "p")
        self._check_t(u0, None, "u0")
        if u0.numel() != B * self.N:
            raise ValueError("forward sensitivities need u0 of B x N entries")
        sv = self._saveat_c(saveat)
        u_save = torch.empty((len(saveat),) + tuple(u0.shape), dtype=self.dtype, device=self.device)
        s_save = torch.empty((len(saveat), self.P) + tuple(u0.shape), dtype=self.dtype, device=self.device)
        st = L.SolveStatsC()
        L.check(L.lib().kanode_forward_sensitivity_tsit5(self._h, _ptr(p), _ptr(u0), B, float(t0), float(tf), sv,
                                                         len(saveat), _ptr(u_save), _ptr(s_save), C.byref(opts),
                                                         C.byref(st), _stream(self.device)),
                self._h, "kanode_forward_sensitivity_tsit5")
        return u_save, s_save, dict(naccept=st.naccept, nreject=st.nreject, nf=st.nf)

    def adjoint_tsit5(self, p: torch.Tensor, dense: "DenseOutput", dl_du: torch.Tensor, opts: "L.SolverOptsC",
                      u_shape):
        """InterpolatingAdjoint over a kept forward solve: (dL/du0, dL/dp, stats)."""
        self._check_t(p, (self.P,), "p")
        self._check_t(dl_du, None, "dl_du")
        du0 = torch.empty(tuple(u_shape), dtype=self.dtype, device=self.device)
        dp = torch.empty_like(p)
        st = L.SolveStatsC()
        L.check(L.lib().kanode_adjoint_tsit5(self._h, _ptr(p), dense.ptr, _ptr(dl_du), _ptr(du0), _ptr(dp),
                                             C.byref(opts), C.byref(st), _stream(self.device)),
                self._h, "kanode_adjoint_tsit5")
        return du0, dp, dict(naccept=st.naccept, nreject=st.nreject, nf=st.nf)

    def table_rejections(self):
        """Intervals the last table builds rejected: (φ, φ', swish), -1 for a table not built yet
        (kanode_table_rejections; their points take the direct formula)."""
        out = (C.c_int32 * 3)()
        L.check(L.lib().kanode_table_rejections(self._h, out), self._h, "kanode_table_rejections")
        return tuple(int(x) for x in out)

    def adjoint_step_sizes(self):
        """The accepted step sizes of the last adjoint_tsit5 (option record_adjoint_steps; else empty)."""
        n = int(L.lib().kanode_adjoint_step_sizes(self._h, None, 0))
        hs = np.zeros(max(n, 0))
        if n > 0:
            L.lib().kanode_adjoint_step_sizes(self._h, hs.ctypes.data, n)
        return hs

    def release_dense(self, dense: "DenseOutput") -> None:
        """Return a dense output's device storage for reuse by the next solve."""
        if not hasattr(self, "_dense_pool"):
            self._dense_pool = []
        if dense is not None and dense.ptr.value and len(self._dense_pool) < 2:
            self._dense_pool.append(dense)

    # -- single layer ----------------------------------------------------------
    def layer_forward(self, layer: int, p_layer: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
        cfg = self.layers[layer]
        K = x.shape[0]
        self._check_t(p_layer, (cfg.param_length,), "p_layer")
        self._check_t(x, (K, cfg.in_dims), "x")
        y = torch.empty((K, cfg.out_dims), dtype=self.dtype, device=self.device)
        L.check(L.lib().kanode_layer_forward(self._h, layer, _ptr(p_layer), _ptr(x), _ptr(y), K,
                                             _stream(self.device)), self._h, "kanode_layer_forward")
        return y

    def layer_forward_stage(self, layer: int, p_layer: torch.Tensor, x: torch.Tensor, ks, c, y_out=None,
                            lam=None, lks=(), lc=(), ls_out=None) -> torch.Tensor:
        """kanode_layer_forward_stage: the layer at y = x + Σ c_j k_j (-> y_out if given) and, with lam,
        λs = lam + Σ lc_j lk_j -> ls_out (required then); returns the layer output (K, O)."""
        cfg = self.layers[layer]
        K = x.shape[0]
        self._check_t(p_layer, (cfg.param_length,), "p_layer")
        for a, nm in [(x, "x")] + [(k, "k") for k in ks] + ([(y_out, "y_out")] if y_out is not None else []):
            self._check_t(a, (K, cfg.in_dims), nm)
        if lam is not None:
            if ls_out is None:
                raise ValueError("layer_forward_stage: lam needs ls_out")
            for a, nm in [(lam, "lam"), (ls_out, "ls_out")] + [(k, "lk") for k in lks]:
                self._check_t(a, (K, cfg.in_dims), nm)
        sx = self._stage_struct(ks, c, y_out)
        sl = self._stage_struct(lks, lc, ls_out) if lam is not None else None
        y = torch.empty((K, cfg.out_dims), dtype=self.dtype, device=self.device)
        L.check(L.lib().kanode_layer_forward_stage(self._h, layer, _ptr(p_layer), _ptr(x), C.byref(sx), _ptr(lam),
                                                   C.byref(sl) if sl is not None else None, _ptr(y), K,
                                                   _stream(self.device)), self._h, "kanode_layer_forward_stage")
        return y

    def layer_vjp(self, layer: int, p_layer: torch.Tensor, x: torch.Tensor, ybar: torch.Tensor):
        cfg = self.layers[layer]
        K = x.shape[0]
        self._check_t(p_layer, (cfg.param_length,), "p_layer")
        self._check_t(x, (K, cfg.in_dims), "x")
        self._check_t(ybar, (K, cfg.out_dims), "ybar")
        xbar = torch.empty_like(x)
        pbar = torch.zeros_like(p_layer)
        L.check(L.lib().kanode_layer_vjp(self._h, layer, _ptr(p_layer), _ptr(x), _ptr(ybar), _ptr(xbar), _ptr(pbar),
                                         K, _stream(self.device)), self._h, "kanode_layer_vjp")
        return xbar, pbar

    def edge_activations(self, layer: int, p_layer: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
        """act (K, I, O) with act[k, i, o] = φ_{o,i}(x[k, i]) (Activation_getter.jl:28-31,48-53)."""
        cfg = self.layers[layer]
        K = x.shape[0]
        self._check_t(p_layer, (cfg.param_length,), "p_layer")
        self._check_t(x, (K, cfg.in_dims), "x")
        act = torch.empty((K, cfg.in_dims, cfg.out_dims), dtype=self.dtype, device=self.device)
        L.check(L.lib().kanode_edge_activations(self._h, layer, _ptr(p_layer), _ptr(x), _ptr(act), K,
                                                _stream(self.device)), self._h, "kanode_edge_activations")
        return act
