"""Lux-style KAN layer API — the host-side mirror of KolmogorovArnold.jl.

Names, arguments and behaviour follow the reference (file:line relative to
/root/reference):
    KDense(in, out, G; normalizer, grid_lims, denominator, basis_func, base_act,
           use_base_act, init_C, init_W, allow_fast_activation)   kdense.jl:20-68
    initialparameters / initialstates / parameterlength / statelength  kdense.jl:70-107
    (l::KDense)(x, p, st) -> (y, st)                              kdense.jl:109-130
    Lux.Chain + Lux.setup + ComponentArray flattening            LV_driver_KANODE.jl:139-143,162,173
The arithmetic runs in libkanode.so (HIP, gfx950); nothing here computes the
layer on the CPU.  A Julia [I, K] array is a torch (K, I) tensor (same memory).
"""
from __future__ import annotations

import numpy as np
import torch

from .handle import KanodeHandle, LayerCfg

# NNlib.fast_act (kdense.jl:57-61): tanh -> tanh_fast, sigmoid -> sigmoid_fast
_FAST = {"tanh": "tanh_fast", "sigmoid": "sigmoid_fast"}


def glorot_uniform(rng: np.random.Generator, out_dims: int, in_dims: int, gain: float = 1.0) -> np.ndarray:
    """WeightInitializers.glorot_uniform: U(-s, s), s = gain*sqrt(6/(fan_in+fan_out)), Float32 [out, in].
    (Init parity with Julia's RNG stream is not required: parameters are an input.)"""
    s = gain * np.sqrt(24.0 / (out_dims + in_dims)) / 2.0
    return ((rng.random((out_dims, in_dims), dtype=np.float64) - 0.5) * 2 * s).astype(np.float32)


def linrange_f32(lo: float, hi: float, n: int) -> np.ndarray:
    """collect(LinRange(lo::Float32, hi::Float32, n)) (kdense.jl:90): Float64 lerp, rounded to Float32."""
    a, b = float(np.float32(lo)), float(np.float32(hi))
    t = np.arange(n, dtype=np.float64) / (n - 1)
    return ((1.0 - t) * a + t * b).astype(np.float32)


class KDense:
    """KolmogorovArnold.KDense (kdense.jl:5-130) backed by the HIP kernels."""

    def __init__(self, in_dims: int, out_dims: int, grid_len: int, *, normalizer: str = "tanh",
                 grid_lims=(-1.0, 1.0), denominator=None, basis_func: str = "rbf", base_act: str = "swish",
                 use_base_act: bool = True, init_C=glorot_uniform, init_W=glorot_uniform,
                 allow_fast_activation: bool = True):
        if base_act != "swish":
            raise NotImplementedError("base_act: only swish (the reference default, kdense.jl:31) is implemented")
        if allow_fast_activation:
            normalizer = _FAST.get(normalizer, normalizer)
        self.in_dims, self.out_dims, self.grid_len = int(in_dims), int(out_dims), int(grid_len)
        self.normalizer = normalizer
        self.grid_lims = (float(np.float32(grid_lims[0])), float(np.float32(grid_lims[1])))
        # kdense.jl:27 — default denominator depends on grid_len only
        self.denominator = float(np.float32(2.0 / (self.grid_len - 1) if denominator is None else denominator))
        self.basis_func = basis_func
        self.base_act = base_act
        self.use_base_act = bool(use_base_act)
        self.init_C, self.init_W = init_C, init_W
        self._handles = {}

    @property
    def cfg(self) -> LayerCfg:
        return LayerCfg(self.in_dims, self.out_dims, self.grid_len, self.normalizer, self.basis_func,
                        self.use_base_act, self.grid_lims, self.denominator)

    # LuxCore interface --------------------------------------------------------
    def initialparameters(self, rng: np.random.Generator) -> dict:
        p = {"C": self.init_C(rng, self.out_dims, self.grid_len * self.in_dims)}  # [O, G, I]
        if self.use_base_act:
            p["W"] = self.init_W(rng, self.out_dims, self.in_dims)
        return p

    def initialstates(self, rng=None) -> dict:
        return {"grid": linrange_f32(self.grid_lims[0], self.grid_lims[1], self.grid_len)}

    def parameterlength(self) -> int:
        return self.cfg.param_length

    def statelength(self) -> int:
        return self.grid_len

    def flatten(self, p: dict) -> np.ndarray:
        """ComponentArray order: C then W, each column-major."""
        parts = [np.asarray(p["C"]).reshape(self.out_dims, -1).flatten(order="F")]
        if self.use_base_act:
            parts.append(np.asarray(p["W"]).reshape(self.out_dims, self.in_dims).flatten(order="F"))
        return np.concatenate(parts)

    def _handle(self, dtype, device) -> KanodeHandle:
        key = (dtype, str(device))
        if key not in self._handles:
            self._handles[key] = KanodeHandle([self.cfg], dtype=dtype, rhs_kind="chain", device=device)
        return self._handles[key]

    def __call__(self, x: torch.Tensor, p, st):
        """(l::KDense)(x, p, st) -> (y, st); x (K, I) or (I,) [Julia x[I, K]]."""
        from .rhs import layer_apply
        if isinstance(p, dict):
            p = torch.as_tensor(self.flatten(p), dtype=x.dtype, device=x.device)
        squeeze = x.dim() == 1
        xx = x.reshape(1, -1) if squeeze else x.reshape(-1, self.in_dims)
        y = layer_apply(self._handle(x.dtype, x.device), 0, p, xx.contiguous())
        return (y.reshape(-1) if squeeze else y), st

    def edge_activations(self, x: torch.Tensor, p) -> torch.Tensor:
        """act (K, I, O): per-edge φ_{o,i}(x_i) (Activation_getter.jl:20-54)."""
        if isinstance(p, dict):
            p = torch.as_tensor(self.flatten(p), dtype=x.dtype, device=x.device)
        return self._handle(x.dtype, x.device).edge_activations(0, p.contiguous(), x.contiguous())


class Chain:
    """Lux.Chain of KDense layers; `setup` returns the flat ComponentArray vector."""

    def __init__(self, *layers: KDense):
        if len(layers) == 1 and isinstance(layers[0], (list, tuple)):
            layers = tuple(layers[0])
        self.layers = list(layers)
        for a, b in zip(self.layers, self.layers[1:]):
            if a.out_dims != b.in_dims:
                raise ValueError("Chain: out_dims of a layer must equal in_dims of the next")
        self._handles = {}

    def __len__(self):
        return len(self.layers)

    def __getitem__(self, i):
        return self.layers[i]

    @property
    def cfgs(self):
        return [l.cfg for l in self.layers]

    def parameterlength(self) -> int:
        return sum(l.parameterlength() for l in self.layers)

    def initialparameters(self, rng) -> list:
        return [l.initialparameters(rng) for l in self.layers]

    def initialstates(self, rng=None) -> list:
        return [l.initialstates(rng) for l in self.layers]

    def setup(self, rng: np.random.Generator):
        """Lux.setup + getdata(ComponentArray(pM)): (flat p float32, st)."""
        pm = self.initialparameters(rng)
        return self.flatten(pm), self.initialstates(rng)

    def flatten(self, pm) -> np.ndarray:
        return np.concatenate([l.flatten(q) for l, q in zip(self.layers, pm)])

    def unflatten(self, p: np.ndarray) -> list:
        out, off = [], 0
        for l in self.layers:
            n = l.parameterlength()
            q = np.asarray(p[off:off + n])
            nC = l.out_dims * l.grid_len * l.in_dims
            d = {"C": q[:nC].reshape(l.grid_len * l.in_dims, l.out_dims).T}
            if l.use_base_act:
                d["W"] = q[nC:].reshape(l.in_dims, l.out_dims).T
            out.append(d)
            off += n
        return out

    def layer_offsets(self):
        offs, o = [], 0
        for l in self.layers:
            offs.append(o)
            o += l.parameterlength()
        return offs

    def handle(self, dtype, device) -> KanodeHandle:
        key = (dtype, str(device))
        if key not in self._handles:
            self._handles[key] = KanodeHandle(self.cfgs, dtype=dtype, rhs_kind="chain", device=device)
        return self._handles[key]

    def __call__(self, x: torch.Tensor, p, st):
        """Chain(x, p, st) -> (y, st), differentiable in x and p."""
        from .rhs import rhs_apply
        if not isinstance(p, torch.Tensor):
            p = torch.as_tensor(self.flatten(p) if isinstance(p, (list, tuple)) else np.asarray(p),
                                dtype=x.dtype, device=x.device)
        squeeze = x.dim() == 1
        xx = x.reshape(1, -1) if squeeze else x
        y = rhs_apply(self.handle(x.dtype, x.device), p, xx.contiguous())
        return (y.reshape(-1) if squeeze else y), st
