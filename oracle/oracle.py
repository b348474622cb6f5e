"""ctypes binding of the CPU ORACLE (oracle/kanode_ref.c) — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker / CPU comparator.  The product package
(kan-odes_amd/kanode) never imports anything under oracle/.

Every function mirrors the reference file:line cited in oracle/kanode_ref.h.
Arrays are numpy, Julia column-major semantics: a [I, K] array is passed as a
numpy array of shape (K, I) in C order (so that x[k, i] == x_julia[i, k]).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

NORM = {"tanh_fast": 0, "tanh": 1, "softsign": 2, "sigmoid": 3, "sigmoid_fast": 4, "identity": 5}
BASIS = {"rbf": 0, "rswaf": 1, "iqf": 2}
SWISH = 100


class KrefLayer(C.Structure):
    _fields_ = [
        ("in_dims", C.c_int32), ("out_dims", C.c_int32), ("grid_len", C.c_int32),
        ("normalizer", C.c_int32), ("basis", C.c_int32), ("use_base_act", C.c_int32),
        ("grid_lo", C.c_float), ("grid_hi", C.c_float), ("denominator", C.c_float),
        ("iqf_reference_quirk", C.c_int32),
    ]


@dataclass
class LayerSpec:
    """KDense constructor arguments (Lotka-Volterra/src/kdense.jl:20-37)."""
    in_dims: int
    out_dims: int
    grid_len: int
    normalizer: str = "tanh"
    basis: str = "rbf"
    use_base_act: bool = True
    grid_lims: tuple = (-1.0, 1.0)
    denominator: float | None = None
    iqf_reference_quirk: bool = True

    def to_c(self) -> KrefLayer:
        den = self.denominator
        if den is None:
            den = float(np.float32(2.0 / (self.grid_len - 1)))  # kdense.jl:27
        return KrefLayer(self.in_dims, self.out_dims, self.grid_len, NORM[self.normalizer],
                         BASIS[self.basis], int(self.use_base_act), float(np.float32(self.grid_lims[0])),
                         float(np.float32(self.grid_lims[1])), float(np.float32(den)),
                         int(self.iqf_reference_quirk))

    def param_length(self) -> int:
        n = self.in_dims * self.grid_len * self.out_dims
        return n + (self.in_dims * self.out_dims if self.use_base_act else 0)


def _build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            _build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        LP = C.POINTER(KrefLayer)
        for dt, ct in (("f64", C.c_double), ("f32", C.c_float)):
            getattr(L, f"kref_act_{dt}").restype = ct
            getattr(L, f"kref_act_{dt}").argtypes = [C.c_int32, ct]
            getattr(L, f"kref_dact_{dt}").restype = ct
            getattr(L, f"kref_dact_{dt}").argtypes = [C.c_int32, ct]
            getattr(L, f"kref_layer_fwd_{dt}").argtypes = [LP, P, P, C.c_int64, P]
            getattr(L, f"kref_layer_vjp_{dt}").argtypes = [LP, P, P, P, C.c_int64, P, P]
            getattr(L, f"kref_chain_fwd_{dt}").argtypes = [C.c_int32, LP, P, P, C.c_int64, P]
            getattr(L, f"kref_chain_vjp_{dt}").argtypes = [C.c_int32, LP, P, P, P, C.c_int64, P, P]
        L.kref_knots.argtypes = [LP, P]
        L.kref_inv_h.restype = C.c_float
        L.kref_inv_h.argtypes = [LP]
        L.kref_layer_param_length.restype = C.c_int64
        L.kref_layer_param_length.argtypes = [LP]
        L.kref_fk_rhs_f64.argtypes = [LP, P, C.c_double, C.c_double, C.c_int64, P, C.c_int64, P, C.c_int32]
        L.kref_fk_vjp_f64.argtypes = [LP, P, C.c_double, C.c_double, C.c_int64, P, P, C.c_int64, P, P]
        L.kref_edge_act_f64.argtypes = [LP, P, P, C.c_int64, P]
        L.kref_bench_fk_rhs_f64.restype = C.c_double
        L.kref_bench_fk_rhs_f64.argtypes = [LP, P, C.c_double, C.c_double, C.c_int64, P, C.c_int64, P,
                                            C.c_int32, C.c_int32]
        L.kref_bench_chain_f64.restype = C.c_double
        L.kref_bench_chain_f64.argtypes = [C.c_int32, LP, P, P, C.c_int64, P, C.c_int32, C.c_int32]
        L.kref_omp_max_threads.restype = C.c_int32
        L.kref_fk_epoch_f64.restype = C.c_int
        L.kref_fk_epoch_f64.argtypes = [LP, P, C.c_double, C.c_double, C.c_int64, P, C.c_int64, C.c_double, P,
                                        C.c_int32, P, C.c_double, C.c_double, C.c_int32, C.c_double, C.c_double,
                                        P, P, P, P]
        L.kref_chain_epoch_f64.restype = C.c_int
        L.kref_chain_epoch_f64.argtypes = [C.c_int32, LP, P, P, C.c_int64, C.c_double, P, C.c_int32, P, C.c_double,
                                           C.c_double, C.c_int32, C.c_double, C.c_double, P, P, P, P]
        L.kref_fk_fsens_solve_f64.restype = C.c_int
        L.kref_fk_fsens_solve_f64.argtypes = [LP, P, C.c_double, C.c_double, C.c_int64, P, C.c_int64, C.c_double, P,
                                              C.c_int32, C.c_double, C.c_double, P, P, P, P]
        L.kref_fk_fsens_epoch_f64.restype = C.c_int
        L.kref_fk_fsens_epoch_f64.argtypes = [LP, P, C.c_double, C.c_double, C.c_int64, P, C.c_int64, C.c_double, P,
                                              C.c_int32, P, C.c_double, C.c_double, C.c_double, P, P, P, P]
        L.kref_chain_solve_f64.restype = C.c_int
        L.kref_chain_solve_f64.argtypes = [C.c_int32, LP, P, P, C.c_int64, C.c_double, P, C.c_int32, C.c_double,
                                           C.c_double, P, P, P]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> C.c_void_p:
    assert a.flags["C_CONTIGUOUS"]
    return C.c_void_p(a.ctypes.data)


def _dt(a: np.ndarray) -> str:
    return {np.dtype(np.float64): "f64", np.dtype(np.float32): "f32"}[a.dtype]


def knots(spec: LayerSpec) -> np.ndarray:
    g = np.zeros(spec.grid_len, np.float32)
    lib().kref_knots(C.byref(spec.to_c()), _ptr(g))
    return g


def inv_h(spec: LayerSpec) -> np.float32:
    return np.float32(lib().kref_inv_h(C.byref(spec.to_c())))


def act(which: str, x: float, dtype=np.float64) -> float:
    w = SWISH if which == "swish" else NORM[which]
    f = lib().kref_act_f64 if dtype == np.float64 else lib().kref_act_f32
    return f(w, x)


def dact(which: str, x: float, dtype=np.float64) -> float:
    w = SWISH if which == "swish" else NORM[which]
    f = lib().kref_dact_f64 if dtype == np.float64 else lib().kref_dact_f32
    return f(w, x)


def layer_fwd(spec: LayerSpec, p: np.ndarray, x: np.ndarray) -> np.ndarray:
    """x: (K, I) -> y: (K, O)."""
    x = np.ascontiguousarray(x)
    p = np.ascontiguousarray(p, dtype=x.dtype)
    K = x.shape[0]
    y = np.zeros((K, spec.out_dims), x.dtype)
    getattr(lib(), f"kref_layer_fwd_{_dt(x)}")(C.byref(spec.to_c()), _ptr(p), _ptr(x), K, _ptr(y))
    return y


def layer_vjp(spec: LayerSpec, p: np.ndarray, x: np.ndarray, ybar: np.ndarray):
    x = np.ascontiguousarray(x)
    p = np.ascontiguousarray(p, dtype=x.dtype)
    ybar = np.ascontiguousarray(ybar, dtype=x.dtype)
    K = x.shape[0]
    xbar = np.zeros_like(x)
    pbar = np.zeros_like(p)
    getattr(lib(), f"kref_layer_vjp_{_dt(x)}")(C.byref(spec.to_c()), _ptr(p), _ptr(x), _ptr(ybar), K,
                                                _ptr(xbar), _ptr(pbar))
    return xbar, pbar


def _layers(specs):
    arr = (KrefLayer * len(specs))(*[s.to_c() for s in specs])
    return arr


def chain_fwd(specs, p: np.ndarray, x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x)
    p = np.ascontiguousarray(p, dtype=x.dtype)
    K = x.shape[0]
    y = np.zeros((K, specs[-1].out_dims), x.dtype)
    getattr(lib(), f"kref_chain_fwd_{_dt(x)}")(len(specs), _layers(specs), _ptr(p), _ptr(x), K, _ptr(y))
    return y


def chain_vjp(specs, p: np.ndarray, x: np.ndarray, ybar: np.ndarray):
    x = np.ascontiguousarray(x)
    p = np.ascontiguousarray(p, dtype=x.dtype)
    ybar = np.ascontiguousarray(ybar, dtype=x.dtype)
    K = x.shape[0]
    xbar = np.zeros_like(x)
    pbar = np.zeros_like(p)
    getattr(lib(), f"kref_chain_vjp_{_dt(x)}")(len(specs), _layers(specs), _ptr(p), _ptr(x), _ptr(ybar), K,
                                                _ptr(xbar), _ptr(pbar))
    return xbar, pbar


def fk_rhs(spec: LayerSpec, p: np.ndarray, D: float, dx: float, u: np.ndarray, dense: bool = False):
    """u: (B, Nx) float64 -> du (B, Nx).  Fisher-KPP_Source.jl:95-98."""
    u = np.ascontiguousarray(u, dtype=np.float64)
    p = np.ascontiguousarray(p, dtype=np.float64)
    B, Nx = u.shape
    du = np.zeros_like(u)
    lib().kref_fk_rhs_f64(C.byref(spec.to_c()), _ptr(p), D, dx, Nx, _ptr(u), B, _ptr(du), int(dense))
    return du


def fk_vjp(spec: LayerSpec, p: np.ndarray, D: float, dx: float, u: np.ndarray, lam: np.ndarray):
    u = np.ascontiguousarray(u, dtype=np.float64)
    lam = np.ascontiguousarray(lam, dtype=np.float64)
    p = np.ascontiguousarray(p, dtype=np.float64)
    B, Nx = u.shape
    lamJ = np.zeros_like(u)
    dp = np.zeros_like(p)
    lib().kref_fk_vjp_f64(C.byref(spec.to_c()), _ptr(p), D, dx, Nx, _ptr(u), _ptr(lam), B, _ptr(lamJ), _ptr(dp))
    return lamJ, dp


def edge_act(spec: LayerSpec, p: np.ndarray, x: np.ndarray) -> np.ndarray:
    """x: (K, I) -> act (K, I, O) with act[k, i, o] (Activation_getter.jl:28-31,48-53)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    p = np.ascontiguousarray(p, dtype=np.float64)
    K = x.shape[0]
    a = np.zeros((K, spec.in_dims, spec.out_dims), np.float64)
    lib().kref_edge_act_f64(C.byref(spec.to_c()), _ptr(p), _ptr(x), K, _ptr(a))
    return a


def bench_fk_rhs(spec: LayerSpec, p, D, dx, u, reps: int, threads: int) -> float:
    u = np.ascontiguousarray(u, dtype=np.float64)
    p = np.ascontiguousarray(p, dtype=np.float64)
    B, Nx = u.shape
    du = np.zeros_like(u)
    return lib().kref_bench_fk_rhs_f64(C.byref(spec.to_c()), _ptr(p), D, dx, Nx, _ptr(u), B, _ptr(du),
                                       reps, threads)


def bench_chain(specs, p, x, reps: int, threads: int) -> float:
    x = np.ascontiguousarray(x, dtype=np.float64)
    p = np.ascontiguousarray(p, dtype=np.float64)
    K = x.shape[0]
    y = np.zeros((K, specs[-1].out_dims), np.float64)
    return lib().kref_bench_chain_f64(len(specs), _layers(specs), _ptr(p), _ptr(x), K, _ptr(y), reps, threads)


def fk_epoch(spec: LayerSpec, p: np.ndarray, D: float, dx: float, u0: np.ndarray, T: float, saveat, target,
             abstol=1e-6, reltol=1e-3, adaptive=True, dt=0.0, eta=1e-2):
    """One Fisher-KPP training epoch in C on one core (oracle/cpu_epoch.c): Tsit5 solve with dense
    output, MSE loss, InterpolatingAdjoint gradient, one Adam step (first step of a fresh optimiser).
    u0 (B, Nx); target (n_save, B, Nx).  Returns (loss, grad, p_new, stats dict, seconds)."""
    u0 = np.ascontiguousarray(u0, dtype=np.float64)
    B, Nx = u0.shape
    sv = np.ascontiguousarray(saveat, dtype=np.float64)
    tg = np.ascontiguousarray(target, dtype=np.float64)
    assert tg.shape == (sv.size, B, Nx)
    pn = np.ascontiguousarray(p, dtype=np.float64).copy()
    grad = np.zeros_like(pn)
    loss = C.c_double()
    secs = C.c_double()
    st = np.zeros(4, np.int64)
    rc = lib().kref_fk_epoch_f64(C.byref(spec.to_c()), _ptr(pn), D, dx, Nx, _ptr(u0), B, T, _ptr(sv), sv.size,
                                 _ptr(tg), abstol, reltol, int(adaptive), dt, eta, C.byref(loss), _ptr(grad),
                                 _ptr(st), C.byref(secs))
    if rc != 0:
        raise RuntimeError(f"kref_fk_epoch_f64 failed ({rc})")
    stats = dict(naccept=int(st[0]), nreject=int(st[1]), adjoint_naccept=int(st[2]), adjoint_nreject=int(st[3]))
    return loss.value, grad, pn, stats, secs.value


def fk_fsens_solve(spec: LayerSpec, p: np.ndarray, D: float, dx: float, u0: np.ndarray, T: float, saveat,
                   abstol=1e-6, reltol=1e-3):
    """The ForwardDiffSensitivity Dual solve in C (oracle/cpu_epoch.c kref_fk_fsens_solve_f64): u0 (B, Nx);
    returns (u_save (n_save, B, Nx), S (n_save, P, B, Nx), stats dict, seconds)."""
    u0 = np.ascontiguousarray(u0, dtype=np.float64)
    B, Nx = u0.shape
    sv = np.ascontiguousarray(saveat, dtype=np.float64)
    P = spec.in_dims * spec.grid_len * spec.out_dims + spec.in_dims * spec.out_dims
    us = np.zeros((sv.size, B, Nx))
    ss = np.zeros((sv.size, P, B, Nx))
    st = np.zeros(2, np.int64)
    secs = C.c_double()
    rc = lib().kref_fk_fsens_solve_f64(C.byref(spec.to_c()), _ptr(np.ascontiguousarray(p, dtype=np.float64)), D, dx,
                                       Nx, _ptr(u0), B, T, _ptr(sv), sv.size, abstol, reltol, _ptr(us), _ptr(ss),
                                       _ptr(st), C.byref(secs))
    if rc != 0:
        raise RuntimeError(f"kref_fk_fsens_solve_f64 failed ({rc})")
    return us, ss, dict(naccept=int(st[0]), nreject=int(st[1])), secs.value


def fk_fsens_epoch(spec: LayerSpec, p: np.ndarray, D: float, dx: float, u0: np.ndarray, T: float, saveat, target,
                   abstol=1e-6, reltol=1e-3, eta=1e-2):
    """One Fisher-KPP training epoch with the ForwardDiffSensitivity gradient in C on one core
    (kref_fk_fsens_epoch_f64).  Returns (loss, grad, p_new, stats dict, seconds)."""
    u0 = np.ascontiguousarray(u0, dtype=np.float64)
    B, Nx = u0.shape
    sv = np.ascontiguousarray(saveat, dtype=np.float64)
    tg = np.ascontiguousarray(target, dtype=np.float64)
    assert tg.shape == (sv.size, B, Nx)
    pn = np.ascontiguousarray(p, dtype=np.float64).copy()
    grad = np.zeros_like(pn)
    loss, secs = C.c_double(), C.c_double()
    st = np.zeros(2, np.int64)
    rc = lib().kref_fk_fsens_epoch_f64(C.byref(spec.to_c()), _ptr(pn), D, dx, Nx, _ptr(u0), B, T, _ptr(sv), sv.size,
                                       _ptr(tg), abstol, reltol, eta, C.byref(loss), _ptr(grad), _ptr(st),
                                       C.byref(secs))
    if rc != 0:
        raise RuntimeError(f"kref_fk_fsens_epoch_f64 failed ({rc})")
    return loss.value, grad, pn, dict(naccept=int(st[0]), nreject=int(st[1])), secs.value


def chain_epoch(specs, p: np.ndarray, u0: np.ndarray, T: float, saveat, target, abstol=1e-6, reltol=1e-3,
                adaptive=True, dt=0.0, eta=5e-4):
    """One NeuralODE (Lux.Chain RHS) training epoch in C on one core (oracle/cpu_epoch.c), the statement of
    kanode.Trainer.step with the InterpolatingAdjoint.  u0 (B, N); target (n_save, B, N).
    Returns (loss, grad, p_new, stats dict, seconds)."""
    u0 = np.ascontiguousarray(u0, dtype=np.float64)
    B, N = u0.shape
    sv = np.ascontiguousarray(saveat, dtype=np.float64)
    tg = np.ascontiguousarray(target, dtype=np.float64)
    assert tg.shape == (sv.size, B, N)
    pn = np.ascontiguousarray(p, dtype=np.float64).copy()
    grad = np.zeros_like(pn)
    loss, secs = C.c_double(), C.c_double()
    st = np.zeros(4, np.int64)
    rc = lib().kref_chain_epoch_f64(len(specs), _layers(specs), _ptr(pn), _ptr(u0), B, T, _ptr(sv), sv.size, _ptr(tg),
                                    abstol, reltol, int(adaptive), dt, eta, C.byref(loss), _ptr(grad), _ptr(st),
                                    C.byref(secs))
    if rc != 0:
        raise RuntimeError(f"kref_chain_epoch_f64 failed ({rc})")
    stats = dict(naccept=int(st[0]), nreject=int(st[1]), adjoint_naccept=int(st[2]), adjoint_nreject=int(st[3]))
    return loss.value, grad, pn, stats, secs.value


def chain_solve(specs, p: np.ndarray, u0: np.ndarray, T: float, saveat, abstol=1e-6, reltol=1e-3):
    """The adaptive forward solve alone (C, one core): (pred (n_save, B, N), stats, seconds)."""
    u0 = np.ascontiguousarray(u0, dtype=np.float64)
    B, N = u0.shape
    sv = np.ascontiguousarray(saveat, dtype=np.float64)
    p = np.ascontiguousarray(p, dtype=np.float64)
    pred = np.zeros((sv.size, B, N))
    st = np.zeros(2, np.int64)
    secs = C.c_double()
    rc = lib().kref_chain_solve_f64(len(specs), _layers(specs), _ptr(p), _ptr(u0), B, T, _ptr(sv), sv.size, abstol,
                                    reltol, _ptr(pred), _ptr(st), C.byref(secs))
    if rc != 0:
        raise RuntimeError(f"kref_chain_solve_f64 failed ({rc})")
    return pred, dict(naccept=int(st[0]), nreject=int(st[1])), secs.value


def omp_max_threads() -> int:
    return int(lib().kref_omp_max_threads())
