"""ctypes binding of libkanode.so (the C-ABI declared in include/kanode.h).

This is the Python side of the drop-in boundary: it binds exactly the entry
points a Julia `ccall` shim binds.  The library is built
in-tree by `make -C kan-odes_amd` (or __graft_entry__.build()); if it is missing
this module raises — there is no CPU fallback in the product path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KANODE_LIB") or os.path.join(_HERE, "libkanode.so")   # override: experiments only

MAX_LAYERS = 8
MAX_GRID = 32

OK, ERR_INVALID_ARG, ERR_UNSUPPORTED, ERR_HIP, ERR_ALLOC, ERR_CAPTURE = range(6)
F32, F64 = 0, 1
NORM = {"tanh_fast": 0, "tanh": 1, "softsign": 2, "sigmoid": 3, "sigmoid_fast": 4, "identity": 5}
BASIS = {"rbf": 0, "rswaf": 1, "iqf": 2}
RHS_CHAIN, RHS_POINTWISE_PERIODIC_LAPLACIAN = 0, 1


class LayerSpecC(C.Structure):
    _fields_ = [
        ("in_dims", C.c_int32), ("out_dims", C.c_int32), ("grid_len", C.c_int32),
        ("normalizer", C.c_int32), ("basis", C.c_int32), ("use_base_act", C.c_int32),
        ("grid_lo", C.c_float), ("grid_hi", C.c_float), ("denominator", C.c_float),
        ("iqf_reference_quirk", C.c_int32),
    ]


class SpecC(C.Structure):
    _fields_ = [
        ("n_layers", C.c_int32),
        ("layers", LayerSpecC * MAX_LAYERS),
        ("dtype", C.c_int32),
        ("rhs_kind", C.c_int32),
        ("nx", C.c_int64),
        ("diffusion", C.c_double),
        ("dx", C.c_double),
        ("device", C.c_int32),
    ]


MAX_STAGES = 8


class StageC(C.Structure):
    """kanode_stage (include/kanode.h): Runge-Kutta stage input and fused error."""
    _fields_ = [
        ("n_prev", C.c_int32),
        ("k", C.c_void_p * MAX_STAGES),
        ("c", C.c_double * MAX_STAGES),
        ("y_out", C.c_void_p),
        ("want_error", C.c_int32),
        ("ec", C.c_double * (MAX_STAGES + 1)),
        ("abstol", C.c_double),
        ("reltol", C.c_double),
        ("error_sumsq", C.c_void_p),
    ]


class SolverOptsC(C.Structure):
    """kanode_solver_options (include/kanode.h)."""
    _fields_ = [
        ("abstol", C.c_double), ("reltol", C.c_double), ("dt", C.c_double), ("adaptive", C.c_int32),
        ("maxiters", C.c_int64), ("dtmin", C.c_double), ("beta1", C.c_double), ("beta2", C.c_double),
        ("gamma", C.c_double), ("qmin", C.c_double), ("qmax", C.c_double), ("qoldinit", C.c_double),
        ("control", C.c_int32), ("graph_steps", C.c_int32),
    ]


class SolveStatsC(C.Structure):
    _fields_ = [("naccept", C.c_int64), ("nreject", C.c_int64), ("nf", C.c_int64)]


# (name, restype, argtypes) for every symbol include/kanode.h declares
_P = C.c_void_p
_H = C.c_void_p
OPT_POINTWISE_TABLE = 1   # kanode_option
OPT_FUSED_STEP = 2
OPT_FUSED_SOLVE = 3
OPT_FUSED_SOLVE_CAP = 4
OPT_GRID_RHS = 5
OPT_GRID_VJP = 6
OPT_GRID_ADJ_STEP = 7
OPT_ADJ_STEP_ROWS = 8
OPT_PAIR_VJP = 9
OPT_PAIR_FUSE = 10
OPT_PAIR_PERSIST = 11
OPT_PAIR_PERSIST_S = 12
OPT_ADJ_FUSED_FINISH = 13
OPT_PAIR_PERSIST_MAX_WG = 14
OPT_PAIR_PERSIST_ABORT = 15
OPT_LAST_ADJOINT = 16      # read-only: a kanode_adjoint_path value
OPT_CHAIN_WIDE = 17
OPT_RECORD_ADJOINT_STEPS = 18
OPT_FK_DEVICE_LOOP = 19
ADJ_NONE, ADJ_HOST_LOOP, ADJ_CHAIN_WG, ADJ_PAIR_PERSIST, ADJ_PAIR_FALLBACK = 0, 1, 2, 3, 4   # kanode_adjoint_path
OPTIONS = {"pointwise_table": OPT_POINTWISE_TABLE, "fused_step": OPT_FUSED_STEP, "fused_solve": OPT_FUSED_SOLVE,
           "fused_solve_cap": OPT_FUSED_SOLVE_CAP, "grid_rhs": OPT_GRID_RHS, "grid_vjp": OPT_GRID_VJP,
           "grid_adj_step": OPT_GRID_ADJ_STEP, "adj_step_rows": OPT_ADJ_STEP_ROWS, "pair_vjp": OPT_PAIR_VJP,
           "pair_fuse": OPT_PAIR_FUSE, "pair_persist": OPT_PAIR_PERSIST, "pair_persist_s": OPT_PAIR_PERSIST_S,
           "adj_fused_finish": OPT_ADJ_FUSED_FINISH, "pair_persist_max_wg": OPT_PAIR_PERSIST_MAX_WG,
           "pair_persist_abort": OPT_PAIR_PERSIST_ABORT, "last_adjoint": OPT_LAST_ADJOINT,
           "chain_wide": OPT_CHAIN_WIDE, "record_adjoint_steps": OPT_RECORD_ADJOINT_STEPS,
           "fk_device_loop": OPT_FK_DEVICE_LOOP}

SIGNATURES = [
    ("kanode_create", C.c_int, [C.POINTER(SpecC), C.POINTER(C.c_void_p)]),
    ("kanode_destroy", None, [_H]),
    ("kanode_last_error", C.c_char_p, [_H]),
    ("kanode_status_string", C.c_char_p, [C.c_int]),
    ("kanode_abi_version", C.c_int32, []),
    ("kanode_param_length", C.c_int64, [_H]),
    ("kanode_layer_param_length", C.c_int64, [_H, C.c_int32]),
    ("kanode_state_length", C.c_int64, [_H]),
    ("kanode_knots", C.c_int, [_H, C.c_int32, _P]),
    ("kanode_reserve", C.c_int, [_H, C.c_int64]),
    ("kanode_set_option", C.c_int, [_H, C.c_int32, C.c_int64]),
    ("kanode_get_option", C.c_int64, [_H, C.c_int32]),
    ("kanode_rhs", C.c_int, [_H, _P, _P, _P, C.c_int64, _P]),
    ("kanode_rhs_stage", C.c_int, [_H, _P, _P, C.POINTER(StageC), _P, C.c_int64, _P]),
    ("kanode_vjp_stage", C.c_int, [_H, _P, _P, C.POINTER(StageC), _P, C.POINTER(StageC), _P, _P, C.c_int64, _P]),
    ("kanode_vjp", C.c_int, [_H, _P, _P, _P, _P, _P, C.c_int64, _P]),
    ("kanode_solver_options_default", None, [C.POINTER(SolverOptsC)]),
    ("kanode_solution_free", None, [_P]),
    ("kanode_solution_steps", C.c_int64, [_P]),
    ("kanode_solution_step_sizes", C.c_int64, [_P, _P, _P, C.c_int64]),
    ("kanode_solve_tsit5", C.c_int, [_H, _P, _P, C.c_int64, C.c_double, C.c_double, C.POINTER(C.c_double), C.c_int64,
                                     _P, C.POINTER(SolverOptsC), C.POINTER(C.c_void_p), C.POINTER(SolveStatsC), _P]),
    ("kanode_adjoint_tsit5", C.c_int, [_H, _P, _P, _P, _P, _P, C.POINTER(SolverOptsC), C.POINTER(SolveStatsC), _P]),
    ("kanode_adjoint_step_sizes", C.c_int64, [_H, _P, C.c_int64]),
    ("kanode_table_rejections", C.c_int, [_H, _P]),
    ("kanode_forward_sensitivity_tsit5", C.c_int, [_H, _P, _P, C.c_int64, C.c_double, C.c_double,
                                                   C.POINTER(C.c_double), C.c_int64, _P, _P, C.POINTER(SolverOptsC),
                                                   C.POINTER(SolveStatsC), _P]),
    ("kanode_forward_sensitivity_supported", C.c_int32, [_H, C.c_int64]),
    ("kanode_forward_sensitivity_step_sizes", C.c_int64, [_H, _P, _P, C.c_int64]),
    ("kanode_rhs_host", C.c_int, [_H, _P, _P, _P, C.c_int64]),
    ("kanode_vjp_host", C.c_int, [_H, _P, _P, _P, _P, _P, C.c_int64]),
    ("kanode_layer_forward", C.c_int, [_H, C.c_int32, _P, _P, _P, C.c_int64, _P]),
    ("kanode_layer_forward_stage", C.c_int, [_H, C.c_int32, _P, _P, C.POINTER(StageC), _P, C.POINTER(StageC), _P,
                                             C.c_int64, _P]),
    ("kanode_layer_vjp", C.c_int, [_H, C.c_int32, _P, _P, _P, _P, _P, C.c_int64, _P]),
    ("kanode_edge_activations", C.c_int, [_H, C.c_int32, _P, _P, _P, C.c_int64, _P]),
    ("kanode_adam_step", C.c_int, [_P, _P, _P, _P, C.c_int64, C.c_int32, C.c_double, C.c_double, C.c_double,
                                   C.c_double, C.c_double, C.c_double, C.c_double, _P]),
    ("kanode_comm_unique_id", C.c_int, [_P]),
    ("kanode_comm_create", C.c_int, [C.c_int32, C.c_int32, _P, C.c_int32, C.POINTER(_P)]),
    ("kanode_comm_allreduce_sum", C.c_int, [_P, _P, C.c_int64, C.c_int32, _P]),
    ("kanode_comm_size", C.c_int32, [_P]),
    ("kanode_comm_rank", C.c_int32, [_P]),
    ("kanode_comm_last_error", C.c_char_p, [_P]),
    ("kanode_comm_destroy", None, [_P]),
]
COMM_ID_BYTES = 128

_lib = None


class KanodeError(RuntimeError):
    pass


def lib() -> C.CDLL:
    """Load libkanode.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise KanodeError(
                f"{LIB_PATH} not found: build it with `make -C kan-odes_amd` "
                "(the HIP extension is required; there is no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(status: int, handle=None, what: str = "") -> None:
    if status != OK:
        L = lib()
        msg = L.kanode_last_error(handle).decode() if handle else ""
        base = L.kanode_status_string(status).decode()
        raise KanodeError(f"{what}: {base}" + (f" ({msg})" if msg else ""))
