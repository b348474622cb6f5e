"""kanode — MI355X-native KAN-ODE right-hand side and adjoint (host-side mirror).

The compute path is libkanode.so (hand-written HIP kernels for gfx950 behind
the C-ABI in include/kanode.h).  This package mirrors the reference's
KolmogorovArnold.jl / Lux interface (KDense, Chain, setup) and the ODE RHS
forms its drivers solve (NeuralODE chain RHS, Fisher-KPP rc_kanode).
"""
from ._lib import KanodeError, LIB_PATH, lib
from .handle import KanodeHandle, LayerCfg
from .layers import Chain, KDense, glorot_uniform, linrange_f32
from .rhs import ChainRHS, FisherKPPRHS, fisher_kpp_laplacian, layer_apply, rhs_apply
from .ode import Solution, Tsit5Options, solve
from .adjoint import DenseRecord, interpolating_adjoint
from .train import Adam, FusedAdam, Trainer, mse_loss, reg_loss
from . import checkpoint, comm, tp
from .tp import GridShardedChainRHS

__all__ = [
    "DenseRecord", "interpolating_adjoint",
    "KanodeError", "LIB_PATH", "lib", "KanodeHandle", "LayerCfg", "Chain", "KDense", "glorot_uniform",
    "linrange_f32", "ChainRHS", "FisherKPPRHS", "fisher_kpp_laplacian", "layer_apply", "rhs_apply",
    "Solution", "Tsit5Options", "solve", "Adam", "FusedAdam", "Trainer", "mse_loss", "reg_loss", "checkpoint", "comm", "tp",
    "GridShardedChainRHS",
]
