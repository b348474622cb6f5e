# KANODEHip.jl — Julia binding of libkanode.so (include/kanode.h), the shim a maintainer adds next to
# src/KolmogorovArnold.jl of the reference (INTEGRATION.md).  Not compiled or executed here: Julia is
# absent from this image; tests/test_julia_shim.py checks it textually against the C header (every
# ccall'd symbol is declared, every mirrored struct has the header's fields in order).
module KANODEHip
using LuxCore, ChainRulesCore, Libdl
const LIB = Ref{Ptr{Cvoid}}(C_NULL)
lib() = (LIB[] == C_NULL && (LIB[] = Libdl.dlopen(get(ENV, "KANODE_LIB", "libkanode.so"))); LIB[])

# mirrors kanode_layer_spec / kanode_spec in include/kanode.h
struct LayerSpec
    in_dims::Int32; out_dims::Int32; grid_len::Int32
    normalizer::Int32; basis::Int32; use_base_act::Int32
    grid_lo::Float32; grid_hi::Float32; denominator::Float32
    iqf_reference_quirk::Int32
end
struct Spec
    n_layers::Int32
    layers::NTuple{8,LayerSpec}
    dtype::Int32; rhs_kind::Int32
    nx::Int64; diffusion::Float64; dx::Float64
    device::Int32
end
const NORM = Dict(:tanh_fast => 0, :tanh => 1, :softsign => 2, :sigmoid => 3, :sigmoid_fast => 4, :identity => 5)
layerspec(I, O, G; normalizer = :tanh_fast) =
    LayerSpec(I, O, G, NORM[normalizer], 0, 1, -1f0, 1f0, 0f0, 1)
pad(ls) = ntuple(i -> i <= length(ls) ? ls[i] : layerspec(1, 1, 2), 8)

mutable struct Handle; ptr::Ptr{Cvoid}; end
function Handle(ls::Vector{LayerSpec}; rhs_kind = 0, nx = 0, D = 0.0, dx = 1.0, device = 0)
    s = Ref(Spec(length(ls), pad(ls), 1, rhs_kind, nx, D, dx, device))
    out = Ref{Ptr{Cvoid}}(C_NULL)
    st = ccall(dlsym(lib(), :kanode_create), Cint, (Ref{Spec}, Ref{Ptr{Cvoid}}), s, out)
    st == 0 || error("kanode_create: ", unsafe_string(ccall(dlsym(lib(), :kanode_last_error), Cstring, (Ptr{Cvoid},), out[])))
    h = Handle(out[]); finalizer(x -> ccall(dlsym(lib(), :kanode_destroy), Cvoid, (Ptr{Cvoid},), x.ptr), h); h
end
check(h, st) = st == 0 || error(unsafe_string(ccall(dlsym(lib(), :kanode_last_error), Cstring, (Ptr{Cvoid},), h.ptr)))

# du = f(u; p) for u::Matrix{Float64} [N, B] (or a Vector: B = 1)
function rhs(h::Handle, p::Vector{Float64}, u::AbstractVecOrMat{Float64}, nout::Int)
    B = size(u, 2); du = similar(u, nout, B)
    GC.@preserve p u du check(h, ccall(dlsym(lib(), :kanode_rhs_host), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int64), h.ptr, p, u, du, B))
    u isa AbstractVector ? vec(du) : du
end
# (λᵀ∂f/∂u, λᵀ∂f/∂p)
function vjp(h::Handle, p::Vector{Float64}, u::AbstractVecOrMat{Float64}, λ::AbstractVecOrMat{Float64})
    B = size(u, 2); λJ = similar(u); dp = zero(p)
    GC.@preserve p u λ λJ dp check(h, ccall(dlsym(lib(), :kanode_vjp_host), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int64),
        h.ptr, p, u, λ, λJ, dp, B))
    λJ, dp
end

# A whole KDense chain as one Lux layer: drop-in for `Lux.Chain(KDense(...), KDense(...))`
# inside NeuralODE (LV_driver_KANODE.jl:139-143,180): out-of-place, differentiable by rrule.
struct KANChainHip <: LuxCore.AbstractLuxLayer
    h::Handle; nin::Int; nout::Int; P::Int
end
KANChainHip(ls::Vector{LayerSpec}) = (h = Handle(ls);
    KANChainHip(h, ls[1].in_dims, ls[end].out_dims, ccall(dlsym(lib(), :kanode_param_length), Int64, (Ptr{Cvoid},), h.ptr)))
LuxCore.parameterlength(l::KANChainHip) = l.P
(l::KANChainHip)(x, p, st) = (rhs(l.h, collect(Float64, p), x, l.nout), st)
function ChainRulesCore.rrule(l::KANChainHip, x, p, st)
    pv = collect(Float64, p); y = rhs(l.h, pv, x, l.nout)
    pullback(ȳ) = ((λJ, dp) = vjp(l.h, pv, x, collect(Float64, first(ȳ)));
                   (NoTangent(), λJ, dp, NoTangent()))
    (y, st), pullback
end

# The whole forward solve + InterpolatingAdjoint on the device (kanode_solve_tsit5 /
# kanode_adjoint_tsit5).  u0, p, the saveat output and dL/du are DEVICE buffers here (e.g.
# hipMalloc'd through the same library's caller, or a ROCArray's pointer); mirrors
# kanode_solver_options / kanode_solve_stats.
struct SolverOptions
    abstol::Float64; reltol::Float64; dt::Float64; adaptive::Int32
    maxiters::Int64; dtmin::Float64; beta1::Float64; beta2::Float64; gamma::Float64
    qmin::Float64; qmax::Float64; qoldinit::Float64
    control::Int32; graph_steps::Int32
end
function default_options()
    o = Ref{SolverOptions}()
    ccall(dlsym(lib(), :kanode_solver_options_default), Cvoid, (Ref{SolverOptions},), o); o[]
end
struct SolveStats
    naccept::Int64; nreject::Int64; nf::Int64
end
# returns (stats, dense::Ptr) ; dense feeds adjoint!, then kanode_solution_free
function solve!(h::Handle, p::Ptr{Float64}, u0::Ptr{Float64}, B, tspan, saveat::Vector{Float64},
                usave::Ptr{Float64}; opt = default_options(), keep_dense = false, stream = C_NULL)
    st = Ref{SolveStats}(); dense = Ref{Ptr{Cvoid}}(C_NULL)
    check(h, ccall(dlsym(lib(), :kanode_solve_tsit5), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Int64, Float64, Float64, Ptr{Float64}, Int64, Ptr{Float64},
         Ref{SolverOptions}, Ptr{Ptr{Cvoid}}, Ref{SolveStats}, Ptr{Cvoid}),
        h.ptr, p, u0, B, tspan[1], tspan[2], saveat, length(saveat), usave, opt,
        keep_dense ? dense : Ptr{Ptr{Cvoid}}(C_NULL), st, stream))
    st[], dense[]
end
function adjoint!(h::Handle, p::Ptr{Float64}, dense::Ptr{Cvoid}, dl_du::Ptr{Float64}, du0::Ptr{Float64},
                  dp::Ptr{Float64}; opt = default_options(), stream = C_NULL)
    st = Ref{SolveStats}()
    check(h, ccall(dlsym(lib(), :kanode_adjoint_tsit5), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ref{SolverOptions},
         Ref{SolveStats}, Ptr{Cvoid}), h.ptr, p, dense, dl_du, du0, dp, opt, st, stream))
    st[]
end
free_dense(d::Ptr{Cvoid}) = ccall(dlsym(lib(), :kanode_solution_free), Cvoid, (Ptr{Cvoid},), d)

# Fisher-KPP: replaces rc_kanode (PDE examples/Fisher-KPP_Source.jl:95-98)
fk_handle(nx, dx; D = 0.01, G = 10) = Handle([layerspec(1, 1, G; normalizer = :softsign)];
                                             rhs_kind = 1, nx = nx, D = D, dx = dx)
rc_kanode_hip(h::Handle, nx) = (u, p, t) -> rhs(h, collect(Float64, p), u, nx)
end # module
