# KANODEHip.jl — Julia binding of libkanode.so (include/kanode.h), the shim a maintainer adds next to
# src/KolmogorovArnold.jl of the reference (INTEGRATION.md).  Not compiled or executed here: Julia is
# absent from this image.  tests/test_julia_shim.py checks it textually against the C header (every
# ccall'd symbol is declared, every mirrored struct has the header's fields in order) and checks that
# the Lux / ChainRules surface below exists and that every kernel call is guarded by the shape checks.
#
# What it replaces (file:line relative to the reference):
#   KANChainHip      Lux.Chain(KDense(...), KDense(...))           Lotka-Volterra/LV_driver_KANODE.jl:139-143
#                    incl. Lux.setup / ComponentArray(pM) axes      :143,162,173-175 (kdense.jl:70-107)
#   RCKanodeHip      rc_kanode(u, p, t)                             PDE examples/Fisher-KPP_Source.jl:95-98
#   solve_tsit5      solve(ODEProblem(f, u0, tspan, p), Tsit5(); saveat) + its InterpolatingAdjoint
#                                                                   LV_driver_KANODE.jl:180-184,
#                                                                   Fisher-KPP_Source.jl:102-103,198
module KANODEHip

using LuxCore, ChainRulesCore, Libdl, Random
using WeightInitializers: glorot_uniform

const LIB = Ref{Ptr{Cvoid}}(C_NULL)
function lib()
    if LIB[] == C_NULL
        LIB[] = Libdl.dlopen(get(ENV, "KANODE_LIB", "libkanode.so"))
    end
    return LIB[]
end
sym(s::Symbol) = Libdl.dlsym(lib(), s)
const HIPLIB = "libamdhip64"

# ---- mirrors of the C structs (include/kanode.h) ------------------------------------------------
# mirrors kanode_layer_spec
struct LayerSpec
    in_dims::Int32; out_dims::Int32; grid_len::Int32
    normalizer::Int32; basis::Int32; use_base_act::Int32
    grid_lo::Float32; grid_hi::Float32; denominator::Float32
    iqf_reference_quirk::Int32
end
# mirrors kanode_spec
struct Spec
    n_layers::Int32
    layers::NTuple{8,LayerSpec}
    dtype::Int32; rhs_kind::Int32
    nx::Int64; diffusion::Float64; dx::Float64
    device::Int32
end

const NORM = Dict(:tanh_fast => 0, :tanh => 1, :softsign => 2, :sigmoid => 3, :σ => 3, :sigmoid_fast => 4,
                  :identity => 5)
const BASIS = Dict(:rbf => 0, :rswaf => 1, :iqf => 2)
# NNlib.fast_act under allow_fast_activation = true (kdense.jl:57-61): tanh -> tanh_fast, sigmoid -> sigmoid_fast
const FAST = Dict(:tanh => :tanh_fast, :sigmoid => :sigmoid_fast, :σ => :sigmoid_fast)
const DTYPE = Dict(Float32 => Int32(0), Float64 => Int32(1))

# the drivers pass the functions themselves (basis_func = rbf, normalizer = softsign); Symbols work too
actname(f::Symbol) = f
actname(f::Function) = nameof(f)

"""layerspec(in, out, G; normalizer, basis_func, use_base_act, grid_lims, denominator, ...) — the KDense
constructor arguments (kdense.jl:20-37), with the reference's defaults: normalizer = tanh (fast_act ->
tanh_fast), basis_func = rbf, use_base_act = true, grid_lims = (-1f0, 1f0), denominator = Float32(2/(G-1))."""
function layerspec(I::Integer, O::Integer, G::Integer; normalizer = :tanh, basis_func = :rbf,
                   use_base_act::Bool = true, grid_lims = (-1.0f0, 1.0f0), denominator = Float32(2 / (G - 1)),
                   allow_fast_activation::Bool = true, iqf_reference_quirk::Bool = true)
    n = actname(normalizer)
    if allow_fast_activation
        n = get(FAST, n, n)
    end
    haskey(NORM, n) || throw(ArgumentError("normalizer $n is not implemented by libkanode"))
    b = actname(basis_func)
    haskey(BASIS, b) || throw(ArgumentError("basis_func $b is not implemented by libkanode"))
    return LayerSpec(Int32(I), Int32(O), Int32(G), Int32(NORM[n]), Int32(BASIS[b]), Int32(use_base_act),
                     Float32(grid_lims[1]), Float32(grid_lims[2]), Float32(denominator), Int32(iqf_reference_quirk))
end
pad(ls) = ntuple(i -> i <= length(ls) ? ls[i] : layerspec(1, 1, 2), 8)

# ---- the handle ----------------------------------------------------------------------------------
mutable struct Handle
    ptr::Ptr{Cvoid}
    T::DataType        # element type of u, p and every output (Float32 or Float64)
    P::Int             # kanode_param_length: the flat ComponentArray length
    nin::Int           # rows of the [N, B] input
    nout::Int          # rows of the [N, B] output
end
errmsg(ptr::Ptr{Cvoid}) = unsafe_string(ccall(sym(:kanode_last_error), Cstring, (Ptr{Cvoid},), ptr))
function Handle(ls::Vector{LayerSpec}; T::Type = Float64, rhs_kind::Integer = 0, nx::Integer = 0, D::Real = 0.0,
                dx::Real = 1.0, device::Integer = 0)
    haskey(DTYPE, T) || throw(ArgumentError("libkanode computes in Float32 or Float64, not $T"))
    s = Ref(Spec(Int32(length(ls)), pad(ls), DTYPE[T], Int32(rhs_kind), Int64(nx), Float64(D), Float64(dx),
                 Int32(device)))
    out = Ref{Ptr{Cvoid}}(C_NULL)
    st = ccall(sym(:kanode_create), Cint, (Ref{Spec}, Ref{Ptr{Cvoid}}), s, out)
    if st != 0
        msg = out[] == C_NULL ? unsafe_string(ccall(sym(:kanode_status_string), Cstring, (Cint,), st)) :
              errmsg(out[])
        out[] == C_NULL || ccall(sym(:kanode_destroy), Cvoid, (Ptr{Cvoid},), out[])
        error("kanode_create: ", msg)
    end
    P = Int(ccall(sym(:kanode_param_length), Int64, (Ptr{Cvoid},), out[]))
    nin = rhs_kind == 1 ? Int(nx) : Int(ls[1].in_dims)
    nout = rhs_kind == 1 ? Int(nx) : Int(ls[end].out_dims)
    h = Handle(out[], T, P, nin, nout)
    finalizer(x -> ccall(sym(:kanode_destroy), Cvoid, (Ptr{Cvoid},), x.ptr), h)
    return h
end
check(h::Handle, st) = st == 0 || error("libkanode: ", errmsg(h.ptr))

# Host copies in the handle's element type.  Duals (ForwardDiff) cannot go through the kernels: the
# automatic sensealg of a small problem (ForwardDiffSensitivity, e.g. Fisher-KPP at Nx = 26) must be
# replaced by InterpolatingAdjoint(autojacvec = ZygoteVJP()), whose VJPs are the rrules below.
function tohost(::Type{T}, a::AbstractArray) where {T}
    eltype(a) <: Real && !(eltype(a) <: Bool) ||
        throw(ArgumentError("libkanode takes real arrays, got eltype $(eltype(a))"))
    eltype(a) <: Union{Float32,Float64,Integer} ||
        throw(ArgumentError("eltype $(eltype(a)) cannot enter the HIP kernels (forward-mode AD?): solve with " *
                            "sensealg = InterpolatingAdjoint(autojacvec = ZygoteVJP())"))
    return a isa Array{T} ? a : Array{T}(a)
end

# every kernel call goes through these checks: the C side trusts the sizes it is given
function checkp(h::Handle, p::AbstractVector)
    length(p) == h.P || throw(DimensionMismatch("p has length $(length(p)); the KAN has $(h.P) parameters " *
                                                "(kanode_param_length)"))
    return nothing
end
function checku(h::Handle, u::AbstractVecOrMat, rows::Int, what::String)
    size(u, 1) == rows || throw(DimensionMismatch("$what has $(size(u, 1)) rows; the handle expects $rows"))
    return nothing
end

"""rhs(h, p, u) -> du: kanode_rhs_host on a Julia [N] or [N, B] array."""
function rhs(h::Handle, p::AbstractVector, u::AbstractVecOrMat)
    checkp(h, p)
    checku(h, u, h.nin, "u")
    T = h.T
    pv, uc = tohost(T, p), tohost(T, u)
    B = size(uc, 2)
    du = Matrix{T}(undef, h.nout, B)
    GC.@preserve pv uc du check(h, ccall(sym(:kanode_rhs_host), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64), h.ptr, pv, uc, du, B))
    return u isa AbstractVector ? vec(du) : du
end

"""vjp(h, p, u, λ) -> (λᵀ∂f/∂u, λᵀ∂f/∂p): kanode_vjp_host (dp starts at zero)."""
function vjp(h::Handle, p::AbstractVector, u::AbstractVecOrMat, λ::AbstractVecOrMat)
    checkp(h, p)
    checku(h, u, h.nin, "u")
    checku(h, λ, h.nout, "λ")
    size(λ, 2) == size(u, 2) || throw(DimensionMismatch("λ and u have different batch sizes"))
    h.nin == h.nout || throw(ArgumentError("the RHS VJP needs a chain with in_dims == out_dims"))
    T = h.T
    pv, uc, λc = tohost(T, p), tohost(T, u), tohost(T, λ)
    B = size(uc, 2)
    λJ = similar(uc)
    dp = zeros(T, h.P)
    GC.@preserve pv uc λc λJ dp check(h, ccall(sym(:kanode_vjp_host), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64),
        h.ptr, pv, uc, λc, λJ, dp, B))
    return λJ, dp
end

# p̄ in p's own type: a ComponentArray keeps its axes (similar), a Vector stays a Vector
ptangent(p::Vector, dp) = dp
ptangent(p::AbstractVector, dp) = copyto!(similar(p, eltype(dp)), dp)
xtangent(x::AbstractVector, g) = vec(g)
xtangent(x::AbstractMatrix, g) = g

# ---- the Lux layer -------------------------------------------------------------------------------
"""KANChainHip(layerspecs; T) — a whole KDense chain as one Lux layer, the drop-in for
`Lux.Chain(KDense(...), KDense(...))` inside NeuralODE (LV_driver_KANODE.jl:139-143,180).
`Lux.setup(rng, kan1)` returns the reference's (layer_1 = (C, W), layer_2 = (C, W)) parameters with the
same Glorot-uniform Float32 init and RNG order (kdense.jl:70-86), so `ComponentArray(pM)` has the
reference axes and `getdata(ComponentArray(pM)) ./ 1e5` (:173-175) is the flat vector the kernels take."""
struct KANChainHip <: LuxCore.AbstractLuxLayer
    h::Handle
    specs::Vector{LayerSpec}
end
KANChainHip(ls::Vector{LayerSpec}; T::Type = Float64, device::Integer = 0) = KANChainHip(Handle(ls; T, device), ls)

layernames(l::KANChainHip) = ntuple(i -> Symbol("layer_", i), length(l.specs))

function initlayer(rng::AbstractRNG, s::LayerSpec)
    C = glorot_uniform(rng, Int(s.out_dims), Int(s.grid_len) * Int(s.in_dims))   # [O, G·I]  kdense.jl:74
    if s.use_base_act == 1
        return (; C, W = glorot_uniform(rng, Int(s.out_dims), Int(s.in_dims)))   # kdense.jl:80
    end
    return (; C)
end
function LuxCore.initialparameters(rng::AbstractRNG, l::KANChainHip)
    return NamedTuple{layernames(l)}(ntuple(i -> initlayer(rng, l.specs[i]), length(l.specs)))
end
# st = (grid = collect(LinRange(grid_lims..., G)),) per layer (kdense.jl:88-92)
function LuxCore.initialstates(::AbstractRNG, l::KANChainHip)
    g(s) = (; grid = collect(LinRange(s.grid_lo, s.grid_hi, Int(s.grid_len))))
    return NamedTuple{layernames(l)}(ntuple(i -> g(l.specs[i]), length(l.specs)))
end
LuxCore.parameterlength(l::KANChainHip) = l.h.P
LuxCore.statelength(l::KANChainHip) = sum(Int(s.grid_len) for s in l.specs)

# the flat parameter vector in ComponentArray order (layer_1.C, layer_1.W, layer_2.C, ...)
flatp(p::AbstractVector) = p
flatp(p::NamedTuple) = reduce(vcat, [vec(q) for layer in values(p) for q in values(layer)])

(l::KANChainHip)(x::AbstractVecOrMat, p, st) = (rhs(l.h, flatp(p), x), st)

function ChainRulesCore.rrule(l::KANChainHip, x::AbstractVecOrMat, p::AbstractVector, st)
    y = rhs(l.h, p, x)
    function kanchain_pullback(Δ)
        ȳ = unthunk(unthunk(Δ)[1])
        if ȳ isa AbstractZero
            return (NoTangent(), ZeroTangent(), ZeroTangent(), NoTangent())
        end
        λJ, dp = vjp(l.h, p, x, ȳ)
        return (NoTangent(), xtangent(x, λJ), ptangent(p, dp), NoTangent())
    end
    return (y, st), kanchain_pullback
end

# ---- Fisher-KPP: replaces rc_kanode (PDE examples/Fisher-KPP_Source.jl:95-98) ----------------------
fk_handle(nx::Integer, dx::Real; D::Real = 0.01, G::Integer = 10, normalizer = :softsign, basis_func = :rbf,
          T::Type = Float64, device::Integer = 0) =
    Handle([layerspec(1, 1, G; normalizer, basis_func)]; T, rhs_kind = 1, nx, D, dx, device)

"""rc_kanode_hip(h)(u, p, t) = D*lap*u + kan1_.(u), differentiable (rrule -> kanode_vjp_host)."""
struct RCKanodeHip
    h::Handle
end
rc_kanode_hip(h::Handle) = RCKanodeHip(h)
(f::RCKanodeHip)(u::AbstractVecOrMat, p::AbstractVector, t) = rhs(f.h, p, u)

function ChainRulesCore.rrule(f::RCKanodeHip, u::AbstractVecOrMat, p::AbstractVector, t)
    du = rhs(f.h, p, u)
    function rc_kanode_pullback(Δ)
        ḡ = unthunk(Δ)
        if ḡ isa AbstractZero
            return (NoTangent(), ZeroTangent(), ZeroTangent(), NoTangent())
        end
        λJ, dp = vjp(f.h, p, u, ḡ)
        return (NoTangent(), xtangent(u, λJ), ptangent(p, dp), NoTangent())
    end
    return du, rc_kanode_pullback
end

# ---- the whole solve + InterpolatingAdjoint on the device (kanode_solve_tsit5 / _adjoint_tsit5) -----
# mirrors kanode_solver_options
struct SolverOptions
    abstol::Float64; reltol::Float64; dt::Float64; adaptive::Int32
    maxiters::Int64; dtmin::Float64; beta1::Float64; beta2::Float64; gamma::Float64
    qmin::Float64; qmax::Float64; qoldinit::Float64
    control::Int32; graph_steps::Int32
end
function default_options()
    o = Ref{SolverOptions}()
    ccall(sym(:kanode_solver_options_default), Cvoid, (Ref{SolverOptions},), o)
    return o[]
end
"""options(; abstol = 1e-6, reltol = 1e-3, dt, adaptive, maxiters, control): solve()'s keywords, with the
OrdinaryDiffEq defaults (include/kanode.h kanode_solver_options)."""
function options(; abstol::Real = 1e-6, reltol::Real = 1e-3, dt::Real = 0.0, adaptive::Bool = true,
                 maxiters::Integer = 100000, control::Integer = 0)
    d = default_options()
    return SolverOptions(abstol, reltol, dt, Int32(adaptive), Int64(maxiters), d.dtmin, d.beta1, d.beta2, d.gamma,
                         d.qmin, d.qmax, d.qoldinit, Int32(control), d.graph_steps)
end
# mirrors kanode_solve_stats
struct SolveStats
    naccept::Int64; nreject::Int64; nf::Int64
end

# device buffers through the HIP runtime (no AMDGPU.jl: hipMalloc / hipMemcpy / hipFree only)
hipcheck(e, what) = e == 0 || error("$what failed with hipError $e")
mutable struct DevBuf
    ptr::Ptr{Cvoid}
    nbytes::Int
end
function DevBuf(nbytes::Integer)
    r = Ref{Ptr{Cvoid}}(C_NULL)
    hipcheck(ccall((:hipMalloc, HIPLIB), Cint, (Ref{Ptr{Cvoid}}, Csize_t), r, max(nbytes, 1)), "hipMalloc")
    b = DevBuf(r[], Int(nbytes))
    finalizer(x -> ccall((:hipFree, HIPLIB), Cint, (Ptr{Cvoid},), x.ptr), b)
    return b
end
function upload(a::Array)
    b = DevBuf(sizeof(a))
    GC.@preserve a hipcheck(ccall((:hipMemcpy, HIPLIB), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t, Cint),
                                  b.ptr, a, sizeof(a), 1), "hipMemcpy H2D")
    return b
end
function download!(a::Array, b::DevBuf)
    sizeof(a) <= b.nbytes || throw(DimensionMismatch("device buffer smaller than the host array"))
    GC.@preserve a hipcheck(ccall((:hipMemcpy, HIPLIB), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t, Cint),
                                  a, b.ptr, sizeof(a), 2), "hipMemcpy D2H")
    return a
end

# the forward dense output (kanode_solution), freed with the object
mutable struct DenseOutput
    ptr::Ptr{Cvoid}
end
function DenseOutput(ptr::Ptr{Cvoid})
    d = DenseOutput(ptr)
    finalizer(x -> (x.ptr == C_NULL || ccall(sym(:kanode_solution_free), Cvoid, (Ptr{Cvoid},), x.ptr)), d)
    return d
end

# raw entry points on device pointers: returns (stats, dense::Ptr) ; dense feeds adjoint!, then free_dense
function solve!(h::Handle, p::Ptr{Cvoid}, u0::Ptr{Cvoid}, B::Integer, tspan, saveat::Vector{Float64},
                usave::Ptr{Cvoid}; opt::SolverOptions = default_options(), keep_dense::Bool = false,
                stream::Ptr{Cvoid} = C_NULL)
    st = Ref{SolveStats}()
    dense = Ref{Ptr{Cvoid}}(C_NULL)
    check(h, ccall(sym(:kanode_solve_tsit5), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64, Float64, Float64, Ptr{Float64}, Int64, Ptr{Cvoid},
         Ref{SolverOptions}, Ptr{Ptr{Cvoid}}, Ref{SolveStats}, Ptr{Cvoid}),
        h.ptr, p, u0, B, tspan[1], tspan[2], saveat, length(saveat), usave, opt,
        keep_dense ? dense : Ptr{Ptr{Cvoid}}(C_NULL), st, stream))
    return st[], dense[]
end
function adjoint!(h::Handle, p::Ptr{Cvoid}, dense::Ptr{Cvoid}, dl_du::Ptr{Cvoid}, du0::Ptr{Cvoid},
                  dp::Ptr{Cvoid}; opt::SolverOptions = default_options(), stream::Ptr{Cvoid} = C_NULL)
    st = Ref{SolveStats}()
    check(h, ccall(sym(:kanode_adjoint_tsit5), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ref{SolverOptions},
         Ref{SolveStats}, Ptr{Cvoid}), h.ptr, p, dense, dl_du, du0, dp, opt, st, stream))
    return st[]
end
free_dense(d::Ptr{Cvoid}) = ccall(sym(:kanode_solution_free), Cvoid, (Ptr{Cvoid},), d)

function solve_impl(h::Handle, u0::AbstractVecOrMat, tspan, p::AbstractVector, saveat::AbstractVector,
                    opt::SolverOptions, keep_dense::Bool)
    checkp(h, p)
    checku(h, u0, h.nin, "u0")
    h.nin == h.nout || throw(ArgumentError("an ODE RHS needs a chain with in_dims == out_dims"))
    T = h.T
    ts = Vector{Float64}(saveat)
    issorted(ts) || throw(ArgumentError("saveat must be ascending"))
    B = size(u0, 2)
    pd, ud = upload(tohost(T, p)), upload(tohost(T, u0))
    out = Array{T}(undef, h.nin, B, length(ts))
    od = DevBuf(sizeof(out))
    st, dense = solve!(h, pd.ptr, ud.ptr, B, tspan, ts, od.ptr; opt, keep_dense)
    download!(out, od)
    sol = u0 isa AbstractVector ? reshape(out, h.nin, length(ts)) : out
    return sol, st, (keep_dense ? DenseOutput(dense) : nothing), pd
end

"""solve_tsit5(h, u0, tspan, p, saveat; abstol, reltol, dt, adaptive) -> Array(sol): [N, n_save] for a
vector u0, [N, B, n_save] for a matrix (the layout of `Array(solve(prob, Tsit5(); saveat))`).
Differentiable in u0 and p by its rrule, whose pullback is kanode_adjoint_tsit5: SciMLSensitivity's
InterpolatingAdjoint, the NeuralODE default (LV_driver_KANODE.jl:180), on the device."""
function solve_tsit5(h::Handle, u0::AbstractVecOrMat, tspan, p::AbstractVector, saveat::AbstractVector; kw...)
    sol, _, _, _ = solve_impl(h, u0, tspan, p, saveat, options(; kw...), false)
    return sol
end

function ChainRulesCore.rrule(::typeof(solve_tsit5), h::Handle, u0::AbstractVecOrMat, tspan, p::AbstractVector,
                              saveat::AbstractVector; kw...)
    opt = options(; kw...)
    sol, _, dense, pd = solve_impl(h, u0, tspan, p, saveat, opt, true)
    function solve_tsit5_pullback(Δ)
        ū = unthunk(Δ)
        if ū isa AbstractZero
            return (NoTangent(), NoTangent(), ZeroTangent(), NoTangent(), ZeroTangent(), NoTangent())
        end
        T = h.T
        size(ū) == size(sol) || throw(DimensionMismatch("cotangent of the solution has the wrong shape"))
        gd = upload(tohost(T, ū))
        du0 = Array{T}(undef, size(u0))
        dp = Array{T}(undef, h.P)
        du0d, dpd = DevBuf(sizeof(du0)), DevBuf(sizeof(dp))
        adjoint!(h, pd.ptr, dense.ptr, gd.ptr, du0d.ptr, dpd.ptr; opt)
        download!(du0, du0d)
        download!(dp, dpd)
        return (NoTangent(), NoTangent(), du0, NoTangent(), ptangent(p, dp), NoTangent())
    end
    return sol, solve_tsit5_pullback
end

# --- ForwardDiffSensitivity (kanode_forward_sensitivity_tsit5): the gradient SciMLSensitivity 7.69 picks for the
# source-term drivers at their own sizes (Fisher-KPP_Source.jl:198, Zygote.gradient(loss, p) with no sensealg and
# length(u0) + length(p) <= 100): the Dual-number solve, one partial per parameter, on the device in one workgroup.
function fsens!(h::Handle, p::Ptr{Cvoid}, u0::Ptr{Cvoid}, B::Integer, tspan, saveat::Vector{Float64},
                usave::Ptr{Cvoid}, ssave::Ptr{Cvoid}; opt::SolverOptions = default_options(),
                stream::Ptr{Cvoid} = C_NULL)
    st = Ref{SolveStats}()
    check(h, ccall(sym(:kanode_forward_sensitivity_tsit5), Cint,
        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64, Float64, Float64, Ptr{Float64}, Int64, Ptr{Cvoid}, Ptr{Cvoid},
         Ref{SolverOptions}, Ref{SolveStats}, Ptr{Cvoid}),
        h.ptr, p, u0, B, tspan[1], tspan[2], saveat, length(saveat), usave, ssave, opt, st, stream))
    return st[]
end
fsens_supported(h::Handle, B::Integer) = ccall(sym(:kanode_forward_sensitivity_supported), Int32,
                                               (Ptr{Cvoid}, Int64), h.ptr, B) == 1

"""solve_tsit5_fwd(h, u0, tspan, p, saveat; abstol, reltol) -> Array(sol), like solve_tsit5, but differentiable in p
by forward sensitivities (ForwardDiffSensitivity, the reference's automatic choice for its small source-term
problems): the rrule's pullback contracts the cotangent with ∂u(saveat)/∂p, computed in the same solve."""
function solve_tsit5_fwd(h::Handle, u0::AbstractVecOrMat, tspan, p::AbstractVector, saveat::AbstractVector; kw...)
    sol, _ = fwd_impl(h, u0, tspan, p, saveat, options(; kw...))
    return sol
end
function fwd_impl(h::Handle, u0::AbstractVecOrMat, tspan, p::AbstractVector, saveat::AbstractVector,
                  opt::SolverOptions)
    checkp(h, p)
    checku(h, u0, h.nin, "u0")
    T = h.T
    ts = Vector{Float64}(saveat)
    issorted(ts) || throw(ArgumentError("saveat must be ascending"))
    B = size(u0, 2)
    fsens_supported(h, B) || throw(ArgumentError("forward sensitivities: not covered for this handle / batch"))
    pd, ud = upload(tohost(T, p)), upload(tohost(T, u0))
    out = Array{T}(undef, h.nin, B, length(ts))
    S = Array{T}(undef, h.nin, B, h.P, length(ts))          # s_save [n_save, P, N, B] in column-major order
    od, sd = DevBuf(sizeof(out)), DevBuf(sizeof(S))
    fsens!(h, pd.ptr, ud.ptr, B, tspan, ts, od.ptr, sd.ptr; opt)
    download!(out, od)
    download!(S, sd)
    sol = u0 isa AbstractVector ? reshape(out, h.nin, length(ts)) : out
    return sol, S
end
function ChainRulesCore.rrule(::typeof(solve_tsit5_fwd), h::Handle, u0::AbstractVecOrMat, tspan, p::AbstractVector,
                              saveat::AbstractVector; kw...)
    sol, S = fwd_impl(h, u0, tspan, p, saveat, options(; kw...))
    function solve_tsit5_fwd_pullback(Δ)
        ū = unthunk(Δ)
        ū isa AbstractZero && return (NoTangent(), NoTangent(), NoTangent(), NoTangent(), ZeroTangent(), NoTangent())
        ub = reshape(ū, h.nin * size(u0, 2), 1, length(saveat))
        Sm = reshape(S, h.nin * size(u0, 2), h.P, length(saveat))
        dp = vec(sum(sum(Sm .* ub; dims = 1); dims = 3))       # Σ_j Σ_i ū_i(t_j) ∂u_i(t_j)/∂p
        return (NoTangent(), NoTangent(), NoTangent(), NoTangent(), ptangent(p, dp), NoTangent())
    end
    return sol, solve_tsit5_fwd_pullback
end

# --- data-parallel training across GPUs (kanode_comm_*): one process per GPU, each with its trajectory
# shard; after the adjoint, the flat [dp; L] (device) is SUM all-reduced over RCCL and the mean applied by
# kanode_adam_step(scale = 1/nranks).  Rank 0 calls comm_unique_id() and the host distributes the bytes
# (MPI.bcast, a file); every rank then calls Comm(nranks, rank, id, device) (collective).
const COMM_ID_BYTES = 128
function comm_unique_id()
    id = zeros(UInt8, COMM_ID_BYTES)
    st = ccall(sym(:kanode_comm_unique_id), Cint, (Ptr{UInt8},), id)
    st == 0 || error("libkanode: ", unsafe_string(ccall(sym(:kanode_comm_last_error), Cstring, (Ptr{Cvoid},), C_NULL)))
    return id
end
mutable struct Comm
    ptr::Ptr{Cvoid}
    nranks::Int
    rank::Int
end
function Comm(nranks::Integer, rank::Integer, id::Vector{UInt8}, device::Integer)
    length(id) == COMM_ID_BYTES || throw(ArgumentError("the unique id is $COMM_ID_BYTES bytes"))
    out = Ref{Ptr{Cvoid}}(C_NULL)
    st = ccall(sym(:kanode_comm_create), Cint, (Int32, Int32, Ptr{UInt8}, Int32, Ref{Ptr{Cvoid}}),
               nranks, rank, id, device, out)
    st == 0 || error("libkanode: ", unsafe_string(ccall(sym(:kanode_comm_last_error), Cstring, (Ptr{Cvoid},), C_NULL)))
    c = Comm(out[], Int(nranks), Int(rank))
    finalizer(x -> (x.ptr == C_NULL || ccall(sym(:kanode_comm_destroy), Cvoid, (Ptr{Cvoid},), x.ptr)), c)
    return c
end
"""allreduce_sum!(c, buf, count, T; stream): buf (device, count entries of T) <- Σ over the ranks, in place."""
function allreduce_sum!(c::Comm, buf::Ptr{Cvoid}, count::Integer, ::Type{T}; stream::Ptr{Cvoid} = C_NULL) where {T}
    haskey(DTYPE, T) || throw(ArgumentError("the all-reduce takes Float32 or Float64, not $T"))
    st = ccall(sym(:kanode_comm_allreduce_sum), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Int64, Int32, Ptr{Cvoid}),
               c.ptr, buf, count, DTYPE[T], stream)
    st == 0 || error("libkanode: ", unsafe_string(ccall(sym(:kanode_comm_last_error), Cstring, (Ptr{Cvoid},), c.ptr)))
    return buf
end

end # module
