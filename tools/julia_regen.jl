# julia_regen.jl — regenerate the golden OUTPUTS with the real reference stack (the reference's
# KolmogorovArnold.jl + Lux + ComponentArrays + Zygote), where Julia exists.  Not run in this image
# (no Julia; DESIGN.md §5): it is the one-command pinning recipe for a machine that has it.
#   python tools/export_golden_for_julia.py            # tests/golden/julia_in/*.mat
#   julia --project=<reference>/Lotka-Volterra tools/julia_regen.jl <reference>/Lotka-Volterra tests/golden
# writes tests/golden/julia_out/<name>.mat (y or du, xbar or lamJ, pbar or dp), which
# tests/test_julia_goldens.py compares against the C oracle (and so, through the GPU parity tests,
# against the HIP path).
using Lux, LuxCore, ComponentArrays, Zygote, MAT, NNlib, Random, LinearAlgebra

const REF = ARGS[1]
const GOLD = ARGS[2]
include(joinpath(REF, "src", "KolmogorovArnold.jl"))
using .KolmogorovArnold

const NORMS = Dict("tanh_fast" => NNlib.tanh_fast, "tanh" => tanh, "softsign" => NNlib.softsign,
                   "sigmoid" => NNlib.sigmoid, "sigmoid_fast" => NNlib.sigmoid_fast, "identity" => identity)
const BASES = Dict("rbf" => KolmogorovArnold.rbf, "rswaf" => KolmogorovArnold.rswaf, "iqf" => KolmogorovArnold.iqf)

# the drivers' KDense calls (LV_driver_KANODE.jl:139-142, Fisher-KPP_Source.jl:83-85): keyword
# arguments exactly as there, allow_fast_activation at its default (true)
function layer(d, i)
    I, O, G = Int(d["l$(i)_in_dims"]), Int(d["l$(i)_out_dims"]), Int(d["l$(i)_grid_len"])
    KDense(I, O, G; use_base_act = d["l$(i)_use_base_act"] == 1, basis_func = BASES[d["l$(i)_basis"]],
           normalizer = NORMS[d["l$(i)_normalizer"]])
end

function run_chain(d)
    n = Int(d["nlayers"])
    kan = Lux.Chain([layer(d, i) for i in 0:n-1]...)
    pM, stM = Lux.setup(Random.default_rng(), kan)
    ax = getaxes(ComponentArray(pM))
    p = ComponentArray(vec(Float64.(d["p"])), ax)
    u = Float64.(d["u"])
    y, back = Zygote.pullback((x, q) -> first(kan(x, q, stM)), u, p)
    xbar, pbar = back(Float64.(d["ybar"]))
    Dict("y" => y, "xbar" => xbar, "pbar" => collect(getdata(pbar)))
end

# rc_kanode (Fisher-KPP_Source.jl:55-59,95-98) with the dense periodic Laplacian, batched over columns
function run_fk(d)
    kan1 = Lux.Chain(layer(d, 0))
    pM, stM = Lux.setup(Random.default_rng(), kan1)
    ax = getaxes(ComponentArray(pM))
    Nx, dx, D = Int(d["nx"]), Float64(d["dx"]), Float64(d["D"])
    lap = diagm(0 => -2.0 * ones(Nx), 1 => ones(Nx - 1), -1 => ones(Nx - 1)) ./ dx^2
    lap[1, end] = 1.0 / dx^2
    lap[end, 1] = 1.0 / dx^2
    function rc(u, p)
        kan1_(x) = kan1([x], ComponentArray(p, ax), stM)[1][1]
        reduce(hcat, [D * lap * u[:, b] + kan1_.(u[:, b]) for b in 1:size(u, 2)])
    end
    p = vec(Float64.(d["p"]))
    u = Float64.(d["u"])
    du, back = Zygote.pullback(rc, u, p)
    lamJ, dp = back(Float64.(d["ybar"]))
    Dict("du" => du, "lamJ" => lamJ, "dp" => dp)
end

function main()
    indir, outdir = joinpath(GOLD, "julia_in"), joinpath(GOLD, "julia_out")
    mkpath(outdir)
    for f in sort(readdir(indir))
        endswith(f, ".mat") || continue
        d = matread(joinpath(indir, f))
        res = d["kind"] == "chain" ? run_chain(d) : run_fk(d)
        matwrite(joinpath(outdir, f), res)
        println("wrote ", f)
    end
end

main()
