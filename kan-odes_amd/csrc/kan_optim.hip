// kan_optim.hip — the optimiser step that follows the gradient all-reduce (gfx950).
//
// Flux 0.14 legacy Optimise.Adam + update!(opt, x, Δ) (LV_driver_KANODE.jl:219,287;
// Fisher-KPP_Source.jl:167,201; Flux pinned at Lotka-Volterra/Manifest.toml, third-party, restated):
//     mt = β1·mt + (1 - β1)·Δ
//     vt = β2·vt + (1 - β2)·Δ²
//     Δ  = mt / (1 - βp1) / (√(vt / (1 - βp2)) + ϵ) · η ;   x .-= Δ ;   βp .*= β
// Flux evaluates these broadcasts with its Float64 hyper-parameters, so a Float32 x, mt, vt is
// promoted, computed in Float64 and rounded on store: the same here.  apply! stores the step into the
// gradient array Δ (`@. Δ = … * η`, Float32 with Float32 parameters) and update! subtracts that array
// (`x .-= Δ`, a Float32 broadcast), so the step is rounded to T before a subtraction in T.  Δ arrives as the SUM
// all-reduce of the ranks' gradients; `scale` (1/world_size) forms their mean in the same pass,
// so the whole post-collective update is ONE launch instead of the ~8 elementwise torch kernels of
// kanode.Adam (kanode/train.py).  The operation order is kanode.Adam's (torch's add_(alpha) and
// addcmul_(value): β·m + (1-β)·Δ, β·v + ((1-β)·Δ)·Δ), every product and sum rounded separately.
#include "kan_common.hpp"
#include "kan_kernels.hpp"

namespace kan {

template <typename T>
__global__ void __launch_bounds__(kBlock)
adam_step_kernel(T* __restrict__ x, T* __restrict__ m, T* __restrict__ v, const T* __restrict__ g, int64_t n,
                 AdamArgs a) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const double d = __dmul_rn((double)g[i], a.scale);
        const double mt = __dadd_rn(__dmul_rn(a.beta1, (double)m[i]), __dmul_rn(a.omb1, d));
        const double vt = __dadd_rn(__dmul_rn(a.beta2, (double)v[i]), __dmul_rn(__dmul_rn(a.omb2, d), d));
        const T ms = (T)mt, vs = (T)vt;          // the stored moments (rounded for T = float)
        m[i] = ms;
        v[i] = vs;
        const double den = __dadd_rn(::sqrt(__ddiv_rn((double)vs, a.c2)), a.eps);
        const double step = __dmul_rn(__ddiv_rn(__ddiv_rn((double)ms, a.c1), den), a.eta);
        if constexpr (std::is_same<T, double>::value) x[i] = __dsub_rn(x[i], step);
        else x[i] = __fsub_rn(x[i], (float)step);
    }
}

template <typename T>
hipError_t launch_adam_step(T* x, T* m, T* v, const T* g, int64_t n, const AdamArgs& a, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int grid = grid_for(n, kBlock, kGridCap);
    hipLaunchKernelGGL((adam_step_kernel<T>), dim3(grid), dim3(kBlock), 0, st, x, m, v, g, n, a);
    return hipGetLastError();
}

template hipError_t launch_adam_step<double>(double*, double*, double*, const double*, int64_t, const AdamArgs&,
                                             hipStream_t);
template hipError_t launch_adam_step<float>(float*, float*, float*, const float*, int64_t, const AdamArgs&,
                                            hipStream_t);

}  // namespace kan
