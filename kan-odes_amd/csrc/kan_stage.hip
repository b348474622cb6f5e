// kan_stage.hip — Runge-Kutta stage plumbing around any RHS (gfx950).
//
// OrdinaryDiffEqTsit5's perform_step! forms each stage input
//     y = uprev + dt·Σ_j a_sj k_j                    (broadcast over the state)
// calls the RHS on it, and after the last stage forms the embedded error
//     utilde = dt·Σ_j btilde_j k_j,   EEst = RMS(utilde / (abstol + reltol·max(|uprev|, |u|)))
// (OrdinaryDiffEq 6.89 calculate_residuals + ODE_DEFAULT_NORM; third-party, restated).
// These generic kernels serve every RHS kind; the Fisher-KPP table path fuses the
// same arithmetic into its streaming kernel instead (kan_pp.hip).
#include "kan_common.hpp"
#include "kan_kernels.hpp"

namespace kan {

// y = u + Σ_{j<nk} c_j k_j, elementwise (fma, ascending j)
template <typename T>
__global__ void __launch_bounds__(kBlock)
stage_lincomb_kernel(const T* __restrict__ u, StageArgs<T> sa, T* __restrict__ y, int64_t n) {
    if (stage_skip(sa.skip)) return;
    const double sc = stage_scale(sa.cscale);
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        T kv[kMaxStages];
        stage_ld<T>(sa, u, i, kv);
        T v = u[i];
#pragma unroll
        for (int j = 0; j < kMaxStages; ++j)
            if (j < sa.nk) v = kfma<T>((T)(sa.c[j] * sc), kv[j], v);
        y[i] = v;
    }
}

// per-block Σ (e/sk)² with e = Σ_j ec_j k_j + ec_nk du, sk = abstol + reltol·max(|u|,|y|)
template <typename T>
__global__ void __launch_bounds__(kBlock)
stage_error_kernel(const T* __restrict__ u, const T* __restrict__ y, const T* __restrict__ du, StageArgs<T> sa,
                   double* __restrict__ slab, int64_t n) {
    __shared__ double red[kBlock / kWave];
    if (stage_skip(sa.skip)) return;
    const double sc = stage_scale(sa.cscale);
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        T kv[kMaxStages];
        stage_ld<T>(sa, u, i, kv);
        double e = 0.0;
#pragma unroll
        for (int j = 0; j < kMaxStages; ++j)
            if (j < sa.nk) e = ::fma(sa.ec[j] * sc, (double)kv[j], e);
        e = ::fma(stage_ec_last(sa) * sc, (double)du[i], e);
        const double sk = ::fma(sa.reltol, fmax(kabs((double)u[i]), kabs((double)y[i])), sa.abstol);
        const double r = e / sk;
        acc = ::fma(r, r, acc);
    }
    const double v[1] = {acc};
    block_sum_to<double, 1>(v, 1, red, slab + blockIdx.x);
}

// out[0] = Σ_b slab[b], fixed order (one block)
__global__ void __launch_bounds__(kBlock) stage_error_final_kernel(const double* __restrict__ slab, int nblk,
                                                                   double* __restrict__ out) {
    __shared__ double red[kBlock / kWave];
    double acc = 0.0;
    for (int b = threadIdx.x; b < nblk; b += kBlock) acc += slab[b];
    const double v[1] = {acc};
    block_sum_to<double, 1>(v, 1, red, out);
}

hipError_t launch_stage_error_final(const double* slab, int nblk, double* out, hipStream_t st) {
    hipLaunchKernelGGL(stage_error_final_kernel, dim3(1), dim3(kBlock), 0, st, slab, nblk, out);
    return hipGetLastError();
}

// The end of an adaptive adjoint step (kanode_solve.cpp adjoint_t, the paths without a fused step
// finish): μ_new = μ + Σ_{j<6} a_j km_j (stage_lincomb_kernel's fma order) and, per block, the partial
// Σ (e/sk)², e = Σ_{j<7} b_j km_j, sk = abstol + reltol·max(|μ|, |μ_new|) (stage_error_kernel's order)
// into slab[block]: the lincomb and the two error launches in one, the host summing the <= 64
// partials in order.
template <typename T>
__global__ void __launch_bounds__(kBlock)
adj_step_finish_kernel(const T* __restrict__ mu, T* __restrict__ mu_new, AdjStepFinish<T> f, double* __restrict__ slab,
                       int64_t n) {
    __shared__ double red[kBlock / kWave];
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        T kv[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) kv[j] = f.km[j][i];
        const T m0 = mu[i];
        T v = m0;
#pragma unroll
        for (int j = 0; j < 6; ++j) v = kfma<T>((T)f.a[j], kv[j], v);
        mu_new[i] = v;
        double e = 0.0;
#pragma unroll
        for (int j = 0; j < 7; ++j) e = ::fma(f.b[j], (double)kv[j], e);
        const double sk = ::fma(f.reltol, fmax(kabs((double)m0), kabs((double)v)), f.abstol);
        const double r = e / sk;
        acc = ::fma(r, r, acc);
    }
    const double w[1] = {acc};
    block_sum_to<double, 1>(w, 1, red, slab + blockIdx.x);
}

template <typename T>
hipError_t launch_adj_step_finish(const T* mu, T* mu_new, const AdjStepFinish<T>& f, double* slab, int64_t n,
                                  int* nblk, hipStream_t st) {
    const int grid = grid_for(n, kBlock, kAdjFinishBlocks);
    *nblk = grid;
    hipLaunchKernelGGL((adj_step_finish_kernel<T>), dim3(grid), dim3(kBlock), 0, st, mu, mu_new, f, slab, n);
    return hipGetLastError();
}
template hipError_t launch_adj_step_finish<double>(const double*, double*, const AdjStepFinish<double>&, double*,
                                                   int64_t, int*, hipStream_t);
template hipError_t launch_adj_step_finish<float>(const float*, float*, const AdjStepFinish<float>&, double*, int64_t,
                                                  int*, hipStream_t);

template <typename T>
hipError_t launch_stage_lincomb(const T* u, const StageArgs<T>& sa, T* y, int64_t n, hipStream_t st) {
    const int grid = grid_for(n, kBlock, kGridCap);
    hipLaunchKernelGGL((stage_lincomb_kernel<T>), dim3(grid), dim3(kBlock), 0, st, u, sa, y, n);
    return hipGetLastError();
}

template <typename T>
__global__ void __launch_bounds__(kBlock) saveat_step_kernel(SaveatStep<T> a, int64_t n) {
    const int j = blockIdx.y;
    T* __restrict__ y = a.dst + (int64_t)j * n;
    const bool copy = (a.exact >> j) & 1ull;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        if (copy) {
            y[i] = a.u_new[i];
            continue;
        }
        T kv[7];
#pragma unroll
        for (int m = 0; m < 7; ++m) kv[m] = (m < a.nk ? a.k[m] : a.u)[i];   // (all loads first)
        T v = a.u[i];
#pragma unroll
        for (int m = 0; m < 7; ++m)
            if (m < a.nk) v = kfma<T>((T)a.w[j][m], kv[m], v);
        y[i] = v;
    }
}

template <typename T>
hipError_t launch_saveat_step(const SaveatStep<T>& a, int64_t n, hipStream_t st) {
    if (a.nsv < 1 || a.nsv > kSaveatPerLaunch || a.nk < 0 || a.nk > 7) return hipErrorInvalidValue;
    const int grid = grid_for(n, kBlock, kGridCap);
    hipLaunchKernelGGL((saveat_step_kernel<T>), dim3(grid, a.nsv), dim3(kBlock), 0, st, a, n);
    return hipGetLastError();
}
template hipError_t launch_saveat_step<double>(const SaveatStep<double>&, int64_t, hipStream_t);
template hipError_t launch_saveat_step<float>(const SaveatStep<float>&, int64_t, hipStream_t);

template <typename T>
hipError_t launch_stage_error(const T* u, const T* y, const T* du, const StageArgs<T>& sa, double* slab,
                              int slab_blocks, double* out, int64_t n, hipStream_t st) {
    const int grid = grid_for(n, kBlock, slab_blocks);
    hipLaunchKernelGGL((stage_error_kernel<T>), dim3(grid), dim3(kBlock), 0, st, u, y, du, sa, slab, n);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_stage_error_final(slab, grid, out, st);
}

template hipError_t launch_stage_lincomb<double>(const double*, const StageArgs<double>&, double*, int64_t,
                                                 hipStream_t);
template hipError_t launch_stage_lincomb<float>(const float*, const StageArgs<float>&, float*, int64_t, hipStream_t);
template hipError_t launch_stage_error<double>(const double*, const double*, const double*, const StageArgs<double>&,
                                               double*, int, double*, int64_t, hipStream_t);
template hipError_t launch_stage_error<float>(const float*, const float*, const float*, const StageArgs<float>&,
                                              double*, int, double*, int64_t, hipStream_t);

}  // namespace kan
