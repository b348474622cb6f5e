// kan_wide.hip — KDense kernels for the full-field surrogate shapes (gfx950).
//
// The surrogate drivers chain KDense(N, 10, G) -> KDense(10, N, G) on a few
// trajectories (PDE examples/Burgers_Surrogate.jl:85-88, Schrodinger_Surrogate.jl:93-96;
// KDense forward kdense.jl:109-130).  With B <= 8 columns the contraction is a
// parameter-streaming GEMV, not a GEMM: VALU + reductions, no MFMA.
//
//   wide-in  (I·G large, O <= 16): one thread per input i computes its basis and
//            its partial y[o] for every column; partials are reduced in the block
//            (fixed order) into a per-block slab, then an ordered slab reduction.
//   wide-out (O large): one thread per output row o; the block stages the (small)
//            basis of its column tile in LDS once; C[o + O*c] reads are coalesced
//            over o (C is column-major [O, G*I]).
// Pullbacks mirror them: wide-out owns its dC/dW rows (no reduction) and emits
// partial basis cotangents per row block; wide-in owns dC/dW of its inputs.
#include "kan_common.hpp"
#include "kan_kernels.hpp"

namespace kan {

constexpr int kKT = 8;        // column tile (trajectories per pass)
constexpr int kOWide = 16;    // max out_dims of a wide-in layer

// basis value/argument/aux for (input value xi, knot g) — direct or recurrence
template <typename T, int PATH>
struct Basis1 {
    T n, z0, F, R, tau, invh;
    __device__ __forceinline__ void init(const Math<T>& M, const LayerConst& lc, T xi) {
        n = normalize<NORM_RUNTIME, T>(M, lc.norm, xi);
        invh = T(lc.invh);
        if constexpr (PATH != PATH_DIRECT) rec_anchor<T>(M, lc, n, z0, F, R, tau);
    }
    __device__ __forceinline__ T next(const Math<T>& M, const LayerConst& lc, int g, T& z, T& aux) {
        if constexpr (PATH == PATH_DIRECT) {
            z = (n - T(lc.grid[g])) * invh;
            aux = T(0);
            return basis_direct<T>(M, lc.basis, z, aux);
        } else {
            T kc = T(lc.K[g]);
            if constexpr (PATH == PATH_REC_CORR) {
                const T e = T(lc.e[g]);
                kc = kc * kfma<T>(tau, kfma<T>(tau, T(0.5) * e * e, e), T(1));
            }
            const T v = F * kc;
            z = z0 - T(lc.Dl[g]);
            aux = T(0);
            F = F * R;
            return v;
        }
    }
};

// ---------------------------------------------------------------------------
// wide-in forward: grid.x = ceil(I/256); slab[(blk*K + k)*O + o] = Σ_{i in blk} (C φ + W sw)
template <typename T, int PATH>
__global__ void __launch_bounds__(kBlock)
kd_fwd_widein_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                     T* __restrict__ slab, int64_t K) {
    __shared__ T red[(kBlock / kWave) * kOWide];
    KAN_EXP_TABLE_LDS(tab);
    const Math<T> M{tab};
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;
    const T* __restrict__ C = p + lc.p_off;
    const T* __restrict__ W = p + lc.w_off;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < I;
    for (int64_t k = 0; k < K; ++k) {
        T acc[kOWide];
#pragma unroll
        for (int o = 0; o < kOWide; ++o) acc[o] = T(0);
        if (valid) {
            const T xi = x[(int64_t)I * k + i];
            Basis1<T, PATH> bs;
            bs.init(M, lc, xi);
            for (int g = 0; g < G; ++g) {
                T z, aux;
                const T phi = bs.next(M, lc, g, z, aux);
                const T* Cc = C + (int64_t)O * (g + (int64_t)G * i);
#pragma unroll
                for (int o = 0; o < kOWide; ++o)
                    if (o < O) acc[o] = kfma<T>(Cc[o], phi, acc[o]);
            }
            if (lc.use_base) {
                const T sw = swish<T>(M, xi);
                const T* Wi = W + (int64_t)O * i;
#pragma unroll
                for (int o = 0; o < kOWide; ++o)
                    if (o < O) acc[o] = kfma<T>(Wi[o], sw, acc[o]);
            }
        }
        block_sum_to<T, kOWide>(acc, O, red, slab + ((int64_t)blockIdx.x * K + k) * O);
    }
}

// y[o + O*k] = Σ_b slab[(b*K + k)*O + o]   (ordered over b)
template <typename T>
__global__ void __launch_bounds__(kBlock)
kd_widein_reduce_kernel(const T* __restrict__ slab, int nblk, int O, int64_t K, T* __restrict__ y) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)O * K) return;
    const int64_t k = idx / O;
    const int o = (int)(idx - k * O);
    T s = T(0);
    for (int b = 0; b < nblk; ++b) s += slab[((int64_t)b * K + k) * O + o];
    y[(int64_t)O * k + o] = s;
}

// ---------------------------------------------------------------------------
// wide-out forward: grid.x = ceil(O/256); each block stages the basis of a column
// tile (GI x KT values + I x KT swish values) in LDS, then thread o contracts.
template <typename T, int PATH>
__global__ void __launch_bounds__(kBlock)
kd_fwd_wideout_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                      T* __restrict__ y, int64_t K) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    KAN_EXP_TABLE_LDS(tab);
    const Math<T> M{tab};
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;
    const int GI = G * I;
    T* phiL = reinterpret_cast<T*>(smem_raw);       // [GI][kKT]
    T* swL = phiL + (int64_t)GI * kKT;              // [I][kKT]
    const T* __restrict__ C = p + lc.p_off;
    const T* __restrict__ W = p + lc.w_off;
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t k0 = 0; k0 < K; k0 += kKT) {
        const int kt = (int)((K - k0) < kKT ? (K - k0) : kKT);
        __syncthreads();
        for (int t = threadIdx.x; t < I * kKT; t += blockDim.x) {
            const int i = t / kKT, kk = t - i * kKT;
            if (kk < kt) {
                const T xi = x[(int64_t)I * (k0 + kk) + i];
                Basis1<T, PATH> bs;
                bs.init(M, lc, xi);
                for (int g = 0; g < G; ++g) {
                    T z, aux;
                    phiL[(g + G * i) * kKT + kk] = bs.next(M, lc, g, z, aux);
                }
                swL[i * kKT + kk] = lc.use_base ? swish<T>(M, xi) : T(0);
            } else {
                for (int g = 0; g < G; ++g) phiL[(g + G * i) * kKT + kk] = T(0);
                swL[i * kKT + kk] = T(0);
            }
        }
        __syncthreads();
        if (o < O) {
            T acc[kKT], bas[kKT];
#pragma unroll
            for (int kk = 0; kk < kKT; ++kk) { acc[kk] = T(0); bas[kk] = T(0); }
            for (int c = 0; c < GI; ++c) {
                const T cv = C[o + (int64_t)O * c];
#pragma unroll
                for (int kk = 0; kk < kKT; ++kk) acc[kk] = kfma<T>(cv, phiL[c * kKT + kk], acc[kk]);
            }
            if (lc.use_base)
                for (int i = 0; i < I; ++i) {
                    const T wv = W[o + (int64_t)O * i];
#pragma unroll
                    for (int kk = 0; kk < kKT; ++kk) bas[kk] = kfma<T>(wv, swL[i * kKT + kk], bas[kk]);
                }
#pragma unroll
            for (int kk = 0; kk < kKT; ++kk)
                if (kk < kt) y[(int64_t)O * (k0 + kk) + o] = lc.use_base ? acc[kk] + bas[kk] : acc[kk];
        }
    }
}

// ---------------------------------------------------------------------------
// wide-out pullback, pass 1: thread o owns dC[o, :], dW[o, :] (accumulated into
// pbar); the block's partial cotangents of the basis (Σ_o C[o,c] ȳ[o,k]) and of
// the base branch (Σ_o W[o,i] ȳ[o,k]) go to slab[(blk*K + k)*(GI+I) + c].
template <typename T, int PATH>
__global__ void __launch_bounds__(kBlock)
kd_vjp_wideout_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                      const T* __restrict__ ybar, T* __restrict__ pbar, T* __restrict__ slab, int64_t K) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    KAN_EXP_TABLE_LDS(tab);
    const Math<T> M{tab};
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;
    const int GI = G * I;
    const int R = GI + I;                            // cotangent rows per column
    T* phiL = reinterpret_cast<T*>(smem_raw);       // [GI][kKT]
    T* swL = phiL + (int64_t)GI * kKT;              // [I][kKT]
    T* redw = swL + (int64_t)I * kKT;               // [wave][R][kKT] wave partials
    const T* __restrict__ C = p + lc.p_off;
    const T* __restrict__ W = p + lc.w_off;
    T* __restrict__ dC = pbar ? pbar + lc.p_off : nullptr;
    T* __restrict__ dW = pbar ? pbar + lc.w_off : nullptr;
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = o < O;
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave, nw = blockDim.x / kWave;
    for (int64_t k0 = 0; k0 < K; k0 += kKT) {
        const int kt = (int)((K - k0) < kKT ? (K - k0) : kKT);
        __syncthreads();
        for (int t = threadIdx.x; t < I * kKT; t += blockDim.x) {
            const int i = t / kKT, kk = t - i * kKT;
            const bool on = kk < kt;
            const T xi = on ? x[(int64_t)I * (k0 + kk) + i] : T(0);
            Basis1<T, PATH> bs;
            bs.init(M, lc, xi);
            for (int g = 0; g < G; ++g) {
                T z, aux;
                const T v = bs.next(M, lc, g, z, aux);
                phiL[(g + G * i) * kKT + kk] = on ? v : T(0);
            }
            swL[i * kKT + kk] = (on && lc.use_base) ? swish<T>(M, xi) : T(0);
        }
        __syncthreads();
        T yb[kKT];
#pragma unroll
        for (int kk = 0; kk < kKT; ++kk) yb[kk] = (valid && kk < kt) ? ybar[(int64_t)O * (k0 + kk) + o] : T(0);
        for (int c = 0; c < R; ++c) {
            const bool isC = c < GI;
            const T coef = valid ? (isC ? C[o + (int64_t)O * c] : (lc.use_base ? W[o + (int64_t)O * (c - GI)] : T(0)))
                                 : T(0);
            const T* row = isC ? phiL + c * kKT : swL + (c - GI) * kKT;
            // owned parameter gradient: Σ_k ȳ[o,k] basis[c,k]
            T g = T(0);
#pragma unroll
            for (int kk = 0; kk < kKT; ++kk) g = kfma<T>(yb[kk], row[kk], g);
            if (valid && pbar && (isC || lc.use_base)) {
                if (isC) dC[o + (int64_t)O * c] += g;
                else dW[o + (int64_t)O * (c - GI)] += g;
            }
            // partial cotangent of basis row c for every column of the tile (wave sums)
#pragma unroll
            for (int kk = 0; kk < kKT; ++kk) {
                const T s = wave_sum(coef * yb[kk]);
                if (lane == 0) redw[((int64_t)wid * R + c) * kKT + kk] = s;
            }
        }
        __syncthreads();
        // block partial = Σ over waves in wave order -> slab
        for (int t = threadIdx.x; t < R * kt; t += blockDim.x) {
            const int c = t / kt, kk = t - c * kt;
            T s = redw[(int64_t)c * kKT + kk];
            for (int w = 1; w < nw; ++w) s += redw[((int64_t)w * R + c) * kKT + kk];
            slab[((int64_t)blockIdx.x * K + (k0 + kk)) * R + c] = s;
        }
    }
}

// wide-out pullback, pass 2: x̄[i,k] from the summed basis cotangents
// (rrule(_rbf) + normalizer + swish rrules; utils.jl:15-21, NNlib).
template <typename T, int PATH>
__global__ void __launch_bounds__(kBlock)
kd_vjp_wideout_finalize_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ x,
                               const T* __restrict__ slab, int nblk, T* __restrict__ xbar, int64_t K) {
    KAN_EXP_TABLE_LDS(tab);
    const Math<T> M{tab};
    const LayerConst& lc = *lcp;
    const int I = lc.I, G = lc.G;
    const int GI = G * I, R = GI + I;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)I * K) return;
    const int64_t k = idx / I;
    const int i = (int)(idx - k * I);
    const T xi = x[(int64_t)I * k + i];
    Basis1<T, PATH> bs;
    bs.init(M, lc, xi);
    const T invh = T(lc.invh);
    T nbar = T(0);
    for (int g = 0; g < G; ++g) {
        T z, aux;
        const T phi = bs.next(M, lc, g, z, aux);
        T bb = T(0);
        for (int b = 0; b < nblk; ++b) bb += slab[((int64_t)b * K + k) * R + g + G * i];
        nbar = nbar + basis_pull<T>(lc.basis, lc.iqf_quirk, z, phi, aux, bb) * invh;
    }
    T xb = nbar * dnormalize<NORM_RUNTIME, T>(lc.norm, bs.n);
    if (lc.use_base) {
        T sb = T(0);
        for (int b = 0; b < nblk; ++b) sb += slab[((int64_t)b * K + k) * R + GI + i];
        T sw, dsw;
        swish_and_grad<T>(M, xi, sw, dsw);
        xb = xb + sb * dsw;
    }
    xbar[(int64_t)I * k + i] = xb;
}

// ---------------------------------------------------------------------------
// wide-in pullback: thread i owns dC[:, g+G i], dW[:, i] and x̄[i, :].
template <typename T, int PATH>
__global__ void __launch_bounds__(kBlock)
kd_vjp_widein_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                     const T* __restrict__ ybar, T* __restrict__ xbar, T* __restrict__ pbar, int64_t K) {
    KAN_EXP_TABLE_LDS(tab);
    const Math<T> M{tab};
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;
    const T* __restrict__ C = p + lc.p_off;
    const T* __restrict__ W = p + lc.w_off;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= I) return;
    const T invh = T(lc.invh);
    T dWacc[kOWide];
#pragma unroll
    for (int o = 0; o < kOWide; ++o) dWacc[o] = T(0);
    for (int64_t k = 0; k < K; ++k) {
        T yb[kOWide];
#pragma unroll
        for (int o = 0; o < kOWide; ++o) yb[o] = o < O ? ybar[(int64_t)O * k + o] : T(0);
        const T xi = x[(int64_t)I * k + i];
        Basis1<T, PATH> bs;
        bs.init(M, lc, xi);
        T nbar = T(0);
        for (int g = 0; g < G; ++g) {
            T z, aux;
            const T phi = bs.next(M, lc, g, z, aux);
            const int64_t col = (int64_t)O * (g + (int64_t)G * i);
            T bb = T(0);
#pragma unroll
            for (int o = 0; o < kOWide; ++o)
                if (o < O) bb = kfma<T>(C[col + o], yb[o], bb);
            nbar = nbar + basis_pull<T>(lc.basis, lc.iqf_quirk, z, phi, aux, bb) * invh;
            if (pbar) {
#pragma unroll
                for (int o = 0; o < kOWide; ++o)
                    if (o < O) pbar[lc.p_off + col + o] += yb[o] * phi;
            }
        }
        T xb = nbar * dnormalize<NORM_RUNTIME, T>(lc.norm, bs.n);
        if (lc.use_base) {
            T sw, dsw;
            swish_and_grad<T>(M, xi, sw, dsw);
            T sb = T(0);
#pragma unroll
            for (int o = 0; o < kOWide; ++o)
                if (o < O) {
                    sb = kfma<T>(W[(int64_t)O * i + o], yb[o], sb);
                    dWacc[o] = kfma<T>(yb[o], sw, dWacc[o]);
                }
            xb = xb + sb * dsw;
        }
        xbar[(int64_t)I * k + i] = xb;
    }
    if (pbar && lc.use_base) {
#pragma unroll
        for (int o = 0; o < kOWide; ++o)
            if (o < O) pbar[lc.w_off + (int64_t)O * i + o] += dWacc[o];
    }
}

// ---------------------------------------------------------------------------
// launchers
static inline size_t wideout_lds(const LayerConst& h, size_t es) { return es * (size_t)(h.G * h.I + h.I) * kKT; }

template <typename T>
hipError_t launch_kd_fwd_widein(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, T* y, T* slab,
                                int64_t K, hipStream_t st) {
    const int nblk = (h.I + kBlock - 1) / kBlock;
    switch (h.path) {
    case PATH_REC_CORR:
        hipLaunchKernelGGL((kd_fwd_widein_kernel<T, PATH_REC_CORR>), dim3(nblk), dim3(kBlock), 0, st, lc, p, x, slab, K);
        break;
    case PATH_REC:
        hipLaunchKernelGGL((kd_fwd_widein_kernel<T, PATH_REC>), dim3(nblk), dim3(kBlock), 0, st, lc, p, x, slab, K);
        break;
    default:
        hipLaunchKernelGGL((kd_fwd_widein_kernel<T, PATH_DIRECT>), dim3(nblk), dim3(kBlock), 0, st, lc, p, x, slab, K);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t n = (int64_t)h.O * K;
    hipLaunchKernelGGL((kd_widein_reduce_kernel<T>), dim3(grid_for(n, kBlock, 1 << 30)), dim3(kBlock), 0, st, slab,
                       nblk, h.O, K, y);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_kd_fwd_wideout(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, T* y, int64_t K,
                                 hipStream_t st) {
    const int nblk = (h.O + kBlock - 1) / kBlock;
    const size_t lds = wideout_lds(h, sizeof(T));
    switch (h.path) {
    case PATH_REC_CORR:
        hipLaunchKernelGGL((kd_fwd_wideout_kernel<T, PATH_REC_CORR>), dim3(nblk), dim3(kBlock), lds, st, lc, p, x, y, K);
        break;
    case PATH_REC:
        hipLaunchKernelGGL((kd_fwd_wideout_kernel<T, PATH_REC>), dim3(nblk), dim3(kBlock), lds, st, lc, p, x, y, K);
        break;
    default:
        hipLaunchKernelGGL((kd_fwd_wideout_kernel<T, PATH_DIRECT>), dim3(nblk), dim3(kBlock), lds, st, lc, p, x, y, K);
    }
    return hipGetLastError();
}

template <typename T>
hipError_t launch_kd_vjp_wideout(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, const T* yb,
                                 T* xb, T* pbar, T* slab, int64_t K, hipStream_t st) {
    const int nblk = (h.O + kBlock - 1) / kBlock;
    const size_t lds = wideout_lds(h, sizeof(T)) + sizeof(T) * (size_t)(kBlock / kWave) * (h.G * h.I + h.I) * kKT;
    const int64_t nfin = (int64_t)h.I * K;
    switch (h.path) {
    case PATH_REC_CORR:
        hipLaunchKernelGGL((kd_vjp_wideout_kernel<T, PATH_REC_CORR>), dim3(nblk), dim3(kBlock), lds, st, lc, p, x, yb,
                           pbar, slab, K);
        hipLaunchKernelGGL((kd_vjp_wideout_finalize_kernel<T, PATH_REC_CORR>), dim3(grid_for(nfin, kBlock, 1 << 30)),
                           dim3(kBlock), 0, st, lc, x, slab, nblk, xb, K);
        break;
    case PATH_REC:
        hipLaunchKernelGGL((kd_vjp_wideout_kernel<T, PATH_REC>), dim3(nblk), dim3(kBlock), lds, st, lc, p, x, yb, pbar,
                           slab, K);
        hipLaunchKernelGGL((kd_vjp_wideout_finalize_kernel<T, PATH_REC>), dim3(grid_for(nfin, kBlock, 1 << 30)),
                           dim3(kBlock), 0, st, lc, x, slab, nblk, xb, K);
        break;
    default:
        hipLaunchKernelGGL((kd_vjp_wideout_kernel<T, PATH_DIRECT>), dim3(nblk), dim3(kBlock), lds, st, lc, p, x, yb,
                           pbar, slab, K);
        hipLaunchKernelGGL((kd_vjp_wideout_finalize_kernel<T, PATH_DIRECT>), dim3(grid_for(nfin, kBlock, 1 << 30)),
                           dim3(kBlock), 0, st, lc, x, slab, nblk, xb, K);
    }
    return hipGetLastError();
}

template <typename T>
hipError_t launch_kd_vjp_widein(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, const T* yb, T* xb,
                                T* pbar, int64_t K, hipStream_t st) {
    const int nblk = (h.I + kBlock - 1) / kBlock;
    switch (h.path) {
    case PATH_REC_CORR:
        hipLaunchKernelGGL((kd_vjp_widein_kernel<T, PATH_REC_CORR>), dim3(nblk), dim3(kBlock), 0, st, lc, p, x, yb, xb,
                           pbar, K);
        break;
    case PATH_REC:
        hipLaunchKernelGGL((kd_vjp_widein_kernel<T, PATH_REC>), dim3(nblk), dim3(kBlock), 0, st, lc, p, x, yb, xb, pbar, K);
        break;
    default:
        hipLaunchKernelGGL((kd_vjp_widein_kernel<T, PATH_DIRECT>), dim3(nblk), dim3(kBlock), 0, st, lc, p, x, yb, xb,
                           pbar, K);
    }
    return hipGetLastError();
}

#define KAN_WIDE_INST(T)                                                                                       \
    template hipError_t launch_kd_fwd_widein<T>(const LayerConst&, const LayerConst*, const T*, const T*, T*, T*, \
                                                int64_t, hipStream_t);                                          \
    template hipError_t launch_kd_fwd_wideout<T>(const LayerConst&, const LayerConst*, const T*, const T*, T*,   \
                                                 int64_t, hipStream_t);                                         \
    template hipError_t launch_kd_vjp_wideout<T>(const LayerConst&, const LayerConst*, const T*, const T*,       \
                                                 const T*, T*, T*, T*, int64_t, hipStream_t);                   \
    template hipError_t launch_kd_vjp_widein<T>(const LayerConst&, const LayerConst*, const T*, const T*,        \
                                                const T*, T*, T*, int64_t, hipStream_t);
KAN_WIDE_INST(double)
KAN_WIDE_INST(float)
#undef KAN_WIDE_INST

}  // namespace kan
