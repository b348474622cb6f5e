// kan_kernels.hip — hand-written HIP kernels (gfx950 / CDNA4) for the KAN-ODE
// right-hand side and its VJP.  No hipify, no CUDA shims; wave64 throughout.
//
// Reference semantics (file:line relative to /root/reference):
//   KDense forward            Lotka-Volterra/src/kdense.jl:109-130
//   KDense pullback           Zygote over kdense.jl:109-130 + rrules utils.jl:15-62
//   Fisher-KPP rc_kanode      PDE examples/Fisher-KPP_Source.jl:55-59,95-98
//   per-edge activations      Lotka-Volterra/Activation_getter.jl:20-54
//
// Memory layout: the reference's Julia column-major arrays, unchanged —
//   state u [N, B] (trajectory contiguous), KDense input x [I, K], C [O, G*I], W [O, I].
// Parameter gradients are reduced deterministically: per-block partial slabs
// (fixed in-block order) + an ordered slab-reduction kernel (no float atomics).
#include "kan_device.hpp"
#include "kan_kernels.hpp"

#include <type_traits>

namespace kan {

constexpr int kBlock = 256;
constexpr int kWave = 64;

// ---------------------------------------------------------------------------
// reductions
template <typename T> __device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

// Sum `n` per-thread values across the block into out[0..n) (thread-0 order
// fixed: wave partials summed in wave order).  `red` is LDS scratch of at
// least (blockDim/64) * n elements.
template <typename T, int N>
__device__ __forceinline__ void block_sum_to(const T (&v)[N], int n, T* red, T* out) {
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    const int nw = blockDim.x / kWave;
#pragma unroll
    for (int q = 0; q < N; ++q) {
        if (q < n) {
            const T s = wave_sum(v[q]);
            if (lane == 0) red[wid * n + q] = s;
        }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < n; q += blockDim.x) {
        T s = red[q];
        for (int w = 1; w < nw; ++w) s += red[w * n + q];
        out[q] = s;
    }
    __syncthreads();
}

// dp[off + q] += sum_b slab[b*P + q]  — one block per parameter, fixed order.
template <typename T>
__global__ void __launch_bounds__(kBlock) slab_reduce_kernel(const T* __restrict__ slab, int64_t nblk,
                                                             int64_t P, T* __restrict__ dp) {
    __shared__ T red[kBlock / kWave];
    const int64_t q = blockIdx.x;
    T s = T(0);
    for (int64_t b = threadIdx.x; b < nblk; b += blockDim.x) s += slab[b * P + q];
    s = wave_sum(s);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        T t = red[0];
        for (int w = 1; w < (int)(blockDim.x / kWave); ++w) t += red[w];
        dp[q] += t;
    }
}

// ---------------------------------------------------------------------------
// Fisher-KPP: pointwise KDense(1,1,G) + periodic 3-point Laplacian.
//
// (D*lap)*u row i with the reference matrix's nonzeros in ascending column order
// and no FMA contraction (the dense gemv adds exact zeros elsewhere).
template <typename T>
__device__ __forceinline__ T lap_row(T um, T u0, T up, T ufirst, T ulast, int i, int Nx, T cd, T co) {
#pragma clang fp contract(off)
    if (Nx >= 3) {
        if (i == 0) { T s = cd * u0; s = s + co * up; s = s + co * ulast; return s; }
        if (i == Nx - 1) { T s = co * ufirst; s = s + co * um; s = s + cd * u0; return s; }
        T s = co * um; s = s + cd * u0; s = s + co * up; return s;
    }
    if (Nx == 2) {
        if (i == 0) { T s = cd * u0; s = s + co * up; return s; }
        T s = co * um; s = s + cd * u0; return s;
    }
    return co * u0;  // Nx == 1: lap[1,end] overwrote the diagonal
}

// Per-thread coefficient registers for the [1,1] KDense (GL = compile-time bound).
template <typename T, int GL>
struct FK11 {
    T A[GL], Bq[GL], Q[GL];   // Horner sets: C_j K_j, C_j K_j e_j, C_j K_j e_j²/2
    T C[GL], K[GL], E[GL], Dl[GL];
    T W;
};

template <typename T, int PATH, int GT>
__device__ __forceinline__ void fk_load_coef(const LayerConst& lc, const T* __restrict__ p, FK11<T, GT ? GT : kMaxGrid>& cf) {
    constexpr int GL = GT ? GT : kMaxGrid;
    const int G = lc.G;
#pragma unroll
    for (int j = 0; j < GL; ++j) {
        const bool on = GT ? true : (j < G);
        const T c = on ? p[j] : T(0);
        const T k = on ? T(lc.K[j]) : T(0);
        const T e = on ? T(lc.e[j]) : T(0);
        cf.C[j] = c;
        cf.K[j] = k;
        cf.E[j] = e;
        cf.Dl[j] = on ? T(lc.Dl[j]) : T(0);
        cf.A[j] = c * k;
        cf.Bq[j] = c * k * e;
        cf.Q[j] = c * k * (T(0.5) * e * e);
    }
    cf.W = lc.use_base ? p[G] : T(0);
}

// KDense(1,1,G)(x) — the reference's per-point `kan1([x], p, st)[1][1]` (:96).
template <typename T, int PATH, int GT>
__device__ __forceinline__ T kan11_fwd(const LayerConst& lc, const FK11<T, GT ? GT : kMaxGrid>& cf, T x) {
    constexpr int GL = GT ? GT : kMaxGrid;
    const int G = GT ? GT : lc.G;
    const T n = normalize<T>(lc.norm, x);
    T spline;
    if constexpr (PATH == PATH_DIRECT) {
        const T invh = T(lc.invh);
        T s = T(0);
#pragma unroll
        for (int j = 0; j < GL; ++j) {
            if (GT || j < G) {
                T aux;
                const T y = (n - T(lc.grid[j])) * invh;
                s = s + cf.C[j] * basis_direct<T>(lc.basis, y, aux);
            }
        }
        spline = s;
    } else {
        T z0, E0, R;
        rec_anchor<T>(lc, n, z0, E0, R);
        // Horner in R over j = G-1 .. 0
        T s0 = T(0), s1 = T(0), s2 = T(0);
#pragma unroll
        for (int j = GL - 1; j >= 0; --j) {
            if (GT || j < G) {
                s0 = kfma<T>(s0, R, cf.A[j]);
                if constexpr (PATH == PATH_REC_CORR) {
                    s1 = kfma<T>(s1, R, cf.Bq[j]);
                    s2 = kfma<T>(s2, R, cf.Q[j]);
                }
            }
        }
        if constexpr (PATH == PATH_REC_CORR) {
            const T tau = z0 + z0;
            spline = E0 * kfma<T>(tau, kfma<T>(tau, s2, s1), s0);
        } else {
            spline = E0 * s0;
        }
    }
    if (lc.use_base) spline = spline + cf.W * swish<T>(x);
    return spline;
}

// One point of the VJP: returns x̄ and accumulates dC_j += λ φ_j, dW += λ swish(x).
template <typename T, int PATH, int GT>
__device__ __forceinline__ T kan11_vjp(const LayerConst& lc, const FK11<T, GT ? GT : kMaxGrid>& cf, T x, T lam,
                                       T (&dC)[GT ? GT : kMaxGrid], T& dW) {
    constexpr int GL = GT ? GT : kMaxGrid;
    const int G = GT ? GT : lc.G;
    const T n = normalize<T>(lc.norm, x);
    const T invh = T(lc.invh);
    T nbar = T(0);
    if constexpr (PATH == PATH_DIRECT) {
#pragma unroll
        for (int j = 0; j < GL; ++j) {
            if (GT || j < G) {
                T aux = T(0);
                const T y = (n - T(lc.grid[j])) * invh;
                const T phi = basis_direct<T>(lc.basis, y, aux);
                const T zb = basis_pull<T>(lc.basis, lc.iqf_quirk, y, phi, aux, cf.C[j] * lam);
                nbar = nbar + zb * invh;
                dC[j] = kfma<T>(lam, phi, dC[j]);
            }
        }
    } else {
        T z0, F, R;
        rec_anchor<T>(lc, n, z0, F, R);
        const T tau = z0 + z0;
#pragma unroll
        for (int j = 0; j < GL; ++j) {
            if (GT || j < G) {
                T phi = F * cf.K[j];
                if constexpr (PATH == PATH_REC_CORR) {
                    const T e = cf.E[j];
                    phi = phi * kfma<T>(tau, kfma<T>(tau, T(0.5) * e * e, e), T(1));
                }
                const T y = z0 - cf.Dl[j];
                const T zb = T(-2) * y * phi * (cf.C[j] * lam);
                nbar = nbar + zb * invh;
                dC[j] = kfma<T>(lam, phi, dC[j]);
                F = F * R;
            }
        }
    }
    T xb = nbar * dnormalize<T>(lc.norm, n);
    if (lc.use_base) {
        T sw, dsw;
        swish_and_grad<T>(x, sw, dsw);
        xb = xb + (cf.W * lam) * dsw;
        dW = kfma<T>(lam, sw, dW);
    }
    return xb;
}

template <typename T, int PATH, int GT>
__global__ void __launch_bounds__(kBlock)
fk_rhs_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, T cd, T co, int32_t Nx,
              const T* __restrict__ u, T* __restrict__ du, int64_t npts) {
    const LayerConst& lc = *lcp;
    FK11<T, GT ? GT : kMaxGrid> cf;
    fk_load_coef<T, PATH, GT>(lc, p, cf);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < npts; idx += stride) {
        const int i = (int)(idx % Nx);
        const int64_t base = idx - i;
        const T u0 = u[idx];
        const T um = (i > 0) ? u[idx - 1] : u[base + Nx - 1];
        const T up = (i < Nx - 1) ? u[idx + 1] : u[base];
        const T lu = lap_row<T>(um, u0, up, u[base], u[base + Nx - 1], i, Nx, cd, co);
        du[idx] = lu + kan11_fwd<T, PATH, GT>(lc, cf, u0);
    }
}

// Nx even: each thread owns an aligned point pair (16-B loads/stores for f64).
template <typename T, int PATH, int GT>
__global__ void __launch_bounds__(kBlock)
fk_rhs_pair_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, T cd, T co, int32_t Nx,
                   const T* __restrict__ u, T* __restrict__ du, int64_t npairs) {
    using V2 = typename std::conditional<sizeof(T) == 8, double2, float2>::type;
    const LayerConst& lc = *lcp;
    FK11<T, GT ? GT : kMaxGrid> cf;
    fk_load_coef<T, PATH, GT>(lc, p, cf);
    const int half = Nx >> 1;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < npairs; q += stride) {
        const int ip = (int)(q % half);
        const int i = ip * 2;
        const int64_t idx = q * 2;
        const int64_t base = idx - i;
        const V2 v = *reinterpret_cast<const V2*>(u + idx);
        const T um = (i > 0) ? u[idx - 1] : u[base + Nx - 1];
        const T up = (i + 2 < Nx) ? u[idx + 2] : u[base];
        const T ufirst = (i == 0) ? v.x : u[base];
        const T ulast = (i + 2 == Nx) ? v.y : u[base + Nx - 1];
        V2 o;
        o.x = lap_row<T>(um, v.x, v.y, ufirst, ulast, i, Nx, cd, co) + kan11_fwd<T, PATH, GT>(lc, cf, v.x);
        o.y = lap_row<T>(v.x, v.y, up, ufirst, ulast, i + 1, Nx, cd, co) + kan11_fwd<T, PATH, GT>(lc, cf, v.y);
        *reinterpret_cast<V2*>(du + idx) = o;
    }
}

template <typename T, int PATH, int GT>
__global__ void __launch_bounds__(kBlock)
fk_vjp_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, T cd, T co, int32_t Nx,
              const T* __restrict__ u, const T* __restrict__ lam, T* __restrict__ lamJ,
              T* __restrict__ slab, int64_t npts) {
    constexpr int GL = GT ? GT : kMaxGrid;
    __shared__ T red[(kBlock / kWave) * (GL + 1)];
    const LayerConst& lc = *lcp;
    FK11<T, GL> cf;
    fk_load_coef<T, PATH, GT>(lc, p, cf);
    T acc[GL + 1];
#pragma unroll
    for (int j = 0; j <= GL; ++j) acc[j] = T(0);
    T dC[GL];
#pragma unroll
    for (int j = 0; j < GL; ++j) dC[j] = T(0);
    T dW = T(0);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < npts; idx += stride) {
        const int i = (int)(idx % Nx);
        const int64_t base = idx - i;
        const T l0 = lam[idx];
        const T lm = (i > 0) ? lam[idx - 1] : lam[base + Nx - 1];
        const T lp = (i < Nx - 1) ? lam[idx + 1] : lam[base];
        // (D*lap)ᵀ λ — lap is symmetric: same row formula on λ
        const T lt = lap_row<T>(lm, l0, lp, lam[base], lam[base + Nx - 1], i, Nx, cd, co);
        lamJ[idx] = lt + kan11_vjp<T, PATH, GT>(lc, cf, u[idx], l0, dC, dW);
    }
    const int G = GT ? GT : lc.G;
    const int P = G + (lc.use_base ? 1 : 0);
#pragma unroll
    for (int j = 0; j < GL; ++j) acc[j] = dC[j];
    // pack (C_0..C_{G-1}, W) contiguously
    acc[GL] = T(0);
    if (!GT) {
#pragma unroll
        for (int j = 0; j <= GL; ++j) if (j == G) acc[j] = dW;
    } else {
        acc[GL] = dW;
    }
    block_sum_to<T, GL + 1>(acc, P, red, slab + (int64_t)blockIdx.x * P);
}

// ---------------------------------------------------------------------------
// Generic KDense, "column" kernels: one thread per column k of x [I, K];
// O <= OMAX accumulators in registers; C/W reads are wave-uniform (scalar path).
template <typename T, int PATH>
struct BasisStream {
    T n, F, R, z0, tau, invh;
    __device__ __forceinline__ void init(const LayerConst& lc, T nn) {
        n = nn;
        invh = T(lc.invh);
        if constexpr (PATH != PATH_DIRECT) {
            rec_anchor<T>(lc, n, z0, F, R);
            tau = z0 + z0;
        }
    }
    // returns φ_g, z_g (the scaled argument), aux (tanh for rswaf)
    __device__ __forceinline__ T next(const LayerConst& lc, int g, T& z, T& aux) {
        if constexpr (PATH == PATH_DIRECT) {
            z = (n - T(lc.grid[g])) * invh;
            aux = T(0);
            return basis_direct<T>(lc.basis, z, aux);
        } else {
            T v = F * T(lc.K[g]);
            if constexpr (PATH == PATH_REC_CORR) {
                const T e = T(lc.e[g]);
                v = v * kfma<T>(tau, kfma<T>(tau, T(0.5) * e * e, e), T(1));
            }
            z = z0 - T(lc.Dl[g]);
            aux = T(0);
            F = F * R;
            return v;
        }
    }
};

template <typename T, int PATH, int OMAX>
__global__ void __launch_bounds__(kBlock)
kd_fwd_col_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                  T* __restrict__ y, int64_t K) {
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;
    const T* __restrict__ C = p + lc.p_off;
    const T* __restrict__ W = p + lc.w_off;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < K; k += stride) {
        T acc[OMAX], bas[OMAX];
#pragma unroll
        for (int o = 0; o < OMAX; ++o) { acc[o] = T(0); bas[o] = T(0); }
        for (int i = 0; i < I; ++i) {
            const T xi = x[(int64_t)I * k + i];
            BasisStream<T, PATH> bs;
            bs.init(lc, normalize<T>(lc.norm, xi));
            for (int g = 0; g < G; ++g) {
                T z, aux;
                const T phi = bs.next(lc, g, z, aux);
                const T* Cc = C + (int64_t)O * (g + (int64_t)G * i);
#pragma unroll
                for (int o = 0; o < OMAX; ++o)
                    if (o < O) acc[o] = kfma<T>(Cc[o], phi, acc[o]);
            }
            if (lc.use_base) {
                const T sw = swish<T>(xi);
                const T* Wi = W + (int64_t)O * i;
#pragma unroll
                for (int o = 0; o < OMAX; ++o)
                    if (o < O) bas[o] = kfma<T>(Wi[o], sw, bas[o]);
            }
        }
#pragma unroll
        for (int o = 0; o < OMAX; ++o)
            if (o < O) y[(int64_t)O * k + o] = lc.use_base ? acc[o] + bas[o] : acc[o];
    }
}

// Column VJP with LDS staging: per tile of TILE columns every thread stages its
// basis values φ[c][t], ȳ[o][t], swish(x)[i][t] in LDS (rows padded to TILE+1),
// then the block computes the tile's dC = ȳ·φᵀ, dW = ȳ·swish(x)ᵀ with each
// thread owning <= NPT parameters (accumulated in registers across tiles).
template <typename T, int PATH, int OMAX, int TILE, int NPT>
__global__ void __launch_bounds__(TILE)
kd_vjp_col_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                  const T* __restrict__ ybar, T* __restrict__ xbar, T* __restrict__ slab, int64_t K) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* smem = reinterpret_cast<T*>(smem_raw);
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;
    const int GI = G * I;
    const int nC = O * GI;
    const int P = nC + (lc.use_base ? O * I : 0);
    constexpr int LD = TILE + 1;
    T* phiL = smem;                        // [GI][LD]
    T* ybL = phiL + (int64_t)GI * LD;      // [O][LD]
    T* swL = ybL + (int64_t)O * LD;        // [I][LD]
    const T* __restrict__ C = p + lc.p_off;
    const T* __restrict__ W = p + lc.w_off;
    const int t = threadIdx.x;
    T dacc[NPT];
#pragma unroll
    for (int q = 0; q < NPT; ++q) dacc[q] = T(0);
    const T invh = T(lc.invh);
    for (int64_t tile = blockIdx.x; tile * TILE < K; tile += gridDim.x) {
        const int64_t k = tile * TILE + t;
        const bool valid = k < K;
        T yb[OMAX];
#pragma unroll
        for (int o = 0; o < OMAX; ++o) yb[o] = (o < O && valid) ? ybar[(int64_t)O * k + o] : T(0);
#pragma unroll
        for (int o = 0; o < OMAX; ++o) if (o < O) ybL[o * LD + t] = yb[o];
        for (int i = 0; i < I; ++i) {
            const T xi = valid ? x[(int64_t)I * k + i] : T(0);
            const T n = normalize<T>(lc.norm, xi);
            BasisStream<T, PATH> bs;
            bs.init(lc, n);
            T nbar = T(0);
            for (int g = 0; g < G; ++g) {
                T z, aux;
                const T phi = bs.next(lc, g, z, aux);
                const int c = g + G * i;
                const T* Cc = C + (int64_t)O * c;
                T bb = T(0);
#pragma unroll
                for (int o = 0; o < OMAX; ++o) if (o < O) bb = kfma<T>(Cc[o], yb[o], bb);
                const T zb = basis_pull<T>(lc.basis, lc.iqf_quirk, z, phi, aux, bb);
                nbar = nbar + zb * invh;
                phiL[c * LD + t] = valid ? phi : T(0);
            }
            T xb = nbar * dnormalize<T>(lc.norm, n);
            if (lc.use_base) {
                T sw, dsw;
                swish_and_grad<T>(xi, sw, dsw);
                const T* Wi = W + (int64_t)O * i;
                T sb = T(0);
#pragma unroll
                for (int o = 0; o < OMAX; ++o) if (o < O) sb = kfma<T>(Wi[o], yb[o], sb);
                xb = xb + sb * dsw;
                swL[i * LD + t] = valid ? sw : T(0);
            }
            if (valid) xbar[(int64_t)I * k + i] = xb;
        }
        __syncthreads();
        const int nt = (int)((K - tile * TILE) < TILE ? (K - tile * TILE) : TILE);
#pragma unroll
        for (int qq = 0; qq < NPT; ++qq) {
            const int q = t + qq * TILE;
            if (q < P) {
                const T* a;
                const T* b;
                if (q < nC) { a = ybL + (q % O) * LD; b = phiL + (q / O) * LD; }
                else { const int r = q - nC; a = ybL + (r % O) * LD; b = swL + (r / O) * LD; }
                T s = T(0);
                for (int tt = 0; tt < nt; ++tt) s = kfma<T>(a[tt], b[tt], s);
                dacc[qq] += s;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int qq = 0; qq < NPT; ++qq) {
        const int q = t + qq * TILE;
        if (q < P) slab[(int64_t)blockIdx.x * P + q] = dacc[qq];
    }
}

// Per-edge activations act[o + O*(i + I*k)] (Activation_getter.jl:28-31,48-53).
template <typename T, int PATH, int OMAX>
__global__ void __launch_bounds__(kBlock)
kd_edge_act_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                   T* __restrict__ act, int64_t K) {
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;
    const T* __restrict__ C = p + lc.p_off;
    const T* __restrict__ W = p + lc.w_off;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < K; k += stride) {
        for (int i = 0; i < I; ++i) {
            const T xi = x[(int64_t)I * k + i];
            T acc[OMAX];
#pragma unroll
            for (int o = 0; o < OMAX; ++o) acc[o] = T(0);
            BasisStream<T, PATH> bs;
            bs.init(lc, normalize<T>(lc.norm, xi));
            for (int g = 0; g < G; ++g) {
                T z, aux;
                const T phi = bs.next(lc, g, z, aux);
                const T* Cc = C + (int64_t)O * (g + (int64_t)G * i);
#pragma unroll
                for (int o = 0; o < OMAX; ++o) if (o < O) acc[o] = kfma<T>(phi, Cc[o], acc[o]);
            }
            const T sw = lc.use_base ? swish<T>(xi) : T(0);
#pragma unroll
            for (int o = 0; o < OMAX; ++o)
                if (o < O)
                    act[(int64_t)O * ((int64_t)I * k + i) + o] =
                        lc.use_base ? kfma<T>(sw, W[(int64_t)O * i + o], acc[o]) : acc[o];
        }
    }
}

// ---------------------------------------------------------------------------
// launchers
static inline int grid_for(int64_t work, int per_block, int cap) {
    int64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    return (int)(g < cap ? g : cap);
}
constexpr int kGridCap = 256 * 16;   // 16 blocks per CU over 256 CUs, grid-stride beyond

template <typename T, int PATH, int GT>
static hipError_t fk_rhs_go(const LayerConst* lc, const T* p, T cd, T co, int Nx, const T* u, T* du,
                            int64_t B, hipStream_t st) {
    const int64_t npts = (int64_t)Nx * B;
    if (Nx % 2 == 0) {
        const int64_t np = npts / 2;
        hipLaunchKernelGGL((fk_rhs_pair_kernel<T, PATH, GT>), dim3(grid_for(np, kBlock, kGridCap)), dim3(kBlock), 0,
                           st, lc, p, cd, co, Nx, u, du, np);
    } else {
        hipLaunchKernelGGL((fk_rhs_kernel<T, PATH, GT>), dim3(grid_for(npts, kBlock, kGridCap)), dim3(kBlock), 0,
                           st, lc, p, cd, co, Nx, u, du, npts);
    }
    return hipGetLastError();
}

template <typename T, int PATH, int GT>
static hipError_t fk_vjp_go(const LayerConst* lc, const T* p, T cd, T co, int Nx, const T* u, const T* lam,
                            T* lamJ, T* dp, int P, T* slab, int slab_blocks, int64_t B, hipStream_t st) {
    const int64_t npts = (int64_t)Nx * B;
    const int nb = grid_for(npts, kBlock, slab_blocks);
    hipLaunchKernelGGL((fk_vjp_kernel<T, PATH, GT>), dim3(nb), dim3(kBlock), 0, st, lc, p, cd, co, Nx, u, lam,
                       lamJ, slab, npts);
    if (dp) hipLaunchKernelGGL((slab_reduce_kernel<T>), dim3(P), dim3(kBlock), 0, st, slab, (int64_t)nb, (int64_t)P, dp);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_fk_rhs(const LayerConst& hlc, const LayerConst* lc, const T* p, T cd, T co, int Nx,
                         const T* u, T* du, int64_t B, hipStream_t st) {
    const int G = hlc.G;
    switch (hlc.path) {
    case PATH_REC_CORR:
        if (G == 10) return fk_rhs_go<T, PATH_REC_CORR, 10>(lc, p, cd, co, Nx, u, du, B, st);
        return fk_rhs_go<T, PATH_REC_CORR, 0>(lc, p, cd, co, Nx, u, du, B, st);
    case PATH_REC:
        if (G == 5) return fk_rhs_go<T, PATH_REC, 5>(lc, p, cd, co, Nx, u, du, B, st);
        return fk_rhs_go<T, PATH_REC, 0>(lc, p, cd, co, Nx, u, du, B, st);
    default:
        return fk_rhs_go<T, PATH_DIRECT, 0>(lc, p, cd, co, Nx, u, du, B, st);
    }
}

template <typename T>
hipError_t launch_fk_vjp(const LayerConst& hlc, const LayerConst* lc, const T* p, T cd, T co, int Nx,
                         const T* u, const T* lam, T* lamJ, T* dp, T* slab, int slab_blocks, int64_t B,
                         hipStream_t st) {
    const int G = hlc.G;
    const int P = G + (hlc.use_base ? 1 : 0);
    switch (hlc.path) {
    case PATH_REC_CORR:
        if (G == 10) return fk_vjp_go<T, PATH_REC_CORR, 10>(lc, p, cd, co, Nx, u, lam, lamJ, dp, P, slab, slab_blocks, B, st);
        return fk_vjp_go<T, PATH_REC_CORR, 0>(lc, p, cd, co, Nx, u, lam, lamJ, dp, P, slab, slab_blocks, B, st);
    case PATH_REC:
        if (G == 5) return fk_vjp_go<T, PATH_REC, 5>(lc, p, cd, co, Nx, u, lam, lamJ, dp, P, slab, slab_blocks, B, st);
        return fk_vjp_go<T, PATH_REC, 0>(lc, p, cd, co, Nx, u, lam, lamJ, dp, P, slab, slab_blocks, B, st);
    default:
        return fk_vjp_go<T, PATH_DIRECT, 0>(lc, p, cd, co, Nx, u, lam, lamJ, dp, P, slab, slab_blocks, B, st);
    }
}

template <typename T, int PATH>
static hipError_t col_fwd_go(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, T* y, int64_t K,
                             hipStream_t st) {
    const int g = grid_for(K, kBlock, kGridCap);
    if (hlc.O <= 4) hipLaunchKernelGGL((kd_fwd_col_kernel<T, PATH, 4>), dim3(g), dim3(kBlock), 0, st, lc, p, x, y, K);
    else if (hlc.O <= 16) hipLaunchKernelGGL((kd_fwd_col_kernel<T, PATH, 16>), dim3(g), dim3(kBlock), 0, st, lc, p, x, y, K);
    else hipLaunchKernelGGL((kd_fwd_col_kernel<T, PATH, 64>), dim3(g), dim3(kBlock), 0, st, lc, p, x, y, K);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_kd_fwd_col(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, T* y, int64_t K,
                             hipStream_t st) {
    switch (hlc.path) {
    case PATH_REC_CORR: return col_fwd_go<T, PATH_REC_CORR>(hlc, lc, p, x, y, K, st);
    case PATH_REC: return col_fwd_go<T, PATH_REC>(hlc, lc, p, x, y, K, st);
    default: return col_fwd_go<T, PATH_DIRECT>(hlc, lc, p, x, y, K, st);
    }
}

template <typename T, int PATH, int OMAX, int TILE, int NPT>
static hipError_t col_vjp_go2(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, const T* yb,
                              T* xb, T* pbar, T* slab, int slab_blocks, int64_t K, hipStream_t st) {
    const int GI = hlc.G * hlc.I;
    const size_t lds = sizeof(T) * (size_t)(GI + hlc.O + hlc.I) * (TILE + 1);
    const int P = hlc.O * GI + (hlc.use_base ? hlc.O * hlc.I : 0);
    const int nb = grid_for(K, TILE, slab_blocks);
    hipLaunchKernelGGL((kd_vjp_col_kernel<T, PATH, OMAX, TILE, NPT>), dim3(nb), dim3(TILE), lds, st, lc, p, x, yb,
                       xb, slab, K);
    if (pbar)
        hipLaunchKernelGGL((slab_reduce_kernel<T>), dim3(P), dim3(kBlock), 0, st, slab, (int64_t)nb, (int64_t)P,
                           pbar + hlc.p_off);
    return hipGetLastError();
}

template <typename T, int PATH>
static hipError_t col_vjp_go(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, const T* yb, T* xb,
                             T* pbar, T* slab, int slab_blocks, int64_t K, hipStream_t st) {
    const int GI = hlc.G * hlc.I;
    const int P = hlc.O * GI + (hlc.use_base ? hlc.O * hlc.I : 0);
    const size_t rows = (size_t)(GI + hlc.O + hlc.I);
    if (rows * 257 * sizeof(T) <= 150 * 1024 && P <= 256 * 8) {
        if (hlc.O <= 4) return col_vjp_go2<T, PATH, 4, 256, 8>(hlc, lc, p, x, yb, xb, pbar, slab, slab_blocks, K, st);
        return col_vjp_go2<T, PATH, 16, 256, 8>(hlc, lc, p, x, yb, xb, pbar, slab, slab_blocks, K, st);
    }
    // narrow tile (64 columns, one wave) for wider layers
    if (hlc.O <= 4) return col_vjp_go2<T, PATH, 4, 64, 32>(hlc, lc, p, x, yb, xb, pbar, slab, slab_blocks, K, st);
    return col_vjp_go2<T, PATH, 16, 64, 32>(hlc, lc, p, x, yb, xb, pbar, slab, slab_blocks, K, st);
}

template <typename T>
hipError_t launch_kd_vjp_col(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, const T* yb,
                             T* xb, T* pbar, T* slab, int slab_blocks, int64_t K, hipStream_t st) {
    switch (hlc.path) {
    case PATH_REC_CORR: return col_vjp_go<T, PATH_REC_CORR>(hlc, lc, p, x, yb, xb, pbar, slab, slab_blocks, K, st);
    case PATH_REC: return col_vjp_go<T, PATH_REC>(hlc, lc, p, x, yb, xb, pbar, slab, slab_blocks, K, st);
    default: return col_vjp_go<T, PATH_DIRECT>(hlc, lc, p, x, yb, xb, pbar, slab, slab_blocks, K, st);
    }
}

template <typename T, int PATH>
static hipError_t edge_go(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, T* act, int64_t K,
                          hipStream_t st) {
    const int g = grid_for(K, kBlock, kGridCap);
    if (hlc.O <= 16) hipLaunchKernelGGL((kd_edge_act_kernel<T, PATH, 16>), dim3(g), dim3(kBlock), 0, st, lc, p, x, act, K);
    else hipLaunchKernelGGL((kd_edge_act_kernel<T, PATH, 64>), dim3(g), dim3(kBlock), 0, st, lc, p, x, act, K);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_kd_edge_act(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, T* act, int64_t K,
                              hipStream_t st) {
    switch (hlc.path) {
    case PATH_REC_CORR: return edge_go<T, PATH_REC_CORR>(hlc, lc, p, x, act, K, st);
    case PATH_REC: return edge_go<T, PATH_REC>(hlc, lc, p, x, act, K, st);
    default: return edge_go<T, PATH_DIRECT>(hlc, lc, p, x, act, K, st);
    }
}

// explicit instantiations
#define KAN_INST(T)                                                                                              \
    template hipError_t launch_fk_rhs<T>(const LayerConst&, const LayerConst*, const T*, T, T, int, const T*, T*, \
                                         int64_t, hipStream_t);                                                   \
    template hipError_t launch_fk_vjp<T>(const LayerConst&, const LayerConst*, const T*, T, T, int, const T*,     \
                                         const T*, T*, T*, T*, int, int64_t, hipStream_t);                        \
    template hipError_t launch_kd_fwd_col<T>(const LayerConst&, const LayerConst*, const T*, const T*, T*,        \
                                             int64_t, hipStream_t);                                               \
    template hipError_t launch_kd_vjp_col<T>(const LayerConst&, const LayerConst*, const T*, const T*, const T*,  \
                                             T*, T*, T*, int, int64_t, hipStream_t);                              \
    template hipError_t launch_kd_edge_act<T>(const LayerConst&, const LayerConst*, const T*, const T*, T*,       \
                                              int64_t, hipStream_t);
KAN_INST(double)
KAN_INST(float)
#undef KAN_INST

}  // namespace kan
