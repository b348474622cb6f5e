// kan_fk.hip — Fisher-KPP source-term RHS and its VJP (gfx950).
//
//   rc_kanode(u, p, t) = D*lap*u + kan1_.(u)      PDE examples/Fisher-KPP_Source.jl:95-98
//   lap: tridiag(1,-2,1)/dx² + periodic corners   PDE examples/Fisher-KPP_Source.jl:55-59
//   kan1 = KDense(1, 1, G) applied pointwise       PDE examples/Fisher-KPP_Source.jl:81-86,96
//
// State u is the reference's [Nx, B] column-major array (trajectory contiguous).
// Thread mapping is division-free: a power-of-two group of TPT threads walks the
// point pairs of one trajectory (aligned 16-byte loads/stores for fp64), 256/TPT
// trajectories per block, blocks grid-stride over trajectories.  Neighbours for
// the stencil come from the same cache lines (L1/L2 hits; HBM traffic stays at
// one read of u and one write of du).
//
// The [1,1] KDense is evaluated with the left-anchored Gaussian recurrence
// (kan_device.hpp): 2 exp per point + Horner sweeps in R = exp(2 z0 δ) over the
// G knots (3 interleaved sweeps when the Float32 knots need the e_j correction).
// Everything the inner loop reads (coefficients, knots, scalars) is loaded into
// registers once per thread (FK11): no scalar loads inside the loop.
#include "kan_common.hpp"
#include "kan_kernels.hpp"
#include "kan_lap.hpp"

namespace kan {

// Per-thread registers for the [1,1] KDense: coefficients, knots and scalars.
template <typename T, int GL>
struct FK11 {
    T A[GL], Bq[GL], Q[GL];     // Horner sets: C_j K_j, C_j K_j e_j, C_j K_j e_j²/2
    T C[GL], CD[GL];            // C_j, C_j Δ_j (pullback)
    T K[GL], KE[GL], KQ[GL];    // K_j, K_j e_j, K_j e_j²/2
    T Dl[GL], grid[GL];
    float Qf[GL];               // Q_j · 2^40 in fp32 (the 2nd-order sweep, relative weight <= 6e-13)
    T W, invh;
    RecScalars<T> rc;
    int G, norm, basis, iqf, use_base;
    __device__ __forceinline__ explicit FK11(const LayerConst& lc) : rc(lc) {}
};

// FWD loads the Horner sets, !FWD the pullback sets; on the compile-time grid the
// hot sets go to SGPRs (to_sgpr) so the VGPR budget is left to the per-point work.
template <typename T, int GT, bool FWD>
__device__ __forceinline__ void fk_load_coef(const LayerConst& lc, const T* __restrict__ p,
                                             FK11<T, GT ? GT : kMaxGrid>& cf) {
    constexpr int GL = GT ? GT : kMaxGrid;
    const int G = lc.G;
#pragma unroll
    for (int j = 0; j < GL; ++j) {
        const bool on = GT ? true : (j < G);
        const T c = on ? p[j] : T(0);
        const T k = on ? T(lc.K[j]) : T(0);
        const T e = on ? T(lc.e[j]) : T(0);
        const T q = T(0.5) * e * e;
        const T dl = on ? T(lc.Dl[j]) : T(0);
        cf.C[j] = c;
        cf.Dl[j] = dl;
        cf.grid[j] = on ? T(lc.grid[j]) : T(0);
        if constexpr (FWD) {
            cf.A[j] = GT ? to_sgpr(c * k) : c * k;
            cf.Bq[j] = GT ? to_sgpr(c * k * e) : c * k * e;
            cf.Q[j] = c * k * q;
            cf.Qf[j] = GT ? to_sgpr((float)((double)(c * k * q) * 0x1p40)) : (float)((double)(c * k * q) * 0x1p40);
        } else {
            cf.K[j] = GT ? to_sgpr(k) : k;
            cf.KE[j] = k * e;
            cf.KQ[j] = k * q;
            cf.C[j] = GT ? to_sgpr(c) : c;
            cf.CD[j] = GT ? to_sgpr(c * dl) : c * dl;
        }
    }
    cf.G = G;
    cf.norm = lc.norm;
    cf.basis = lc.basis;
    cf.iqf = lc.iqf_quirk;
    cf.use_base = lc.use_base;
    cf.invh = T(lc.invh);
    cf.W = lc.use_base ? p[G] : T(0);
}

// KDense(1,1,G)(x) — the reference's per-point `kan1([x], p, st)[1][1]` (:96).
template <typename T, int NORM, int PATH, int GT>
__device__ __forceinline__ T kan11_fwd(const Math<T>& M, const FK11<T, GT ? GT : kMaxGrid>& cf, T x) {
    constexpr int GL = GT ? GT : kMaxGrid;
    const int G = GT ? GT : cf.G;
    const T n = normalize<NORM, T>(M, cf.norm, x);
    T spline;
    if constexpr (PATH == PATH_DIRECT) {
        T s = T(0);
#pragma unroll
        for (int j = 0; j < GL; ++j) {
            if (GT || j < G) {
                T aux;
                const T y = (n - cf.grid[j]) * cf.invh;
                s = s + cf.C[j] * basis_direct<T>(M, cf.basis, y, aux);
            }
        }
        spline = s;
    } else {
        T z0, E0, R, taup;
        rec_anchor<T>(M, cf.rc, n, z0, E0, R, taup);
        // Horner in R over j = G-1 .. 0 (GT > 0: starts from the top coefficient)
        T s0 = GT ? cf.A[GL - 1] : T(0), s1 = GT ? cf.Bq[GL - 1] : T(0), s2 = GT ? cf.Q[GL - 1] : T(0);
#pragma unroll
        for (int j = (GT ? GL - 2 : GL - 1); j >= 0; --j) {
            if (GT || j < G) {
                s0 = kfma<T>(s0, R, cf.A[j]);
                if constexpr (PATH == PATH_REC_CORR) {
                    s1 = kfma<T>(s1, R, cf.Bq[j]);
                    s2 = kfma<T>(s2, R, cf.Q[j]);
                }
            }
        }
        if constexpr (PATH == PATH_REC_CORR) spline = E0 * kfma<T>(taup, kfma<T>(taup, s2, s1), s0);
        else spline = E0 * s0;
    }
    if (cf.use_base) spline = spline + cf.W * swish<T>(M, x);   // spline + W*swish.(x) (kdense.jl:123-124)
    return spline;
}

// Two points at once, branch-free (recurrence paths, compile-time grid): the two
// independent dependency chains interleave.
template <typename T, int NORM, int PATH, int GT, bool BASE>
__device__ __forceinline__ void kan11_fwd2(const Math<T>& M, const FK11<T, GT>& cf, const T (&x)[2], T (&y)[2]) {
    static_assert(GT > 0 && PATH != PATH_DIRECT, "pair path needs a compile-time grid");
    T n[2], z0[2], E0[2], R[2], tp[2], s0[2], s1[2];
    float r32[2], s2[2];   // 2nd-order sweep in fp32 (scaled by 2^40): its weight is <= 6e-13
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        n[k] = normalize<NORM, T>(M, cf.norm, x[k]);
        rec_anchor<T>(M, cf.rc, n[k], z0[k], E0[k], R[k], tp[k]);
        s0[k] = cf.A[GT - 1];
        s1[k] = cf.Bq[GT - 1];
        s2[k] = cf.Qf[GT - 1];
        r32[k] = (float)R[k];
    }
#pragma unroll
    for (int j = GT - 2; j >= 0; --j) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            s0[k] = kfma<T>(s0[k], R[k], cf.A[j]);
            if constexpr (PATH == PATH_REC_CORR) {
                s1[k] = kfma<T>(s1[k], R[k], cf.Bq[j]);
                s2[k] = fmaf(s2[k], r32[k], cf.Qf[j]);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const T q2 = T((double)s2[k] * 0x1p-40);
        T sp = (PATH == PATH_REC_CORR) ? E0[k] * kfma<T>(tp[k], kfma<T>(tp[k], q2, s1[k]), s0[k]) : E0[k] * s0[k];
        if constexpr (BASE) sp = sp + cf.W * swish<T>(M, x[k]);
        y[k] = sp;
    }
}

// One point of the pullback: returns x̄, accumulates dC_j += λ φ_j, dW += λ swish(x).
//   x̄ = n̄ N'(Ω) + (W λ) swish'(x),  n̄ = Σ_j (-2 z_j φ_j C_j λ)(1/h)   (utils.jl:18 rrule)
template <typename T, int NORM, int PATH, int GT>
__device__ __forceinline__ T kan11_vjp(const Math<T>& M, const FK11<T, GT ? GT : kMaxGrid>& cf, T x, T lam,
                                       T (&dC)[GT ? GT : kMaxGrid], T& dW) {
    constexpr int GL = GT ? GT : kMaxGrid;
    const int G = GT ? GT : cf.G;
    const T n = normalize<NORM, T>(M, cf.norm, x);
    T nbar;
    if constexpr (PATH == PATH_DIRECT) {
        nbar = T(0);
#pragma unroll
        for (int j = 0; j < GL; ++j) {
            if (GT || j < G) {
                T aux = T(0);
                const T y = (n - cf.grid[j]) * cf.invh;
                const T phi = basis_direct<T>(M, cf.basis, y, aux);
                const T zb = basis_pull<T>(cf.basis, cf.iqf, y, phi, aux, cf.C[j] * lam);
                nbar = nbar + zb * cf.invh;
                dC[j] = kfma<T>(lam, phi, dC[j]);
            }
        }
    } else {
        T z0, F, R, taup;
        rec_anchor<T>(M, cf.rc, n, z0, F, R, taup);
        T sa = T(0), sb = T(0);   // Σ C_j φ_j, Σ C_j Δ_j φ_j  ->  Σ C_j z_j φ_j = z0·sa - sb
#pragma unroll
        for (int j = 0; j < GL; ++j) {
            if (GT || j < G) {
                T kc = cf.K[j];
                if constexpr (PATH == PATH_REC_CORR) kc = kfma<T>(taup, kfma<T>(taup, cf.KQ[j], cf.KE[j]), cf.K[j]);
                const T phi = F * kc;
                dC[j] = kfma<T>(lam, phi, dC[j]);
                sa = kfma<T>(cf.C[j], phi, sa);
                sb = kfma<T>(cf.CD[j], phi, sb);
                F = F * R;
            }
        }
        nbar = (T(-2) * cf.invh) * lam * kfma<T>(z0, sa, -sb);
    }
    T xb = nbar * dnormalize<NORM, T>(cf.norm, n);
    if (cf.use_base) {
        T sw, dsw;
        swish_and_grad<T>(M, x, sw, dsw);
        xb = xb + (cf.W * lam) * dsw;
        dW = kfma<T>(lam, sw, dW);
    }
    return xb;
}

// SHORT: one unit (point or pair) per thread per trajectory (Nx <= 512) — the hot
// shape; the long-grid loop is a separate instantiation so it cannot inflate the
// short kernel's register allocation.
template <typename T, int NORM, int PATH, int GT, bool PAIR, bool SHORT>
__global__ void __launch_bounds__(kBlock)
fk_rhs_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, T cd, T co, int Nx, int tpt_log2,
              const T* __restrict__ u, T* __restrict__ du, int64_t B) {
    using V2 = typename Vec2<T>::type;
    constexpr int GL = GT ? GT : kMaxGrid;
    KAN_EXP_TABLE_LDS(tab);
    const Math<T> M{tab};
    FK11<T, GL> cf(*lcp);
    fk_load_coef<T, GT, true>(*lcp, p, cf);
    const int tpt = 1 << tpt_log2;
    const int tpb = kBlock >> tpt_log2;
    const int lt = threadIdx.x & (tpt - 1);
    const int units = PAIR ? (Nx >> 1) : Nx;
    const int64_t b0 = (int64_t)blockIdx.x * tpb + (threadIdx.x >> tpt_log2);
    const int64_t bstride = (int64_t)gridDim.x * tpb;
    if constexpr (SHORT) {
        // one unit (point or pair) per thread per trajectory: Nx <= 512
        const int q = lt;
        if (q >= units) return;
        const int i = PAIR ? 2 * q : q;
        const int im = i > 0 ? i - 1 : Nx - 1;
        const int ip = (i + (PAIR ? 2 : 1)) < Nx ? i + (PAIR ? 2 : 1) : 0;
        for (int64_t b = b0; b < B; b += bstride) {
            const T* __restrict__ ub = u + b * Nx;
            T* __restrict__ db = du + b * Nx;
            if constexpr (PAIR) {
                const V2 v = *reinterpret_cast<const V2*>(ub + i);
                const T um = ub[im], up = ub[ip];
                T k0, k1, l0, l1;
                if constexpr (GT > 0 && PATH != PATH_DIRECT) {
                    // both points in one branch-free body (interleaved chains)
                    const T xs[2] = {v.x, v.y};
                    T ks[2];
                    if (cf.use_base) kan11_fwd2<T, NORM, PATH, GT, true>(M, cf, xs, ks);
                    else kan11_fwd2<T, NORM, PATH, GT, false>(M, cf, xs, ks);
                    k0 = ks[0];
                    k1 = ks[1];
                } else {
                    k0 = kan11_fwd<T, NORM, PATH, GT>(M, cf, v.x);
                    k1 = kan11_fwd<T, NORM, PATH, GT>(M, cf, v.y);
                }
                if (Nx >= 4) {
                    lap_pair<T>(um, v.x, v.y, up, i, Nx, cd, co, l0, l1);
                } else {
                    l0 = lap3<T>(um, v.x, v.y, i, Nx, cd, co);
                    l1 = lap3<T>(v.x, v.y, up, i + 1, Nx, cd, co);
                }
                V2 o;
                o.x = l0 + k0;
                o.y = l1 + k1;
                *reinterpret_cast<V2*>(db + i) = o;
            } else {
                const T u0 = ub[i], um = ub[im], up = ub[ip];
                db[i] = lap3<T>(um, u0, up, i, Nx, cd, co) + kan11_fwd<T, NORM, PATH, GT>(M, cf, u0);
            }
        }
        return;
    }
    (void)units;
    for (int64_t b = b0; b < B; b += bstride) {
        const T* __restrict__ ub = u + b * Nx;
        T* __restrict__ db = du + b * Nx;
        for (int q = lt; q < units; q += tpt) {
            if constexpr (PAIR) {
                const int i = 2 * q;
                const V2 v = *reinterpret_cast<const V2*>(ub + i);
                const T um = ub[i > 0 ? i - 1 : Nx - 1];
                const T up = ub[i + 2 < Nx ? i + 2 : 0];
                V2 o;
                o.x = lap3<T>(um, v.x, v.y, i, Nx, cd, co) + kan11_fwd<T, NORM, PATH, GT>(M, cf, v.x);
                o.y = lap3<T>(v.x, v.y, up, i + 1, Nx, cd, co) + kan11_fwd<T, NORM, PATH, GT>(M, cf, v.y);
                *reinterpret_cast<V2*>(db + i) = o;
            } else {
                const int i = q;
                const T u0 = ub[i];
                const T um = ub[i > 0 ? i - 1 : Nx - 1];
                const T up = ub[i + 1 < Nx ? i + 1 : 0];
                db[i] = lap3<T>(um, u0, up, i, Nx, cd, co) + kan11_fwd<T, NORM, PATH, GT>(M, cf, u0);
            }
        }
    }
}

template <typename T, int NORM, int PATH, int GT, bool PAIR>
__global__ void __launch_bounds__(kBlock)
fk_vjp_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, T cd, T co, int Nx, int tpt_log2,
              const T* __restrict__ u, const T* __restrict__ lam, T* __restrict__ lamJ, T* __restrict__ slab,
              int64_t B) {
    using V2 = typename Vec2<T>::type;
    constexpr int GL = GT ? GT : kMaxGrid;
    __shared__ T red[(kBlock / kWave) * (GL + 1)];
    KAN_EXP_TABLE_LDS(tab);
    const Math<T> M{tab};
    FK11<T, GL> cf(*lcp);
    fk_load_coef<T, GT, false>(*lcp, p, cf);
    T dC[GL];
#pragma unroll
    for (int j = 0; j < GL; ++j) dC[j] = T(0);
    T dW = T(0);
    const int tpt = 1 << tpt_log2;
    const int tpb = kBlock >> tpt_log2;
    const int lt = threadIdx.x & (tpt - 1);
    const int units = PAIR ? (Nx >> 1) : Nx;
    const int64_t b0 = (int64_t)blockIdx.x * tpb + (threadIdx.x >> tpt_log2);
    const int64_t bstride = (int64_t)gridDim.x * tpb;
    for (int64_t b = b0; b < B; b += bstride) {
        const T* __restrict__ ub = u + b * Nx;
        const T* __restrict__ lb = lam + b * Nx;
        T* __restrict__ ob = lamJ + b * Nx;
        for (int q = lt; q < units; q += tpt) {
            // (D*lap)ᵀ λ : lap is symmetric, same row formula on λ
            if constexpr (PAIR) {
                const int i = 2 * q;
                const V2 lv = *reinterpret_cast<const V2*>(lb + i);
                const V2 uv = *reinterpret_cast<const V2*>(ub + i);
                const T lm = lb[i > 0 ? i - 1 : Nx - 1];
                const T lp = lb[i + 2 < Nx ? i + 2 : 0];
                T l0, l1;
                if (Nx >= 4) {
                    lap_pair<T>(lm, lv.x, lv.y, lp, i, Nx, cd, co, l0, l1);
                } else {
                    l0 = lap3<T>(lm, lv.x, lv.y, i, Nx, cd, co);
                    l1 = lap3<T>(lv.x, lv.y, lp, i + 1, Nx, cd, co);
                }
                V2 o;
                o.x = l0 + kan11_vjp<T, NORM, PATH, GT>(M, cf, uv.x, lv.x, dC, dW);
                o.y = l1 + kan11_vjp<T, NORM, PATH, GT>(M, cf, uv.y, lv.y, dC, dW);
                *reinterpret_cast<V2*>(ob + i) = o;
            } else {
                const int i = q;
                const T l0 = lb[i];
                const T lm = lb[i > 0 ? i - 1 : Nx - 1];
                const T lp = lb[i + 1 < Nx ? i + 1 : 0];
                ob[i] = lap3<T>(lm, l0, lp, i, Nx, cd, co) + kan11_vjp<T, NORM, PATH, GT>(M, cf, ub[i], l0, dC, dW);
            }
        }
    }
    const int G = GT ? GT : cf.G;
    const int P = G + (cf.use_base ? 1 : 0);
    T acc[GL + 1];
#pragma unroll
    for (int j = 0; j < GL; ++j) acc[j] = dC[j];
    acc[GL] = T(0);
#pragma unroll
    for (int j = 0; j <= GL; ++j)   // pack (C_0..C_{G-1}, W) contiguously
        if (j == G) acc[j] = dW;
    block_sum_to<T, GL + 1>(acc, P, red, slab + (int64_t)blockIdx.x * P);
}

// ---------------------------------------------------------------------------
template <typename T, int NORM, int PATH, int GT>
static hipError_t fk_rhs_go(const LayerConst* lc, const T* p, T cd, T co, int Nx, const T* u, T* du, int64_t B,
                            hipStream_t st) {
    const bool pair = (Nx % 2 == 0);
    const int units = pair ? Nx / 2 : Nx;
    const int tl = ceil_log2(units < kBlock ? units : kBlock);
    const int tpb = kBlock >> tl;
    const int grid = grid_for(B, tpb, kGridCap);
    const bool shortg = units <= kBlock;
    if (pair && shortg)
        hipLaunchKernelGGL((fk_rhs_kernel<T, NORM, PATH, GT, true, true>), dim3(grid), dim3(kBlock), 0, st, lc, p, cd,
                           co, Nx, tl, u, du, B);
    else if (pair)
        hipLaunchKernelGGL((fk_rhs_kernel<T, NORM, PATH, GT, true, false>), dim3(grid), dim3(kBlock), 0, st, lc, p,
                           cd, co, Nx, tl, u, du, B);
    else if (shortg)
        hipLaunchKernelGGL((fk_rhs_kernel<T, NORM, PATH, GT, false, true>), dim3(grid), dim3(kBlock), 0, st, lc, p,
                           cd, co, Nx, tl, u, du, B);
    else
        hipLaunchKernelGGL((fk_rhs_kernel<T, NORM, PATH, GT, false, false>), dim3(grid), dim3(kBlock), 0, st, lc, p,
                           cd, co, Nx, tl, u, du, B);
    return hipGetLastError();
}

template <typename T, int NORM, int PATH, int GT>
static hipError_t fk_vjp_go(const LayerConst* lc, const T* p, T cd, T co, int Nx, const T* u, const T* lam, T* lamJ,
                            T* dp, int P, T* slab, int slab_blocks, int64_t B, hipStream_t st) {
    const bool pair = (Nx % 2 == 0);
    const int units = pair ? Nx / 2 : Nx;
    const int tl = ceil_log2(units < kBlock ? units : kBlock);
    const int tpb = kBlock >> tl;
    const int grid = grid_for(B, tpb, slab_blocks);
    if (pair)
        hipLaunchKernelGGL((fk_vjp_kernel<T, NORM, PATH, GT, true>), dim3(grid), dim3(kBlock), 0, st, lc, p, cd, co,
                           Nx, tl, u, lam, lamJ, slab, B);
    else
        hipLaunchKernelGGL((fk_vjp_kernel<T, NORM, PATH, GT, false>), dim3(grid), dim3(kBlock), 0, st, lc, p, cd,
                           co, Nx, tl, u, lam, lamJ, slab, B);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !dp) return e;
    return launch_slab_reduce<T>(slab, grid, P, dp, st);
}

// Specialised instantiations for the reference configurations (softsign G=10,
// tanh_fast G=5), a generic runtime-normalizer kernel for everything else.
template <typename T>
hipError_t launch_fk_rhs(const LayerConst& hlc, const LayerConst* lc, const T* p, T cd, T co, int Nx, const T* u,
                         T* du, int64_t B, hipStream_t st) {
    const int G = hlc.G;
    if (hlc.norm == NORM_SOFTSIGN && hlc.path == PATH_REC_CORR && G == 10)
        return fk_rhs_go<T, NORM_SOFTSIGN, PATH_REC_CORR, 10>(lc, p, cd, co, Nx, u, du, B, st);
    if (hlc.norm == NORM_SOFTSIGN && hlc.path == PATH_REC && G == 5)
        return fk_rhs_go<T, NORM_SOFTSIGN, PATH_REC, 5>(lc, p, cd, co, Nx, u, du, B, st);
    if (hlc.norm == NORM_TANH_FAST && hlc.path == PATH_REC && G == 5)
        return fk_rhs_go<T, NORM_TANH_FAST, PATH_REC, 5>(lc, p, cd, co, Nx, u, du, B, st);
    switch (hlc.path) {
    case PATH_REC_CORR: return fk_rhs_go<T, NORM_RUNTIME, PATH_REC_CORR, 0>(lc, p, cd, co, Nx, u, du, B, st);
    case PATH_REC: return fk_rhs_go<T, NORM_RUNTIME, PATH_REC, 0>(lc, p, cd, co, Nx, u, du, B, st);
    default: return fk_rhs_go<T, NORM_RUNTIME, PATH_DIRECT, 0>(lc, p, cd, co, Nx, u, du, B, st);
    }
}

template <typename T>
hipError_t launch_fk_vjp(const LayerConst& hlc, const LayerConst* lc, const T* p, T cd, T co, int Nx, const T* u,
                         const T* lam, T* lamJ, T* dp, T* slab, int slab_blocks, int64_t B, hipStream_t st) {
    const int G = hlc.G;
    const int P = G + (hlc.use_base ? 1 : 0);
    if (hlc.norm == NORM_SOFTSIGN && hlc.path == PATH_REC_CORR && G == 10)
        return fk_vjp_go<T, NORM_SOFTSIGN, PATH_REC_CORR, 10>(lc, p, cd, co, Nx, u, lam, lamJ, dp, P, slab,
                                                              slab_blocks, B, st);
    if (hlc.norm == NORM_SOFTSIGN && hlc.path == PATH_REC && G == 5)
        return fk_vjp_go<T, NORM_SOFTSIGN, PATH_REC, 5>(lc, p, cd, co, Nx, u, lam, lamJ, dp, P, slab, slab_blocks,
                                                        B, st);
    if (hlc.norm == NORM_TANH_FAST && hlc.path == PATH_REC && G == 5)
        return fk_vjp_go<T, NORM_TANH_FAST, PATH_REC, 5>(lc, p, cd, co, Nx, u, lam, lamJ, dp, P, slab, slab_blocks,
                                                         B, st);
    switch (hlc.path) {
    case PATH_REC_CORR:
        return fk_vjp_go<T, NORM_RUNTIME, PATH_REC_CORR, 0>(lc, p, cd, co, Nx, u, lam, lamJ, dp, P, slab, slab_blocks,
                                                            B, st);
    case PATH_REC:
        return fk_vjp_go<T, NORM_RUNTIME, PATH_REC, 0>(lc, p, cd, co, Nx, u, lam, lamJ, dp, P, slab, slab_blocks, B,
                                                       st);
    default:
        return fk_vjp_go<T, NORM_RUNTIME, PATH_DIRECT, 0>(lc, p, cd, co, Nx, u, lam, lamJ, dp, P, slab, slab_blocks,
                                                          B, st);
    }
}

#define KAN_FK_INST(T)                                                                                           \
    template hipError_t launch_fk_rhs<T>(const LayerConst&, const LayerConst*, const T*, T, T, int, const T*, T*, \
                                         int64_t, hipStream_t);                                                   \
    template hipError_t launch_fk_vjp<T>(const LayerConst&, const LayerConst*, const T*, T, T, int, const T*,     \
                                         const T*, T*, T*, T*, int, int64_t, hipStream_t);
KAN_FK_INST(double)
KAN_FK_INST(float)
#undef KAN_FK_INST

}  // namespace kan
