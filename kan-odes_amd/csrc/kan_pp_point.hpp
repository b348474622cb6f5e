// kan_pp_point.hpp — per-point evaluation of the piecewise-polynomial pointwise KAN (kan_pp.hip): the
// reference formula (the tables' build and the cold path), the table lookup, and one point of the
// pullback with its dC moments.  Shared by the Fisher-KPP table kernels (kan_pp.hip) and the
// one-workgroup small-field solve and adjoint (kan_small.hip).  Reference: kdense.jl:109-130,
// utils.jl:8-21, PDE examples/Fisher-KPP_Source.jl:95-98 (relative to /root/reference).
#pragma once
#include "kan_common.hpp"

#ifndef KAN_VJP_PACKED
#define KAN_VJP_PACKED 1
#endif

namespace kan {
#ifdef KAN_CLOCK_PROBE
extern __device__ unsigned long long kan_clock_probe[32];   // (kan_pp.hip, diagnostic build only)
#endif

// φ(u) by the reference's formula: normalizer, Σ_j C_j basis((n - g_j)/h) in
// ascending j, + W swish(u).  `sc` returns Σ|terms|.  NORM / BASIS >= 0 fix the
// normalizer / basis at compile time (-1: runtime switch).
template <int NORM, int BASIS, typename TC, typename TG>
__device__ __forceinline__ double pp_direct(const Math<double>& M, const LayerConst& lc, const TC* __restrict__ C,
                                            const TG* __restrict__ grid, double u, double& sc) {
    const double n = normalize<NORM, double>(M, lc.norm, u);
    const int basis = BASIS >= 0 ? BASIS : lc.basis;
    const double invh = (double)lc.invh;
    const int G = lc.G;
    double s = 0.0, a = 0.0;
#pragma unroll 1
    for (int j = 0; j < G; ++j) {
        double aux;
        const double y = (n - (double)grid[j]) * invh;
        const double t = (double)C[j] * basis_direct<double>(M, basis, y, aux);
        s = s + t;
        a = a + kabs(t);
    }
    if (lc.use_base) {
        const double t = (double)C[G] * swish<double>(M, u);
        s = s + t;
        a = a + kabs(t);
    }
    sc = a;
    return s;
}

// φ(u) from the LDS table; ok = false outside [lo, -lo) or in a rejected interval.
__device__ __forceinline__ double pp_eval(const double2* __restrict__ tl, int ni, double inv_w, double x0, double u,
                                          bool& ok) {
    const double x = ::fma(u, inv_w, x0);
    const bool in = (x >= 0.0) && (x < (double)ni);     // false for NaN
    const double xc = in ? x : 0.0;
    const double fl = __builtin_floor(xc);
    const int k = (int)fl;
    const double t = ::fma(2.0, xc - fl, -1.0);           // exact
    const double2* __restrict__ e = tl + k;
    const double2 c8 = e[4 * ni], c6 = e[3 * ni], c4 = e[2 * ni], c2 = e[ni], c0 = e[0];
    double y = ::fma(c8.y, t, c8.x);
    y = ::fma(y, t, c6.y);
    y = ::fma(y, t, c6.x);
    y = ::fma(y, t, c4.y);
    y = ::fma(y, t, c4.x);
    y = ::fma(y, t, c2.y);
    y = ::fma(y, t, c2.x);
    y = ::fma(y, t, c0.y);
    y = ::fma(y, t, c0.x);
    ok = in && (y == y);
    return y;
}

// ---------------------------------------------------------------------------
// VJP of the Fisher-KPP RHS (the pullback SciMLSensitivity requests per stage):
//   λᵀJ = (D lap)ᵀλ + λ ⊙ φ'(u)      lap symmetric; φ' = the rrule chain (utils.jl:15-21)
//   dC_j += Σ λ B_j(N(u)),  dW += Σ λ swish(u)
// φ'(u) and swish(u) come from the PP_DPHI / PP_SWISH tables (same interval index);
// the G basis values for dC from the Gaussian recurrence (kan_device.hpp), in the
// form g = λ·E0, dC_j += g·kc_j, g *= R.

// φ'(u) and swish(u) by the reference formulas (slow path: out of range / rejected).
template <int NORM, int BASIS>
__device__ __forceinline__ void pp_direct_dphi_sw(const Math<double>& M, const LayerConst& lc,
                                                  const double* __restrict__ p, double u, double& dphi,
                                                  double& sw) {
    const double n = normalize<NORM, double>(M, lc.norm, u);
    const int basis = BASIS >= 0 ? BASIS : lc.basis;
    const double invh = (double)lc.invh;
    const int G = lc.G;
    double s = 0.0;
#pragma unroll 1
    for (int j = 0; j < G; ++j) {
        double aux = 0.0;
        const double y = (n - (double)lc.grid[j]) * invh;
        const double phi = basis_direct<double>(M, basis, y, aux);
        s = s + basis_pull<double>(basis, lc.iqf_quirk, y, phi, aux, p[j]) * invh;
    }
    double dsw;
    swish_and_grad<double>(M, u, sw, dsw);
    dphi = dnormalize<NORM, double>(lc.norm, n) * s + (lc.use_base ? p[G] * dsw : 0.0);
}

#ifndef KAN_VJP_SPLIT_HORNER
#define KAN_VJP_SPLIT_HORNER 1
#endif
// Two tables sharing one interval index: φ'(u) from td, swish(u) from ts.  SPLITH: the two Horner
// chains run one after the other (a scheduling barrier between them) so only one table's five 16-byte
// LDS reads are live at a time (the adjoint-stage and adjoint-step kernels, where registers limit the
// occupancy); otherwise the compiler interleaves the two independent chains (the standalone VJP, round 4:
// 160 VGPRs, still 3 waves/SIMD; 1M trajectories 1539 -> 1481 us in one interleaved process,
// profiles/r04/ab/vjp_interleaved_horner_ab.txt; the adjoint rows step measured 58.1 -> 58.6 us with it).
template <bool SPLITH = (KAN_VJP_SPLIT_HORNER != 0)>
__device__ __forceinline__ bool pp_eval2(const double2* __restrict__ td, const double2* __restrict__ ts, int ni,
                                         double inv_w, double x0, double u, double& d, double& s) {
    // interval index without selects: v_cvt_i32_f64 saturates out-of-range values (and gives 0 for NaN,
    // whose t and so y are NaN: rejected below), so one unsigned compare is the range check, and the masked
    // index keeps the LDS reads in the table for the points the direct formula takes (ni: a power of two).
    // In range, k and t are those of the clamped form (the same bits).
    const double x = ::fma(u, inv_w, x0);
    const double fl = __builtin_floor(x);
    int ki;
    asm("v_cvt_i32_f64 %0, %1" : "=v"(ki) : "v"(fl));
    const bool in = (unsigned)ki < (unsigned)ni;
    const int k = ki & (ni - 1);
    const double t = ::fma(2.0, x - fl, -1.0);
    const double2* __restrict__ a = td + k;
    const double2* __restrict__ b = ts + k;
    double y, z;
    {
        const double2 a8 = a[4 * ni], a6 = a[3 * ni], a4 = a[2 * ni], a2 = a[ni], a0 = a[0];
        y = ::fma(a8.y, t, a8.x);
        y = ::fma(y, t, a6.y);
        y = ::fma(y, t, a6.x);
        y = ::fma(y, t, a4.y);
        y = ::fma(y, t, a4.x);
        y = ::fma(y, t, a2.y);
        y = ::fma(y, t, a2.x);
        y = ::fma(y, t, a0.y);
        y = ::fma(y, t, a0.x);
    }
    if constexpr (SPLITH) __builtin_amdgcn_sched_barrier(0);
    {
        const double2 b8 = b[4 * ni], b6 = b[3 * ni], b4 = b[2 * ni], b2 = b[ni], b0 = b[0];
        z = ::fma(b8.y, t, b8.x);
        z = ::fma(z, t, b6.y);
        z = ::fma(z, t, b6.x);
        z = ::fma(z, t, b4.y);
        z = ::fma(z, t, b4.x);
        z = ::fma(z, t, b2.y);
        z = ::fma(z, t, b2.x);
        z = ::fma(z, t, b0.y);
        z = ::fma(z, t, b0.x);
    }
    d = y;
    s = z;
    return in && (y == y) && (z == z);
}

// One point of the pullback: returns λ φ'(x); accumulates the dC moments and dW.
// With v_j = λ E0 R^j and the knot correction kc_j = K_j (1 + τ' e_j + τ'² e_j²/2):
//     Σ_points λ B_j = K_j (S0_j + e_j S1_j + e_j²/2 S2_j),
//     S0_j = Σ v_j,  S1_j = Σ v_j τ',  S2_j = Σ v_j τ'²
// so the loop over knots needs no per-knot constants (they would not fit in SGPRs
// next to the rest of the kernel).  S1/S2 carry weights |τ' e_j| <= 1.1e-6 and
// (τ' e_j)²/2 <= 6e-13 of S0 (G=10), so they run in fp32 on their own fp32 power
// chain: their rounding reaches dC at < 1e-13 relative.
template <int NORM, int PATH, int GT, bool SPLITH = (KAN_VJP_SPLIT_HORNER != 0)>
__device__ __forceinline__ double pp_vjp_point(const Math<double>& M, const LayerConst& lc,
                                               const double* __restrict__ p, const RecScalars<double>& rc,
                                               const double2* __restrict__ td, const double2* __restrict__ ts,
                                               int ni, double inv_w, double x0, double x, double l,
                                               double (&S0)[GT], float (&S1)[GT], float (&S2)[GT], double& dW,
                                               bool init = false) {
    // init: the moments and dW start at this point (the same bits as adding it to zeros; saves the
    // zeroing of 30 accumulator registers per stage in the adjoint step kernels)
    double dphi, sw;
    if (__builtin_expect(!pp_eval2<SPLITH>(td, ts, ni, inv_w, x0, x, dphi, sw), 0)) {
#ifdef KAN_CLOCK_PROBE   // (diagnostic build: points that take the direct formula, tools/vjp_drift.py --count)
        atomicAdd(&kan_clock_probe[7], 1ull);
#endif
        pp_direct_dphi_sw<NORM, BASIS_RBF>(M, lc, p, x, dphi, sw);
    }
    dW = init ? l * sw : ::fma(l, sw, dW);
    const double n = normalize<NORM, double>(M, lc.norm, x);
    double z0, E0, R, taup;
    rec_anchor<double>(M, rc, n, z0, E0, R, taup);
    double v = l * E0;
    float v32 = (float)v, R32 = (float)R;
    const float t32 = (float)taup, t2 = t32 * t32;
#if KAN_VJP_PACKED
    // fp32 correction moments two knots at a time: (v_j, v_j+1) advanced by R² with one packed
    // multiply (their weight in dC is <= 1.1e-6, so the fp32 rounding of R² does not show)
    typedef float kf2 __attribute__((ext_vector_type(2)));
    kf2 vp = {v32, v32 * R32};
    const float R2 = R32 * R32;
    const kf2 R2v = {R2, R2};
#endif
#pragma unroll
    for (int j = 0; j < GT; ++j) {
        S0[j] = init ? v : S0[j] + v;
        v = v * R;
        if constexpr (PATH == PATH_REC_CORR) {
#if KAN_VJP_PACKED
            const float vj = (j & 1) ? vp.y : vp.x;
            S1[j] = init ? vj * t32 : fmaf(vj, t32, S1[j]);
            S2[j] = init ? vj * t2 : fmaf(vj, t2, S2[j]);
            if (j & 1) vp = vp * R2v;
#else
            S1[j] = init ? v32 * t32 : fmaf(v32, t32, S1[j]);
            S2[j] = init ? v32 * t2 : fmaf(v32, t2, S2[j]);
            v32 = v32 * R32;
#endif
        }
    }
    return l * dphi;
}

}  // namespace kan
