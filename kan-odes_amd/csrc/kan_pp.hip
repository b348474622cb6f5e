// kan_pp.hip — Fisher-KPP RHS through a piecewise-polynomial form of the pointwise KAN (gfx950).
//
//   rc_kanode(u, p, t) = D*lap*u + kan1_.(u)       PDE examples/Fisher-KPP_Source.jl:95-98
//
// kan1 is a scalar function of u alone, φ(u) = Σ_j C_j B_j(N(u)) + W swish(u)
// (kdense.jl:116-124), fixed for the whole launch.  Instead of G basis functions
// per grid point (2 exp + Horner sweeps + swish ≈ 120 fp64 VALU per point), each
// launch first tabulates φ as a degree-9 polynomial on each interval of width w
// (interpolated at Chebyshev nodes from the direct formula, then accepted only if
// it matches the direct formula to tol·Σ|terms| at three check points), and the
// RHS kernel evaluates one Horner polynomial from LDS: ≈25 VALU per point, which
// leaves the kernel bound by HBM (one read of u, one write of du).
//
// Points outside the tabulated range, and points in an interval that failed its
// acceptance test (marked NaN), take the direct formula (pp_direct) — the exact
// reference arithmetic, register-light, rarely executed.
//
// Error: interpolation <= ~1e-16 of Σ|C_j| at w <= 0.16 h (host rule, kanode_abi.cpp);
// measured <= 1.3e-15 of the scale over 2M points, the fp64 rounding floor of the
// direct 11-term sum itself.
#include "kan_common.hpp"
#include "kan_kernels.hpp"
#include "kan_lap.hpp"
#include "kan_pp_point.hpp"
#include "kan_adjloop.hpp"
#include "kan_tsit5.hpp"

#include <cstdlib>


namespace kan {

// Diagnostic build only (-DKAN_CLOCK_PROBE, tools/build_var.sh; tools/clock_probe.py): thread 0 of every block of
// the adjoint rows step (slot 0) and the standalone VJP (slot 1) adds its lifetime in shader clocks (s_memtime) and
// in the 100 MHz reference clock (s_memrealtime); their ratio is the in-kernel clock (MI355X_MICROARCH.md, DVFS
// give-back item 6).  Vector atomics only.  Absent from the product build.
// Slots 2.. (same build): s_memrealtime phase sums of the device-controlled loops' kernels (tools/clock_probe.py
// --phases): the finish launch's last workgroup (reduce, arrive, decide, plan) and the forward DEV step's
// workgroups (decision, rows).
#ifdef KAN_CLOCK_PROBE
__device__ unsigned long long kan_clock_probe[32];
#define KAN_PROBE_T(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime();
#define KAN_PROBE_ADD(slot, val) atomicAdd(&kan_clock_probe[(slot)], (unsigned long long)(val));
#define KAN_PROBE_BEGIN                                                                                   \
    const unsigned long long kan_ck0_ = __builtin_amdgcn_s_memtime(), kan_rt0_ = __builtin_amdgcn_s_memrealtime();
#define KAN_PROBE_END(slot)                                                                               \
    if (threadIdx.x == 0) {                                                                               \
        const unsigned long long c1_ = __builtin_amdgcn_s_memtime(), r1_ = __builtin_amdgcn_s_memrealtime(); \
        atomicAdd(&kan_clock_probe[2 * (slot)], c1_ - kan_ck0_);                                          \
        atomicAdd(&kan_clock_probe[2 * (slot) + 1], r1_ - kan_rt0_);                                      \
    }
#else
#define KAN_PROBE_BEGIN
#define KAN_PROBE_END(slot)
#define KAN_PROBE_T(v)
#define KAN_PROBE_ADD(slot, val)
#endif

constexpr int kPPEvals = kPPCoef + kPPChecks;        // direct evaluations per interval

// One block builds kPPPerBlock intervals of one tabulated function (blockIdx.y
// picks it from `fns`): 13 direct evaluations per interval (10 nodes + 3 checks),
// node values -> monomial coefficients (Q, host-built), acceptance.
//   PP_PHI    φ(u)  = Σ_j C_j B_j(N(u)) + W swish(u)                 (kdense.jl:116-124)
//   PP_DPHI   φ'(u) = N'(u) Σ_j ∂B_j C_j / h + W swish'(u)  — the rrule chain of
//             utils.jl:15-21 and NNlib's Ω-form derivatives, i.e. x̄/λ of the pullback
//   PP_SWISH  swish(u)                                               (the dW weight)
// Each evaluation is split over a quad of lanes (terms j ≡ sub mod 4, combined in
// a fixed order) so the dependent chain is ~3 exponentials, not G+1: the build is
// latency-bound and sits between two dependent launches.
// Table layout per function: [kPPCoef/2][ni] pairs (a_2c, a_2c+1), so lanes at
// neighbouring intervals read neighbouring 16-byte LDS words.
struct PPFns {
    int fn[kPPMaxFns];
};

// Parameter stamp (pp_stamp): block b of function fn built its intervals from the parameters in its own stamp.
// When p matches it bit for bit the block skips its build.  Every block compares and rewrites only its own stamp,
// so there is no cross-block ordering to establish (round 5 and before: one stamp per function written by the
// last block to arrive on a counter, i.e. 64 serialised atomics per build).  The constants a build needs are
// loaded together with the stamp, so a build costs one memory round trip before its evaluations.
__global__ void __launch_bounds__(kBlock)
fk_pp_build_kernel(const LayerConst* __restrict__ lcp, const PPConst* __restrict__ pcp,
                   const double* __restrict__ p, double* __restrict__ tables, PPFns fns) {
    KAN_PROBE_T(pb0)
    __shared__ double sQ[kPPCoef * kPPCoef];
    __shared__ double sT[kPPEvals];              // nodes, then check points
    __shared__ double sC[kMaxGrid + 1];          // C_0..C_{G-1}, W
    __shared__ double sG[kMaxGrid];              // knots
    __shared__ double fv[kPPPerBlock][kPPEvals];
    __shared__ double sv[kPPPerBlock][kPPChecks];
    __shared__ double cf[kPPPerBlock][kPPCoef];
    __shared__ int bad[kPPPerBlock];
    __shared__ int same;
    const LayerConst& lc = *lcp;
    const PPConst& pc = *pcp;
    const int tid = threadIdx.x;
    const int G = lc.G;
    const int fn = fns.fn[blockIdx.y];
    double* __restrict__ stamp = pp_stamp(tables, pc.ni, fn, blockIdx.x);
    // every constant the build needs and the stamp comparison, in one round of loads
    if (tid < kPPCoef * kPPCoef) sQ[tid] = (&pc.Q[0][0])[tid];
    if (tid < kPPEvals) sT[tid] = tid < kPPCoef ? pc.xi[tid] : pc.tchk[tid - kPPCoef];
    if (tid <= G) sC[tid] = (tid < G || lc.use_base) ? p[tid] : 0.0;
    if (tid < G) sG[tid] = (double)lc.grid[tid];
    if (tid < kPPPerBlock) bad[tid] = 0;
    if (tid < kWave) {
        const int j = tid;
        const double pj = j <= G && (j < G || lc.use_base) ? p[j] : 0.0;
        const bool ne = j <= G && __double_as_longlong(stamp[j]) != __double_as_longlong(pj);
        const bool valid = stamp[kPPStampValid] == 1.0;
        const bool any_ne = __any(ne);
        if (j == 0) same = valid && !any_ne;
    }
    KAN_EXP_TABLE_LDS(tab);   // its __syncthreads publishes the constants and `same` too
    KAN_PROBE_T(pb1)
    if (same) return;          // (block-uniform)
    const Math<double> M{tab};
    double* __restrict__ table = tables + (int64_t)fn * kPPCoef * pc.ni;
    const int k0 = blockIdx.x * kPPPerBlock;
    {
        // evaluation e = tid / 4 (all lanes of a quad take part in the shuffles)
        const int e = tid >> 2, sub = tid & 3;
        const bool live = e < kPPPerBlock * kPPEvals;
        const int kl = live ? e / kPPEvals : 0, m = live ? e - kl * kPPEvals : 0;
        const double c = pc.lo + ((double)(k0 + kl) + 0.5) * pc.w;   // exact: w is a power of two
        const double u = ::fma(sT[m], 0.5 * pc.w, c);
        const double n = normalize<NORM_RUNTIME, double>(M, lc.norm, u);
        const double invh = (double)lc.invh;
        double s = 0.0, a = 0.0, base = 0.0;    // spline-part sum, Σ|spline terms|, base term
        if (fn != PP_SWISH) {
            for (int j = sub; j < G; j += 4) {
                double aux = 0.0;
                const double y = (n - sG[j]) * invh;
                const double phi = basis_direct<double>(M, lc.basis, y, aux);
                const double t = fn == PP_PHI ? sC[j] * phi
                                              : basis_pull<double>(lc.basis, lc.iqf_quirk, y, phi, aux, sC[j]) * invh;
                s = s + t;
                a = a + kabs(t);
            }
        }
        if (sub == 3) {
            double sw, dsw;
            swish_and_grad<double>(M, u, sw, dsw);
            base = fn == PP_SWISH ? sw : (lc.use_base ? sC[G] * (fn == PP_PHI ? sw : dsw) : 0.0);
        }
        s = s + __shfl_xor(s, 1, 4);
        a = a + __shfl_xor(a, 1, 4);
        s = s + __shfl_xor(s, 2, 4);
        a = a + __shfl_xor(a, 2, 4);
        base = __shfl(base, 3, 4);
        if (live && sub == 0) {
            // acceptance scale: Σ|terms| at the point, floored at 4·w·(the function's natural
            // magnitude: Σ|C| (/h) + |W|, or 1 + |u| for swish).  The node -> monomial
            // conversion rounds at ~|Q|·eps·(variation over the interval, ~w·|f'|), so
            // where every term vanishes (swish(0) = 0) the floor keeps a correct fit from
            // being rejected; it admits absolute errors <= 2.5e-15 of that magnitude.
            // (magnitudes by compare-and-negate: with the |x| source modifier the swish branch's scale came out
            // as base + 4w(1 + u), negative below u ≈ -0.2, which rejected every swish interval there and sent
            // those points of the VJP to the direct formula; tools/pp_direct_scan.py)
            auto mag = [](double x) { return x < 0.0 ? -x : x; };
            double csum = 0.0;
            for (int j = 0; j < G; ++j) csum += mag(sC[j]);
            const double wabs = lc.use_base ? mag(sC[G]) : 0.0;
            double v, sc, ref;
            if (fn == PP_PHI) {
                v = s + base;
                sc = a + mag(base);
                ref = csum + wabs;
            } else if (fn == PP_DPHI) {
                const double dn = dnormalize<NORM_RUNTIME, double>(lc.norm, n);
                v = dn * s + base;
                sc = dn * a + mag(base);
                ref = csum * invh + wabs;
            } else {
                v = base;
                sc = mag(base);
                ref = 1.0 + mag(u);
            }
            sc += 4.0 * pc.w * ref;
            fv[kl][m] = v;
            if (m >= kPPCoef) sv[kl][m - kPPCoef] = sc;
        }
    }
    __syncthreads();
    if (tid < kPPPerBlock * kPPCoef) {
        // a = Q (f - f_0) + f_0 e_0: the constant is carried exactly, Q only sees the variation
        const int kl = tid / kPPCoef, i = tid - kl * kPPCoef;
        const double f0 = fv[kl][0];
        double s = 0.0;
#pragma unroll
        for (int m = 0; m < kPPCoef; ++m) s = ::fma(sQ[i * kPPCoef + m], fv[kl][m] - f0, s);
        cf[kl][i] = i == 0 ? s + f0 : s;
    }
    __syncthreads();
    if (tid < kPPPerBlock * kPPChecks) {
        const int kl = tid / kPPChecks, c = tid - kl * kPPChecks;
        const double t = sT[kPPCoef + c];
        double y = cf[kl][kPPCoef - 1];
#pragma unroll
        for (int i = kPPCoef - 2; i >= 0; --i) y = ::fma(y, t, cf[kl][i]);
        if (!(kabs(y - fv[kl][kPPCoef + c]) <= pc.tol * sv[kl][c])) {
            bad[kl] = 1;
#ifdef KAN_CLOCK_PROBE   // (diagnostic build: rejected intervals per function and the worst residual / tolerance)
            atomicAdd(&kan_clock_probe[16 + fn], 1ull);
            const double r = kabs(y - fv[kl][kPPCoef + c]) / (pc.tol * sv[kl][c]);
            atomicMax(&kan_clock_probe[19], (unsigned long long)__double_as_longlong(r == r ? r : 1e300));
            atomicMax(&kan_clock_probe[20 + fn], (unsigned long long)(k0 + kl));
#endif
        }
    }
    __syncthreads();
    if (tid < kPPPerBlock * kPPCoef) {
        const int kl = tid / kPPCoef, i = tid - kl * kPPCoef;
        const int64_t k = k0 + kl;
        table[((int64_t)(i >> 1) * pc.ni + k) * 2 + (i & 1)] = bad[kl] ? __builtin_nan("") : cf[kl][i];
    }
    // this block's stamp (read only by this block of later launches; published to them by the kernel boundary)
    if (tid <= G) stamp[tid] = sC[tid];
    if (tid == 0) {
        stamp[kPPStampValid] = 1.0;
        int nbad = 0;
        for (int q = 0; q < kPPPerBlock; ++q) nbad += bad[q];
        stamp[kPPStampRejected] = (double)nbad;   // (kanode_table_rejections)
    }
    KAN_PROBE_T(pb2)
    if (tid == 0) {
        KAN_PROBE_ADD(12, pb1 - pb0)   // (diagnostic build) constants + stamp comparison
        KAN_PROBE_ADD(13, pb2 - pb1)   // the build
        KAN_PROBE_ADD(15, 1)
    }
}

// RHS of the point pair (i, i+1) of one trajectory row `ub` -> `db`.
template <int NORM, int BASIS>
__device__ __forceinline__ void pp_pair_finish(const Math<double>& M, const LayerConst& lc,
                                               const double* __restrict__ p, const double2* __restrict__ tl, int ni,
                                               double inv_w, double x0, double cd, double co, int Nx, int i,
                                               double2 v, double um, double up, double* __restrict__ db) {
    bool ok0, ok1;
    double k0 = pp_eval(tl, ni, inv_w, x0, v.x, ok0);
    double k1 = pp_eval(tl, ni, inv_w, x0, v.y, ok1);
#ifndef KAN_PP_NO_SLOW
    if (__builtin_expect(!(ok0 && ok1), 0)) {
        double sc;
        if (!ok0) k0 = pp_direct<NORM, BASIS>(M, lc, p, lc.grid, v.x, sc);
        if (!ok1) k1 = pp_direct<NORM, BASIS>(M, lc, p, lc.grid, v.y, sc);
    }
#endif
    double l0, l1;
    if (Nx >= 4) {
        lap_pair<double>(um, v.x, v.y, up, i, Nx, cd, co, l0, l1);
    } else {
        l0 = lap3<double>(um, v.x, v.y, i, Nx, cd, co);
        l1 = lap3<double>(v.x, v.y, up, i + 1, Nx, cd, co);
    }
    double2 o;
    o.x = l0 + k0;
    o.y = l1 + k1;
    *reinterpret_cast<double2*>(db + i) = o;
}

// Point pairs (Nx even): 2^tpt_log2 threads per trajectory, 256 >> tpt_log2
// trajectories per block, blocks grid-stride over trajectories.  SHORT (Nx/2 <=
// 256): one pair per thread per trajectory, two trajectories per iteration (both
// rows' loads issued before either is used).  Dynamic LDS: the table,
// [kPPCoef/2][ni] double2.
#ifndef KAN_PP_WPE
#define KAN_PP_WPE 1
#endif
#ifndef KAN_PP_UNR
#define KAN_PP_UNR 2
#endif
template <int NORM, int BASIS, bool SHORT>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KAN_PP_WPE)))
fk_rhs_pp_kernel(const LayerConst* __restrict__ lcp, const double* __restrict__ p,
                 const double2* __restrict__ table, int ni, double inv_w, double x0, double cd, double co, int Nx,
                 int tpt_log2, const double* __restrict__ u, double* __restrict__ du, int64_t B) {
    extern __shared__ double2 tl[];
    for (int i = threadIdx.x; i < (kPPCoef / 2) * ni; i += kBlock) tl[i] = table[i];   // (register copy: glds here cost occupancy)
    KAN_EXP_TABLE_LDS(tab);   // (its __syncthreads also publishes tl)
    const Math<double> M{tab};
    const LayerConst& lc = *lcp;
    const int tpt = 1 << tpt_log2;
    const int tpb = kBlock >> tpt_log2;
    const int lt = threadIdx.x & (tpt - 1);
    const int units = Nx >> 1;
    const int64_t b0 = (int64_t)blockIdx.x * tpb + (threadIdx.x >> tpt_log2);
    const int64_t bstride = (int64_t)gridDim.x * tpb;
    if constexpr (SHORT) {
        if (lt >= units) return;
        const int i = 2 * lt;
        const int im = i > 0 ? i - 1 : Nx - 1;
        const int ip = i + 2 < Nx ? i + 2 : 0;
        int64_t b = b0;
        for (; KAN_PP_UNR == 2 && b + bstride < B; b += 2 * bstride) {
            const double* __restrict__ ua = u + b * Nx;
            const double* __restrict__ uc = ua + bstride * Nx;
            const double2 va = *reinterpret_cast<const double2*>(ua + i);
            const double2 vc = *reinterpret_cast<const double2*>(uc + i);
            const double uma = ua[im], upa = ua[ip], umc = uc[im], upc = uc[ip];
            pp_pair_finish<NORM, BASIS>(M, lc, p, tl, ni, inv_w, x0, cd, co, Nx, i, va, uma, upa, du + b * Nx);
            pp_pair_finish<NORM, BASIS>(M, lc, p, tl, ni, inv_w, x0, cd, co, Nx, i, vc, umc, upc,
                                        du + (b + bstride) * Nx);
        }
        for (; b < B; b += bstride) {
            const double* __restrict__ ua = u + b * Nx;
            pp_pair_finish<NORM, BASIS>(M, lc, p, tl, ni, inv_w, x0, cd, co, Nx, i,
                                        *reinterpret_cast<const double2*>(ua + i), ua[im], ua[ip], du + b * Nx);
        }
        return;
    }
    for (int64_t b = b0; b < B; b += bstride) {
        const double* __restrict__ ub = u + b * Nx;
        for (int q = lt; q < units; q += tpt) {
            const int i = 2 * q;
            pp_pair_finish<NORM, BASIS>(M, lc, p, tl, ni, inv_w, x0, cd, co, Nx, i,
                                        *reinterpret_cast<const double2*>(ub + i), ub[i > 0 ? i - 1 : Nx - 1],
                                        ub[i + 2 < Nx ? i + 2 : 0], du + b * Nx);
        }
    }
}

// Whole-wave rotations (DPP wave_ror:1 / wave_rol:1, GFX9 family): lane i receives
// lane (i-1) mod 64 / (i+1) mod 64.  Two 32-bit moves per double, no LDS.
__device__ __forceinline__ double wave_ror1(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x13C, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x13C, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_rol1(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x134, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x134, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

typedef double kd2 __attribute__((ext_vector_type(2)));

// (D*lap)*λ at the 2·NP consecutive points a lane holds (pair k = v[k].x, v[k].y; the wave's lanes hold
// the row in order): lap3's ascending-column orders, no FMA contraction.  co·v is formed once per point and
// shared by both neighbours' rows (the same product bits as lap_pair's), the two cross-lane neighbours
// arrive by one wave rotation each (lane 0's left neighbour is lane 63's last point: the periodic wrap),
// and only the row's first (lane 0) and last (lane 63) points take their boundary orders.
template <int NP>
__device__ __forceinline__ void lap_lane(const kd2 (&v)[NP], int lane, double cd, double co, double (&r)[2 * NP]) {
#pragma clang fp contract(off)
    constexpr int L = 2 * NP;
    double cu[L], du[L];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        cu[2 * k] = co * v[k].x;
        cu[2 * k + 1] = co * v[k].y;
        du[2 * k] = cd * v[k].x;
        du[2 * k + 1] = cd * v[k].y;
    }
    const double cl = wave_ror1(cu[L - 1]), cr = wave_rol1(cu[0]);
#pragma unroll
    for (int m = 0; m < L; ++m) r[m] = ((m == 0 ? cl : cu[m - 1]) + du[m]) + (m == L - 1 ? cr : cu[m + 1]);
    const double first = (du[0] + cu[1]) + cl;            // row 0: (cd·u0 + co·up) + co·um
    const double last = (cr + cu[L - 2]) + du[L - 1];     // row Nx-1: (co·up + co·um) + cd·u0
    r[0] = lane == 0 ? first : r[0];
    r[L - 1] = lane == kWave - 1 ? last : r[L - 1];
}

#ifndef KAN_PP_NT
#define KAN_PP_NT 1
#endif
#ifndef KAN_PP_ROWS
#define KAN_PP_ROWS 1
#endif
#ifndef KAN_PP_COLD_GLOBAL_EXP
#define KAN_PP_COLD_GLOBAL_EXP 1
#endif
__device__ __forceinline__ kd2 ld_stream(const double* p) {
#if KAN_PP_NT
    return __builtin_nontemporal_load(reinterpret_cast<const kd2*>(p));
#else
    return *reinterpret_cast<const kd2*>(p);
#endif
}

// Adjoint step kernel: u_i, λ, Q_m and kλ_j are re-read by later stages of the same launch.
// They are read and written with the default cache policy, so the re-reads can hit in L2
// (KAN_VSTEP_KEEP=0: nontemporal, as the streaming kernels; FK256 epoch at 4096 trajectories
// 7.6 -> 6.6 ms, profiles/r01/epoch/vstep_keep_ab.txt)
#ifndef KAN_VSTEP_KEEP
#define KAN_VSTEP_KEEP 1
#endif
__device__ __forceinline__ kd2 ld_vstep(const double* p) {
#if KAN_VSTEP_KEEP
    return *reinterpret_cast<const kd2*>(p);
#else
    return ld_stream(p);
#endif
}

// a[k] += Σ_{j<N} (sc·c_j)·K_j[k], e[k] += Σ_{j<N} (sc·ec_j)·K_j[k] (E) over the NP pairs of one
// row at offset off: all N·NP loads are issued before the first FMA.  (An unrolled loop over
// j < kMaxStages guarded by j < nk compiles to one branch per array, and the loads, which
// cannot move above their guard, then wait one after the other.)
template <int N, int NP, bool E>
__device__ __forceinline__ void stage_sum_n(const StageArgs<double>& sa, int64_t off, double sc, kd2 (&a)[NP],
                                            kd2 (&e)[NP]) {
    kd2 v[N][NP];
#pragma unroll
    for (int j = 0; j < N; ++j)
#pragma unroll
        for (int k = 0; k < NP; ++k) v[j][k] = ld_stream(sa.k[j] + off + 128 * k);
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const double cj = sa.c[j] * sc;
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            a[k].x = ::fma(cj, v[j][k].x, a[k].x);
            a[k].y = ::fma(cj, v[j][k].y, a[k].y);
        }
        if constexpr (E) {
            const double ej = sa.ec[j] * sc;
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                e[k].x = ::fma(ej, v[j][k].x, e[k].x);
                e[k].y = ::fma(ej, v[j][k].y, e[k].y);
            }
        }
    }
}
template <int NP, bool E>
__device__ __forceinline__ void stage_sum(const StageArgs<double>& sa, int64_t off, double sc, kd2 (&a)[NP],
                                          kd2 (&e)[NP]) {
    switch (sa.nk) {
    case 1: stage_sum_n<1, NP, E>(sa, off, sc, a, e); break;
    case 2: stage_sum_n<2, NP, E>(sa, off, sc, a, e); break;
    case 3: stage_sum_n<3, NP, E>(sa, off, sc, a, e); break;
    case 4: stage_sum_n<4, NP, E>(sa, off, sc, a, e); break;
    case 5: stage_sum_n<5, NP, E>(sa, off, sc, a, e); break;
    case 6: stage_sum_n<6, NP, E>(sa, off, sc, a, e); break;
    case 7: stage_sum_n<7, NP, E>(sa, off, sc, a, e); break;
    case 8: stage_sum_n<8, NP, E>(sa, off, sc, a, e); break;
    default: break;
    }
}
static_assert(kMaxStages == 8, "stage_sum covers nk <= 8");
__device__ __forceinline__ void st_stream(double* p, kd2 v) {
#if KAN_PP_NT
    __builtin_nontemporal_store(v, reinterpret_cast<kd2*>(p));
#else
    *reinterpret_cast<kd2*>(p) = v;
#endif
}
__device__ __forceinline__ void st_vstep(double* p, kd2 v) {   // see ld_vstep
#if KAN_VSTEP_KEEP
    *reinterpret_cast<kd2*>(p) = v;
#else
    st_stream(p, v);
#endif
}
// Forward step kernel: u_new and k_7 are read by the next step (KAN_FSTEP_KEEP=1: default
// cache policy for those loads and stores; measured no faster, profiles/r01/epoch/fstep_keep_ab.txt)
#ifndef KAN_FSTEP_KEEP
#define KAN_FSTEP_KEEP 0
#endif
__device__ __forceinline__ kd2 ld_fstep(const double* p) {
#if KAN_FSTEP_KEEP
    return *reinterpret_cast<const kd2*>(p);
#else
    return ld_stream(p);
#endif
}
__device__ __forceinline__ void st_fstep(double* p, kd2 v) {
#if KAN_FSTEP_KEEP
    *reinterpret_cast<kd2*>(p) = v;
#else
    st_stream(p, v);
#endif
}

// Nx = 128·NP: one wave per trajectory row.  Lane l holds the pairs (128k + 2l,
// 128k + 2l + 1), k < NP, each a fully coalesced 1 KB wave load; the stencil
// neighbours u[128k + 2l - 1] and u[128k + 2l + 2] are the neighbouring lanes'
// values (wave rotations), the periodic wrap included: u is read from HBM once, by
// streaming (nontemporal) loads, and du written once by streaming stores.
// Row mapping (chunk = rows per wave): chunk > 0 gives block k the contiguous rows
// [k·4·chunk, (k+1)·4·chunk), wave j taking rows j, j+4, ... of it, and the grid covers the batch
// (ceil(B / (4 chunk)) blocks, dispatched as the hardware frees slots); chunk = 0 is the persistent
// grid-stride form.  At 1M trajectories the contiguous chunks stream faster than a persistent grid
// (the table staging is amortised over 4·chunk rows; profiles/r02/ab/).
#ifndef KAN_PP_RHS_BS
#define KAN_PP_RHS_BS 256
#endif
constexpr int kRhsBlock = KAN_PP_RHS_BS;   // threads per block of the table RHS kernel
template <int NORM, int BASIS, int NP>
__global__ void __launch_bounds__(kRhsBlock) __attribute__((amdgpu_waves_per_eu(KAN_PP_WPE)))
fk_rhs_pp_wave_kernel(const LayerConst* __restrict__ lcp, const double* __restrict__ p,
                      const double2* __restrict__ table, int ni, double inv_w, double x0, double cd, double co,
                      const double* __restrict__ u, double* __restrict__ du, int64_t B, int chunk) {
    constexpr int Nx = 128 * NP;
    extern __shared__ double2 tl[];
    constexpr int R = KAN_PP_ROWS;   // rows per wave per pipeline step
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t rstride = chunk > 0 ? (int64_t)(kRhsBlock / kWave) : (int64_t)gridDim.x * (kRhsBlock / kWave);
    int64_t b = (int64_t)blockIdx.x * (kRhsBlock / kWave) * (chunk > 0 ? chunk : 1) + (threadIdx.x >> 6);
    if (chunk > 0) {
        const int64_t end = ((int64_t)blockIdx.x + 1) * (kRhsBlock / kWave) * chunk;
        B = end < B ? end : B;
    }
    // the first rows' loads are in flight while the block stages its table
    kd2 v[R][NP];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t br = b + r * rstride;
        if (br < B) {
#pragma unroll
            for (int k = 0; k < NP; ++k) v[r][k] = ld_stream(u + br * Nx + 128 * k + 2 * lane);
        }
    }
    for (int i = threadIdx.x; i < (kPPCoef / 2) * ni; i += kRhsBlock) tl[i] = table[i];   // (direct-to-LDS: 0.8 % slower here)
#if KAN_PP_COLD_GLOBAL_EXP
    // only the cold direct-formula branch takes exponentials: it reads the 2 KB 2^(j/256) table from
    // global memory instead of every block staging it in LDS
    __syncthreads();
    const Math<double> M{kExp2Tab256};
#else
    KAN_EXP_TABLE_LDS(tab);   // (its __syncthreads also publishes tl)
    const Math<double> M{tab};
#endif
    const LayerConst& lc = *lcp;
    for (; b < B; b += R * rstride) {
        // software pipeline: the next R rows' loads are issued before these rows' math
        kd2 vn[R][NP];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t bn = b + (R + r) * rstride;
            if (bn < B) {
#pragma unroll
                for (int k = 0; k < NP; ++k) vn[r][k] = ld_stream(u + bn * Nx + 128 * k + 2 * lane);
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t br = b + r * rstride;
            if (R > 1 && br >= B) break;
            double* __restrict__ db = du + br * Nx;
            double rr[NP], rl[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                rr[k] = wave_ror1(v[r][k].y);
                rl[k] = wave_rol1(v[r][k].x);
            }
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                const double um = lane == 0 ? rr[(k + NP - 1) % NP] : rr[k];
                const double up = lane == kWave - 1 ? rl[(k + 1) % NP] : rl[k];
                const int i = 128 * k + 2 * lane;
                bool ok0, ok1;
                double k0 = pp_eval(tl, ni, inv_w, x0, v[r][k].x, ok0);
                double k1 = pp_eval(tl, ni, inv_w, x0, v[r][k].y, ok1);
                if (__builtin_expect(!(ok0 && ok1), 0)) {
                    double sc;
                    if (!ok0) k0 = pp_direct<NORM, BASIS>(M, lc, p, lc.grid, v[r][k].x, sc);
                    if (!ok1) k1 = pp_direct<NORM, BASIS>(M, lc, p, lc.grid, v[r][k].y, sc);
                }
                double l0, l1;
                lap_pair<double>(um, v[r][k].x, v[r][k].y, up, i, Nx, cd, co, l0, l1);
                kd2 o;
                o.x = l0 + k0;
                o.y = l1 + k1;
                st_stream(db + i, o);
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int k = 0; k < NP; ++k) v[r][k] = vn[r][k];
    }
}

// Block size of the VJP kernels: LDS (two 20 KB tables + the exp table, 42 KB) allows 3 blocks
// per CU and the registers (~140 VGPRs) 3 waves/SIMD, so 256-thread blocks fill both.  Measured
// (tools/ab_rhs.py --op vjp, 1M trajectories): 256/3 waves 1639 us; 512-thread blocks at 3 or 4
// waves/SIMD (the latter spilling) 1740-1746 us.
#ifndef KAN_VJP_BLOCK
#define KAN_VJP_BLOCK 256
#endif
#ifndef KAN_VJP_UNROLL_PAIRS
#define KAN_VJP_UNROLL_PAIRS 1
#endif
#ifndef KAN_VJP_WPE
#define KAN_VJP_WPE 3
#endif
#ifndef KAN_VJP_STG_WPE
#define KAN_VJP_STG_WPE 3
#endif

constexpr int kVjpBlock = KAN_VJP_BLOCK;
#ifndef KAN_VJP_CHUNK
#define KAN_VJP_CHUNK 8
#endif
constexpr int kVjpChunk = KAN_VJP_CHUNK;   // rows per wave of the standalone table VJP (0 = persistent grid)
// Nx = 128·NP, one wave per trajectory row (as fk_rhs_pp_wave_kernel): u and λ by
// nontemporal 16-B loads, λ's stencil neighbours by wave rotation, λᵀJ by
// nontemporal stores; per-thread dC/dW registers, block-summed into the slab row
// of this block (ordered: bitwise reproducible for a given grid).  Dynamic LDS:
// the PP_DPHI and PP_SWISH tables, [2][kPPCoef/2][ni] double2.
// STG (kanode_vjp_stage, the adjoint stage): the forward dense output y = u + Σ su.c_j su.k_j
// and the adjoint stage input λs = lam + Σ sl.c_j sl.k_j are formed in registers (λs written
// to lam_out when non-null); with err_slab the λ error Σ (e/sk)², e = Σ sl.ec_j sl.k_j +
// sl.ec_nk λᵀJ, sk = abstol + reltol·max(|lam|,|λs|), is block-summed into err_slab[block].
// NI > 0: the table's interval count as a compile-time constant, so the LDS row offsets of the
// Horner coefficients are instruction immediates instead of per-point address adds (with the
// unrolled pairs: 1M trajectories 1557 -> 1460 us); 0: runtime ni.
template <int NORM, int PATH, int GT, int NP, bool STG, int NI>
__global__ void __launch_bounds__(kVjpBlock) __attribute__((amdgpu_waves_per_eu(STG ? KAN_VJP_STG_WPE : KAN_VJP_WPE)))
fk_vjp_pp_wave_kernel(const LayerConst* __restrict__ lcp, const double* __restrict__ p,
                      const double2* __restrict__ tables, int ni_rt, double inv_w, double x0, double cd, double co,
                      const double* __restrict__ u, const double* __restrict__ lam, double* __restrict__ lamJ,
                      double* __restrict__ slab, int64_t B, StageArgs<double> su, StageArgs<double> sl,
                      double* __restrict__ lam_out, double* __restrict__ err_slab, int chunk) {
    constexpr int Nx = 128 * NP;
    const int ni = NI > 0 ? NI : ni_rt;
    extern __shared__ double2 tl[];
    __shared__ double red[(kVjpBlock / kWave) * (GT + 1)];
    if (STG && stage_skip(sl.skip)) return;
    KAN_PROBE_BEGIN
    const int tsz = (kPPCoef / 2) * ni;   // double2 per table
    if constexpr (STG) {   // (the stage form keeps the register copy: the direct-to-LDS loads cost it scratch)
        for (int i = threadIdx.x; i < tsz; i += kVjpBlock) {
            tl[i] = tables[PP_DPHI * tsz + i];
            tl[tsz + i] = tables[PP_SWISH * tsz + i];
        }
    } else {
        lds_copy16(tl, tables + PP_DPHI * tsz, tsz);
        lds_copy16(tl + tsz, tables + PP_SWISH * tsz, tsz);
    }
    KAN_EXP_TABLE_LDS(tab);   // (its __syncthreads also publishes tl)
    const Math<double> M{tab};
    const double2* __restrict__ td = tl;
    const double2* __restrict__ ts = tl + tsz;
    const LayerConst& lc = *lcp;
    const RecScalars<double> rc(lc);
    double S0[GT];
    float S1[GT], S2[GT];
#pragma unroll
    for (int j = 0; j < GT; ++j) {
        S0[j] = 0.0;
        S1[j] = S2[j] = 0.0f;
    }
    double dW = 0.0;
    const bool want_err = STG && err_slab != nullptr;
    const double suc = STG ? stage_scale(su.cscale) : 1.0, slc = STG ? stage_scale(sl.cscale) : 1.0;
    double eacc = 0.0;
    const int lane = threadIdx.x & (kWave - 1);
    // row mapping as fk_rhs_pp_wave_kernel: chunk > 0 = contiguous rows per block (grid covers B)
    const int64_t rstride = chunk > 0 ? (int64_t)(kVjpBlock / kWave) : (int64_t)gridDim.x * (kVjpBlock / kWave);
    if (chunk > 0) {
        const int64_t end = ((int64_t)blockIdx.x + 1) * (kVjpBlock / kWave) * chunk;
        B = end < B ? end : B;
    }
    for (int64_t b = (int64_t)blockIdx.x * (kVjpBlock / kWave) * (chunk > 0 ? chunk : 1) + (threadIdx.x >> 6); b < B;
         b += rstride) {
        const int64_t rb = b * Nx + 2 * lane;
        kd2 uv[NP], lv[NP], l0[NP], ev[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            uv[k] = ld_stream(u + rb + 128 * k);
            lv[k] = ld_stream(lam + rb + 128 * k);
        }
        if constexpr (STG) {
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                l0[k] = lv[k];
                ev[k] = kd2{0.0, 0.0};
            }
            // Σ c_j k_j with the kernel-argument coefficients as the scalar operands, scaled
            // once at the end (device step control: c_j·dt): premultiplied coefficients
            // would occupy VGPRs for the whole kernel and push it into scratch
            kd2 ta[NP], te[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) ta[k] = kd2{0.0, 0.0};
            stage_sum<NP, false>(su, rb, 1.0, ta, te);
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                uv[k].x = ::fma(suc, ta[k].x, uv[k].x);
                uv[k].y = ::fma(suc, ta[k].y, uv[k].y);
                ta[k] = kd2{0.0, 0.0};
                te[k] = kd2{0.0, 0.0};
            }
            if (want_err) stage_sum<NP, true>(sl, rb, 1.0, ta, te);
            else stage_sum<NP, false>(sl, rb, 1.0, ta, te);
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                lv[k].x = ::fma(slc, ta[k].x, lv[k].x);
                lv[k].y = ::fma(slc, ta[k].y, lv[k].y);
                ev[k].x = slc * te[k].x;
                ev[k].y = slc * te[k].y;
            }
            if (lam_out) {
#pragma unroll
                for (int k = 0; k < NP; ++k) st_stream(lam_out + rb + 128 * k, lv[k]);
            }
        }
        double rr[NP], rl[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            rr[k] = wave_ror1(lv[k].y);
            rl[k] = wave_rol1(lv[k].x);
        }
        double la[NP][2];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            const double lm = lane == 0 ? rr[(k + NP - 1) % NP] : rr[k];
            const double lp = lane == kWave - 1 ? rl[(k + 1) % NP] : rl[k];
            lap_pair<double>(lm, lv[k].x, lv[k].y, lp, 128 * k + 2 * lane, Nx, cd, co, la[k][0], la[k][1]);
        }
        // the row's pairs of the standalone VJP (NP <= 2): unrolled, with a scheduling barrier between
        // them so only one pair's table reads and exponentials are live next to the 40 accumulator
        // VGPRs (1M trajectories 1557 -> 1460 us, profiles/r02/ab/vjp_unroll_ab.txt).  Elsewhere a real
        // loop selecting the pair's registers (unrolled, the stage and NP = 4 forms spill).
        constexpr int kPairUnroll = (KAN_VJP_UNROLL_PAIRS && !STG && NP <= 2) ? NP : 1;
#pragma unroll kPairUnroll
        for (int k = 0; k < NP; ++k) {
            kd2 uk = uv[0], lk = lv[0], l0k = l0[0], ek = ev[0];
            double a0 = la[0][0], a1 = la[0][1];
#pragma unroll
            for (int q = 1; q < NP; ++q) {
                if (k == q) {
                    uk = uv[q];
                    lk = lv[q];
                    a0 = la[q][0];
                    a1 = la[q][1];
                    if constexpr (STG) {
                        l0k = l0[q];
                        ek = ev[q];
                    }
                }
            }
            if constexpr (kPairUnroll > 1) __builtin_amdgcn_sched_barrier(0);
            const double x0b = pp_vjp_point<NORM, PATH, GT, STG>(M, lc, p, rc, td, ts, ni, inv_w, x0, uk.x, lk.x, S0, S1,
                                                           S2, dW);
            __builtin_amdgcn_sched_barrier(0);
            const double x1b = pp_vjp_point<NORM, PATH, GT, STG>(M, lc, p, rc, td, ts, ni, inv_w, x0, uk.y, lk.y, S0, S1,
                                                           S2, dW);
            kd2 o;
            o.x = a0 + x0b;
            o.y = a1 + x1b;
            st_stream(lamJ + rb + 128 * k, o);
            if (want_err) {
                const double en = stage_ec_last(sl) * slc;
                const double ex = ::fma(en, o.x, ek.x), ey = ::fma(en, o.y, ek.y);
                const double sx = ::fma(sl.reltol, fmax(kabs(l0k.x), kabs(lk.x)), sl.abstol);
                const double sy = ::fma(sl.reltol, fmax(kabs(l0k.y), kabs(lk.y)), sl.abstol);
                const double rx = ex / sx, ry = ey / sy;
                eacc = ::fma(rx, rx, eacc);
                eacc = ::fma(ry, ry, eacc);
            }
        }
    }
    const int P = GT + (lc.use_base ? 1 : 0);
    double acc[GT + 1];
#pragma unroll
    for (int j = 0; j < GT; ++j) {
        const double e = lc.e[j];
        acc[j] = PATH == PATH_REC_CORR ? lc.K[j] * ::fma(lc.h2[j], (double)S2[j], ::fma(e, (double)S1[j], S0[j]))
                                       : lc.K[j] * S0[j];
    }
    acc[GT] = dW;
    block_sum_to<double, GT + 1>(acc, P, red, slab + (int64_t)blockIdx.x * P);
    if (want_err) {
        __syncthreads();   // red is reused
        const double v[1] = {eacc};
        block_sum_to<double, 1>(v, 1, red, err_slab + blockIdx.x);
    }
    KAN_PROBE_END(1)
}

// The six stages of one InterpolatingAdjoint step in ONE launch (Fisher-KPP table path, dense
// output in Q form): the stage loop runs inside the kernel and every wave keeps its rows across
// the stages (row b -> the same wave in every stage), so stage s+1 reads the kλ_{s+1} values its
// own wave wrote in stage s and no grid barrier is needed.  Per stage the same arithmetic as
// fk_vjp_pp_wave_kernel<…, STG>: u(t_s) = u_i + Σ_m θ^m Q_m, λs = λ + Σ_{j<=s} h a_sj kλ_j, the
// pullback, the moments block-summed into that stage's slab rows; stage 6 also writes λs (the
// new λ) and the λ error partials.  The tables are staged and the kernel launched once per step
// instead of once per stage.
template <int NORM, int PATH, int GT, int NP>
__global__ void __launch_bounds__(kVjpBlock) __attribute__((amdgpu_waves_per_eu(KAN_VJP_STG_WPE)))
fk_vjp_step_pp_wave_kernel(const LayerConst* __restrict__ lcp, const double* __restrict__ p,
                           const double2* __restrict__ tables, int ni, double inv_w, double x0, double cd, double co,
                           int64_t B, AdjStepArgs a) {
    constexpr int Nx = 128 * NP;
    extern __shared__ double2 tl[];
    __shared__ double red[(kVjpBlock / kWave) * (GT + 1)];
    const int tsz = (kPPCoef / 2) * ni;
    for (int i = threadIdx.x; i < tsz; i += kVjpBlock) {   // (register copy: direct-to-LDS loads cost scratch here)
        tl[i] = tables[PP_DPHI * tsz + i];
        tl[tsz + i] = tables[PP_SWISH * tsz + i];
    }
    KAN_EXP_TABLE_LDS(tab);
    const Math<double> M{tab};
    const double2* __restrict__ td = tl;
    const double2* __restrict__ ts = tl + tsz;
    const LayerConst& lc = *lcp;
    const RecScalars<double> rc(lc);
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t rstride = (int64_t)gridDim.x * (kVjpBlock / kWave);
    const int P = GT + (lc.use_base ? 1 : 0);
    double eacc = 0.0;
#ifndef KAN_VSTEP_UNROLL
#define KAN_VSTEP_UNROLL 6   // unrolled: static stage offsets and coefficients (132 -> 32 B/lane scratch, epoch -12%)
#endif
#pragma unroll KAN_VSTEP_UNROLL
    for (int s = 0; s < 6; ++s) {
        double S0[GT];
        float S1[GT], S2[GT];
#pragma unroll
        for (int j = 0; j < GT; ++j) {
            S0[j] = 0.0;
            S1[j] = S2[j] = 0.0f;
        }
        double dW = 0.0;
        const bool last = s == 5;
        const bool want_err = last && a.err_slab != nullptr;
        const double* __restrict__ uu = a.su_u[s];
        for (int64_t b = (int64_t)blockIdx.x * (kVjpBlock / kWave) + (threadIdx.x >> 6); b < B; b += rstride) {
            const int64_t rb = b * Nx + 2 * lane;
            kd2 uv[NP], lv[NP], l0[NP], ev[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                uv[k] = ld_vstep(uu + rb + 128 * k);
                lv[k] = ld_vstep(a.lam + rb + 128 * k);
                l0[k] = lv[k];
            }
            {   // u(t_s) = u_i + Σ_m θ^m Q_m (stage_sum order: Σ first, then added)
                kd2 q[4][NP];
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int k = 0; k < NP; ++k) q[m][k] = ld_vstep(a.su_q[s][m] + rb + 128 * k);
#pragma unroll
                for (int k = 0; k < NP; ++k) {
                    kd2 t{0.0, 0.0};
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        t.x = ::fma(a.su_c[s][m], q[m][k].x, t.x);
                        t.y = ::fma(a.su_c[s][m], q[m][k].y, t.y);
                    }
                    uv[k].x = ::fma(1.0, t.x, uv[k].x);
                    uv[k].y = ::fma(1.0, t.y, uv[k].y);
                }
            }
            {   // λs = λ + Σ_{j<=s} h a_sj kλ_j (and the error sum at the last stage)
                kd2 t[NP], e[NP];
#pragma unroll
                for (int k = 0; k < NP; ++k) {
                    t[k] = kd2{0.0, 0.0};
                    e[k] = kd2{0.0, 0.0};
                }
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    if (j <= s) {
                        const double c = a.a[s][j], ce = a.ec[j];
#pragma unroll
                        for (int k = 0; k < NP; ++k) {
                            const kd2 kj = ld_vstep(a.kl[j] + rb + 128 * k);
                            t[k].x = ::fma(c, kj.x, t[k].x);
                            t[k].y = ::fma(c, kj.y, t[k].y);
                            if (want_err) {
                                e[k].x = ::fma(ce, kj.x, e[k].x);
                                e[k].y = ::fma(ce, kj.y, e[k].y);
                            }
                        }
                    }
                }
#pragma unroll
                for (int k = 0; k < NP; ++k) {
                    lv[k].x = ::fma(1.0, t[k].x, lv[k].x);
                    lv[k].y = ::fma(1.0, t[k].y, lv[k].y);
                    ev[k] = e[k];
                }
            }
            if (last && a.lam_out) {   // (read by the next adjoint step)
#pragma unroll
                for (int k = 0; k < NP; ++k) st_vstep(a.lam_out + rb + 128 * k, lv[k]);
            }
            double rr[NP], rl[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                rr[k] = wave_ror1(lv[k].y);
                rl[k] = wave_rol1(lv[k].x);
            }
            double la[NP][2];
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                const double lm = lane == 0 ? rr[(k + NP - 1) % NP] : rr[k];
                const double lp = lane == kWave - 1 ? rl[(k + 1) % NP] : rl[k];
                lap_pair<double>(lm, lv[k].x, lv[k].y, lp, 128 * k + 2 * lane, Nx, cd, co, la[k][0], la[k][1]);
            }
            double* __restrict__ out = a.kl[s + 1];
#pragma unroll 1
            for (int k = 0; k < NP; ++k) {
                kd2 uk = uv[0], lk = lv[0], l0k = l0[0], ek = ev[0];
                double a0 = la[0][0], a1 = la[0][1];
#pragma unroll
                for (int q = 1; q < NP; ++q) {
                    if (k == q) {
                        uk = uv[q];
                        lk = lv[q];
                        a0 = la[q][0];
                        a1 = la[q][1];
                        l0k = l0[q];
                        ek = ev[q];
                    }
                }
                const double x0b = pp_vjp_point<NORM, PATH, GT>(M, lc, p, rc, td, ts, ni, inv_w, x0, uk.x, lk.x, S0,
                                                               S1, S2, dW);
                __builtin_amdgcn_sched_barrier(0);
                const double x1b = pp_vjp_point<NORM, PATH, GT>(M, lc, p, rc, td, ts, ni, inv_w, x0, uk.y, lk.y, S0,
                                                               S1, S2, dW);
                kd2 o;
                o.x = a0 + x0b;
                o.y = a1 + x1b;
                st_vstep(out + rb + 128 * k, o);
                if (want_err) {
                    const double en = a.ec[6];
                    const double ex = ::fma(en, o.x, ek.x), ey = ::fma(en, o.y, ek.y);
                    const double sx = ::fma(a.reltol, fmax(kabs(l0k.x), kabs(lk.x)), a.abstol);
                    const double sy = ::fma(a.reltol, fmax(kabs(l0k.y), kabs(lk.y)), a.abstol);
                    const double rx = ex / sx, ry = ey / sy;
                    eacc = ::fma(rx, rx, eacc);
                    eacc = ::fma(ry, ry, eacc);
                }
            }
        }
        double acc[GT + 1];
#pragma unroll
        for (int j = 0; j < GT; ++j) {
            const double e = lc.e[j];
            acc[j] = PATH == PATH_REC_CORR ? lc.K[j] * ::fma(lc.h2[j], (double)S2[j], ::fma(e, (double)S1[j], S0[j]))
                                           : lc.K[j] * S0[j];
        }
        acc[GT] = dW;
        block_sum_to<double, GT + 1>(acc, P, red, a.slab[s] + (int64_t)blockIdx.x * P);
        // kλ_{s+1} written by this wave is read back by it in the next stage: a workgroup-scope
        // release/acquire (wait for the stores, invalidate the CU's L1) suffices, the rows never
        // change wave; an agent-scope __threadfence would write back the whole L2 every stage
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();   // (red is reused)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    if (a.err_slab) {
        const double v[1] = {eacc};
        block_sum_to<double, 1>(v, 1, red, a.err_slab + blockIdx.x);
    }
}

// The same adjoint step with one trajectory row per wave and the row's stage values in registers
// (batches up to 4 rows x the slab's blocks; fk_vjp_step_pp_wave_kernel beyond).  The wave keeps
// λ, kλ_1..kλ_6 and the dense-output arrays u_i, Q_1..Q_4 of its row across the six stages, so a
// step reads λ, kλ_1 and the dense output once (again only when a stage falls in another forward
// step: a.reload) and writes λ_new and kλ_7: 7 to 12 state passes per step instead of ~58.  The
// per-point arithmetic is fk_vjp_step_pp_wave_kernel's, statement for statement (λᵀJ, λ_new and
// kλ_7 bitwise equal); the moment partials are block-summed per stage into the same slab rows
// (the grid differs, so dp differs from that kernel in the last bits of the reduction order).
#ifndef KAN_VROWS_WPE
#define KAN_VROWS_WPE 2
#endif
#ifndef KAN_VROWS_SB
#define KAN_VROWS_SB 1
#endif
#ifndef KAN_VROWS_NORED
#define KAN_VROWS_NORED 0
#endif
#ifndef KAN_VROWS_SKEL
#define KAN_VROWS_SKEL 0
#endif
#ifndef KAN_VROWS_CONTIG
#define KAN_VROWS_CONTIG 1
#endif
#ifndef KAN_VROWS_L2LOAD
#define KAN_VROWS_L2LOAD 0
#endif
// NI > 0: the table's interval count compiled in, so the Horner coefficients' LDS offsets are instruction
// immediates (as fk_vjp_pp_wave_kernel; round 4: the per-point address arithmetic of the runtime count
// was ~8 VALU per point and stage)
#ifndef KAN_VROWS_NI
#define KAN_VROWS_NI 1
#endif
// KAN_ADJ_FIN_BLOCK threads: with 1024 the slab rows of a step kernel's grid (up to 1024 blocks) are one load
// per slab per thread, all in flight at once
#ifndef KAN_ADJ_FIN_BLOCK
#define KAN_ADJ_FIN_BLOCK 256
#endif
constexpr int kAdjFinBlock = KAN_ADJ_FIN_BLOCK;
// Block q of the adaptive adjoint step's finish (adj_finish_kernel; q == P: the λ error partials).  AG: the
// rows were stored by other workgroups of the running launch (the rows kernel's fused finish) and are read
// with agent-scope loads.  The order depends only on blockDim, so both callers give the same bits.
template <bool AG>
__device__ __forceinline__ double fin_ld(const double* p) {
    if constexpr (AG) return ld_agent(p);
    else return *p;
}
template <bool AG, bool AGW = false, class F = AdjFinish>
__device__ __forceinline__ void adj_finish_block(const F& f, int64_t P, int64_t q, double* red, double* sums) {
    // four of each thread's rows per pass, all loads issued before the adds (same order of the adds)
    const int64_t bs = blockDim.x;
    if (q == P) {   // the λ error partials
        double s = 0.0;
        int64_t b = threadIdx.x;
        for (; b + 3 * bs < f.nblk; b += 4 * bs) {
            double v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = fin_ld<AG>(f.err_slab + b + r * bs);
#pragma unroll
            for (int r = 0; r < 4; ++r) s += v[r];
        }
        for (; b < f.nblk; b += bs) s += fin_ld<AG>(f.err_slab + b);
        const double v[1] = {s};
        block_sum_to<double, 1>(v, 1, red, sums);
        __syncthreads();
        if (threadIdx.x == 0) {
            if constexpr (AGW) st_agent(f.out, sums[0]);   // (read by the controller of this launch)
            else f.out[0] = sums[0];
        }
        return;
    }
    double acc[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) acc[i] = 0.0;
    const int64_t rs = f.tr ? 1 : P, qo = f.tr ? q * f.nblk : q;   // row b of parameter q at b·rs + qo
    int64_t b = threadIdx.x;
    if (f.nslab <= 3) {
        for (; b + 3 * bs < f.nblk; b += 4 * bs) {
            double v[4][3];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int i = 0; i < 3; ++i) v[r][i] = i < f.nslab ? fin_ld<AG>(f.slab[i] + (b + r * bs) * rs + qo) : 0.0;
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int i = 0; i < 3; ++i) acc[i] += v[r][i];
        }
    }
    for (; b < f.nblk; b += bs) {
        double v[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) v[i] = i < f.nslab ? fin_ld<AG>(f.slab[i] + b * rs + qo) : 0.0;   // all loads first
#pragma unroll
        for (int i = 0; i < 6; ++i) acc[i] += v[i];
    }
    block_sum_to<double, 6>(acc, f.nslab, red, sums);
    __syncthreads();
    if (threadIdx.x == 0) {
        double cm = 0.0, ce = 0.0, k7 = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            if (i < f.nslab) {
                cm = ::fma(f.ca[i], sums[i], cm);
                ce = ::fma(f.ce[i], sums[i], ce);
                if (i == f.k7) k7 = sums[i];
            }
        }
        const double m0 = f.mu[q], k1 = f.km1[q];
        const double mn = ::fma(1.0, cm, ::fma(f.a0, k1, m0));
        f.mu_new[q] = mn;
        f.km7[q] = k7;
        const double e = ::fma(f.e0, k1, ce);
        const double r = e / ::fma(f.reltol, fmax(kabs(m0), kabs(mn)), f.abstol);
        if constexpr (AGW) st_agent(f.out + 1 + q, r * r);
        else f.out[1 + q] = r * r;
    }
}

// The rows kernel's fused finish (AdjStepArgs::fin_ctr): every workgroup has stored its rows (agent-scope
// stores) and arrives; the last P + 1 to arrive wait for the rest (the one arriving last does not wait) and
// each runs one block of the finish.  Every wait is bounded: on a time-out the terms are not written and the
// host's wait on them fails when the stream drains.  The finishers count themselves out; the last one puts
// both counters back to zero for the next launch.
constexpr unsigned kFinSpinMax = 1u << 22;
__device__ __forceinline__ void rows_fused_finish(const AdjFinish& f, unsigned* ctr, int64_t P) {
    __shared__ double fred[(kVjpBlock / kWave) * 6];
    __shared__ double fsums[6];
    __shared__ unsigned farr;
    __shared__ int fok;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's row stores have landed
    __syncthreads();
    if (threadIdx.x == 0) farr = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned G = gridDim.x;
    const unsigned back = G - 1u - farr;   // 0: the last to arrive
    if (back > (unsigned)P) return;
    if (threadIdx.x == 0) {
        int ok = 1;
        for (unsigned spins = 0; __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < G; ++spins) {
            if (spins > kFinSpinMax) {
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        fok = ok;
    }
    __syncthreads();
    if (fok) adj_finish_block<true>(f, P, P - (int64_t)back, fred, fsums);
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned d = __hip_atomic_fetch_add(ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == (unsigned)P) {
            __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// The rows step's body (kan_rows_body.inc) reads its arguments as `a`: the kernel's own (by value), or in
// fk_vjp_step_rows_loop_kernel (the device step control, kan_adjloop.hpp) the attempt's plan through the
// constant address space.  (A reference to the by-value argument made the compiler form the arguments'
// products per use: +23% VALU.)
template <int NORM, int PATH, int GT, int NP, int CMB, int NI = 0>
__global__ void __launch_bounds__(kVjpBlock) __attribute__((amdgpu_waves_per_eu(KAN_VROWS_WPE)))
fk_vjp_step_rows_kernel(const LayerConst* __restrict__ lcp, const double* __restrict__ p,
                        const double2* __restrict__ tables, int ni_rt, double inv_w, double x0, double cd, double co,
                        int64_t B, AdjStepArgs a) {
#define KAN_ROWS_BODY_DEV 0
#include "kan_rows_body.inc"
#undef KAN_ROWS_BODY_DEV
}

template <int NORM, int PATH, int GT, int NP, int CMB, int NI = 0>
__global__ void __launch_bounds__(kVjpBlock) __attribute__((amdgpu_waves_per_eu(KAN_VROWS_WPE)))
fk_vjp_step_rows_loop_kernel(const LayerConst* __restrict__ lcp, const double* __restrict__ p,
                             const double2* __restrict__ tables, int ni_rt, double inv_w, double x0, double cd,
                             double co, int64_t B, const AdjLoopCtl* __restrict__ lctl, const AdjLoopPlan* lplan) {
    if (lctl->status != 0) return;   // the adjoint has ended or paused: a launch the host queued ahead
    typedef const __attribute__((address_space(4))) AdjStepArgs CArgs;
    const CArgs& a = *(CArgs*)&lplan[lctl->it & 1].a;
#define KAN_ROWS_BODY_DEV 1
#include "kan_rows_body.inc"
#undef KAN_ROWS_BODY_DEV
}

// dp[q] (= or +=) Σ_b slab[b·P + q] for q < P (block q), and err_out[0] = Σ_b err_slab[b]
// (block P): the adjoint stage's reductions in one launch, fixed order.
__global__ void __launch_bounds__(kBlock)
vjp_finish_kernel(const double* __restrict__ slab, int64_t nblk, int64_t P, double* __restrict__ dp, int assign,
                  const double* __restrict__ err_slab, double* __restrict__ err_out) {
    __shared__ double red[kBlock / kWave];
    const int64_t q = blockIdx.x;
    double s = 0.0;
    if (q < P) {
        s = strided_rows_sum(slab + q, nblk, P, s);
    } else {
        s = strided_rows_sum(err_slab, nblk, 1, s);
    }
    s = wave_sum(s);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = red[0];
        for (int w = 1; w < (int)(blockDim.x / kWave); ++w) t += red[w];
        if (q < P) dp[q] = assign ? t : dp[q] + t;
        else err_out[0] = t;
    }
}

// vjp_finish_kernel over several jobs: blockIdx.y = job, blockIdx.x = q (< P: dp_q; == P: error)
__global__ void __launch_bounds__(kBlock) vjp_finish_jobs_kernel(FinishJobs jobs, int64_t P) {
    __shared__ double red[kBlock / kWave];
    FinishJob jb{};
#pragma unroll
    for (int j = 0; j < kMaxFinishJobs; ++j)   // static indices: no copy of the argument to scratch
        if (j == (int)blockIdx.y) jb = jobs.j[j];
    const int64_t q = blockIdx.x;
    if (q < P ? !jb.dp : !jb.err_out) return;
    double s = 0.0;
    if (q < P) {
        s = jb.tr ? strided_rows_sum(jb.slab + q * jb.nblk, jb.nblk, 1, s) : strided_rows_sum(jb.slab + q, jb.nblk, P, s);
    } else {
        s = strided_rows_sum(jb.err_slab, jb.nblk, 1, s);
    }
    s = wave_sum(s);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = red[0];
        for (int w = 1; w < (int)(blockDim.x / kWave); ++w) t += red[w];
        if (q < P) {
            if (jb.base) jb.dp[q] = ::fma(1.0, t, ::fma(jb.coef, jb.other[q], jb.base[q]));
            else jb.dp[q] = jb.assign ? t : jb.dp[q] + t;
        } else {
            jb.err_out[0] = t;
        }
    }
}

hipError_t launch_vjp_finish_jobs(const FinishJobs& jobs, int njobs, int64_t P, hipStream_t st) {
    if (njobs <= 0) return hipSuccess;
    if (njobs > kMaxFinishJobs) return hipErrorInvalidValue;
    hipLaunchKernelGGL(vjp_finish_jobs_kernel, dim3((unsigned)P + 1, (unsigned)njobs), dim3(kBlock), 0, st, jobs, P);
    return hipGetLastError();
}

__global__ void __launch_bounds__(kAdjFinBlock) adj_finish_kernel(AdjFinish f, int64_t P) {
    __shared__ double red[(kAdjFinBlock / kWave) * 6];
    __shared__ double sums[6];
    adj_finish_block<false>(f, P, blockIdx.x, red, sums);
}

hipError_t launch_adj_finish(const AdjFinish& f, int64_t P, hipStream_t st) {
    if (f.nslab < 1 || f.nslab > 6 || P < 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(adj_finish_kernel, dim3((unsigned)P + 1), dim3(kAdjFinBlock), 0, st, f, P);
    return hipGetLastError();
}

// ---- the adjoint's device step control (kan_adjloop.hpp) --------------------------------------------------
// The forward steps the next plan's stages can fall in, staged in LDS by the controlling workgroup: the window
// ends a few steps above the last planned stage's (the adjoint runs backward in t); beyond it, global loads.
constexpr int kAdjWin = 256;
struct AdjFwWindow {
    const double* wts;
    const double* wdts;
    void* const* wsl;
    int64_t w0, wn;
    const double* gts;
    const double* gdts;
    void* const* gsl;
    __device__ bool in(int64_t i) const { return i >= w0 && i < w0 + wn; }
    __device__ double ts(int64_t i) const { return in(i) ? wts[i - w0] : gts[i]; }
    __device__ double dts(int64_t i) const { return in(i) ? wdts[i - w0] : gdts[i]; }
    __device__ const void* slot(int64_t i) const { return in(i) ? wsl[i - w0] : gsl[i]; }
};

// The finish launch of an attempt: each workgroup runs its block of adj_finish_kernel (the error terms by
// agent-scope stores), then counts itself in; the last to arrive sums the terms in adjoint_t's order and
// thread 0 applies its PI controller.  The next attempt's plan differs from the current one only in its
// step-dependent fields (the host wrote the rest into both buffers, kan_adjloop.hpp adj_loop_plan): those the
// workgroup's threads write in parallel, stage s's forward-step search on thread s.  Every workgroup stages
// the forward-step window and reads the state at its start, so the controller's inputs are on chip when the
// last one arrives.  The host's mirror is written when the state needs it (a stop, the end) and every 8
// attempts (the host's queue refill reads the attempt count from it).
constexpr int kAdjMaxTerms = kMaxGrid + 2;   // 1 + P, P <= G + 1
__global__ void __launch_bounds__(kAdjFinBlock) adj_finish_loop_kernel(AdjLoopArgs la) {
    using K = Tsit5Tab;
    __shared__ double red[(kAdjFinBlock / kWave) * 6];
    __shared__ double sums[6];
    __shared__ double wts[kAdjWin], wdts[kAdjWin];
    __shared__ void* wsl[kAdjWin];
    __shared__ double terms[kAdjMaxTerms];
    __shared__ unsigned arr;
    __shared__ AdjLoopCtl cs;   // the state after the decision
    __shared__ int64_t fis[6];
    KAN_PROBE_T(pf0)
    const AdjLoopCtl* cp = la.ctl;
    if (cp->status != 0) return;
    AdjLoopCtl c = *cp;
    // the controller's inputs that do not depend on the error terms, on thread 0 while the reduction runs
    // (only the last workgroup to arrive uses them)
    double qb2 = 0.0, stop_si = 0.0;
    if (threadIdx.x == 0) {
        qb2 = ::pow(c.qold, la.beta2);
        stop_si = la.stops[c.si];
    }
    int64_t w0 = c.fi - (kAdjWin - 8);
    if (w0 < 0) w0 = 0;
    const int64_t wn = la.nsteps - w0 < kAdjWin ? la.nsteps - w0 : kAdjWin;
    for (int64_t i = threadIdx.x; i < wn; i += blockDim.x) {   // (published by the finish block's barriers)
        wts[i] = la.fts[w0 + i];
        wdts[i] = la.fdts[w0 + i];
        wsl[i] = la.slots[w0 + i];
    }
    typedef const __attribute__((address_space(4))) AdjFinish CFin;
    adj_finish_block<false, true>(*(CFin*)&la.plan[c.it & 1].f, la.P, blockIdx.x, red, sums);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this workgroup's error term has landed
    __syncthreads();
    KAN_PROBE_T(pf1)
    if (threadIdx.x == 0) arr = __hip_atomic_fetch_add(la.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (arr != gridDim.x - 1u) return;
    if (threadIdx.x <= la.P) terms[threadIdx.x] = ld_agent(la.out + threadIdx.x);
    __syncthreads();
    KAN_PROBE_T(pf2)
    if (threadIdx.x == 0) {
        double mus = 0.0;   // the μ terms in order, then the λ total (adjoint_t)
        for (int64_t q = 0; q < la.P; ++q) mus += terms[1 + q];
        const double sumsq = terms[0] + mus;
        const double eest = ::sqrt(sumsq / la.ntot);
        const double q11 = eest > 0 ? ::pow(eest, la.beta1) : 0.0;
        ++c.it;
        c.nf += 6;
        if (eest > 1.0 && c.h > la.dtmin) {
            ++c.nreject;
            c.h = c.h / ::fmin(1.0 / la.qmin, q11 / la.gamma);
        } else {
            double q = q11 / qb2;
            q = ::fmax(1.0 / la.qmax, ::fmin(1.0 / la.qmin, q / la.gamma));
            const double hnew = q > 0 ? c.h / q : c.h * la.qmax;
            c.qold = ::fmax(eest, la.qoldinit);
            if (la.hs && c.naccept < la.hs_cap) la.hs[c.naccept] = c.h;
            c.tau = c.tau + c.h;
            c.lc ^= 1;
            c.mc ^= 1;
            c.fs ^= 1;   // FSAL: kλ_7, kμ_7 become the next step's first stage values
            ++c.naccept;
            c.h = hnew;
            if (::fabs(c.tau - stop_si) <= 1e-12 * ::fmax(1.0, la.TT)) {
                c.tau = stop_si;
                if (c.si + 1 < la.nstops) c.status = 3;   // the host takes the saveat jump and the next stop
            }
        }
        if (c.status == 0) adj_loop_top(la, c, stop_si);
        cs = c;
    }
    __syncthreads();
    KAN_PROBE_T(pf3)
    c = cs;
    const int t = threadIdx.x;
    if (c.status == 0) {   // the next attempt's step-dependent fields
        AdjLoopPlan& pl = la.plan[c.it & 1];
        AdjStepArgs& a = pl.a;
        const double h = c.h, tau = c.tau;
        if (t < 6) {
            const double ts = la.tf - (t == 5 ? tau + h : tau + K::TC[t] * h);
            const AdjFwWindow fw{wts, wdts, wsl, w0, wn, la.fts, la.fdts, la.slots};
            const int64_t fi = adj_loop_interval(fw, la.nsteps, ts, c.fi);
            const double r = (ts - fw.ts(fi)) / fw.dts(fi);
            const double th = r < 0.0 ? 0.0 : (r > 1.0 ? 1.0 : r);
            const double* su = static_cast<const double*>(fw.slot(fi));
            a.su_u[t] = su;
            for (int m = 0; m < 4; ++m) a.su_q[t][m] = su + (m + 1) * la.n;
            a.su_c[t][0] = th;
            a.su_c[t][1] = th * th;
            a.su_c[t][2] = th * th * th;
            a.su_c[t][3] = th * th * th * th;
            fis[t] = fi;
        } else if (t < 42) {
            const int ii = (t - 6) / 6, jj = (t - 6) % 6;
            a.a[ii][jj] = jj <= ii ? h * K::TA[ii][jj] : 0.0;
        } else if (t < 49) {
            a.ec[t - 42] = h * K::BT[t - 42];
        } else if (t == 49) {
            a.kl[0] = c.fs ? la.kl[6] : la.kl[0];
            a.kl[6] = c.fs ? la.kl[0] : la.kl[6];
            a.lam = la.lam[c.lc];
            a.lam_out = la.lam[c.lc ^ 1];
            AdjFinish& f = pl.f;
            f.a0 = h * K::TA[5][0];
            f.e0 = h * K::BT[0];
            f.mu = la.mu[c.mc];
            f.mu_new = la.mu[c.mc ^ 1];
            f.km1 = c.fs ? la.km[6] : la.km[0];
            f.km7 = c.fs ? la.km[0] : la.km[6];
        }
        __syncthreads();
        if (t == 0) {
            a.reload[0] = 1;
            for (int q = 1; q < 6; ++q) a.reload[q] = fis[q] == fis[q - 1] ? 0 : 1;   // (same slot: same u_i, Q_m)
            c.fi = fis[5];
        }
    }
    if (t == 0) {
        *la.ctl = c;
        if (c.status != 0 || (c.it & 7) == 0) *la.mirror = c;
        __hip_atomic_store(la.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        KAN_PROBE_T(pf4)
        KAN_PROBE_ADD(2, pf1 - pf0)   // the last workgroup: start -> its error term landed
        KAN_PROBE_ADD(3, pf2 - pf1)   // arrival, the terms' loads
        KAN_PROBE_ADD(4, pf3 - pf2)   // the decision (thread 0)
        KAN_PROBE_ADD(5, pf4 - pf3)   // the plan fields, the state's store
        KAN_PROBE_ADD(6, 1)
    }
}

// du = D·lap·y + KAN(y) for one trajectory row held by one wave (lane: pairs 128k + 2·lane),
// stencil neighbours by wave rotation, the KAN from the LDS table (direct formula off-table)
template <int NORM, int BASIS, int NP>
__device__ __forceinline__ void fk_row_rhs(const Math<double>& M, const LayerConst& lc, const double* __restrict__ p,
                                           const double2* __restrict__ tl, int ni, double inv_w, double x0, double cd,
                                           double co, int lane, const kd2 (&y)[NP], kd2 (&du)[NP]) {
    constexpr int Nx = 128 * NP;
    double rr[NP], rl[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        rr[k] = wave_ror1(y[k].y);
        rl[k] = wave_rol1(y[k].x);
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const double um = lane == 0 ? rr[(k + NP - 1) % NP] : rr[k];
        const double up = lane == kWave - 1 ? rl[(k + 1) % NP] : rl[k];
        const int i = 128 * k + 2 * lane;
        bool ok0, ok1;
        double k0 = pp_eval(tl, ni, inv_w, x0, y[k].x, ok0);
        double k1 = pp_eval(tl, ni, inv_w, x0, y[k].y, ok1);
        if (__builtin_expect(!(ok0 && ok1), 0)) {
            double sc;
            if (!ok0) k0 = pp_direct<NORM, BASIS>(M, lc, p, lc.grid, y[k].x, sc);
            if (!ok1) k1 = pp_direct<NORM, BASIS>(M, lc, p, lc.grid, y[k].y, sc);
        }
        double l0, l1;
        lap_pair<double>(um, y[k].x, y[k].y, up, i, Nx, cd, co, l0, l1);
        du[k].x = l0 + k0;
        du[k].y = l1 + k1;
    }
}

// A whole Tsit5 step per trajectory row (kanode_solve_tsit5, host control, Fisher-KPP table
// path): the Laplacian stencil couples only the points of one row, so the six stages run
// with the row in registers: u and k_1 are read once, k_2..k_7 and u_new written once (the
// dense output slot), instead of six stage launches re-reading u and k_1..k_s.  Same
// arithmetic and order as six fk_stage_pp_wave_kernel launches (bitwise equal results);
// the embedded-error partial Σ (e/sk)² goes to err_slab[block] (ordered).
struct StepOut {
    double* k[6];     // k_2..k_7, or (qform) Q_1..Q_4, -, k_7
    double* u_new;
    int32_t qform;    // dense output as u_n + Σ_m θ^(m+1) Q_m, Q_m = dt Σ_i RI[i][m] k_i
};
#ifndef KAN_FSTEP_WPE
#define KAN_FSTEP_WPE KAN_PP_WPE
#endif

// The step control of a device-controlled solve (FkLoopArgs), at the head of the NEXT launch: every workgroup
// of launch q sums launch q - 1's error partials in the same order and applies solve_t's PI controller to its
// attempt, so all reach the same decision with no grid-wide wait; workgroup 0 records an accepted step and
// writes the state launch q + 1 reads (and the host's mirror).  Returns false when the solve has ended.
__device__ __forceinline__ bool fk_loop_decide(const FkLoopArgs& la, int64_t q, FkLoopCtl& c, double* red,
                                               double* lsum) {
    // the previous launch's partials are loaded with the state, not after it (one round trip)
    const double* pp = la.parts + ((q + 1) & 1) * la.max_grid;
    double s = 0.0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += kBlock) s += pp[b];
    const FkLoopCtl* sp = la.state + ((q + 1) & 1);
    c = *sp;
    const bool w0 = blockIdx.x == 0 && threadIdx.x == 0;
    FkLoopCtl* out = la.state + (q & 1);
    if (c.status != 0) {   // ended earlier: a launch queued ahead passes the state on
        if (w0) *out = c;
        return false;
    }
    if (c.pending) {
        // qold^β2 does not depend on the error: formed while the partials are in flight
        const double qb2 = ::pow(c.qold, la.beta2);
        const double v[1] = {s};
        block_sum_to<double, 1>(v, 1, red, lsum);   // (the same order in every workgroup)
        const double eest = ::sqrt(*lsum / (double)la.n);
        const double q11 = eest > 0 ? ::pow(eest, la.beta1) : 0.0;
        ++c.it;
        if (eest > 1.0 && c.dt > la.dtmin) {
            ++c.nreject;
            c.dt = c.dt / ::fmin(1.0 / la.qmin, q11 / la.gamma);
        } else {
            double qq = q11 / qb2;
            qq = ::fmax(1.0 / la.qmax, ::fmin(1.0 / la.qmin, qq / la.gamma));
            if (1.0 <= qq && qq <= 1.0) qq = 1.0;   // qsteady_min = qsteady_max = 1
            const double dtnew = qq > 0 ? c.dt / qq : c.dt * la.qmax;
            c.qold = ::fmax(eest, la.qoldinit);
            if (w0) {
                la.ts[c.step] = c.t;
                la.dts[c.step] = c.dt;
            }
            c.t = c.t + c.dt;
            ++c.step;
            c.dt = dtnew;
            for (int k = 0; k < 3; ++k) c.cand[k] = c.cand[k + 1];   // slots[step - 1 .. step + 1]
            c.cand[3] = nullptr;
        }
    }
    if (c.t >= la.tf - 1e-14 * ::fmax(1.0, ::fabs(la.tf))) c.status = 1;
    else if (c.it >= la.maxiters) c.status = 2;
    else c.dt = ::fmin(c.dt, la.tf - c.t);   // (solve_t clips at the top of its next iteration)
    c.pending = c.status == 0 ? 1 : 0;
    if (w0) {
        FkLoopCtl o = c;
        if (o.status == 0) o.cand[3] = la.slots[o.step + 2];
        *out = o;
        if (o.status != 0 || (o.it & 7) == 0) *la.mirror = o;   // (the host's queue refill reads it; 1 in 8)
    }
    return c.status == 0;
}
// DEV (FkLoopArgs, solve_fk_loop, launch q): the attempt's step and size come from fk_loop_decide, its
// coefficients (dt times the tableau, as the host forms them) from LDS, its vectors are the slots of the
// table, and the error partials go to la.parts for launch q + 1.
template <int NORM, int BASIS, int NP, bool DEV = false>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KAN_FSTEP_WPE)))
fk_step_pp_wave_kernel(const LayerConst* __restrict__ lcp, const double* __restrict__ p,
                       const double2* __restrict__ table, int ni, double inv_w, double x0, double cd, double co,
                       const double* __restrict__ u, const double* __restrict__ k1, StepOut so, StepCoef sc,
                       double* __restrict__ err_slab, int64_t B, FkLoopArgs la, int64_t lq) {
    constexpr int Nx = 128 * NP;
    KAN_PROBE_T(pw0)
    extern __shared__ double2 tl[];
    __shared__ double red[kBlock / kWave];
    // DEV: the attempt's coefficients in LDS (published by the table staging's barrier below)
    __shared__ StepCoef lsc[1];
    __shared__ double lsum;
    // the table's loads first: under DEV they overlap the state and partials loads of the decision
    for (int i = threadIdx.x; i < (kPPCoef / 2) * ni; i += kBlock) tl[i] = table[i];   // (register copy: glds here cost occupancy)
    // DEV: this wave's first row is loaded before the decision, for the attempt it will most likely take
    // (the previous one accepted: the next step's u and k_1); a rejection reloads it below
    const int64_t b0 = (int64_t)blockIdx.x * (kBlock / kWave) + (threadIdx.x >> 6);
    const double* su_spec = nullptr;
    const double* sk_spec = nullptr;
    kd2 us0[NP], ks0[NP];
    if constexpr (DEV) {
        const FkLoopCtl* sp = la.state + ((lq + 1) & 1);
        if (sp->status == 0) {
            const int64_t st0 = sp->step;
            su_spec = static_cast<const double*>(sp->pending ? sp->cand[2] : sp->cand[1]);
            sk_spec = sp->pending ? static_cast<const double*>(sp->cand[1]) + 5 * la.n
                                  : (st0 == 0 ? la.k1_0 : static_cast<const double*>(sp->cand[0]) + 5 * la.n);
            if (b0 < B) {
                const int64_t rb = b0 * Nx + 2 * (threadIdx.x & (kWave - 1));
#pragma unroll
                for (int k = 0; k < NP; ++k) {
                    us0[k] = ld_fstep(su_spec + rb + 128 * k);
                    ks0[k] = ld_fstep(sk_spec + rb + 128 * k);
                }
            }
        }
    }
    if constexpr (DEV) {
        FkLoopCtl c;
        if (!fk_loop_decide(la, lq, c, red, &lsum)) return;   // the solve has ended: a launch queued ahead
        double* const cur = static_cast<double*>(c.cand[1]);
        u = cur;
        k1 = c.step == 0 ? la.k1_0 : static_cast<const double*>(c.cand[0]) + 5 * la.n;
#pragma unroll
        for (int m = 0; m < 4; ++m) so.k[m] = cur + (m + 1) * la.n;
        so.k[5] = cur + 5 * la.n;
        so.u_new = static_cast<double*>(c.cand[2]);
        err_slab = la.parts + (lq & 1) * la.max_grid;
        const int t = threadIdx.x;
        if (t < 36) lsc[0].a[t / 6][t % 6] = t % 6 <= t / 6 ? c.dt * Tsit5Tab::TA[t / 6][t % 6] : 0.0;
        else if (t < 43) lsc[0].e[t - 36] = c.dt * Tsit5Tab::BT[t - 36];
        else if (t < 71) lsc[0].q[(t - 43) / 7][(t - 43) % 7] = c.dt * Tsit5Tab::RI[(t - 43) % 7][(t - 43) / 7];
    }
    auto ca = [&](int s_, int j) { return DEV ? lsc[0].a[s_][j] : sc.a[s_][j]; };   // dt·a_sj
    auto ce = [&](int j) { return DEV ? lsc[0].e[j] : sc.e[j]; };                     // dt·btilde_j
    auto cq = [&](int m, int i) { return DEV ? lsc[0].q[m][i] : sc.q[m][i]; };        // dt·RI[i][m]
    const double abstol = DEV ? la.abstol : sc.abstol, reltol = DEV ? la.reltol : sc.reltol;
    KAN_EXP_TABLE_LDS(tab);   // (its __syncthreads also publishes tl)
    KAN_PROBE_T(pw1)
    const Math<double> M{tab};
    const LayerConst& lc = *lcp;
    const int lane = threadIdx.x & (kWave - 1);
    const bool want_err = err_slab != nullptr;
    const int64_t rstride = (int64_t)gridDim.x * (kBlock / kWave);
    double eacc = 0.0;
    for (int64_t b = b0; b < B; b += rstride) {
        const int64_t rb = b * Nx + 2 * lane;
        kd2 uv[NP], kk[7][NP], y[NP];
        if (DEV && b == b0 && u == su_spec && k1 == sk_spec) {
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                uv[k] = us0[k];
                kk[0][k] = ks0[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                uv[k] = ld_fstep(u + rb + 128 * k);
                kk[0][k] = ld_fstep(k1 + rb + 128 * k);
            }
        }
#pragma unroll
        for (int s = 0; s < 6; ++s) {
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                y[k] = uv[k];
#pragma unroll
                for (int j = 0; j <= s; ++j) {
                    y[k].x = ::fma(ca(s, j), kk[j][k].x, y[k].x);
                    y[k].y = ::fma(ca(s, j), kk[j][k].y, y[k].y);
                }
            }
            fk_row_rhs<NORM, BASIS, NP>(M, lc, p, tl, ni, inv_w, x0, cd, co, lane, y, kk[s + 1]);
            if (!DEV && !so.qform) {
#pragma unroll
                for (int k = 0; k < NP; ++k) st_stream(so.k[s] + rb + 128 * k, kk[s + 1][k]);
            }
        }
        if (DEV || so.qform) {   // the interpolation polynomials of the dense output, then k_7 (FSAL)
#pragma unroll
            for (int m = 0; m < 4; ++m) {
#pragma unroll
                for (int k = 0; k < NP; ++k) {
                    kd2 q{0.0, 0.0};
#pragma unroll
                    for (int i = 0; i < 7; ++i) {
                        q.x = ::fma(cq(m, i), kk[i][k].x, q.x);
                        q.y = ::fma(cq(m, i), kk[i][k].y, q.y);
                    }
                    st_stream(so.k[m] + rb + 128 * k, q);
                }
            }
#pragma unroll
            for (int k = 0; k < NP; ++k) st_fstep(so.k[5] + rb + 128 * k, kk[6][k]);
        }
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            st_fstep(so.u_new + rb + 128 * k, y[k]);
            if (want_err) {
                kd2 e{0.0, 0.0};
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    e.x = ::fma(ce(j), kk[j][k].x, e.x);
                    e.y = ::fma(ce(j), kk[j][k].y, e.y);
                }
                const double ex = ::fma(ce(6), kk[6][k].x, e.x), ey = ::fma(ce(6), kk[6][k].y, e.y);
                const double sx = ::fma(reltol, fmax(kabs(uv[k].x), kabs(y[k].x)), abstol);
                const double sy = ::fma(reltol, fmax(kabs(uv[k].y), kabs(y[k].y)), abstol);
                const double rx = ex / sx, ry = ey / sy;
                eacc = ::fma(rx, rx, eacc);
                eacc = ::fma(ry, ry, eacc);
            }
        }
    }
    if constexpr (DEV) {
        KAN_PROBE_T(pw2)
        const double v[1] = {eacc};
        block_sum_to<double, 1>(v, 1, red, err_slab + blockIdx.x);
        if (threadIdx.x == 0) {
            KAN_PROBE_T(pw3)
            KAN_PROBE_ADD(8, pw1 - pw0)    // decision + table staging
            KAN_PROBE_ADD(9, pw2 - pw1)    // rows
            KAN_PROBE_ADD(10, pw3 - pw2)   // error partial
            KAN_PROBE_ADD(11, 1)
        }
    } else if (want_err) {
        const double v[1] = {eacc};
        block_sum_to<double, 1>(v, 1, red, err_slab + blockIdx.x);
    }
}


// Runge-Kutta stage, fused (kanode_rhs_stage): the stage input y = u + Σ_j c_j k_j is
// formed in registers from nontemporal loads of u and the k_j, the stencil
// neighbours of y come from the wave rotations, du = f(y) as above.  Optionally y
// is written (the adjoint's saved input; Tsit5's u_new) and the embedded error
// Σ (e/sk)², e = Σ ec_j k_j + ec_nk du, sk = abstol + reltol·max(|u|,|y|), is
// block-summed into err_slab[blockIdx.x] (ordered: reproducible).
template <int NORM, int BASIS, int NP>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KAN_PP_WPE)))
fk_stage_pp_wave_kernel(const LayerConst* __restrict__ lcp, const double* __restrict__ p,
                        const double2* __restrict__ table, int ni, double inv_w, double x0, double cd, double co,
                        const double* __restrict__ u, StageArgs<double> sa, double* __restrict__ y_out,
                        double* __restrict__ err_slab, double* __restrict__ du, int64_t B) {
    constexpr int Nx = 128 * NP;
    extern __shared__ double2 tl[];
    __shared__ double red[kBlock / kWave];
    if (stage_skip(sa.skip)) return;
    for (int i = threadIdx.x; i < (kPPCoef / 2) * ni; i += kBlock) tl[i] = table[i];
    KAN_EXP_TABLE_LDS(tab);   // (its __syncthreads also publishes tl)
    const Math<double> M{tab};
    const LayerConst& lc = *lcp;
    const int lane = threadIdx.x & (kWave - 1);
    const bool want_err = err_slab != nullptr;
    const double sac = stage_scale(sa.cscale);
    const int64_t rstride = (int64_t)gridDim.x * (kBlock / kWave);
    double eacc = 0.0;
    for (int64_t b = (int64_t)blockIdx.x * (kBlock / kWave) + (threadIdx.x >> 6); b < B; b += rstride) {
        const int64_t rb = b * Nx + 2 * lane;
        kd2 uv[NP], y[NP], e[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            uv[k] = ld_stream(u + rb + 128 * k);
            y[k] = uv[k];
            e[k] = kd2{0.0, 0.0};
        }
        if (want_err) stage_sum<NP, true>(sa, rb, sac, y, e);
        else stage_sum<NP, false>(sa, rb, sac, y, e);
        kd2 dv[NP];
        fk_row_rhs<NORM, BASIS, NP>(M, lc, p, tl, ni, inv_w, x0, cd, co, lane, y, dv);
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            const int i = 128 * k + 2 * lane;
            const kd2 o = dv[k];
            st_stream(du + b * Nx + i, o);
            if (y_out) st_stream(y_out + b * Nx + i, y[k]);
            if (want_err) {
                const double en = stage_ec_last(sa) * sac;
                const double ex = ::fma(en, o.x, e[k].x), ey = ::fma(en, o.y, e[k].y);
                const double sx = ::fma(sa.reltol, fmax(kabs(uv[k].x), kabs(y[k].x)), sa.abstol);
                const double sy = ::fma(sa.reltol, fmax(kabs(uv[k].y), kabs(y[k].y)), sa.abstol);
                const double rx = ex / sx, ry = ey / sy;
                eacc = ::fma(rx, rx, eacc);
                eacc = ::fma(ry, ry, eacc);
            }
        }
    }
    if (want_err) {
        const double v[1] = {eacc};
        block_sum_to<double, 1>(v, 1, red, err_slab + blockIdx.x);
    }
}

// Persistent grid: min(resident blocks per CU, 4) x CUs, each block stages the table
// once.  4 blocks (16 waves) per CU streamed fastest in the grid sweep (tools/pp_grid.sh:
// 98.7 us at 1024 blocks vs 101.4 us at the 6-block occupancy limit); the nontemporal
// copy microbenchmark peaks at the same shape.  KANODE_OPT_GRID_RHS overrides (tuning only).
template <typename K>
static int pp_grid_cap(K kernel, size_t lds, int bs = kBlock) {
    int dev = 0, cus = 256, nb = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, bs, lds) != hipSuccess || nb < 1) nb = 4;
    return (nb < 4 ? nb : 4) * cus;
}

hipError_t launch_fk_pp_build(const PPConst& hpc, const LayerConst* lc, const PPConst* pc, const double* p,
                              double* tables, const int* fns, int nfn, hipStream_t st) {
    if (hpc.ni <= 0 || hpc.ni % kPPPerBlock || hpc.ni > kPPMaxIntervals || nfn < 1 || nfn > kPPMaxFns)
        return hipErrorInvalidValue;
    PPFns f{};
    for (int i = 0; i < nfn; ++i) f.fn[i] = fns[i];
    hipLaunchKernelGGL(fk_pp_build_kernel, dim3(hpc.ni / kPPPerBlock, nfn), dim3(kBlock), 0, st, lc, pc, p, tables,
                       f);
    return hipGetLastError();
}

#ifndef KAN_PP_CHUNK
#define KAN_PP_CHUNK 4
#endif
constexpr int kPPChunk = KAN_PP_CHUNK;   // rows per wave of the table RHS kernel (0 = persistent grid)

hipError_t launch_fk_rhs_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc, const double* p,
                            double* table, double cd, double co, int Nx, const double* u, double* du, int64_t B,
                            hipStream_t st, bool build, int grid_ovr) {
    if (Nx < 2 || (Nx & 1)) return hipErrorInvalidValue;
    const int fn_phi = PP_PHI;
    if (build) {
        hipError_t e = launch_fk_pp_build(hpc, lc, pc, p, table, &fn_phi, 1, st);
        if (e != hipSuccess) return e;
    }
    const int units = Nx / 2;
    const int tl = ceil_log2(units < kBlock ? units : kBlock);
    const int tpb = kBlock >> tl;
    const size_t lds = sizeof(double2) * (kPPCoef / 2) * (size_t)hpc.ni;
#define KAN_PP_WAVE(NORM, BASIS, NP)                                                                             \
    do {                                                                                                         \
        static int cap = 0;                                                                                      \
        if (!cap) cap = pp_grid_cap(fk_rhs_pp_wave_kernel<NORM, BASIS, NP>, lds, kRhsBlock);                   \
        const int chunk = grid_ovr > 0 ? 0 : kPPChunk;                                                          \
        const int grid = chunk > 0 ? grid_for(B, (kRhsBlock / kWave) * chunk, 1 << 30)                            \
                                   : grid_for(B, kRhsBlock / kWave, grid_ovr > 0 ? grid_ovr : cap);             \
        hipLaunchKernelGGL((fk_rhs_pp_wave_kernel<NORM, BASIS, NP>), dim3(grid), dim3(kRhsBlock), lds, st, lc, p, \
                           (const double2*)table, hpc.ni, hpc.inv_w, hpc.x0, cd, co, u, du, B, chunk);           \
    } while (0)
#define KAN_PP_PAIR(NORM, BASIS, SHORT)                                                                          \
    do {                                                                                                         \
        static int cap = 0;                                                                                      \
        if (!cap) cap = pp_grid_cap(fk_rhs_pp_kernel<NORM, BASIS, SHORT>, lds);                                 \
        const int grid = grid_for(B, tpb, cap);                                                                  \
        hipLaunchKernelGGL((fk_rhs_pp_kernel<NORM, BASIS, SHORT>), dim3(grid), dim3(kBlock), lds, st, lc, p,     \
                           (const double2*)table, hpc.ni, hpc.inv_w, hpc.x0, cd, co, Nx, tl, u, du, B);          \
    } while (0)
#define KAN_PP_GO(NORM, BASIS)                                                                                   \
    do {                                                                                                         \
        if (Nx == 256) KAN_PP_WAVE(NORM, BASIS, 2);                                                              \
        else if (Nx == 128) KAN_PP_WAVE(NORM, BASIS, 1);                                                         \
        else if (Nx == 512) KAN_PP_WAVE(NORM, BASIS, 4);                                                         \
        else if (units <= kBlock) KAN_PP_PAIR(NORM, BASIS, true);                                                \
        else KAN_PP_PAIR(NORM, BASIS, false);                                                                    \
    } while (0)
    if (hlc.basis == BASIS_RBF && hlc.norm == NORM_SOFTSIGN) KAN_PP_GO(NORM_SOFTSIGN, BASIS_RBF);
    else if (hlc.basis == BASIS_RBF && hlc.norm == NORM_TANH_FAST) KAN_PP_GO(NORM_TANH_FAST, BASIS_RBF);
    else KAN_PP_GO(NORM_RUNTIME, -1);
#undef KAN_PP_GO
#undef KAN_PP_PAIR
#undef KAN_PP_WAVE
    return hipGetLastError();
}

bool fk_stage_pp_supported(const PPConst& hpc, int Nx) { return hpc.enabled && (Nx == 128 || Nx == 256 || Nx == 512); }

hipError_t launch_fk_stage_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc,
                              const double* p, double* table, double cd, double co, int Nx, const double* u,
                              const StageArgs<double>& sa, double* y_out, double* err_slab, int slab_blocks,
                              double* err_out, double* du, int64_t B, hipStream_t st, bool build, int grid_ovr) {
    if (!fk_stage_pp_supported(hpc, Nx)) return hipErrorInvalidValue;
    const int fn_phi = PP_PHI;
    hipError_t e = hipSuccess;
    if (build && (e = launch_fk_pp_build(hpc, lc, pc, p, table, &fn_phi, 1, st)) != hipSuccess) return e;
    const size_t lds = sizeof(double2) * (kPPCoef / 2) * (size_t)hpc.ni;
    int grid = 0;
    double* slab = err_out ? err_slab : nullptr;
#define KAN_STAGE_WAVE(NORM, BASIS, NP)                                                                          \
    do {                                                                                                         \
        static int cap = 0;                                                                                      \
        if (!cap) cap = pp_grid_cap(fk_stage_pp_wave_kernel<NORM, BASIS, NP>, lds);                             \
        const int gcap = grid_ovr > 0 ? grid_ovr : cap;                                                          \
        grid = grid_for(B, kBlock / kWave, gcap < slab_blocks ? gcap : slab_blocks);                            \
        hipLaunchKernelGGL((fk_stage_pp_wave_kernel<NORM, BASIS, NP>), dim3(grid), dim3(kBlock), lds, st, lc, p, \
                           (const double2*)table, hpc.ni, hpc.inv_w, hpc.x0, cd, co, u, sa, y_out, slab, du, B);  \
    } while (0)
#define KAN_STAGE_GO(NORM, BASIS)                                                                                \
    do {                                                                                                         \
        if (Nx == 256) KAN_STAGE_WAVE(NORM, BASIS, 2);                                                           \
        else if (Nx == 128) KAN_STAGE_WAVE(NORM, BASIS, 1);                                                      \
        else KAN_STAGE_WAVE(NORM, BASIS, 4);                                                                     \
    } while (0)
    if (hlc.basis == BASIS_RBF && hlc.norm == NORM_SOFTSIGN) KAN_STAGE_GO(NORM_SOFTSIGN, BASIS_RBF);
    else if (hlc.basis == BASIS_RBF && hlc.norm == NORM_TANH_FAST) KAN_STAGE_GO(NORM_TANH_FAST, BASIS_RBF);
    else KAN_STAGE_GO(NORM_RUNTIME, -1);
#undef KAN_STAGE_GO
#undef KAN_STAGE_WAVE
    e = hipGetLastError();
    if (e != hipSuccess || !err_out) return e;
    return launch_stage_error_final(err_slab, grid, err_out, st);
}

hipError_t launch_fk_step_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc,
                             const double* p, double* table, double cd, double co, int Nx, const double* u,
                             const double* k1, double* const* kout, double* u_new, const double* a6x6,
                             const double* e7, const double* q4x7, double abstol, double reltol, double* err_slab,
                             int slab_blocks, double* err_out, int64_t B, hipStream_t st, bool build, int grid_ovr,
                             int* parts_out) {
    if (!fk_stage_pp_supported(hpc, Nx)) return hipErrorInvalidValue;
    const int fn_phi = PP_PHI;
    hipError_t e = hipSuccess;
    if (build && (e = launch_fk_pp_build(hpc, lc, pc, p, table, &fn_phi, 1, st)) != hipSuccess) return e;
    const size_t lds = sizeof(double2) * (kPPCoef / 2) * (size_t)hpc.ni;
    StepOut so{};
    for (int j = 0; j < 6; ++j) so.k[j] = kout[j];
    so.u_new = u_new;
    so.qform = q4x7 ? 1 : 0;
    StepCoef sc{};
    if (q4x7)
        for (int m = 0; m < 4; ++m)
            for (int i = 0; i < 7; ++i) sc.q[m][i] = q4x7[7 * m + i];
    for (int s = 0; s < 6; ++s)
        for (int j = 0; j < 6; ++j) sc.a[s][j] = a6x6[6 * s + j];
    for (int j = 0; j < 7; ++j) sc.e[j] = e7 ? e7[j] : 0.0;
    sc.abstol = abstol;
    sc.reltol = reltol;
    int grid = 0;
    double* slab = err_out ? err_slab : nullptr;
#define KAN_STEP_WAVE(NORM, BASIS, NP)                                                                           \
    do {                                                                                                         \
        static int cap = 0;                                                                                      \
        if (!cap) cap = pp_grid_cap(fk_step_pp_wave_kernel<NORM, BASIS, NP>, lds);                              \
        const int gcap = grid_ovr > 0 ? grid_ovr : cap;                                                          \
        grid = grid_for(B, kBlock / kWave, gcap < slab_blocks ? gcap : slab_blocks);                            \
        hipLaunchKernelGGL((fk_step_pp_wave_kernel<NORM, BASIS, NP>), dim3(grid), dim3(kBlock), lds, st, lc, p,  \
                           (const double2*)table, hpc.ni, hpc.inv_w, hpc.x0, cd, co, u, k1, so, sc, slab, B,    \
                           FkLoopArgs{}, (int64_t)0);                                                            \
    } while (0)
#define KAN_STEP_GO(NORM, BASIS)                                                                                 \
    do {                                                                                                         \
        if (Nx == 256) KAN_STEP_WAVE(NORM, BASIS, 2);                                                            \
        else if (Nx == 128) KAN_STEP_WAVE(NORM, BASIS, 1);                                                       \
        else KAN_STEP_WAVE(NORM, BASIS, 4);                                                                      \
    } while (0)
    if (hlc.basis == BASIS_RBF && hlc.norm == NORM_SOFTSIGN) KAN_STEP_GO(NORM_SOFTSIGN, BASIS_RBF);
    else if (hlc.basis == BASIS_RBF && hlc.norm == NORM_TANH_FAST) KAN_STEP_GO(NORM_TANH_FAST, BASIS_RBF);
    else KAN_STEP_GO(NORM_RUNTIME, -1);
#undef KAN_STEP_GO
#undef KAN_STEP_WAVE
    e = hipGetLastError();
    if (e != hipSuccess || !err_out) return e;
    if (parts_out) {
        *parts_out = grid;
        return hipSuccess;
    }
    return launch_stage_error_final(err_slab, grid, err_out, st);
}

// Launch lq of the device-controlled solve (FkLoopArgs): the step kernel's DEV instantiation over a grid of at
// most la.max_grid workgroups (the same grid every launch).  The tables must already be built.
hipError_t launch_fk_step_pp_loop(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, double cd,
                                  double co, int Nx, const double* p, const double* table, const FkLoopArgs& la,
                                  int64_t lq, int64_t B, hipStream_t st, int grid_ovr) {
    const int max_grid = (int)la.max_grid;
    if (!fk_stage_pp_supported(hpc, Nx)) return hipErrorInvalidValue;
    const size_t lds = sizeof(double2) * (kPPCoef / 2) * (size_t)hpc.ni;
#define KAN_LOOP_WAVE(NORM, BASIS, NP)                                                                           \
    do {                                                                                                         \
        static int cap = 0;                                                                                      \
        if (!cap) cap = pp_grid_cap(fk_step_pp_wave_kernel<NORM, BASIS, NP, true>, lds);                        \
        const int gcap = grid_ovr > 0 ? grid_ovr : cap;                                                          \
        const int grid = grid_for(B, kBlock / kWave, gcap < max_grid ? gcap : max_grid);                        \
        hipLaunchKernelGGL((fk_step_pp_wave_kernel<NORM, BASIS, NP, true>), dim3(grid), dim3(kBlock), lds, st,  \
                           lc, p, (const double2*)table, hpc.ni, hpc.inv_w, hpc.x0, cd, co, nullptr, nullptr,  \
                           StepOut{}, StepCoef{}, nullptr, B, la, lq);                                           \
    } while (0)
#define KAN_LOOP_GO(NORM, BASIS)                                                                                 \
    do {                                                                                                         \
        if (Nx == 256) KAN_LOOP_WAVE(NORM, BASIS, 2);                                                            \
        else if (Nx == 128) KAN_LOOP_WAVE(NORM, BASIS, 1);                                                       \
        else KAN_LOOP_WAVE(NORM, BASIS, 4);                                                                      \
    } while (0)
    if (hlc.basis == BASIS_RBF && hlc.norm == NORM_SOFTSIGN) KAN_LOOP_GO(NORM_SOFTSIGN, BASIS_RBF);
    else if (hlc.basis == BASIS_RBF && hlc.norm == NORM_TANH_FAST) KAN_LOOP_GO(NORM_TANH_FAST, BASIS_RBF);
    else KAN_LOOP_GO(NORM_RUNTIME, -1);
#undef KAN_LOOP_GO
#undef KAN_LOOP_WAVE
    return hipGetLastError();
}

// The table VJP covers the recurrence configurations the Fisher-KPP drivers use.
bool fk_vjp_pp_supported(const LayerConst& hlc, int Nx) {
    const bool shape = Nx == 128 || Nx == 256 || Nx == 512;
    const bool cfg = hlc.basis == BASIS_RBF && hlc.path != PATH_DIRECT &&
                     ((hlc.G == 10 && (hlc.norm == NORM_SOFTSIGN || hlc.norm == NORM_TANH_FAST)) ||
                      (hlc.G == 5 && (hlc.norm == NORM_SOFTSIGN || hlc.norm == NORM_TANH_FAST)));
    return shape && cfg;
}

template <int NORM, int PATH, int GT, bool STG>
static hipError_t fk_vjp_pp_go(const PPConst& hpc, const LayerConst* lc, const double* p, const double* tables,
                               double cd, double co, int Nx, const double* u, const double* lam, double* lamJ,
                               double* slab, int slab_blocks, int64_t B, int& grid, const StageArgs<double>& su,
                               const StageArgs<double>& sl, double* lam_out, double* err_slab, hipStream_t st,
                               int grid_ovr) {
    const size_t lds = 2 * sizeof(double2) * (kPPCoef / 2) * (size_t)hpc.ni;
#define KAN_VJP_WAVE(NP, NI)                                                                                      \
    do {                                                                                                         \
        static int cap = 0;                                                                                      \
        if (!cap) cap = pp_grid_cap(fk_vjp_pp_wave_kernel<NORM, PATH, GT, NP, STG, NI>, lds, kVjpBlock);        \
        const int gcap = grid_ovr > 0 ? grid_ovr : cap;                                                          \
        /* the standalone VJP (not a stage): contiguous chunks over a batch-covering grid, chunk */             \
        /* grown until the grid fits the slab */                                                                 \
        int chunk = 0;                                                                                           \
        if (!STG && grid_ovr == 0 && kVjpChunk > 0) {                                                            \
            chunk = kVjpChunk;                                                                                   \
            while ((B + (int64_t)(kVjpBlock / kWave) * chunk - 1) / ((int64_t)(kVjpBlock / kWave) * chunk) >     \
                   slab_blocks)                                                                                  \
                chunk *= 2;                                                                                      \
            grid = grid_for(B, (kVjpBlock / kWave) * chunk, slab_blocks);                                        \
        } else {                                                                                                 \
            grid = grid_for(B, kVjpBlock / kWave, gcap < slab_blocks ? gcap : slab_blocks);                      \
        }                                                                                                        \
        hipLaunchKernelGGL((fk_vjp_pp_wave_kernel<NORM, PATH, GT, NP, STG, NI>), dim3(grid), dim3(kVjpBlock), lds, st, \
                           lc, p, (const double2*)tables, hpc.ni, hpc.inv_w, hpc.x0, cd, co, u, lam, lamJ, slab, B, \
                           su, sl, lam_out, err_slab ? slab + (int64_t)grid * (GT + 1) : nullptr, chunk);        \
    } while (0)
    if (Nx == 256 && !STG && hpc.ni == 256) KAN_VJP_WAVE(2, 256);   // the FK256 tables (w = 1/32 on [-4, 4))
    else if (Nx == 256) KAN_VJP_WAVE(2, 0);
    else if (Nx == 128) KAN_VJP_WAVE(1, 0);
    else KAN_VJP_WAVE(4, 0);
#undef KAN_VJP_WAVE
    return hipGetLastError();
}

template <bool STG>
static hipError_t fk_vjp_pp_dispatch(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const double* p,
                                     const double* tables, double cd, double co, int Nx, const double* u,
                                     const double* lam, double* lamJ, double* slab, int slab_blocks, int64_t B,
                                     int& grid, const StageArgs<double>& su, const StageArgs<double>& sl,
                                     double* lam_out, double* err_slab, hipStream_t st, int grid_ovr) {
#define KAN_VJP_GO(NORM, PATH, GT)                                                                               \
    return fk_vjp_pp_go<NORM, PATH, GT, STG>(hpc, lc, p, tables, cd, co, Nx, u, lam, lamJ, slab, slab_blocks, B, \
                                             grid, su, sl, lam_out, err_slab, st, grid_ovr)
    if (hlc.path == PATH_REC_CORR) {
        if (hlc.G == 10 && hlc.norm == NORM_SOFTSIGN) KAN_VJP_GO(NORM_SOFTSIGN, PATH_REC_CORR, 10);
        else if (hlc.G == 10) KAN_VJP_GO(NORM_TANH_FAST, PATH_REC_CORR, 10);
        else if (hlc.norm == NORM_SOFTSIGN) KAN_VJP_GO(NORM_SOFTSIGN, PATH_REC_CORR, 5);
        else KAN_VJP_GO(NORM_TANH_FAST, PATH_REC_CORR, 5);
    } else {
        if (hlc.G == 10 && hlc.norm == NORM_SOFTSIGN) KAN_VJP_GO(NORM_SOFTSIGN, PATH_REC, 10);
        else if (hlc.G == 10) KAN_VJP_GO(NORM_TANH_FAST, PATH_REC, 10);
        else if (hlc.norm == NORM_SOFTSIGN) KAN_VJP_GO(NORM_SOFTSIGN, PATH_REC, 5);
        else KAN_VJP_GO(NORM_TANH_FAST, PATH_REC, 5);
    }
#undef KAN_VJP_GO
}

hipError_t launch_fk_vjp_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc,
                            const double* p, double* tables, double cd, double co, int Nx, const double* u,
                            const double* lam, double* lamJ, double* dp, double* slab, int slab_blocks, int64_t B,
                            hipStream_t st, bool build, int grid_ovr) {
    if (!fk_vjp_pp_supported(hlc, Nx)) return hipErrorInvalidValue;
    const int fns[2] = {PP_DPHI, PP_SWISH};
    hipError_t e = hipSuccess;
    if (build && (e = launch_fk_pp_build(hpc, lc, pc, p, tables, fns, 2, st)) != hipSuccess) return e;
    int grid = 0;
    const StageArgs<double> none{};
    e = fk_vjp_pp_dispatch<false>(hpc, hlc, lc, p, tables, cd, co, Nx, u, lam, lamJ, slab, slab_blocks, B, grid, none,
                                  none, nullptr, nullptr, st, grid_ovr);
    if (e != hipSuccess || !dp) return e;
    return launch_slab_reduce<double>(slab, grid, hlc.G + (hlc.use_base ? 1 : 0), dp, st);
}

hipError_t launch_fk_vjp_stage_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc,
                                  const double* p, double* tables, double cd, double co, int Nx, const double* u,
                                  const StageArgs<double>& su, const double* lam, const StageArgs<double>& sl,
                                  double* lam_out, double* lamJ, double* dp, bool dp_assign, double* err_out,
                                  double* slab, int slab_blocks, int64_t B, hipStream_t st, bool build,
                                  int* deferred_grid, int grid_ovr) {
    if (!fk_vjp_pp_supported(hlc, Nx)) return hipErrorInvalidValue;
    const int fns[2] = {PP_DPHI, PP_SWISH};
    hipError_t e = hipSuccess;
    if (build && (e = launch_fk_pp_build(hpc, lc, pc, p, tables, fns, 2, st)) != hipSuccess) return e;
    int grid = 0;
    // slab: [grid][P] dC/dW partials, then [grid] error partials (grid <= slab_blocks / 2);
    // with deferred_grid the reduction is left to launch_vjp_finish_jobs
    const int cap = slab_blocks / 2;
    e = fk_vjp_pp_dispatch<true>(hpc, hlc, lc, p, tables, cd, co, Nx, u, lam, lamJ, slab, cap, B, grid, su, sl,
                                 lam_out, err_out ? slab : nullptr, st, grid_ovr);
    if (e != hipSuccess) return e;
    const int P = hlc.G + (hlc.use_base ? 1 : 0);
    if (deferred_grid) {
        *deferred_grid = grid;
        return hipSuccess;
    }
    if (!dp && !err_out) return hipSuccess;
    hipLaunchKernelGGL(vjp_finish_kernel, dim3((unsigned)(dp ? P : 0) + (err_out ? 1 : 0)), dim3(kBlock), 0, st,
                       slab, (int64_t)grid, (int64_t)P, dp, dp_assign ? 1 : 0,
                       slab + (int64_t)grid * (hlc.G + 1), err_out);
    return hipGetLastError();
}

hipError_t launch_fk_vjp_step_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc,
                                 const double* p, double* tables, double cd, double co, int Nx,
                                 const AdjStepArgs& a_in, double* slab_base, int slab_blocks, int64_t B,
                                 int* grid_out, hipStream_t st, bool build, int grid_ovr, bool rows,
                                 int* combined_out, bool* fused_finish_out) {
    if (!fk_vjp_pp_supported(hlc, Nx)) return hipErrorInvalidValue;
    const int fns[2] = {PP_DPHI, PP_SWISH};
    hipError_t e = hipSuccess;
    if (build && (e = launch_fk_pp_build(hpc, lc, pc, p, tables, fns, 2, st)) != hipSuccess) return e;
    const size_t lds = 2 * sizeof(double2) * (kPPCoef / 2) * (size_t)hpc.ni;
    const int P = hlc.G + (hlc.use_base ? 1 : 0);
    AdjStepArgs a = a_in;
    int grid = 0;
    // one row per wave, the row's stages in registers, where the grid of one row per wave fits the slab
    const bool use_rows = rows && grid_ovr == 0 && Nx <= 256 && B <= (int64_t)(kVjpBlock / kWave) * slab_blocks;
    // only the rows kernel combines: fixed steps (1) through A alone, adaptive steps (2) through A and the
    // μ error combination E (the caller asks for 2 with the error slab)
    if (!use_rows || (a.err_slab && a.combine != 2) || (!a.err_slab && a.combine == 2)) a.combine = 0;
    if (combined_out) *combined_out = a.combine;
    // the fused finish: the combined adaptive rows step with at least 1 + P workgroups
    if (a.combine != 2 || grid_for(B, kVjpBlock / kWave, slab_blocks) < P + 1) a.fin_ctr = nullptr;
    if (fused_finish_out) *fused_finish_out = a.fin_ctr != nullptr;
    // the arrival counters start every fused launch at zero (a timed-out wait in an earlier launch
    // may leave a late arrival behind in them, which would let the next launch's finishers start early)
    if (a.fin_ctr && (e = hipMemsetAsync(a.fin_ctr, 0, 2 * sizeof(unsigned), st)) != hipSuccess) return e;
    a.reload[0] = 1;
    for (int s = 1; s < 6; ++s) {
        bool same = a.su_u[s] == a.su_u[s - 1];
        for (int m = 0; m < 4; ++m) same = same && a.su_q[s][m] == a.su_q[s - 1][m];
        a.reload[s] = same ? 0 : 1;
    }
#define KAN_VSTEP(NORM, PATH, GT, NP)                                                                              \
    do {                                                                                                         \
        if (use_rows) {                                                                                          \
            grid = grid_for(B, kVjpBlock / kWave, slab_blocks);                                                  \
            for (int s = 0; s < 6; ++s) a.slab[s] = slab_base + (int64_t)s * grid * P;                            \
            if (a.err_slab) a.err_slab = slab_base + (int64_t)6 * grid * P;                                       \
            if (a.fin_ctr) {                                                                                     \
                const int which[3] = {0, 1, 5}; /* A, E, kμ_7 (as kanode_internal_fk_adjoint_step) */            \
                for (int q = 0; q < 3; ++q) {                                                                    \
                    a.fin.slab[q] = a.slab[which[q]];                                                            \
                    a.fin.ca[q] = q == 0 ? 1.0 : 0.0;                                                            \
                    a.fin.ce[q] = q == 1 ? 1.0 : 0.0;                                                            \
                }                                                                                                \
                a.fin.nslab = 3;                                                                                 \
                a.fin.k7 = 2;                                                                                    \
                a.fin.tr = 1;                                                                                    \
                a.fin.nblk = grid;                                                                               \
                a.fin.err_slab = a.err_slab;                                                                     \
            }                                                                                                    \
            if (KAN_VROWS_NI && NP == 2 && hpc.ni == 256) {                                                     \
                if (a.combine == 2)                                                                              \
                    hipLaunchKernelGGL((fk_vjp_step_rows_kernel<NORM, PATH, GT, 2, 2, 256>), dim3(grid),           \
                                       dim3(kVjpBlock), lds, st, lc, p, (const double2*)tables, hpc.ni, hpc.inv_w,\
                                       hpc.x0, cd, co, B, a);                                   \
                else                                                                                             \
                    hipLaunchKernelGGL((fk_vjp_step_rows_kernel<NORM, PATH, GT, 2, 0, 256>), dim3(grid),           \
                                       dim3(kVjpBlock), lds, st, lc, p, (const double2*)tables, hpc.ni, hpc.inv_w,\
                                       hpc.x0, cd, co, B, a);                                   \
            } else if (a.combine == 2)                                                                           \
                hipLaunchKernelGGL((fk_vjp_step_rows_kernel<NORM, PATH, GT, (NP < 4 ? NP : 2), 2>), dim3(grid),    \
                                   dim3(kVjpBlock), lds, st, lc, p, (const double2*)tables, hpc.ni, hpc.inv_w,    \
                                   hpc.x0, cd, co, B, a);                                       \
            else                                                                                                 \
                hipLaunchKernelGGL((fk_vjp_step_rows_kernel<NORM, PATH, GT, (NP < 4 ? NP : 2), 0>), dim3(grid),    \
                                   dim3(kVjpBlock), lds, st, lc, p, (const double2*)tables, hpc.ni, hpc.inv_w,    \
                                   hpc.x0, cd, co, B, a);                                       \
            break;                                                                                               \
        }                                                                                                        \
        static int cap = 0;                                                                                      \
        if (!cap) cap = pp_grid_cap(fk_vjp_step_pp_wave_kernel<NORM, PATH, GT, NP>, lds, kVjpBlock);             \
        const int gcap = grid_ovr > 0 ? grid_ovr : cap;                                                          \
        grid = grid_for(B, kVjpBlock / kWave, gcap < slab_blocks ? gcap : slab_blocks);                            \
        for (int s = 0; s < 6; ++s) a.slab[s] = slab_base + (int64_t)s * grid * P;                                \
        if (a.err_slab) a.err_slab = slab_base + (int64_t)6 * grid * P;                                           \
        hipLaunchKernelGGL((fk_vjp_step_pp_wave_kernel<NORM, PATH, GT, NP>), dim3(grid), dim3(kVjpBlock), lds, st,  \
                           lc, p, (const double2*)tables, hpc.ni, hpc.inv_w, hpc.x0, cd, co, B, a);              \
    } while (0)
#define KAN_VSTEP_NP(NORM, PATH, GT)                                                                              \
    do {                                                                                                         \
        if (Nx == 256) KAN_VSTEP(NORM, PATH, GT, 2);                                                             \
        else if (Nx == 128) KAN_VSTEP(NORM, PATH, GT, 1);                                                        \
        else KAN_VSTEP(NORM, PATH, GT, 4);                                                                       \
    } while (0)
    if (hlc.path == PATH_REC_CORR) {
        if (hlc.G == 10 && hlc.norm == NORM_SOFTSIGN) KAN_VSTEP_NP(NORM_SOFTSIGN, PATH_REC_CORR, 10);
        else if (hlc.G == 10) KAN_VSTEP_NP(NORM_TANH_FAST, PATH_REC_CORR, 10);
        else if (hlc.norm == NORM_SOFTSIGN) KAN_VSTEP_NP(NORM_SOFTSIGN, PATH_REC_CORR, 5);
        else KAN_VSTEP_NP(NORM_TANH_FAST, PATH_REC_CORR, 5);
    } else {
        if (hlc.G == 10 && hlc.norm == NORM_SOFTSIGN) KAN_VSTEP_NP(NORM_SOFTSIGN, PATH_REC, 10);
        else if (hlc.G == 10) KAN_VSTEP_NP(NORM_TANH_FAST, PATH_REC, 10);
        else if (hlc.norm == NORM_SOFTSIGN) KAN_VSTEP_NP(NORM_SOFTSIGN, PATH_REC, 5);
        else KAN_VSTEP_NP(NORM_TANH_FAST, PATH_REC, 5);
    }
#undef KAN_VSTEP_NP
#undef KAN_VSTEP
    *grid_out = grid;
    return hipGetLastError();
}

// One attempt of the device-controlled adaptive adjoint (kan_adjloop.hpp): the rows kernel's DEV instantiation
// over la.grid workgroups and the finish launch with the controller.  Supported where launch_fk_vjp_step_pp
// takes the rows kernel with the combined adaptive step (fk_adjoint_loop_supported).
bool fk_adjoint_loop_supported(const PPConst& hpc, const LayerConst& hlc, int Nx) {
    return fk_vjp_pp_supported(hlc, Nx) && (Nx == 128 || Nx == 256) && hpc.ni > 0;
}
int fk_adjoint_loop_grid(int64_t B, int slab_blocks) {   // the rows step's grid (0: the batch is above its cap)
    return B >= 1 && B <= (int64_t)(kVjpBlock / kWave) * slab_blocks ? grid_for(B, kVjpBlock / kWave, slab_blocks) : 0;
}
hipError_t launch_fk_adjoint_loop(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc,
                                  const double* p, double* tables, double cd, double co, int Nx, const AdjLoopArgs& la,
                                  int64_t B, hipStream_t st, bool build) {
    if (!fk_adjoint_loop_supported(hpc, hlc, Nx) || la.grid < 1) return hipErrorInvalidValue;
    const int fns[2] = {PP_DPHI, PP_SWISH};
    hipError_t e = hipSuccess;
    if (build && (e = launch_fk_pp_build(hpc, lc, pc, p, tables, fns, 2, st)) != hipSuccess) return e;
    const size_t lds = 2 * sizeof(double2) * (kPPCoef / 2) * (size_t)hpc.ni;
#define KAN_ALOOP(NORM, PATH, GT)                                                                                 \
    do {                                                                                                         \
        if (Nx == 256 && hpc.ni == 256)                                                                          \
            hipLaunchKernelGGL((fk_vjp_step_rows_loop_kernel<NORM, PATH, GT, 2, 2, 256>), dim3(la.grid),          \
                               dim3(kVjpBlock), lds, st, lc, p, (const double2*)tables, hpc.ni, hpc.inv_w, hpc.x0,  \
                               cd, co, B, la.ctl, la.plan);                                                 \
        else if (Nx == 256)                                                                                      \
            hipLaunchKernelGGL((fk_vjp_step_rows_loop_kernel<NORM, PATH, GT, 2, 2, 0>), dim3(la.grid),            \
                               dim3(kVjpBlock), lds, st, lc, p, (const double2*)tables, hpc.ni, hpc.inv_w, hpc.x0,  \
                               cd, co, B, la.ctl, la.plan);                                                 \
        else                                                                                                     \
            hipLaunchKernelGGL((fk_vjp_step_rows_loop_kernel<NORM, PATH, GT, 1, 2, 0>), dim3(la.grid),            \
                               dim3(kVjpBlock), lds, st, lc, p, (const double2*)tables, hpc.ni, hpc.inv_w, hpc.x0,  \
                               cd, co, B, la.ctl, la.plan);                                                 \
    } while (0)
    if (hlc.path == PATH_REC_CORR) {
        if (hlc.G == 10 && hlc.norm == NORM_SOFTSIGN) KAN_ALOOP(NORM_SOFTSIGN, PATH_REC_CORR, 10);
        else if (hlc.G == 10) KAN_ALOOP(NORM_TANH_FAST, PATH_REC_CORR, 10);
        else if (hlc.norm == NORM_SOFTSIGN) KAN_ALOOP(NORM_SOFTSIGN, PATH_REC_CORR, 5);
        else KAN_ALOOP(NORM_TANH_FAST, PATH_REC_CORR, 5);
    } else {
        if (hlc.G == 10 && hlc.norm == NORM_SOFTSIGN) KAN_ALOOP(NORM_SOFTSIGN, PATH_REC, 10);
        else if (hlc.G == 10) KAN_ALOOP(NORM_TANH_FAST, PATH_REC, 10);
        else if (hlc.norm == NORM_SOFTSIGN) KAN_ALOOP(NORM_SOFTSIGN, PATH_REC, 5);
        else KAN_ALOOP(NORM_TANH_FAST, PATH_REC, 5);
    }
#undef KAN_ALOOP
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(adj_finish_loop_kernel, dim3((unsigned)la.P + 1), dim3(kAdjFinBlock), 0, st, la);
    return hipGetLastError();
}

#ifdef KAN_CLOCK_PROBE
extern "C" int kan_clock_probe_read(unsigned long long* out) {   // [32]: slot 0 clocks, realtime; slot 1 ...; phases
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(kan_clock_probe), sizeof(unsigned long long) * 32);
}
extern "C" int kan_clock_probe_reset() {
    const unsigned long long z[32] = {};
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(kan_clock_probe), z, sizeof(z));
}
#endif
}  // namespace kan
