// kan_device.hpp — device-side math for the KAN-ODE hot path on gfx950 (CDNA4).
//
// Scalar semantics restate the reference (file:line relative to /root/reference):
//   normalizer / base activation  Lotka-Volterra/src/kdense.jl:25-31,57-61,116,123
//   rbf / rswaf / iqf + pullbacks Lotka-Volterra/src/utils.jl:8-62
//   NNlib 0.9.24 tanh_fast, sigmoid, sigmoid_fast, swish, softsign and their
//   rrules (Lotka-Volterra/Manifest.toml:1776).
//
// fp64 is VALU-bound on MI355X (a wave64 fp64 op occupies a SIMD for 4 cycles;
// measured ~1.87 GHz under this load), so the fp64 elementary functions are
// written for VALU instruction count:
//   exp  — x·256/ln2 rounded by the 1.5·2^52 magic add (no rndne/cvt), |r| <= ln2/512,
//          2^(j/256) from a 256-entry LDS table, degree-4 Taylor (remainder 3.7e-17),
//          one ldexp: 13 VALU, <= 2 ulp.
//   rcp  — v_rcp_f64 + two Newton steps (0.5-1 ulp); a/b = a·rcp(b).
// fp32 uses the hardware-accelerated library functions.
//
// The RBF basis on the reference's uniform Float32 knot grid is evaluated with a
// left-anchored Gaussian recurrence:
//     z_j = z_0 - Δ_j,  Δ_j = (g_j - g_0)·s = j·δ + e_j   (e_j: Float32 knot rounding)
//     exp(-z_j²) = exp(-z_0²) · R^j · exp(-Δ_j²) · exp(2 z_0 e_j),  R = exp(2 z_0 δ)
// i.e. 2 exp per input element instead of G.  exp(-z_0²) is formed from the exact
// square z_0² = p + perr (fma); exp(2 z_0 e_j) = exp(τ_c e_j)·exp(τ' e_j) with
// τ' = 2 z_0 - τ_c centred on the normalizer's range, the first factor folded into
// the constants and the second taken to 2nd order (|τ' e_j| <= 1.1e-6 for G=10).
// Relative error vs per-knot exp: <= ~3e-15 of Σ|C_j φ_j| (tools/ and tests).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kan_exp_table.hpp"

namespace kan {

constexpr int kMaxGrid = 32;    // knots per layer handled by the kernels
constexpr int kMaxLayers = 8;

enum Norm : int { NORM_TANH_FAST = 0, NORM_TANH = 1, NORM_SOFTSIGN = 2, NORM_SIGMOID = 3,
                  NORM_SIGMOID_FAST = 4, NORM_IDENTITY = 5, NORM_RUNTIME = -1 };
enum Basis : int { BASIS_RBF = 0, BASIS_RSWAF = 1, BASIS_IQF = 2 };
// basis evaluation path chosen on the host from the layer's constants
enum Path : int { PATH_DIRECT = 0, PATH_REC = 1, PATH_REC_CORR = 2 };

// Per-layer constants, computed once on the host at handle creation and stored
// in a device buffer (wave-uniform reads -> scalar loads).
struct LayerConst {
    int32_t I, O, G;
    int32_t norm, basis, use_base, iqf_quirk, path;
    int64_t p_off;            // offset of this layer's C in the flat parameter vector
    int64_t w_off;            // offset of W (p_off + O*G*I)
    float grid[kMaxGrid];     // Float32 knots (LinRange semantics, kdense.jl:90)
    float invh;               // Float32 1/h (utils.jl:9)
    int32_t unit_delta;       // δ == 1 exactly (default grids): R = exp(2 z0)
    double g0, s, delta;      // recurrence anchor constants (f64; cast per dtype)
    double gs;                // -g0·s  (z0 = fma(n, s, gs))
    double tau_c;             // centre of 2·z0 over the normalizer's range
    double K[kMaxGrid];       // exp(-Δ_j²) · exp(tau_c·e_j)
    double e[kMaxGrid];       // Δ_j - j·δ
    double Dl[kMaxGrid];      // Δ_j
    double h2[kMaxGrid];      // 0.5·e_j·e_j as the kernels form it, (0.5·e_j)·e_j: the 2nd-order correction weight
};

// Piecewise-polynomial form of a pointwise KDense(1,1,G) (kan_pp.hip): φ(u) on
// [lo, -lo) cut into `ni` intervals of width w (a power of two), each a degree-9
// polynomial in t = 2(x - k) - 1, x = u/w + ni/2.  Built per launch from p.
constexpr int kPPCoef = 10;
constexpr int kPPChecks = 3;
constexpr int kPPMaxIntervals = 512;
constexpr int kPPMaxFns = 3;
enum PPFn : int { PP_PHI = 0, PP_DPHI = 1, PP_SWISH = 2 };   // tabulated functions (slot = id)
constexpr int kPPPerBlock = 4;   // intervals built per block of fk_pp_build_kernel (13·4·4 = 208 lanes)
// After the kPPMaxFns table slots (kPPCoef·ni doubles each), one stamp per slot and build block: the parameters
// C_0..C_{G-1}, W that block's intervals were last built from and a valid flag (fk_pp_build_kernel: a block
// skips its build when p matches its own stamp; each block reads and writes only its own, so no block waits for
// another).  pp_tables_doubles() sizes the whole buffer.
constexpr int kPPStampValid = kMaxGrid + 1;
constexpr int kPPStampRejected = kMaxGrid + 2;   // intervals of the block the last build rejected (direct formula)
constexpr int kPPStampStride = kMaxGrid + 3;
__host__ __device__ inline double* pp_stamp(double* tables, int ni, int fn, int blk) {
    return tables + (int64_t)kPPMaxFns * kPPCoef * ni + ((int64_t)fn * (ni / kPPPerBlock) + blk) * kPPStampStride;
}
inline int64_t pp_tables_doubles(int ni) {
    return (int64_t)kPPMaxFns * kPPCoef * ni + (int64_t)kPPMaxFns * (ni / kPPPerBlock) * kPPStampStride;
}
struct PPConst {
    int32_t ni;                       // intervals (power of two, multiple of 16)
    int32_t enabled;                  // host admissibility (f64, rbf/rswaf, even Nx)
    double w, inv_w, x0, lo;          // width, 1/w, ni/2, -ni·w/2
    double tol;                       // acceptance: |poly - direct| <= tol·Σ|terms| at the checks
    double xi[kPPCoef];               // Chebyshev nodes cos(π(2m+1)/20)
    double tchk[kPPChecks];           // acceptance points in t
    double Q[kPPCoef][kPPCoef];       // node values -> monomial coefficients in t
};

// Every kernel that evaluates fp64 exponentials stages the table in LDS once.
#define KAN_EXP_TABLE_LDS(name)                                                         \
    __shared__ double name[256];                                                        \
    for (int i_ = threadIdx.x; i_ < 256; i_ += blockDim.x) name[i_] = kExp2Tab256[i_]; \
    __syncthreads();

// ---------------------------------------------------------------------------
// elementary functions, per dtype
template <typename T> struct Math;

template <> struct Math<double> {
    const double* __restrict__ tab;   // LDS copy of kExp2Tab256
    // exp for -745 <= x <= 709 (no special-case handling; callers bound or clamp x)
    __device__ __forceinline__ double exp(double x) const {
        const double magic = 0x1.8p52;
        const double t = ::fma(x, k256oLn2, magic);      // round(x·256/ln2) in the low mantissa bits
        const int k = (int)__double2loint(t);
        const double kd = t - magic;
        double r = ::fma(-kd, kLn2o256Hi, x);
        r = ::fma(-kd, kLn2o256Lo, r);
        double p = ::fma(r, 0x1.5555555555555p-5, 0x1.5555555555555p-3);   // 1/24, 1/6
        p = ::fma(r, p, 0.5);
        p = ::fma(r, p, 1.0);
        p = ::fma(r, p, 1.0);
        return __builtin_amdgcn_ldexp(tab[k & 255] * p, k >> 8);
    }
    // exp of a non-positive argument, clamped below (underflow -> 0)
    // exp of a non-positive argument (underflow -> 0).  Only |x| < 5.8e6 keeps the int32
    // exponent exact; clamp there (ldexp flushes anything below -1075 to 0 anyway).
    __device__ __forceinline__ double exp_neg(double x) const { return exp(x < -7.0e5 ? -7.0e5 : x); }
    __device__ __forceinline__ double exp_clamped(double x) const { return exp(fmin(fmax(x, -745.0), 709.0)); }
    __device__ __forceinline__ double rcp(double d) const {
        double r = __builtin_amdgcn_rcp(d);
        double e = ::fma(-d, r, 1.0);
        r = ::fma(r, e, r);
        e = ::fma(-d, r, 1.0);
        return ::fma(r, e, r);
    }
    __device__ __forceinline__ double div(double a, double d) const { return a * rcp(d); }
    __device__ __forceinline__ double fma(double a, double b, double c) const { return ::fma(a, b, c); }
    __device__ __forceinline__ double tanh(double x) const { return ::tanh(x); }
};

template <> struct Math<float> {
    const double* __restrict__ tab;   // unused
    __device__ __forceinline__ float exp(float x) const { return ::expf(x); }
    __device__ __forceinline__ float exp_neg(float x) const { return ::expf(x); }
    __device__ __forceinline__ float exp_clamped(float x) const { return ::expf(x); }
    __device__ __forceinline__ float rcp(float d) const { return 1.0f / d; }
    __device__ __forceinline__ float div(float a, float d) const { return a / d; }
    __device__ __forceinline__ float fma(float a, float b, float c) const { return ::fmaf(a, b, c); }
    __device__ __forceinline__ float tanh(float x) const { return ::tanhf(x); }
};

// Move a wave-uniform value into SGPRs (v_readfirstlane): coefficients computed
// once per thread with VALU ops then live in SGPRs and feed VALU ops as the one
// scalar operand, instead of occupying VGPRs (occupancy).
__device__ __forceinline__ double to_sgpr(double v) {
    const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
    const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ float to_sgpr(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

__device__ __forceinline__ double kabs(double x) { return __builtin_fabs(x); }   // |x| source modifier
__device__ __forceinline__ float kabs(float x) { return __builtin_fabsf(x); }
template <typename T> __device__ __forceinline__ T kfma(T a, T b, T c);
template <> __device__ __forceinline__ double kfma<double>(double a, double b, double c) { return ::fma(a, b, c); }
template <> __device__ __forceinline__ float kfma<float>(float a, float b, float c) { return ::fmaf(a, b, c); }

// NNlib.tanh_fast (Float64: exp form + small-|x| polynomial; Float32: rational)
__device__ __forceinline__ double tanh_fast(const Math<double>& M, double x) {
    const double x2 = x * x;
    double p = -0.008697141630499953;
    p = ::fma(x2, p, 0.02186660872609521);
    p = ::fma(x2, p, -0.05396823125794372);
    p = ::fma(x2, p, 0.13333333325511604);
    p = ::fma(x2, p, -0.33333333333324583);
    p = ::fma(x2, p, 1.0);
    const double ypoly = x * p;
    const double e2x = M.exp(fmin(fmax(x + x, -700.0), 700.0));
    const double y = (e2x - 1.0) * M.rcp(e2x + 1.0);
    const double sg = x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : x);
    return x2 > 900.0 ? sg : (x2 < 0.017 ? ypoly : y);
}
__device__ __forceinline__ float tanh_fast(const Math<float>&, float x) {
    const float x2 = x * x;
    float n = 1.587199e-8f;
    n = fmaf(x2, n, 2.2332108e-5f);
    n = fmaf(x2, n, 0.0035974074f);
    n = fmaf(x2, n, 0.1346604f);
    n = fmaf(x2, n, 1.0f);
    float d = 8.7767893e-7f;
    d = fmaf(x2, d, 0.0003453992f);
    d = fmaf(x2, d, 0.026262015f);
    d = fmaf(x2, d, 0.4679937f);
    d = fmaf(x2, d, 1.0f);
    const float sg = x > 0.f ? 1.f : (x < 0.f ? -1.f : x);
    return x2 < 66.0f ? x * (n / d) : sg;
}

// NNlib.sigmoid: t = exp(-|x|); x >= 0 ? 1/(1+t) : t/(1+t)
template <typename T> __device__ __forceinline__ T sigmoid(const Math<T>& M, T x) {
    const T t = M.exp_neg(-kabs(x));
    return (x >= T(0) ? T(1) : t) * M.rcp(T(1) + t);
}
template <typename T> __device__ __forceinline__ T sigmoid_fast(const Math<T>& M, T x) {
    const T y = sigmoid(M, x);
    return x > T(40) ? T(1) : (x < T(-80) ? T(0) : y);
}
// swish(x) = x * sigmoid(x): one exp + one reciprocal
template <typename T> __device__ __forceinline__ T swish(const Math<T>& M, T x) { return x * sigmoid(M, x); }
// swish and its rrule derivative  Ω + sigmoid_fast(x)(1 - Ω)  sharing one exp
template <typename T> __device__ __forceinline__ void swish_and_grad(const Math<T>& M, T x, T& om, T& d) {
    const T sg = sigmoid(M, x);
    om = x * sg;
    const T sf = x > T(40) ? T(1) : (x < T(-80) ? T(0) : sg);
    d = om + sf * (T(1) - om);
}
template <typename T> __device__ __forceinline__ T softsign(const Math<T>& M, T x) { return M.div(x, T(1) + kabs(x)); }

// normalizer; NORM >= 0 selects at compile time, NORM_RUNTIME switches on `rt`
template <int NORM, typename T> __device__ __forceinline__ T normalize(const Math<T>& M, int rt, T x) {
    const int n = NORM < 0 ? rt : NORM;
    if (n == NORM_SOFTSIGN) return softsign(M, x);
    if (n == NORM_TANH_FAST) return tanh_fast(M, x);
    if (n == NORM_TANH) return M.tanh(x);
    if (n == NORM_SIGMOID) return sigmoid(M, x);
    if (n == NORM_SIGMOID_FAST) return sigmoid_fast(M, x);
    return x;
}
// rrule derivative in NNlib's Ω form
template <int NORM, typename T> __device__ __forceinline__ T dnormalize(int rt, T om) {
    const int n = NORM < 0 ? rt : NORM;
    switch (n) {
    case NORM_TANH_FAST:
    case NORM_TANH: return T(1) - om * om;
    case NORM_SOFTSIGN: { const T a = T(1) - kabs(om); return a * a; }
    case NORM_SIGMOID:
    case NORM_SIGMOID_FAST: return om * (T(1) - om);
    default: return T(1);
    }
}

// direct basis value (utils.jl:13,32-34,54); aux = tanh(y) for rswaf
template <typename T> __device__ __forceinline__ T basis_direct(const Math<T>& M, int basis, T y, T& aux) {
    if (basis == BASIS_RBF) return M.exp_neg(-(y * y));
    if (basis == BASIS_RSWAF) { aux = M.tanh(y); return T(1) - aux * aux; }
    return M.rcp(T(1) + y * y);
}
// pullback dy for a basis value (utils.jl:15-21, 36-42, 56-62)
template <typename T> __device__ __forceinline__ T basis_pull(int basis, int iqf_quirk, T y, T phi, T aux, T bbar) {
    if (basis == BASIS_RBF) return T(-2) * y * phi * bbar;
    if (basis == BASIS_RSWAF) return T(-2) * aux * phi * bbar;
    return iqf_quirk ? T(-2) * y * phi * bbar : T(-2) * y * phi * phi * bbar;
}

// The recurrence's per-layer scalars, hoisted into registers once per thread
// (reading them through the LayerConst pointer inside the loop re-issues scalar
// loads whose lgkmcnt waits serialise with the LDS exp-table reads).
template <typename T> struct RecScalars {
    T s, gs, delta, tau_c;
    int unit_delta;
    __device__ __forceinline__ explicit RecScalars(const LayerConst& lc)
        : s(T(lc.s)), gs(T(lc.gs)), delta(T(lc.delta)), tau_c(T(lc.tau_c)), unit_delta(lc.unit_delta) {}
};

// Recurrence anchor for a normalised input n:
//   z0 = (n - g0)·s,  E0 = exp(-z0²) (exact square),  R = exp(2 z0 δ),  τ' = 2 z0 - τ_c
template <typename T> __device__ __forceinline__ void rec_anchor(const Math<T>& M, const RecScalars<T>& rc, T n, T& z0,
                                                                  T& E0, T& R, T& taup) {
    z0 = kfma<T>(n, rc.s, rc.gs);
    const T p2 = z0 * z0;
    const T perr = kfma<T>(z0, z0, -p2);          // z0² = p2 + perr exactly
    const T E = M.exp(-p2);
    E0 = kfma<T>(-E, perr, E);                    // exp(-p2 - perr), |perr| <= ulp(p2)/2
    const T tw = z0 + z0;                         // the correction exp(2 z0 e_j) is in 2·z0
    R = M.exp(tw * rc.delta);                     // (δ = 1 exactly on the default grids: the same bits as exp(tw))
    taup = tw - rc.tau_c;
}
template <typename T> __device__ __forceinline__ void rec_anchor(const Math<T>& M, const LayerConst& lc, T n, T& z0,
                                                                  T& E0, T& R, T& taup) {
    rec_anchor<T>(M, RecScalars<T>(lc), n, z0, E0, R, taup);
}

}  // namespace kan
