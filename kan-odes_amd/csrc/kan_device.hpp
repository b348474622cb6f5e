// kan_device.hpp — device-side math for the KAN-ODE hot path on gfx950 (CDNA4).
//
// Scalar semantics restate the reference (file:line relative to /root/reference):
//   normalizer / base activation  Lotka-Volterra/src/kdense.jl:25-31,57-61,116,123
//   rbf / rswaf / iqf + pullbacks Lotka-Volterra/src/utils.jl:8-62
//   NNlib 0.9.24 tanh_fast, sigmoid, sigmoid_fast, swish, softsign and their
//   rrules (Lotka-Volterra/Manifest.toml:1776).
//
// The RBF basis on the reference's uniform Float32 knot grid is evaluated with a
// left-anchored Gaussian recurrence:
//     z_j = z_0 - Δ_j,  Δ_j = (g_j - g_0)·s = j·δ + e_j   (e_j: Float32 knot rounding)
//     exp(-z_j²) = exp(-z_0²) · R^j · exp(-Δ_j²) · exp(2 z_0 e_j),  R = exp(2 z_0 δ)
// i.e. 2 exp per input element instead of G, with exp(-z_0²) formed from the
// exact square z_0² = p + perr (fma) and exp(2 z_0 e_j) by its 2nd-order Taylor
// series (|2 z_0 e_j| < 3e-6).  Relative error vs per-knot exp: <= ~12 ulp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kan {

constexpr int kMaxGrid = 32;    // knots per layer handled by the kernels
constexpr int kMaxLayers = 8;

enum Norm : int { NORM_TANH_FAST = 0, NORM_TANH = 1, NORM_SOFTSIGN = 2, NORM_SIGMOID = 3,
                  NORM_SIGMOID_FAST = 4, NORM_IDENTITY = 5 };
enum Basis : int { BASIS_RBF = 0, BASIS_RSWAF = 1, BASIS_IQF = 2 };
// basis evaluation path chosen on the host from the layer's constants
enum Path : int { PATH_DIRECT = 0, PATH_REC = 1, PATH_REC_CORR = 2 };

// Per-layer constants, computed once on the host at handle creation and passed
// by value as a kernel argument (lives in the kernarg segment -> SGPR loads).
struct LayerConst {
    int32_t I, O, G;
    int32_t norm, basis, use_base, iqf_quirk, path;
    int64_t p_off;            // offset of this layer's C in the flat parameter vector
    int64_t w_off;            // offset of W (p_off + O*G*I)
    float grid[kMaxGrid];     // Float32 knots (LinRange semantics, kdense.jl:90)
    float invh;               // Float32 1/h (utils.jl:9)
    double g0, s, delta;      // recurrence anchor constants (f64; cast per dtype)
    double K[kMaxGrid];       // exp(-Δ_j²)
    double e[kMaxGrid];       // Δ_j - j·δ
    double Dl[kMaxGrid];      // Δ_j
};

// ---------------------------------------------------------------------------
// elementary functions
template <typename T> __device__ __forceinline__ T kexp(T x);
template <> __device__ __forceinline__ double kexp<double>(double x) { return exp(x); }
template <> __device__ __forceinline__ float kexp<float>(float x) { return expf(x); }
template <typename T> __device__ __forceinline__ T ktanh(T x);
template <> __device__ __forceinline__ double ktanh<double>(double x) { return tanh(x); }
template <> __device__ __forceinline__ float ktanh<float>(float x) { return tanhf(x); }
template <typename T> __device__ __forceinline__ T kabs(T x) { return x < T(0) ? -x : x; }
template <typename T> __device__ __forceinline__ T kfma(T a, T b, T c);
template <> __device__ __forceinline__ double kfma<double>(double a, double b, double c) { return fma(a, b, c); }
template <> __device__ __forceinline__ float kfma<float>(float a, float b, float c) { return fmaf(a, b, c); }

// NNlib.tanh_fast (Float64: exp form + small-|x| polynomial; Float32: rational)
__device__ __forceinline__ double tanh_fast(double x) {
    const double x2 = x * x;
    double p = -0.008697141630499953;
    p = fma(x2, p, 0.02186660872609521);
    p = fma(x2, p, -0.05396823125794372);
    p = fma(x2, p, 0.13333333325511604);
    p = fma(x2, p, -0.33333333333324583);
    p = fma(x2, p, 1.0);
    const double ypoly = x * p;
    const double e2x = exp(fmin(x + x, 700.0));
    const double y = (e2x - 1.0) / (e2x + 1.0);
    const double sg = x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : x);
    return x2 > 900.0 ? sg : (x2 < 0.017 ? ypoly : y);
}
__device__ __forceinline__ float tanh_fast(float x) {
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
template <typename T> __device__ __forceinline__ T sigmoid(T x) {
    const T t = kexp<T>(-kabs(x));
    return (x >= T(0) ? T(1) : t) / (T(1) + t);
}
template <typename T> __device__ __forceinline__ T sigmoid_fast(T x) {
    const T y = sigmoid(x);
    return x > T(40) ? T(1) : (x < T(-80) ? T(0) : y);
}
// swish(x) = x * sigmoid(x), one exp + one division
template <typename T> __device__ __forceinline__ T swish(T x) {
    const T t = kexp<T>(-kabs(x));
    return x * ((x >= T(0) ? T(1) : t) / (T(1) + t));
}
// swish and its rrule derivative  Ω + sigmoid_fast(x)(1 - Ω)  sharing one exp
template <typename T> __device__ __forceinline__ void swish_and_grad(T x, T& om, T& d) {
    const T t = kexp<T>(-kabs(x));
    const T sg = (x >= T(0) ? T(1) : t) / (T(1) + t);
    om = x * sg;
    const T sf = x > T(40) ? T(1) : (x < T(-80) ? T(0) : sg);
    d = om + sf * (T(1) - om);
}
template <typename T> __device__ __forceinline__ T softsign(T x) { return x / (T(1) + kabs(x)); }

template <typename T> __device__ __forceinline__ T normalize(int norm, T x) {
    switch (norm) {
    case NORM_TANH_FAST: return tanh_fast(x);
    case NORM_TANH: return ktanh<T>(x);
    case NORM_SOFTSIGN: return softsign(x);
    case NORM_SIGMOID: return sigmoid(x);
    case NORM_SIGMOID_FAST: return sigmoid_fast(x);
    default: return x;
    }
}
// rrule derivative in NNlib's Ω form
template <typename T> __device__ __forceinline__ T dnormalize(int norm, T om) {
    switch (norm) {
    case NORM_TANH_FAST:
    case NORM_TANH: return T(1) - om * om;
    case NORM_SOFTSIGN: { const T a = T(1) - kabs(om); return a * a; }
    case NORM_SIGMOID:
    case NORM_SIGMOID_FAST: return om * (T(1) - om);
    default: return T(1);
    }
}

// direct basis value (utils.jl:13,32-34,54); aux = tanh(y) for rswaf
template <typename T> __device__ __forceinline__ T basis_direct(int basis, T y, T& aux) {
    if (basis == BASIS_RBF) return kexp<T>(-(y * y));
    if (basis == BASIS_RSWAF) { aux = ktanh<T>(y); return T(1) - aux * aux; }
    return T(1) / (T(1) + y * y);
}
// pullback dy for a basis value (utils.jl:15-21, 36-42, 56-62)
template <typename T> __device__ __forceinline__ T basis_pull(int basis, int iqf_quirk, T y, T phi, T aux, T bbar) {
    if (basis == BASIS_RBF) return T(-2) * y * phi * bbar;
    if (basis == BASIS_RSWAF) return T(-2) * aux * phi * bbar;
    return iqf_quirk ? T(-2) * y * phi * bbar : T(-2) * y * phi * phi * bbar;
}

// Recurrence anchor: E0 = exp(-z0²) with exact square, R = exp(2 z0 δ).
template <typename T> __device__ __forceinline__ void rec_anchor(const LayerConst& lc, T n, T& z0, T& E0, T& R) {
    z0 = (n - T(lc.g0)) * T(lc.s);
    const T p2 = z0 * z0;
    const T perr = kfma<T>(z0, z0, -p2);          // z0² = p2 + perr exactly
    E0 = kexp<T>(-p2) * (T(1) - perr);            // exp(-p2 - perr), |perr| <= ulp(p2)/2
    R = kexp<T>((z0 + z0) * T(lc.delta));
}

// All G basis values of one normalised input n (into phi[]), plus z_j for the
// pullback (zv[]).  PATH_DIRECT matches the reference formula term by term.
template <typename T, int PATH>
__device__ __forceinline__ void basis_all(const LayerConst& lc, T n, T* phi, T* zv, T* aux) {
    const int G = lc.G;
    if constexpr (PATH == PATH_DIRECT) {
        const T invh = T(lc.invh);
#pragma unroll 4
        for (int g = 0; g < G; ++g) {
            const T y = (n - T(lc.grid[g])) * invh;
            zv[g] = y;
            phi[g] = basis_direct<T>(lc.basis, y, aux[g]);
        }
    } else {
        T z0, F, R;
        rec_anchor<T>(lc, n, z0, F, R);
        const T tau = z0 + z0;
#pragma unroll 4
        for (int g = 0; g < G; ++g) {
            T v = F * T(lc.K[g]);
            if constexpr (PATH == PATH_REC_CORR) {
                const T e = T(lc.e[g]);
                v = v * kfma<T>(tau, kfma<T>(tau, T(0.5) * e * e, e), T(1));
            }
            phi[g] = v;
            zv[g] = z0 - T(lc.Dl[g]);
            aux[g] = T(0);
            F = F * R;
        }
    }
}

}  // namespace kan
