// fkbench.hip — standalone variant microbenchmark for the Fisher-KPP RHS kernel body
// (development tool; not part of libkanode.so).  Each variant removes or swaps one
// ingredient so its cost can be read off directly on the GPU:
//   V0 table exp (production math)        V1 polynomial exp (no LDS table)
//   V2 no swish term                      V3 Horner S0 only (no knot correction)
//   V4 V0 with 128-thread blocks          V5 exp only (no Horner, no swish)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I kan-odes_amd/csrc tools/fkbench.hip -o fkbench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "kan_device.hpp"

using namespace kan;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// polynomial exp: k = round(x/ln2), |r| <= ln2/2, degree-12 Taylor (no table)
__device__ __forceinline__ double exp_poly(double x) {
    const double magic = 0x1.8p52;
    const double t = fma(x, 0x1.71547652b82fep0, magic);
    const int k = (int)__double2loint(t);
    const double kd = t - magic;
    double r = fma(-kd, 0x1.62e42fefa39efp-1, x);
    r = fma(-kd, 0x1.abc9e3b39803fp-56, r);
    double p = 1.0 / 479001600.0;
    p = fma(r, p, 1.0 / 39916800.0);
    p = fma(r, p, 1.0 / 3628800.0);
    p = fma(r, p, 1.0 / 362880.0);
    p = fma(r, p, 1.0 / 40320.0);
    p = fma(r, p, 1.0 / 5040.0);
    p = fma(r, p, 1.0 / 720.0);
    p = fma(r, p, 1.0 / 120.0);
    p = fma(r, p, 1.0 / 24.0);
    p = fma(r, p, 1.0 / 6.0);
    p = fma(r, p, 0.5);
    p = fma(r, p, 1.0);
    p = fma(r, p, 1.0);
    return __builtin_amdgcn_ldexp(p, k);
}

struct Coef { double A[10], Bq[10], Q[10], W, s, gs, tc; };

template <int V>
__device__ __forceinline__ double EXP(const Math<double>& M, double x) {
    if constexpr (V == 1) return exp_poly(x);
    else return M.exp(x);
}

template <int V>
__device__ __forceinline__ double kanf(const Math<double>& M, const Coef& c, double x) {
    const double n = x * M.rcp(1.0 + __builtin_fabs(x));
    const double z0 = fma(n, c.s, c.gs);
    const double p2 = z0 * z0, perr = fma(z0, z0, -p2);
    const double E = EXP<V>(M, -p2);
    const double E0 = fma(-E, perr, E);
    const double tw = z0 + z0;
    const double R = EXP<V>(M, tw);
    if constexpr (V == 5) return E0 + R;
    const double tp = tw - c.tc;
    double s0 = c.A[9], s1 = c.Bq[9], s2 = c.Q[9];
#pragma unroll
    for (int j = 8; j >= 0; --j) {
        s0 = fma(s0, R, c.A[j]);
        if constexpr (V != 3) { s1 = fma(s1, R, c.Bq[j]); s2 = fma(s2, R, c.Q[j]); }
    }
    double sp = (V != 3) ? E0 * fma(tp, fma(tp, s2, s1), s0) : E0 * s0;
    if constexpr (V != 2) {
        const double t = EXP<V>(M, -__builtin_fabs(x) < -7e5 ? -7e5 : -__builtin_fabs(x));
        const double sg = (x >= 0 ? 1.0 : t) * M.rcp(1.0 + t);
        sp = fma(c.W, x * sg, sp);
    }
    return sp;
}

template <int V, int BS>
__global__ void __launch_bounds__(BS) kern(const Coef* __restrict__ cp, const double* __restrict__ u,
                                           double* __restrict__ du, int64_t B, double cd, double co) {
    KAN_EXP_TABLE_LDS(tab);
    const Math<double> M{tab};
    const Coef c = *cp;
    const int Nx = 256;
    const int tpb = BS / 128;
    const int q = threadIdx.x & 127;
    const int i = 2 * q;
    const int im = i > 0 ? i - 1 : Nx - 1, ip = i + 2 < Nx ? i + 2 : 0;
    for (int64_t b = (int64_t)blockIdx.x * tpb + threadIdx.x / 128; b < B; b += (int64_t)gridDim.x * tpb) {
        const double* ub = u + b * Nx;
        const double2 v = *reinterpret_cast<const double2*>(ub + i);
        const double um = ub[im], up = ub[ip];
        double2 o;
        o.x = (co * um + cd * v.x) + co * v.y + kanf<V>(M, c, v.x);
        o.y = (co * v.x + cd * v.y) + co * up + kanf<V>(M, c, v.y);
        *reinterpret_cast<double2*>(du + b * Nx + i) = o;
    }
}

template <int V, int BS>
float run(const Coef* c, const double* u, double* du, int64_t B, int reps) {
    const int tpb = BS / 128;
    int grid = (int)std::min<int64_t>((B + tpb - 1) / tpb, 4096 * (256 / BS));
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL((kern<V, BS>), dim3(grid), dim3(BS), 0, 0, c, u, du, B, -1300.5, 650.25);
    (void)hipEventRecord(a);
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((kern<V, BS>), dim3(grid), dim3(BS), 0, 0, c, u, du, B, -1300.5, 650.25);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps * 1000.f;
}

int main() {
    const int64_t B = 131072, Nx = 256, N = B * Nx;
    std::vector<double> hu(N);
    for (int64_t k = 0; k < N; ++k) hu[k] = 0.5 + 0.5 * std::sin(0.001 * (double)k);
    Coef hc;
    for (int j = 0; j < 10; ++j) { hc.A[j] = 0.1 * (j + 1) * std::exp(-j * j * 1.0); hc.Bq[j] = 1e-7 * hc.A[j]; hc.Q[j] = 1e-14 * hc.A[j]; }
    hc.W = 0.3; hc.s = 4.5; hc.gs = 4.5; hc.tc = 9.0;
    double *u, *du;
    Coef* c;
    CK(hipMalloc(&u, N * 8));
    CK(hipMalloc(&du, N * 8));
    CK(hipMalloc(&c, sizeof(Coef)));
    CK(hipMemcpy(u, hu.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(c, &hc, sizeof(Coef), hipMemcpyHostToDevice));
    const int reps = 20;
    printf("V0 table exp        %8.1f us\n", run<0, 256>(c, u, du, B, reps));
    printf("V1 poly exp         %8.1f us\n", run<1, 256>(c, u, du, B, reps));
    printf("V2 no swish         %8.1f us\n", run<2, 256>(c, u, du, B, reps));
    printf("V3 S0 only          %8.1f us\n", run<3, 256>(c, u, du, B, reps));
    printf("V4 V0 block128      %8.1f us\n", run<0, 128>(c, u, du, B, reps));
    printf("V5 exp only         %8.1f us\n", run<5, 256>(c, u, du, B, reps));
    printf("V0 again            %8.1f us\n", run<0, 256>(c, u, du, B, reps));
    CK(hipDeviceSynchronize());
    return 0;
}
