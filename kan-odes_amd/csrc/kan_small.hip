// kan_small.hip — the Fisher-KPP source-term problem at the reference's own size (PDE examples/
// Fisher-KPP_Source.jl:34-49,95-103,194-213: 26 grid points, one initial condition, T = 5, saveat 0.5,
// the default tolerances) as ONE workgroup for the whole forward solve and ONE for the whole
// InterpolatingAdjoint (the drivers of kan_onewg.hpp), instead of a host loop of per-step launches and
// host round trips over a field that fills a tenth of one wave.
//
// Layout: wave w holds trajectory w (B <= 16 waves), lane j grid point j (Nx <= 64, even: the table path's
// condition).  The periodic Laplacian's neighbours come from lanes (j ± 1) mod Nx of the same wave
// (ds_bpermute), in lap3's ascending-column order; the pointwise KAN is the piecewise-polynomial table
// (kan_pp_point.hpp) staged in LDS, with the reference formula for points off the table.  The forward is
// then the same arithmetic as the host loop's fk_rhs_pp_kernel per point, and the adjoint stage the same
// per-point pullback as the Fisher-KPP adjoint kernels (pp_vjp_point), its eleven moments block-summed per
// stage into kμ.
#include "kan_onewg.hpp"
#include "kan_lap.hpp"
#include "kan_pp_point.hpp"

namespace kan {

namespace {

// MAXT: the block bound the kernels are compiled for (256: B <= 4, one wave per SIMD and up to 256 VGPRs;
// 1024: B <= 16 at 128 VGPRs)

// The Fisher-KPP RHS and its pullback for the one-workgroup drivers.
template <int NORM, int PATH, int GT>
struct FkSmallModel {
    const Math<double>& M;
    const LayerConst& lc;
    const RecScalars<double> rc;
    const double* __restrict__ p;      // the parameters (the cold path's reference formula)
    const double2* __restrict__ tf;    // PP_PHI table (forward) or PP_DPHI (adjoint), LDS
    const double2* __restrict__ ts;    // PP_SWISH table (adjoint), LDS
    int ni;
    double inv_w, x0, cd, co;
    int Nx, j, jm, jp;                 // this lane's point and its periodic neighbours
    double* red;                       // LDS, (blockDim / 64)·(GT + 1) doubles (per-stage moment sums)
    int P;
    bool act;
    int64_t idx, n;

    __device__ double lap(double v) const {
        const double um = __shfl(v, jm, kWave), up = __shfl(v, jp, kWave);
        return lap3<double>(um, v, up, j, Nx, cd, co);
    }
    // f(y)_j = (D lap y)_j + φ(y_j)  (fk_rhs_pp_kernel: pp_pair_finish's per-point order)
    __device__ double rhs(double y) {
        const double l = lap(y);
        bool ok;
        double k = pp_eval(tf, ni, inv_w, x0, y, ok);
        if (__builtin_expect(!ok, 0)) {
            double sc;
            k = pp_direct<NORM, BASIS_RBF>(M, lc, p, lc.grid, y, sc);
        }
        return l + k;
    }
    // λsᵀ∂f/∂u at y (entry j) and kμ = Σ_points λs ∂φ/∂p, the eleven moments summed over the block
    __device__ double vjp(double y, double ls, double* __restrict__ km) {
        const double l = lap(ls);   // (D lap)ᵀ = D lap
        double S0[GT], dW;
        float S1[GT], S2[GT];
        const double xb = pp_vjp_point<NORM, PATH, GT>(M, lc, p, rc, tf, ts, ni, inv_w, x0, y, ls, S0, S1, S2, dW, true);
        double acc[GT + 1];
#pragma unroll
        for (int q = 0; q < GT; ++q) {
            const double e = lc.e[q];
            acc[q] = PATH == PATH_REC_CORR ? lc.K[q] * ::fma(lc.h2[q], (double)S2[q], ::fma(e, (double)S1[q], S0[q]))
                                           : lc.K[q] * S0[q];
        }
        acc[GT] = dW;
        block_sum_to<double, GT + 1>(acc, P, red, km);   // (ends with a block barrier)
        return act ? l + xb : 0.0;
    }
};

template <int NORM, int PATH, int GT>
__device__ __forceinline__ FkSmallModel<NORM, PATH, GT> fk_small_model(const Math<double>& M, const LayerConst& lc,
                                                                       const double* p, const double2* tf,
                                                                       const double2* ts, const FkSmallArgs& s,
                                                                       int64_t B, double* red) {
    const int j = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const bool act = j < s.Nx && w < B;
    return FkSmallModel<NORM, PATH, GT>{M, lc, RecScalars<double>(lc), p, tf, ts, s.ni, s.inv_w, s.x0, s.cd, s.co,
                                        s.Nx, j, (j + s.Nx - 1) % s.Nx, (j + 1) % s.Nx, red,
                                        GT + (lc.use_base ? 1 : 0), act, (int64_t)s.Nx * w + j,
                                        (int64_t)s.Nx * B};
}

// Stage `nt` tables of [kPPCoef/2][ni] double2 from the handle's table buffer (slots fns[0..nt)) into LDS.
__device__ __forceinline__ void stage_tables(double2* tl, const double2* __restrict__ tables, int ni, const int* fns,
                                             int nt) {
    const int tsz = (kPPCoef / 2) * ni;
    for (int f = 0; f < nt; ++f)
        for (int i = threadIdx.x; i < tsz; i += blockDim.x) tl[f * tsz + i] = tables[fns[f] * tsz + i];
}

template <int NORM, int PATH, int GT, int MAXT>
__global__ void __launch_bounds__(MAXT)
fk_small_tsit5_kernel(const LayerConst* __restrict__ lcp, const double* __restrict__ p,
                      const double2* __restrict__ tables, FkSmallArgs s, const double* __restrict__ u0, int64_t B,
                      ChainSolveArgs a) {
    extern __shared__ double2 tl[];
    __shared__ double red[MAXT / kWave];
    const int fns[1] = {PP_PHI};
    stage_tables(tl, tables, s.ni, fns, 1);
    KAN_EXP_TABLE_LDS(tab);   // (its barrier also publishes tl)
    const Math<double> M{tab};
    const LayerConst& lc = *lcp;
    auto m = fk_small_model<NORM, PATH, GT>(M, lc, p, tl, nullptr, s, B, nullptr);
    onewg_tsit5<double>(m, u0, a, red);
}

template <int NORM, int PATH, int GT, int MAXT>
__global__ void __launch_bounds__(MAXT)
fk_small_adjoint_kernel(const LayerConst* __restrict__ lcp, const double* __restrict__ p,
                        const double2* __restrict__ tables, FkSmallArgs s, int64_t B, ChainAdjointArgs a,
                        int stage_rec) {
    extern __shared__ double2 tl[];
    __shared__ double red[MAXT / kWave];
    __shared__ double mred[(MAXT / kWave) * (GT + 1)];
    const int tsz = (kPPCoef / 2) * s.ni;
    const int fns[2] = {PP_DPHI, PP_SWISH};
    stage_tables(tl, tables, s.ni, fns, 2);
    const int P = GT + 1;   // (the launcher admits use_base layers only)
    double* mu = reinterpret_cast<double*>(tl + 2 * tsz);   // [2][P]
    double* km = mu + 2 * P;                                // [7][P]
    double* tsl = km + 7 * P;                               // [nsteps]
    double* dtsl = tsl + a.nsteps;
    for (int i = threadIdx.x; i < 9 * P; i += blockDim.x) mu[i] = 0.0;
    for (int64_t i = threadIdx.x; i < a.nsteps; i += blockDim.x) {
        tsl[i] = a.ts[i];
        dtsl[i] = a.dts[i];
    }
    KAN_EXP_TABLE_LDS(tab);
    const Math<double> M{tab};
    const LayerConst& lc = *lcp;
    double* recl = nullptr;
    if (stage_rec) {
        recl = dtsl + a.nsteps;
        onewg_stage_rec<double>(recl, a, (int64_t)s.Nx * B);
    }
    auto m = fk_small_model<NORM, PATH, GT>(M, lc, p, tl, tl + tsz, s, B, mred);
    onewg_adjoint<double>(m, a, mu, km, tsl, dtsl, red, recl);
}

}  // namespace

bool fk_small_supported(const LayerConst& hlc, const PPConst& hpc, int Nx, int64_t B) {
    return Nx >= 4 && Nx <= kWave && Nx % 2 == 0 && B >= 1 && B <= kFkSmallMaxBatch && hpc.enabled &&
           hlc.basis == BASIS_RBF && hlc.path != PATH_DIRECT && hlc.use_base &&
           (hlc.G == 10 || hlc.G == 5) && (hlc.norm == NORM_SOFTSIGN || hlc.norm == NORM_TANH_FAST);
}

#define KAN_SMALL_GO(KERNEL, ...)                                                                                   \
    do {                                                                                                          \
        if (hlc.path == PATH_REC_CORR) {                                                                          \
            if (hlc.G == 10 && hlc.norm == NORM_SOFTSIGN) KERNEL(NORM_SOFTSIGN, PATH_REC_CORR, 10);               \
            else if (hlc.G == 10) KERNEL(NORM_TANH_FAST, PATH_REC_CORR, 10);                                      \
            else if (hlc.norm == NORM_SOFTSIGN) KERNEL(NORM_SOFTSIGN, PATH_REC_CORR, 5);                          \
            else KERNEL(NORM_TANH_FAST, PATH_REC_CORR, 5);                                                        \
        } else {                                                                                                  \
            if (hlc.G == 10 && hlc.norm == NORM_SOFTSIGN) KERNEL(NORM_SOFTSIGN, PATH_REC, 10);                    \
            else if (hlc.G == 10) KERNEL(NORM_TANH_FAST, PATH_REC, 10);                                           \
            else if (hlc.norm == NORM_SOFTSIGN) KERNEL(NORM_SOFTSIGN, PATH_REC, 5);                               \
            else KERNEL(NORM_TANH_FAST, PATH_REC, 5);                                                             \
        }                                                                                                         \
    } while (0)

hipError_t launch_fk_small_tsit5(const LayerConst& hlc, const PPConst& hpc, const LayerConst* lc, const double* p,
                                 const double* tables, const FkSmallArgs& s, const double* u0, int64_t B,
                                 const ChainSolveArgs& a, hipStream_t st) {
    if (!fk_small_supported(hlc, hpc, s.Nx, B) || s.ni != hpc.ni) return hipErrorNotSupported;
    const size_t lds = sizeof(double2) * (kPPCoef / 2) * (size_t)hpc.ni;
    const int threads = (int)B * kWave;
#define KAN_SMALL_FWD(NORM, PATH, GT)                                                                              \
    do {                                                                                                         \
        if (threads <= 256)                                                                                      \
            hipLaunchKernelGGL((fk_small_tsit5_kernel<NORM, PATH, GT, 256>), dim3(1), dim3(threads), lds, st, lc, p, \
                               (const double2*)tables, s, u0, B, a);                                             \
        else                                                                                                     \
            hipLaunchKernelGGL((fk_small_tsit5_kernel<NORM, PATH, GT, 1024>), dim3(1), dim3(threads), lds, st, lc, \
                               p, (const double2*)tables, s, u0, B, a);                                          \
    } while (0)
    KAN_SMALL_GO(KAN_SMALL_FWD);
#undef KAN_SMALL_FWD
    return hipGetLastError();
}

hipError_t launch_fk_small_adjoint(const LayerConst& hlc, const PPConst& hpc, const LayerConst* lc, const double* p,
                                   const double* tables, const FkSmallArgs& s, int64_t B, const ChainAdjointArgs& a,
                                   hipStream_t st) {
    if (!fk_small_supported(hlc, hpc, s.Nx, B) || s.ni != hpc.ni || a.nsteps < 1) return hipErrorNotSupported;
    const int P = hlc.G + 1;
    size_t lds = 2 * sizeof(double2) * (kPPCoef / 2) * (size_t)hpc.ni + sizeof(double) * (9 * (size_t)P + 2 * a.nsteps);
    if (lds > 150 * 1024) return hipErrorNotSupported;   // (~6,000 forward steps at ni = 256)
    // the forward's dense output staged in LDS too where it fits (the reference's 26-point problem: ~45 steps,
    // 65 KB): every adjoint stage interpolates it
    const size_t rec = sizeof(double) * ((size_t)a.nsteps * 7 + 1) * (size_t)s.Nx * B;
    const int stage_rec = lds + rec <= 150 * 1024 ? 1 : 0;
    if (stage_rec) lds += rec;
    const int threads = (int)B * kWave;
#define KAN_SMALL_ADJ1(NORM, PATH, GT, MAXT)                                                                       \
    do {                                                                                                         \
        {                                                                                                        \
            const void* fn = reinterpret_cast<const void*>(&fk_small_adjoint_kernel<NORM, PATH, GT, MAXT>);        \
            hipError_t e_ = ensure_dynamic_lds(fn, lds);                                                         \
            if (e_ != hipSuccess) return e_;                                                                     \
        }                                                                                                        \
        hipLaunchKernelGGL((fk_small_adjoint_kernel<NORM, PATH, GT, MAXT>), dim3(1), dim3(threads), lds, st, lc, p, \
                           (const double2*)tables, s, B, a, stage_rec);                                          \
    } while (0)
#define KAN_SMALL_ADJ(NORM, PATH, GT)                                                                              \
    do {                                                                                                         \
        if (threads <= 256) KAN_SMALL_ADJ1(NORM, PATH, GT, 256);                                                 \
        else KAN_SMALL_ADJ1(NORM, PATH, GT, 1024);                                                               \
    } while (0)
    KAN_SMALL_GO(KAN_SMALL_ADJ);
#undef KAN_SMALL_ADJ
#undef KAN_SMALL_ADJ1
    return hipGetLastError();
}
#undef KAN_SMALL_GO

}  // namespace kan
