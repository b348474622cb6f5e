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


// ---- forward sensitivities (SciMLSensitivity 7.69 ForwardDiffSensitivity) ---------------------------------
// The reference's Fisher-KPP gradient at its own size: Zygote.gradient(x -> loss(x), p) with no sensealg
// (Fisher-KPP_Source.jl:198; the Allen-Cahn source driver likewise).  With length(u0) + length(p) = 26 + 11
// <= 100 SciMLSensitivity picks ForwardDiffSensitivity: the solve runs over ForwardDiff.Dual numbers with one
// partial per parameter (chunk = P = 11), i.e. over the state [u; S_1..S_P], S_k = ∂u/∂p_k, with
//     S_k' = (D lap) S_k + φ'(u) S_k + ∂φ/∂p_k(u),   ∂φ/∂C_k = B_k(N(u)),  ∂φ/∂W = swish(u)
// (kdense.jl:116-124), integrated by the same Tsit5 (third-party semantics, restated from the pinned
// SciMLSensitivity 7.69 / DiffEqBase / OrdinaryDiffEq 6.89; verify where Julia exists).  What the Dual solve
// changes in the step control: DiffEqBase's ODE_DEFAULT_NORM over Dual numbers counts the partials.  The
// residual scale of state entry i is abstol + reltol·max(‖u_i‖, ‖unew_i‖) with ‖x‖ = sqrt(value² + Σ_k
// partial_k²) (calculate_residuals calls the scalar Dual norm), the residual's value and partials are divided by
// it, and EEst = sqrt(Σ_i (value² + Σ_k partial_k²) / (n·(1 + P))); the Hairer-Wanner initial step takes the same
// norms; saveat values and partials come from the same interpolant.
//
// Layout: wave 0 carries the values, wave 1 + k the partial S_k (k < G: C_k, k = G: W); lane l is point l % Nx
// of trajectory l / Nx (Nx·B <= 64).  Wave 0 alone evaluates the RHS at the values and hands φ'(y), swish(y) and
// N(y) of every stage to the partial waves through LDS (one barrier per stage, two slots); a partial wave's
// evaluation is then a stencil, an fma and one exponential.  The other exchanges are the per-entry Dual norms (one
// LDS round per step) and the error norm's block sum.  TAB: φ, φ' and swish from the
// piecewise-polynomial tables (PP_PHI, PP_DPHI, PP_SWISH staged in LDS, the reference formula off the table);
// otherwise the reference formula throughout (odd Nx, table path off).
template <int NORM, int GT, bool TAB>
__global__ void __launch_bounds__((GT + 2) * kWave)
fk_small_fsens_kernel(const LayerConst* __restrict__ lcp, const double* __restrict__ p,
                      const double2* __restrict__ tables, FkSmallArgs s, const double* __restrict__ u0, int64_t B,
                      ChainSolveArgs a, double* __restrict__ s_save) {
    using K = Tsit5Tab;
    extern __shared__ double2 tl[];
    __shared__ double red[kFsensMaxWaves];
    const int tsz = TAB ? (kPPCoef / 2) * s.ni : 0;
    if constexpr (TAB) {
        const int fns[3] = {PP_PHI, PP_DPHI, PP_SWISH};
        stage_tables(tl, tables, s.ni, fns, 3);
    }
    double* __restrict__ xv = reinterpret_cast<double*>(tl + 3 * tsz);   // [waves][64] per-entry exchange
    KAN_EXP_TABLE_LDS(tab);   // (its barrier also publishes the tables)
    const Math<double> M{tab};
    const LayerConst& lc = *lcp;
    constexpr int P = GT + 1;
    const int w = threadIdx.x / kWave, l = threadIdx.x & (kWave - 1);
    const int nw = (int)(blockDim.x / kWave);
    const int Nx = s.Nx;
    const int64_t n = (int64_t)Nx * B;
    const bool act = l < n;
    const int j = l % Nx, b0 = l - j;
    const int jm = act ? b0 + (j + Nx - 1) % Nx : l, jp = act ? b0 + (j + 1) % Nx : l;
    const bool sens = w > 0;   // (wave-uniform)
    const int kq = w - 1;
    const double2* tphi = tl;
    const double2* tdphi = tl + tsz;
    const double2* tsw = tl + 2 * tsz;
    auto lap = [&](double v) -> double {
        const double um = __shfl(v, jm, kWave), up = __shfl(v, jp, kWave);
        return lap3<double>(um, v, up, j, Nx, s.cd, s.co);
    };
    // One evaluation of the Dual RHS at the stage input z (wave 0: the values y; wave 1 + k: the partial s_k):
    //   wave 0:      f(y) = (D lap y) + φ(y)                    (FkSmallModel::rhs), and the quantities every
    //                partial needs at y -- φ'(y), swish(y), N(y) -- into LDS slot `slot`;
    //   wave 1 + k:  ((D lap) s_k + s_k φ'(y)) + ∂φ/∂p_k(y),  ∂φ/∂C_k = B_k(N(y)) by the reference formula,
    //                ∂φ/∂W = swish(y), read from that slot after the block barrier.
    // Only wave 0 evaluates at the values, so a partial wave costs a stencil, one fma and one exponential.
    double* __restrict__ shv = xv + kFsensMaxWaves * kWave;   // [2][3][64]: φ', swish, N by slot
    auto F = [&](double z, int slot) -> double {
        double r = 0.0;
        double* sh = shv + slot * 3 * kWave;
        if (!sens) {
            const double lp = lap(z);
            double k = 0.0, dphi = 0.0, sw = 0.0;
            bool ok = false, ok2 = false;
            if constexpr (TAB) {
                k = pp_eval(tphi, s.ni, s.inv_w, s.x0, z, ok);
                ok2 = pp_eval2<true>(tdphi, tsw, s.ni, s.inv_w, s.x0, z, dphi, sw);
            }
            if (!ok) {
                double sc;
                k = pp_direct<NORM, BASIS_RBF>(M, lc, p, lc.grid, z, sc);
            }
            if (!ok2) pp_direct_dphi_sw<NORM, BASIS_RBF>(M, lc, p, z, dphi, sw);
            r = lp + k;
            sh[l] = dphi;
            sh[kWave + l] = sw;
            sh[2 * kWave + l] = normalize<NORM, double>(M, lc.norm, z);
        }
        __syncthreads();
        if (sens) {
            const double lp = lap(z);
            const double dphi = sh[l];
            double dp = sh[kWave + l];
            if (kq < GT) {
                const double y = (sh[2 * kWave + l] - (double)lc.grid[kq]) * (double)lc.invh;
                double aux;
                dp = basis_direct<double>(M, BASIS_RBF, y, aux);
            }
            r = (lp + z * dphi) + dp;
        }
        return r;
    };
    // Σ over the waves of v at this lane's entry (value first, then the partials in order: the entry's Dual
    // sse), the same total in every wave
    auto pt_sum = [&](double v) -> double {
        xv[w * kWave + l] = v;
        __syncthreads();
        double t = xv[l];
        for (int q = 1; q < nw; ++q) t += xv[q * kWave + l];
        __syncthreads();
        return t;
    };
    auto bsum = [&](double v) -> double { return onewg_bsum(act ? v : 0.0, red); };
    double* __restrict__ usave = reinterpret_cast<double*>(a.u_save);
    auto put = [&](int64_t si, double v) {
        if (!act) return;
        if (!sens) {
            if (usave) usave[si * n + l] = v;
        } else if (s_save) {
            s_save[(si * P + kq) * n + l] = v;
        }
    };
    // this wave's entry of the Dual state (the value, or partial kq) and its seven stage values
    double z = sens ? 0.0 : (act ? u0[l] : 0.0);
    double k[7];
    k[0] = F(z, 0);
    const double t0 = a.t0, tf = a.tf;
    const double ntot = (double)n * (double)(P + 1);
    int64_t si = 0;
    while (si < a.n_save && a.saveat[si] <= t0 + 1e-14 * ::fmax(1.0, ::fabs(t0))) {
        put(si, z);
        ++si;
    }
    double nrm = 0.0;   // ‖u_i‖ of this lane's entry (the Dual norm over value and partials)
    if (a.adaptive) nrm = ::sqrt(pt_sum(act ? z * z : 0.0));
    double dt = a.dt;
    if (a.adaptive && !(a.dt > 0)) {   // Hairer & Wanner over the Dual state
        const double sk = ::fma(a.reltol, nrm, a.abstol);
        const double e0 = z / sk, e1 = k[0] / sk;
        const double d0 = ::sqrt(bsum(e0 * e0) / ntot);
        const double d1 = ::sqrt(bsum(e1 * e1) / ntot);
        double dt0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        dt0 = ::fmin(dt0, tf - t0);
        const double f1 = F(::fma(dt0, k[0], z), 1);
        const double e = ::fma(-1.0, k[0], f1) / sk;
        const double d2 = ::sqrt(bsum(e * e) / ntot) / dt0;
        const double mx = ::fmax(d1, d2);
        const double dt1 = mx <= 1e-15 ? ::fmax(1e-6, dt0 * 1e-3) : ::pow(0.01 / mx, 1.0 / 5.0);
        dt = ::fmin(::fmin(100 * dt0, dt1), tf - t0);
    }
    double qold = a.qoldinit, t = t0;
    int64_t naccept = 0, nreject = 0, nf = 0, it = 0, status = 0;
    for (; it < a.maxiters; ++it) {
        if (t >= tf - 1e-14 * ::fmax(1.0, ::fabs(tf))) break;
        dt = ::fmin(dt, tf - t);
        double y = z;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            y = z;
#pragma unroll
            for (int q = 0; q <= i; ++q) y = ::fma(dt * K::TA[i][q], k[q], y);
            k[i + 1] = F(y, i & 1);
        }
        nf += 6;
        double dtnew = dt, nn = nrm;
        if (a.adaptive) {
            double ev = 0.0;
#pragma unroll
            for (int q = 0; q < 6; ++q) ev = ::fma(dt * K::BT[q], k[q], ev);
            const double e = ::fma(dt * K::BT[6], k[6], ev);
            nn = ::sqrt(pt_sum(act ? y * y : 0.0));
            const double sk = ::fma(a.reltol, ::fmax(nrm, nn), a.abstol);
            const double r = e / sk;
            const double eest = ::sqrt(bsum(r * r) / ntot);
            const double q11 = eest > 0 ? ::pow(eest, a.beta1) : 0.0;
            if (eest > 1.0 && dt > a.dtmin) {
                ++nreject;
                dt = dt / ::fmin(1.0 / a.qmin, q11 / a.gamma);
                continue;
            }
            double q = q11 / ::pow(qold, a.beta2);
            q = ::fmax(1.0 / a.qmax, ::fmin(1.0 / a.qmin, q / a.gamma));
            if (1.0 <= q && q <= 1.0) q = 1.0;   // qsteady_min = qsteady_max = 1
            dtnew = q > 0 ? dt / q : dt * a.qmax;
            qold = ::fmax(eest, a.qoldinit);
        }
        const double tn = t + dt;
        while (si < a.n_save && a.saveat[si] <= tn + 1e-12 * ::fmax(1.0, ::fabs(tn))) {
            const double tsv = a.saveat[si];
            double v = y;
            if (!(::fabs(tsv - tn) <= 1e-12 * ::fmax(1.0, ::fabs(tn)))) {
                double wt[7];
                tsit5_interp_weights((tsv - t) / dt, wt);
                v = z;
#pragma unroll
                for (int q = 0; q < 7; ++q) v = ::fma(wt[q] * dt, k[q], v);
            }
            put(si, v);
            ++si;
        }
        if (a.ts && threadIdx.x == 0 && naccept < a.cap) {   // the accepted steps (diagnostics: step-size replay)
            a.ts[naccept] = t;
            a.dts[naccept] = dt;
        }
        z = y;   // commit (value and partials), FSAL
        k[0] = k[6];
        nrm = nn;
        t = tn;
        ++naccept;
        dt = dtnew;
    }
    if (it == a.maxiters && !(t >= tf - 1e-14 * ::fmax(1.0, ::fabs(tf)))) status = 1;
    if (threadIdx.x == 0) {
        a.out[0] = naccept;
        a.out[1] = nreject;
        a.out[2] = nf + 1;
        a.out[3] = status;
    }
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

bool fk_small_fsens_supported(const LayerConst& hlc, int Nx, int64_t B) {
    const int P = hlc.G + 1;
    return Nx >= 3 && B >= 1 && (int64_t)Nx * B <= kWave && P + 1 <= kFsensMaxWaves && hlc.basis == BASIS_RBF &&
           hlc.use_base && (hlc.G == 10 || hlc.G == 5) && (hlc.norm == NORM_SOFTSIGN || hlc.norm == NORM_TANH_FAST);
}

hipError_t launch_fk_small_fsens(const LayerConst& hlc, const PPConst& hpc, bool tab, const LayerConst* lc,
                                 const double* p, const double* tables, const FkSmallArgs& s, const double* u0,
                                 int64_t B, const ChainSolveArgs& a, double* s_save, hipStream_t st) {
    if (!fk_small_fsens_supported(hlc, s.Nx, B) || (tab && (!hpc.enabled || s.ni != hpc.ni || !tables)))
        return hipErrorNotSupported;
    const int threads = (hlc.G + 2) * kWave;
    const size_t lds = (tab ? 3 * sizeof(double2) * (kPPCoef / 2) * (size_t)hpc.ni : 0) +
                       sizeof(double) * (size_t)(kFsensMaxWaves + 6) * kWave;   // exchange + the two slots
#define KAN_FSENS1(NORM, GT, TAB)                                                                                  \
    do {                                                                                                         \
        const void* fn = reinterpret_cast<const void*>(&fk_small_fsens_kernel<NORM, GT, TAB>);                   \
        hipError_t e_ = ensure_dynamic_lds(fn, lds);                                                             \
        if (e_ != hipSuccess) return e_;                                                                         \
        hipLaunchKernelGGL((fk_small_fsens_kernel<NORM, GT, TAB>), dim3(1), dim3(threads), lds, st, lc, p,         \
                           (const double2*)tables, s, u0, B, a, s_save);                                         \
    } while (0)
#define KAN_FSENS(NORM, GT)                                                                                        \
    do {                                                                                                         \
        if (tab) KAN_FSENS1(NORM, GT, true);                                                                     \
        else KAN_FSENS1(NORM, GT, false);                                                                        \
    } while (0)
    if (hlc.G == 10 && hlc.norm == NORM_SOFTSIGN) KAN_FSENS(NORM_SOFTSIGN, 10);
    else if (hlc.G == 10) KAN_FSENS(NORM_TANH_FAST, 10);
    else if (hlc.norm == NORM_SOFTSIGN) KAN_FSENS(NORM_SOFTSIGN, 5);
    else KAN_FSENS(NORM_TANH_FAST, 5);
#undef KAN_FSENS
#undef KAN_FSENS1
    return hipGetLastError();
}

}  // namespace kan
