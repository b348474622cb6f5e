// kan_kernels.hpp — internal launcher declarations (C++ linkage, not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kan_device.hpp"

namespace kan {

// `hlc` is the host copy of the layer constants (selects the kernel variant),
// `lc` the device copy the kernels read.  All pointers are device pointers.
template <typename T>
hipError_t launch_fk_rhs(const LayerConst& hlc, const LayerConst* lc, const T* p, T cd, T co, int Nx,
                         const T* u, T* du, int64_t B, hipStream_t st);
template <typename T>
hipError_t launch_fk_vjp(const LayerConst& hlc, const LayerConst* lc, const T* p, T cd, T co, int Nx,
                         const T* u, const T* lam, T* lamJ, T* dp, T* slab, int slab_blocks, int64_t B,
                         hipStream_t st);
// Runge-Kutta stage arguments (kanode_rhs_stage): y = u + Σ_{j<nk} c_j k_j; optional
// embedded error e = Σ_{j<nk} ec_j k_j + ec_nk du, Σ (e / (abstol + reltol·max(|u|,|y|)))².
constexpr int kMaxStages = 8;
// cscale (nullable, device): c_j and ec_j are multiplied by *cscale inside the kernel — the
// step size of a device-controlled solve (kanode_solve.cpp graph mode) lives in device memory.
template <typename T>
struct StageArgs {
    const T* k[kMaxStages];
    double c[kMaxStages];
    double ec[kMaxStages + 1];
    double abstol, reltol;
    int nk;
    const double* cscale;
    const int32_t* skip;    // nullable, device: the launch does nothing while *skip != 0 (a finished solve)
};
__device__ __forceinline__ double stage_scale(const double* cscale) { return cscale ? *cscale : 1.0; }
__device__ __forceinline__ bool stage_skip(const int32_t* skip) { return skip && *skip; }
// ec[nk] with static indices only: a runtime index into the by-value StageArgs would make the
// compiler copy the whole struct to scratch
template <typename SA>
__device__ __forceinline__ double stage_ec_last(const SA& sa) {
    double e = 0.0;
#pragma unroll
    for (int j = 0; j <= kMaxStages; ++j)
        if (j == sa.nk) e = sa.ec[j];
    return e;
}
// Element idx of every stage array, all loads issued before any value is used.  An unused slot
// (j >= nk) reads `safe` instead, so no load sits behind a branch: a branch per load made the
// compiler wait for each array before loading the next (one memory round trip per stage array,
// up to 7 per stage input).  Callers combine kv[j] under `j < nk` exactly as before.
template <typename T>
__device__ __forceinline__ void stage_ld(const StageArgs<T>& sa, const T* safe, int64_t idx, T (&kv)[kMaxStages]) {
    if (sa.nk == 0) return;   // a plain RHS call (nothing combined): no loads at all
#pragma unroll
    for (int j = 0; j < kMaxStages; ++j) kv[j] = (j < sa.nk ? sa.k[j] : safe)[idx];
}
template <typename T>
hipError_t launch_stage_lincomb(const T* u, const StageArgs<T>& sa, T* y, int64_t n, hipStream_t st);
// The saveat values that fall in one accepted Tsit5 step in one launch (round 4; kanode_solve.cpp solve_t):
// saveat j (< nsv) is y_j = u + Σ_m w[j][m] k_m in stage_lincomb_kernel's fma order, or u_new itself when bit j
// of `exact` is set (a saveat on the step's end), written to dst + j·n.  A surrogate forward step holds up to
// ~40 saveat points (Burgers: 200 stops over 5 steps), each of which was one launch.
constexpr int kSaveatPerLaunch = 48;
template <typename T> struct SaveatStep {
    const T* u;
    const T* u_new;
    const T* k[7];
    T* dst;
    uint64_t exact;
    int32_t nk, nsv;
    double w[kSaveatPerLaunch][7];
};
template <typename T>
hipError_t launch_saveat_step(const SaveatStep<T>& a, int64_t n, hipStream_t st);
// per-block partials into `slab` (<= slab_blocks rows), then out[0] = ordered total
template <typename T>
hipError_t launch_stage_error(const T* u, const T* y, const T* du, const StageArgs<T>& sa, double* slab,
                              int slab_blocks, double* out, int64_t n, hipStream_t st);
hipError_t launch_stage_error_final(const double* slab, int nblk, double* out, hipStream_t st);
// μ update + μ error partials of an adaptive adjoint step (kan_stage.hip adj_step_finish_kernel)
constexpr int kAdjFinishBlocks = 64;
template <typename T>
struct AdjStepFinish {
    const T* km[7];
    double a[6], b[7];
    double abstol, reltol;
};
template <typename T>
hipError_t launch_adj_step_finish(const T* mu, T* mu_new, const AdjStepFinish<T>& f, double* slab, int64_t n,
                                  int* nblk, hipStream_t st);

// Flux Adam step after the gradient all-reduce (kan_optim.hip, kanode_adam_step)
struct AdamArgs {
    double scale;          // Δ = scale·g (1/world_size after a SUM all-reduce)
    double beta1, beta2;   // β
    double omb1, omb2;     // 1 - β
    double c1, c2;         // 1 - βp (βp = β^t, Flux's running powers before this step advances them)
    double eps, eta;
};
template <typename T>
hipError_t launch_adam_step(T* x, T* m, T* v, const T* g, int64_t n, const AdamArgs& a, hipStream_t st);

// piecewise-polynomial Fisher-KPP RHS / VJP (kan_pp.hip).  build = false reuses the
// tables of an earlier launch with the same p (the integrator holds them per solve).  `tables` holds
// kPPMaxFns slots of kPPCoef·ni doubles (slot = PPFn id); the build fills the listed
// functions from p, the RHS then reads slot PP_PHI (fp64, Nx even).
// Persistent-grid overrides of the table kernels (kanode_set_option KANODE_OPT_GRID_*; 0 = the
// occupancy-derived default).  Tuning sweeps only: the grid fixes the dp reduction order.
struct GridOverride {
    int rhs = 0, vjp = 0, vstep = 0;
    bool vstep_rows = true;   // KANODE_OPT_ADJ_STEP_ROWS
};
hipError_t launch_fk_pp_build(const PPConst& hpc, const LayerConst* lc, const PPConst* pc, const double* p,
                              double* tables, const int* fns, int nfn, hipStream_t st);
hipError_t launch_fk_rhs_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc, const double* p,
                            double* table, double cd, double co, int Nx, const double* u, double* du, int64_t B,
                            hipStream_t st, bool build = true, int grid_ovr = 0);
bool fk_vjp_pp_supported(const LayerConst& hlc, int Nx);
bool fk_stage_pp_supported(const PPConst& hpc, int Nx);
// fused stage: du = f(u + Σ c_j k_j), optional y_out, optional error total into err_out[0]
hipError_t launch_fk_stage_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc,
                              const double* p, double* table, double cd, double co, int Nx, const double* u,
                              const StageArgs<double>& sa, double* y_out, double* err_slab, int slab_blocks,
                              double* err_out, double* du, int64_t B, hipStream_t st, bool build = true,
                              int grid_ovr = 0);
// A whole Tsit5 step of the Fisher-KPP table RHS per trajectory row (fk_step_pp_wave_kernel):
// a6x6[6s + j] = dt·a_sj, e7 = dt·btilde (error with err_out), k_2..k_7 -> kout[0..5]; with
// q4x7[7m + i] = dt·RI[i][m] the dense output is Q_1..Q_4 -> kout[0..3] and k_7 -> kout[5]
hipError_t launch_fk_step_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc,
                             const double* p, double* table, double cd, double co, int Nx, const double* u,
                             const double* k1, double* const* kout, double* u_new, const double* a6x6,
                             const double* e7, const double* q4x7, double abstol, double reltol, double* err_slab,
                             int slab_blocks, double* err_out, int64_t B, hipStream_t st, bool build,
                             int grid_ovr = 0, int* parts_out = nullptr);
// (parts_out != nullptr with err_out: the per-block error partials are left in err_slab[0, *parts_out)
// for the caller to sum -- the host, from mapped memory -- instead of a final reduction launch)

// The adaptive Fisher-KPP solve with the step control on the device (kanode_solve.cpp solve_fk_loop): launch q
// of the step kernel decides launch q - 1's attempt at its head (every workgroup sums the same error partials
// and applies solve_t's PI controller: accept/reject, the step record, the next step size), then takes the
// next attempt into the dense-output slots.  The host enqueues launches ahead without waiting on any of them;
// a launch after the end passes the final state on and returns.
struct StepCoef {
    double a[6][6];   // dt·a_sj
    double e[7];      // dt·btilde_j
    double q[4][7];   // dt·RI[i][m] (qform)
    double abstol, reltol;
};
struct FkLoopCtl {
    double t, dt, qold;
    int64_t step, nreject, it;   // accepted steps, rejections, decided attempts
    int32_t status;              // 0 running, 1 done, 2 maxiters reached
    int32_t pending;             // the launch that wrote this state took an attempt (the next launch decides it)
    void* cand[4];               // slots[step - 1 .. step + 2] (cand[0]: none at step 0)
};
struct FkLoopArgs {
    FkLoopCtl* state;      // [2]: launch q reads state[(q + 1) & 1] (launch q - 1's, the host's for q = 0); its
                           // workgroup 0 writes state[q & 1] and the host's mirror
    FkLoopCtl* mirror;     // the host's mapped copy (device address)
    void* const* slots;    // dense-output slots (u_n, Q_1..Q_4, k_7 of n entries each), up to step + 2
    const double* k1_0;    // k_1 of the first step
    double* ts;            // accepted steps: start time, step size
    double* dts;
    double* parts;         // [2][max_grid] error partials, by launch parity
    int64_t max_grid;
    int64_t n;             // state entries (Nx·B): the error norm's count and the slot vector stride
    double tf, abstol, reltol, dtmin, beta1, beta2, gamma, qmin, qmax, qoldinit;
    int64_t maxiters;
};
struct AdjLoopArgs;
struct AdjLoopCtl;
struct AdjLoopPlan;
bool fk_adjoint_loop_supported(const PPConst& hpc, const LayerConst& hlc, int Nx);
int fk_adjoint_loop_grid(int64_t B, int slab_blocks);
hipError_t launch_fk_adjoint_loop(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc,
                                  const double* p, double* tables, double cd, double co, int Nx, const AdjLoopArgs& la,
                                  int64_t B, hipStream_t st, bool build);
hipError_t launch_fk_step_pp_loop(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, double cd,
                                  double co, int Nx, const double* p, const double* table, const FkLoopArgs& la,
                                  int64_t lq, int64_t B, hipStream_t st, int grid_ovr = 0);
hipError_t launch_fk_vjp_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc,
                            const double* p, double* tables, double cd, double co, int Nx, const double* u,
                            const double* lam, double* lamJ, double* dp, double* slab, int slab_blocks, int64_t B,
                            hipStream_t st, bool build = true, int grid_ovr = 0);
// adjoint stage, fused (kanode_vjp_stage): y = u + Σ su.c_j su.k_j, λs = lam + Σ sl.c_j sl.k_j
// in registers (λs -> lam_out if non-null), λᵀJ at y, dp (= if dp_assign, else +=), the λ
// error total -> err_out[0] when non-null (sl.ec / abstol / reltol)
hipError_t launch_fk_vjp_stage_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc,
                                  const double* p, double* tables, double cd, double co, int Nx, const double* u,
                                  const StageArgs<double>& su, const double* lam, const StageArgs<double>& sl,
                                  double* lam_out, double* lamJ, double* dp, bool dp_assign, double* err_out,
                                  double* slab, int slab_blocks, int64_t B, hipStream_t st, bool build = true,
                                  int* deferred_grid = nullptr, int grid_ovr = 0);
// The reductions of several adjoint stages launched with deferred_grid (their slabs in
// separate regions) in one launch: job j sums slab_j rows into dp_j (= or +=) and err_slab_j
// into err_out_j, each in the fixed order of vjp_finish_kernel.
// One InterpolatingAdjoint step (six stages) of the Fisher-KPP table path in one launch
// (fk_vjp_step_pp_wave_kernel); the dense output must be in Q form.  slab_base receives the six
// stages' [grid][P] moment rows and then the [grid] error partials; grid_out the grid.
// The finish of an ADAPTIVE Fisher-KPP adjoint step in one launch (kan_pp.hip adj_finish_kernel):
// block q < P forms the stage sums S_i[q] = Σ_b slab_i[b·P + q] (i < nslab, one pass, fixed order),
//     μ_new[q] = fma(1, Σ_i ca_i S_i, fma(a0, km1[q], μ[q]))       (μ + h Σ_j a6_j kμ_j)
//     km7[q]   = S_{k7}[q]                                         (the next step's FSAL kμ_1)
//     out[1 + q] = (e / (abstol + reltol·max(|μ|, |μ_new|)))²,  e = e0·km1[q] + Σ_i ce_i S_i
//                                                                  (the μ part of the [λ; μ] norm)
// and block P sums the λ error partials into out[0]: the step's μ update, FSAL and error norm,
// which otherwise take the reduction, lincomb and two error launches.
struct AdjFinish {
    const double* slab[6];
    double ca[6], ce[6];
    int32_t nslab, k7;
    int32_t tr, pad;           // tr: slab i holds its rows parameter-major, [P][nblk] (the rows kernel's
                               // combined adaptive step), so block q reads one contiguous row of nblk
    int64_t nblk;
    double a0, e0, abstol, reltol;
    const double* mu;
    double* mu_new;
    const double* km1;
    double* km7;
    const double* err_slab;
    double* out;
};
struct AdjStepArgs {
    double* kl[7];             // kλ_1 (FSAL, read) .. kλ_7 (written by stage s into kl[s + 1])
    double a[6][6];            // h·a_sj
    const double* su_u[6];     // u_i of the forward step holding stage s
    const double* su_q[6][4];  // its Q_1..Q_4
    double su_c[6][4];         // θ_s^m
    double ec[7];              // h·btilde (stage 6 error)
    double abstol, reltol;
    const double* lam;
    double* lam_out;
    double* slab[6];           // per stage: [grid][P] moment rows
    double* err_slab;          // [grid] (null: no error)
    int32_t reload[6];         // (set by the launcher) stage s reads u_i, Q_m other than stage s-1's
    // combine (fixed step): stages 0..4 are not reduced one by one; each thread accumulates
    // A = Σ_{s<5} a[5][s+1]·moments_s and the block rows of A go to slab[0], stage 5's (kμ_7, the
    // next step's FSAL kμ_1) to slab[5]: 2 block reductions per step instead of 6.  Only the rows
    // kernel combines; the launcher clears it otherwise.
    int32_t combine;
    // fin_ctr non-null (combine = 2): the step's finish runs inside the rows kernel -- the last P + 1
    // workgroups to arrive (fin_ctr[0] counts arrivals, fin_ctr[1] finishers; both back to 0 at the end)
    // each do one block of adj_finish_kernel's work on `fin` in its order (bitwise the same results), so
    // no finish launch follows the step.  The launcher fills fin.slab / err_slab / nblk / nslab / k7.
    unsigned* fin_ctr;
    AdjFinish fin;
};
hipError_t launch_fk_vjp_step_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc,
                                 const double* p, double* tables, double cd, double co, int Nx,
                                 const AdjStepArgs& a, double* slab_base, int slab_blocks, int64_t B, int* grid_out,
                                 hipStream_t st, bool build, int grid_ovr = 0, bool rows = true,
                                 int* combined_out = nullptr, bool* fused_finish_out = nullptr);
constexpr int kMaxFinishJobs = 8;
struct FinishJob {
    const double* slab;
    const double* err_slab;
    double* dp;
    double* err_out;
    int64_t nblk;
    int32_t assign;
    int32_t tr;                // slab rows parameter-major, [P][nblk] (the rows kernel's combined steps)
    // base != null: dp[q] = fma(1, Σ, fma(coef, other[q], base[q])) -- a two-term stage_lincomb of
    // (base; other, Σ) in its own order, so the μ update of a combined adjoint step needs no launch
    const double* base;
    const double* other;
    double coef;
};
struct FinishJobs {
    FinishJob j[kMaxFinishJobs];
};
hipError_t launch_vjp_finish_jobs(const FinishJobs& jobs, int njobs, int64_t P, hipStream_t st);
hipError_t launch_adj_finish(const AdjFinish& f, int64_t P, hipStream_t st);
template <typename T>
hipError_t launch_kd_fwd_col(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, T* y, int64_t K,
                             hipStream_t st);
// whole chain, one launch (all layers I, O <= 16); hipErrorNotSupported otherwise.  With `sa` it is
// a Runge-Kutta stage (kanode_rhs_stage): input x + Σ c_j k_j, optional y_out, and with err_out the
// embedded-error total (per-block partials in err_slab, <= slab_rows blocks)
template <typename T>
hipError_t launch_kd_chain_col(const LayerConst* hlcs, int nl, const LayerConst* lcs, const T* p, int64_t P,
                               const T* x, T* y, int64_t K, hipStream_t st, const StageArgs<T>* sa = nullptr,
                               T* y_out = nullptr, double* err_slab = nullptr, int slab_rows = 0,
                               double* err_out = nullptr);
// adjoint stage of a whole small chain in one launch + one reduction launch (dp = or +=; the λ
// error total into err_out when non-null); hipErrorNotSupported outside its shapes
template <typename T>
hipError_t launch_kd_chain_vjp_stage(const LayerConst* hlcs, int nl, const LayerConst* lcs, const T* p, int64_t P,
                                     const T* u, const StageArgs<T>& su, const T* lam, const StageArgs<T>& sl,
                                     T* lam_out, T* lamJ, T* dp, bool dp_assign, double* err_out, void* slab,
                                     size_t slab_bytes, int64_t K, hipStream_t st);
template <typename T>
hipError_t launch_kd_vjp_col(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, const T* yb,
                             T* xb, T* pbar, T* slab, int slab_blocks, int64_t K, hipStream_t st);
template <typename T>
hipError_t launch_kd_edge_act(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, T* act, int64_t K,
                              hipStream_t st);

// device-side Tsit5 step control (kan_solve.hip; kanode_solve.cpp graph mode)
struct SolveCtl {
    double t, dt, qold, eest;
    int64_t naccept, nreject, attempts, si;
    int32_t done, status, accepted, pad;   // status: 0 ok, 1 maxiters, 2 dense-output storage full
};
template <typename T>
struct Tsit5Bufs {
    T* U;               // u_n (committed on accept)
    T* K[7];            // k_1 .. k_7 (k_1 <- k_7 on accept)
    const T* UNEW;      // stage-7 output u_{n+1}
    T* save;            // [n_save][n] saveat values
    void* const* slots; // dense-output slot n: [u_n, k_2..k_7] (record)
};
struct Tsit5PostArgs {
    double tf, dtmin, beta1, beta2, gamma, qmin, qmax, qoldinit;
    int32_t adaptive, record;
    int64_t maxiters, n_save, slot_cap;
    const double* saveat;
    double* ts_rec;
    double* dts_rec;
};
template <typename T>
hipError_t launch_tsit5_post(const SolveCtl* cin, SolveCtl* cout, const double* sumsq, const Tsit5Bufs<T>& bf,
                             const Tsit5PostArgs& pa, int64_t n, hipStream_t st);

// Tsit5Interp b_i(θ) = Σ_m RI[i][m] θ^(m+1) (OrdinaryDiffEqTsit5 1.1.0), on the device
__device__ __forceinline__ void tsit5_interp_weights(double th, double w[7]) {
    constexpr double RI[7][4] = {
        {1.0, -2.763706197274826, 2.9132554618219126, -1.0530884977290216},
        {0.0, 0.13169999999999998, -0.2234, 0.1017},
        {0.0, 3.9302962368947516, -5.941033872131505, 2.490627285651253},
        {0.0, -12.411077166933676, 30.33818863028232, -16.548102889244902},
        {0.0, 37.50931341651104, -88.1789048947664, 47.37952196281928},
        {0.0, -27.896526289197286, 65.09189467479366, -34.87065786149661},
        {0.0, 1.5, -4.0, 2.5},
    };
    const double th2 = th * th, tp[4] = {th, th2, th2 * th, th2 * th2};   // θ^(m+1) (pow would cost ~4 calls)
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        double s = 0.0;
#pragma unroll
        for (int m = 0; m < 4; ++m) s += RI[i][m] * tp[m];
        w[i] = s;
    }
}

// A whole Tsit5 solve of a small chain in one workgroup (kd_chain_tsit5_kernel, kan_col.hip):
// the options and storage of kanode_solve_tsit5 (solve_t semantics), status out[3]:
// 0 done, 1 maxiters, 2 dense-output capacity (the caller falls back to the host loop).
struct ChainSolveArgs {
    double t0, tf, dt, abstol, reltol, dtmin, beta1, beta2, gamma, qmin, qmax, qoldinit;
    int32_t adaptive, pad;
    int64_t maxiters, n_save, cap;
    const double* saveat;
    void* u_save;     // [n_save][n] or null
    void* rec;        // [cap][7][n]: u_n, k_2..k_7 of accepted step n (null: no dense output)
    void* k1_0;       // k_1 of step 0 (with rec)
    double* ts;       // [cap] step start times (with rec)
    double* dts;      // [cap] step sizes (with rec)
    int64_t* out;     // naccept, nreject, nf, status
    double* hts;      // or null: mapped host copy of ts | dts ([2][cap], with rec), fenced before out is written
};
// InterpolatingAdjoint of a small chain in one workgroup (kd_chain_adjoint_kernel): the backward
// Tsit5 over [λ; μ] of kanode_solve.cpp adjoint_t, reading the dense output that
// kd_chain_tsit5_kernel recorded.  Jump rows of dl_du come grouped: group 0 at τ = 0 (t = tf),
// group 1 + si at stop si (si < nstops - 1), group nstops at t0 (after the loop).
struct ChainAdjointArgs {
    double t0, tf, dt, abstol, reltol, dtmin, beta1, beta2, gamma, qmin, qmax, qoldinit;
    int32_t adaptive, pad;
    int64_t maxiters;
    const void* rec;        // [nsteps][7][n] (kd_chain_tsit5_kernel layout)
    const void* k1_0;
    const double* ts;       // [nsteps]
    const double* dts;      // [nsteps]
    int64_t nsteps;
    const void* dl_du;      // [n_save][n] or null
    const double* stops;    // [nstops], ascending τ, the last = tf - t0
    int64_t nstops;
    const int32_t* jrows;   // dl_du rows, grouped
    const int32_t* joff;    // [nstops + 2] group offsets into jrows
    void* du0;              // [n] or null
    void* dp;               // [P] or null
    int64_t* out;           // naccept, nreject, nf, status (0 ok, 1 maxiters)
    double* hs;             // [hs_cap] accepted adjoint step sizes, in order (KANODE_OPT_RECORD_ADJOINT_STEPS), or null
    int64_t hs_cap;
};
// The whole InterpolatingAdjoint of a surrogate pair KDense(N -> H) + KDense(H -> N) in ONE launch
// (kd_pair_adjoint_kernel, kan_pair_adj.hip): the grid split over workgroups of S points, two exchanges
// of H·B partials per adjoint stage.  c.rec is the device table of the forward solve's slot pointers
// ([nsteps]; slot i = u_i, k_2..k_7, each n = N·B entries), c.k1_0 the first step's k_1.
constexpr int kPairAdjXW = 512;   // doubles per workgroup and exchange slot
struct PairAdjArgs {
    ChainAdjointArgs c;
    double* xbuf;     // [2][nwg][kPairAdjXW] exchange slots (write-through stores and loads)
    unsigned* ctr;    // arrival counter; ctr[1]: abort word (the 16 bytes are zeroed before every launch)
    unsigned* abrt;
    int64_t P;        // parameters of the chain (the error norm's count)
    int S;            // grid points per workgroup (0: 8)
    int max_wg;       // co-resident workgroups assumed at most (0: the occupancy query's capacity)
    int force_abort;  // tests: the abort word raised at launch (as an exchange time-out raises it)
};
// The Fisher-KPP problem at small sizes (kan_small.hip): the whole forward solve / adjoint in one workgroup,
// wave = trajectory (B <= kFkSmallMaxBatch), lane = grid point (Nx <= 64, even), the pointwise KAN from the
// piecewise-polynomial tables (built by the caller: PP_PHI for the solve, PP_DPHI + PP_SWISH for the adjoint).
constexpr int kFkSmallMaxBatch = 16;
struct FkSmallArgs {
    int Nx, ni;
    double inv_w, x0;   // PPConst
    double cd, co;      // D·(-2/dx²), D/dx²
};
bool fk_small_supported(const LayerConst& hlc, const PPConst& hpc, int Nx, int64_t B);
hipError_t launch_fk_small_tsit5(const LayerConst& hlc, const PPConst& hpc, const LayerConst* lc, const double* p,
                                 const double* tables, const FkSmallArgs& s, const double* u0, int64_t B,
                                 const ChainSolveArgs& a, hipStream_t st);
hipError_t launch_fk_small_adjoint(const LayerConst& hlc, const PPConst& hpc, const LayerConst* lc, const double* p,
                                   const double* tables, const FkSmallArgs& s, int64_t B, const ChainAdjointArgs& a,
                                   hipStream_t st);
// Forward sensitivities of a small Fisher-KPP field (SciMLSensitivity ForwardDiffSensitivity, kan_small.hip):
// one workgroup of G + 2 waves (the values and one partial per parameter), Nx·B <= 64 points; u_save [n_save][n],
// s_save [n_save][P][n].  tab: the PP_PHI / PP_DPHI / PP_SWISH tables (built by the caller) or the reference formula.
constexpr int kFsensMaxWaves = 16;
bool fk_small_fsens_supported(const LayerConst& hlc, int Nx, int64_t B);
hipError_t launch_fk_small_fsens(const LayerConst& hlc, const PPConst& hpc, bool tab, const LayerConst* lc,
                                 const double* p, const double* tables, const FkSmallArgs& s, const double* u0,
                                 int64_t B, const ChainSolveArgs& a, double* s_save, hipStream_t st);
int pair_adjoint_workgroups(const LayerConst* hl, int64_t B, int S);
hipError_t launch_kd_pair_adjoint(const LayerConst* hl, const LayerConst* dlc, const double* p, int64_t B,
                                  PairAdjArgs pa, hipStream_t st);
constexpr int kChainAdjointMaxSteps = 1024;   // forward steps held in LDS
template <typename T>
hipError_t launch_kd_chain_adjoint(const LayerConst* hlcs, int nl, const LayerConst* lcs, const T* p, int64_t P,
                                   int64_t B, const ChainAdjointArgs& a, hipStream_t st, bool wide);
// A whole InterpolatingAdjoint step of a small chain per trajectory column (kd_chain_vjp_step_kernel, kan_col.hip):
// the six adjoint stages of kanode_solve.cpp adjoint_t in one launch, λ and kλ_1..kλ_7 of a column in registers.
// Stage s reads the forward dense output u_i + Σ_q su_c[s][q] k_{i,q} (K form, the forward step holding stage s)
// and the adjoint stage input λ + Σ_{q<=s} a[s][q] kλ_q; its kμ rows go to slab region s ([P][grid] of T: the
// stage kernel's per-block sums), the λ error partials (with want_error) after the six regions ([grid] doubles).
// chain_vjp_step_finish reduces the regions into km_out[0..5] (= kμ_2..kμ_7) and the error total, each in the
// order chain_vjp_finish_kernel uses: the step is bitwise the six kd_chain_vjp_stage_kernel launches.
template <typename T>
struct ChainKmOut {
    T* k[7];
};
template <typename T>
struct ChainAdjStep {
    const T* su_u[6];
    const T* su_k[6][7];
    double su_c[6][7];
    double a[6][6];   // h·a_sj
    double ec[7];     // h·btilde_j (the λ error of stage 6)
    double abstol, reltol;
    const T* lam;
    T* lam_out;       // λ_new (stage 6's input)
    const T* kl1;     // kλ_1 (FSAL)
    T* kl7;           // kλ_7
    int32_t want_error;
    // fsal = 1: the step follows a saveat stop whose jump and FSAL re-evaluation the host folded into it: first
    // λ' = λ + Σ_r jump[r] (the jump rows, in order) and kλ_1 = λ'ᵀ∂f/∂u at the forward dense output at the stop
    // (j_u + Σ_q j_c[q] j_k[q]), its kμ_1 into slab region 6 (km_out[6]); the step then starts from λ'
    int32_t fsal;
    int32_t njump, pad;
    const T* jump[8];
    const T* j_u;
    const T* j_k[7];
    double j_c[7];
};
template <typename T>
hipError_t launch_kd_chain_vjp_step(const LayerConst* hlcs, int nl, const LayerConst* lcs, const T* p, int64_t P,
                                    int64_t K, const ChainAdjStep<T>& a, int grid_cap, void* slab, size_t slab_bytes,
                                    T* const* km_out /* [6], [7] with fsal */, double* err_out, hipStream_t st);
// slab bytes launch_kd_chain_vjp_step needs for K columns over at most grid_cap blocks
size_t chain_vjp_step_slab_bytes(int64_t P, int64_t K, size_t esize, int grid_cap);
// whether launch_kd_chain_vjp_step covers this chain (no launch)
bool chain_vjp_step_supported(const LayerConst* hlcs, int nl, int64_t P, size_t esize);
// One Tsit5 step of a small chain per trajectory column (kd_chain_step_kernel, kan_col.hip)
struct ChainStepArgs {
    double a[6][6];   // dt·a_sj
    double e[7];      // dt·btilde_j
    double abstol, reltol;
    const void* u;
    const void* k1;
    void* k[6];       // k_2..k_7
    void* u_new;
};
template <typename T>
hipError_t launch_kd_chain_step(const LayerConst* hlcs, int nl, const LayerConst* lcs, const T* p, int64_t P,
                                int64_t K, const ChainStepArgs& a, double* err_slab, int slab_rows, double* err_out,
                                hipStream_t st);
constexpr int kChainSolveMaxBatch = 16;   // columns of one workgroup (256 lanes / 16)
template <typename T>
hipError_t launch_kd_chain_tsit5(const LayerConst* hlcs, int nl, const LayerConst* lcs, const T* p, int64_t P,
                                 const T* u0, int64_t B, const ChainSolveArgs& a, hipStream_t st);

// surrogate shapes (kan_wide.hip)
constexpr int kWideKT = 8;       // column tile of the wide-out kernels
constexpr int kWideOMax = 16;    // max out_dims of a wide-in layer
// Stage inputs formed by the wide-in forward of a surrogate pair (kanode_rhs_stage /
// kanode_vjp_stage): block (chunk, column) forms its inputs y = x + Σ su.c·su.k (the order of
// stage_lincomb_kernel) -> y_out, and, with lam, the adjoint stage input λs = lam + Σ sl.c·sl.k
// over the same index range -> ls_out (N_in == N_out), so no separate combination launches.
template <typename T>
struct WideStageIn {
    StageArgs<T> su;
    T* y_out;
    const T* lam;
    StageArgs<T> sl;
    T* ls_out;
};
template <typename T>
hipError_t launch_kd_fwd_widein(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, T* y, T* slab,
                                int64_t K, hipStream_t st, const WideStageIn<T>* si = nullptr);
// xslab (nullable): the layer input is the nblk chunk partials of the wide-in layer before it
// (launch_kd_fwd_widein with y == nullptr), summed in the reduce kernel's order by the consumer
template <typename T>
hipError_t launch_kd_fwd_wideout(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, T* y, int64_t K,
                                 hipStream_t st, const T* xslab = nullptr, int xnblk = 0);
// assign: the parameter cotangents are written (=) instead of accumulated (+=); every pbar entry of
// the layer has exactly one writer
template <typename T>
hipError_t launch_kd_vjp_wideout(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, const T* yb,
                                 T* xb, T* pbar, T* slab, int64_t K, hipStream_t st, const T* xslab = nullptr,
                                 int xnblk = 0, bool assign = false);
// inputs per block of the wide-in forward (kd_fwd_widein_co_kernel: at most kWIMaxV C and kWIMaxW W
// entries per thread of 256) and its chunk count
constexpr int kWideInMaxInputs = 64;
#ifndef KAN_WIDEIN_MAXV
#define KAN_WIDEIN_MAXV 32
#endif
constexpr int kWIMaxV = KAN_WIDEIN_MAXV;
constexpr int kWIMaxW = 8;
// The launch is latency-bound at a few columns: a wide input (I >= 32·kWideInMinChunks) gets at
// least kWideInMinChunks chunks (blocks per column), so Burgers' I = 512 is not left to 8
// long-running blocks (RHS 12.3 -> 9.5 us at B = 4).  Narrower inputs keep one chunk per
// kWIMaxV·tn entries (their launches are short anyway, and the summation order stays the one the
// narrow-layer parity tests were pinned with).
#ifndef KAN_WIDEIN_MIN_CHUNKS
#define KAN_WIDEIN_MIN_CHUNKS 16
#endif
constexpr int kWideInMinChunks = KAN_WIDEIN_MIN_CHUNKS;
__host__ __device__ inline int widein_cw(int O, int G, int I) {
    const int tn = (256 / O) * O;
    int cw = (kWIMaxV * tn) / (O * G);
    if (cw > kWideInMaxInputs) cw = kWideInMaxInputs;
    if (cw * O > kWIMaxW * tn) cw = (kWIMaxW * tn) / O;
    if (kWideInMinChunks > 0 && I >= 32 * kWideInMinChunks) {
        const int cmin = (I + kWideInMinChunks - 1) / kWideInMinChunks;
        if (cw > cmin) cw = cmin;
    }
    return cw < 1 ? 1 : cw;
}
inline int widein_chunks(const LayerConst& h) {
    const int cw = widein_cw(h.O, h.G, h.I);
    return (h.I + cw - 1) / cw;
}
template <typename T>
hipError_t launch_kd_vjp_widein(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, const T* yb, T* xb,
                                T* pbar, int64_t K, hipStream_t st, bool assign = false);
// The surrogate pair's whole pullback in two launches (kan_wide.hip): lc = the two layers' device
// constants (lc[0] wide-in, lc[1] wide-out); x = layer-1 input (u; with si the stage base u, y formed
// and written to si->y_out, λs to si->ls_out); ybar = λ (no si); xvjp = the layer-1 input the pullback
// reads (u, or si->y_out); pslab = the wide-in chunk partials (widein_chunks·K·H), S = the wide-out dot
// products' chunk partials (widein_chunks·H·(G+1)·K).  hipErrorNotSupported: K > kPairMaxK or the LDS
// would not fit (use the 4 launches).
constexpr int64_t kPairMaxK = 64;
// err_out (with si): the adjoint stage's λ error total, from per-block partials in err_slab (<= err_rows)
// bas (nullable): the wide-in basis store the forward blocks fill and the pullback blocks read
template <typename T>
hipError_t launch_kd_vjp_pair(const LayerConst& h0, const LayerConst& h1, const LayerConst* lc, const T* p,
                              const T* x, const WideStageIn<T>* si, const T* ybar, const T* xvjp, T* pslab, T* S,
                              T* xb, T* pbar, int64_t K, hipStream_t st, bool assign, double* err_slab = nullptr,
                              int err_rows = 0, double* err_out = nullptr, T* bas = nullptr);
// elements of the pair's wide-in basis store (bas above: φ [K][I][G], swish and swish' [K][I])
inline int64_t pair_basis_elems(const LayerConst& h0, int64_t K) { return K * h0.I * (h0.G + 2); }

// The pair pullback as a plan of its two launches (kan_wide.hip), so that a caller running adjoint stages
// back to back (the solver's deferred stages, kanode_abi.cpp) can hold a stage's second launch until the
// next stage is known and run the two together (launch_pair_second with `next`: kd_vjp_pair_ba_kernel).
// The wide-in basis store (WideBasisG): phi [K][I][G] = φ_g(x_ik), sw / dsw [K][I] = swish(x_ik), swish'.
template <typename T>
struct WideBasisG {
    T* phi;
    T* sw;
    T* dsw;
};
template <typename T>
struct PairBArgs {   // the second launch's kernel arguments
    const T* x;          // the layer-1 input the pullback reads (u, or the stage's y)
    const T* pslab;      // the first launch's hidden-layer chunk partials
    int nblk;
    const T* ybar;       // λ, or the stage's λs
    const T* S;          // the dot products' chunk partials
    T* xbar;
    T* pbar;
    int64_t K;
    int nP, nrc, np, nxg, cw, nbx, hb_off, assign;
    WideStageIn<T> si;
    double* err_slab;
    WideBasisG<T> bg;
};
template <typename T>
struct PairAArgs {   // the first launch's (a stage's) kernel arguments beyond the layer constants
    const T* x;          // the stage base u
    T* pslab;
    T* spart;
    WideStageIn<T> si;
    WideBasisG<T> bg;
};
template <typename T>
struct PairPlan {
    const LayerConst* lc;
    const T* p;
    int path;            // the wide-out layer's basis path
    bool stage;          // an adjoint stage (si given): the first launch forms y and λs
    PairAArgs<T> a;
    const T* ybar_a;     // (no stage) λ
    int nF, nblk, mv;    // first launch: blocks, wide-in chunks, load-slot instantiation (0 = <8,2>)
    PairBArgs<T> b;
    int gridB;
    size_t ldsB;
    double* err_out;     // the λ error total (b.err_slab != nullptr), summed over err_rows partials
    int err_rows;
    bool fuse_ok;        // this plan's second launch can carry the next stage's first (same chunking)
};
template <typename T>
hipError_t plan_kd_vjp_pair(const LayerConst& h0, const LayerConst& h1, const LayerConst* lc, const T* p, const T* x,
                            const WideStageIn<T>* si, const T* ybar, const T* xvjp, T* pslab, T* S, T* xb, T* pbar,
                            int64_t K, bool assign, double* err_slab, int err_rows, double* err_out, T* bas,
                            PairPlan<T>* out);
template <typename T>
hipError_t launch_pair_first(const PairPlan<T>& pl, hipStream_t st);
// next != nullptr: also runs next's first launch, inside this launch when the two fuse (*fused = true)
template <typename T>
hipError_t launch_pair_second(const PairPlan<T>& pl, const PairPlan<T>* next, hipStream_t st, bool* fused = nullptr);

}  // namespace kan
