// kanode_internal.hpp — handle accessors shared between the C-ABI translation units
// (kanode_abi.cpp owns the handle; kanode_solve.cpp is the integrator around it).
// C++ linkage, not part of the C-ABI.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "kanode.h"

namespace kan {
struct ChainSolveArgs;
struct ChainAdjointArgs;
struct AdjStepArgs;
struct PairAdjArgs;
struct FkLoopArgs;
struct AdjLoopArgs;
}

kanode_status kanode_internal_fail(kanode_handle* h, kanode_status s, const std::string& msg);
kanode_status kanode_internal_check(kanode_handle* h);     // non-null, sets the handle's device
int kanode_internal_dtype(const kanode_handle* h);
int64_t kanode_internal_state_length(const kanode_handle* h);
bool kanode_internal_square(const kanode_handle* h);       // N_in == N_out (an ODE right-hand side)
// While held, each RHS / VJP table set is built by the first launch only (p must not change).
void kanode_internal_hold_tables(kanode_handle* h, bool on);
// handle scratch: kanode_internal_scratch_rows() doubles of per-block partials (stream-ordered use)
double* kanode_internal_scratch(kanode_handle* h);
int kanode_internal_scratch_rows(const kanode_handle* h);
// kanode_vjp_stage with dp either accumulated (+=, the C-ABI semantics) or assigned (dp_assign)
// su_scale / sl_scale (nullable, device): the state / adjoint stage coefficients are multiplied
// by *scale in the kernels (device-resident step sizes)
// defer: on the Fisher-KPP table path, leave the stage's dp / error reduction pending until
// kanode_internal_vjp_flush (up to kMaxFinishJobs stages reduced in one launch); the stage's
// dp and error_sumsq outputs are valid only after the flush
kanode_status kanode_internal_vjp_stage(kanode_handle* h, const void* p, const void* u, const kanode_stage* state,
                                        const void* lam, const kanode_stage* adj, void* lamJ, void* dp, bool dp_assign,
                                        int64_t batch, void* stream, const double* su_scale = nullptr,
                                        const double* sl_scale = nullptr,
                                        bool defer = false);
kanode_status kanode_internal_vjp_flush(kanode_handle* h, void* stream);
void kanode_internal_vjp_discard(kanode_handle* h);
// the one-workgroup small-chain solve (kd_chain_tsit5_kernel): whether this handle's RHS and a
// batch qualify, and the launch (launched = false when the kernel does not cover the shape)
bool kanode_internal_chain_tsit5_ok(const kanode_handle* h, int64_t batch);
// KANODE_OPT_FUSED_SOLVE_CAP: dense-output slots of the one-workgroup solve (0 = its default)
int kanode_internal_fused_solve_cap(const kanode_handle* h);
kanode_status kanode_internal_chain_tsit5(kanode_handle* h, const void* p, const void* u0, int64_t batch,
                                          const kan::ChainSolveArgs* a, void* stream, bool& launched);
// a whole Tsit5 step per row on the Fisher-KPP table path (fk_step_pp_wave_kernel); launched =
// false when the handle is not that path (the caller runs the six stages)
// (q4x7: write the dense output as the interpolation polynomials Q_1..Q_4 and k_7)
bool kanode_internal_fk_step_ok(const kanode_handle* h);
// the device-controlled adaptive Fisher-KPP solve (KANODE_OPT_FK_DEVICE_LOOP): whether the handle takes it,
// and one step attempt (builds the table first when the solve has not)
bool kanode_internal_fk_loop_ok(const kanode_handle* h);
// the adaptive adjoint's device loop (kan_adjloop.hpp): ok when the handle takes it for this batch, with the
// rows step's slab base and grid (allocating the slabs); one attempt (rows + finish launches)
kanode_status kanode_internal_fk_adjoint_loop_geometry(kanode_handle* h, int64_t batch, void* stream, bool& ok,
                                                      double** slab, int64_t* grid);
kanode_status kanode_internal_fk_adjoint_loop(kanode_handle* h, const void* p, const kan::AdjLoopArgs* la,
                                              int64_t batch, void* stream);
kanode_status kanode_internal_fk_step_loop(kanode_handle* h, const void* p, const kan::FkLoopArgs* la, int64_t lq,
                                           int64_t batch, void* stream);
kanode_status kanode_internal_fk_step(kanode_handle* h, const void* p, const void* u, const void* k1,
                                      void* const* kout, void* u_new, const double* a6x6, const double* e7,
                                      const double* q4x7, double abstol, double reltol, double* err_out,
                                      int64_t batch, void* stream, bool& launched, double* err_parts = nullptr,
                                      int* nparts = nullptr);
// (err_parts, nparts: the step's per-block error partials written to err_parts -- at most
// kanode_internal_max_parts() of them, device-visible memory -- and their count returned for the caller
// to sum, instead of the total into err_out)
int kanode_internal_max_parts();
// the surrogate pair's adjoint stages run lazily when deferred (KANODE_OPT_PAIR_FUSE)
bool kanode_internal_pair_lazy(const kanode_handle* h);
// the integrator's mapped error-partial buffer for lazy pair stages (nullptr: off), see kanode_abi.cpp
void kanode_internal_set_err_parts(kanode_handle* h, double* parts, int* nparts);
// a whole Tsit5 step of a small chain per column (kd_chain_step_kernel); K-form dense output
kanode_status kanode_internal_chain_step(kanode_handle* h, const void* p, const void* u, const void* k1,
                                         void* const* kout, void* u_new, const double* a6x6, const double* e7,
                                         double abstol, double reltol, double* err_out, int64_t batch, void* stream,
                                         bool& launched);
// one InterpolatingAdjoint step on the Fisher-KPP table path (fk_vjp_step_pp_wave_kernel) plus
// its reductions: kμ of the six stages -> km[0..5] (assigned), the λ error -> err_out
// μ update a combined (fixed-step) adjoint step applies itself: mu_new = mu + a61·km1 + A
struct AdjMuUpdate {
    const double* mu;
    double* mu_new;
    const double* km1;
    double a61;
};
// An adaptive step's μ update, FSAL kμ_7 and μ error terms formed by one finish launch (AdjFinish):
// out[0] = the λ error sum, out[1 + q] = the μ terms (device, 1 + P doubles); *done set when it ran.
struct AdjAdaptiveFinish {
    const double* mu;
    double* mu_new;
    const double* km1;
    double* km7;
    double a6[6], bt[7];   // h·a6_j, h·btilde_j
    double abstol, reltol;
    double* out;
    bool* done;
};
kanode_status kanode_internal_fk_adjoint_step(kanode_handle* h, const void* p, kan::AdjStepArgs* a, void* const* km,
                                              double* err_out, int64_t batch, void* stream, bool& launched,
                                              bool* combined = nullptr, const AdjMuUpdate* mu = nullptr,
                                              const AdjAdaptiveFinish* af = nullptr);
kanode_status kanode_internal_chain_adjoint(kanode_handle* h, const void* p, int64_t batch,
                                            const kan::ChainAdjointArgs* a, void* stream, bool& launched);   // drop pending reductions (error paths)
// the persistent surrogate-pair adjoint (kd_pair_adjoint_kernel): whether the handle takes it
// (KANODE_OPT_PAIR_PERSIST, fp64 surrogate pair), its workgroup count, and the launch (launched =
// false when the kernel does not cover the shape / batch)
bool kanode_internal_pair_persist_ok(const kanode_handle* h);
int64_t kanode_internal_param_length(const kanode_handle* h);
int kanode_internal_pair_adjoint_workgroups(const kanode_handle* h, int64_t batch);
// KANODE_OPT_LAST_ADJOINT: record the path kanode_adjoint_tsit5 took (a kanode_adjoint_path value)
void kanode_internal_set_last_adjoint(kanode_handle* h, int path);
// KANODE_OPT_RECORD_ADJOINT_STEPS: the handle's record of the accepted adjoint step sizes, or null when off
// a whole InterpolatingAdjoint step of a small chain in one launch (+ its reduction): args = kan::ChainAdjStep<T>
// of the handle's dtype; km_out[0..5] <- kμ_2..kμ_7; launched = false where not covered
// (km_out[6] <- kμ_1 at the folded stop when args.fsal)
kanode_status kanode_internal_chain_adjoint_step(kanode_handle* h, const void* p, const void* args, void* const* km_out,
                                                 double* err_out, int64_t batch, void* stream, bool& launched);
// whether kanode_internal_chain_adjoint_step launches for this handle (the host may then fold stops into it)
bool kanode_internal_chain_adjoint_step_ok(const kanode_handle* h);
// forward sensitivities of a small Fisher-KPP field in one workgroup (kanode_forward_sensitivity_tsit5)
bool kanode_internal_fsens_ok(const kanode_handle* h, int64_t batch);
kanode_status kanode_internal_fk_fsens(kanode_handle* h, const void* p, const void* u0, int64_t batch,
                                       const kan::ChainSolveArgs* a, void* s_save, void* stream);
void kanode_internal_clear_adjoint_steps(kanode_handle* h);
std::vector<double>* kanode_internal_adjoint_steps(kanode_handle* h);
kanode_status kanode_internal_pair_adjoint(kanode_handle* h, const void* p, int64_t batch, kan::PairAdjArgs* a,
                                           void* stream, bool& launched);
// kanode_rhs_stage with the stage coefficients (c, ec) multiplied by *cscale (device) in the kernels;
// while *skip != 0 (device, nullable) the stage kernels return at once (a finished graph-mode solve)
kanode_status kanode_internal_rhs_stage(kanode_handle* h, const void* p, const void* u, const kanode_stage* sg,
                                        void* du, int64_t batch, void* stream, const double* cscale,
                                        const int32_t* skip = nullptr);
// allocate every workspace the stage calls of this batch use (before hipGraph capture)
kanode_status kanode_internal_prepare(kanode_handle* h, int64_t batch, hipStream_t st);
// address of the handle's kanode_solution* slot for solves without a dense output (freed by kanode_destroy)
void* kanode_internal_solution_cache(kanode_handle* h);
