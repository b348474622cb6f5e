// kan_adjloop.hpp — the adaptive Fisher-KPP InterpolatingAdjoint with its step control on the device
// (kanode_solve.cpp adjoint_t's device loop, KANODE_OPT_FK_DEVICE_LOOP).
//
// One attempt = the rows kernel (fk_vjp_step_rows_kernel, DEV) + the finish kernel (adj_finish_kernel, DEV),
// both reading their arguments from plan[it & 1]; the finish's last workgroup to arrive sums the error
// terms, runs adjoint_t's PI controller and writes plan[(it + 1) & 1] for the next attempt.  A step that
// lands on a saveat stop pauses the loop (status 3): the host takes the jump λ += ∂L/∂u(t_j) and the FSAL
// re-evaluation exactly as its own loop does, then resumes.  The plan builder below is shared by the host
// (the first attempt and every resume) and the device, so both form the same coefficients and pointers.
#pragma once
#include "kan_kernels.hpp"
#include "kan_tsit5.hpp"

namespace kan {

struct AdjLoopCtl {
    double tau, h, qold;
    int64_t si, naccept, nreject, it, nf;
    int64_t fi;                 // forward step of the last planned stage (the interval search starts there)
    int32_t status;             // 0 running, 1 done, 2 maxiters reached, 3 paused on a saveat stop
    int32_t lc, mc, fs;         // λ and μ buffer parity; FSAL swap of kλ_1 / kλ_7 and kμ_1 / kμ_7
};
struct AdjLoopPlan {
    AdjStepArgs a;
    AdjFinish f;
};
struct AdjLoopArgs {
    AdjLoopCtl* ctl;
    AdjLoopCtl* mirror;         // the host's mapped copy (device address)
    AdjLoopPlan* plan;          // [2], by attempt parity
    unsigned* arrive;           // the finish launch's arrival counter (0 between launches)
    double* lam[2];
    double* kl[7];
    double* mu[2];
    double* km[7];
    void* const* slots;         // forward dense-output slots (u_i, Q_1..Q_4, k_7)
    const double* fts;          // forward accepted steps: start time, size
    const double* fdts;
    int64_t nsteps;
    double* slab;               // the rows kernel's slab base
    int64_t grid;               // its grid
    int64_t P, n;
    double* out;                // [1 + P] the finish's error terms
    const double* stops;        // [nstops] τ of the saveat stops, the last = TT
    int64_t nstops;
    double tf, TT, abstol, reltol, dtmin, beta1, beta2, gamma, qmin, qmax, qoldinit, ntot;
    int64_t maxiters;
    double* hs;                 // accepted step sizes (KANODE_OPT_RECORD_ADJOINT_STEPS) or null
    int64_t hs_cap;
};

// the largest i < nsteps with ts[i] <= t (0 if none): std::upper_bound - 1, clamped, searched from `i`
template <class FW>
__host__ __device__ inline int64_t adj_loop_interval(const FW& fw, int64_t nsteps, double t, int64_t i) {
    if (i > nsteps - 1) i = nsteps - 1;
    if (i < 0) i = 0;
    while (i > 0 && fw.ts(i) > t) --i;
    while (i + 1 < nsteps && fw.ts(i + 1) <= t) ++i;
    return i;
}

// The arguments of the attempt at state c (adjoint_t's per-step host code and kanode_internal_fk_adjoint_step
// / launch_fk_vjp_step_pp's fields, in their arithmetic).  fw: ts(i), dts(i), slot(i) of the forward steps.
template <class FW>
__host__ __device__ inline void adj_loop_plan(const AdjLoopArgs& la, AdjLoopCtl& c, AdjLoopPlan& pl, const FW& fw) {
    using K = Tsit5Tab;
    AdjStepArgs& a = pl.a;
    const double h = c.h, tau = c.tau;
    double* const kl0 = c.fs ? la.kl[6] : la.kl[0];
    double* const kl6 = c.fs ? la.kl[0] : la.kl[6];
    double* const km0 = c.fs ? la.km[6] : la.km[0];
    double* const km6 = c.fs ? la.km[0] : la.km[6];
    a.kl[0] = kl0;
    for (int j = 1; j < 6; ++j) a.kl[j] = la.kl[j];
    a.kl[6] = kl6;
    int64_t fi = c.fi;
    for (int i = 0; i < 6; ++i) {
        for (int j = 0; j < 6; ++j) a.a[i][j] = j <= i ? h * K::TA[i][j] : 0.0;
        const double t = la.tf - (i == 5 ? tau + h : tau + K::TC[i] * h);
        fi = adj_loop_interval(fw, la.nsteps, t, fi);
        const double r = (t - fw.ts(fi)) / fw.dts(fi);
        const double th = r < 0.0 ? 0.0 : (r > 1.0 ? 1.0 : r);   // std::min(1, std::max(0, r))
        const double* su = static_cast<const double*>(fw.slot(fi));
        a.su_u[i] = su;
        for (int m = 0; m < 4; ++m) a.su_q[i][m] = su + (m + 1) * la.n;
        a.su_c[i][0] = th;
        a.su_c[i][1] = th * th;
        a.su_c[i][2] = th * th * th;
        a.su_c[i][3] = th * th * th * th;
    }
    c.fi = fi;
    for (int j = 0; j < 7; ++j) a.ec[j] = h * K::BT[j];
    a.abstol = la.abstol;
    a.reltol = la.reltol;
    a.lam = la.lam[c.lc];
    a.lam_out = la.lam[c.lc ^ 1];
    for (int s = 0; s < 6; ++s) a.slab[s] = la.slab + (int64_t)s * la.grid * la.P;
    a.err_slab = la.slab + (int64_t)6 * la.grid * la.P;
    a.reload[0] = 1;
    for (int s = 1; s < 6; ++s) a.reload[s] = a.su_u[s] == a.su_u[s - 1] ? 0 : 1;   // (the Q_m follow u_i)
    a.combine = 2;
    a.fin_ctr = nullptr;
    AdjFinish& f = pl.f;
    const int which[3] = {0, 1, 5};   // A, E, kμ_7 (kanode_internal_fk_adjoint_step)
    for (int q = 0; q < 6; ++q) {
        f.slab[q] = q < 3 ? a.slab[which[q]] : nullptr;
        f.ca[q] = q == 0 ? 1.0 : 0.0;
        f.ce[q] = q == 1 ? 1.0 : 0.0;
    }
    f.nslab = 3;
    f.k7 = 2;
    f.tr = 1;
    f.pad = 0;
    f.nblk = la.grid;
    f.a0 = h * K::TA[5][0];
    f.e0 = h * K::BT[0];
    f.abstol = la.abstol;
    f.reltol = la.reltol;
    f.mu = la.mu[c.mc];
    f.mu_new = la.mu[c.mc ^ 1];
    f.km1 = km0;
    f.km7 = km6;
    f.err_slab = a.err_slab;
    f.out = la.out;
}

// adjoint_t's loop top: done / maxiters, else the step clipped to the next stop (status stays 0)
// stop = stops[c.si] (the host passes its own copy: la.stops is device memory)
__host__ __device__ inline void adj_loop_top(const AdjLoopArgs& la, AdjLoopCtl& c, double stop) {
    if (c.tau >= la.TT - 1e-14 * (la.TT > 1.0 ? la.TT : 1.0)) c.status = 1;
    else if (c.it >= la.maxiters) c.status = 2;
    else {
        const double room = stop - c.tau;
        c.h = c.h < room ? c.h : room;
    }
}

}  // namespace kan
