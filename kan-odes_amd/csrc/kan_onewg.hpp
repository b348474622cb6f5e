// kan_onewg.hpp — a whole Tsit5 solve and a whole InterpolatingAdjoint in ONE workgroup, for problems
// small enough that launches and host round trips, not arithmetic, decide the time: the reference's own
// driver sizes (one Lotka-Volterra trajectory, LV_driver_KANODE.jl:180-184,279-291; one 26-point
// Fisher-KPP field, PDE examples/Fisher-KPP_Source.jl:34-49,95-103,194-213).
//
// The drivers restate kanode_solve.cpp solve_t / adjoint_t (OrdinaryDiffEqTsit5 1.1.0 tableau and PI
// controller, Hairer-Wanner initial step, saveat from the dense output, FSAL; SciMLSensitivity 7.69
// InterpolatingAdjoint over [λ; μ] with the saveat jumps and the FSAL re-evaluation after each jump).
// Every thread takes every step-control decision itself on block sums that all threads receive in the
// same order, so no thread ever waits on a host.  The right-hand side is a model class:
//
//   bool act; int64_t idx, n; int P;     this thread's state entry (idx < n when act), its parameters
//   T rhs(T y);                          f(y)_idx (collective: every thread of the block calls it)
//   T vjp(T y, T ls, T* km);             λsᵀ∂f/∂u at y for this entry (0 when !act), and the adjoint's
//                                        kμ = (∂f/∂p)ᵀλs summed over the state, written to km[0..P) (LDS);
//                                        collective, ends with a block barrier
//
// ChainModel (kan_col.hip) is the small-chain network; FkSmallModel (kan_small.hip) the Fisher-KPP RHS of
// a field of <= 64 points per wave.  The dense-output layout is the host loop's K form, one contiguous
// block [step][u_n, k_2..k_7][n] (ChainSolveArgs::rec), so the host-loop adjoint can read it as well.
#pragma once
#include "kan_common.hpp"
#include "kan_kernels.hpp"
#include "kan_tsit5.hpp"

namespace kan {

// The step controller's powers EEst^β1 and qold^β2 as exp2(y·log2 x) (x > 0 here): on one wave the full pow
// sits on each step's dependency chain, and this form took the FK26 forward solve 169 -> 148 us, its adjoint
// 647 -> 623 us (profiles/r05/small/onewg_pow_ab.txt).  It can differ from pow in the last bits, so a step size
// can differ from the host loop's at rounding level (the tests' bars allow for that).  KAN_ONEWG_STDPOW: pow.
#ifdef KAN_ONEWG_STDPOW
#define KAN_ONEWG_POW(x, y) ::pow(x, y)
#else
#define KAN_ONEWG_POW(x, y) ::exp2((y) * ::log2(x))
#endif

// Σ over the block of v (inactive entries give 0), the same ordered total in every thread.  red: LDS of
// blockDim / 64 doubles.
__device__ __forceinline__ double onewg_bsum(double v, double* red) {
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = v;
    __syncthreads();
    double t = red[0];
    for (int w = 1; w < (int)(blockDim.x / kWave); ++w) t += red[w];
    return t;
}

// The forward solve (solve_t): u0[n] -> u_save [n_save][n], the dense output and the counters in a.out.
template <typename T, class Mdl>
__device__ __forceinline__ void onewg_tsit5(Mdl& m, const T* __restrict__ u0, const ChainSolveArgs& a, double* red) {
    using K = Tsit5Tab;
    const bool act = m.act;
    const int64_t idx = m.idx, n = m.n;
    T* __restrict__ usave = reinterpret_cast<T*>(a.u_save);
    T* __restrict__ rec = reinterpret_cast<T*>(a.rec);
    auto bsum = [&](double v) -> double { return onewg_bsum(act ? v : 0.0, red); };
    T u = act ? u0[idx] : T(0);
    T k[7];
    k[0] = m.rhs(u);
    if (rec && act) reinterpret_cast<T*>(a.k1_0)[idx] = k[0];
    const double t0 = a.t0, tf = a.tf;
    int64_t si = 0;
    while (si < a.n_save && a.saveat[si] <= t0 + 1e-14 * ::fmax(1.0, ::fabs(t0))) {
        if (act && usave) usave[si * n + idx] = u;
        ++si;
    }
    double dt = a.dt;
    if (a.adaptive && !(a.dt > 0)) {   // Hairer & Wanner (solve_t initdt)
        const double sk = ::fma(a.reltol, kabs((double)u), a.abstol);
        const double d0 = ::sqrt(bsum(((double)u / sk) * ((double)u / sk)) / (double)n);
        const double d1 = ::sqrt(bsum(((double)k[0] / sk) * ((double)k[0] / sk)) / (double)n);
        double dt0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        dt0 = ::fmin(dt0, tf - t0);
        const T f1 = m.rhs(kfma<T>((T)dt0, k[0], u));
        const double e = ::fma(-1.0, (double)k[0], (double)f1) / sk;
        const double d2 = ::sqrt(bsum(e * e) / (double)n) / dt0;
        const double mx = ::fmax(d1, d2);
        const double dt1 = mx <= 1e-15 ? ::fmax(1e-6, dt0 * 1e-3) : ::pow(0.01 / mx, 1.0 / 5.0);
        dt = ::fmin(::fmin(100 * dt0, dt1), tf - t0);
    }
    double qold = a.qoldinit, t = t0;
    int64_t naccept = 0, nreject = 0, nf = 0, it = 0, status = 0;
    for (; it < a.maxiters; ++it) {
        if (t >= tf - 1e-14 * ::fmax(1.0, ::fabs(tf))) break;
        dt = ::fmin(dt, tf - t);
        T y = u;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            y = u;
#pragma unroll
            for (int q = 0; q <= i; ++q) y = kfma<T>((T)(dt * K::TA[i][q]), k[q], y);
            k[i + 1] = m.rhs(y);
        }
        nf += 6;
        double dtnew = dt;
        if (a.adaptive) {
            double ev = 0.0;
#pragma unroll
            for (int q = 0; q < 6; ++q) ev = ::fma(dt * K::BT[q], (double)k[q], ev);
            const double e = ::fma(dt * K::BT[6], (double)k[6], ev);
            const double sk = ::fma(a.reltol, ::fmax(kabs((double)u), kabs((double)y)), a.abstol);
            const double r = e / sk;
            const double eest = ::sqrt(bsum(r * r) / (double)n);
            const double q11 = eest > 0 ? KAN_ONEWG_POW(eest, a.beta1) : 0.0;
            if (eest > 1.0 && dt > a.dtmin) {
                ++nreject;
                dt = dt / ::fmin(1.0 / a.qmin, q11 / a.gamma);
                continue;
            }
            double q = q11 / KAN_ONEWG_POW(qold, a.beta2);
            q = ::fmax(1.0 / a.qmax, ::fmin(1.0 / a.qmin, q / a.gamma));
            if (1.0 <= q && q <= 1.0) q = 1.0;   // qsteady_min = qsteady_max = 1
            dtnew = q > 0 ? dt / q : dt * a.qmax;
            qold = ::fmax(eest, a.qoldinit);
        }
        if (rec && naccept >= a.cap) {   // dense-output storage exhausted
            status = 2;
            break;
        }
        const double tn = t + dt;
        while (si < a.n_save && a.saveat[si] <= tn + 1e-12 * ::fmax(1.0, ::fabs(tn))) {
            const double tsv = a.saveat[si];
            T v = y;
            if (!(::fabs(tsv - tn) <= 1e-12 * ::fmax(1.0, ::fabs(tn)))) {
                double w[7];
                tsit5_interp_weights((tsv - t) / dt, w);
                v = u;
#pragma unroll
                for (int q = 0; q < 7; ++q) v = kfma<T>((T)(w[q] * dt), k[q], v);
            }
            if (act && usave) usave[si * n + idx] = v;
            ++si;
        }
        if (rec) {
            T* __restrict__ r = rec + naccept * 7 * n;
            if (act) {
                r[idx] = u;
#pragma unroll
                for (int q = 1; q < 7; ++q) r[(int64_t)q * n + idx] = k[q];
            }
            if (threadIdx.x == 0) {
                a.ts[naccept] = t;
                a.dts[naccept] = dt;
                if (a.hts) {
                    a.hts[naccept] = t;
                    a.hts[a.cap + naccept] = dt;
                }
            }
        }
        u = y;   // commit u <- u_new, k_1 <- k_7 (FSAL)
        k[0] = k[6];
        t = tn;
        ++naccept;
        dt = dtnew;
    }
    if (status == 0 && it == a.maxiters && !(t >= tf - 1e-14 * ::fmax(1.0, ::fabs(tf)))) status = 1;
    if (threadIdx.x == 0) {
        if (a.hts) __threadfence_system();   // the host reads the step records once it sees the counters
        a.out[0] = naccept;
        a.out[1] = nreject;
        a.out[2] = nf + 1;
        a.out[3] = status;
    }
}

// (the generic small-chain shapes are too large for the stage loop to be unrolled; their stage values then
// live in scratch, which only the non-LV small chains pay for)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wpass-failed"
// Copy the forward's dense output ([nsteps][7][n]) and k1_0 ([n]) into LDS at dst (the caller's sizing:
// (nsteps·7 + 1)·n elements): at one or a few trajectories every adjoint stage interpolates it, and the global
// loads' latency would sit on each stage's dependency chain.  Ends with a barrier.
template <typename T>
__device__ __forceinline__ void onewg_stage_rec(T* __restrict__ dst, const ChainAdjointArgs& a, int64_t n) {
    const T* __restrict__ rec = reinterpret_cast<const T*>(a.rec);
    const T* __restrict__ k1 = reinterpret_cast<const T*>(a.k1_0);
    const int64_t m = a.nsteps * 7 * n;
    for (int64_t i = threadIdx.x; i < m; i += blockDim.x) dst[i] = rec[i];
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) dst[m + i] = k1[i];
    __syncthreads();
}

// The adjoint (adjoint_t): the backward Tsit5 over [λ; μ] in τ = tf - t, reading the forward's dense output
// (a.rec).  λ and its seven stage values stay in registers; μ ([2][P], zeroed by the caller) and its seven
// stage vectors km ([7][P]) live in LDS, as do the forward step times tsl / dtsl ([nsteps] each, copied by
// the caller).  recl: the dense output ([nsteps][7][n]) followed by k1_0 ([n]) in LDS when the caller staged
// it there (onewg_stage_rec), else null (read from a.rec).  Writes du0, dp and the counters.
template <typename T, class Mdl>
__device__ __forceinline__ void onewg_adjoint(Mdl& m, const ChainAdjointArgs& a, T* __restrict__ mu,
                                              T* __restrict__ km, const double* __restrict__ tsl,
                                              const double* __restrict__ dtsl, double* red,
                                              const T* __restrict__ recl = nullptr) {
    using K = Tsit5Tab;
    const int P = m.P;
    const bool act = m.act;
    const int64_t idx = m.idx, n = m.n;
    const T* __restrict__ rec = recl ? recl : reinterpret_cast<const T*>(a.rec);
    const T* __restrict__ rk1 = recl ? recl + a.nsteps * 7 * n : reinterpret_cast<const T*>(a.k1_0);
    const T* __restrict__ dl = reinterpret_cast<const T*>(a.dl_du);
    const double t0 = a.t0, tf = a.tf, TT = tf - t0;
    const int64_t ntot = n + P;
    auto bsum = [&](double v) -> double { return onewg_bsum(v, red); };
    auto add_rows = [&](int gidx, T l) -> T {   // λ += Σ dl_du[r] (rows in order)
        for (int32_t q = a.joff[gidx]; q < a.joff[gidx + 1]; ++q)
            if (act) l = l + dl[(int64_t)a.jrows[q] * n + idx];
        return l;
    };
    int64_t cur = a.nsteps - 1;   // forward step holding t (moves back as τ grows)
    // adjoint RHS at τ with adjoint stage input ls: returns λsᵀ∂f/∂u, kμ -> km[slot]
    auto adj = [&](double tau, T ls, int slot) -> T {
        const double t = tf - tau;
        while (cur > 0 && tsl[cur] > t) --cur;
        while (cur + 1 < a.nsteps && tsl[cur + 1] <= t) ++cur;
        const double dti = dtsl[cur];
        const double th = ::fmin(1.0, ::fmax(0.0, (t - tsl[cur]) / dti));
        T y = T(0);
        if (act) {
            const T* __restrict__ r = rec + cur * 7 * n;
            const T* __restrict__ k1 = cur == 0 ? rk1 : rec + (cur - 1) * 7 * n + 6 * n;
            T kv[7];
            kv[0] = k1[idx];
#pragma unroll
            for (int q = 1; q < 7; ++q) kv[q] = r[(int64_t)q * n + idx];
            y = r[idx];
#pragma unroll
            for (int q = 0; q < 7; ++q) {
                const double b = th * (K::RI[q][0] + th * (K::RI[q][1] + th * (K::RI[q][2] + th * K::RI[q][3])));
                y = kfma<T>((T)(b * dti), kv[q], y);
            }
        }
#ifdef KAN_ONEWG_NOVJP   // timing experiment only: the driver without the model's pullback (wrong results)
        (void)slot;
        return y * ls;
#else
        return m.vjp(y, act ? ls : T(0), km + (size_t)slot * P);
#endif
    };
    T lam = T(0);
    if (dl) lam = add_rows(0, lam);
    int mc = 0;   // mu[mc] holds μ (zero)
    T kl[7];
    kl[0] = adj(0.0, lam, 0);
    int64_t nf = 1;
    double h = a.dt;
    if (a.adaptive && !(a.dt > 0)) {   // Hairer-Wanner on [λ; μ]
        double s0 = 0.0, s1 = 0.0;
        {
            const double sk = ::fma(a.reltol, kabs((double)lam), a.abstol);
            const double r0 = (double)lam / sk, r1 = (double)kl[0] / sk;
            s0 = act ? r0 * r0 : 0.0;
            s1 = act ? r1 * r1 : 0.0;
        }
        for (int q = threadIdx.x; q < P; q += blockDim.x) {
            const double mv = (double)mu[q];
            const double sk = ::fma(a.reltol, kabs(mv), a.abstol);
            const double r0 = mv / sk, r1 = (double)km[q] / sk;
            s0 += r0 * r0;
            s1 += r1 * r1;
        }
        const double d0 = ::sqrt(bsum(s0) / (double)ntot), d1 = ::sqrt(bsum(s1) / (double)ntot);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        h0 = ::fmin(h0, TT);
        kl[1] = adj(h0, kfma<T>((T)h0, kl[0], lam), 1);
        ++nf;
        double s2 = 0.0;
        {
            const double sk = ::fma(a.reltol, kabs((double)lam), a.abstol);
            const double e = ::fma(-1.0, (double)kl[0], (double)kl[1]) / sk;
            s2 = act ? e * e : 0.0;
        }
        for (int q = threadIdx.x; q < P; q += blockDim.x) {
            const double sk = ::fma(a.reltol, kabs((double)mu[q]), a.abstol);
            const double e = ::fma(-1.0, (double)km[q], (double)km[P + q]) / sk;
            s2 += e * e;
        }
        const double d2 = ::sqrt(bsum(s2) / (double)ntot) / h0;
        const double mx = ::fmax(d1, d2);
        const double h1 = mx <= 1e-15 ? ::fmax(1e-6, h0 * 1e-3) : ::pow(0.01 / mx, 1.0 / 5.0);
        h = ::fmin(::fmin(100 * h0, h1), TT);
    }
    double qold = a.qoldinit, tau = 0.0;
    int64_t si = 0, naccept = 0, nreject = 0, it = 0, status = 0;
    int k0 = 0;   // km slot of kμ_1 (FSAL swaps slots 0 and 6)
    for (; it < a.maxiters; ++it) {
        if (tau >= TT - 1e-14 * ::fmax(1.0, TT)) break;
        h = ::fmin(h, a.stops[si] - tau);
        int ks[7];
        ks[0] = k0;
#pragma unroll
        for (int q = 1; q < 6; ++q) ks[q] = q;
        ks[6] = k0 == 0 ? 6 : 0;
        T ls = lam;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            ls = lam;
#pragma unroll
            for (int q = 0; q <= i; ++q) ls = kfma<T>((T)(h * K::TA[i][q]), kl[q], ls);
            kl[i + 1] = adj(i == 5 ? tau + h : tau + K::TC[i] * h, ls, ks[i + 1]);
        }
        nf += 6;
        // μ_new = μ + h Σ a_6j kμ_j (and its error), λ error
        T* __restrict__ mu0 = mu + (size_t)mc * P;
        T* __restrict__ mu1 = mu + (size_t)(mc ^ 1) * P;
        double s = 0.0;
        for (int q = threadIdx.x; q < P; q += blockDim.x) {
            T v = mu0[q];
#pragma unroll
            for (int r = 0; r < 6; ++r) v = kfma<T>((T)(h * K::TA[5][r]), km[(size_t)ks[r] * P + q], v);
            mu1[q] = v;
            if (a.adaptive) {
                double ev = 0.0;
#pragma unroll
                for (int r = 0; r < 6; ++r) ev = ::fma(h * K::BT[r], (double)km[(size_t)ks[r] * P + q], ev);
                const double e = ::fma(h * K::BT[6], (double)km[(size_t)ks[6] * P + q], ev);
                const double sk = ::fma(a.reltol, ::fmax(kabs((double)mu0[q]), kabs((double)v)), a.abstol);
                s += (e / sk) * (e / sk);
            }
        }
        double hnew = h;
        if (a.adaptive) {
            if (act) {
                double ev = 0.0;
#pragma unroll
                for (int r = 0; r < 6; ++r) ev = ::fma(h * K::BT[r], (double)kl[r], ev);
                const double e = ::fma(h * K::BT[6], (double)kl[6], ev);
                const double sk = ::fma(a.reltol, ::fmax(kabs((double)lam), kabs((double)ls)), a.abstol);
                s += (e / sk) * (e / sk);
            }
            const double eest = ::sqrt(bsum(s) / (double)ntot);
            const double q11 = eest > 0 ? KAN_ONEWG_POW(eest, a.beta1) : 0.0;
            if (eest > 1.0 && h > a.dtmin) {
                ++nreject;
                h = h / ::fmin(1.0 / a.qmin, q11 / a.gamma);
                __syncthreads();   // mu1 is rewritten by the retry
                continue;
            }
            double q = q11 / KAN_ONEWG_POW(qold, a.beta2);
            q = ::fmax(1.0 / a.qmax, ::fmin(1.0 / a.qmin, q / a.gamma));
            if (1.0 <= q && q <= 1.0) q = 1.0;
            hnew = q > 0 ? h / q : h * a.qmax;
            qold = ::fmax(eest, a.qoldinit);
        }
        __syncthreads();   // mu1 complete
        tau = tau + h;
        lam = ls;          // λ <- the last stage input (λ + h Σ a_6j kλ_j)
        mc ^= 1;
        kl[0] = kl[6];     // FSAL
        k0 = ks[6];
        if (a.hs && threadIdx.x == 0 && naccept < a.hs_cap) a.hs[naccept] = h;
        ++naccept;
        if (::fabs(tau - a.stops[si]) <= 1e-12 * ::fmax(1.0, TT)) {
            tau = a.stops[si];
            if (si + 1 < a.nstops) {
                if (dl && a.joff[si + 2] > a.joff[si + 1]) {
                    lam = add_rows((int)si + 1, lam);   // callback: λ += ∂L/∂u(t_j)
                    kl[0] = adj(tau, lam, k0);          // u_modified!: FSAL re-evaluated
                    ++nf;
                }
            }
            si = si + 1 < a.nstops ? si + 1 : a.nstops - 1;
        }
        h = hnew;
    }
    if (it == a.maxiters && !(tau >= TT - 1e-14 * ::fmax(1.0, TT))) status = 1;
    if (dl) lam = add_rows((int)a.nstops, lam);
    if (a.du0 && act) reinterpret_cast<T*>(a.du0)[idx] = lam;
    if (a.dp)
        for (int q = threadIdx.x; q < P; q += blockDim.x) reinterpret_cast<T*>(a.dp)[q] = mu[(size_t)mc * P + q];
    if (threadIdx.x == 0) {
        a.out[0] = naccept;
        a.out[1] = nreject;
        a.out[2] = nf;
        a.out[3] = status;
    }
}
#pragma clang diagnostic pop

}  // namespace kan
