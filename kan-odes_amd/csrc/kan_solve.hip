// kan_solve.hip — device-side step control of the Tsit5 integrator (kanode_solve.cpp graph mode).
//
// In graph mode a solve is a hipGraph of K step slots, replayed until the control block says
// done: each slot is the six stage launches (the step size read from device memory through
// StageArgs::cscale) and one tsit5_post_kernel, which takes the accept/reject decision of
// OrdinaryDiffEq's PI controller from the embedded-error total, writes the saveat values that
// fall inside an accepted step from the dense output, records the step for the adjoint and
// commits u <- u_new, k_1 <- k_7 (FSAL).  Every thread takes the same decision from the same
// inputs; thread 0 of block 0 writes the next control block (double-buffered by slot parity,
// so no block reads a control block that is being written).  Same controller arithmetic and
// order as the host loop (kanode_solve.cpp solve_t).
#include "kan_common.hpp"
#include "kan_kernels.hpp"

namespace kan {


template <typename T>
__global__ void __launch_bounds__(kBlock)
tsit5_post_kernel(const SolveCtl* __restrict__ cin, SolveCtl* __restrict__ cout, const double* __restrict__ sumsq,
                  Tsit5Bufs<T> bf, Tsit5PostArgs pa, int64_t n) {
    const SolveCtl c = *cin;
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    if (c.done) {
        if (lead) *cout = c;
        return;
    }
    const double t = c.t, dt = c.dt;
    bool accept = true;
    double dtnew = dt, qold = c.qold, eest = 0.0;
    if (pa.adaptive) {
        eest = ::sqrt(*sumsq / (double)n);
        const double q11 = eest > 0 ? ::pow(eest, pa.beta1) : 0.0;
        if (eest > 1.0 && dt > pa.dtmin) {
            accept = false;
            dtnew = dt / ::fmin(1.0 / pa.qmin, q11 / pa.gamma);
        } else {
            double q = q11 / ::pow(qold, pa.beta2);
            q = ::fmax(1.0 / pa.qmax, ::fmin(1.0 / pa.qmin, q / pa.gamma));
            if (1.0 <= q && q <= 1.0) q = 1.0;   // qsteady_min = qsteady_max = 1
            dtnew = q > 0 ? dt / q : dt * pa.qmax;
            qold = ::fmax(eest, pa.qoldinit);
        }
    }
    const bool full = accept && pa.record && c.naccept >= pa.slot_cap;   // storage exhausted: stop before it
    SolveCtl o = c;
    o.attempts = c.attempts + 1;
    o.eest = eest;
    if (full) {
        o.done = 1;
        o.status = 2;
        if (lead) *cout = o;
        return;
    }
    if (!accept) {
        o.dt = dtnew;
        o.nreject = c.nreject + 1;
        o.accepted = 0;
    } else {
        const double tn = t + dt;
        int64_t si1 = c.si;
        while (si1 < pa.n_save && pa.saveat[si1] <= tn + 1e-12 * ::fmax(1.0, ::fabs(tn))) ++si1;
        T* __restrict__ rec = pa.record ? reinterpret_cast<T*>(bf.slots[c.naccept]) : nullptr;
        for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
            const T ui = bf.U[i];
            T kv[7];
#pragma unroll
            for (int j = 0; j < 7; ++j) kv[j] = bf.K[j][i];
            const T un = bf.UNEW[i];
            for (int64_t s = c.si; s < si1; ++s) {
                const double ts = pa.saveat[s];
                T v;
                if (::fabs(ts - tn) <= 1e-12 * ::fmax(1.0, ::fabs(tn))) {
                    v = un;
                } else {
                    double w[7];
                    tsit5_interp_weights((ts - t) / dt, w);
                    v = ui;
#pragma unroll
                    for (int j = 0; j < 7; ++j) v = kfma<T>((T)(w[j] * dt), kv[j], v);
                }
                bf.save[s * n + i] = v;
            }
            if (rec) {
                rec[i] = ui;
#pragma unroll
                for (int j = 1; j < 7; ++j) rec[(int64_t)j * n + i] = kv[j];
            }
            bf.U[i] = un;           // commit: u <- u_new, k_1 <- k_7 (FSAL)
            bf.K[0][i] = kv[6];
        }
        if (lead && pa.record) {
            pa.ts_rec[c.naccept] = t;
            pa.dts_rec[c.naccept] = dt;
        }
        o.t = tn;
        o.dt = ::fmin(dtnew, pa.tf - tn);
        o.qold = qold;
        o.naccept = c.naccept + 1;
        o.si = si1;
        o.accepted = 1;
        if (tn >= pa.tf - 1e-14 * ::fmax(1.0, ::fabs(pa.tf))) o.done = 1;
    }
    if (!o.done && o.attempts >= pa.maxiters) {
        o.done = 1;
        o.status = 1;
    }
    if (lead) *cout = o;
}

template <typename T>
hipError_t launch_tsit5_post(const SolveCtl* cin, SolveCtl* cout, const double* sumsq, const Tsit5Bufs<T>& bf,
                             const Tsit5PostArgs& pa, int64_t n, hipStream_t st) {
    const int grid = grid_for(n, kBlock, kGridCap);
    hipLaunchKernelGGL((tsit5_post_kernel<T>), dim3(grid), dim3(kBlock), 0, st, cin, cout, sumsq, bf, pa, n);
    return hipGetLastError();
}

template hipError_t launch_tsit5_post<double>(const SolveCtl*, SolveCtl*, const double*, const Tsit5Bufs<double>&,
                                              const Tsit5PostArgs&, int64_t, hipStream_t);
template hipError_t launch_tsit5_post<float>(const SolveCtl*, SolveCtl*, const double*, const Tsit5Bufs<float>&,
                                             const Tsit5PostArgs&, int64_t, hipStream_t);

}  // namespace kan
