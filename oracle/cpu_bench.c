/*
 * cpu_bench.c — CPU BASELINE timing harness (test infrastructure only; called
 * only by bench.py's cpu_baseline leg).  Times the faithful CPU restatement of
 * the reference Fisher-KPP RHS (PDE examples/Fisher-KPP_Source.jl:95-98):
 *   du = (D*lap) * u  — the reference's DENSE Nx x Nx matvec (lap :55-59), written
 *                        in column-axpy form (gemv 'N'), ascending column order;
 *      + kan1_.(u)   — one scalar KDense(1,1,G) evaluation per grid point (:96).
 * Threads: OpenMP over trajectories (threads=1 is the single-threaded reference
 * shape; the Julia driver is single-threaded apart from BLAS).
 */
#include "kanode_ref.h"
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* Returns wall seconds for `reps` full RHS evaluations over B trajectories. */
double kref_bench_fk_rhs_f64(const kref_layer* L, const double* p, double D, double dx, int64_t Nx,
                             const double* u, int64_t B, double* du, int32_t reps, int32_t threads) {
    const double dx2 = dx * dx;
    const double cd = D * (-2.0 / dx2), co = D * (1.0 / dx2);
    double* A = (double*)calloc((size_t)(Nx * Nx), sizeof(double));
    for (int64_t i = 0; i < Nx; ++i) {
        A[i + Nx * i] = cd;
        if (i + 1 < Nx) { A[i + Nx * (i + 1)] = co; A[(i + 1) + Nx * i] = co; }
    }
    A[0 + Nx * (Nx - 1)] = co; A[(Nx - 1) + Nx * 0] = co;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
    double t0 = now_s();
    for (int32_t r = 0; r < reps; ++r) {
#pragma omp parallel for schedule(static)
        for (int64_t b = 0; b < B; ++b) {
            const double* ub = u + Nx * b;
            double* db = du + Nx * b;
            memset(db, 0, sizeof(double) * (size_t)Nx);
            for (int64_t j = 0; j < Nx; ++j) {          /* gemv 'N': y += A[:,j] * u[j] */
                const double uj = ub[j];
                const double* Aj = A + Nx * j;
                for (int64_t i = 0; i < Nx; ++i) db[i] += Aj[i] * uj;
            }
            for (int64_t i = 0; i < Nx; ++i) {           /* kan1_.(u) */
                double kan;
                kref_layer_fwd_f64(L, p, &ub[i], 1, &kan);
                db[i] = db[i] + kan;
            }
        }
    }
    double t1 = now_s();
    free(A);
    return t1 - t0;
}

/* Chain RHS (NeuralODE dudt = Chain(u)) timing: `reps` evaluations of a [I0,K] batch. */
double kref_bench_chain_f64(int32_t n, const kref_layer* Ls, const double* p, const double* x,
                            int64_t K, double* y, int32_t reps, int32_t threads) {
    const int64_t I0 = Ls[0].in_dims, IL = Ls[n - 1].out_dims;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
    double t0 = now_s();
    for (int32_t r = 0; r < reps; ++r) {
#pragma omp parallel for schedule(static)
        for (int64_t k = 0; k < K; ++k) kref_chain_fwd_f64(n, Ls, p, x + I0 * k, 1, y + IL * k);
    }
    return now_s() - t0;
}

int32_t kref_omp_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
