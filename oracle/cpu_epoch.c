/*
 * cpu_epoch.c — CPU BASELINE of one KAN-ODE training epoch (test infrastructure only; called
 * only by bench.py's epoch / lv1_train legs and tests/test_cpu_epoch.py).
 *
 * One iteration of the reference's training loop (PDE examples/Fisher-KPP_Source.jl:101-109,
 * 195-201): predict(p) = solve(ODEProblem(rc_kanode, u0, (0, T), p), Tsit5(); saveat), the MSE loss,
 * its gradient by SciMLSensitivity's InterpolatingAdjoint, and one Flux Adam update — all in C on one
 * core, so the "reference CPU path" of the epoch metric is timed without an interpreter in the loop.
 *   RHS: D*lap*u as the reference's DENSE Nx x Nx matvec (:55-59,97) + kan1_.(u) per point (:96);
 *   VJP: (D*lap)^T λ as the dense transposed matvec (what Zygote's pullback of the matvec does) +
 *        the per-point KAN pullback (kref_fk_vjp_f64 with D = 0);
 *   Tsit5 / controller / dense output / adjoint: the statements of kan-odes_amd/kanode/ode.py and
 *   kanode/adjoint.py (OrdinaryDiffEqTsit5 1.1.0 and SciMLSensitivity 7.69, restated there):
 *   Hairer-Wanner initial step, PI controller (beta1 7/50, beta2 2/25, gamma 9/10, qmin 1/5, qmax 10,
 *   qoldinit 1e-4), RMS error norm over the whole state ([λ; μ] in the adjoint), saveat from the
 *   free interpolant, λ jumps at the saveat times with FSAL re-evaluated.
 * The same epoch for a Lux.Chain NeuralODE RHS (kref_chain_epoch_f64; LV_driver_KANODE.jl:180-219,
 * 279-287: dudt = Chain(u), its pullback by kref_chain_vjp_f64), and the forward solve alone
 * (kref_chain_solve_f64: the driver's loss_train / loss_test solves, :290-291).
 * u, targets: [N, B] column-major (trajectory contiguous); targets [n_save][N*B].
 */
#include "kanode_ref.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static const double TC[6] = {0.161, 0.327, 0.9, 0.9800255409045097, 1.0, 1.0};
static const double TA[6][6] = {
    {0.161},
    {-0.008480655492356989, 0.335480655492357},
    {2.897153057105493, -6.359448489975075, 4.3622954328695815},
    {5.325864828439257, -11.748883564062828, 7.4955393428898365, -0.09249506636175525},
    {5.86145544294642, -12.92096931784711, 8.159367898576159, -0.071584973281401, -0.028269050394068383},
    {0.09646076681806523, 0.01, 0.4798896504144996, 1.379008574103742, -3.290069515436081, 2.324710524099774}};
static const double TB[7] = {-0.00178001105222577714, -0.0008164344596567469, 0.007880878010261995,
                             -0.1447110071732629,     0.5823571654525552,     -0.45808210592918697,
                             0.015151515151515152};
static const double RI[7][4] = {{1.0, -2.763706197274826, 2.9132554618219126, -1.0530884977290216},
                                {0.0, 0.13169999999999998, -0.2234, 0.1017},
                                {0.0, 3.9302962368947516, -5.941033872131505, 2.490627285651253},
                                {0.0, -12.411077166933676, 30.33818863028232, -16.548102889244902},
                                {0.0, 37.50931341651104, -88.1789048947664, 47.37952196281928},
                                {0.0, -27.896526289197286, 65.09189467479366, -34.87065786149661},
                                {0.0, 1.5, -4.0, 2.5}};

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

typedef struct epoch_ctx epoch_ctx;
struct epoch_ctx {
    void (*rhs)(epoch_ctx* c, const double* u, double* du);
    /* lamJ = (∂f/∂u)^T lam ; dp = Σ lam ∂f/∂p (overwritten) */
    void (*vjp)(epoch_ctx* c, const double* u, const double* lam, double* lamJ, double* dp);
    const double* p;
    int64_t B, n, P;
    /* Fisher-KPP */
    const kref_layer* L;
    int64_t Nx;
    double D, dx;
    double* A;      /* dense D*lap, column-major */
    double* tmp;    /* [Nx] */
    /* chain */
    int32_t nl;
    const kref_layer* Ls;
};

static void fk_rhs(epoch_ctx* c, const double* u, double* du) {
    kref_fk_rhs_f64(c->L, c->p, 0.0, c->dx, c->Nx, u, c->B, du, 0);   /* kan1_.(u) (D = 0: no stencil) */
    for (int64_t b = 0; b < c->B; ++b) {                                /* + (D*lap) u, dense gemv 'N' */
        const double* ub = u + c->Nx * b;
        double* db = c->tmp;
        memset(db, 0, sizeof(double) * (size_t)c->Nx);
        for (int64_t j = 0; j < c->Nx; ++j) {
            const double uj = ub[j];
            const double* Aj = c->A + c->Nx * j;
            for (int64_t i = 0; i < c->Nx; ++i) db[i] += Aj[i] * uj;
        }
        for (int64_t i = 0; i < c->Nx; ++i) du[c->Nx * b + i] += db[i];
    }
}

static void fk_vjp(epoch_ctx* c, const double* u, const double* lam, double* lamJ, double* dp) {
    memset(dp, 0, sizeof(double) * (size_t)c->P);
    kref_fk_vjp_f64(c->L, c->p, 0.0, c->dx, c->Nx, u, lam, c->B, lamJ, dp);
    for (int64_t b = 0; b < c->B; ++b) {                                /* + (D*lap)^T λ, dense gemv 'T' */
        const double* lb = lam + c->Nx * b;
        for (int64_t j = 0; j < c->Nx; ++j) {
            const double* Aj = c->A + c->Nx * j;
            double s = 0.0;
            for (int64_t i = 0; i < c->Nx; ++i) s += Aj[i] * lb[i];
            lamJ[c->Nx * b + j] += s;
        }
    }
}

/* NeuralODE dudt(u, p, t) = first(Chain(u, p, st)) (LV_driver_KANODE.jl:180) and its Zygote pullback */
static void chain_rhs(epoch_ctx* c, const double* u, double* du) { kref_chain_fwd_f64(c->nl, c->Ls, c->p, u, c->B, du); }

static void chain_vjp(epoch_ctx* c, const double* u, const double* lam, double* lamJ, double* dp) {
    memset(dp, 0, sizeof(double) * (size_t)c->P);
    kref_chain_vjp_f64(c->nl, c->Ls, c->p, u, lam, c->B, lamJ, dp);
}

static void interp_w(double th, double* w) {
    for (int i = 0; i < 7; ++i) {
        double s = 0.0, tp = th;
        for (int m = 0; m < 4; ++m) { s += RI[i][m] * tp; tp *= th; }
        w[i] = s;
    }
}

typedef struct {   /* the forward dense output: accepted steps */
    int64_t n, cap;
    double *t, *dt, *u, *k;    /* u: [cap][n]; k: [cap][7][n] */
} dense_rec;

static int rec_add(dense_rec* r, int64_t n, double t, double dt, const double* u, double* const* ks) {
    if (r->n == r->cap) {
        int64_t cap = r->cap ? 2 * r->cap : 256;
        double* nt = realloc(r->t, sizeof(double) * cap);
        double* nd = realloc(r->dt, sizeof(double) * cap);
        double* nu = realloc(r->u, sizeof(double) * cap * n);
        double* nk = realloc(r->k, sizeof(double) * cap * n * 7);
        if (!nt || !nd || !nu || !nk) return -1;
        r->t = nt; r->dt = nd; r->u = nu; r->k = nk; r->cap = cap;
    }
    r->t[r->n] = t;
    r->dt[r->n] = dt;
    memcpy(r->u + r->n * n, u, sizeof(double) * n);
    for (int i = 0; i < 7; ++i) memcpy(r->k + (r->n * 7 + i) * n, ks[i], sizeof(double) * n);
    r->n++;
    return 0;
}

/* u(t) from the dense record (DenseRecord.locate: the step with t_s <= t, θ clamped to [0, 1]) */
static void rec_eval(const dense_rec* r, int64_t n, double t, double* out) {
    int64_t lo = 0, hi = r->n;          /* bisect_right(t_list, t) - 1 */
    while (lo < hi) { int64_t mid = (lo + hi) / 2; if (t < r->t[mid]) hi = mid; else lo = mid + 1; }
    int64_t s = lo - 1;
    if (s < 0) s = 0;
    if (s > r->n - 1) s = r->n - 1;
    const double dt = r->dt[s];
    double th = (t - r->t[s]) / dt;
    th = th < 0.0 ? 0.0 : (th > 1.0 ? 1.0 : th);
    double w[7];
    interp_w(th, w);
    const double* u = r->u + s * n;
    for (int64_t e = 0; e < n; ++e) {
        double acc = 0.0;
        for (int i = 0; i < 7; ++i) acc += (dt * w[i]) * r->k[(s * 7 + i) * n + e];
        out[e] = u[e] + acc;
    }
}

static double sumsq_scaled(const double* x, const double* sk, int64_t n) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) { const double v = x[i] / sk[i]; s += v * v; }
    return s;
}

/* The forward solve: solve(prob, Tsit5(); saveat) from t = 0 to T, pred[n_save][n]; the dense output kept
 * in rec when rec != NULL.  Returns 0, or -1 when out of memory. */
static int forward(epoch_ctx* c, const double* u0, double T, const double* saveat, int32_t n_save, double abstol,
                   double reltol, int32_t adaptive, double dt_fixed, double* pred, dense_rec* rec, int64_t* nacc_out,
                   int64_t* nrej_out) {
    const int64_t n = c->n;
    double* buf = malloc(sizeof(double) * n * 12);
    if (!buf) return -1;
    double *u = buf, *unew = buf + n, *y = buf + 2 * n, *sk = buf + 3 * n, *e = buf + 4 * n;
    double* ks[7];
    for (int i = 0; i < 7; ++i) ks[i] = buf + (5 + i) * n;
    const double beta1 = 7.0 / 50.0, beta2 = 2.0 / 25.0, gamma = 0.9, qmin = 0.2, qmax = 10.0, qoldinit = 1e-4;
    memcpy(u, u0, sizeof(double) * n);
    int32_t si = 0;
    while (si < n_save && saveat[si] <= 1e-14) { memcpy(pred + si * n, u0, sizeof(double) * n); ++si; }
    double t = 0.0, dt;
    c->rhs(c, u, ks[0]);
    if (adaptive) {   /* _initdt */
        for (int64_t i = 0; i < n; ++i) sk[i] = abstol + fabs(u[i]) * reltol;
        const double d0 = sqrt(sumsq_scaled(u, sk, n) / n), d1 = sqrt(sumsq_scaled(ks[0], sk, n) / n);
        double dt0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        if (dt0 > T) dt0 = T;
        for (int64_t i = 0; i < n; ++i) y[i] = u[i] + dt0 * ks[0][i];
        c->rhs(c, y, ks[1]);
        for (int64_t i = 0; i < n; ++i) e[i] = ks[1][i] - ks[0][i];
        const double d2 = sqrt(sumsq_scaled(e, sk, n) / n) / dt0;
        const double mx = d1 > d2 ? d1 : d2;
        const double dt1 = mx <= 1e-15 ? fmax(1e-6, dt0 * 1e-3) : pow(0.01 / mx, 1.0 / 5.0);
        dt = fmin(fmin(100 * dt0, dt1), T);
    } else {
        dt = dt_fixed;
    }
    double qold = qoldinit;
    int64_t nacc = 0, nrej = 0;
    while (t < T - 1e-14 * fmax(1.0, T)) {
        if (dt > T - t) dt = T - t;
        for (int s = 0; s < 6; ++s) {
            for (int64_t i = 0; i < n; ++i) {
                double acc = u[i];
                for (int j = 0; j <= s; ++j) acc = acc + (dt * TA[s][j]) * ks[j][i];
                y[i] = acc;
            }
            if (s == 5) memcpy(unew, y, sizeof(double) * n);
            c->rhs(c, y, ks[s + 1]);
        }
        double dtnew = dt;
        if (adaptive) {
            for (int64_t i = 0; i < n; ++i) {
                double acc = 0.0;
                for (int j = 0; j < 7; ++j) acc += TB[j] * ks[j][i];
                e[i] = dt * acc;
                sk[i] = abstol + fmax(fabs(u[i]), fabs(unew[i])) * reltol;
            }
            const double EEst = sqrt(sumsq_scaled(e, sk, n) / n);
            const double q11 = EEst > 0 ? pow(EEst, beta1) : 0.0;
            if (EEst > 1.0) { ++nrej; dt = dt / fmin(1.0 / qmin, q11 / gamma); continue; }
            double q = q11 / pow(qold, beta2);
            q = fmax(1.0 / qmax, fmin(1.0 / qmin, q / gamma));
            dtnew = q > 0 ? dt / q : dt * qmax;
            qold = fmax(EEst, qoldinit);
        }
        const double tn = t + dt;
        while (si < n_save && saveat[si] <= tn + 1e-12 * fmax(1.0, fabs(tn))) {
            const double ts = saveat[si];
            if (fabs(ts - tn) <= 1e-12 * fmax(1.0, fabs(tn))) {
                memcpy(pred + si * n, unew, sizeof(double) * n);
            } else {
                double w[7];
                interp_w((ts - t) / dt, w);
                for (int64_t i = 0; i < n; ++i) {
                    double acc = 0.0;
                    for (int j = 0; j < 7; ++j) acc += (dt * w[j]) * ks[j][i];
                    pred[si * n + i] = u[i] + acc;
                }
            }
            ++si;
        }
        if (rec && rec_add(rec, n, t, dt, u, ks)) { free(buf); return -1; }
        t = tn;
        memcpy(u, unew, sizeof(double) * n);
        memcpy(ks[0], ks[6], sizeof(double) * n);
        ++nacc;
        dt = dtnew;
        if (nacc + nrej > 100000) { free(buf); return -3; }   /* maxiters */
    }
    *nacc_out = nacc;
    *nrej_out = nrej;
    free(buf);
    return 0;
}

/* One epoch on the context's RHS.  Returns 0 on success; loss, grad[P] (dL/dp) and the stats out. */
static int run_epoch(epoch_ctx* cp, double* p, const double* u0, double T, const double* saveat, int32_t n_save,
                     const double* target, double abstol, double reltol, int32_t adaptive, double dt_fixed, double eta,
                     double* loss_out, double* grad, int64_t* stats) {
    epoch_ctx c = *cp;
    const int64_t n = c.n, P = c.P;
    const double beta1 = 7.0 / 50.0, beta2 = 2.0 / 25.0, gamma = 0.9, qmin = 0.2, qmax = 10.0, qoldinit = 1e-4;
    if (n_save < 1) return -2;
    double* buf = malloc(sizeof(double) * n * 24);
    double* pred = malloc(sizeof(double) * n * n_save);
    dense_rec rec = {0, 0, NULL, NULL, NULL, NULL};
    int64_t nacc = 0, nrej = 0;
    int rc = forward(&c, u0, T, saveat, n_save, abstol, reltol, adaptive, dt_fixed, pred, &rec, &nacc, &nrej);
    if (rc) return rc;
    double *y = buf + 2 * n, *sk = buf + 3 * n, *e = buf + 4 * n;
    /* ---- loss = mean(abs2, target - pred); ∂L/∂u(t_j) = -2 (target - pred) / numel ---- */
    const double numel = (double)n * n_save;
    double loss = 0.0;
    double* g = malloc(sizeof(double) * n * n_save);
    for (int64_t i = 0; i < n * n_save; ++i) {
        const double r = target[i] - pred[i];
        loss += r * r;
        g[i] = -2.0 * r / numel;
    }
    loss /= numel;

    /* ---- InterpolatingAdjoint (kanode/adjoint.py, statement for statement) ---- */
    double *lam = buf + 12 * n, *ls = buf + 13 * n, *lnew = buf + 14 * n;
    double* kl[7];
    for (int i = 0; i < 7; ++i) kl[i] = buf + (15 + i) * n;
    double* km = malloc(sizeof(double) * P * 7);
    double* mu = calloc(P, sizeof(double));
    double* munew = malloc(sizeof(double) * P);
    double* emu = malloc(sizeof(double) * P);
    double* skm = malloc(sizeof(double) * P);
    memset(lam, 0, sizeof(double) * n);
    int32_t* used = calloc((size_t)n_save, sizeof(int32_t));   /* (the surrogates have 201 saveat stops) */
    double* stops = malloc(sizeof(double) * ((size_t)n_save + 1));
    const double eps = 1e-12 * fmax(1.0, fabs(T));
    for (int32_t j = 0; j < n_save; ++j)
        if (fabs(saveat[j] - T) <= 0.0 && !used[j]) {   /* the jump at tf sets the initial λ */
            for (int64_t i = 0; i < n; ++i) lam[i] += g[j * n + i];
            used[j] = 1;
        }
    int nst = 0;
    for (int32_t j = n_save - 1; j >= 0; --j)     /* interior saveat times in τ = T - t, ascending */
        if (!used[j] && saveat[j] > eps && saveat[j] < T - eps) {
            const double s = T - saveat[j];
            if (nst == 0 || s > stops[nst - 1]) stops[nst++] = s;
        }
    stops[nst++] = T;
    double tau = 0.0, h;
    rec_eval(&rec, n, T - 0.0, y);
    c.vjp(&c, y, lam, kl[0], km);
    const double ntot = (double)(n + P);
    if (adaptive) {
        for (int64_t i = 0; i < n; ++i) sk[i] = abstol + fabs(lam[i]) * reltol;
        for (int64_t q = 0; q < P; ++q) skm[q] = abstol + fabs(mu[q]) * reltol;
        const double d0 = sqrt((sumsq_scaled(lam, sk, n) + sumsq_scaled(mu, skm, P)) / ntot);
        const double d1 = sqrt((sumsq_scaled(kl[0], sk, n) + sumsq_scaled(km, skm, P)) / ntot);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        if (h0 > T) h0 = T;
        for (int64_t i = 0; i < n; ++i) ls[i] = lam[i] + h0 * kl[0][i];
        rec_eval(&rec, n, T - h0, y);
        c.vjp(&c, y, ls, kl[1], km + P);
        for (int64_t i = 0; i < n; ++i) e[i] = kl[1][i] - kl[0][i];
        for (int64_t q = 0; q < P; ++q) emu[q] = km[P + q] - km[q];
        const double d2 = sqrt((sumsq_scaled(e, sk, n) + sumsq_scaled(emu, skm, P)) / ntot) / h0;
        const double mx = d1 > d2 ? d1 : d2;
        const double h1 = mx <= 1e-15 ? fmax(1e-6, h0 * 1e-3) : pow(0.01 / mx, 1.0 / 5.0);
        h = fmin(fmin(100 * h0, h1), T);
    } else {
        h = dt_fixed;
    }
    double qold = qoldinit;
    int32_t sti = 0;
    int64_t aacc = 0, arej = 0;
    while (tau < T - 1e-14 * fmax(1.0, T)) {
        if (h > stops[sti] - tau) h = stops[sti] - tau;
        for (int s = 0; s < 6; ++s) {
            for (int64_t i = 0; i < n; ++i) {
                double acc = lam[i];
                for (int j = 0; j <= s; ++j) acc = acc + (h * TA[s][j]) * kl[j][i];
                ls[i] = acc;
            }
            if (s == 5) memcpy(lnew, ls, sizeof(double) * n);
            rec_eval(&rec, n, T - (tau + TC[s] * h), y);
            c.vjp(&c, y, ls, kl[s + 1], km + (s + 1) * P);
        }
        for (int64_t q = 0; q < P; ++q) {
            double acc = 0.0;
            for (int j = 0; j < 6; ++j) acc += (h * TA[5][j]) * km[j * P + q];
            munew[q] = mu[q] + acc;
        }
        double hnew = h;
        if (adaptive) {
            for (int64_t i = 0; i < n; ++i) {
                double acc = 0.0;
                for (int j = 0; j < 7; ++j) acc += (h * TB[j]) * kl[j][i];
                e[i] = acc;
                sk[i] = abstol + reltol * fmax(fabs(lam[i]), fabs(lnew[i]));
            }
            for (int64_t q = 0; q < P; ++q) {
                double acc = 0.0;
                for (int j = 0; j < 7; ++j) acc += (h * TB[j]) * km[j * P + q];
                emu[q] = acc;
                skm[q] = abstol + fmax(fabs(mu[q]), fabs(munew[q])) * reltol;
            }
            const double EEst = sqrt((sumsq_scaled(e, sk, n) + sumsq_scaled(emu, skm, P)) / ntot);
            const double q11 = EEst > 0 ? pow(EEst, beta1) : 0.0;
            if (EEst > 1.0) { ++arej; h = h / fmin(1.0 / qmin, q11 / gamma); continue; }
            double q = q11 / pow(qold, beta2);
            q = fmax(1.0 / qmax, fmin(1.0 / qmin, q / gamma));
            hnew = q > 0 ? h / q : h * qmax;
            qold = fmax(EEst, qoldinit);
        }
        tau = tau + h;
        memcpy(lam, lnew, sizeof(double) * n);
        memcpy(mu, munew, sizeof(double) * P);
        memcpy(kl[0], kl[6], sizeof(double) * n);
        memcpy(km, km + 6 * P, sizeof(double) * P);
        ++aacc;
        if (fabs(tau - stops[sti]) <= 1e-12 * fmax(1.0, T)) {
            tau = stops[sti];
            const double ts = T - tau;
            if (sti < nst - 1) {
                for (int32_t j = 0; j < n_save; ++j)   /* λ += ∂L/∂u(t_j) at every saveat equal to ts */
                    if (!used[j] && fabs(saveat[j] - ts) <= eps) {
                        for (int64_t i = 0; i < n; ++i) lam[i] += g[j * n + i];
                        used[j] = 1;
                    }
                rec_eval(&rec, n, T - tau, y);           /* u_modified!: FSAL re-evaluated */
                c.vjp(&c, y, lam, kl[0], km);
            }
            sti = sti + 1 < nst ? sti + 1 : nst - 1;
        }
        h = hnew;
    }
    /* dL/dp = μ(t0); a saveat at t0 adds to dL/du0 only */
    memcpy(grad, mu, sizeof(double) * P);
    /* ---- Flux Adam step (first step of a fresh optimiser: βp = β) ---- */
    for (int64_t q = 0; q < P; ++q) {
        const double m = 0.1 * grad[q], v = 0.001 * grad[q] * grad[q];
        p[q] -= m / (1 - 0.9) / (sqrt(v / (1 - 0.999)) + 1e-8) * eta;
    }
    *loss_out = loss;
    stats[0] = nacc; stats[1] = nrej; stats[2] = aacc; stats[3] = arej;
    free(buf); free(pred); free(g); free(km); free(mu); free(munew); free(emu); free(skm);
    free(used); free(stops);
    free(rec.t); free(rec.dt); free(rec.u); free(rec.k);
    return 0;
}

int kref_fk_epoch_f64(const kref_layer* L, double* p, double D, double dx, int64_t Nx, const double* u0, int64_t B,
                      double T, const double* saveat, int32_t n_save, const double* target, double abstol,
                      double reltol, int32_t adaptive, double dt_fixed, double eta, double* loss_out, double* grad,
                      int64_t* stats /* [4]: fwd accept, fwd reject, adj accept, adj reject */, double* seconds) {
    const double t_start = now_s();
    epoch_ctx c = {0};
    c.rhs = fk_rhs;
    c.vjp = fk_vjp;
    c.p = p;
    c.B = B;
    c.n = Nx * B;
    c.P = kref_layer_param_length(L);
    c.L = L;
    c.Nx = Nx;
    c.D = D;
    c.dx = dx;
    c.A = calloc((size_t)(Nx * Nx), sizeof(double));
    c.tmp = malloc(sizeof(double) * Nx);
    const double dx2 = dx * dx, cd = D * (-2.0 / dx2), co = D * (1.0 / dx2);
    for (int64_t i = 0; i < Nx; ++i) {
        c.A[i + Nx * i] = cd;
        if (i + 1 < Nx) { c.A[i + Nx * (i + 1)] = co; c.A[(i + 1) + Nx * i] = co; }
    }
    c.A[0 + Nx * (Nx - 1)] = co;
    c.A[(Nx - 1) + Nx * 0] = co;
    const int rc = run_epoch(&c, p, u0, T, saveat, n_save, target, abstol, reltol, adaptive, dt_fixed, eta, loss_out,
                             grad, stats);
    free(c.A);
    free(c.tmp);
    *seconds = now_s() - t_start;
    return rc;
}

static epoch_ctx chain_ctx(int32_t nl, const kref_layer* Ls, const double* p, int64_t B) {
    epoch_ctx c = {0};
    c.rhs = chain_rhs;
    c.vjp = chain_vjp;
    c.p = p;
    c.B = B;
    c.n = (int64_t)Ls[0].in_dims * B;
    c.P = 0;
    for (int32_t l = 0; l < nl; ++l) c.P += kref_layer_param_length(&Ls[l]);
    c.nl = nl;
    c.Ls = Ls;
    return c;
}

int kref_chain_epoch_f64(int32_t nl, const kref_layer* Ls, double* p, const double* u0, int64_t B, double T,
                         const double* saveat, int32_t n_save, const double* target, double abstol, double reltol,
                         int32_t adaptive, double dt_fixed, double eta, double* loss_out, double* grad, int64_t* stats,
                         double* seconds) {
    const double t_start = now_s();
    if (nl < 1 || Ls[nl - 1].out_dims != Ls[0].in_dims) return -4;
    epoch_ctx c = chain_ctx(nl, Ls, p, B);
    const int rc = run_epoch(&c, p, u0, T, saveat, n_save, target, abstol, reltol, adaptive, dt_fixed, eta, loss_out,
                             grad, stats);
    *seconds = now_s() - t_start;
    return rc;
}

int kref_chain_solve_f64(int32_t nl, const kref_layer* Ls, const double* p, const double* u0, int64_t B, double T,
                         const double* saveat, int32_t n_save, double abstol, double reltol, double* pred,
                         int64_t* stats /* [2] */, double* seconds) {
    const double t_start = now_s();
    if (nl < 1 || Ls[nl - 1].out_dims != Ls[0].in_dims) return -4;
    epoch_ctx c = chain_ctx(nl, Ls, p, B);
    const int rc = forward(&c, u0, T, saveat, n_save, abstol, reltol, 1, 0.0, pred, NULL, &stats[0], &stats[1]);
    *seconds = now_s() - t_start;
    return rc;
}

/* ---- ForwardDiffSensitivity (SciMLSensitivity 7.69's automatic sensealg for the small source-term drivers:
 * Fisher-KPP_Source.jl:198 Zygote.gradient(loss, p), length(u0) + length(p) <= 100; third-party semantics
 * restated, the same statement as kan-odes_amd/csrc/kan_small.hip fk_small_fsens_kernel and
 * tests/test_gpu_fsens.py dual_tsit5).  The Dual-number solve over z = [u; S_1; ...; S_P] (rows of n entries),
 * S_k = ∂u/∂p_k:  S_k' = (D lap) S_k + φ'(u) S_k + ∂φ/∂p_k(u), φ' and ∂φ/∂p from the oracle's pullback of
 * one KDense(1,1,G) point with ȳ = 1.  DiffEqBase's Dual norm: entry i's residual scale is
 * abstol + reltol·max(‖z_i‖, ‖znew_i‖), ‖z_i‖² = Σ_r z[r][i]², and the RMS runs over all (1 + P)·n values. */
static void fk_fsens_rhs(epoch_ctx* c, const double* z, double* dz, double* g /* [P] scratch */) {
    const int64_t n = c->n, P = c->P, Nx = c->Nx;
    c->rhs(c, z, dz);                                    /* the values */
    for (int64_t k = 0; k < P; ++k) {                    /* (D*lap) S_k, dense gemv 'N' */
        for (int64_t b = 0; b < c->B; ++b) {
            const double* sb = z + (1 + k) * n + Nx * b;
            double* db = dz + (1 + k) * n + Nx * b;
            memset(db, 0, sizeof(double) * (size_t)Nx);
            for (int64_t j = 0; j < Nx; ++j) {
                const double sj = sb[j];
                const double* Aj = c->A + Nx * j;
                for (int64_t i = 0; i < Nx; ++i) db[i] += Aj[i] * sj;
            }
        }
    }
    for (int64_t i = 0; i < n; ++i) {                    /* + φ'(u_i) S_k,i + ∂φ/∂p_k(u_i) */
        const double one = 1.0;
        double dphi = 0.0;
        memset(g, 0, sizeof(double) * (size_t)P);
        kref_layer_vjp_f64(c->L, c->p, z + i, &one, 1, &dphi, g);
        for (int64_t k = 0; k < P; ++k) {
            double* d = dz + (1 + k) * n + i;
            *d = (*d + z[(1 + k) * n + i] * dphi) + g[k];
        }
    }
}

/* Σ over all (1 + P)·n values of (x / sk_entry)² with the per-entry scales sk[n] */
static double dual_sumsq(const double* x, const double* sk, int64_t n, int64_t rows) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i)
        for (int64_t r = 0; r < rows; ++r) { const double v = x[r * n + i] / sk[i]; s += v * v; }
    return s;
}
static double dual_nrm(const double* z, int64_t i, int64_t n, int64_t rows) {
    double s = 0.0;
    for (int64_t r = 0; r < rows; ++r) s += z[r * n + i] * z[r * n + i];
    return sqrt(s);
}

/* The Dual solve from t = 0 to T: zsave [n_save][(1 + P)·n] (values then the P sensitivities), stats[2]. */
static int fsens_forward(epoch_ctx* c, const double* u0, double T, const double* saveat, int32_t n_save, double abstol,
                         double reltol, double* zsave, int64_t* stats) {
    const int64_t n = c->n, P = c->P, rows = 1 + P, m = rows * n;
    double* buf = malloc(sizeof(double) * (m * 12 + n + P));
    if (!buf) return -1;
    double *z = buf, *znew = buf + m, *y = buf + 2 * m, *e = buf + 3 * m;
    double* ks[7];
    for (int i = 0; i < 7; ++i) ks[i] = buf + (4 + i) * m;
    double* sk = buf + 11 * m;
    double* g = sk + n;
    const double beta1 = 7.0 / 50.0, beta2 = 2.0 / 25.0, gamma = 0.9, qmin = 0.2, qmax = 10.0, qoldinit = 1e-4;
    memset(z, 0, sizeof(double) * m);
    memcpy(z, u0, sizeof(double) * n);
    int32_t si = 0;
    while (si < n_save && saveat[si] <= 1e-14) { memcpy(zsave + si * m, z, sizeof(double) * m); ++si; }
    double t = 0.0;
    fk_fsens_rhs(c, z, ks[0], g);
    for (int64_t i = 0; i < n; ++i) sk[i] = abstol + dual_nrm(z, i, n, rows) * reltol;   /* _initdt */
    const double d0 = sqrt(dual_sumsq(z, sk, n, rows) / m), d1 = sqrt(dual_sumsq(ks[0], sk, n, rows) / m);
    double dt0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
    if (dt0 > T) dt0 = T;
    for (int64_t q = 0; q < m; ++q) y[q] = z[q] + dt0 * ks[0][q];
    fk_fsens_rhs(c, y, ks[1], g);
    for (int64_t q = 0; q < m; ++q) e[q] = ks[1][q] - ks[0][q];
    const double d2 = sqrt(dual_sumsq(e, sk, n, rows) / m) / dt0;
    const double mx = d1 > d2 ? d1 : d2;
    const double dt1 = mx <= 1e-15 ? fmax(1e-6, dt0 * 1e-3) : pow(0.01 / mx, 1.0 / 5.0);
    double dt = fmin(fmin(100 * dt0, dt1), T);
    double qold = qoldinit;
    int64_t nacc = 0, nrej = 0;
    while (t < T - 1e-14 * fmax(1.0, T)) {
        if (dt > T - t) dt = T - t;
        for (int s = 0; s < 6; ++s) {
            for (int64_t q = 0; q < m; ++q) {
                double acc = z[q];
                for (int j = 0; j <= s; ++j) acc = acc + (dt * TA[s][j]) * ks[j][q];
                y[q] = acc;
            }
            if (s == 5) memcpy(znew, y, sizeof(double) * m);
            fk_fsens_rhs(c, y, ks[s + 1], g);
        }
        for (int64_t q = 0; q < m; ++q) {
            double acc = 0.0;
            for (int j = 0; j < 7; ++j) acc += TB[j] * ks[j][q];
            e[q] = dt * acc;
        }
        for (int64_t i = 0; i < n; ++i) sk[i] = abstol + fmax(dual_nrm(z, i, n, rows), dual_nrm(znew, i, n, rows)) * reltol;
        const double EEst = sqrt(dual_sumsq(e, sk, n, rows) / m);
        const double q11 = EEst > 0 ? pow(EEst, beta1) : 0.0;
        if (EEst > 1.0) { ++nrej; dt = dt / fmin(1.0 / qmin, q11 / gamma); continue; }
        double q = q11 / pow(qold, beta2);
        q = fmax(1.0 / qmax, fmin(1.0 / qmin, q / gamma));
        const double dtnew = q > 0 ? dt / q : dt * qmax;
        qold = fmax(EEst, qoldinit);
        const double tn = t + dt;
        while (si < n_save && saveat[si] <= tn + 1e-12 * fmax(1.0, fabs(tn))) {
            const double ts = saveat[si];
            if (fabs(ts - tn) <= 1e-12 * fmax(1.0, fabs(tn))) {
                memcpy(zsave + si * m, znew, sizeof(double) * m);
            } else {
                double w[7];
                interp_w((ts - t) / dt, w);
                for (int64_t q = 0; q < m; ++q) {
                    double acc = 0.0;
                    for (int j = 0; j < 7; ++j) acc += (dt * w[j]) * ks[j][q];
                    zsave[si * m + q] = z[q] + acc;
                }
            }
            ++si;
        }
        t = tn;
        memcpy(z, znew, sizeof(double) * m);
        memcpy(ks[0], ks[6], sizeof(double) * m);
        ++nacc;
        dt = dtnew;
        if (nacc + nrej > 100000) { free(buf); return -3; }   /* maxiters */
    }
    stats[0] = nacc;
    stats[1] = nrej;
    free(buf);
    return 0;
}

static epoch_ctx fk_ctx(const kref_layer* L, const double* p, double D, double dx, int64_t Nx, int64_t B) {
    epoch_ctx c = {0};
    c.rhs = fk_rhs;
    c.vjp = fk_vjp;
    c.p = p;
    c.B = B;
    c.n = Nx * B;
    c.P = kref_layer_param_length(L);
    c.L = L;
    c.Nx = Nx;
    c.D = D;
    c.dx = dx;
    c.A = calloc((size_t)(Nx * Nx), sizeof(double));
    c.tmp = malloc(sizeof(double) * Nx);
    const double dx2 = dx * dx, cd = D * (-2.0 / dx2), co = D * (1.0 / dx2);
    for (int64_t i = 0; i < Nx; ++i) {
        c.A[i + Nx * i] = cd;
        if (i + 1 < Nx) { c.A[i + Nx * (i + 1)] = co; c.A[(i + 1) + Nx * i] = co; }
    }
    c.A[0 + Nx * (Nx - 1)] = co;
    c.A[(Nx - 1) + Nx * 0] = co;
    return c;
}

/* The Dual solve alone: usave [n_save][n], ssave [n_save][P][n], stats [2] (accepted, rejected). */
int kref_fk_fsens_solve_f64(const kref_layer* L, const double* p, double D, double dx, int64_t Nx, const double* u0,
                            int64_t B, double T, const double* saveat, int32_t n_save, double abstol, double reltol,
                            double* usave, double* ssave, int64_t* stats, double* seconds) {
    const double t_start = now_s();
    epoch_ctx c = fk_ctx(L, p, D, dx, Nx, B);
    const int64_t n = c.n, m = (1 + c.P) * n;
    double* zs = malloc(sizeof(double) * (size_t)(m * (n_save > 0 ? n_save : 1)));
    int rc = zs ? fsens_forward(&c, u0, T, saveat, n_save, abstol, reltol, zs, stats) : -1;
    if (rc == 0)
        for (int32_t j = 0; j < n_save; ++j) {
            memcpy(usave + j * n, zs + j * m, sizeof(double) * n);
            memcpy(ssave + j * c.P * n, zs + j * m + n, sizeof(double) * c.P * n);
        }
    free(zs);
    free(c.A);
    free(c.tmp);
    *seconds = now_s() - t_start;
    return rc;
}

/* One Fisher-KPP training epoch with the reference's ForwardDiffSensitivity gradient: the Dual solve, the MSE loss,
 * dL/dp_k = Σ_j Σ_i 2 (pred - X)/numel · S_k, one Adam step (first step of a fresh optimiser); stats [2]. */
int kref_fk_fsens_epoch_f64(const kref_layer* L, double* p, double D, double dx, int64_t Nx, const double* u0,
                            int64_t B, double T, const double* saveat, int32_t n_save, const double* target,
                            double abstol, double reltol, double eta, double* loss_out, double* grad, int64_t* stats,
                            double* seconds) {
    const double t_start = now_s();
    if (n_save < 1) return -2;
    epoch_ctx c = fk_ctx(L, p, D, dx, Nx, B);
    const int64_t n = c.n, P = c.P, m = (1 + P) * n;
    double* zs = malloc(sizeof(double) * (size_t)(m * n_save));
    int rc = zs ? fsens_forward(&c, u0, T, saveat, n_save, abstol, reltol, zs, stats) : -1;
    if (rc == 0) {
        const double numel = (double)n * n_save;
        double loss = 0.0;
        memset(grad, 0, sizeof(double) * (size_t)P);
        for (int32_t j = 0; j < n_save; ++j)
            for (int64_t i = 0; i < n; ++i) {
                const double r = zs[j * m + i] - target[j * n + i];
                loss += r * r;
                const double dl = 2.0 * r / numel;
                for (int64_t k = 0; k < P; ++k) grad[k] += dl * zs[j * m + (1 + k) * n + i];
            }
        *loss_out = loss / numel;
        for (int64_t q = 0; q < P; ++q) {   /* Flux Adam, first step */
            const double mm = 0.1 * grad[q], v = 0.001 * grad[q] * grad[q];
            p[q] -= mm / (1 - 0.9) / (sqrt(v / (1 - 0.999)) + 1e-8) * eta;
        }
    }
    free(zs);
    free(c.A);
    free(c.tmp);
    *seconds = now_s() - t_start;
    return rc;
}
