/*
 * kanode_ref.h — CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference KAN-ODE hot path, used ONLY by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker / CPU comparator.  It is never linked into, loaded by or called
 * from the product library (kan-odes_amd/, libkanode.so).
 *
 * What it restates (file:line relative to /root/reference):
 *   - KDense ctor constants        Lotka-Volterra/src/kdense.jl:20-68
 *   - knot grid (Julia LinRange)   Lotka-Volterra/src/kdense.jl:88-92
 *   - parameter layout             Lotka-Volterra/src/kdense.jl:70-107, LV_driver_KANODE.jl:162,173-175
 *   - KDense forward               Lotka-Volterra/src/kdense.jl:109-130 (PDE copy: PDE examples/src/kdense.jl:109-130)
 *   - rbf / rswaf / iqf + rrules   Lotka-Volterra/src/utils.jl:8-62
 *   - Fisher-KPP RHS rc_kanode     PDE examples/Fisher-KPP_Source.jl:34,55-59,95-98
 *   - per-edge activations         Lotka-Volterra/Activation_getter.jl:3-63
 *   - NNlib 0.9.24 scalar activations (tanh_fast, sigmoid, sigmoid_fast, swish,
 *     softsign) and their ChainRules rrules — third-party, pinned at
 *     Lotka-Volterra/Manifest.toml:1776; restated from the published package.
 *
 * Parity status: the reference holds NO numeric fixtures for this path
 * (SURVEY.md §4, §8c C4).  This oracle is pinned by: the exact knot constants
 * (LinRange semantics), the Activation_getter identity (Σ edges == layer output),
 * the rrule formulas checked by finite differences, and an independent numpy +
 * mpmath restatement (oracle/kanode_np.py).  See DESIGN.md §Parity.
 *
 * Layout: Julia column-major.  x is [I, K] with x[i + I*k]; C is [O, G*I] with
 * C[o + O*(g + G*i)]; W is [O, I] with W[o + O*i].  The flat parameter vector of
 * a chain is the ComponentArray order: layer_1.C, layer_1.W, layer_2.C, ...
 */
#ifndef KANODE_REF_H
#define KANODE_REF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* enums share values with include/kanode.h */
enum { KREF_NORM_TANH_FAST = 0, KREF_NORM_TANH = 1, KREF_NORM_SOFTSIGN = 2,
       KREF_NORM_SIGMOID = 3, KREF_NORM_SIGMOID_FAST = 4, KREF_NORM_IDENTITY = 5 };
enum { KREF_BASIS_RBF = 0, KREF_BASIS_RSWAF = 1, KREF_BASIS_IQF = 2 };

typedef struct {
    int32_t in_dims, out_dims, grid_len;
    int32_t normalizer;     /* KREF_NORM_* */
    int32_t basis;          /* KREF_BASIS_* */
    int32_t use_base_act;   /* base_act = swish when 1 */
    float grid_lo, grid_hi; /* grid_lims, Float32 (kdense.jl:26,38,65) */
    float denominator;      /* Float32(2/(G-1)) by default (kdense.jl:27) */
    int32_t iqf_reference_quirk; /* reproduce utils.jl:59's pullback for IQF */
} kref_layer;

/* constants */
int64_t kref_layer_param_length(const kref_layer* L);
void    kref_knots(const kref_layer* L, float* grid /*[G]*/);
float   kref_inv_h(const kref_layer* L);
float   kref_default_denominator(int32_t grid_len);

/* scalar activations (exposed for tests) */
double kref_act_f64(int32_t which, double x);   /* which: KREF_NORM_* or 100 = swish */
float  kref_act_f32(int32_t which, float x);
double kref_dact_f64(int32_t which, double x);  /* rrule derivative, NNlib form */
float  kref_dact_f32(int32_t which, float x);

/* one KDense layer: x [I,K] -> y [O,K]; p = (C, W) flat */
void kref_layer_fwd_f64(const kref_layer* L, const double* p, const double* x, int64_t K, double* y);
void kref_layer_fwd_f32(const kref_layer* L, const float*  p, const float*  x, int64_t K, float*  y);
/* pullback: xbar [I,K] overwritten; pbar [P] ACCUMULATED (+=) */
void kref_layer_vjp_f64(const kref_layer* L, const double* p, const double* x, const double* ybar,
                        int64_t K, double* xbar, double* pbar);
void kref_layer_vjp_f32(const kref_layer* L, const float* p, const float* x, const float* ybar,
                        int64_t K, float* xbar, float* pbar);

/* Lux.Chain of n layers, flat p in ComponentArray order */
void kref_chain_fwd_f64(int32_t n, const kref_layer* Ls, const double* p, const double* x, int64_t K, double* y);
void kref_chain_fwd_f32(int32_t n, const kref_layer* Ls, const float*  p, const float*  x, int64_t K, float*  y);
void kref_chain_vjp_f64(int32_t n, const kref_layer* Ls, const double* p, const double* x, const double* ybar,
                        int64_t K, double* xbar, double* pbar);
void kref_chain_vjp_f32(int32_t n, const kref_layer* Ls, const float* p, const float* x, const float* ybar,
                        int64_t K, float* xbar, float* pbar);

/* Fisher-KPP source-term RHS (Fisher-KPP_Source.jl:95-98): du = D*lap*u + kan1_.(u)
 * u, du: [Nx, B]; the KAN is a [1,1] KDense applied pointwise.  dense=1 runs the
 * reference's dense Nx x Nx matvec (timing-faithful); dense=0 the 3 nonzeros in
 * the same ascending-column order (bitwise identical results). */
void kref_fk_rhs_f64(const kref_layer* L, const double* p, double D, double dx, int64_t Nx,
                     const double* u, int64_t B, double* du, int32_t dense);
/* lamJ = (d f/d u)^T lam ; dp += sum_points lam * d f/d p */
void kref_fk_vjp_f64(const kref_layer* L, const double* p, double D, double dx, int64_t Nx,
                     const double* u, const double* lam, int64_t B, double* lamJ, double* dp);

/* One Fisher-KPP training epoch on one core (cpu_epoch.c; bench comparator): solve + loss +
 * InterpolatingAdjoint gradient + Adam, u0 [Nx, B], target [n_save][Nx, B]; p updated in place. */
int kref_fk_epoch_f64(const kref_layer* L, double* p, double D, double dx, int64_t Nx, const double* u0, int64_t B,
                      double T, const double* saveat, int32_t n_save, const double* target, double abstol,
                      double reltol, int32_t adaptive, double dt_fixed, double eta, double* loss_out, double* grad,
                      int64_t* stats, double* seconds);

/* ForwardDiffSensitivity (the reference's automatic sensealg at Fisher-KPP_Source.jl:198): the Dual solve alone
 * (usave [n_save][Nx, B], ssave [n_save][P][Nx, B], stats [2]) and one training epoch with that gradient. */
int kref_fk_fsens_solve_f64(const kref_layer* L, const double* p, double D, double dx, int64_t Nx, const double* u0,
                            int64_t B, double T, const double* saveat, int32_t n_save, double abstol, double reltol,
                            double* usave, double* ssave, int64_t* stats, double* seconds);
int kref_fk_fsens_epoch_f64(const kref_layer* L, double* p, double D, double dx, int64_t Nx, const double* u0,
                            int64_t B, double T, const double* saveat, int32_t n_save, const double* target,
                            double abstol, double reltol, double eta, double* loss_out, double* grad, int64_t* stats,
                            double* seconds);

/* The same epoch for a Lux.Chain NeuralODE RHS (LV_driver_KANODE.jl:180-219,279-287), u0 [N, B] with
 * N = Ls[0].in_dims = Ls[nl-1].out_dims; and the forward solve alone from t = 0 to T at the adaptive
 * tolerances (the driver's loss_train / loss_test solves, :290-291), pred [n_save][N, B], stats [2]. */
int kref_chain_epoch_f64(int32_t nl, const kref_layer* Ls, double* p, const double* u0, int64_t B, double T,
                         const double* saveat, int32_t n_save, const double* target, double abstol, double reltol,
                         int32_t adaptive, double dt_fixed, double eta, double* loss_out, double* grad, int64_t* stats,
                         double* seconds);
int kref_chain_solve_f64(int32_t nl, const kref_layer* Ls, const double* p, const double* u0, int64_t B, double T,
                         const double* saveat, int32_t n_save, double abstol, double reltol, double* pred,
                         int64_t* stats, double* seconds);

/* per-edge activations (Activation_getter.jl:3-63): act [O, I, K] (o fastest) */
void kref_edge_act_f64(const kref_layer* L, const double* p, const double* x, int64_t K, double* act);

#ifdef __cplusplus
}
#endif
#endif
