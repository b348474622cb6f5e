/*
 * kanode.h — C-ABI of the MI355X-native KAN-ODE right-hand side and its VJP.
 *
 * This is the drop-in boundary for the reference's hot path.  A
 * host (the Julia `ccall` shim in INTEGRATION.md, or the Python harness in
 * kan-odes_amd/kanode) binds exactly these entry points.  Plain C: integer status
 * codes, plain pointers and sizes, no exceptions across the ABI.
 *
 * Reference interfaces replaced (file:line relative to /root/reference):
 *   kanode_create / kanode_param_length / kanode_knots
 *       KDense ctor + LuxCore.initialparameters/initialstates/parameterlength/statelength
 *       Lotka-Volterra/src/kdense.jl:20-107 (PDE copy: PDE examples/src/kdense.jl:20-107)
 *   kanode_layer_forward
 *       (l::KDense)(x, p, st) -> (y, st)                     Lotka-Volterra/src/kdense.jl:109-130
 *   kanode_layer_forward_stage
 *       the same call at a Runge-Kutta stage input (grid-sharded surrogate, PDE examples/Burgers_Surrogate.jl:85-97)
 *   kanode_layer_vjp
 *       Zygote pullback of the above incl. rrule(_rbf)        Lotka-Volterra/src/utils.jl:15-21
 *   kanode_rhs  (rhs_kind = CHAIN)
 *       NeuralODE dudt(u,p,t) = first(Chain(u, p, st))      Lotka-Volterra/LV_driver_KANODE.jl:139-143,180
 *                                                           PDE examples/Burgers_Surrogate.jl:85-97,
 *                                                           PDE examples/Schrodinger_Surrogate.jl:93-104
 *   kanode_rhs  (rhs_kind = POINTWISE_PERIODIC_LAPLACIAN)
 *       rc_kanode(u,p,t) = D*lap*u + kan1_.(u)              PDE examples/Fisher-KPP_Source.jl:55-59,95-98
 *   kanode_vjp
 *       the RHS pullback SciMLSensitivity requests per adjoint stage (λᵀ∂f/∂u, λᵀ∂f/∂p)
 *   kanode_edge_activations
 *       per-edge activations                                 Lotka-Volterra/Activation_getter.jl:3-63
 *
 * Layout: the reference's Julia column-major arrays.  A state / layer input is
 * [N, B] with element (n, b) at n + N*b (one trajectory contiguous).  The flat
 * parameter vector p is the ComponentArray order of the Lux chain:
 * layer_1.C [O,G*I] col-major, layer_1.W [O,I], layer_2.C, ... (kdense.jl:70-86,
 * LV_driver_KANODE.jl:173-175) — the same vector the reference stores in `.mat`
 * p_list rows.
 *
 * Ownership / threading: the caller owns every buffer passed in.  Device
 * variants take DEVICE pointers and are asynchronous on `stream` (a hipStream_t,
 * NULL = default stream); they never allocate once kanode_reserve() covered the
 * batch, so they can be captured into a hipGraph.  *_host variants take host
 * pointers, stage through handle-owned device buffers and return after the
 * stream synchronises.  A handle is bound to one device, is NOT thread-safe,
 * and separate handles are independent.  A handle's device calls must be stream-ordered: issue
 * them on one stream at a time (the Fisher-KPP table kernels keep per-handle build state in device
 * memory; kanode_reserve resets it).  `dp`/`pbar` ACCUMULATE (+=): the adjoint
 * integrates μ across stages, so zeroing is the caller's job.
 */
#ifndef KANODE_H
#define KANODE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KANODE_ABI_VERSION 1
#define KANODE_MAX_LAYERS 8
#define KANODE_MAX_GRID 32

typedef enum {
    KANODE_OK = 0,
    KANODE_ERR_INVALID_ARG = 1,
    KANODE_ERR_UNSUPPORTED = 2,
    KANODE_ERR_HIP = 3,
    KANODE_ERR_ALLOC = 4,
    KANODE_ERR_CAPTURE = 5 /* would need to allocate during stream capture: call kanode_reserve first */
} kanode_status;

typedef enum { KANODE_F32 = 0, KANODE_F64 = 1 } kanode_dtype;

/* normalizer (kdense.jl:25,57-61; NNlib.fast_act maps tanh -> tanh_fast when
 * allow_fast_activation, the reference default) */
typedef enum {
    KANODE_NORM_TANH_FAST = 0,
    KANODE_NORM_TANH = 1,
    KANODE_NORM_SOFTSIGN = 2,
    KANODE_NORM_SIGMOID = 3,
    KANODE_NORM_SIGMOID_FAST = 4,
    KANODE_NORM_IDENTITY = 5
} kanode_normalizer;

/* basis_func (utils.jl:8-62) */
typedef enum { KANODE_BASIS_RBF = 0, KANODE_BASIS_RSWAF = 1, KANODE_BASIS_IQF = 2 } kanode_basis;

typedef enum {
    KANODE_RHS_CHAIN = 0,                        /* du = Chain(u)                           */
    KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN = 1  /* du = D*lap*u + KDense(1,1,G).(u)        */
} kanode_rhs_kind;

/* One KDense layer (kdense.jl:20-37). */
typedef struct {
    int32_t in_dims;
    int32_t out_dims;
    int32_t grid_len;               /* G, 2 <= G <= KANODE_MAX_GRID */
    int32_t normalizer;             /* kanode_normalizer */
    int32_t basis;                  /* kanode_basis */
    int32_t use_base_act;           /* 1: y += W * swish.(x) */
    float grid_lo, grid_hi;         /* grid_lims, Float32 (default -1f0, 1f0) */
    float denominator;              /* <= 0: Float32(2/(G-1)) (kdense.jl:27) */
    int32_t iqf_reference_quirk;    /* 1: IQF pullback exactly as utils.jl:59 */
} kanode_layer_spec;

typedef struct {
    int32_t n_layers;
    kanode_layer_spec layers[KANODE_MAX_LAYERS];
    int32_t dtype;                  /* kanode_dtype of u, p and every output */
    int32_t rhs_kind;               /* kanode_rhs_kind */
    /* POINTWISE_PERIODIC_LAPLACIAN only: state [nx, B], one [1,1] layer */
    int64_t nx;
    double diffusion;               /* D (Fisher-KPP_Source.jl:34) */
    double dx;                      /* grid spacing (lap = tridiag(1,-2,1)/dx^2 + periodic corners) */
    int32_t device;                 /* HIP device ordinal */
} kanode_spec;

typedef struct kanode_handle kanode_handle;

/* --- lifecycle ------------------------------------------------------------- */
kanode_status kanode_create(const kanode_spec* spec, kanode_handle** out);
void kanode_destroy(kanode_handle* h);
const char* kanode_last_error(const kanode_handle* h);   /* message of the last failure on h */
const char* kanode_status_string(kanode_status s);
int32_t kanode_abi_version(void);

/* --- introspection (LuxCore.parameterlength / statelength / initialstates) -- */
int64_t kanode_param_length(const kanode_handle* h);     /* whole chain */
int64_t kanode_layer_param_length(const kanode_handle* h, int32_t layer);
int64_t kanode_state_length(const kanode_handle* h);     /* N of the [N, B] state */
kanode_status kanode_knots(const kanode_handle* h, int32_t layer, float* grid_out /* [G] host */);

/* Pre-size handle workspaces for batches up to max_batch (no allocation in later
 * device calls with batch <= max_batch; required before hipGraph capture).  A device
 * call that would still need to allocate while its stream is capturing returns
 * KANODE_ERR_CAPTURE instead.  It takes no stream, so it SYNCHRONISES THE WHOLE DEVICE
 * (hipDeviceSynchronize, then a synchronous reset of the table stamps): call it outside the
 * timed / overlapped region, and never while any stream of the process is being captured (a
 * device-wide synchronisation invalidates a global-mode capture on another thread). */
kanode_status kanode_reserve(kanode_handle* h, int64_t max_batch);

/* Evaluation-strategy switches (no reference counterpart: they select between
 * HIP kernels computing the same function).
 *   KANODE_OPT_POINTWISE_TABLE (POINTWISE rhs, f64): 1 = evaluate kan1_.(u)
 *     through the per-launch piecewise-polynomial table (default where admissible:
 *     rbf/rswaf basis, even nx), 0 = the per-point basis recurrence.  Setting 1
 *     where inadmissible returns KANODE_ERR_UNSUPPORTED.
 *   KANODE_OPT_FUSED_STEP (default 1): the integrator issues one launch per Tsit5 /
 *     adjoint step where a fused step kernel covers the RHS (Fisher-KPP table path,
 *     small chains); 0 = one kanode_rhs_stage / kanode_vjp_stage launch per stage with
 *     the K-form dense output.
 *   KANODE_OPT_FUSED_SOLVE (default 1): control = auto may run a small-chain solve as
 *     one workgroup; 0 = always the host loop.
 *   KANODE_OPT_FUSED_SOLVE_CAP (default 0): dense-output slots of that one-workgroup
 *     solve (0 = its own block; small values exercise the host-loop fallback).
 *   KANODE_OPT_GRID_RHS / _GRID_VJP / _GRID_ADJ_STEP (default 0): persistent grid of
 *     the Fisher-KPP table kernels: RHS, RK stage and one-launch Tsit5 step / VJP and
 *     adjoint stage / one-launch adjoint step (0 = occupancy-derived).
 *     Tuning only: the grid fixes the order of the dp reduction, so gradients are
 *     bitwise reproducible for a given grid, not across grids.
 *   KANODE_OPT_ADJ_STEP_ROWS (default 1): the one-launch Fisher-KPP adjoint step keeps each
 *     trajectory row's stage values in the registers of one wave (batches up to 8192 rows
 *     of <= 256 points, GRID_ADJ_STEP unset); 0 = the persistent-grid step kernel, whose
 *     stages pass kλ through memory.  Same λᵀJ and λ bitwise; dp to the reduction order.
 *   KANODE_OPT_PAIR_VJP (default 1): the VJP / adjoint stage of a surrogate chain KAN [N, H, N]
 *     (wide-in then wide-out layer) runs as two launches (batches up to 64); 0 = the four-launch
 *     path.  Equal to the summation order of the wide-out dot products (both fixed-order).
 *   KANODE_OPT_PAIR_FUSE (default 1): the integrator's adjoint stages of such a chain hold each
 *     stage's second launch until the next stage is issued and run the two in one launch (the
 *     x̄ block of stage s forms stage s+1's input λs over its own chunk); 0 = two launches per
 *     stage.  Bitwise equal.
 *   KANODE_OPT_PAIR_PERSIST (default 1): kanode_adjoint_tsit5 of such a chain (fp64, after a
 *     host-loop forward solve) runs the whole InterpolatingAdjoint as ONE launch where its LDS
 *     carve fits (e.g. Burgers [512, 10, 512] with up to 8 trajectories): the grid split over
 *     workgroups of KANODE_OPT_PAIR_PERSIST_S points (4, 8 or 16; 0 = 8), one exchange of the
 *     hidden pre-activations per step and one of the hidden cotangents per adjoint stage between
 *     workgroups, μ and its stage vectors resident in LDS, the step control on the device; other
 *     shapes take the launch-per-stage path.  Same algorithm; sums in another fixed order.
 *   KANODE_OPT_ADJ_FUSED_FINISH (default 0): 1 = an adaptive Fisher-KPP adjoint step on the rows
 *     kernel (ADJ_STEP_ROWS, >= 1 + P workgroups) finishes inside that launch: the last 1 + P
 *     workgroups to arrive each sum one parameter's stage rows (or the λ error partials) and write
 *     μ_new, kμ_7 and the error terms in the finish kernel's order (bitwise equal); 0 = the separate
 *     finish launch per step.  Measured equal on the adaptive epoch (the finish's cost is its memory
 *     round trips, not its launch), so the simpler path is the default.
 *   KANODE_OPT_PAIR_PERSIST_MAX_WG (default 0): the persistent pair adjoint's workgroups spin on each
 *     other, so it is launched only when all of them can be resident at once: 0 = the capacity the
 *     device reports (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs); n > 0 = at most n (a
 *     partitioned or shared device).  A grid above the capacity takes the launch-per-stage path.
 *   KANODE_OPT_PAIR_PERSIST_ABORT (default 0, tests only): 1 raises the kernel's abort word at
 *     launch, which is what an exchange time-out does (e.g. workgroups kept off the device by other
 *     work): the adjoint then re-runs on the launch-per-stage path.
 *   KANODE_OPT_LAST_ADJOINT (read-only): the path the handle's last kanode_adjoint_tsit5 took,
 *     a kanode_adjoint_path value.
 *   KANODE_OPT_CHAIN_WIDE (default 1): the one-workgroup adjoint of ONE trajectory of a two-layer chain
 *     with base activations (the Lotka-Volterra driver's shape) spreads the pullback over the whole
 *     workgroup, one basis function per lane (kd_chain_adjoint_wide_kernel); 0 = the 16-lane group of
 *     the batched kernel.  Same formulas; sums in another order.
 *   KANODE_OPT_RECORD_ADJOINT_STEPS (default 0): 1 = kanode_adjoint_tsit5 keeps the accepted step
 *     sizes of its backward integration on the handle (kanode_adjoint_step_sizes), on every path
 *     (the one-launch adjoints write them from the device, up to 4 x the forward steps + 1024).
 *     Diagnostics: two solvers' step sequences show whether their controllers took the same path.
 *   KANODE_OPT_FK_DEVICE_LOOP (default 1): the adaptive Fisher-KPP table path (control = auto, dense
 *     output kept) runs its step control on the device.  Forward: launch q of the step kernel decides
 *     attempt q - 1 at its head (every workgroup sums the same error partials and applies the PI
 *     controller) and takes the next step; the saveat values are formed from the dense output afterwards.
 *     Adjoint (the combined rows step, Nx = 128 / 256): the finish launch's last workgroup decides the
 *     attempt and plans the next one; a step landing on a saveat stop pauses the loop for the host's jump.
 *     The host queues launches ahead and never waits on a step.  0 = the host loops (one norm read per
 *     step).  Same controller arithmetic; the device sums the terms in another order and its pow may round
 *     differently, so step sizes agree to rounding, not bitwise.
 * Options are read when a call is issued (never from the environment).  kanode_get_option
 * returns the current value, or -1 for an unknown option. */
typedef enum {
    KANODE_OPT_POINTWISE_TABLE = 1,
    KANODE_OPT_FUSED_STEP = 2,
    KANODE_OPT_FUSED_SOLVE = 3,
    KANODE_OPT_FUSED_SOLVE_CAP = 4,
    KANODE_OPT_GRID_RHS = 5,
    KANODE_OPT_GRID_VJP = 6,
    KANODE_OPT_GRID_ADJ_STEP = 7,
    KANODE_OPT_ADJ_STEP_ROWS = 8,
    KANODE_OPT_PAIR_VJP = 9,
    KANODE_OPT_PAIR_FUSE = 10,
    KANODE_OPT_PAIR_PERSIST = 11,
    KANODE_OPT_PAIR_PERSIST_S = 12,
    KANODE_OPT_ADJ_FUSED_FINISH = 13,
    KANODE_OPT_PAIR_PERSIST_MAX_WG = 14,
    KANODE_OPT_PAIR_PERSIST_ABORT = 15,
    KANODE_OPT_LAST_ADJOINT = 16,
    KANODE_OPT_CHAIN_WIDE = 17,
    KANODE_OPT_RECORD_ADJOINT_STEPS = 18,
    KANODE_OPT_FK_DEVICE_LOOP = 19
} kanode_option;
typedef enum {
    KANODE_ADJ_NONE = 0,            /* no adjoint on this handle yet */
    KANODE_ADJ_HOST_LOOP = 1,       /* the host-loop integrator (per-step / per-stage launches) */
    KANODE_ADJ_CHAIN_WG = 2,        /* a small chain's whole adjoint in one workgroup (kd_chain_adjoint_kernel) */
    KANODE_ADJ_PAIR_PERSIST = 3,    /* a surrogate pair's whole adjoint in one launch (kd_pair_adjoint_kernel) */
    KANODE_ADJ_PAIR_FALLBACK = 4    /* that launch timed out on an exchange; re-run on the host loop */
} kanode_adjoint_path;
kanode_status kanode_set_option(kanode_handle* h, int32_t option, int64_t value);
int64_t kanode_get_option(const kanode_handle* h, int32_t option);

/* --- the RHS and its VJP (device pointers, async on stream) ----------------- */
/* du[N,B] = f(u[N,B]; p) */
kanode_status kanode_rhs(kanode_handle* h, const void* p, const void* u, void* du, int64_t batch, void* stream);

/* Runge-Kutta stage (OrdinaryDiffEqTsit5 perform_step!: the stage broadcast plus the dudt
 * call, and after the last stage the embedded-error residual of calculate_residuals):
 *     y  = u + Σ_{j<n_prev} c[j]·k[j]            (formed in registers where the kernel allows)
 *     du = f(y; p)
 *     y_out (nullable) <- y
 *     want_error: *error_sumsq = Σ_i (e_i / (abstol + reltol·max(|u_i|, |y_i|)))²,
 *                 e = Σ_{j<n_prev} ec[j]·k[j] + ec[n_prev]·du,  over all N·B entries
 * k, y_out, du are device [N,B] arrays of the state dtype; error_sumsq is a device double.
 * n_prev = 0 makes this kanode_rhs (plus the optional copy / error). */
#define KANODE_MAX_STAGES 8
typedef struct {
    int32_t n_prev;
    const void* k[KANODE_MAX_STAGES];
    double c[KANODE_MAX_STAGES];
    void* y_out;
    int32_t want_error;
    double ec[KANODE_MAX_STAGES + 1];
    double abstol, reltol;
    void* error_sumsq;
} kanode_stage;
kanode_status kanode_rhs_stage(kanode_handle* h, const void* p, const void* u, const kanode_stage* stage, void* du,
                               int64_t batch, void* stream);

/* Adjoint stage (SciMLSensitivity InterpolatingAdjoint with a VJP of the RHS: one RHS
 * evaluation of the adjoint ODE, written in reversed time τ = t_f - t as
 * dλ/dτ = λᵀ∂f/∂u, dμ/dτ = λᵀ∂f/∂p):
 *     y    = u + Σ_{j<state->n_prev} state->c[j]·state->k[j]  (the forward dense output at t)
 *     λs   = lam + Σ_{j<adj->n_prev} adj->c[j]·adj->k[j]      (adjoint stage input; -> adj->y_out)
 *     lamJ = λsᵀ ∂f/∂u at y;   dp (nullable) += λsᵀ ∂f/∂p at y
 *     adj->want_error: *adj->error_sumsq = Σ (e/sk)² over the λ entries,
 *                      e = Σ adj->ec[j] adj->k[j] + adj->ec[n]·lamJ, sk = abstol + reltol·max(|lam|, |λs|)
 * state->y_out and state->want_error are ignored. */
kanode_status kanode_vjp_stage(kanode_handle* h, const void* p, const void* u, const kanode_stage* state,
                               const void* lam, const kanode_stage* adj, void* lamJ, void* dp, int64_t batch,
                               void* stream);
/* lam_J[N,B] = (∂f/∂u)ᵀ lam   (nullable: skip)
 * dp[P]     += Σ_b (∂f/∂p)ᵀ lam  (nullable: skip) */
kanode_status kanode_vjp(kanode_handle* h, const void* p, const void* u, const void* lam, void* lam_J, void* dp,
                         int64_t batch, void* stream);

/* --- the integrator around the RHS ------------------
 * solve(ODEProblem(f, u0, (t0, tf), p), Tsit5(); saveat, abstol, reltol[, dt, adaptive])
 *     (LV_driver_KANODE.jl:122,180-184; Fisher-KPP_Source.jl:102-103), run as a
 *     native host loop issuing stream-ordered kernels: every stage is one
 *     kanode_rhs_stage (the stage combination formed inside the RHS kernel), the
 *     RHS tables are built once per solve (p is constant within it), saveat values
 *     come from the dense output on the device.  Semantics restate OrdinaryDiffEqTsit5
 *     1.1.0 / OrdinaryDiffEq 6.89 (third-party, pinned at Lotka-Volterra/Manifest.toml):
 *     Tsitouras 5(4) with FSAL, error norm = RMS over ALL N*B state entries (a batched
 *     state is one ODE), PI controller, Hairer-Wanner initial step, saveat from the
 *     free 4th-order interpolant.
 *   control = host: adaptive = 1 reads the 8-byte error norm once per step (the
 *     accept/reject decision on the host); adaptive = 0 (fixed dt) never synchronises,
 *     so the whole solve can be captured into a hipGraph by the caller.
 *   control = device: the controller runs on the GPU (tsit5_post_kernel: accept/reject,
 *     step size, saveat, dense-output record, u <- u_new commit) and the solve is a
 *     hipGraph of graph_steps step slots (stage launches read the step size from device
 *     memory) replayed until done: one host read per replay instead of per step.  The
 *     graph is cached in the kanode_solution.  Opt-in (it rarely pays on ROCm 7.2).
 *   control = auto: a chain of small layers (<= 16 wide) with <= 16 trajectories runs
 *     the whole solve in ONE workgroup (controller, saveat and dense output on the
 *     device), and with its dense output kept the whole adjoint too (one Lotka-Volterra
 *     trajectory: the adjoint on one wave); so does a Fisher-KPP field of <= 64 points
 *     (even Nx, <= 16 trajectories, rbf basis, G = 5 or 10, softsign / tanh_fast: one wave
 *     per trajectory, the pointwise KAN from the tables).  On the Fisher-KPP table path at
 *     Nx = 128/256/512 (fp64) each Tsit5 step is one launch (all six stages per trajectory
 *     row), the dense output is kept as u_n and the interpolation polynomials Q_1..Q_4
 *     (plus k_7), and the adjoint step is one launch (+ its finish); adaptive solves with
 *     the dense output kept run their step control on the device
 *     (KANODE_OPT_FK_DEVICE_LOOP).  Everything else runs as control = host.
 * kanode_adjoint_tsit5 is SciMLSensitivity 7.69's InterpolatingAdjoint (the NeuralODE
 * default; the reference's gradients): the adjoint ODE [λ; μ] integrated backward
 * with Tsit5 at the same tolerances, u(t) from the forward dense output, λ += ∂L/∂u
 * at every saveat time (tstops, FSAL re-evaluated after each jump); an adjoint stage
 * is one kanode_vjp_stage (or the fused step / one-workgroup kernels above). */
typedef struct {
    double abstol, reltol;          /* 1e-6, 1e-3 */
    double dt;                      /* adaptive = 0: the fixed step; adaptive = 1: initial step, 0 = Hairer-Wanner */
    int32_t adaptive;               /* 1 */
    int64_t maxiters;               /* 100000 */
    double dtmin;                   /* 0 */
    double beta1, beta2, gamma;     /* 7/50, 2/25, 9/10 */
    double qmin, qmax, qoldinit;    /* 1/5, 10, 1e-4 */
    int32_t control;                /* step control: 0 = auto (one-workgroup solve for small chains, else
                                       host), 1 = host (one 8-byte norm read per step), 2 = device (hipGraph
                                       of graph_steps step slots, replayed until done) */
    int32_t graph_steps;            /* step slots per graph replay (device control; even, 0 = 16) */
} kanode_solver_options;
void kanode_solver_options_default(kanode_solver_options* opt);

typedef struct {
    int64_t naccept, nreject, nf;   /* accepted / rejected steps, RHS (or VJP) evaluations */
} kanode_solve_stats;

/* Dense output of one forward solve (device memory owned by the object: u_n and the
 * 7 stage vectors of every accepted step).  Reusable: passing an existing object to
 * kanode_solve_tsit5 reuses its storage when large enough. */
typedef struct kanode_solution kanode_solution;
void kanode_solution_free(kanode_solution* sol);
int64_t kanode_solution_steps(const kanode_solution* sol);
/* The accepted steps of the solve: ts[i] (start time) and dts[i] (step size) for
 * i < min(steps, cap) (host arrays, either may be NULL).  Returns the step count, -1 for NULL. */
int64_t kanode_solution_step_sizes(const kanode_solution* sol, double* ts, double* dts, int64_t cap);

/* u_save[n_save, N, B] (device) <- u(saveat[j]); saveat (host, ascending, within
 * [t0, tf]).  dense: NULL = no dense output kept; else *dense (NULL or an object to
 * reuse) receives it, for kanode_adjoint_tsit5. */
kanode_status kanode_solve_tsit5(kanode_handle* h, const void* p, const void* u0, int64_t batch, double t0,
                                 double tf, const double* saveat, int64_t n_save, void* u_save,
                                 const kanode_solver_options* opt, kanode_solution** dense,
                                 kanode_solve_stats* stats, void* stream);

/* Given the forward solution `dense` (same h, p, batch) and dl_du[n_save, N, B] (device;
 * ∂L/∂u at the forward saveat times), writes du0[N, B] = dL/du0 and dp[P] = dL/dp
 * (both device, overwritten).  Either output may be NULL. */
kanode_status kanode_adjoint_tsit5(kanode_handle* h, const void* p, const kanode_solution* dense,
                                   const void* dl_du, void* du0, void* dp, const kanode_solver_options* opt,
                                   kanode_solve_stats* stats, void* stream);
/* Forward sensitivities: SciMLSensitivity 7.69 ForwardDiffSensitivity, the gradient the reference computes for its
 * small source-term problems (Fisher-KPP_Source.jl:198 and the Allen-Cahn source driver: Zygote.gradient(loss, p)
 * with no sensealg, length(u0) + length(p) <= 100, so the automatic choice is forward mode over ForwardDiff.Dual
 * numbers with one partial per parameter).  The solve of u together with S_k = ∂u/∂p_k, the Dual error norm over
 * value and partials (per entry the scale abstol + reltol·max(‖u_i‖, ‖unew_i‖), ‖x‖² = value² + Σ partials²; the
 * RMS over n·(1 + P) values), saveat from the same interpolant:
 *     u_save[n_save, N, B] <- u(saveat[j]);  s_save[n_save, P, N, B] <- ∂u(saveat[j])/∂p   (device, either nullable)
 * so dL/dp = Σ_j Σ_i ∂L/∂u_i(t_j) · s_save[j, :, i] (the host's contraction, as the Dual pullback's).  Covered: the
 * pointwise + periodic Laplacian RHS (fp64, rbf, G = 5 or 10, base activation, softsign / tanh_fast) with
 * nx·batch <= 64, as ONE workgroup (control is ignored); KANODE_ERR_UNSUPPORTED otherwise.  Synchronous (reads the
 * step counters). */
kanode_status kanode_forward_sensitivity_tsit5(kanode_handle* h, const void* p, const void* u0, int64_t batch,
                                               double t0, double tf, const double* saveat, int64_t n_save,
                                               void* u_save, void* s_save, const kanode_solver_options* opt,
                                               kanode_solve_stats* stats, void* stream);
/* 1 when kanode_forward_sensitivity_tsit5 covers this handle at `batch` trajectories, else 0 (no GPU work). */
/* The accepted steps of the handle's last kanode_forward_sensitivity_tsit5 (until the next solve without a dense output
 * on the handle): ts[i], dts[i] for i < min(count, cap) (host arrays, either NULL); returns the count (the first 4096
 * steps are recorded), -1 for a NULL handle.  Diagnostics: another solver can replay the same step sequence. */
int64_t kanode_forward_sensitivity_step_sizes(kanode_handle* h, double* ts, double* dts, int64_t cap);
int32_t kanode_forward_sensitivity_supported(const kanode_handle* h, int64_t batch);
/* KANODE_OPT_RECORD_ADJOINT_STEPS: the accepted step sizes of the handle's last kanode_adjoint_tsit5
 * (in backward order), out[i] for i < min(count, cap) (out may be NULL).  Returns the count (0 when not
 * recorded), -1 for NULL. */
int64_t kanode_adjoint_step_sizes(const kanode_handle* h, double* out, int64_t cap);
/* Fisher-KPP table path diagnostics (no reference counterpart): out[f] = the intervals of table f (0 φ, 1 φ', 2 swish)
   its last build rejected (their points take the direct formula), -1 for a table not built yet.  Synchronous
   (reads the device stamps after the handle's work); KANODE_ERR_UNSUPPORTED without a table path. */
kanode_status kanode_table_rejections(kanode_handle* h, int32_t out[3]);

/* --- the optimiser step after the gradient all-reduce -----------
 * Flux 0.14 Optimise.Adam + update!(opt, x, Δ) (LV_driver_KANODE.jl:219,287; Fisher-KPP_Source.jl:
 * 167,201), one stream-ordered launch over the n entries of x (x, m, v, g device arrays of `dtype`):
 *     Δ = scale·g            (scale = 1/world_size when g is the SUM all-reduce of [dp; L])
 *     m = β1·m + (1-β1)·Δ;   v = β2·v + ((1-β2)·Δ)·Δ
 *     x -= η · (m / (1 - β1ᵗ)) / (√(v / (1 - β2ᵗ)) + ε)
 * computed in double (Flux's Float64 hyper-parameters) and rounded to `dtype` on store.  beta1_t = β1ᵗ, beta2_t = β2ᵗ are Flux's running powers βp at this step (β at
 * the first step; the caller advances them).  m and v are caller-owned, persist across steps and
 * start at zero.  No handle: KANODE_ERR_INVALID_ARG on bad sizes / hyper-parameters,
 * KANODE_ERR_HIP when the launch fails. */
kanode_status kanode_adam_step(void* x, void* m, void* v, const void* g, int64_t n, int32_t dtype, double scale,
                               double eta, double beta1, double beta2, double eps, double beta1_t, double beta2_t,
                               void* stream);

/* --- the data-parallel gradient all-reduce (one process per GPU) -----------------
 * For hosts without a collective of their own (Julia, C): after kanode_adjoint_tsit5 on each rank's
 * trajectory shard, the flat [dp; L] is SUM all-reduced in place over RCCL (xGMI inside a node), then
 * kanode_adam_step(..., scale = 1/nranks, ...) applies the mean (the same step as kanode.Trainer with
 * torch.distributed, LV_driver_KANODE.jl:219-291 per rank).  Rank 0 makes the unique id and the host
 * hands its KANODE_COMM_ID_BYTES bytes to every rank (a file, MPI, an environment variable); every rank
 * then calls kanode_comm_create with the same nranks and id and its own rank and device (collective:
 * it returns when all ranks have joined).  Each rank needs its own GPU (RCCL refuses a second rank on a
 * device: kanode_comm_create then fails on both ranks instead of hanging); the calling thread's current
 * device is left as it was.  The all-reduce is stream-ordered (stream = the handle's). */
#define KANODE_COMM_ID_BYTES 128
typedef struct kanode_comm kanode_comm;
kanode_status kanode_comm_unique_id(uint8_t* id /* [KANODE_COMM_ID_BYTES] */);
kanode_status kanode_comm_create(int32_t nranks, int32_t rank, const uint8_t* id, int32_t device, kanode_comm** out);
kanode_status kanode_comm_allreduce_sum(kanode_comm* c, void* buf, int64_t count, int32_t dtype, void* stream);
int32_t kanode_comm_size(const kanode_comm* c);
int32_t kanode_comm_rank(const kanode_comm* c);
const char* kanode_comm_last_error(const kanode_comm* c);   /* NULL: the last failure without a communicator */
void kanode_comm_destroy(kanode_comm* c);

/* host-pointer variants (synchronous) */
kanode_status kanode_rhs_host(kanode_handle* h, const void* p, const void* u, void* du, int64_t batch);
kanode_status kanode_vjp_host(kanode_handle* h, const void* p, const void* u, const void* lam, void* lam_J,
                              void* dp, int64_t batch);

/* --- single-layer entry points (one Lux KDense call) ------------------------ */
/* y[O,K] = KDense_layer(x[I,K]; p_layer)  (p_layer = that layer's (C, W) slice) */
kanode_status kanode_layer_forward(kanode_handle* h, int32_t layer, const void* p_layer, const void* x, void* y,
                                   int64_t K, void* stream);
/* The same layer at a Runge-Kutta / adjoint stage input (the grid-sharded surrogate's first layer,
 * kanode/tp.py; Burgers_Surrogate.jl:85-97 "grid sharded"):
 *     y  = x + Σ_{j<sx->n_prev} sx->c[j]·sx->k[j]        -> sx->y_out (nullable)
 *     λs = lam + Σ_{j<sl->n_prev} sl->c[j]·sl->k[j]      -> sl->y_out (only when lam != NULL)
 *     out[O,K] = KDense_layer(y; p_layer)
 * k, lam, y_out are [I,K] arrays; want_error is ignored.  A wide input layer forms y and λs inside its
 * forward kernel (no combination launches); other layers run the combinations as separate launches. */
kanode_status kanode_layer_forward_stage(kanode_handle* h, int32_t layer, const void* p_layer, const void* x,
                                         const kanode_stage* sx, const void* lam, const kanode_stage* sl, void* out,
                                         int64_t K, void* stream);
/* xbar[I,K] = pullback(ybar)  (nullable); pbar_layer[P_l] += ... (nullable) */
kanode_status kanode_layer_vjp(kanode_handle* h, int32_t layer, const void* p_layer, const void* x,
                               const void* ybar, void* xbar, void* pbar_layer, int64_t K, void* stream);
/* act[O, I, K] with act(o,i,k) = Σ_g C[o,g+G i] φ_g(x[i,k]) + W[o,i] swish(x[i,k])
 * (Σ_i act(o,i,k) == y(o,k): the Activation_getter.jl:33-36,55-61 identity) */
kanode_status kanode_edge_activations(kanode_handle* h, int32_t layer, const void* p_layer, const void* x,
                                      void* act, int64_t K, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* KANODE_H */
