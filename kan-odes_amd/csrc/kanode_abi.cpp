// kanode_abi.cpp — the C-ABI (include/kanode.h) over the HIP kernels.
//
// Host-side responsibilities: validate the spec exactly as the reference ctor
// would accept it (kdense.jl:20-68), precompute the per-layer constants the
// kernels read (knots with Julia LinRange semantics, Float32 1/h, recurrence
// constants), own the device workspaces, and dispatch each layer to its kernel.
// No C++ exception crosses the ABI: every entry point returns a kanode_status.
#include "kanode.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "kan_device.hpp"
#include "kan_kernels.hpp"
#include "kanode_internal.hpp"

using kan::LayerConst;

namespace {

#ifndef KAN_SLAB_BLOCKS
#define KAN_SLAB_BLOCKS 4096
#endif
constexpr int kSlabBlocks = KAN_SLAB_BLOCKS;   // grid cap of the VJP kernels = slab rows

// column: thread per batch column (small I·G, O <= 16; e.g. LV [2,10,2]);
// wide-in / wide-out: the surrogate shapes (kan_wide.hip)
enum LayerKind { KIND_COL = 0, KIND_WIDE_IN = 1, KIND_WIDE_OUT = 2 };

}  // namespace

struct kanode_handle {
    kanode_spec spec{};
    int n_layers = 0;
    LayerConst hlc[KANODE_MAX_LAYERS];
    LayerKind kind[KANODE_MAX_LAYERS];
    LayerConst* dlc = nullptr;        // device copy
    int64_t P = 0;
    int64_t n_in = 0, n_out = 0;      // state length (input / output of the RHS)
    size_t esize = 8;
    int max_layer_P = 0;
    int max_dim = 0;
    // workspaces (device)
    void* slab = nullptr;
    size_t slab_bytes = 0;
    void* ws = nullptr;               // chain activations / gradients
    size_t ws_bytes = 0;
    int64_t reserved_batch = 0;
    // piecewise-polynomial pointwise RHS (kan_pp.hip)
    kan::PPConst hpc{};
    kan::PPConst* dpc = nullptr;
    double* dtable = nullptr;
    bool pp_on = false;
    // evaluation-strategy options (kanode_set_option; read here, never from the environment per launch)
    bool fused_step = true;           // KANODE_OPT_FUSED_STEP
    bool fused_solve = true;          // KANODE_OPT_FUSED_SOLVE
    bool pair_vjp = true;             // KANODE_OPT_PAIR_VJP
    bool pair_fuse = true;            // KANODE_OPT_PAIR_FUSE
    bool pair_persist = true;         // KANODE_OPT_PAIR_PERSIST
    int pair_persist_s = 0;           // KANODE_OPT_PAIR_PERSIST_S (0: the kernel's default)
    int pair_persist_max_wg = 0;      // KANODE_OPT_PAIR_PERSIST_MAX_WG (0: the device's co-resident capacity)
    bool pair_persist_abort = false;  // KANODE_OPT_PAIR_PERSIST_ABORT (tests: raise the abort word at launch)
    int last_adjoint = KANODE_ADJ_NONE;   // KANODE_OPT_LAST_ADJOINT (read-only)
    bool chain_wide = true;           // KANODE_OPT_CHAIN_WIDE
    bool record_adj_steps = false;    // KANODE_OPT_RECORD_ADJOINT_STEPS
    bool fk_loop = true;              // KANODE_OPT_FK_DEVICE_LOOP
    std::vector<double> adj_steps;    // the last kanode_adjoint_tsit5's accepted step sizes (when recorded)
    bool adj_fused_finish = false;    // KANODE_OPT_ADJ_FUSED_FINISH (measured even with the finish launch)
    unsigned* fin_ctr = nullptr;      // its two arrival counters (device, zeroed at allocation)
    // the surrogate pair's deferred adjoint stage: its second launch, held until the next stage is issued
    // (then both run as kd_vjp_pair_ba_kernel) or kanode_internal_vjp_flush; pair_par picks the buffers of
    // the ping-pong pairs (hidden / dot-product partials, basis store, y, λs) the next stage writes
    kan::PairPlan<double> pend_d{};
    kan::PairPlan<float> pend_f{};
    bool pend_valid = false;
    int pair_par = 0;
    // (set by the integrator) a lazy pair stage's λ error as per-block partials in err_parts (mapped host
    // memory, summed by the host), their count in *err_nparts, instead of a final-reduction launch
    double* err_parts = nullptr;
    int* err_nparts = nullptr;
    int fused_solve_cap = 0;          // KANODE_OPT_FUSED_SOLVE_CAP (0 = the kernel's block)
    kan::GridOverride grid_ovr{};     // KANODE_OPT_GRID_{RHS,VJP,ADJ_STEP} (0 = default)
    // the integrator's storage for solves without a dense output (kanode_solve.cpp)
    kanode_solution* solve_cache = nullptr;
    // table reuse inside one integrator solve (p constant): build each table set once
    bool hold_tables = false;
    bool built_phi = false, built_vjp = false;
    // adjoint stages whose dp / error reductions wait for kanode_internal_vjp_flush (one launch)
    void* defer_slab = nullptr;
    void* cstep_slab = nullptr;       // the fused small-chain adjoint step's six stage regions (grown on demand)
    size_t cstep_bytes = 0;
    void* step_slab = nullptr;        // fused adjoint step: six stages' moment rows + error partials
    kan::FinishJobs jobs{};
    int njobs = 0;
    // stage input y for kanode_rhs_stage's unfused path
    void* stage_ws = nullptr;
    size_t stage_ws_bytes = 0;
    // host staging (device buffers) for *_host calls
    void* stage = nullptr;
    size_t stage_bytes = 0;
    std::string err;
};

namespace {

kanode_status fail(kanode_handle* h, kanode_status s, const std::string& msg) {
    if (h) h->err = msg;
    return s;
}

// true when the launch must (re)build its table set; under hold_tables only the first does
bool table_build(kanode_handle* h, bool& built) {
    if (!h->hold_tables) return true;
    if (built) return false;
    built = true;
    return true;
}

#define HIP_TRY(h, expr)                                                                         \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return fail((h), KANODE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// Julia LinRange{Float32}(a, b, G)[j] = Float32((1-t)*a + t*b), t = j/(G-1) in Float64.
void knots_linrange(float lo, float hi, int G, float* out) {
    const double a = (double)lo, b = (double)hi;
    for (int j = 0; j < G; ++j) {
        const double t = (double)j / (double)(G - 1);
        out[j] = (float)((1.0 - t) * a + t * b);
    }
}

bool norm_range(int norm, double& lo, double& hi) {
    switch (norm) {
    case KANODE_NORM_TANH_FAST:
    case KANODE_NORM_TANH:
    case KANODE_NORM_SOFTSIGN: lo = -1.0; hi = 1.0; return true;
    case KANODE_NORM_SIGMOID:
    case KANODE_NORM_SIGMOID_FAST: lo = 0.0; hi = 1.0; return true;
    default: return false;   // identity: unbounded
    }
}

// Host-side layer constants (see kan_device.hpp for the recurrence).
kanode_status make_layer_const(kanode_handle* h, const kanode_layer_spec& s, int dtype, int64_t p_off,
                               LayerConst& lc) {
    std::memset(&lc, 0, sizeof(lc));
    if (s.in_dims < 1 || s.out_dims < 1)
        return fail(h, KANODE_ERR_INVALID_ARG, "in_dims and out_dims must be >= 1");
    if (s.grid_len < 2 || s.grid_len > KANODE_MAX_GRID)
        return fail(h, KANODE_ERR_UNSUPPORTED, "grid_len must be in [2, " + std::to_string(KANODE_MAX_GRID) + "]");
    if (s.normalizer < 0 || s.normalizer > KANODE_NORM_IDENTITY)
        return fail(h, KANODE_ERR_INVALID_ARG, "unknown normalizer");
    if (s.basis < 0 || s.basis > KANODE_BASIS_IQF) return fail(h, KANODE_ERR_INVALID_ARG, "unknown basis");
    if (!(s.grid_hi > s.grid_lo)) return fail(h, KANODE_ERR_INVALID_ARG, "grid_lims must satisfy lo < hi");
    lc.I = s.in_dims;
    lc.O = s.out_dims;
    lc.G = s.grid_len;
    lc.norm = s.normalizer;
    lc.basis = s.basis;
    lc.use_base = s.use_base_act ? 1 : 0;
    lc.iqf_quirk = s.iqf_reference_quirk ? 1 : 0;
    lc.p_off = p_off;
    lc.w_off = p_off + (int64_t)lc.O * lc.G * lc.I;
    knots_linrange(s.grid_lo, s.grid_hi, lc.G, lc.grid);
    volatile float den = s.denominator > 0.f ? s.denominator : (float)(2.0 / (double)(lc.G - 1));
    volatile float one = 1.0f;
    lc.invh = one / den;   // Float32 1/h (utils.jl:9)
    const double sd = (double)lc.invh;
    lc.g0 = (double)lc.grid[0];
    lc.s = sd;
    lc.gs = -lc.g0 * sd;
    lc.delta = ((double)s.grid_hi - (double)s.grid_lo) * sd / (double)(lc.G - 1);
    lc.unit_delta = lc.delta == 1.0 ? 1 : 0;
    // the knot-rounding correction exp(2·z0·e_j) is expanded around the centre of
    // 2·z0 ∈ [2 z_lo, 2 z_hi] over the normalizer's range
    double nlo = -1.0, nhi = 1.0;
    const bool bounded = norm_range(lc.norm, nlo, nhi);
    const double zlo = (nlo - lc.g0) * sd, zhi = (nhi - lc.g0) * sd;
    lc.tau_c = bounded ? (zlo + zhi) : 0.0;
    double emax = 0.0;
    bool exact = true;
    for (int j = 0; j < lc.G; ++j) {
        const double D = ((double)lc.grid[j] - (double)lc.grid[0]) * sd;
        lc.Dl[j] = D;
        lc.e[j] = D - (double)j * lc.delta;
        lc.h2[j] = 0.5 * lc.e[j] * lc.e[j];   // (kan_pp.hip's moment transforms read it; same order, same bits)
        const long double DL = D;
        lc.K[j] = (double)(std::exp(-DL * DL) * std::exp((long double)lc.tau_c * (long double)lc.e[j]));
        emax = std::max(emax, std::fabs(lc.e[j]));
        if (lc.e[j] != 0.0) exact = false;
    }
    // recurrence admissibility: bounded normalizer, no overflow of exp(-z0²) or
    // R^(G-1), and a centred 2nd-order correction accurate to < 1 ulp.
    lc.path = kan::PATH_DIRECT;
    if (lc.basis == KANODE_BASIS_RBF && bounded) {
        const double zmax = std::max(std::fabs(zlo), std::fabs(zhi));
        const double lim = (dtype == KANODE_F64) ? 600.0 : 80.0;
        const double tmax = (zhi - zlo) * emax;   // max |τ' e_j|
        const bool ok = zmax * zmax <= lim && 2.0 * zmax * std::fabs(lc.delta) * (lc.G - 1) <= lim &&
                        lc.delta > 0.0 && (dtype == KANODE_F64 ? tmax <= 1e-5 : tmax <= 1e-3);
        if (ok) lc.path = exact ? kan::PATH_REC : kan::PATH_REC_CORR;
    }
    return KANODE_OK;
}

// Piecewise-polynomial table constants for a pointwise KDense(1,1,G) (kan_pp.hip).
// Interval width: the largest power of two <= 0.16·h_u, h_u the knot spacing seen
// in u (h / max N'(u)), capped at 1/16; with degree 9 the Chebyshev interpolation
// error of a Gaussian of width h_u is then <= ~1e-16 of |C|.  ni <= 512 intervals
// centred on 0 (so softsign's kink at 0 is an interval edge).
void make_pp_const(const LayerConst& lc, int dtype, int64_t nx, kan::PPConst& pc) {
    std::memset(&pc, 0, sizeof(pc));
    pc.enabled = dtype == KANODE_F64 && (lc.basis == KANODE_BASIS_RBF || lc.basis == KANODE_BASIS_RSWAF) &&
                 nx >= 2 && nx % 2 == 0;
    const double slope = (lc.norm == KANODE_NORM_SIGMOID || lc.norm == KANODE_NORM_SIGMOID_FAST) ? 0.25 : 1.0;
    const double hu = (1.0 / (double)lc.invh) / slope;
    double w = 1.0 / 16.0;
    while (w > 0.16 * hu && w > 0x1p-20) w *= 0.5;
    int ni = kan::kPPMaxIntervals;
    while (ni > 16 && ni * w > 8.0) ni >>= 1;   // domain at most [-4, 4)
    pc.ni = ni;
    pc.w = w;
    pc.inv_w = 1.0 / w;
    pc.x0 = ni / 2;
    pc.lo = -(ni / 2) * w;
    pc.tol = 2e-14;
    const int N = kan::kPPCoef;
    const long double pi = 3.141592653589793238462643383279502884L;
    for (int m = 0; m < N; ++m) pc.xi[m] = (double)std::cos(pi * (2 * m + 1) / (2.0L * N));
    pc.tchk[0] = -1.0;
    pc.tchk[1] = 0.0;
    pc.tchk[2] = 1.0;
    // Q = (Chebyshev -> monomial) · DCT, in long double
    long double T[kan::kPPCoef][kan::kPPCoef] = {};
    T[0][0] = 1;
    T[1][1] = 1;
    for (int l = 2; l < N; ++l) {
        for (int i = 1; i < N; ++i) T[l][i] = 2 * T[l - 1][i - 1];
        for (int i = 0; i < N; ++i) T[l][i] -= T[l - 2][i];
    }
    for (int i = 0; i < N; ++i)
        for (int m = 0; m < N; ++m) {
            long double s = 0;
            for (int l = 0; l < N; ++l) {
                const long double d = (2.0L / N) * std::cos(pi * l * (2 * m + 1) / (2.0L * N)) * (l == 0 ? 0.5L : 1.0L);
                s += T[l][i] * d;
            }
            pc.Q[i][m] = (double)s;
        }
}

int64_t layer_P(const LayerConst& lc) {
    return (int64_t)lc.O * lc.G * lc.I + (lc.use_base ? (int64_t)lc.O * lc.I : 0);
}

bool is_capturing(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess) return false;
    return cs != hipStreamCaptureStatusNone;
}

// Partial-sum slab of the surrogate-shape kernels for a batch of B columns.
int64_t wide_slab_elems(const kanode_handle* h, int64_t B) {
    int64_t m = 0;
    for (int l = 0; l < h->n_layers; ++l) {
        const LayerConst& c = h->hlc[l];
        if (h->kind[l] == KIND_WIDE_IN) m = std::max<int64_t>(m, (int64_t)kan::widein_chunks(c) * B * c.O);
        if (h->kind[l] == KIND_WIDE_OUT) m = std::max<int64_t>(m, (int64_t)c.I * (c.G + 1) * B);
    }
    return m;
}

// The full-field surrogate shape KAN [N, H, N] (Burgers_Surrogate.jl:85-88,
// Schrodinger_Surrogate.jl:93-96): a wide-in layer feeding a wide-out layer.  Its RHS and VJP
// hand the hidden layer over as the wide-in chunk partials (no reduce launch).
bool surrogate_pair(const kanode_handle* h) {
    return h->n_layers == 2 && h->kind[0] == KIND_WIDE_IN && h->kind[1] == KIND_WIDE_OUT;
}

// Chain workspace layout (elements of the dtype), for a batch of B columns:
//   [hidden activations: Σ_{l>=1} I_l·B][grad ping: max_dim·B][grad pong: max_dim·B][wide slab]
//   [surrogate pair: the wide-in layer's chunk partials, chunks·B·H]
struct WsLayout {
    int64_t acts, g0, g1, wslab, pslab, sslab, bslab, pair2, total;   // pair2: offset of the second copy of [pslab, pair2)
};
WsLayout ws_layout(const kanode_handle* h, int64_t B) {
    WsLayout w{};
    int64_t e = 0;
    w.acts = e;
    for (int l = 1; l < h->n_layers; ++l) e += (int64_t)h->hlc[l].I * B;
    w.g0 = e;
    e += (int64_t)h->max_dim * B;
    w.g1 = e;
    e += (int64_t)h->max_dim * B;
    w.wslab = e;
    e += wide_slab_elems(h, B);
    w.pslab = e;
    if (surrogate_pair(h)) e += (int64_t)kan::widein_chunks(h->hlc[0]) * B * h->hlc[0].O;
    // [surrogate pair, two-launch pullback: the wide-out dot products' chunk partials, chunks·H·(G+1)·B]
    w.sslab = e;
    if (surrogate_pair(h)) e += (int64_t)kan::widein_chunks(h->hlc[0]) * h->hlc[1].I * (h->hlc[1].G + 1) * B;
    // [surrogate pair, two-launch pullback: the wide-in layer's basis store, B·I·(G + 2)]
    w.bslab = e;
    if (surrogate_pair(h)) e += kan::pair_basis_elems(h->hlc[0], B);
    // [surrogate pair: the second buffer of the ping-pong pairs pslab .. bslab (fused deferred stages)]
    w.pair2 = e;
    if (surrogate_pair(h)) e += e - w.pslab;
    w.total = e;
    return w;
}

size_t chain_ws_bytes(const kanode_handle* h, int64_t B) { return (size_t)ws_layout(h, B).total * h->esize; }

kanode_status flush_pair(kanode_handle* h, hipStream_t st);

kanode_status ensure_ws(kanode_handle* h, int64_t B, hipStream_t st) {
    const size_t need = h->spec.rhs_kind == KANODE_RHS_CHAIN ? chain_ws_bytes(h, B) : 0;
    if (need <= h->ws_bytes) return KANODE_OK;
    if (is_capturing(st))
        return fail(h, KANODE_ERR_CAPTURE, "batch exceeds reserved workspace during stream capture; call kanode_reserve");
    // a deferred surrogate-pair stage reads the old workspace: launch it before the buffer goes away
    if (kanode_status s = flush_pair(h, st); s != KANODE_OK) return s;
    HIP_TRY(h, hipStreamSynchronize(st));
    if (h->ws) HIP_TRY(h, hipFree(h->ws));
    h->ws = nullptr;
    h->ws_bytes = 0;
    HIP_TRY(h, hipMalloc(&h->ws, need));
    h->ws_bytes = need;
    return KANODE_OK;
}

// The wide kernels need the chain workspace's slab (sized by ensure_ws(K)).
template <typename T>
T* wide_slab(kanode_handle* h, int64_t K) {
    return (T*)h->ws + ws_layout(h, K).wslab;
}

template <typename T>
kanode_status layer_fwd_t(kanode_handle* h, int l, const T* p_full, const T* x, T* y, int64_t K, hipStream_t st) {
    const LayerConst& hl = h->hlc[l];
    switch (h->kind[l]) {
    case KIND_COL:
        HIP_TRY(h, kan::launch_kd_fwd_col<T>(hl, h->dlc + l, p_full, x, y, K, st));
        return KANODE_OK;
    case KIND_WIDE_IN:
        HIP_TRY(h, kan::launch_kd_fwd_widein<T>(hl, h->dlc + l, p_full, x, y, wide_slab<T>(h, K), K, st));
        return KANODE_OK;
    case KIND_WIDE_OUT:
        HIP_TRY(h, kan::launch_kd_fwd_wideout<T>(hl, h->dlc + l, p_full, x, y, K, st));
        return KANODE_OK;
    }
    return fail(h, KANODE_ERR_UNSUPPORTED, "layer kind");
}

template <typename T>
kanode_status layer_vjp_t(kanode_handle* h, int l, const T* p_full, const T* x, const T* yb, T* xb, T* pbar_full,
                          int64_t K, hipStream_t st) {
    const LayerConst& hl = h->hlc[l];
    switch (h->kind[l]) {
    case KIND_COL:
        HIP_TRY(h, kan::launch_kd_vjp_col<T>(hl, h->dlc + l, p_full, x, yb, xb, pbar_full, (T*)h->slab, kSlabBlocks,
                                             K, st));
        return KANODE_OK;
    case KIND_WIDE_IN:
        HIP_TRY(h, kan::launch_kd_vjp_widein<T>(hl, h->dlc + l, p_full, x, yb, xb, pbar_full, K, st));
        return KANODE_OK;
    case KIND_WIDE_OUT:
        HIP_TRY(h, kan::launch_kd_vjp_wideout<T>(hl, h->dlc + l, p_full, x, yb, xb, pbar_full, wide_slab<T>(h, K), K,
                                                 st));
        return KANODE_OK;
    }
    return fail(h, KANODE_ERR_UNSUPPORTED, "layer kind");
}

template <typename T>
kanode_status rhs_t(kanode_handle* h, const T* p, const T* u, T* du, int64_t B, hipStream_t st) {
    if (h->spec.rhs_kind == KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN) {
        const double dx2 = h->spec.dx * h->spec.dx;
        const T cd = (T)(h->spec.diffusion * (-2.0 / dx2)), co = (T)(h->spec.diffusion * (1.0 / dx2));
        if constexpr (std::is_same<T, double>::value) {
            if (h->pp_on) {
                HIP_TRY(h, kan::launch_fk_rhs_pp(h->hpc, h->hlc[0], h->dlc, h->dpc, p, h->dtable, cd, co, (int)h->spec.nx, u, du,
                                                 B, st, table_build(h, h->built_phi), h->grid_ovr.rhs));
                return KANODE_OK;
            }
        }
        HIP_TRY(h, kan::launch_fk_rhs<T>(h->hlc[0], h->dlc, p, cd, co, (int)h->spec.nx, u, du, B, st));
        return KANODE_OK;
    }
    bool all_col = h->n_layers > 1;
    for (int l = 0; l < h->n_layers; ++l) all_col = all_col && h->kind[l] == KIND_COL;
    if (all_col) {
        const hipError_t e = kan::launch_kd_chain_col<T>(h->hlc, h->n_layers, h->dlc, p, h->P, u, du, B, st);
        if (e == hipSuccess) return KANODE_OK;
        if (e != hipErrorNotSupported) return fail(h, KANODE_ERR_HIP, std::string("launch_kd_chain_col: ") + hipGetErrorString(e));
    }
    kanode_status s = ensure_ws(h, B, st);
    if (s != KANODE_OK) return s;
    T* ws = (T*)h->ws;
    const WsLayout wl = ws_layout(h, B);
    if (surrogate_pair(h)) {   // two launches: wide-in partials -> wide-out summing them itself
        T* ps = ws + wl.pslab;
        HIP_TRY(h, kan::launch_kd_fwd_widein<T>(h->hlc[0], h->dlc, p, u, (T*)nullptr, ps, B, st));
        HIP_TRY(h, kan::launch_kd_fwd_wideout<T>(h->hlc[1], h->dlc + 1, p, (const T*)nullptr, du, B, st, ps,
                                                  kan::widein_chunks(h->hlc[0])));
        return KANODE_OK;
    }
    const T* cur = u;
    for (int l = 0; l < h->n_layers; ++l) {
        T* out = (l == h->n_layers - 1) ? du : ws + ((l % 2) ? wl.g1 : wl.g0);
        s = layer_fwd_t<T>(h, l, p, cur, out, B, st);
        if (s != KANODE_OK) return s;
        cur = out;
    }
    return KANODE_OK;
}

template <typename T>
kanode_status vjp_t(kanode_handle* h, const T* p, const T* u, const T* lam, T* lamJ, T* dp, int64_t B,
                    hipStream_t st) {
    if (h->spec.rhs_kind == KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN) {
        const double dx2 = h->spec.dx * h->spec.dx;
        const T cd = (T)(h->spec.diffusion * (-2.0 / dx2)), co = (T)(h->spec.diffusion * (1.0 / dx2));
        // lam_J is needed for the kernel's store; use workspace when the caller passes NULL
        T* out = lamJ;
        if (!out) {
            kanode_status s = ensure_ws(h, B, st);
            if (s != KANODE_OK) return s;
            if (h->ws_bytes < (size_t)(h->spec.nx * B) * h->esize) {
                if (is_capturing(st)) return fail(h, KANODE_ERR_CAPTURE, "workspace too small during capture");
                HIP_TRY(h, hipStreamSynchronize(st));
                if (h->ws) HIP_TRY(h, hipFree(h->ws));
                HIP_TRY(h, hipMalloc(&h->ws, (size_t)(h->spec.nx * B) * h->esize));
                h->ws_bytes = (size_t)(h->spec.nx * B) * h->esize;
            }
            out = (T*)h->ws;
        }
        if constexpr (std::is_same<T, double>::value) {
            if (h->pp_on && kan::fk_vjp_pp_supported(h->hlc[0], (int)h->spec.nx)) {
                HIP_TRY(h, kan::launch_fk_vjp_pp(h->hpc, h->hlc[0], h->dlc, h->dpc, p, h->dtable, cd, co,
                                                 (int)h->spec.nx, u, lam, out, dp, (double*)h->slab, kSlabBlocks, B,
                                                 st, table_build(h, h->built_vjp), h->grid_ovr.vjp));
                return KANODE_OK;
            }
        }
        HIP_TRY(h, kan::launch_fk_vjp<T>(h->hlc[0], h->dlc, p, cd, co, (int)h->spec.nx, u, lam, out, dp, (T*)h->slab,
                                         kSlabBlocks, B, st));
        return KANODE_OK;
    }
    if (lamJ && h->n_in == h->n_out) {
        bool all_col = true;
        for (int l = 0; l < h->n_layers; ++l) all_col = all_col && h->kind[l] == KIND_COL;
        if (all_col) {
            const kan::StageArgs<T> none{};
            const hipError_t e = kan::launch_kd_chain_vjp_stage<T>(h->hlc, h->n_layers, h->dlc, p, h->P, u, none, lam,
                                                                   none, nullptr, lamJ, dp, false, nullptr, h->slab,
                                                                   h->slab_bytes, B, st);
            if (e == hipSuccess) return KANODE_OK;
            if (e != hipErrorNotSupported)
                return fail(h, KANODE_ERR_HIP, std::string("launch_kd_chain_vjp_stage: ") + hipGetErrorString(e));
        }
    }
    kanode_status s = ensure_ws(h, B, st);
    if (s != KANODE_OK) return s;
    T* ws = (T*)h->ws;
    const WsLayout wl = ws_layout(h, B);
    if (surrogate_pair(h)) {
        T* ps = ws + wl.pslab;
        T* hbar = ws + wl.g0;
        const int nb = kan::widein_chunks(h->hlc[0]);
        if (lamJ && h->pair_vjp) {
            // two launches (launch_kd_vjp_pair): the wide-in forward blocks also form the wide-out dot
            // products' chunk partials; the wide-out parameter cotangents beside the wide-in pullback
            // (x̄ of the hidden layer formed per block)
            const hipError_t e = kan::launch_kd_vjp_pair<T>(h->hlc[0], h->hlc[1], h->dlc, p, u, nullptr, lam, u, ps,
                                                            ws + wl.sslab, lamJ, dp, B, st, false, nullptr, 0,
                                                            nullptr, ws + wl.bslab);
            if (e == hipSuccess) return KANODE_OK;
            if (e != hipErrorNotSupported)
                return fail(h, KANODE_ERR_HIP, std::string("launch_kd_vjp_pair: ") + hipGetErrorString(e));
        }
        // four launches: wide-in partials; the wide-out pullback's dot products and parameter
        // cotangents in one launch; its input cotangent; the wide-in pullback
        HIP_TRY(h, kan::launch_kd_fwd_widein<T>(h->hlc[0], h->dlc, p, u, (T*)nullptr, ps, B, st));
        HIP_TRY(h, kan::launch_kd_vjp_wideout<T>(h->hlc[1], h->dlc + 1, p, (const T*)nullptr, lam, hbar, dp,
                                                  ws + wl.wslab, B, st, ps, nb));
        if (lamJ || dp) HIP_TRY(h, kan::launch_kd_vjp_widein<T>(h->hlc[0], h->dlc, p, u, hbar, lamJ, dp, B, st));
        return KANODE_OK;
    }
    // forward recompute, keeping every hidden layer's input
    const T* acts[KANODE_MAX_LAYERS];
    acts[0] = u;
    T* wp = ws + wl.acts;
    for (int l = 1; l < h->n_layers; ++l) {
        T* out = wp;
        wp += (int64_t)h->hlc[l].I * B;
        s = layer_fwd_t<T>(h, l - 1, p, acts[l - 1], out, B, st);
        if (s != KANODE_OK) return s;
        acts[l] = out;
    }
    T* g0 = ws + wl.g0;
    T* g1 = ws + wl.g1;
    const T* g = lam;
    for (int l = h->n_layers - 1; l >= 0; --l) {
        T* out = (l == 0) ? lamJ : ((l % 2) ? g0 : g1);
        if (l == 0 && !out) out = (g == g0) ? g1 : g0;   // caller skipped lam_J
        s = layer_vjp_t<T>(h, l, p, acts[l], g, out, dp, B, st);
        if (s != KANODE_OK) return s;
        g = out;
    }
    return KANODE_OK;
}

kanode_status ensure_stage_ws(kanode_handle* h, size_t need, hipStream_t st);

template <typename T>
kanode_status stage_t(kanode_handle* h, const T* p, const T* u, const kanode_stage* sg, T* du, int64_t B,
                      hipStream_t st, const double* cscale = nullptr, const int32_t* skip = nullptr) {
    if (sg->n_prev < 0 || sg->n_prev > KANODE_MAX_STAGES)
        return fail(h, KANODE_ERR_INVALID_ARG, "n_prev must be in [0, KANODE_MAX_STAGES]");
    if (h->n_in != h->n_out) return fail(h, KANODE_ERR_INVALID_ARG, "stage needs an RHS with N_in == N_out");
    if (sg->want_error && !sg->error_sumsq) return fail(h, KANODE_ERR_INVALID_ARG, "want_error needs error_sumsq");
    kan::StageArgs<T> sa{};
    sa.nk = sg->n_prev;
    for (int j = 0; j < sg->n_prev; ++j) {
        if (!sg->k[j]) return fail(h, KANODE_ERR_INVALID_ARG, "null stage vector k[" + std::to_string(j) + "]");
        sa.k[j] = (const T*)sg->k[j];
        sa.c[j] = sg->c[j];
    }
    for (int j = 0; j <= sg->n_prev; ++j) sa.ec[j] = sg->want_error ? sg->ec[j] : 0.0;
    sa.abstol = sg->abstol;
    sa.reltol = sg->reltol;
    sa.cscale = cscale;
    sa.skip = skip;
    double* err_out = sg->want_error ? (double*)sg->error_sumsq : nullptr;
    if constexpr (std::is_same<T, double>::value) {
        if (h->spec.rhs_kind == KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN && h->pp_on &&
            kan::fk_stage_pp_supported(h->hpc, (int)h->spec.nx)) {
            const double dx2 = h->spec.dx * h->spec.dx;
            const double cd = h->spec.diffusion * (-2.0 / dx2), co = h->spec.diffusion * (1.0 / dx2);
            HIP_TRY(h, kan::launch_fk_stage_pp(h->hpc, h->hlc[0], h->dlc, h->dpc, p, h->dtable, cd, co,
                                               (int)h->spec.nx, u, sa, (double*)sg->y_out, (double*)h->slab,
                                               kSlabBlocks, err_out, du, B, st, table_build(h, h->built_phi),
                                               h->grid_ovr.rhs));
            return KANODE_OK;
        }
    }
    if (h->spec.rhs_kind == KANODE_RHS_CHAIN) {
        // a small chain: stage input, RHS and error partials in one kernel (kd_chain_col_kernel)
        bool all_col = true;
        for (int l = 0; l < h->n_layers; ++l) all_col = all_col && h->kind[l] == KIND_COL;
        if (all_col) {
            const hipError_t e = kan::launch_kd_chain_col<T>(h->hlc, h->n_layers, h->dlc, p, h->P, u, du, B, st, &sa,
                                                             (T*)sg->y_out, (double*)h->slab, kSlabBlocks, err_out);
            if (e == hipSuccess) return KANODE_OK;
            if (e != hipErrorNotSupported)
                return fail(h, KANODE_ERR_HIP, std::string("launch_kd_chain_col: ") + hipGetErrorString(e));
        }
    }
    const int64_t n = h->n_in * B;
    if (h->spec.rhs_kind == KANODE_RHS_CHAIN && surrogate_pair(h) && !skip) {
        // surrogate pair: the wide-in forward forms y itself (kd_fwd_widein_co_kernel stage input)
        kanode_status s = ensure_ws(h, B, st);
        if (s != KANODE_OK) return s;
        T* y = (T*)sg->y_out;
        if (!y && err_out) {
            if ((s = ensure_stage_ws(h, (size_t)n * sizeof(T), st)) != KANODE_OK) return s;
            y = (T*)h->stage_ws;
        }
        T* ps = (T*)h->ws + ws_layout(h, B).pslab;
        kan::WideStageIn<T> si{};
        si.su = sa;
        si.y_out = y;
        HIP_TRY(h, kan::launch_kd_fwd_widein<T>(h->hlc[0], h->dlc, p, u, (T*)nullptr, ps, B, st, &si));
        HIP_TRY(h, kan::launch_kd_fwd_wideout<T>(h->hlc[1], h->dlc + 1, p, (const T*)nullptr, du, B, st, ps,
                                                  kan::widein_chunks(h->hlc[0])));
        if (err_out) HIP_TRY(h, kan::launch_stage_error<T>(u, y, du, sa, (double*)h->slab, kSlabBlocks, err_out, n, st));
        return KANODE_OK;
    }
    // unfused: y materialised (into y_out or the handle's stage workspace), RHS, error pass
    T* y = (T*)sg->y_out;
    if (!y) {
        kanode_status s = ensure_stage_ws(h, (size_t)n * sizeof(T), st);
        if (s != KANODE_OK) return s;
        y = (T*)h->stage_ws;
    }
    HIP_TRY(h, kan::launch_stage_lincomb<T>(u, sa, y, n, st));
    kanode_status s = rhs_t<T>(h, p, y, du, B, st);
    if (s != KANODE_OK) return s;
    if (err_out) HIP_TRY(h, kan::launch_stage_error<T>(u, y, du, sa, (double*)h->slab, kSlabBlocks, err_out, n, st));
    return KANODE_OK;
}

// stage workspace of at least `need` bytes (the unfused stage paths)
kanode_status ensure_stage_ws(kanode_handle* h, size_t need, hipStream_t st) {
    if (need <= h->stage_ws_bytes) return KANODE_OK;
    if (is_capturing(st)) return fail(h, KANODE_ERR_CAPTURE, "stage workspace too small during capture");
    if (kanode_status s = flush_pair(h, st); s != KANODE_OK) return s;   // (reads the old stage workspace)
    HIP_TRY(h, hipStreamSynchronize(st));
    if (h->stage_ws) HIP_TRY(h, hipFree(h->stage_ws));
    h->stage_ws = nullptr;
    h->stage_ws_bytes = 0;
    HIP_TRY(h, hipMalloc(&h->stage_ws, need));
    h->stage_ws_bytes = need;
    return KANODE_OK;
}

template <typename T>
kanode_status stage_args(kanode_handle* h, const kanode_stage* sg, kan::StageArgs<T>& sa) {
    if (sg->n_prev < 0 || sg->n_prev > KANODE_MAX_STAGES)
        return fail(h, KANODE_ERR_INVALID_ARG, "n_prev must be in [0, KANODE_MAX_STAGES]");
    sa = kan::StageArgs<T>{};
    sa.nk = sg->n_prev;
    for (int j = 0; j < sg->n_prev; ++j) {
        if (!sg->k[j]) return fail(h, KANODE_ERR_INVALID_ARG, "null stage vector k[" + std::to_string(j) + "]");
        sa.k[j] = (const T*)sg->k[j];
        sa.c[j] = sg->c[j];
    }
    for (int j = 0; j <= sg->n_prev; ++j) sa.ec[j] = sg->want_error ? sg->ec[j] : 0.0;
    sa.abstol = sg->abstol;
    sa.reltol = sg->reltol;
    return KANODE_OK;
}

// one region of the deferred reduction slab: [grid][G+1] partials + [grid] error partials, grid <= kSlabBlocks/2
constexpr size_t kDeferRegion = (size_t)(kSlabBlocks / 2) * (kan::kMaxGrid + 2);

// The fixed-size reduction slabs of the Fisher-KPP table adjoint (deferred stage reductions and the
// one-launch adjoint step).  kanode_create allocates them for handles that can take that path; this
// covers a handle whose table path was switched on later, and refuses to allocate under capture.
kanode_status ensure_adjoint_slabs(kanode_handle* h, hipStream_t st, bool at_create = false) {
    if (h->defer_slab && h->step_slab && h->fin_ctr) return KANODE_OK;
    if (!at_create && is_capturing(st))
        return fail(h, KANODE_ERR_CAPTURE, "adjoint reduction slabs would be allocated during capture");
    const size_t defer = kDeferRegion * sizeof(double) * kan::kMaxFinishJobs;
    const size_t step = (size_t)(kSlabBlocks / 2) * (6 * (kan::kMaxGrid + 1) + 1) * sizeof(double);
    if ((!h->defer_slab && hipMalloc(&h->defer_slab, defer) != hipSuccess) ||
        (!h->step_slab && hipMalloc(&h->step_slab, step) != hipSuccess)) {
        (void)hipGetLastError();
        return fail(h, KANODE_ERR_ALLOC, "adjoint reduction slabs");
    }
    if (!h->fin_ctr) {   // the fused finish's arrival counters: zero here, and back to zero after every step
        if (hipMalloc(&h->fin_ctr, 2 * sizeof(unsigned)) != hipSuccess ||
            hipMemset(h->fin_ctr, 0, 2 * sizeof(unsigned)) != hipSuccess) {
            (void)hipGetLastError();
            if (h->fin_ctr) (void)hipFree(h->fin_ctr);
            h->fin_ctr = nullptr;
            return fail(h, KANODE_ERR_ALLOC, "adjoint finish counters");
        }
    }
    return KANODE_OK;
}

template <typename T>
kan::PairPlan<T>& pair_pending(kanode_handle* h);
template <>
kan::PairPlan<double>& pair_pending<double>(kanode_handle* h) { return h->pend_d; }
template <>
kan::PairPlan<float>& pair_pending<float>(kanode_handle* h) { return h->pend_f; }

// the deferred surrogate-pair stage's second launch, alone (nothing to fuse it with)
kanode_status flush_pair(kanode_handle* h, hipStream_t st) {
    if (!h->pend_valid) return KANODE_OK;
    h->pend_valid = false;
    const hipError_t e = h->spec.dtype == KANODE_F64 ? kan::launch_pair_second<double>(h->pend_d, nullptr, st)
                                                     : kan::launch_pair_second<float>(h->pend_f, nullptr, st);
    if (e != hipSuccess) return fail(h, KANODE_ERR_HIP, std::string("launch_pair_second: ") + hipGetErrorString(e));
    return KANODE_OK;
}

kanode_status vjp_flush(kanode_handle* h, hipStream_t st) {
    if (kanode_status s = flush_pair(h, st); s != KANODE_OK) return s;
    if (h->njobs == 0) return KANODE_OK;
    const int n = h->njobs;
    h->njobs = 0;
    HIP_TRY(h, kan::launch_vjp_finish_jobs(h->jobs, n, h->hlc[0].G + (h->hlc[0].use_base ? 1 : 0), st));
    return KANODE_OK;
}

template <typename T>
kanode_status vjp_stage_t(kanode_handle* h, const T* p, const T* u, const kanode_stage* state, const T* lam,
                          const kanode_stage* adj, T* lamJ, T* dp, int64_t B, hipStream_t st, bool dp_assign = false,
                          const double* su_scale = nullptr, const double* sl_scale = nullptr, bool defer = false) {
    if (h->n_in != h->n_out) return fail(h, KANODE_ERR_INVALID_ARG, "adjoint stage needs an RHS with N_in == N_out");
    if (adj->want_error && !adj->error_sumsq) return fail(h, KANODE_ERR_INVALID_ARG, "want_error needs error_sumsq");
    kan::StageArgs<T> su, sl;
    kanode_status s = stage_args<T>(h, state, su);
    if (s != KANODE_OK) return s;
    s = stage_args<T>(h, adj, sl);
    if (s != KANODE_OK) return s;
    su.cscale = su_scale;
    sl.cscale = sl_scale;
    const int64_t n = h->n_in * B;
    if constexpr (std::is_same<T, double>::value) {
        // Fisher-KPP table path: the whole adjoint stage in one streaming kernel + one reduction
        if (h->spec.rhs_kind == KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN && h->pp_on && lamJ &&
            kan::fk_vjp_pp_supported(h->hlc[0], (int)h->spec.nx)) {
            const double dx2 = h->spec.dx * h->spec.dx;
            const double cd = h->spec.diffusion * (-2.0 / dx2), co = h->spec.diffusion * (1.0 / dx2);
            double* err_out = adj->want_error ? (double*)adj->error_sumsq : nullptr;
            if (defer && (dp || err_out)) {
                if (h->njobs == kan::kMaxFinishJobs && (s = vjp_flush(h, st)) != KANODE_OK) return s;
                if ((s = ensure_adjoint_slabs(h, st)) != KANODE_OK) return s;
                double* region = (double*)h->defer_slab + (size_t)h->njobs * kDeferRegion;
                int grid = 0;
                HIP_TRY(h, kan::launch_fk_vjp_stage_pp(h->hpc, h->hlc[0], h->dlc, h->dpc, p, h->dtable, cd, co,
                                                       (int)h->spec.nx, u, su, lam, sl, (double*)adj->y_out, lamJ,
                                                       dp, dp_assign, err_out, region, kSlabBlocks, B, st,
                                                       table_build(h, h->built_vjp), &grid, h->grid_ovr.vjp));
                kan::FinishJob& jb = h->jobs.j[h->njobs++];
                jb.slab = region;
                jb.err_slab = region + (int64_t)grid * (h->hlc[0].G + 1);
                jb.dp = dp;
                jb.err_out = err_out;
                jb.nblk = grid;
                jb.assign = dp_assign ? 1 : 0;
                return KANODE_OK;
            }
            HIP_TRY(h, kan::launch_fk_vjp_stage_pp(h->hpc, h->hlc[0], h->dlc, h->dpc, p, h->dtable, cd, co,
                                                   (int)h->spec.nx, u, su, lam, sl, (double*)adj->y_out, lamJ, dp,
                                                   dp_assign, err_out, (double*)h->slab, kSlabBlocks, B, st,
                                                   table_build(h, h->built_vjp), nullptr, h->grid_ovr.vjp));
            return KANODE_OK;
        }
    }
    if (h->spec.rhs_kind == KANODE_RHS_CHAIN && lamJ) {
        // a small chain: the whole adjoint stage in one kernel (kd_chain_vjp_stage_kernel) + one reduction
        bool all_col = true;
        for (int l = 0; l < h->n_layers; ++l) all_col = all_col && h->kind[l] == KIND_COL;
        if (all_col) {
            const hipError_t e = kan::launch_kd_chain_vjp_stage<T>(
                h->hlc, h->n_layers, h->dlc, p, h->P, u, su, lam, sl, (T*)adj->y_out, lamJ, dp, dp_assign,
                adj->want_error ? (double*)adj->error_sumsq : nullptr, h->slab, h->slab_bytes, B, st);
            if (e == hipSuccess) return KANODE_OK;
            if (e != hipErrorNotSupported)
                return fail(h, KANODE_ERR_HIP, std::string("launch_kd_chain_vjp_stage: ") + hipGetErrorString(e));
        }
    }
    if (h->spec.rhs_kind == KANODE_RHS_CHAIN && surrogate_pair(h) && lamJ) {
        // surrogate pair: y and λs formed by the wide-in forward (no combination launches), the
        // parameter cotangents written with = when dp_assign (no memset): four launches per stage.
        // Deferred stages (the integrator's, `defer`) run lazily: a stage's second launch waits for the next
        // stage and both run as one (launch_pair_second with next), alternating the ping-pong buffers.
        const bool lazy = defer && h->pair_vjp && h->pair_fuse;
        if (!lazy || chain_ws_bytes(h, B) > h->ws_bytes || 4 * (size_t)n * sizeof(T) > h->stage_ws_bytes)
            if ((s = flush_pair(h, st)) != KANODE_OK) return s;   // (and before any buffer is reallocated)
        if ((s = ensure_ws(h, B, st)) != KANODE_OK) return s;
        if ((s = ensure_stage_ws(h, 4 * (size_t)n * sizeof(T), st)) != KANODE_OK) return s;
        const int par = lazy ? h->pair_par : 0;
        const WsLayout wl = ws_layout(h, B);
        T* ws = (T*)h->ws;
        const int64_t pp = par ? wl.pair2 - wl.pslab : 0;   // the ping-pong pairs' second buffer
        T* y = (T*)h->stage_ws + (size_t)par * 2 * n;
        T* ls = adj->y_out ? (T*)adj->y_out : y + n;
        T* ps = ws + wl.pslab + pp;
        T* hbar = ws + wl.g0;
        const int nb = kan::widein_chunks(h->hlc[0]);
        kan::WideStageIn<T> si{};
        si.su = su;
        si.y_out = y;
        si.lam = lam;
        si.sl = sl;
        si.ls_out = ls;
        hipError_t e = hipErrorNotSupported;
        bool err_done = false;
        if (lazy) {
            double* err_out = adj->want_error ? (double*)adj->error_sumsq : nullptr;
            kan::PairPlan<T> pl;
            const bool host_parts = err_out && h->err_parts && h->err_nparts;
            e = kan::plan_kd_vjp_pair<T>(h->hlc[0], h->hlc[1], h->dlc, p, u, &si, lam, y, ps, ws + wl.sslab + pp, lamJ,
                                         dp, B, dp_assign, host_parts ? h->err_parts : (double*)h->slab, kSlabBlocks,
                                         err_out, ws + wl.bslab + pp, &pl);
            if (e == hipSuccess) {
                if (host_parts && pl.err_out) {   // the host sums the partials: no final launch
                    *h->err_nparts = pl.err_rows;
                    pl.err_out = nullptr;
                }
                kan::PairPlan<T>& pend = pair_pending<T>(h);
                if (h->pend_valid) e = kan::launch_pair_second<T>(pend, &pl, st);
                else e = kan::launch_pair_first<T>(pl, st);
                if (e != hipSuccess)
                    return fail(h, KANODE_ERR_HIP, std::string("pair stage: ") + hipGetErrorString(e));
                pend = pl;
                h->pend_valid = true;
                h->pair_par ^= 1;
                return KANODE_OK;
            }
            if (e != hipErrorNotSupported)
                return fail(h, KANODE_ERR_HIP, std::string("plan_kd_vjp_pair: ") + hipGetErrorString(e));
            if ((s = flush_pair(h, st)) != KANODE_OK) return s;
        } else if (h->pair_vjp) {   // two launches (see vjp_t), plus the λ error's final sum
            double* err_out = adj->want_error ? (double*)adj->error_sumsq : nullptr;
            const bool host_parts = err_out && h->err_parts && h->err_nparts;   // (as the lazy path)
            kan::PairPlan<T> pl;
            e = kan::plan_kd_vjp_pair<T>(h->hlc[0], h->hlc[1], h->dlc, p, u, &si, lam, y, ps, ws + wl.sslab + pp, lamJ,
                                         dp, B, dp_assign, host_parts ? h->err_parts : (double*)h->slab, kSlabBlocks,
                                         err_out, ws + wl.bslab + pp, &pl);
            if (e == hipSuccess) {
                if (host_parts && pl.err_out) {
                    *h->err_nparts = pl.err_rows;
                    pl.err_out = nullptr;
                }
                if ((e = kan::launch_pair_first<T>(pl, st)) == hipSuccess) e = kan::launch_pair_second<T>(pl, nullptr, st);
                if (e != hipSuccess) return fail(h, KANODE_ERR_HIP, std::string("pair stage: ") + hipGetErrorString(e));
            } else if (e != hipErrorNotSupported) {
                return fail(h, KANODE_ERR_HIP, std::string("plan_kd_vjp_pair: ") + hipGetErrorString(e));
            }
            err_done = e == hipSuccess && err_out != nullptr;
        }
        if (e != hipSuccess) {
            HIP_TRY(h, kan::launch_kd_fwd_widein<T>(h->hlc[0], h->dlc, p, u, (T*)nullptr, ps, B, st, &si));
            HIP_TRY(h, kan::launch_kd_vjp_wideout<T>(h->hlc[1], h->dlc + 1, p, (const T*)nullptr, ls, hbar, dp,
                                                      ws + wl.wslab, B, st, ps, nb, dp_assign));
            HIP_TRY(h, kan::launch_kd_vjp_widein<T>(h->hlc[0], h->dlc, p, y, hbar, lamJ, dp, B, st, dp_assign));
        }
        if (adj->want_error && !err_done)
            HIP_TRY(h, kan::launch_stage_error<T>(lam, ls, lamJ, sl, (double*)h->slab, kSlabBlocks,
                                                  (double*)adj->error_sumsq, n, st));
        return KANODE_OK;
    }
    if (dp && dp_assign) HIP_TRY(h, hipMemsetAsync(dp, 0, (size_t)h->P * sizeof(T), st));
    if ((s = ensure_stage_ws(h, 2 * (size_t)n * sizeof(T), st)) != KANODE_OK) return s;
    T* y = su.nk ? (T*)h->stage_ws : (T*)u;
    T* ls = adj->y_out ? (T*)adj->y_out : (sl.nk ? (T*)h->stage_ws + n : (T*)lam);
    if (su.nk) HIP_TRY(h, kan::launch_stage_lincomb<T>(u, su, y, n, st));
    if (sl.nk || adj->y_out) HIP_TRY(h, kan::launch_stage_lincomb<T>(lam, sl, ls, n, st));
    if ((s = vjp_t<T>(h, p, y, ls, lamJ, dp, B, st)) != KANODE_OK) return s;
    if (adj->want_error)
        HIP_TRY(h, kan::launch_stage_error<T>(lam, ls, lamJ, sl, (double*)h->slab, kSlabBlocks,
                                              (double*)adj->error_sumsq, n, st));
    return KANODE_OK;
}

kanode_status check_handle(kanode_handle* h) {
    if (!h) return KANODE_ERR_INVALID_ARG;
    hipError_t e = hipSetDevice(h->spec.device);
    if (e != hipSuccess) return fail(h, KANODE_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
    return KANODE_OK;
}

}  // namespace

namespace {
// one layer at a stage input (kanode_layer_forward_stage): y = x + Σ c·k (and λs = lam + Σ c·k) formed by the
// wide-in forward's blocks themselves (kd_fwd_widein_stage_kernel, the fma order of stage_lincomb_kernel);
// any other layer kind gets the combinations as their own launches first
template <typename T>
kanode_status layer_fwd_stage_t(kanode_handle* h, int l, const T* p_full, const T* x, const kanode_stage* sx,
                                const T* lam, const kanode_stage* sl, T* out, int64_t K, hipStream_t st) {
    kan::StageArgs<T> su{}, sla{};
    kanode_status s = stage_args<T>(h, sx, su);
    if (s != KANODE_OK) return s;
    if (lam && (s = stage_args<T>(h, sl, sla)) != KANODE_OK) return s;
    const LayerConst& hl = h->hlc[l];
    const int64_t n = (int64_t)hl.I * K;
    if (h->kind[l] == KIND_WIDE_IN) {
        kan::WideStageIn<T> si{};
        si.su = su;
        si.y_out = (T*)sx->y_out;
        si.lam = lam;
        si.sl = sla;
        si.ls_out = lam ? (T*)sl->y_out : nullptr;
        HIP_TRY(h, kan::launch_kd_fwd_widein<T>(hl, h->dlc + l, p_full, x, out, wide_slab<T>(h, K), K, st, &si));
        return KANODE_OK;
    }
    T* y = (T*)sx->y_out;
    if (!y) {
        if ((s = ensure_stage_ws(h, (size_t)n * sizeof(T), st)) != KANODE_OK) return s;
        y = (T*)h->stage_ws;
    }
    HIP_TRY(h, kan::launch_stage_lincomb<T>(x, su, y, n, st));
    if (lam) HIP_TRY(h, kan::launch_stage_lincomb<T>(lam, sla, (T*)sl->y_out, n, st));
    return layer_fwd_t<T>(h, l, p_full, y, out, K, st);
}
}  // namespace

extern "C" {

int32_t kanode_abi_version(void) { return KANODE_ABI_VERSION; }

const char* kanode_status_string(kanode_status s) {
    switch (s) {
    case KANODE_OK: return "ok";
    case KANODE_ERR_INVALID_ARG: return "invalid argument";
    case KANODE_ERR_UNSUPPORTED: return "unsupported configuration";
    case KANODE_ERR_HIP: return "HIP runtime error";
    case KANODE_ERR_ALLOC: return "allocation failure";
    case KANODE_ERR_CAPTURE: return "allocation needed during stream capture";
    }
    return "unknown status";
}

const char* kanode_last_error(const kanode_handle* h) { return h ? h->err.c_str() : "null handle"; }

kanode_status kanode_create(const kanode_spec* spec, kanode_handle** out) {
    if (!spec || !out) return KANODE_ERR_INVALID_ARG;
    *out = nullptr;
    kanode_handle* h = new (std::nothrow) kanode_handle();
    if (!h) return KANODE_ERR_ALLOC;
    h->spec = *spec;
    auto bail = [&](kanode_status s) {
        // keep the handle so the caller can read kanode_last_error, then destroy
        *out = h;
        return s;
    };
    if (spec->dtype != KANODE_F32 && spec->dtype != KANODE_F64)
        return bail(fail(h, KANODE_ERR_INVALID_ARG, "dtype must be KANODE_F32 or KANODE_F64"));
    h->esize = spec->dtype == KANODE_F64 ? 8 : 4;
    if (spec->n_layers < 1 || spec->n_layers > KANODE_MAX_LAYERS)
        return bail(fail(h, KANODE_ERR_INVALID_ARG, "n_layers must be in [1, 8]"));
    h->n_layers = spec->n_layers;
    int64_t off = 0;
    for (int l = 0; l < h->n_layers; ++l) {
        kanode_status s = make_layer_const(h, spec->layers[l], spec->dtype, off, h->hlc[l]);
        if (s != KANODE_OK) return bail(s);
        if (l > 0 && spec->layers[l].in_dims != spec->layers[l - 1].out_dims)
            return bail(fail(h, KANODE_ERR_INVALID_ARG,
                             "layer " + std::to_string(l) + " in_dims != previous out_dims (Lux.Chain)"));
        off += layer_P(h->hlc[l]);
        h->max_layer_P = std::max<int>(h->max_layer_P, (int)layer_P(h->hlc[l]));
        h->max_dim = std::max({h->max_dim, h->hlc[l].I, h->hlc[l].O});
        // kernel class for this layer
        const LayerConst& lc = h->hlc[l];
        const size_t rows = (size_t)(lc.G * lc.I + lc.I);
        if (lc.O <= 16 && (size_t)(lc.G * lc.I + lc.O + lc.I) * 65 * h->esize <= 150 * 1024 &&
            layer_P(lc) <= 64 * 32) {
            h->kind[l] = KIND_COL;
        } else if (lc.O <= kan::kWideOMax) {
            h->kind[l] = KIND_WIDE_IN;
        } else if (rows * kan::kWideKT * h->esize <= 150 * 1024) {
            h->kind[l] = KIND_WIDE_OUT;
        } else {
            return bail(fail(h, KANODE_ERR_UNSUPPORTED,
                             "layer " + std::to_string(l) + " shape (I=" + std::to_string(lc.I) + ", O=" +
                                 std::to_string(lc.O) + ") is not supported by this build"));
        }
    }
    h->P = off;
    if (spec->rhs_kind == KANODE_RHS_CHAIN) {
        h->n_in = spec->layers[0].in_dims;
        h->n_out = spec->layers[h->n_layers - 1].out_dims;
    } else if (spec->rhs_kind == KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN) {
        if (h->n_layers != 1 || spec->layers[0].in_dims != 1 || spec->layers[0].out_dims != 1)
            return bail(fail(h, KANODE_ERR_INVALID_ARG, "pointwise RHS needs exactly one KDense(1, 1, G)"));
        if (spec->nx < 1 || spec->nx > (1 << 30)) return bail(fail(h, KANODE_ERR_INVALID_ARG, "nx must be >= 1"));
        if (!(spec->dx > 0.0)) return bail(fail(h, KANODE_ERR_INVALID_ARG, "dx must be > 0"));
        h->n_in = h->n_out = spec->nx;
    } else {
        return bail(fail(h, KANODE_ERR_INVALID_ARG, "unknown rhs_kind"));
    }
    hipError_t e = hipSetDevice(spec->device);
    if (e != hipSuccess) return bail(fail(h, KANODE_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e)));
    if ((e = hipMalloc(&h->dlc, sizeof(LayerConst) * h->n_layers)) != hipSuccess)
        return bail(fail(h, KANODE_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e)));
    if ((e = hipMemcpy(h->dlc, h->hlc, sizeof(LayerConst) * h->n_layers, hipMemcpyHostToDevice)) != hipSuccess)
        return bail(fail(h, KANODE_ERR_HIP, std::string("hipMemcpy: ") + hipGetErrorString(e)));
    if (spec->rhs_kind == KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN) {
        make_pp_const(h->hlc[0], spec->dtype, spec->nx, h->hpc);
        if (h->hpc.enabled) {
            if ((e = hipMalloc(&h->dpc, sizeof(kan::PPConst))) != hipSuccess ||
                (e = hipMemcpy(h->dpc, &h->hpc, sizeof(kan::PPConst), hipMemcpyHostToDevice)) != hipSuccess ||
                (e = hipMalloc(&h->dtable, sizeof(double) * kan::pp_tables_doubles(h->hpc.ni))) != hipSuccess ||
                (e = hipMemset(h->dtable, 0, sizeof(double) * kan::pp_tables_doubles(h->hpc.ni))) != hipSuccess)
                return bail(fail(h, KANODE_ERR_HIP, std::string("pp table: ") + hipGetErrorString(e)));
            h->pp_on = true;
            if (kan::fk_vjp_pp_supported(h->hlc[0], (int)spec->nx)) {
                kanode_status s = ensure_adjoint_slabs(h, nullptr, true);
                if (s != KANODE_OK) return bail(s);
            }
        }
    }
    // per-block partial rows: the column-kernel VJPs need a layer's (an all-column chain's) P per row;
    // the wide kernels keep their partials in the chain workspace; stage / error / table-VJP rows
    // need at most kMaxGrid + 2 doubles
    {
        bool all_col = true;
        int64_t col_P = 0;
        for (int l = 0; l < h->n_layers; ++l) {
            if (h->kind[l] == KIND_COL) col_P = std::max<int64_t>(col_P, layer_P(h->hlc[l]));
            else all_col = false;
        }
        if (all_col) col_P = std::max<int64_t>(col_P, h->P);
        const size_t row = std::max<size_t>((size_t)col_P * h->esize, (size_t)(kan::kMaxGrid + 2) * sizeof(double));
        h->slab_bytes = (size_t)kSlabBlocks * row;
    }
    if ((e = hipMalloc(&h->slab, h->slab_bytes)) != hipSuccess)
        return bail(fail(h, KANODE_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e)));
    *out = h;
    return KANODE_OK;
}

void kanode_destroy(kanode_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->spec.device);
    if (h->dlc) (void)hipFree(h->dlc);
    if (h->slab) (void)hipFree(h->slab);
    if (h->ws) (void)hipFree(h->ws);
    if (h->stage) (void)hipFree(h->stage);
    if (h->dpc) (void)hipFree(h->dpc);
    if (h->stage_ws) (void)hipFree(h->stage_ws);
    if (h->dtable) (void)hipFree(h->dtable);
    if (h->defer_slab) (void)hipFree(h->defer_slab);
    if (h->cstep_slab) (void)hipFree(h->cstep_slab);
    if (h->step_slab) (void)hipFree(h->step_slab);
    if (h->fin_ctr) (void)hipFree(h->fin_ctr);
    if (h->solve_cache) kanode_solution_free(h->solve_cache);
    delete h;
}

int64_t kanode_param_length(const kanode_handle* h) { return h ? h->P : -1; }
int64_t kanode_layer_param_length(const kanode_handle* h, int32_t layer) {
    if (!h || layer < 0 || layer >= h->n_layers) return -1;
    return layer_P(h->hlc[layer]);
}
int64_t kanode_state_length(const kanode_handle* h) { return h ? h->n_in : -1; }

kanode_status kanode_knots(const kanode_handle* h, int32_t layer, float* grid_out) {
    if (!h || !grid_out || layer < 0 || layer >= h->n_layers) return KANODE_ERR_INVALID_ARG;
    std::memcpy(grid_out, h->hlc[layer].grid, sizeof(float) * h->hlc[layer].G);
    return KANODE_OK;
}

kanode_status kanode_reserve(kanode_handle* h, int64_t max_batch) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if (max_batch < 0) return fail(h, KANODE_ERR_INVALID_ARG, "max_batch < 0");
    s = ensure_ws(h, max_batch, nullptr);
    if (s != KANODE_OK) return s;
    if (h->spec.rhs_kind == KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN) {
        const size_t need = (size_t)(h->spec.nx * max_batch) * h->esize;
        if (need > h->ws_bytes) {
            HIP_TRY(h, hipDeviceSynchronize());
            if (h->ws) HIP_TRY(h, hipFree(h->ws));
            HIP_TRY(h, hipMalloc(&h->ws, need));
            h->ws_bytes = need;
        }
    }
    // Reset the table stamps: re-zeroing the stamp region here (the call before graph capture / a
    // new batch) invalidates every build block's stamp, so the next launch rebuilds every table.
    if (h->dtable) {
        const int64_t off = (int64_t)kan::kPPMaxFns * kan::kPPCoef * h->hpc.ni;
        HIP_TRY(h, hipDeviceSynchronize());
        HIP_TRY(h, hipMemset(h->dtable + off, 0, sizeof(double) * (size_t)(kan::pp_tables_doubles(h->hpc.ni) - off)));
    }
    h->reserved_batch = std::max(h->reserved_batch, max_batch);
    return KANODE_OK;
}

kanode_status kanode_set_option(kanode_handle* h, int32_t option, int64_t value) {
    if (!h) return KANODE_ERR_INVALID_ARG;
    auto flag = [&](bool& dst, const char* name) {
        if (value != 0 && value != 1) return fail(h, KANODE_ERR_INVALID_ARG, std::string(name) + " takes 0 or 1");
        dst = value == 1;
        return KANODE_OK;
    };
    auto count = [&](int& dst, const char* name, int64_t hi) {
        if (value < 0 || value > hi)
            return fail(h, KANODE_ERR_INVALID_ARG, std::string(name) + " takes 0.." + std::to_string(hi));
        dst = (int)value;
        return KANODE_OK;
    };
    switch (option) {
    case KANODE_OPT_POINTWISE_TABLE:
        if (value != 0 && value != 1) return fail(h, KANODE_ERR_INVALID_ARG, "POINTWISE_TABLE takes 0 or 1");
        if (value == 1 && !h->hpc.enabled)
            return fail(h, KANODE_ERR_UNSUPPORTED,
                        "POINTWISE_TABLE needs a pointwise f64 RHS with rbf/rswaf basis and even nx");
        h->pp_on = value == 1;
        return KANODE_OK;
    case KANODE_OPT_FUSED_STEP: return flag(h->fused_step, "FUSED_STEP");
    case KANODE_OPT_FUSED_SOLVE: return flag(h->fused_solve, "FUSED_SOLVE");
    case KANODE_OPT_FUSED_SOLVE_CAP: return count(h->fused_solve_cap, "FUSED_SOLVE_CAP", 1 << 20);
    case KANODE_OPT_GRID_RHS: return count(h->grid_ovr.rhs, "GRID_RHS", 1 << 24);
    case KANODE_OPT_GRID_VJP: return count(h->grid_ovr.vjp, "GRID_VJP", kSlabBlocks / 2);
    case KANODE_OPT_GRID_ADJ_STEP: return count(h->grid_ovr.vstep, "GRID_ADJ_STEP", kSlabBlocks / 2);
    case KANODE_OPT_ADJ_STEP_ROWS: return flag(h->grid_ovr.vstep_rows, "ADJ_STEP_ROWS");
    case KANODE_OPT_PAIR_VJP: return flag(h->pair_vjp, "PAIR_VJP");
    case KANODE_OPT_PAIR_FUSE: return flag(h->pair_fuse, "PAIR_FUSE");
    case KANODE_OPT_PAIR_PERSIST: return flag(h->pair_persist, "PAIR_PERSIST");
    case KANODE_OPT_PAIR_PERSIST_S:
        // the kernel is instantiated for 4, 8 and 16 points per workgroup
        if (value != 0 && value != 4 && value != 8 && value != 16)
            return fail(h, KANODE_ERR_INVALID_ARG, "PAIR_PERSIST_S takes 0 (default), 4, 8 or 16");
        h->pair_persist_s = (int)value;
        return KANODE_OK;
    case KANODE_OPT_ADJ_FUSED_FINISH: return flag(h->adj_fused_finish, "ADJ_FUSED_FINISH");
    case KANODE_OPT_PAIR_PERSIST_MAX_WG: return count(h->pair_persist_max_wg, "PAIR_PERSIST_MAX_WG", 1 << 20);
    case KANODE_OPT_PAIR_PERSIST_ABORT: return flag(h->pair_persist_abort, "PAIR_PERSIST_ABORT");
    case KANODE_OPT_LAST_ADJOINT: return fail(h, KANODE_ERR_INVALID_ARG, "LAST_ADJOINT is read-only");
    case KANODE_OPT_CHAIN_WIDE: return flag(h->chain_wide, "CHAIN_WIDE");
    case KANODE_OPT_RECORD_ADJOINT_STEPS: return flag(h->record_adj_steps, "RECORD_ADJOINT_STEPS");
    case KANODE_OPT_FK_DEVICE_LOOP: return flag(h->fk_loop, "FK_DEVICE_LOOP");
    }
    return fail(h, KANODE_ERR_INVALID_ARG, "unknown option " + std::to_string(option));
}

int64_t kanode_get_option(const kanode_handle* h, int32_t option) {
    if (!h) return -1;
    switch (option) {
    case KANODE_OPT_POINTWISE_TABLE: return h->pp_on ? 1 : 0;
    case KANODE_OPT_FUSED_STEP: return h->fused_step ? 1 : 0;
    case KANODE_OPT_FUSED_SOLVE: return h->fused_solve ? 1 : 0;
    case KANODE_OPT_FUSED_SOLVE_CAP: return h->fused_solve_cap;
    case KANODE_OPT_GRID_RHS: return h->grid_ovr.rhs;
    case KANODE_OPT_GRID_VJP: return h->grid_ovr.vjp;
    case KANODE_OPT_GRID_ADJ_STEP: return h->grid_ovr.vstep;
    case KANODE_OPT_ADJ_STEP_ROWS: return h->grid_ovr.vstep_rows ? 1 : 0;
    case KANODE_OPT_PAIR_VJP: return h->pair_vjp ? 1 : 0;
    case KANODE_OPT_PAIR_FUSE: return h->pair_fuse ? 1 : 0;
    case KANODE_OPT_PAIR_PERSIST: return h->pair_persist ? 1 : 0;
    case KANODE_OPT_PAIR_PERSIST_S: return h->pair_persist_s;
    case KANODE_OPT_ADJ_FUSED_FINISH: return h->adj_fused_finish ? 1 : 0;
    case KANODE_OPT_PAIR_PERSIST_MAX_WG: return h->pair_persist_max_wg;
    case KANODE_OPT_PAIR_PERSIST_ABORT: return h->pair_persist_abort ? 1 : 0;
    case KANODE_OPT_LAST_ADJOINT: return h->last_adjoint;
    case KANODE_OPT_CHAIN_WIDE: return h->chain_wide ? 1 : 0;
    case KANODE_OPT_RECORD_ADJOINT_STEPS: return h->record_adj_steps ? 1 : 0;
    case KANODE_OPT_FK_DEVICE_LOOP: return h->fk_loop ? 1 : 0;
    }
    return -1;
}

kanode_status kanode_rhs(kanode_handle* h, const void* p, const void* u, void* du, int64_t batch, void* stream) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if (batch < 0) return fail(h, KANODE_ERR_INVALID_ARG, "batch < 0");
    if (batch == 0) return KANODE_OK;
    if (!p || !u || !du) return fail(h, KANODE_ERR_INVALID_ARG, "null pointer");
    hipStream_t st = (hipStream_t)stream;
    if (h->spec.dtype == KANODE_F64) return rhs_t<double>(h, (const double*)p, (const double*)u, (double*)du, batch, st);
    return rhs_t<float>(h, (const float*)p, (const float*)u, (float*)du, batch, st);
}

kanode_status kanode_rhs_stage(kanode_handle* h, const void* p, const void* u, const kanode_stage* stage, void* du,
                               int64_t batch, void* stream) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if (!stage) return fail(h, KANODE_ERR_INVALID_ARG, "null stage");
    if (batch < 0) return fail(h, KANODE_ERR_INVALID_ARG, "batch < 0");
    if (batch == 0) return KANODE_OK;
    if (!p || !u || !du) return fail(h, KANODE_ERR_INVALID_ARG, "null p/u/du");
    hipStream_t st = (hipStream_t)stream;
    if (h->spec.dtype == KANODE_F64) return stage_t<double>(h, (const double*)p, (const double*)u, stage, (double*)du,
                                                            batch, st);
    return stage_t<float>(h, (const float*)p, (const float*)u, stage, (float*)du, batch, st);
}

kanode_status kanode_vjp_stage(kanode_handle* h, const void* p, const void* u, const kanode_stage* state,
                               const void* lam, const kanode_stage* adj, void* lamJ, void* dp, int64_t batch,
                               void* stream) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if (!state || !adj) return fail(h, KANODE_ERR_INVALID_ARG, "null stage");
    if (batch < 0) return fail(h, KANODE_ERR_INVALID_ARG, "batch < 0");
    if (batch == 0) return KANODE_OK;
    if (!p || !u || !lam || !lamJ) return fail(h, KANODE_ERR_INVALID_ARG, "null p/u/lam/lamJ");
    hipStream_t st = (hipStream_t)stream;
    if (h->spec.dtype == KANODE_F64)
        return vjp_stage_t<double>(h, (const double*)p, (const double*)u, state, (const double*)lam, adj,
                                   (double*)lamJ, (double*)dp, batch, st);
    return vjp_stage_t<float>(h, (const float*)p, (const float*)u, state, (const float*)lam, adj, (float*)lamJ,
                              (float*)dp, batch, st);
}

kanode_status kanode_vjp(kanode_handle* h, const void* p, const void* u, const void* lam, void* lam_J, void* dp,
                         int64_t batch, void* stream) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if (batch < 0) return fail(h, KANODE_ERR_INVALID_ARG, "batch < 0");
    if (batch == 0) return KANODE_OK;
    if (!p || !u || !lam) return fail(h, KANODE_ERR_INVALID_ARG, "null pointer");
    hipStream_t st = (hipStream_t)stream;
    if (h->spec.dtype == KANODE_F64)
        return vjp_t<double>(h, (const double*)p, (const double*)u, (const double*)lam, (double*)lam_J, (double*)dp,
                             batch, st);
    return vjp_t<float>(h, (const float*)p, (const float*)u, (const float*)lam, (float*)lam_J, (float*)dp, batch, st);
}

static kanode_status stage_alloc(kanode_handle* h, size_t bytes) {
    if (bytes <= h->stage_bytes) return KANODE_OK;
    if (h->stage) HIP_TRY(h, hipFree(h->stage));
    h->stage = nullptr;
    h->stage_bytes = 0;
    HIP_TRY(h, hipMalloc(&h->stage, bytes));
    h->stage_bytes = bytes;
    return KANODE_OK;
}

kanode_status kanode_rhs_host(kanode_handle* h, const void* p, const void* u, void* du, int64_t batch) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if (batch <= 0) return batch == 0 ? KANODE_OK : fail(h, KANODE_ERR_INVALID_ARG, "batch < 0");
    const size_t bp = (size_t)h->P * h->esize, bu = (size_t)(h->n_in * batch) * h->esize,
                 bo = (size_t)(h->n_out * batch) * h->esize;
    if ((s = stage_alloc(h, bp + bu + bo)) != KANODE_OK) return s;
    char* d = (char*)h->stage;
    HIP_TRY(h, hipMemcpy(d, p, bp, hipMemcpyHostToDevice));
    HIP_TRY(h, hipMemcpy(d + bp, u, bu, hipMemcpyHostToDevice));
    if ((s = kanode_rhs(h, d, d + bp, d + bp + bu, batch, nullptr)) != KANODE_OK) return s;
    HIP_TRY(h, hipMemcpy(du, d + bp + bu, bo, hipMemcpyDeviceToHost));
    return KANODE_OK;
}

kanode_status kanode_vjp_host(kanode_handle* h, const void* p, const void* u, const void* lam, void* lam_J, void* dp,
                              int64_t batch) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if (batch <= 0) return batch == 0 ? KANODE_OK : fail(h, KANODE_ERR_INVALID_ARG, "batch < 0");
    const size_t bp = (size_t)h->P * h->esize, bu = (size_t)(h->n_in * batch) * h->esize,
                 bo = (size_t)(h->n_out * batch) * h->esize;
    if ((s = stage_alloc(h, 2 * bp + 2 * bu + bo)) != KANODE_OK) return s;
    char* d = (char*)h->stage;
    char* dp_d = d + bp;
    char* u_d = dp_d + bp;
    char* lam_d = u_d + bu;
    char* lj_d = lam_d + bo;
    HIP_TRY(h, hipMemcpy(d, p, bp, hipMemcpyHostToDevice));
    HIP_TRY(h, hipMemcpy(u_d, u, bu, hipMemcpyHostToDevice));
    HIP_TRY(h, hipMemcpy(lam_d, lam, bo, hipMemcpyHostToDevice));
    if (dp) HIP_TRY(h, hipMemcpy(dp_d, dp, bp, hipMemcpyHostToDevice));
    if ((s = kanode_vjp(h, d, u_d, lam_d, lam_J ? lj_d : nullptr, dp ? dp_d : nullptr, batch, nullptr)) != KANODE_OK)
        return s;
    if (lam_J) HIP_TRY(h, hipMemcpy(lam_J, lj_d, bu, hipMemcpyDeviceToHost));
    if (dp) HIP_TRY(h, hipMemcpy(dp, dp_d, bp, hipMemcpyDeviceToHost));
    return KANODE_OK;
}

kanode_status kanode_layer_forward(kanode_handle* h, int32_t layer, const void* p_layer, const void* x, void* y,
                                   int64_t K, void* stream) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if (layer < 0 || layer >= h->n_layers) return fail(h, KANODE_ERR_INVALID_ARG, "layer out of range");
    if (K < 0) return fail(h, KANODE_ERR_INVALID_ARG, "K < 0");
    if (K == 0) return KANODE_OK;
    if (!p_layer || !x || !y) return fail(h, KANODE_ERR_INVALID_ARG, "null pointer");
    // kernels index p_full + p_off: shift the caller's layer slice back
    const int64_t off = h->hlc[layer].p_off;
    hipStream_t st = (hipStream_t)stream;
    if ((s = ensure_ws(h, K, st)) != KANODE_OK) return s;
    if (h->spec.dtype == KANODE_F64)
        return layer_fwd_t<double>(h, layer, (const double*)p_layer - off, (const double*)x, (double*)y, K, st);
    return layer_fwd_t<float>(h, layer, (const float*)p_layer - off, (const float*)x, (float*)y, K, st);
}

kanode_status kanode_layer_forward_stage(kanode_handle* h, int32_t layer, const void* p_layer, const void* x,
                                         const kanode_stage* sx, const void* lam, const kanode_stage* sl, void* out,
                                         int64_t K, void* stream) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if (layer < 0 || layer >= h->n_layers) return fail(h, KANODE_ERR_INVALID_ARG, "layer out of range");
    if (K < 0) return fail(h, KANODE_ERR_INVALID_ARG, "K < 0");
    if (K == 0) return KANODE_OK;
    if (!p_layer || !x || !sx || !out) return fail(h, KANODE_ERR_INVALID_ARG, "null pointer");
    if (lam && (!sl || !sl->y_out)) return fail(h, KANODE_ERR_INVALID_ARG, "lam needs sl with y_out (the λs output)");
    const int64_t off = h->hlc[layer].p_off;
    hipStream_t st = (hipStream_t)stream;
    if ((s = ensure_ws(h, K, st)) != KANODE_OK) return s;
    if (h->spec.dtype == KANODE_F64)
        return layer_fwd_stage_t<double>(h, layer, (const double*)p_layer - off, (const double*)x, sx,
                                         (const double*)lam, sl, (double*)out, K, st);
    return layer_fwd_stage_t<float>(h, layer, (const float*)p_layer - off, (const float*)x, sx, (const float*)lam, sl,
                                    (float*)out, K, st);
}

kanode_status kanode_layer_vjp(kanode_handle* h, int32_t layer, const void* p_layer, const void* x, const void* ybar,
                               void* xbar, void* pbar_layer, int64_t K, void* stream) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if (layer < 0 || layer >= h->n_layers) return fail(h, KANODE_ERR_INVALID_ARG, "layer out of range");
    if (K < 0) return fail(h, KANODE_ERR_INVALID_ARG, "K < 0");
    if (K == 0) return KANODE_OK;
    if (!p_layer || !x || !ybar || !xbar) return fail(h, KANODE_ERR_INVALID_ARG, "null pointer (xbar is required)");
    const int64_t off = h->hlc[layer].p_off;
    hipStream_t st = (hipStream_t)stream;
    if ((s = ensure_ws(h, K, st)) != KANODE_OK) return s;
    if (h->spec.dtype == KANODE_F64)
        return layer_vjp_t<double>(h, layer, (const double*)p_layer - off, (const double*)x, (const double*)ybar,
                                   (double*)xbar, pbar_layer ? (double*)pbar_layer - off : nullptr, K, st);
    return layer_vjp_t<float>(h, layer, (const float*)p_layer - off, (const float*)x, (const float*)ybar, (float*)xbar,
                              pbar_layer ? (float*)pbar_layer - off : nullptr, K, st);
}

kanode_status kanode_edge_activations(kanode_handle* h, int32_t layer, const void* p_layer, const void* x, void* act,
                                      int64_t K, void* stream) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if (layer < 0 || layer >= h->n_layers) return fail(h, KANODE_ERR_INVALID_ARG, "layer out of range");
    if (K < 0) return fail(h, KANODE_ERR_INVALID_ARG, "K < 0");
    if (K == 0) return KANODE_OK;
    if (!p_layer || !x || !act) return fail(h, KANODE_ERR_INVALID_ARG, "null pointer");
    const int64_t off = h->hlc[layer].p_off;
    hipStream_t st = (hipStream_t)stream;
    if (h->hlc[layer].O > 64) return fail(h, KANODE_ERR_UNSUPPORTED, "edge activations need out_dims <= 64");
    if (h->spec.dtype == KANODE_F64) {
        HIP_TRY(h, kan::launch_kd_edge_act<double>(h->hlc[layer], h->dlc + layer, (const double*)p_layer - off,
                                                   (const double*)x, (double*)act, K, st));
    } else {
        HIP_TRY(h, kan::launch_kd_edge_act<float>(h->hlc[layer], h->dlc + layer, (const float*)p_layer - off,
                                                  (const float*)x, (float*)act, K, st));
    }
    return KANODE_OK;
}

kanode_status kanode_adam_step(void* x, void* m, void* v, const void* g, int64_t n, int32_t dtype, double scale,
                               double eta, double beta1, double beta2, double eps, double beta1_t, double beta2_t,
                               void* stream) {
    if (n < 0 || (dtype != KANODE_F32 && dtype != KANODE_F64)) return KANODE_ERR_INVALID_ARG;
    if (n == 0) return KANODE_OK;
    if (!x || !m || !v || !g) return KANODE_ERR_INVALID_ARG;
    // 1 - β^t must stay positive (t >= 1 with 0 <= β < 1): the bias corrections divide by it
    if (!(beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && beta1_t < 1.0 && beta2_t < 1.0))
        return KANODE_ERR_INVALID_ARG;
    kan::AdamArgs a;
    a.scale = scale;
    a.beta1 = beta1;
    a.beta2 = beta2;
    a.omb1 = 1.0 - beta1;
    a.omb2 = 1.0 - beta2;
    a.c1 = 1.0 - beta1_t;
    a.c2 = 1.0 - beta2_t;
    a.eps = eps;
    a.eta = eta;
    const hipStream_t st = (hipStream_t)stream;
    const hipError_t e = dtype == KANODE_F64
        ? kan::launch_adam_step<double>((double*)x, (double*)m, (double*)v, (const double*)g, n, a, st)
        : kan::launch_adam_step<float>((float*)x, (float*)m, (float*)v, (const float*)g, n, a, st);
    return e == hipSuccess ? KANODE_OK : KANODE_ERR_HIP;
}

}  // extern "C"

// ---- internal entry points for the integrator (kanode_solve.cpp) ----------------
kanode_status kanode_internal_fail(kanode_handle* h, kanode_status s, const std::string& msg) { return fail(h, s, msg); }
int kanode_internal_dtype(const kanode_handle* h) { return h->spec.dtype; }
int64_t kanode_internal_state_length(const kanode_handle* h) { return h->n_in; }
bool kanode_internal_square(const kanode_handle* h) { return h->n_in == h->n_out; }
void kanode_internal_hold_tables(kanode_handle* h, bool on) {
    h->hold_tables = on;
    h->built_phi = h->built_vjp = false;
}
double* kanode_internal_scratch(kanode_handle* h) { return (double*)h->slab; }
void* kanode_internal_solution_cache(kanode_handle* h) { return &h->solve_cache; }
int kanode_internal_scratch_rows(const kanode_handle*) { return kSlabBlocks; }
kanode_status kanode_internal_check(kanode_handle* h) { return check_handle(h); }
kanode_status kanode_internal_vjp_flush(kanode_handle* h, void* stream) {
    return vjp_flush(h, (hipStream_t)stream);
}
void kanode_internal_vjp_discard(kanode_handle* h) {
    h->njobs = 0;
    h->pend_valid = false;
}
// the Fisher-KPP RHS at the reference's own sizes (kan_small.hip): one workgroup per solve / adjoint
static bool fk_small_ok(const kanode_handle* h, int64_t batch) {
    return h->spec.rhs_kind == KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN && h->spec.dtype == KANODE_F64 && h->pp_on &&
           h->fused_solve && kan::fk_small_supported(h->hlc[0], h->hpc, (int)h->spec.nx, batch);
}
static kan::FkSmallArgs fk_small_args(const kanode_handle* h) {
    kan::FkSmallArgs s{};
    const double dx2 = h->spec.dx * h->spec.dx;
    s.Nx = (int)h->spec.nx;
    s.ni = h->hpc.ni;
    s.inv_w = h->hpc.inv_w;
    s.x0 = h->hpc.x0;
    s.cd = h->spec.diffusion * (-2.0 / dx2);
    s.co = h->spec.diffusion * (1.0 / dx2);
    return s;
}
bool kanode_internal_chain_tsit5_ok(const kanode_handle* h, int64_t batch) {
    if (fk_small_ok(h, batch)) return true;
    if (h->spec.rhs_kind != KANODE_RHS_CHAIN || batch < 1 || batch > kan::kChainSolveMaxBatch) return false;
    if (!h->fused_solve) return false;
    for (int l = 0; l < h->n_layers; ++l)
        if (h->kind[l] != KIND_COL) return false;
    return true;
}
int kanode_internal_fused_solve_cap(const kanode_handle* h) { return h->fused_solve_cap; }
bool kanode_internal_fk_step_ok(const kanode_handle* h) {
    return h->spec.dtype == KANODE_F64 && h->spec.rhs_kind == KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN && h->pp_on &&
           kan::fk_stage_pp_supported(h->hpc, (int)h->spec.nx) && h->fused_step;
}
bool kanode_internal_fk_loop_ok(const kanode_handle* h) { return h->fk_loop && kanode_internal_fk_step_ok(h); }
kanode_status kanode_internal_fk_step_loop(kanode_handle* h, const void* p, const kan::FkLoopArgs* la, int64_t lq,
                                           int64_t batch, void* stream) {
    const hipStream_t st = (hipStream_t)stream;
    if (table_build(h, h->built_phi)) {
        const int fn_phi = kan::PP_PHI;
        HIP_TRY(h, kan::launch_fk_pp_build(h->hpc, h->dlc, h->dpc, (const double*)p, h->dtable, &fn_phi, 1, st));
    }
    const double dx2 = h->spec.dx * h->spec.dx;
    const double cd = h->spec.diffusion * (-2.0 / dx2), co = h->spec.diffusion * (1.0 / dx2);
    HIP_TRY(h, kan::launch_fk_step_pp_loop(h->hpc, h->hlc[0], h->dlc, cd, co, (int)h->spec.nx, (const double*)p,
                                           h->dtable, *la, lq, batch, st, h->grid_ovr.rhs));
    return KANODE_OK;
}
kanode_status kanode_internal_fk_step(kanode_handle* h, const void* p, const void* u, const void* k1,
                                      void* const* kout, void* u_new, const double* a6x6, const double* e7,
                                      const double* q4x7, double abstol, double reltol, double* err_out,
                                      int64_t batch, void* stream, bool& launched, double* err_parts,
                                      int* nparts) {
    launched = false;
    if (nparts) *nparts = 0;
    if (!kanode_internal_fk_step_ok(h)) return KANODE_OK;
    const double dx2 = h->spec.dx * h->spec.dx;
    const double cd = h->spec.diffusion * (-2.0 / dx2), co = h->spec.diffusion * (1.0 / dx2);
    HIP_TRY(h, kan::launch_fk_step_pp(h->hpc, h->hlc[0], h->dlc, h->dpc, (const double*)p, h->dtable, cd, co,
                                      (int)h->spec.nx, (const double*)u, (const double*)k1, (double* const*)kout,
                                      (double*)u_new, a6x6, e7, q4x7, abstol, reltol,
                                      err_parts && nparts ? err_parts : (double*)h->slab, kSlabBlocks, err_out, batch,
                                      (hipStream_t)stream, table_build(h, h->built_phi), h->grid_ovr.rhs,
                                      err_parts && nparts ? nparts : nullptr));
    launched = true;
    return KANODE_OK;
}
int kanode_internal_max_parts() { return kSlabBlocks; }
void kanode_internal_set_err_parts(kanode_handle* h, double* parts, int* nparts) {
    h->err_parts = parts;
    h->err_nparts = nparts;
}
bool kanode_internal_pair_lazy(const kanode_handle* h) {
    return h->spec.rhs_kind == KANODE_RHS_CHAIN && surrogate_pair(h) && h->pair_vjp && h->pair_fuse;
}
kanode_status kanode_internal_chain_step(kanode_handle* h, const void* p, const void* u, const void* k1,
                                         void* const* kout, void* u_new, const double* a6x6, const double* e7,
                                         double abstol, double reltol, double* err_out, int64_t batch, void* stream,
                                         bool& launched) {
    launched = false;
    if (h->spec.rhs_kind != KANODE_RHS_CHAIN || !h->fused_step) return KANODE_OK;
    for (int l = 0; l < h->n_layers; ++l)
        if (h->kind[l] != KIND_COL) return KANODE_OK;
    kan::ChainStepArgs a{};
    for (int s = 0; s < 6; ++s)
        for (int j = 0; j < 6; ++j) a.a[s][j] = a6x6[6 * s + j];
    for (int j = 0; j < 7; ++j) a.e[j] = e7 ? e7[j] : 0.0;
    a.abstol = abstol;
    a.reltol = reltol;
    a.u = u;
    a.k1 = k1;
    for (int j = 0; j < 6; ++j) a.k[j] = kout[j];
    a.u_new = u_new;
    const hipStream_t st = (hipStream_t)stream;
    const hipError_t e =
        h->spec.dtype == KANODE_F64
            ? kan::launch_kd_chain_step<double>(h->hlc, h->n_layers, h->dlc, (const double*)p, h->P, batch, a,
                                                (double*)h->slab, kSlabBlocks, err_out, st)
            : kan::launch_kd_chain_step<float>(h->hlc, h->n_layers, h->dlc, (const float*)p, h->P, batch, a,
                                               (double*)h->slab, kSlabBlocks, err_out, st);
    if (e == hipErrorNotSupported) return KANODE_OK;
    if (e != hipSuccess) return fail(h, KANODE_ERR_HIP, std::string("launch_kd_chain_step: ") + hipGetErrorString(e));
    launched = true;
    return KANODE_OK;
}
// a whole InterpolatingAdjoint step of a small chain (kd_chain_vjp_step_kernel + its finish): km_out[0..5] <- kμ_2..kμ_7,
// *err_out <- the λ error total (with want_error); launched = false where the kernel does not cover the chain
template <typename T>
static kanode_status chain_adjoint_step_t(kanode_handle* h, const T* p, const kan::ChainAdjStep<T>& a,
                                          void* const* km_out, double* err_out, int64_t batch, hipStream_t st,
                                          bool& launched) {
    const size_t row = (size_t)h->P * sizeof(T) + sizeof(double);
    int64_t cap = (int64_t)(h->slab_bytes / row) - 1;   // the stage kernel's grid cap (launch_kd_chain_vjp_stage)
    if (cap > 1024) cap = 1024;
    if (cap < 1) return KANODE_OK;
    const size_t need = kan::chain_vjp_step_slab_bytes(h->P, batch, sizeof(T), (int)cap);
    if (h->cstep_bytes < need) {
        if (is_capturing(st)) return fail(h, KANODE_ERR_CAPTURE, "chain adjoint step slab grows during capture");
        HIP_TRY(h, hipStreamSynchronize(st));
        if (h->cstep_slab) HIP_TRY(h, hipFree(h->cstep_slab));
        h->cstep_slab = nullptr;
        h->cstep_bytes = 0;
        HIP_TRY(h, hipMalloc(&h->cstep_slab, need));
        h->cstep_bytes = need;
    }
    T* km[7];
    for (int s = 0; s < (a.fsal ? 7 : 6); ++s) km[s] = (T*)km_out[s];
    const hipError_t e = kan::launch_kd_chain_vjp_step<T>(h->hlc, h->n_layers, h->dlc, p, h->P, batch, a, (int)cap,
                                                          h->cstep_slab, h->cstep_bytes, km, err_out, st);
    if (e == hipErrorNotSupported) return KANODE_OK;
    if (e != hipSuccess) return fail(h, KANODE_ERR_HIP, std::string("launch_kd_chain_vjp_step: ") + hipGetErrorString(e));
    launched = true;
    return KANODE_OK;
}
bool kanode_internal_chain_adjoint_step_ok(const kanode_handle* h) {
    if (h->spec.rhs_kind != KANODE_RHS_CHAIN || !h->fused_step) return false;
    for (int l = 0; l < h->n_layers; ++l)
        if (h->kind[l] != KIND_COL) return false;
    const size_t esize = h->spec.dtype == KANODE_F64 ? sizeof(double) : sizeof(float);
    if ((int64_t)(h->slab_bytes / ((size_t)h->P * esize + sizeof(double))) - 1 < 1) return false;
    return kan::chain_vjp_step_supported(h->hlc, h->n_layers, h->P, esize);
}
kanode_status kanode_internal_chain_adjoint_step(kanode_handle* h, const void* p, const void* args, void* const* km_out,
                                                 double* err_out, int64_t batch, void* stream, bool& launched) {
    launched = false;
    if (!kanode_internal_chain_adjoint_step_ok(h)) return KANODE_OK;
    const hipStream_t st = (hipStream_t)stream;
    return h->spec.dtype == KANODE_F64
               ? chain_adjoint_step_t<double>(h, (const double*)p, *(const kan::ChainAdjStep<double>*)args, km_out,
                                              err_out, batch, st, launched)
               : chain_adjoint_step_t<float>(h, (const float*)p, *(const kan::ChainAdjStep<float>*)args, km_out,
                                             err_out, batch, st, launched);
}
kanode_status kanode_internal_fk_adjoint_loop_geometry(kanode_handle* h, int64_t batch, void* stream, bool& ok,
                                                      double** slab, int64_t* grid) {
    ok = false;
    const int P = h->hlc[0].G + (h->hlc[0].use_base ? 1 : 0);
    if (!h->fk_loop || h->spec.dtype != KANODE_F64 || h->spec.rhs_kind != KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN ||
        !h->pp_on || !h->fused_step || !kan::fk_adjoint_loop_supported(h->hpc, h->hlc[0], (int)h->spec.nx) ||
        h->grid_ovr.vstep != 0 || !h->grid_ovr.vstep_rows || h->adj_fused_finish || P > KANODE_MAX_GRID + 1 ||
        kan::fk_adjoint_loop_grid(batch, kSlabBlocks / 2) < 1)
        return KANODE_OK;
    if (kanode_status s = ensure_adjoint_slabs(h, (hipStream_t)stream); s != KANODE_OK) return s;
    *slab = (double*)h->step_slab;
    *grid = kan::fk_adjoint_loop_grid(batch, kSlabBlocks / 2);
    ok = true;
    return KANODE_OK;
}
kanode_status kanode_internal_fk_adjoint_loop(kanode_handle* h, const void* p, const kan::AdjLoopArgs* la,
                                              int64_t batch, void* stream) {
    const double dx2 = h->spec.dx * h->spec.dx;
    const double cd = h->spec.diffusion * (-2.0 / dx2), co = h->spec.diffusion * (1.0 / dx2);
    HIP_TRY(h, kan::launch_fk_adjoint_loop(h->hpc, h->hlc[0], h->dlc, h->dpc, (const double*)p, h->dtable, cd, co,
                                           (int)h->spec.nx, *la, batch, (hipStream_t)stream,
                                           table_build(h, h->built_vjp)));
    return KANODE_OK;
}
kanode_status kanode_internal_fk_adjoint_step(kanode_handle* h, const void* p, kan::AdjStepArgs* a, void* const* km,
                                              double* err_out, int64_t batch, void* stream, bool& launched,
                                              bool* combined, const AdjMuUpdate* mu, const AdjAdaptiveFinish* af) {
    launched = false;
    if (combined) *combined = false;
    if (af) *af->done = false;
    if (h->spec.dtype != KANODE_F64 || h->spec.rhs_kind != KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN || !h->pp_on ||
        !kan::fk_vjp_pp_supported(h->hlc[0], (int)h->spec.nx) || !h->fused_step)
        return KANODE_OK;
    const hipStream_t st = (hipStream_t)stream;
    const int P = h->hlc[0].G + (h->hlc[0].use_base ? 1 : 0);
    if (kanode_status s = ensure_adjoint_slabs(h, st); s != KANODE_OK) return s;
    const double dx2 = h->spec.dx * h->spec.dx;
    const double cd = h->spec.diffusion * (-2.0 / dx2), co = h->spec.diffusion * (1.0 / dx2);
    a->err_slab = err_out ? (double*)h->step_slab : nullptr;   // relocated by the launcher
    int grid = 0, comb = 0;
    a->combine = err_out && af ? 2 : (combined != nullptr && err_out == nullptr ? 1 : 0);
    a->fin_ctr = nullptr;
    if (err_out && af && h->adj_fused_finish) {   // the finish inside the rows kernel (the launcher may decline)
        a->fin_ctr = h->fin_ctr;
        a->fin = kan::AdjFinish{};
        a->fin.a0 = af->a6[0];
        a->fin.e0 = af->bt[0];
        a->fin.abstol = af->abstol;
        a->fin.reltol = af->reltol;
        a->fin.mu = af->mu;
        a->fin.mu_new = af->mu_new;
        a->fin.km1 = af->km1;
        a->fin.km7 = af->km7;
        a->fin.out = af->out;
        // the arrival counters re-zeroed on the stream before every fused launch: a wait that timed
        // out in an earlier launch cannot leave them off by one for this one
        HIP_TRY(h, hipMemsetAsync(h->fin_ctr, 0, 2 * sizeof(unsigned), st));
    }
    bool fused_fin = false;
    HIP_TRY(h, kan::launch_fk_vjp_step_pp(h->hpc, h->hlc[0], h->dlc, h->dpc, (const double*)p, h->dtable, cd, co,
                                          (int)h->spec.nx, *a, (double*)h->step_slab, kSlabBlocks / 2, batch, &grid, st,
                                          table_build(h, h->built_vjp), h->grid_ovr.vstep,
                                          h->grid_ovr.vstep_rows, &comb, &fused_fin));
    if (fused_fin) {   // μ_new, kμ_7 and the error terms are written by the step kernel itself
        *af->done = true;
        launched = true;
        return KANODE_OK;
    }
    kan::FinishJobs jobs{};
    double* base = (double*)h->step_slab;
    if (comb == 1) {
        // km[0] <- Σ_{s<5} h·a6_{s+1}·kμ_{s+2} (the kernel's combined rows), km[5] <- kμ_7
        for (int q = 0; q < 2; ++q) {
            const int s = q == 0 ? 0 : 5;
            kan::FinishJob& jb = jobs.j[q];
            jb.slab = base + (int64_t)s * grid * P;
            jb.dp = (double*)km[s];
            jb.nblk = grid;
            jb.assign = 1;
            jb.tr = 1;   // the rows kernel stores combined rows parameter-major
            if (q == 0 && mu) {   // μ_new = μ + a61·kμ_1 + A in the same launch (A itself is not stored)
                jb.dp = mu->mu_new;
                jb.base = mu->mu;
                jb.other = mu->km1;
                jb.coef = mu->a61;
            }
        }
        HIP_TRY(h, kan::launch_vjp_finish_jobs(jobs, 2, P, st));
        *combined = true;
        launched = true;
        return KANODE_OK;
    }
    if (err_out && af) {
        // adaptive step: the six stage sums, μ_new = μ + Σ h a6_j kμ_j, kμ_7 and the μ error terms in one
        // launch (slab s holds kμ_{s+2})
        kan::AdjFinish f{};
        if (comb == 2) {
            // the rows kernel reduced A = Σ_{s<5} h a6_{s+1} kμ_{s+2} (slab 0), E = Σ_s h b̃_{s+1} kμ_{s+2}
            // (slab 1) and kμ_7 (slab 5) instead of the six stage sums
            const int which[3] = {0, 1, 5};
            for (int q = 0; q < 3; ++q) {
                f.slab[q] = base + (int64_t)which[q] * grid * P;
                f.ca[q] = q == 0 ? 1.0 : 0.0;
                f.ce[q] = q == 1 ? 1.0 : 0.0;
            }
            f.nslab = 3;
            f.k7 = 2;
            f.tr = 1;   // the rows kernel stores the combined rows parameter-major
        } else {
            for (int s = 0; s < 6; ++s) {
                f.slab[s] = base + (int64_t)s * grid * P;
                f.ca[s] = s < 5 ? af->a6[s + 1] : 0.0;
                f.ce[s] = af->bt[s + 1];
            }
            f.nslab = 6;
            f.k7 = 5;
        }
        f.nblk = grid;
        f.a0 = af->a6[0];
        f.e0 = af->bt[0];
        f.abstol = af->abstol;
        f.reltol = af->reltol;
        f.mu = af->mu;
        f.mu_new = af->mu_new;
        f.km1 = af->km1;
        f.km7 = af->km7;
        f.err_slab = base + (int64_t)6 * grid * P;
        f.out = af->out;
        HIP_TRY(h, kan::launch_adj_finish(f, P, st));
        *af->done = true;
        launched = true;
        return KANODE_OK;
    }
    for (int s = 0; s < 6; ++s) {
        kan::FinishJob& jb = jobs.j[s];
        jb.slab = base + (int64_t)s * grid * P;
        jb.dp = (double*)km[s];
        jb.nblk = grid;
        jb.assign = 1;
        if (s == 5 && err_out) {
            jb.err_slab = base + (int64_t)6 * grid * P;
            jb.err_out = err_out;
        }
    }
    HIP_TRY(h, kan::launch_vjp_finish_jobs(jobs, 6, P, st));
    launched = true;
    return KANODE_OK;
}
kanode_status kanode_internal_chain_adjoint(kanode_handle* h, const void* p, int64_t batch,
                                            const kan::ChainAdjointArgs* a, void* stream, bool& launched) {
    launched = false;
    const hipStream_t st = (hipStream_t)stream;
    if (fk_small_ok(h, batch)) {
        const int fns[2] = {kan::PP_DPHI, kan::PP_SWISH};
        if (table_build(h, h->built_vjp))
            HIP_TRY(h, kan::launch_fk_pp_build(h->hpc, h->dlc, h->dpc, (const double*)p, h->dtable, fns, 2, st));
        const hipError_t e = kan::launch_fk_small_adjoint(h->hlc[0], h->hpc, h->dlc, (const double*)p, h->dtable,
                                                          fk_small_args(h), batch, *a, st);
        if (e == hipErrorNotSupported) return KANODE_OK;
        if (e != hipSuccess) return fail(h, KANODE_ERR_HIP, std::string("launch_fk_small_adjoint: ") + hipGetErrorString(e));
        launched = true;
        return KANODE_OK;
    }
    const hipError_t e =
        h->spec.dtype == KANODE_F64
            ? kan::launch_kd_chain_adjoint<double>(h->hlc, h->n_layers, h->dlc, (const double*)p, h->P, batch, *a, st,
                                                   h->chain_wide)
            : kan::launch_kd_chain_adjoint<float>(h->hlc, h->n_layers, h->dlc, (const float*)p, h->P, batch, *a, st,
                                                  h->chain_wide);
    if (e == hipErrorNotSupported) return KANODE_OK;
    if (e != hipSuccess) return fail(h, KANODE_ERR_HIP, std::string("launch_kd_chain_adjoint: ") + hipGetErrorString(e));
    launched = true;
    return KANODE_OK;
}
bool kanode_internal_pair_persist_ok(const kanode_handle* h) {
    return h->pair_persist && h->spec.dtype == KANODE_F64 && h->spec.rhs_kind == KANODE_RHS_CHAIN && surrogate_pair(h);
}
int64_t kanode_internal_param_length(const kanode_handle* h) { return h->P; }
kanode_status kanode_internal_pair_adjoint(kanode_handle* h, const void* p, int64_t batch, kan::PairAdjArgs* a,
                                           void* stream, bool& launched) {
    launched = false;
    if (!kanode_internal_pair_persist_ok(h)) return KANODE_OK;
    a->S = h->pair_persist_s;
    a->P = h->P;
    a->max_wg = h->pair_persist_max_wg;
    a->force_abort = h->pair_persist_abort ? 1 : 0;
    const hipError_t e = kan::launch_kd_pair_adjoint(h->hlc, h->dlc, (const double*)p, batch, *a, (hipStream_t)stream);
    if (e == hipErrorNotSupported) return KANODE_OK;
    if (e != hipSuccess) return fail(h, KANODE_ERR_HIP, std::string("launch_kd_pair_adjoint: ") + hipGetErrorString(e));
    launched = true;
    return KANODE_OK;
}
void kanode_internal_set_last_adjoint(kanode_handle* h, int path) { h->last_adjoint = path; }

void kanode_internal_clear_adjoint_steps(kanode_handle* h) { h->adj_steps.clear(); }
std::vector<double>* kanode_internal_adjoint_steps(kanode_handle* h) {
    return h->record_adj_steps ? &h->adj_steps : nullptr;
}

extern "C" kanode_status kanode_table_rejections(kanode_handle* h, int32_t out[3]) {
    if (!h || !out) return KANODE_ERR_INVALID_ARG;
    if (!h->dtable || !h->pp_on) return fail(h, KANODE_ERR_UNSUPPORTED, "no pointwise table on this handle");
    const int ni = h->hpc.ni, nb = ni / kan::kPPPerBlock;
    const int64_t off = (int64_t)kan::kPPMaxFns * kan::kPPCoef * ni;
    std::vector<double> st((size_t)kan::kPPMaxFns * nb * kan::kPPStampStride);
    HIP_TRY(h, hipDeviceSynchronize());
    HIP_TRY(h, hipMemcpy(st.data(), h->dtable + off, st.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (int f = 0; f < kan::kPPMaxFns; ++f) {
        int32_t n = 0;
        bool built = true;
        for (int b = 0; b < nb; ++b) {
            const double* sp = st.data() + ((size_t)f * nb + b) * kan::kPPStampStride;
            if (sp[kan::kPPStampValid] != 1.0) built = false;
            else n += (int32_t)sp[kan::kPPStampRejected];
        }
        out[f] = built ? n : -1;
    }
    return KANODE_OK;
}
extern "C" int64_t kanode_adjoint_step_sizes(const kanode_handle* h, double* out, int64_t cap) {
    if (!h) return -1;
    const int64_t n = (int64_t)h->adj_steps.size();
    if (out && cap > 0) std::memcpy(out, h->adj_steps.data(), (size_t)std::min(n, cap) * sizeof(double));
    return n;
}
int kanode_internal_pair_adjoint_workgroups(const kanode_handle* h, int64_t batch) {
    return kan::pair_adjoint_workgroups(h->hlc, batch, h->pair_persist_s);
}
// forward sensitivities of a small Fisher-KPP field (kan_small.hip fk_small_fsens_kernel)
bool kanode_internal_fsens_ok(const kanode_handle* h, int64_t batch) {
    return h->spec.rhs_kind == KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN && h->spec.dtype == KANODE_F64 &&
           kan::fk_small_fsens_supported(h->hlc[0], (int)h->spec.nx, batch);
}
kanode_status kanode_internal_fk_fsens(kanode_handle* h, const void* p, const void* u0, int64_t batch,
                                       const kan::ChainSolveArgs* a, void* s_save, void* stream) {
    const hipStream_t st = (hipStream_t)stream;
    const bool tab = h->pp_on && h->hpc.enabled;
    if (tab) {
        const int fns[3] = {kan::PP_PHI, kan::PP_DPHI, kan::PP_SWISH};
        HIP_TRY(h, kan::launch_fk_pp_build(h->hpc, h->dlc, h->dpc, (const double*)p, h->dtable, fns, 3, st));
    }
    const hipError_t e = kan::launch_fk_small_fsens(h->hlc[0], h->hpc, tab, h->dlc, (const double*)p,
                                                    tab ? h->dtable : nullptr, fk_small_args(h), (const double*)u0,
                                                    batch, *a, (double*)s_save, st);
    if (e == hipErrorNotSupported)
        return fail(h, KANODE_ERR_UNSUPPORTED, "forward sensitivities: shape not covered by the one-workgroup kernel");
    if (e != hipSuccess) return fail(h, KANODE_ERR_HIP, std::string("launch_fk_small_fsens: ") + hipGetErrorString(e));
    return KANODE_OK;
}
kanode_status kanode_internal_chain_tsit5(kanode_handle* h, const void* p, const void* u0, int64_t batch,
                                          const kan::ChainSolveArgs* a, void* stream, bool& launched) {
    launched = false;
    const hipStream_t st = (hipStream_t)stream;
    if (fk_small_ok(h, batch)) {
        const int fn = kan::PP_PHI;
        if (table_build(h, h->built_phi))
            HIP_TRY(h, kan::launch_fk_pp_build(h->hpc, h->dlc, h->dpc, (const double*)p, h->dtable, &fn, 1, st));
        const hipError_t e = kan::launch_fk_small_tsit5(h->hlc[0], h->hpc, h->dlc, (const double*)p, h->dtable,
                                                        fk_small_args(h), (const double*)u0, batch, *a, st);
        if (e == hipErrorNotSupported) return KANODE_OK;
        if (e != hipSuccess) return fail(h, KANODE_ERR_HIP, std::string("launch_fk_small_tsit5: ") + hipGetErrorString(e));
        launched = true;
        return KANODE_OK;
    }
    const hipError_t e =
        h->spec.dtype == KANODE_F64
            ? kan::launch_kd_chain_tsit5<double>(h->hlc, h->n_layers, h->dlc, (const double*)p, h->P,
                                                 (const double*)u0, batch, *a, st)
            : kan::launch_kd_chain_tsit5<float>(h->hlc, h->n_layers, h->dlc, (const float*)p, h->P, (const float*)u0,
                                                batch, *a, st);
    if (e == hipErrorNotSupported) return KANODE_OK;
    if (e != hipSuccess) return fail(h, KANODE_ERR_HIP, std::string("launch_kd_chain_tsit5: ") + hipGetErrorString(e));
    launched = true;
    return KANODE_OK;
}
kanode_status kanode_internal_vjp_stage(kanode_handle* h, const void* p, const void* u, const kanode_stage* state,
                                        const void* lam, const kanode_stage* adj, void* lamJ, void* dp, bool dp_assign,
                                        int64_t batch, void* stream, const double* su_scale, const double* sl_scale,
                                        bool defer) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if (!p || !u || !lam || !state || !adj || batch < 1) return fail(h, KANODE_ERR_INVALID_ARG, "null argument or batch < 1");
    hipStream_t st = (hipStream_t)stream;
    if (h->spec.dtype == KANODE_F64)
        return vjp_stage_t<double>(h, (const double*)p, (const double*)u, state, (const double*)lam, adj, (double*)lamJ,
                                   (double*)dp, batch, st, dp_assign, su_scale, sl_scale, defer);
    return vjp_stage_t<float>(h, (const float*)p, (const float*)u, state, (const float*)lam, adj, (float*)lamJ,
                              (float*)dp, batch, st, dp_assign, su_scale, sl_scale);
}

kanode_status kanode_internal_rhs_stage(kanode_handle* h, const void* p, const void* u, const kanode_stage* sg,
                                        void* du, int64_t batch, void* stream, const double* cscale,
                                        const int32_t* skip) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if (!p || !u || !du || !sg || batch < 1) return fail(h, KANODE_ERR_INVALID_ARG, "null argument or batch < 1");
    hipStream_t st = (hipStream_t)stream;
    if (h->spec.dtype == KANODE_F64)
        return stage_t<double>(h, (const double*)p, (const double*)u, sg, (double*)du, batch, st, cscale, skip);
    return stage_t<float>(h, (const float*)p, (const float*)u, sg, (float*)du, batch, st, cscale, skip);
}

// every workspace a stage / adjoint-stage call of this batch may need, allocated now
// (so the calls can be captured into a hipGraph)
kanode_status kanode_internal_prepare(kanode_handle* h, int64_t batch, hipStream_t st) {
    kanode_status s = check_handle(h);
    if (s != KANODE_OK) return s;
    if ((s = ensure_ws(h, batch, st)) != KANODE_OK) return s;
    if (h->spec.rhs_kind == KANODE_RHS_POINTWISE_PERIODIC_LAPLACIAN && h->ws_bytes < (size_t)(h->spec.nx * batch) * h->esize) {
        HIP_TRY(h, hipStreamSynchronize(st));
        if (h->ws) HIP_TRY(h, hipFree(h->ws));
        HIP_TRY(h, hipMalloc(&h->ws, (size_t)(h->spec.nx * batch) * h->esize));
        h->ws_bytes = (size_t)(h->spec.nx * batch) * h->esize;
    }
    return ensure_stage_ws(h, 2 * (size_t)(h->n_in * batch) * h->esize, st);
}
