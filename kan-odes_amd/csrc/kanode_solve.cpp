// kanode_solve.cpp — the Tsit5 integrator and the InterpolatingAdjoint around the HIP
// RHS / VJP (include/kanode.h: kanode_solve_tsit5, kanode_adjoint_tsit5).
//
// A native host loop: every Runge-Kutta stage is one kanode_rhs_stage (the stage
// combination u + dt·Σ a_sj k_j is formed inside the RHS kernel, the last stage also
// writes u_new and the embedded-error sum of squares), every adjoint stage one
// kanode_vjp_stage.  The only device->host traffic is the 8-byte error norm of an
// adaptive step (the accept/reject decision); a fixed-step solve never synchronises.
// The step sequence, controller and saveat handling restate OrdinaryDiffEqTsit5 1.1.0 /
// OrdinaryDiffEq 6.89 and SciMLSensitivity 7.69 (third-party, pinned in
// Lotka-Volterra/Manifest.toml; the Python driver kanode/ode.py + kanode/adjoint.py is
// the same algorithm statement and the parity reference of the tests).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <string>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <type_traits>
#include <vector>

#include "kan_adjloop.hpp"
#include "kan_kernels.hpp"
#include "kanode.h"
#include "kanode_internal.hpp"

namespace {

// Tsitouras 5(4) (OrdinaryDiffEq tsit_tableaus.jl)
constexpr double TC[6] = {0.161, 0.327, 0.9, 0.9800255409045097, 1.0, 1.0};
constexpr double TA[6][6] = {
    {0.161, 0, 0, 0, 0, 0},
    {-0.008480655492356989, 0.335480655492357, 0, 0, 0, 0},
    {2.897153057105493, -6.359448489975075, 4.3622954328695815, 0, 0, 0},
    {5.325864828439257, -11.748883564062828, 7.4955393428898365, -0.09249506636175525, 0, 0},
    {5.86145544294642, -12.92096931784711, 8.159367898576159, -0.071584973281401, -0.028269050394068383, 0},
    {0.09646076681806523, 0.01, 0.4798896504144996, 1.379008574103742, -3.290069515436081, 2.324710524099774},
};
constexpr double BT[7] = {-0.00178001105222577714, -0.0008164344596567469, 0.007880878010261995,
                          -0.1447110071732629,     0.5823571654525552,     -0.45808210592918697,
                          0.015151515151515152};
// dense output b_i(θ) = Σ_m RI[i][m] θ^(m+1)  (Tsit5Interp)
constexpr double RI[7][4] = {
    {1.0, -2.763706197274826, 2.9132554618219126, -1.0530884977290216},
    {0.0, 0.13169999999999998, -0.2234, 0.1017},
    {0.0, 3.9302962368947516, -5.941033872131505, 2.490627285651253},
    {0.0, -12.411077166933676, 30.33818863028232, -16.548102889244902},
    {0.0, 37.50931341651104, -88.1789048947664, 47.37952196281928},
    {0.0, -27.896526289197286, 65.09189467479366, -34.87065786149661},
    {0.0, 1.5, -4.0, 2.5},
};

void interp_weights(double theta, double w[7]) {
    for (int i = 0; i < 7; ++i) {
        double s = 0.0;
        for (int m = 0; m < 4; ++m) s += RI[i][m] * std::pow(theta, (double)(m + 1));
        w[i] = s;
    }
}

kanode_solver_options resolved(const kanode_solver_options* o) {
    kanode_solver_options d;
    kanode_solver_options_default(&d);
    return o ? *o : d;
}

}  // namespace

extern "C" void kanode_solver_options_default(kanode_solver_options* o) {
    if (!o) return;
    o->abstol = 1e-6;
    o->reltol = 1e-3;
    o->dt = 0.0;
    o->adaptive = 1;
    o->maxiters = 100000;
    o->dtmin = 0.0;
    o->beta1 = 7.0 / 50.0;
    o->beta2 = 2.0 / 25.0;
    o->gamma = 0.9;
    o->qmin = 0.2;
    o->qmax = 10.0;
    o->qoldinit = 1e-4;
    o->control = 0;
    o->graph_steps = 16;
}

// Dense output: step n keeps u_n and k_2..k_7 in slot n (7 states); k_1 of step n is
// k_7 of step n-1 (FSAL), k_1 of step 0 has its own buffer.  Without recording only
// two slots are used, alternately.
// device / pinned scalar slots of a solution: 8 norm totals, then an adaptive adjoint step's finish
// terms at 8 (the FK step: 1 + P <= 34) or its <= kAdjFinishBlocks partials at 16
constexpr int kScalars = 16 + kan::kAdjFinishBlocks + 16;

struct kanode_solution {
    kanode_handle* h = nullptr;
    int dtype = 0;
    size_t esize = 8;
    int64_t n = 0;                   // elements of one state (N·B)
    int64_t batch = 0;
    double t0 = 0, tf = 0;
    std::vector<double> saveat;
    std::vector<double> ts, dts;     // accepted steps: start time, step
    std::vector<void*> slots;
    bool slots_borrowed = false;     // slots point into fused.block (one-workgroup solve), not owned
    bool qform = false;              // slots hold u_n, Q_1..Q_4, k_7 (fk_step_pp_wave_kernel) instead of u_n, k_2..k_7
    void* k1_0 = nullptr;
    bool record = true;
    // one-workgroup small-chain solve (kd_chain_tsit5_kernel): contiguous dense output and the
    // device copies of saveat, step times and the result block
    struct Fused {
        void* block = nullptr;
        int64_t cap = 0;                   // steps the block holds
        double* saveat = nullptr;
        int64_t saveat_cap = 0;
        double* ts = nullptr;              // [cap] then dts [cap]
        int64_t ts_cap = 0;
        double* hts = nullptr;             // pinned host staging of ts | dts (mapped, coherent)
        double* mts = nullptr;             // its device address (null: copied)
        int64_t hts_cap = 0;
        int64_t* out = nullptr;            // naccept, nreject, nf, status
        void* adj_meta = nullptr;          // adjoint: stops, jump rows and offsets
        size_t adj_meta_bytes = 0;
        void* hup = nullptr;               // pinned staging of the small uploads (staged_upload)
        size_t hup_bytes = 0;
        hipEvent_t hup_ev = nullptr;       // recorded after the last upload from hup
        bool hup_pending = false;
        // the bytes last uploaded into saveat / adj_meta: a training loop passes the same saveat and stops every
        // iteration, and an unchanged upload is skipped (each one is a copy launch on the stream's critical path)
        std::vector<char> saveat_last, meta_last;
    } fused;
    double* dscal = nullptr;         // device scalars (norm totals; an adaptive FK adjoint step's 1 + P terms)
    double* hscal = nullptr;         // pinned host mirror (mapped, coherent)
    // device address of hscal: the host-controlled adaptive loops have their step-control scalars written
    // there by the producing kernels, so reading them costs a stream synchronisation and no copy launch
    // (a D2H hipMemcpyAsync of 8 bytes ran as a ~4.4 us blit kernel, twice per FK training step).
    // nullptr if the runtime gave no device address: those loops then copy from dscal as before.
    double* mscal = nullptr;
    // mapped, coherent pinned host memory for a step's per-block error partials (the FK step path: the
    // host sums them, so no final-reduction launch per adaptive step); hparts / its device address
    double* hparts = nullptr;
    double* mparts = nullptr;
    // a call on this solution failed: its kernels may still be in flight and its mapped step-control slots
    // may hold written values; the next call drains the stream and re-arms every slot first (ctl_begin)
    bool ctl_dirty = false;
    // the persistent pair adjoint's device buffer: [arrival counter, abort word][slot table | ts | dts][exchange slots]
    void* padj = nullptr;
    size_t padj_bytes = 0;
    double* hs_dev = nullptr;        // KANODE_OPT_RECORD_ADJOINT_STEPS: the one-launch adjoints' step sizes
    int64_t hs_cap = 0;
    // the device-controlled Fisher-KPP solve (solve_fk_loop): its state and host mirror, the error partials,
    // the device copy of the slot table (staged through pinned memory) and the step records
    struct Loop {
        kan::FkLoopCtl* ctl = nullptr;     // [2]
        kan::FkLoopCtl* hmir = nullptr;    // pinned, mapped
        kan::FkLoopCtl* dmir = nullptr;    // its device address
        double* parts = nullptr;
        void** dslots = nullptr;
        void** hslots = nullptr;           // pinned
        double* ts = nullptr;              // [cap] then dts [cap]
        int64_t cap = 0, synced = 0;
    } loop;
    // the device-controlled Fisher-KPP adjoint (adjoint_fk_loop): state, mirror, plans, host staging, tables
    struct AdjLoop {
        kan::AdjLoopCtl* ctl = nullptr;
        kan::AdjLoopCtl* hmir = nullptr;   // pinned, mapped
        kan::AdjLoopCtl* dmir = nullptr;
        kan::AdjLoopPlan* plan = nullptr;  // [2]
        void* hplan = nullptr;             // pinned staging: a plan and a state
        unsigned* arrive = nullptr;
        void* meta = nullptr;
        size_t meta_bytes = 0;
    } aloop;
    // adjoint scratch (sized on first use)
    void* adj = nullptr;
    size_t adj_bytes = 0;
    // device step control (graph mode): U, K_1..K_7, U_new; control blocks; saveat staging;
    // the dense-output slot table and step times as the device writes them; the cached graph
    struct Graph {
        void* bufs = nullptr;
        size_t bufs_bytes = 0;
        kan::SolveCtl* ctl = nullptr;      // [2], parity-buffered
        kan::SolveCtl* hctl = nullptr;     // pinned mirror
        double* saveat = nullptr;
        int64_t saveat_cap = 0;
        void* save = nullptr;
        size_t save_bytes = 0;
        void** slots = nullptr;            // device copy of the slot pointers
        double* ts = nullptr;
        double* dts = nullptr;
        int64_t cap = 0;                   // capacity of slots / ts / dts
        int64_t slots_synced = 0;
        hipStream_t cap_stream = nullptr;
        hipGraphExec_t exec = nullptr;
        // what the graph baked in
        const void* key_p = nullptr;
        int64_t key_nsave = -1, key_cap = -1;
        int key_record = -1, key_steps = -1;
        double key_tf = 0;
        kanode_solver_options key_opt{};
    } g;

    ~kanode_solution() {
        if (!slots_borrowed)
            for (void* s : slots) (void)hipFree(s);
        for (void* q : {fused.block, (void*)fused.saveat, (void*)fused.ts, (void*)fused.out, fused.adj_meta})
            if (q) (void)hipFree(q);
        if (k1_0) (void)hipFree(k1_0);
        if (dscal) (void)hipFree(dscal);
        if (hscal) (void)hipHostFree(hscal);
        if (hparts) (void)hipHostFree(hparts);
        if (adj) (void)hipFree(adj);
        if (padj) (void)hipFree(padj);
        if (hs_dev) (void)hipFree(hs_dev);
        if (fused.hts) (void)hipHostFree(fused.hts);
        if (fused.hup_ev) {
            if (fused.hup_pending) (void)hipEventSynchronize(fused.hup_ev);
            (void)hipEventDestroy(fused.hup_ev);
        }
        if (fused.hup) (void)hipHostFree(fused.hup);
        for (void* q : {(void*)loop.ctl, (void*)loop.parts, (void*)loop.dslots, (void*)loop.ts})
            if (q) (void)hipFree(q);
        for (void* q : {(void*)loop.hmir, (void*)loop.hslots})
            if (q) (void)hipHostFree(q);
        for (void* q : {(void*)aloop.ctl, (void*)aloop.plan, (void*)aloop.arrive, aloop.meta})
            if (q) (void)hipFree(q);
        for (void* q : {(void*)aloop.hmir, aloop.hplan})
            if (q) (void)hipHostFree(q);
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
        if (g.cap_stream) (void)hipStreamDestroy(g.cap_stream);
        for (void* p : {(void*)g.bufs, (void*)g.ctl, (void*)g.saveat, g.save, (void*)g.slots, (void*)g.ts, (void*)g.dts})
            if (p) (void)hipFree(p);
        if (g.hctl) (void)hipHostFree(g.hctl);
    }
    size_t state_bytes() const { return (size_t)n * esize; }
    char* slot(int64_t i) const { return (char*)slots[record ? i : (i & 1)]; }
    void* u(int64_t i) const { return slot(i); }
    // stage vector k_j (j = 1..7) of step i
    void* k(int64_t i, int j) const {
        if (j == 1) return i == 0 ? k1_0 : k(i - 1, 7);
        if (qform && j == 7) return slot(i) + 5 * state_bytes();
        return slot(i) + (size_t)(j - 1) * state_bytes();
    }
    // interpolation polynomial Q_m (m = 1..4) of step i (qform): u(t_i + θ dt_i) = u_i + Σ_m θ^m Q_m
    void* q(int64_t i, int m) const { return slot(i) + (size_t)m * state_bytes(); }
};

extern "C" void kanode_solution_free(kanode_solution* s) { delete s; }
extern "C" int64_t kanode_solution_steps(const kanode_solution* s) { return s ? (int64_t)s->ts.size() : -1; }
extern "C" int64_t kanode_solution_step_sizes(const kanode_solution* s, double* ts, double* dts, int64_t cap) {
    if (!s) return -1;
    const int64_t n = (int64_t)s->ts.size(), m = std::max<int64_t>(0, std::min(n, cap));
    if (ts && m) std::memcpy(ts, s->ts.data(), (size_t)m * sizeof(double));
    if (dts && m) std::memcpy(dts, s->dts.data(), (size_t)m * sizeof(double));
    return n;
}

namespace {

#define SOLVE_HIP(h, expr)                                                                                    \
    do {                                                                                                      \
        hipError_t e_ = (expr);                                                                               \
        if (e_ != hipSuccess)                                                                                 \
            return kanode_internal_fail((h), KANODE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define SOLVE_TRY(expr)                            \
    do {                                           \
        kanode_status s_ = (expr);                 \
        if (s_ != KANODE_OK) return s_;            \
    } while (0)

bool capturing(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive;
}

// slots [0, need) exist (allocating — not allowed during capture)
kanode_status ensure_slots(kanode_handle* h, kanode_solution* s, int64_t need, hipStream_t st) {
    if (s->slots_borrowed) {   // the previous solve used the fused block: start a slot list of our own
        s->slots.clear();
        s->slots_borrowed = false;
    }
    if (!s->record) need = std::min<int64_t>(need, 2);
    if ((int64_t)s->slots.size() >= need) return KANODE_OK;
    if (capturing(st)) return kanode_internal_fail(h, KANODE_ERR_CAPTURE, "dense-output storage grows during capture");
    while ((int64_t)s->slots.size() < need) {
        void* p = nullptr;
        if (hipMalloc(&p, 7 * s->state_bytes()) != hipSuccess) {
            (void)hipGetLastError();
            return kanode_internal_fail(h, KANODE_ERR_ALLOC, "dense output: out of device memory at step " +
                                                                 std::to_string(s->slots.size()));
        }
        s->slots.push_back(p);
    }
    return KANODE_OK;
}

// Σ over n entries of ((Σ_j ec_j k_j + ec_last·du) / (abstol + reltol·max(|u|,|y|)))² -> dst (device)
template <typename T>
kanode_status wsumsq(kanode_handle* h, const void* u, const void* y, int nk, const void* const* k, const double* ec,
                     const void* du, double abstol, double reltol, int64_t n, double* dst, hipStream_t st) {
    kan::StageArgs<T> sa{};
    sa.nk = nk;
    for (int j = 0; j < nk; ++j) sa.k[j] = (const T*)k[j];
    for (int j = 0; j <= nk; ++j) sa.ec[j] = ec[j];
    sa.abstol = abstol;
    sa.reltol = reltol;
    SOLVE_HIP(h, kan::launch_stage_error<T>((const T*)u, (const T*)y, (const T*)du, sa, kanode_internal_scratch(h),
                                            kanode_internal_scratch_rows(h), dst, n, st));
    return KANODE_OK;
}

// y = u + Σ_j c_j k_j over n entries (y may alias u)
template <typename T>
kanode_status lincomb(kanode_handle* h, const void* u, int nk, const void* const* k, const double* c, void* y,
                      int64_t n, hipStream_t st) {
    kan::StageArgs<T> sa{};
    sa.nk = nk;
    for (int j = 0; j < nk; ++j) {
        sa.k[j] = (const T*)k[j];
        sa.c[j] = c[j];
    }
    SOLVE_HIP(h, kan::launch_stage_lincomb<T>((const T*)u, sa, (T*)y, n, st));
    return KANODE_OK;
}

kanode_status read_scalars(kanode_handle* h, kanode_solution* s, int cnt, hipStream_t st) {
    if (capturing(st)) return kanode_internal_fail(h, KANODE_ERR_CAPTURE, "adaptive step control reads the error norm");
    SOLVE_HIP(h, hipMemcpyAsync(s->hscal, s->dscal, cnt * sizeof(double), hipMemcpyDeviceToHost, st));
    SOLVE_HIP(h, hipStreamSynchronize(st));
    return KANODE_OK;
}

// Step-control scalars of the host-controlled adaptive loops: where the producing kernels write them
// (ctl) and how the host gets slots [off, off + cnt) into hscal (read_ctl).
inline double* ctl(kanode_solution* s) { return s->mscal ? s->mscal : s->dscal; }
kanode_status read_ctl(kanode_handle* h, kanode_solution* s, int off, int cnt, hipStream_t st) {
    if (capturing(st)) return kanode_internal_fail(h, KANODE_ERR_CAPTURE, "adaptive step control reads the error norm");
    if (!s->mscal)
        SOLVE_HIP(h, hipMemcpyAsync(s->hscal + off, s->dscal + off, cnt * sizeof(double), hipMemcpyDeviceToHost, st));
    SOLVE_HIP(h, hipStreamSynchronize(st));
    return KANODE_OK;
}

// Mapped step control without a stream synchronisation: the host marks the slots a step's kernels will
// write with a NaN bit pattern no kernel produces (arm_ctl), launches, and spins until every slot has been
// written (wait_ctl).  A GPU store to coherent host memory is visible to the host within about a
// microsecond, while hipStreamSynchronize's wake-up put ~20 us between the kernel's end and the host's
// next launch (the FK adaptive epoch's kernel trace: a 24 us gap before every step kernel).  The stream
// is queried every few hundred polls: when it has drained, every slot must have been written (kernel
// completion releases the stores), otherwise the call fails instead of spinning forever.
constexpr uint64_t kCtlUnset = 0x7FF4DEADBEEF0001ull;   // a signalling-NaN payload
inline void arm_ctl(double* p, int n) {
    for (int i = 0; i < n; ++i) __atomic_store_n(reinterpret_cast<uint64_t*>(p + i), kCtlUnset, __ATOMIC_RELAXED);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
}
inline bool ctl_ready(const double* p, int n) {
    for (int i = 0; i < n; ++i)
        if (__atomic_load_n(reinterpret_cast<const uint64_t*>(p + i), __ATOMIC_ACQUIRE) == kCtlUnset) return false;
    return true;
}
struct CtlRange {
    const double* p;
    int n;
};
// spin-wait hint for the host polls of mapped control words
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#elif defined(__aarch64__)
    asm volatile("yield" ::: "memory");
#else
    std::atomic_signal_fence(std::memory_order_seq_cst);
#endif
}
kanode_status wait_ctl(kanode_handle* h, hipStream_t st, std::initializer_list<CtlRange> rs) {
    if (capturing(st)) return kanode_internal_fail(h, KANODE_ERR_CAPTURE, "adaptive step control reads the error norm");
    auto ready = [&] {
        for (const CtlRange& r : rs)
            if (!ctl_ready(r.p, r.n)) return false;
        return true;
    };
    for (uint64_t it = 1;; ++it) {
        if (ready()) return KANODE_OK;
        if ((it & 255) == 0) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess) {
                if (ready()) return KANODE_OK;
                return kanode_internal_fail(h, KANODE_ERR_HIP, "step control: the stream drained without the error terms");
            }
            if (q != hipErrorNotReady) SOLVE_HIP(h, q);
        }
        cpu_relax();
    }
}

// Before a solve / adjoint on a solution whose previous call failed: wait for that call's kernels (they may
// still write the mapped slots), then arm every partials slot again, so a polled step control never reads
// an earlier call's values.  The happy path costs nothing.
kanode_status ctl_begin(kanode_handle* h, kanode_solution* s, hipStream_t st) {
    if (!s->ctl_dirty) return KANODE_OK;
    if (!capturing(st)) SOLVE_HIP(h, hipStreamSynchronize(st));
    s->fused.saveat_last.clear();   // (an upload of the failed call may not have run)
    s->fused.meta_last.clear();
    if (s->hparts) arm_ctl(s->hparts, kanode_internal_max_parts());
    if (s->hscal) arm_ctl(s->hscal, kScalars);
    s->ctl_dirty = false;
    return KANODE_OK;
}

kanode_stage make_stage(int nk, void* const* k, const double* c) {
    kanode_stage sg{};
    sg.n_prev = nk;
    for (int j = 0; j < nk; ++j) {
        sg.k[j] = k[j];
        sg.c[j] = c[j];
    }
    return sg;
}

struct TableHold {   // p is constant for one solve: each table set is built once
    kanode_handle* h;
    explicit TableHold(kanode_handle* hh) : h(hh) { kanode_internal_hold_tables(h, true); }
    ~TableHold() { kanode_internal_hold_tables(h, false); }
};

// Hairer & Wanner initial step (OrdinaryDiffEq ode_determine_initdt, order 5); kanode/ode.py _initdt
template <typename T>
kanode_status initdt(kanode_handle* h, kanode_solution* s, const void* p, const void* u0, const void* f0,
                     double tdist, const kanode_solver_options& o, double& dt, hipStream_t st, void* tmp) {
    const double one = 1.0;
    double e1[2] = {1.0, 0.0};
    SOLVE_TRY(wsumsq<T>(h, u0, u0, 0, nullptr, &one, u0, o.abstol, o.reltol, s->n, s->dscal + 0, st));
    SOLVE_TRY(wsumsq<T>(h, u0, u0, 0, nullptr, &one, f0, o.abstol, o.reltol, s->n, s->dscal + 1, st));
    SOLVE_TRY(read_scalars(h, s, 2, st));
    const double d0 = std::sqrt(s->hscal[0] / (double)s->n), d1 = std::sqrt(s->hscal[1] / (double)s->n);
    double dt0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
    dt0 = std::min(dt0, tdist);
    void* kk[1] = {(void*)f0};
    kanode_stage sg = make_stage(1, kk, &dt0);
    SOLVE_TRY(kanode_rhs_stage(h, p, u0, &sg, tmp, s->batch, st));
    const void* kd[1] = {tmp};
    e1[1] = -1.0;
    SOLVE_TRY(wsumsq<T>(h, u0, u0, 1, kd, e1, f0, o.abstol, o.reltol, s->n, s->dscal + 2, st));
    SOLVE_TRY(read_scalars(h, s, 3, st));
    const double d2 = std::sqrt(s->hscal[2] / (double)s->n) / dt0;
    const double mx = std::max(d1, d2);
    const double dt1 = mx <= 1e-15 ? std::max(1e-6, dt0 * 1e-3) : std::pow(0.01 / mx, 1.0 / 5.0);
    dt = std::min(std::min(100 * dt0, dt1), tdist);
    return KANODE_OK;
}

// The saveat values inside step `step` (t, t + dt] from its dense output: one launch for all of them (the same
// arithmetic as one stage_lincomb / copy each; kan::SaveatStep).  ks: the step's k_1..k_7 (K form).
template <typename T>
kanode_status saveat_in_step(kanode_handle* h, kanode_solution* s, int64_t step, double t, double dt,
                             void* const* ks, const double* saveat, int64_t n_save, int64_t& si, void* u_save,
                             hipStream_t st) {
    const size_t sb = s->state_bytes();
    const double tn = t + dt;
    kan::SaveatStep<T> sv{};
    sv.u = (const T*)s->u(step);
    sv.u_new = (const T*)s->u(step + 1);
    sv.nk = s->qform ? 4 : 7;
    for (int j = 0; j < sv.nk; ++j) sv.k[j] = (const T*)(s->qform ? s->q(step, j + 1) : ks[j]);
    auto flush_sv = [&]() -> kanode_status {
        if (sv.nsv == 0) return KANODE_OK;
        SOLVE_HIP(h, kan::launch_saveat_step<T>(sv, s->n, st));
        sv.nsv = 0;
        sv.exact = 0;
        return KANODE_OK;
    };
    while (si < n_save && saveat[si] <= tn + 1e-12 * std::max(1.0, std::fabs(tn))) {
        const double tsv = saveat[si];
        if (sv.nsv == 0) sv.dst = (T*)((char*)u_save + si * sb);
        const int jv = sv.nsv;
        if (std::fabs(tsv - tn) <= 1e-12 * std::max(1.0, std::fabs(tn))) {
            sv.exact |= 1ull << jv;
        } else if (s->qform) {
            const double th = (tsv - t) / dt;
            sv.w[jv][0] = th;
            sv.w[jv][1] = th * th;
            sv.w[jv][2] = th * th * th;
            sv.w[jv][3] = th * th * th * th;
        } else {
            double w[7];
            interp_weights((tsv - t) / dt, w);
            for (int j = 0; j < 7; ++j) sv.w[jv][j] = w[j] * dt;
        }
        ++sv.nsv;
        ++si;
        if (sv.nsv == kan::kSaveatPerLaunch) SOLVE_TRY(flush_sv());
    }
    return flush_sv();
}

template <typename T>
kanode_status solve_t(kanode_handle* h, const void* p, const void* u0, double t0, double tf, const double* saveat,
                      int64_t n_save, void* u_save, const kanode_solver_options& o, kanode_solution* s,
                      kanode_solve_stats* stats, hipStream_t st) {
    const size_t sb = s->state_bytes();
    int64_t si = 0;
    while (si < n_save && saveat[si] <= t0 + 1e-14 * std::max(1.0, std::fabs(t0))) {
        SOLVE_HIP(h, hipMemcpyAsync((char*)u_save + si * sb, u0, sb, hipMemcpyDeviceToDevice, st));
        ++si;
    }
    // fixed step: the whole step sequence is known, allocate it up front
    if (!o.adaptive) {
        int64_t nst = 0;
        for (double t = t0, dt = o.dt; nst < o.maxiters && !(t >= tf - 1e-14 * std::max(1.0, std::fabs(tf)));) {
            dt = std::min(dt, tf - t);
            t = t + dt;
            ++nst;
        }
        SOLVE_TRY(ensure_slots(h, s, nst + 1, st));
    } else {
        SOLVE_TRY(ensure_slots(h, s, 2, st));
    }
    // Fisher-KPP table path: one launch per step and the dense output in Q form
    s->qform = kanode_internal_fk_step_ok(h);
    SOLVE_HIP(h, hipMemcpyAsync(s->u(0), u0, sb, hipMemcpyDeviceToDevice, st));
    kanode_stage s0{};
    SOLVE_TRY(kanode_rhs_stage(h, p, s->u(0), &s0, s->k1_0, s->batch, st));   // k1 = f(u0)
    double dt = o.dt;
    if (o.adaptive && !(o.dt > 0)) SOLVE_TRY(initdt<T>(h, s, p, s->u(0), s->k1_0, tf - t0, o, dt, st, s->q(0, 1)));
    double qold = o.qoldinit;
    double t = t0;
    int64_t step = 0, naccept = 0, nreject = 0, nf = 0;
    int64_t it = 0;
    for (; it < o.maxiters; ++it) {
        if (t >= tf - 1e-14 * std::max(1.0, std::fabs(tf))) break;
        dt = std::min(dt, tf - t);
        SOLVE_TRY(ensure_slots(h, s, step + 2, st));
        void* ks[7];
        for (int j = 0; j < 7; ++j) ks[j] = s->k(step, j + 1);
        bool fused_step = false;   // Fisher-KPP table path: the six stages in one launch
        int nparts = 0;            // > 0: the error is that many partials in hparts (not hscal[0])
        if (o.adaptive && s->mscal) arm_ctl(s->hscal, 1);
        if (s->qform) {
            double a66[36] = {}, e7[7], q47[28];
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j <= i; ++j) a66[6 * i + j] = dt * TA[i][j];
            for (int j = 0; j < 7; ++j) e7[j] = dt * BT[j];
            for (int m = 0; m < 4; ++m)
                for (int i = 0; i < 7; ++i) q47[7 * m + i] = dt * RI[i][m];
            void* kout[6] = {s->q(step, 1), s->q(step, 2), s->q(step, 3), s->q(step, 4), nullptr, s->k(step, 7)};
            SOLVE_TRY(kanode_internal_fk_step(h, p, s->u(step), ks[0], kout, s->u(step + 1), a66,
                                              o.adaptive ? e7 : nullptr, q47, o.abstol, o.reltol,
                                              o.adaptive ? ctl(s) : nullptr, s->batch, st, fused_step,
                                              o.adaptive ? s->mparts : nullptr, &nparts));
            if (!fused_step) return kanode_internal_fail(h, KANODE_ERR_HIP, "Tsit5: fused step not launched");
        } else {   // a small chain: the six stages per column in one launch
            double a66[36] = {}, e7[7];
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j <= i; ++j) a66[6 * i + j] = dt * TA[i][j];
            for (int j = 0; j < 7; ++j) e7[j] = dt * BT[j];
            SOLVE_TRY(kanode_internal_chain_step(h, p, s->u(step), ks[0], ks + 1, s->u(step + 1), a66,
                                                 o.adaptive ? e7 : nullptr, o.abstol, o.reltol,
                                                 o.adaptive ? ctl(s) : nullptr, s->batch, st, fused_step));
        }
        for (int i = 0; i < 6 && !fused_step; ++i) {
            double c[6];
            for (int j = 0; j <= i; ++j) c[j] = dt * TA[i][j];
            kanode_stage sg = make_stage(i + 1, ks, c);
            if (i == 5) {
                sg.y_out = s->u(step + 1);
                if (o.adaptive) {
                    sg.want_error = 1;
                    for (int j = 0; j < 7; ++j) sg.ec[j] = dt * BT[j];
                    sg.abstol = o.abstol;
                    sg.reltol = o.reltol;
                    sg.error_sumsq = ctl(s);
                }
            }
            SOLVE_TRY(kanode_rhs_stage(h, p, s->u(step), &sg, ks[i + 1], s->batch, st));
        }
        nf += 6;
        double dtnew = dt;
        if (o.adaptive) {
            double sumsq;
            if (nparts > 0) {   // the step kernel's per-block partials, summed here in block order
                SOLVE_TRY(wait_ctl(h, st, {{s->hparts, nparts}}));
                sumsq = 0.0;
                for (int b = 0; b < nparts; ++b) sumsq += s->hparts[b];
                arm_ctl(s->hparts, nparts);   // (every slot stays armed between steps)
            } else {
                if (s->mscal) SOLVE_TRY(wait_ctl(h, st, {{s->hscal, 1}}));
                else SOLVE_TRY(read_ctl(h, s, 0, 1, st));
                sumsq = s->hscal[0];
            }
            const double EEst = std::sqrt(sumsq / (double)s->n);
            const double q11 = EEst > 0 ? std::pow(EEst, o.beta1) : 0.0;
            if (EEst > 1.0 && dt > o.dtmin) {
                ++nreject;
                dt = dt / std::min(1.0 / o.qmin, q11 / o.gamma);
                continue;
            }
            double q = q11 / std::pow(qold, o.beta2);
            q = std::max(1.0 / o.qmax, std::min(1.0 / o.qmin, q / o.gamma));
            if (1.0 <= q && q <= 1.0) q = 1.0;   // qsteady_min = qsteady_max = 1
            dtnew = q > 0 ? dt / q : dt * o.qmax;
            qold = std::max(EEst, o.qoldinit);
        }
        const double tn = t + dt;
        SOLVE_TRY(saveat_in_step<T>(h, s, step, t, dt, ks, saveat, n_save, si, u_save, st));
        s->ts.push_back(t);
        s->dts.push_back(dt);
        t = tn;
        ++step;
        ++naccept;
        dt = dtnew;
    }
    if (it == o.maxiters && !(t >= tf - 1e-14 * std::max(1.0, std::fabs(tf))))
        return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "Tsit5: maxiters reached");
    if (stats) {
        stats->naccept = naccept;
        stats->nreject = nreject;
        stats->nf = nf + 1;
    }
    return KANODE_OK;
}

// ---- one-workgroup solve of a small chain (kd_chain_tsit5_kernel) ------------------------
// A stream-ordered upload of host bytes through the solution's pinned staging: unlike hipMemcpy from pageable
// memory it does not hold the host until the stream drains.  The staging is rewritten only after the previous
// upload from it has run (its event).
kanode_status staged_upload(kanode_handle* h, kanode_solution* s, void* dst, const void* src, size_t bytes,
                            hipStream_t st, std::vector<char>* last = nullptr) {
    auto& f = s->fused;
    if (last && last->size() == bytes && std::memcmp(last->data(), src, bytes) == 0) return KANODE_OK;
    if (!f.hup_ev) SOLVE_HIP(h, hipEventCreateWithFlags(&f.hup_ev, hipEventDisableTiming));
    if (f.hup_pending) {
        SOLVE_HIP(h, hipEventSynchronize(f.hup_ev));
        f.hup_pending = false;
    }
    if (f.hup_bytes < bytes) {
        if (f.hup) (void)hipHostFree(f.hup);
        f.hup = nullptr;
        f.hup_bytes = 0;
        SOLVE_HIP(h, hipHostMalloc(&f.hup, bytes));
        f.hup_bytes = bytes;
    }
    std::memcpy(f.hup, src, bytes);
    SOLVE_HIP(h, hipMemcpyAsync(dst, f.hup, bytes, hipMemcpyHostToDevice, st));
    SOLVE_HIP(h, hipEventRecord(f.hup_ev, st));
    f.hup_pending = true;
    if (last) last->assign((const char*)src, (const char*)src + bytes);
    return KANODE_OK;
}

// The whole forward solve in one launch for a chain of small layers and <= 16 trajectories (the
// Lotka-Volterra shape).  done = false when the shape is not covered or the dense-output block
// filled up: the caller then runs the host loop (solve_t) from scratch.
template <typename T>
kanode_status solve_fused_t(kanode_handle* h, const void* p, const void* u0, double t0, double tf, const double* saveat,
                            int64_t n_save, void* u_save, const kanode_solver_options& o, kanode_solution* s,
                            kanode_solve_stats* stats, hipStream_t st, bool& done) {
    done = false;
    if (capturing(st) || !kanode_internal_chain_tsit5_ok(h, s->batch)) return KANODE_OK;
    const size_t sb = s->state_bytes();
    auto& f = s->fused;
    int64_t cap = 0;
    if (s->record) {
        if (!o.adaptive) {
            for (double t = t0, dt = o.dt; cap < o.maxiters && !(t >= tf - 1e-14 * std::max(1.0, std::fabs(tf)));) {
                dt = std::min(dt, tf - t);
                t = t + dt;
                ++cap;
            }
        } else {
            cap = std::min<int64_t>(o.maxiters, 4096);
            if (const int c = kanode_internal_fused_solve_cap(h)) cap = c;   // KANODE_OPT_FUSED_SOLVE_CAP
        }
        cap = std::max<int64_t>(cap, 1);
        if (f.cap < cap) {
            if (s->slots_borrowed) s->slots.clear();
            if (f.block) (void)hipFree(f.block);
            f.block = nullptr;
            f.cap = 0;
            if (hipMalloc(&f.block, (size_t)cap * 7 * sb) != hipSuccess) {
                (void)hipGetLastError();
                return KANODE_OK;   // no room for the contiguous block: the host loop allocates per step
            }
            f.cap = cap;
        }
        if (f.ts_cap < f.cap) {
            if (f.ts) (void)hipFree(f.ts);
            f.ts = nullptr;
            f.ts_cap = 0;
            SOLVE_HIP(h, hipMalloc((void**)&f.ts, 2 * (size_t)f.cap * sizeof(double)));
            f.ts_cap = f.cap;
        }
    }
    if (f.saveat_cap < n_save) {
        if (f.saveat) (void)hipFree(f.saveat);
        f.saveat = nullptr;
        f.saveat_cap = 0;
        f.saveat_last.clear();
        SOLVE_HIP(h, hipMalloc((void**)&f.saveat, (size_t)n_save * sizeof(double)));
        f.saveat_cap = n_save;
    }
    if (!f.out) SOLVE_HIP(h, hipMalloc((void**)&f.out, 4 * sizeof(int64_t)));
    if (n_save > 0) SOLVE_TRY(staged_upload(h, s, f.saveat, saveat, (size_t)n_save * sizeof(double), st, &f.saveat_last));
    kan::ChainSolveArgs a{};
    a.t0 = t0;
    a.tf = tf;
    a.dt = o.dt;
    a.abstol = o.abstol;
    a.reltol = o.reltol;
    a.dtmin = o.dtmin;
    a.beta1 = o.beta1;
    a.beta2 = o.beta2;
    a.gamma = o.gamma;
    a.qmin = o.qmin;
    a.qmax = o.qmax;
    a.qoldinit = o.qoldinit;
    a.adaptive = o.adaptive ? 1 : 0;
    a.maxiters = o.maxiters;
    a.n_save = n_save;
    a.cap = s->record ? f.cap : 0;
    a.saveat = f.saveat;
    a.u_save = n_save > 0 ? u_save : nullptr;
    a.rec = s->record ? f.block : nullptr;
    a.k1_0 = s->k1_0;
    a.ts = s->record ? f.ts : nullptr;
    a.dts = s->record ? f.ts + f.cap : nullptr;
    // the counters straight into the mapped host mirror when there is one (no copy launch to read them); without
    // step records to fetch, the host then spins on them instead of synchronising the stream (wait_ctl: the
    // wake-up of hipStreamSynchronize is ~20 us; what follows on the stream is ordered after the kernel anyway)
    // the step records: pinned, mapped host staging the kernel writes alongside the device copy (else copied)
    if (s->record && f.hts_cap < f.cap) {
        if (f.hts) (void)hipHostFree(f.hts);
        f.hts = nullptr;
        f.mts = nullptr;
        f.hts_cap = 0;
        SOLVE_HIP(h, hipHostMalloc((void**)&f.hts, 2 * (size_t)f.cap * sizeof(double),
                                   hipHostMallocMapped | hipHostMallocCoherent));
        f.hts_cap = f.cap;
        if (hipHostGetDevicePointer((void**)&f.mts, f.hts, 0) != hipSuccess) {
            (void)hipGetLastError();
            f.mts = nullptr;
        }
    }
    a.out = s->mscal ? (int64_t*)s->mscal : f.out;
    a.hts = s->record && s->mscal ? f.mts : nullptr;
    const bool spin = s->mscal && (!s->record || a.hts);
    if (spin) arm_ctl(s->hscal, 4);
    bool launched = false;
    SOLVE_TRY(kanode_internal_chain_tsit5(h, p, u0, s->batch, &a, st, launched));
    if (!launched) return KANODE_OK;
    if (!s->mscal) SOLVE_HIP(h, hipMemcpyAsync(s->hscal, f.out, 4 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    if (s->record && !a.hts)
        SOLVE_HIP(h, hipMemcpyAsync(f.hts, f.ts, 2 * (size_t)f.cap * sizeof(double), hipMemcpyDeviceToHost, st));
    if (spin) SOLVE_TRY(wait_ctl(h, st, {{s->hscal, 4}}));
    else SOLVE_HIP(h, hipStreamSynchronize(st));
    int64_t res[4];
    std::memcpy(res, s->hscal, sizeof(res));
    if (res[3] == 2) return KANODE_OK;   // dense output full: the host loop redoes the solve
    if (res[3] == 1) return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "Tsit5: maxiters reached");
    const int64_t na = res[0];
    if (s->record) {
        s->ts.assign(f.hts, f.hts + na);
        s->dts.assign(f.hts + f.cap, f.hts + f.cap + na);
        if (!s->slots_borrowed)
            for (void* q : s->slots) (void)hipFree(q);
        s->slots.resize(f.cap);
        for (int64_t i = 0; i < f.cap; ++i) s->slots[i] = (char*)f.block + (size_t)i * 7 * sb;
        s->slots_borrowed = true;
    }
    if (stats) {
        stats->naccept = res[0];
        stats->nreject = res[1];
        stats->nf = res[2];
    }
    done = true;
    return KANODE_OK;
}

// ---- device step control: the solve as a replayed hipGraph ------------------------------
kanode_status dev_alloc(kanode_handle* h, void** p, size_t bytes, const char* what) {
    if (hipMalloc(p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
        return kanode_internal_fail(h, KANODE_ERR_ALLOC, std::string("device control: out of device memory (") + what + ")");
    }
    return KANODE_OK;
}

bool same_opts(const kanode_solver_options& a, const kanode_solver_options& b) {
    return a.abstol == b.abstol && a.reltol == b.reltol && a.adaptive == b.adaptive && a.maxiters == b.maxiters &&
           a.dtmin == b.dtmin && a.beta1 == b.beta1 && a.beta2 == b.beta2 && a.gamma == b.gamma && a.qmin == b.qmin &&
           a.qmax == b.qmax && a.qoldinit == b.qoldinit;
}

template <typename T>
kan::Tsit5Bufs<T> graph_bufs(kanode_solution* s) {
    kan::Tsit5Bufs<T> bf{};
    char* b = (char*)s->g.bufs;
    const size_t sb = s->state_bytes();
    bf.U = (T*)b;
    for (int j = 0; j < 7; ++j) bf.K[j] = (T*)(b + (1 + j) * sb);
    bf.UNEW = (const T*)(b + 8 * sb);
    bf.save = (T*)s->g.save;
    bf.slots = s->g.slots;
    return bf;
}

// Capture `steps` step slots (six stage launches + tsit5_post_kernel each) into a graph.
template <typename T>
kanode_status build_graph(kanode_handle* h, kanode_solution* s, const void* p, double tf, int64_t n_save,
                          const kanode_solver_options& o, int steps) {
    auto& g = s->g;
    if (g.exec) {
        (void)hipGraphExecDestroy(g.exec);
        g.exec = nullptr;
    }
    if (!g.cap_stream) SOLVE_HIP(h, hipStreamCreateWithFlags(&g.cap_stream, hipStreamNonBlocking));
    const kan::Tsit5Bufs<T> bf = graph_bufs<T>(s);
    kan::Tsit5PostArgs pa{};
    pa.tf = tf;
    pa.dtmin = o.dtmin;
    pa.beta1 = o.beta1;
    pa.beta2 = o.beta2;
    pa.gamma = o.gamma;
    pa.qmin = o.qmin;
    pa.qmax = o.qmax;
    pa.qoldinit = o.qoldinit;
    pa.adaptive = o.adaptive;
    pa.record = s->record;
    pa.maxiters = o.maxiters;
    pa.n_save = n_save;
    pa.slot_cap = g.cap;
    pa.saveat = g.saveat;
    pa.ts_rec = g.ts;
    pa.dts_rec = g.dts;
    kanode_internal_hold_tables(h, true);   // the first captured stage rebuilds the tables on every replay
    SOLVE_HIP(h, hipStreamBeginCapture(g.cap_stream, hipStreamCaptureModeRelaxed));
    kanode_status r = KANODE_OK;
    for (int sl = 0; sl < steps && r == KANODE_OK; ++sl) {
        kan::SolveCtl* cin = g.ctl + (sl & 1);
        kan::SolveCtl* cout = g.ctl + ((sl + 1) & 1);
        void* ks[7];
        for (int j = 0; j < 7; ++j) ks[j] = bf.K[j];
        for (int i = 0; i < 6 && r == KANODE_OK; ++i) {
            kanode_stage sg = make_stage(i + 1, ks, TA[i]);
            if (i == 5) {
                sg.y_out = (void*)bf.UNEW;
                if (o.adaptive) {
                    sg.want_error = 1;
                    for (int j = 0; j < 7; ++j) sg.ec[j] = BT[j];
                    sg.abstol = o.abstol;
                    sg.reltol = o.reltol;
                    sg.error_sumsq = s->dscal;
                }
            }
            r = kanode_internal_rhs_stage(h, p, bf.U, &sg, ks[i + 1], s->batch, g.cap_stream, &cin->dt, &cin->done);
        }
        if (r == KANODE_OK) {
            const hipError_t e = kan::launch_tsit5_post<T>(cin, cout, s->dscal, bf, pa, s->n, g.cap_stream);
            if (e != hipSuccess) r = kanode_internal_fail(h, KANODE_ERR_HIP, std::string("tsit5_post: ") + hipGetErrorString(e));
        }
    }
    hipGraph_t graph = nullptr;
    const hipError_t ec = hipStreamEndCapture(g.cap_stream, &graph);
    if (r != KANODE_OK) {
        if (graph) (void)hipGraphDestroy(graph);
        return r;
    }
    if (ec != hipSuccess) return kanode_internal_fail(h, KANODE_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ec));
    const hipError_t ei = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (ei != hipSuccess) {
        g.exec = nullptr;
        return kanode_internal_fail(h, KANODE_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
    }
    g.key_p = p;
    g.key_nsave = n_save;
    g.key_cap = g.cap;
    g.key_record = s->record;
    g.key_steps = steps;
    g.key_tf = tf;
    g.key_opt = o;
    return KANODE_OK;
}

// dense-output capacity for `need` accepted steps: slots (host + device pointer table) and the
// device step-time records; growing the tables invalidates the graph
kanode_status graph_capacity(kanode_handle* h, kanode_solution* s, int64_t need, hipStream_t st) {
    auto& g = s->g;
    if (s->record) SOLVE_TRY(ensure_slots(h, s, need, st));
    if (need > g.cap) {
        int64_t cap = std::max<int64_t>(64, g.cap);
        while (cap < need) cap *= 2;
        SOLVE_HIP(h, hipStreamSynchronize(st));
        void *nslots = nullptr, *nts = nullptr, *ndts = nullptr;
        SOLVE_TRY(dev_alloc(h, &nslots, cap * sizeof(void*), "slot table"));
        SOLVE_TRY(dev_alloc(h, &nts, cap * sizeof(double), "step times"));
        SOLVE_TRY(dev_alloc(h, &ndts, cap * sizeof(double), "step sizes"));
        if (g.cap > 0) {
            SOLVE_HIP(h, hipMemcpy(nts, g.ts, g.cap * sizeof(double), hipMemcpyDeviceToDevice));
            SOLVE_HIP(h, hipMemcpy(ndts, g.dts, g.cap * sizeof(double), hipMemcpyDeviceToDevice));
        }
        for (void* q : {(void*)g.slots, (void*)g.ts, (void*)g.dts})
            if (q) (void)hipFree(q);
        g.slots = (void**)nslots;
        g.ts = (double*)nts;
        g.dts = (double*)ndts;
        g.cap = cap;
        g.slots_synced = 0;
    }
    if (s->record && g.slots_synced < (int64_t)s->slots.size()) {
        const int64_t a = g.slots_synced, b = std::min<int64_t>((int64_t)s->slots.size(), g.cap);
        SOLVE_HIP(h, hipMemcpy(g.slots + a, s->slots.data() + a, (b - a) * sizeof(void*), hipMemcpyHostToDevice));
        g.slots_synced = b;
    }
    return KANODE_OK;
}

template <typename T>
kanode_status solve_graph_t(kanode_handle* h, const void* p, const void* u0, double t0, double tf,
                            const double* saveat, int64_t n_save, void* u_save, const kanode_solver_options& o,
                            kanode_solution* s, kanode_solve_stats* stats, hipStream_t st) {
    auto& g = s->g;
    const size_t sb = s->state_bytes();
    const int steps = o.graph_steps > 0 ? (o.graph_steps + 1) / 2 * 2 : 16;
    if (g.bufs_bytes < 9 * sb) {
        SOLVE_HIP(h, hipStreamSynchronize(st));
        if (g.bufs) (void)hipFree(g.bufs);
        g.bufs = nullptr;
        g.bufs_bytes = 0;
        SOLVE_TRY(dev_alloc(h, &g.bufs, 9 * sb, "stage vectors"));
        g.bufs_bytes = 9 * sb;
        if (g.exec) {
            (void)hipGraphExecDestroy(g.exec);
            g.exec = nullptr;
        }
    }
    if (!g.ctl) {
        SOLVE_TRY(dev_alloc(h, (void**)&g.ctl, 2 * sizeof(kan::SolveCtl), "control"));
        SOLVE_HIP(h, hipHostMalloc((void**)&g.hctl, sizeof(kan::SolveCtl)));
    }
    if (g.saveat_cap < std::max<int64_t>(n_save, 1) || g.save_bytes < (size_t)n_save * sb) {
        SOLVE_HIP(h, hipStreamSynchronize(st));
        if (g.saveat) (void)hipFree(g.saveat);
        if (g.save) (void)hipFree(g.save);
        g.saveat = nullptr;
        g.save = nullptr;
        SOLVE_TRY(dev_alloc(h, (void**)&g.saveat, std::max<int64_t>(n_save, 1) * sizeof(double), "saveat"));
        SOLVE_TRY(dev_alloc(h, &g.save, std::max<size_t>((size_t)n_save * sb, 1), "saveat values"));
        g.saveat_cap = std::max<int64_t>(n_save, 1);
        g.save_bytes = (size_t)n_save * sb;
        if (g.exec) {
            (void)hipGraphExecDestroy(g.exec);
            g.exec = nullptr;
        }
    }
    SOLVE_TRY(kanode_internal_prepare(h, s->batch, st));
    const kan::Tsit5Bufs<T> bf = graph_bufs<T>(s);
    int64_t si = 0;
    while (si < n_save && saveat[si] <= t0 + 1e-14 * std::max(1.0, std::fabs(t0))) {
        SOLVE_HIP(h, hipMemcpyAsync((char*)g.save + si * sb, u0, sb, hipMemcpyDeviceToDevice, st));
        ++si;
    }
    if (n_save > 0) SOLVE_HIP(h, hipMemcpyAsync(g.saveat, saveat, n_save * sizeof(double), hipMemcpyHostToDevice, st));
    SOLVE_HIP(h, hipMemcpyAsync(bf.U, u0, sb, hipMemcpyDeviceToDevice, st));
    kanode_stage s0{};
    SOLVE_TRY(kanode_rhs_stage(h, p, bf.U, &s0, bf.K[0], s->batch, st));   // k1 = f(u0)
    if (s->record) {
        SOLVE_TRY(ensure_slots(h, s, 1, st));
        SOLVE_HIP(h, hipMemcpyAsync(s->k1_0, bf.K[0], sb, hipMemcpyDeviceToDevice, st));
    }
    double dt = o.dt;
    if (o.adaptive && !(o.dt > 0)) SOLVE_TRY(initdt<T>(h, s, p, bf.U, bf.K[0], tf - t0, o, dt, st, bf.K[1]));
    kan::SolveCtl c0{};
    c0.t = t0;
    c0.dt = std::min(dt, tf - t0);
    c0.qold = o.qoldinit;
    c0.si = si;
    c0.done = t0 >= tf - 1e-14 * std::max(1.0, std::fabs(tf)) ? 1 : 0;
    SOLVE_HIP(h, hipStreamSynchronize(st));   // the pinned control block is rewritten below
    *g.hctl = c0;
    SOLVE_HIP(h, hipMemcpyAsync(g.ctl, g.hctl, sizeof(c0), hipMemcpyHostToDevice, st));
    int64_t naccept = 0;
    for (;;) {
        SOLVE_TRY(graph_capacity(h, s, naccept + steps + 1, st));
        if (!g.exec || g.key_p != p || g.key_nsave != n_save || g.key_cap != g.cap || g.key_record != (int)s->record ||
            g.key_steps != steps || g.key_tf != tf || !same_opts(g.key_opt, o))
            SOLVE_TRY(build_graph<T>(h, s, p, tf, n_save, o, steps));
        SOLVE_HIP(h, hipGraphLaunch(g.exec, st));
        SOLVE_HIP(h, hipMemcpyAsync(g.hctl, g.ctl, sizeof(kan::SolveCtl), hipMemcpyDeviceToHost, st));
        SOLVE_HIP(h, hipStreamSynchronize(st));
        naccept = g.hctl->naccept;
        if (g.hctl->done) break;
    }
    const kan::SolveCtl c = *g.hctl;
    if (c.status == 1) return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "Tsit5: maxiters reached");
    if (c.status != 0) return kanode_internal_fail(h, KANODE_ERR_ALLOC, "Tsit5 (device control): dense-output storage full");
    if (s->record && c.naccept > 0) {
        s->ts.resize(c.naccept);
        s->dts.resize(c.naccept);
        SOLVE_HIP(h, hipMemcpy(s->ts.data(), g.ts, c.naccept * sizeof(double), hipMemcpyDeviceToHost));
        SOLVE_HIP(h, hipMemcpy(s->dts.data(), g.dts, c.naccept * sizeof(double), hipMemcpyDeviceToHost));
    }
    if (n_save > 0) SOLVE_HIP(h, hipMemcpyAsync(u_save, g.save, n_save * sb, hipMemcpyDeviceToDevice, st));
    if (stats) {
        stats->naccept = c.naccept;
        stats->nreject = c.nreject;
        stats->nf = 6 * c.attempts + 1;
    }
    return KANODE_OK;
}

// ---- the adaptive Fisher-KPP solve with the step control on the device ------------------------------
// KANODE_OPT_FK_DEVICE_LOOP, control = auto, fp64 table path, dense output kept: solve_t's algorithm with every
// attempt one launch of the step kernel's DEV instantiation (kan::FkLoopArgs): launch q decides attempt q - 1 at
// its head (every workgroup, the same sums) and takes the next, so the host queues launches ahead in batches of
// kBatch and only polls the mapped mirror of the state; launches queued past the end return at once.  The saveat values come from the dense output afterwards (saveat_in_step, as solve_t).
// done = false when not covered (solve_t runs instead).
kanode_status solve_fk_loop(kanode_handle* h, const void* p, const void* u0, double t0, double tf,
                            const double* saveat, int64_t n_save, void* u_save, const kanode_solver_options& o,
                            kanode_solution* s, kanode_solve_stats* stats, hipStream_t st, bool& done) {
    done = false;
    if (o.control != 0 || !o.adaptive || !s->record || s->dtype != KANODE_F64 || capturing(st) ||
        !kanode_internal_fk_loop_ok(h) || t0 >= tf - 1e-14 * std::max(1.0, std::fabs(tf)))
        return KANODE_OK;
    constexpr int64_t kBatch = 16;
    const size_t sb = s->state_bytes();
    auto& L = s->loop;
    // the slot table and step records grow geometrically with the launches queued (a solve that reaches
    // maxiters stops on the device's status 2, not on the table size)
    const int64_t cap_max = o.maxiters + 2 * kBatch + 3;
    auto grow = [&](int64_t want) -> kanode_status {
        if (L.cap >= want) return KANODE_OK;
        int64_t cap = std::max<int64_t>(L.cap, 1024);
        while (cap < want) cap *= 2;
        cap = std::max(std::min(cap, cap_max), want);
        SOLVE_HIP(h, hipStreamSynchronize(st));   // (the queued launches write the old records)
        void** nslots = nullptr;
        double* nts = nullptr;
        void** nh = nullptr;
        SOLVE_TRY(dev_alloc(h, (void**)&nslots, cap * sizeof(void*), "slot table"));
        if (kanode_status r = dev_alloc(h, (void**)&nts, 2 * cap * sizeof(double), "step records"); r != KANODE_OK) {
            (void)hipFree(nslots);
            return r;
        }
        if (hipHostMalloc((void**)&nh, cap * sizeof(void*)) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipFree(nslots);
            (void)hipFree(nts);
            return kanode_internal_fail(h, KANODE_ERR_ALLOC, "Tsit5 (device loop): pinned slot staging");
        }
        if (L.cap > 0) {   // keep what is recorded: slots [0, synced), ts | dts (each cap long)
            SOLVE_HIP(h, hipMemcpy(nslots, L.dslots, L.cap * sizeof(void*), hipMemcpyDeviceToDevice));
            SOLVE_HIP(h, hipMemcpy(nts, L.ts, L.cap * sizeof(double), hipMemcpyDeviceToDevice));
            SOLVE_HIP(h, hipMemcpy(nts + cap, L.ts + L.cap, L.cap * sizeof(double), hipMemcpyDeviceToDevice));
            std::memcpy(nh, L.hslots, L.cap * sizeof(void*));
        }
        for (void* q : {(void*)L.dslots, (void*)L.ts})
            if (q) (void)hipFree(q);
        if (L.hslots) (void)hipHostFree(L.hslots);
        L.dslots = nslots;
        L.ts = nts;
        L.hslots = nh;
        L.cap = cap;
        return KANODE_OK;
    };
    SOLVE_TRY(grow(std::min<int64_t>(cap_max, 4 * kBatch + 3)));
    if (!L.ctl) {
        SOLVE_TRY(dev_alloc(h, (void**)&L.ctl, 2 * sizeof(kan::FkLoopCtl), "loop state"));
        SOLVE_TRY(dev_alloc(h, (void**)&L.parts, 2 * kanode_internal_max_parts() * sizeof(double), "loop partials"));
        SOLVE_HIP(h, hipHostMalloc((void**)&L.hmir, sizeof(kan::FkLoopCtl), hipHostMallocMapped | hipHostMallocCoherent));
        SOLVE_HIP(h, hipHostGetDevicePointer((void**)&L.dmir, L.hmir, 0));
    }
    L.synced = 0;
    int64_t si = 0;
    while (si < n_save && saveat[si] <= t0 + 1e-14 * std::max(1.0, std::fabs(t0))) {
        SOLVE_HIP(h, hipMemcpyAsync((char*)u_save + si * sb, u0, sb, hipMemcpyDeviceToDevice, st));
        ++si;
    }
    SOLVE_TRY(ensure_slots(h, s, 3, st));
    s->qform = true;
    SOLVE_HIP(h, hipMemcpyAsync(s->u(0), u0, sb, hipMemcpyDeviceToDevice, st));
    kanode_stage s0{};
    SOLVE_TRY(kanode_rhs_stage(h, p, s->u(0), &s0, s->k1_0, s->batch, st));   // k1 = f(u0)
    double dt = o.dt;
    if (!(o.dt > 0)) SOLVE_TRY(initdt<double>(h, s, p, s->u(0), s->k1_0, tf - t0, o, dt, st, s->q(0, 1)));
    SOLVE_HIP(h, hipStreamSynchronize(st));   // (the mirror is the init copy's source and the device's target)
    kan::FkLoopCtl c0{};   // launch 0 reads state[1]: no attempt pending
    c0.t = t0;
    c0.dt = dt;
    c0.qold = o.qoldinit;
    c0.cand[1] = s->slots[0];
    c0.cand[2] = s->slots[1];
    c0.cand[3] = s->slots[2];
    *L.hmir = c0;
    SOLVE_HIP(h, hipMemcpy(L.ctl + 1, &c0, sizeof(c0), hipMemcpyHostToDevice));
    kan::FkLoopArgs la{};
    la.state = L.ctl;
    la.mirror = L.dmir;
    la.slots = L.dslots;
    la.k1_0 = (const double*)s->k1_0;
    la.ts = L.ts;
    la.dts = L.ts + L.cap;
    la.parts = L.parts;
    la.max_grid = kanode_internal_max_parts();
    la.n = s->n;
    la.tf = tf;
    la.abstol = o.abstol;
    la.reltol = o.reltol;
    la.dtmin = o.dtmin;
    la.beta1 = o.beta1;
    la.beta2 = o.beta2;
    la.gamma = o.gamma;
    la.qmin = o.qmin;
    la.qmax = o.qmax;
    la.qoldinit = o.qoldinit;
    la.maxiters = o.maxiters;
    const volatile kan::FkLoopCtl* mir = L.hmir;
    int64_t queued = 0;
    for (;;) {
        if (queued + kBatch + 3 > L.cap) {
            if (queued + kBatch + 3 > cap_max)
                return kanode_internal_fail(h, KANODE_ERR_ALLOC, "Tsit5 (device loop): step table full");
            SOLVE_TRY(grow(queued + kBatch + 3));
            la.slots = L.dslots;
            la.ts = L.ts;
            la.dts = L.ts + L.cap;
        }
        // slots for every step the queued launches can reach (each launch advances at most one step; a state
        // names the slots up to its step + 2)
        SOLVE_TRY(ensure_slots(h, s, queued + kBatch + 3, st));
        const int64_t ns = (int64_t)s->slots.size();
        if (L.synced < ns) {
            std::memcpy(L.hslots + L.synced, s->slots.data() + L.synced, (ns - L.synced) * sizeof(void*));
            SOLVE_HIP(h, hipMemcpyAsync(L.dslots + L.synced, L.hslots + L.synced, (ns - L.synced) * sizeof(void*),
                                        hipMemcpyHostToDevice, st));
            L.synced = ns;
        }
        for (int64_t i = 0; i < kBatch; ++i)
            SOLVE_TRY(kanode_internal_fk_step_loop(h, p, &la, queued + i, s->batch, st));
        queued += kBatch;
        // keep one batch queued behind the running one: wait until the device has decided the previous batch's
        // attempts (launch q decides attempt q - 1)
        for (uint64_t it = 1; mir->status == 0 && mir->it + 1 < queued - kBatch; ++it) {
            if ((it & 255) == 0) {
                const hipError_t q = hipStreamQuery(st);
                if (q == hipSuccess) break;
                if (q != hipErrorNotReady) SOLVE_HIP(h, q);
            }
            cpu_relax();
        }
        if (mir->status != 0) break;
        if (hipStreamQuery(st) == hipSuccess && mir->status == 0 && mir->it + 1 < queued - kBatch)
            return kanode_internal_fail(h, KANODE_ERR_HIP, "Tsit5 (device loop): the stream drained without progress");
    }
    SOLVE_HIP(h, hipStreamSynchronize(st));
    const kan::FkLoopCtl c = *(const kan::FkLoopCtl*)L.hmir;
    if (c.status == 2) return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "Tsit5: maxiters reached");
    s->ts.resize(c.step);
    s->dts.resize(c.step);
    if (c.step > 0) {
        SOLVE_HIP(h, hipMemcpy(s->ts.data(), L.ts, c.step * sizeof(double), hipMemcpyDeviceToHost));
        SOLVE_HIP(h, hipMemcpy(s->dts.data(), L.ts + L.cap, c.step * sizeof(double), hipMemcpyDeviceToHost));
    }
    for (int64_t i = 0; i < c.step && si < n_save; ++i)
        SOLVE_TRY(saveat_in_step<double>(h, s, i, s->ts[i], s->dts[i], nullptr, saveat, n_save, si, u_save, st));
    if (stats) {
        stats->naccept = c.step;
        stats->nreject = c.nreject;
        stats->nf = 6 * c.it + 1;
    }
    done = true;
    return KANODE_OK;
}

// ---- the adaptive Fisher-KPP adjoint with its step control on the device (kan_adjloop.hpp) ----------------
// adjoint_t's loop for the combined adaptive rows step (KANODE_OPT_FK_DEVICE_LOOP): one attempt = the rows
// launch + the finish launch, whose last workgroup runs the controller and plans the next attempt; the host
// queues attempts in batches and only polls the mapped mirror of the state.  A step landing on a saveat stop
// pauses the loop: the host drains the stream, takes the stop (take_stop: the jump and the FSAL
// re-evaluation, as its own loop), plans the next attempt and resumes.  On return the loop's variables hold
// adjoint_t's values at its end.
template <class TakeStop>
kanode_status adjoint_fk_loop(kanode_handle* h, const void* p, kanode_solution* s, const kanode_solver_options& o,
                              const std::vector<double>& stops, double* slab, int64_t grid, void* const* lam,
                              void* const* kl, void* const* mu, void* const* km, double& hstep, double& qold,
                              double& tau, size_t& si, int64_t& naccept, int64_t& nreject, int64_t& it, int64_t& nf,
                              int& lcur, int& mcur, std::vector<double>* hrec, TakeStop& take_stop, hipStream_t st) {
    constexpr int64_t kBatch = 16;
    const int64_t nsteps = (int64_t)s->ts.size(), P = kanode_param_length(h), nst = (int64_t)stops.size();
    auto& A = s->aloop;
    // device copies: forward slot table | ts | dts | stops, then the error terms [1 + P]
    const size_t meta = (size_t)(3 * nsteps + nst + 1 + P + 8) * sizeof(double);
    if (A.meta_bytes < meta) {
        SOLVE_HIP(h, hipStreamSynchronize(st));
        if (A.meta) (void)hipFree(A.meta);
        A.meta = nullptr;
        A.meta_bytes = 0;
        SOLVE_TRY(dev_alloc(h, &A.meta, meta, "adjoint loop tables"));
        A.meta_bytes = meta;
    }
    if (!A.ctl) {
        SOLVE_TRY(dev_alloc(h, (void**)&A.ctl, sizeof(kan::AdjLoopCtl), "adjoint loop state"));
        SOLVE_TRY(dev_alloc(h, (void**)&A.plan, 2 * sizeof(kan::AdjLoopPlan), "adjoint loop plans"));
        SOLVE_TRY(dev_alloc(h, (void**)&A.arrive, 64, "adjoint loop counter"));
        SOLVE_HIP(h, hipHostMalloc((void**)&A.hmir, sizeof(kan::AdjLoopCtl), hipHostMallocMapped | hipHostMallocCoherent));
        SOLVE_HIP(h, hipHostGetDevicePointer((void**)&A.dmir, A.hmir, 0));
        SOLVE_HIP(h, hipHostMalloc((void**)&A.hplan, sizeof(kan::AdjLoopPlan) + sizeof(kan::AdjLoopCtl)));
    }
    void** dslots = (void**)A.meta;
    double* dts_ = (double*)A.meta + nsteps;   // [ts | dts]
    double* dstops = dts_ + 2 * nsteps;
    double* dout = dstops + nst;
    {
        std::vector<char> host((3 * nsteps + nst) * sizeof(double));
        std::memcpy(host.data(), s->slots.data(), nsteps * sizeof(void*));
        std::memcpy(host.data() + nsteps * sizeof(double), s->ts.data(), nsteps * sizeof(double));
        std::memcpy(host.data() + 2 * nsteps * sizeof(double), s->dts.data(), nsteps * sizeof(double));
        std::memcpy(host.data() + 3 * nsteps * sizeof(double), stops.data(), nst * sizeof(double));
        SOLVE_HIP(h, hipStreamSynchronize(st));
        SOLVE_HIP(h, hipMemcpy(A.meta, host.data(), host.size(), hipMemcpyHostToDevice));
    }
    SOLVE_HIP(h, hipMemsetAsync(A.arrive, 0, sizeof(unsigned), st));
    kan::AdjLoopArgs la{};
    la.ctl = A.ctl;
    la.mirror = A.dmir;
    la.plan = A.plan;
    la.arrive = A.arrive;
    for (int i = 0; i < 2; ++i) {
        la.lam[i] = (double*)lam[i];
        la.mu[i] = (double*)mu[i];
    }
    for (int j = 0; j < 7; ++j) {
        la.kl[j] = (double*)kl[j];
        la.km[j] = (double*)km[j];
    }
    la.slots = dslots;
    la.fts = dts_;
    la.fdts = dts_ + nsteps;
    la.nsteps = nsteps;
    la.slab = slab;
    la.grid = grid;
    la.P = P;
    la.n = s->n;
    la.out = dout;
    la.stops = dstops;
    la.nstops = nst;
    la.tf = s->tf;
    la.TT = s->tf - s->t0;
    la.abstol = o.abstol;
    la.reltol = o.reltol;
    la.dtmin = o.dtmin;
    la.beta1 = o.beta1;
    la.beta2 = o.beta2;
    la.gamma = o.gamma;
    la.qmin = o.qmin;
    la.qmax = o.qmax;
    la.qoldinit = o.qoldinit;
    la.ntot = (double)(s->n + P);
    la.maxiters = o.maxiters;
    if (hrec) {
        const int64_t cap = 4 * nsteps + 1024;
        if (s->hs_cap < cap) {
            if (s->hs_dev) SOLVE_HIP(h, hipFree(s->hs_dev));
            s->hs_dev = nullptr;
            s->hs_cap = 0;
            SOLVE_HIP(h, hipMalloc((void**)&s->hs_dev, (size_t)cap * sizeof(double)));
            s->hs_cap = cap;
        }
        la.hs = s->hs_dev;
        la.hs_cap = s->hs_cap;
    }
    // the host's view of the forward steps for the plans it builds (the same values as the device's)
    struct HostFw {
        const kanode_solution* s;
        double ts(int64_t i) const { return s->ts[i]; }
        double dts(int64_t i) const { return s->dts[i]; }
        const void* slot(int64_t i) const { return s->u(i); }
    } hfw{s};
    kan::AdjLoopCtl c{};
    c.tau = tau;
    c.h = hstep;
    c.qold = qold;
    c.si = (int64_t)si;
    c.naccept = naccept;
    c.nreject = nreject;
    c.it = it;
    c.nf = nf;
    c.fi = nsteps - 1;
    c.lc = lcur;
    c.mc = mcur;
    c.fs = 0;
    const volatile kan::AdjLoopCtl* mir = A.hmir;
    for (;;) {
        // (re)start at c: the loop top, the attempt's plan, the state (the stream is drained: the staging is free)
        kan::adj_loop_top(la, c, stops[(size_t)c.si]);   // (la.stops is the device copy)
        if (c.status != 0) break;
        kan::AdjLoopPlan* hp = (kan::AdjLoopPlan*)A.hplan;
        kan::adj_loop_plan(la, c, *hp, hfw);
        std::memcpy((char*)A.hplan + sizeof(kan::AdjLoopPlan), &c, sizeof(c));
        *A.hmir = c;
        // both buffers: the device rewrites only a plan's step-dependent fields (adj_finish_loop_kernel)
        for (int b = 0; b < 2; ++b)
            SOLVE_HIP(h, hipMemcpyAsync(A.plan + b, hp, sizeof(kan::AdjLoopPlan), hipMemcpyHostToDevice, st));
        SOLVE_HIP(h, hipMemcpyAsync(A.ctl, (char*)A.hplan + sizeof(kan::AdjLoopPlan), sizeof(c), hipMemcpyHostToDevice,
                                    st));
        const int64_t base = c.it;
        int64_t queued = 0;
        for (;;) {
            for (int64_t i = 0; i < kBatch; ++i) SOLVE_TRY(kanode_internal_fk_adjoint_loop(h, p, &la, s->batch, st));
            queued += kBatch;
            for (uint64_t k = 1; mir->status == 0 && mir->it < base + queued - kBatch; ++k) {
                if ((k & 255) == 0) {
                    const hipError_t q = hipStreamQuery(st);
                    if (q == hipSuccess) break;
                    if (q != hipErrorNotReady) SOLVE_HIP(h, q);
                }
                cpu_relax();
            }
            if (mir->status != 0) break;
            if (hipStreamQuery(st) == hipSuccess && mir->status == 0 && mir->it < base + queued - kBatch)
                return kanode_internal_fail(h, KANODE_ERR_HIP, "adjoint Tsit5 (device loop): the stream drained without progress");
        }
        SOLVE_HIP(h, hipStreamSynchronize(st));
        c = *(const kan::AdjLoopCtl*)A.hmir;
        if (c.status != 3) break;
        // paused on stops[si]: the stop's jump and FSAL re-evaluation on the host, then the next stop
        tau = c.tau;
        si = (size_t)c.si;
        lcur = c.lc;
        nf = c.nf;
        SOLVE_TRY(take_stop(c.fs ? kl[6] : kl[0], c.fs ? km[6] : km[0]));
        SOLVE_TRY(kanode_internal_vjp_flush(h, st));
        c.lc = lcur;
        c.si = (int64_t)si;
        c.nf = nf;
        c.status = 0;
    }
    if (c.status == 2) {
        it = o.maxiters;   // (adjoint_t reports it)
        tau = c.tau;
        return KANODE_OK;
    }
    tau = c.tau;
    hstep = c.h;
    qold = c.qold;
    si = (size_t)c.si;
    naccept = c.naccept;
    nreject = c.nreject;
    it = c.it;
    nf = c.nf;
    lcur = c.lc;
    mcur = c.mc;
    if (hrec && la.hs) {
        hrec->resize((size_t)std::min(naccept, la.hs_cap));
        if (!hrec->empty())
            SOLVE_HIP(h, hipMemcpy(hrec->data(), la.hs, hrec->size() * sizeof(double), hipMemcpyDeviceToHost));
    }
    return KANODE_OK;
}

// ---- InterpolatingAdjoint -----------------------------------------------------------
template <typename T>
kanode_status adjoint_t(kanode_handle* h, const void* p, kanode_solution* s, const void* dl_du, void* du0, void* dp,
                        const kanode_solver_options& o, kanode_solve_stats* stats, hipStream_t st) {
    const int64_t n = s->n, P = kanode_param_length(h);
    const size_t sb = s->state_bytes(), pb = (size_t)P * s->esize;
    const int64_t nsteps = (int64_t)s->ts.size();
    if (nsteps < 1) return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "adjoint: the forward solve took no steps");
    // scratch: lam[2], kl[7] (states), mu[2], km[7] (parameter vectors)
    const size_t need = 9 * sb + 9 * pb + 256;
    if (s->adj_bytes < need) {
        if (capturing(st)) return kanode_internal_fail(h, KANODE_ERR_CAPTURE, "adjoint scratch grows during capture");
        SOLVE_HIP(h, hipStreamSynchronize(st));
        if (s->adj) SOLVE_HIP(h, hipFree(s->adj));
        s->adj = nullptr;
        s->adj_bytes = 0;
        if (hipMalloc(&s->adj, need) != hipSuccess) {
            (void)hipGetLastError();
            return kanode_internal_fail(h, KANODE_ERR_ALLOC, "adjoint scratch: out of device memory");
        }
        s->adj_bytes = need;
    }
    auto align = [](size_t x) { return (x + 255) & ~(size_t)255; };
    char* w = (char*)s->adj;
    void *lam[2], *kl[7], *mu[2], *km[7];
    for (auto& x : lam) { x = w; w += sb; }
    for (auto& x : kl) { x = w; w += sb; }
    w = (char*)s->adj + align(9 * sb);
    for (auto& x : mu) { x = w; w += pb; }
    for (auto& x : km) { x = w; w += pb; }

    const double t0 = s->t0, tf = s->tf, TT = tf - t0;
    const double eps = 1e-12 * std::max(1.0, std::fabs(tf));
    // jumps: distinct saveat values, each with the rows of dl_du that land on it
    struct Jump { double ts; std::vector<int64_t> rows; bool live; };
    std::vector<Jump> jumps;
    for (int64_t j = 0; j < (int64_t)s->saveat.size(); ++j) {
        auto f = std::find_if(jumps.begin(), jumps.end(), [&](const Jump& x) { return x.ts == s->saveat[j]; });
        if (f == jumps.end()) jumps.push_back({s->saveat[j], {j}, true});
        else f->rows.push_back(j);
    }
    auto add_jump = [&](Jump& jm, void* l) -> kanode_status {
        for (int64_t r : jm.rows) {
            const void* g[1] = {(const char*)dl_du + r * sb};
            const double one = 1.0;
            SOLVE_TRY(lincomb<T>(h, l, 1, g, &one, l, n, st));
        }
        jm.live = false;
        return KANODE_OK;
    };
    SOLVE_HIP(h, hipMemsetAsync(lam[0], 0, sb, st));
    SOLVE_HIP(h, hipMemsetAsync(mu[0], 0, pb, st));
    if (dl_du) {
        for (auto& jm : jumps)
            if (jm.live && jm.ts == tf) SOLVE_TRY(add_jump(jm, lam[0]));
    } else {
        for (auto& jm : jumps) jm.live = false;
    }
    std::vector<double> stops;
    for (auto& jm : jumps)
        if (jm.live && t0 + eps < jm.ts && jm.ts < tf - eps) stops.push_back(tf - jm.ts);
    std::sort(stops.begin(), stops.end());
    stops.push_back(TT);

    // adjoint RHS at τ: u(tf - τ) from the dense output, λ stage input l + Σ lc_j lks_j
    // (-> lam_out), lamJ = λsᵀ∂f/∂u, dpo = λsᵀ∂f/∂p; ec != NULL adds the λ error total -> err
    // defer: the dp / error reductions of this stage wait for flush() (one launch per step)
    kanode_internal_vjp_discard(h);   // nothing pending from an earlier failed call
    int lam_parts = 0;                // > 0: the step's λ error as that many partials in hparts
    struct PartsOff {                 // the handle must not keep the solution's buffer past this call
        kanode_handle* h;
        ~PartsOff() { kanode_internal_set_err_parts(h, nullptr, nullptr); }
    } parts_off{h};
    if (o.adaptive && s->mparts) kanode_internal_set_err_parts(h, s->mparts, &lam_parts);
    auto adj_rhs = [&](double tau, const void* l, int nl, void* const* lks, const double* lc, void* lamJ, void* dpo,
                       void* lam_out, const double* ec, double* err, bool defer = false) -> kanode_status {
        const double t = tf - tau;
        int64_t i = (int64_t)(std::upper_bound(s->ts.begin(), s->ts.end(), t) - s->ts.begin()) - 1;
        i = std::max<int64_t>(0, std::min<int64_t>(nsteps - 1, i));
        const double dti = s->dts[i];
        const double theta = std::min(1.0, std::max(0.0, (t - s->ts[i]) / dti));
        kanode_stage su;
        if (s->qform) {   // u_i + Σ_m θ^m Q_m
            const double c[4] = {theta, theta * theta, theta * theta * theta, theta * theta * theta * theta};
            void* qs[4] = {s->q(i, 1), s->q(i, 2), s->q(i, 3), s->q(i, 4)};
            su = make_stage(4, qs, c);
        } else {
            double c[7];
            interp_weights(theta, c);
            for (double& x : c) x *= dti;
            void* ks[7];
            for (int j = 0; j < 7; ++j) ks[j] = s->k(i, j + 1);
            su = make_stage(7, ks, c);
        }
        kanode_stage sl = make_stage(nl, lks, lc);
        sl.y_out = lam_out;
        if (ec) {
            sl.want_error = 1;
            for (int j = 0; j <= nl; ++j) sl.ec[j] = ec[j];
            sl.abstol = o.abstol;
            sl.reltol = o.reltol;
            sl.error_sumsq = err;
        }
        return kanode_internal_vjp_stage(h, p, s->u(i), &su, l, &sl, lamJ, dpo, true, s->batch, st, nullptr, nullptr,
                                         defer);
    };
    const int64_t ntot = n + P;
    int lcur = 0, mcur = 0;   // lam[lcur], mu[mcur] hold λ, μ (a saveat jump flips λ alone)
    SOLVE_TRY(adj_rhs(0.0, lam[lcur], 0, nullptr, nullptr, kl[0], km[0], nullptr, nullptr, nullptr));
    int64_t nf = 1;
    double hstep = o.dt;
    if (o.adaptive && !(o.dt > 0)) {
        // Hairer-Wanner on the augmented state [λ; μ] (kanode/adjoint.py)
        const double one = 1.0;
        SOLVE_TRY(wsumsq<T>(h, lam[lcur], lam[lcur], 0, nullptr, &one, lam[lcur], o.abstol, o.reltol, n, s->dscal + 0, st));
        SOLVE_TRY(wsumsq<T>(h, mu[mcur], mu[mcur], 0, nullptr, &one, mu[mcur], o.abstol, o.reltol, P, s->dscal + 1, st));
        SOLVE_TRY(wsumsq<T>(h, lam[lcur], lam[lcur], 0, nullptr, &one, kl[0], o.abstol, o.reltol, n, s->dscal + 2, st));
        SOLVE_TRY(wsumsq<T>(h, mu[mcur], mu[mcur], 0, nullptr, &one, km[0], o.abstol, o.reltol, P, s->dscal + 3, st));
        SOLVE_TRY(read_scalars(h, s, 4, st));
        const double d0 = std::sqrt((s->hscal[0] + s->hscal[1]) / (double)ntot);
        const double d1 = std::sqrt((s->hscal[2] + s->hscal[3]) / (double)ntot);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        h0 = std::min(h0, TT);
        void* k1l[1] = {kl[0]};
        SOLVE_TRY(adj_rhs(h0, lam[lcur], 1, k1l, &h0, kl[1], km[1], nullptr, nullptr, nullptr));
        ++nf;
        const double e2[2] = {1.0, -1.0};
        const void* a1[1] = {kl[1]};
        const void* b1[1] = {km[1]};
        SOLVE_TRY(wsumsq<T>(h, lam[lcur], lam[lcur], 1, a1, e2, kl[0], o.abstol, o.reltol, n, s->dscal + 0, st));
        SOLVE_TRY(wsumsq<T>(h, mu[mcur], mu[mcur], 1, b1, e2, km[0], o.abstol, o.reltol, P, s->dscal + 1, st));
        SOLVE_TRY(read_scalars(h, s, 2, st));
        const double d2 = std::sqrt((s->hscal[0] + s->hscal[1]) / (double)ntot) / h0;
        const double mx = std::max(d1, d2);
        const double h1 = mx <= 1e-15 ? std::max(1e-6, h0 * 1e-3) : std::pow(0.01 / mx, 1.0 / 5.0);
        hstep = std::min(std::min(100 * h0, h1), TT);
    } else if (!(hstep > 0)) {
        return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "fixed-step adjoint needs opt->dt > 0");
    }
    double qold = o.qoldinit, tau = 0.0;
    size_t si = 0;
    int64_t naccept = 0, nreject = 0, it = 0;
    std::vector<double>* hrec = kanode_internal_adjoint_steps(h);
    if (hrec) hrec->clear();
    // a small chain whose steps run as one launch each: a stop's jump and FSAL re-evaluation ride in the next
    // step's launch (ChainAdjStep::fsal) instead of a launch of their own; `pend` holds them until that step
    // is accepted (a rejected attempt forms them again)
    const bool fold_stops = !s->qform && kanode_internal_chain_adjoint_step_ok(h);
    struct {
        bool on = false;
        int ng = 0;
        const void* g[8];
    } pend;
    // A step that landed on stops[si] (tau == stops[si]): the saveat jump there, if any, and the next stop.
    // k0l / k0m: the current kλ_1 / kμ_1 buffers (the FSAL re-evaluation's outputs).
    auto take_stop = [&](void* k0l, void* k0m) -> kanode_status {
        const double tsv = tf - tau;
        Jump* key = nullptr;
        for (auto& jm : jumps)
            if (jm.live && (!key || std::fabs(jm.ts - tsv) < std::fabs(key->ts - tsv))) key = &jm;
        if (key && std::fabs(key->ts - tsv) <= eps && si + 1 < stops.size()) {
            if (fold_stops && key->rows.size() <= 8) {
                pend.on = true;
                pend.ng = 0;
                for (int64_t r : key->rows) pend.g[pend.ng++] = (const char*)dl_du + r * sb;
                key->live = false;
            } else if (key->rows.size() <= (size_t)KANODE_MAX_STAGES) {
                // callback λ += ∂L/∂u(t_j) and the FSAL re-evaluation (u_modified!) as ONE adjoint
                // stage: λs = λ + Σ_r 1·g_r (the lincombs' fma order) -> λ_new, kλ_1 = λsᵀJ at λs
                void* g[KANODE_MAX_STAGES];
                double ones[KANODE_MAX_STAGES];
                int ng = 0;
                for (int64_t r : key->rows) {
                    g[ng] = (char*)dl_du + r * sb;
                    ones[ng++] = 1.0;
                }
                key->live = false;
                // (deferred where the surrogate pair's stages run lazily: its second launch then runs
                // together with the next step's first stage, whose λs starts from this kλ_1)
                SOLVE_TRY(adj_rhs(tau, lam[lcur], ng, g, ones, k0l, k0m, lam[lcur ^ 1], nullptr, nullptr,
                                  kanode_internal_pair_lazy(h)));
                lcur ^= 1;
            } else {
                SOLVE_TRY(add_jump(*key, lam[lcur]));                   // callback: λ += ∂L/∂u(t_j)
                SOLVE_TRY(adj_rhs(tau, lam[lcur], 0, nullptr, nullptr, k0l, k0m, nullptr, nullptr, nullptr));
            }
            ++nf;                                                      // u_modified!: FSAL re-evaluated
        }
        si = std::min(si + 1, stops.size() - 1);
        return KANODE_OK;
    };
    bool dev_loop = false;
    if constexpr (std::is_same<T, double>::value) {
        if (s->qform && o.adaptive && o.control == 0 && !capturing(st) && s->record) {
            double* lslab = nullptr;
            int64_t lgrid = 0;
            SOLVE_TRY(kanode_internal_fk_adjoint_loop_geometry(h, s->batch, st, dev_loop, &lslab, &lgrid));
            if (dev_loop) {
                SOLVE_TRY(adjoint_fk_loop(h, p, s, o, stops, lslab, lgrid, lam, kl, mu, km, hstep, qold, tau, si,
                                          naccept, nreject, it, nf, lcur, mcur, hrec, take_stop, st));
            }
        }
    }
    for (; !dev_loop && it < o.maxiters; ++it) {
        if (tau >= TT - 1e-14 * std::max(1.0, TT)) break;
        hstep = std::min(hstep, stops[si] - tau);
        bool fused_step = false;   // Fisher-KPP table path, Q-form dense output: the six stages in one launch
        // combined (fixed step, kanode_internal_fk_adjoint_step): the step's reduction launch reduces the
        // stage moments through the combinations the step consumes and writes μ_new itself (AdjMuUpdate)
        // and the FSAL kμ_7 into km[6]; km[1..5] are NOT written on such a step and hold stale values,
        // so nothing may read them when `combined` is set
        bool combined = false;
        bool finished = false;     // adaptive step: μ_new, kμ_7 and the μ error terms formed by the finish launch
        if (o.adaptive && s->mscal) arm_ctl(s->hscal, kScalars);
        lam_parts = 0;
        if (s->qform) {
            kan::AdjStepArgs a{};
            for (int j = 0; j < 7; ++j) a.kl[j] = (double*)kl[j];
            for (int i = 0; i < 6; ++i) {
                for (int j = 0; j <= i; ++j) a.a[i][j] = hstep * TA[i][j];
                const double t = tf - (i == 5 ? tau + hstep : tau + TC[i] * hstep);
                int64_t fi = (int64_t)(std::upper_bound(s->ts.begin(), s->ts.end(), t) - s->ts.begin()) - 1;
                fi = std::max<int64_t>(0, std::min<int64_t>(nsteps - 1, fi));
                const double th = std::min(1.0, std::max(0.0, (t - s->ts[fi]) / s->dts[fi]));
                a.su_u[i] = (const double*)s->u(fi);
                for (int m = 0; m < 4; ++m) a.su_q[i][m] = (const double*)s->q(fi, m + 1);
                a.su_c[i][0] = th;
                a.su_c[i][1] = th * th;
                a.su_c[i][2] = th * th * th;
                a.su_c[i][3] = th * th * th * th;
            }
            for (int j = 0; j < 7; ++j) a.ec[j] = hstep * BT[j];
            a.abstol = o.abstol;
            a.reltol = o.reltol;
            a.lam = (const double*)lam[lcur];
            a.lam_out = (double*)lam[lcur ^ 1];
            void* kms[6] = {km[1], km[2], km[3], km[4], km[5], km[6]};
            const AdjMuUpdate mup{(const double*)mu[mcur], (double*)mu[mcur ^ 1], (const double*)km[0], hstep * TA[5][0]};
            AdjAdaptiveFinish af{};
            af.mu = (const double*)mu[mcur];
            af.mu_new = (double*)mu[mcur ^ 1];
            af.km1 = (const double*)km[0];
            af.km7 = (double*)km[6];
            for (int j = 0; j < 6; ++j) af.a6[j] = hstep * TA[5][j];
            for (int j = 0; j < 7; ++j) af.bt[j] = hstep * BT[j];
            af.abstol = o.abstol;
            af.reltol = o.reltol;
            af.out = ctl(s) + 8;
            af.done = &finished;
            SOLVE_TRY(kanode_internal_fk_adjoint_step(h, p, &a, kms, o.adaptive ? ctl(s) + 0 : nullptr, s->batch,
                                                      st, fused_step, &combined, &mup,
                                                      o.adaptive && P <= KANODE_MAX_GRID + 1 ? &af : nullptr));
        } else {
            // a small chain: the six stages in one launch (kd_chain_vjp_step_kernel), kμ_2..kμ_7 into km[1..6] and
            // the λ error into slot 0 by its reduction launch: the same values as the six adj_rhs calls below
            kan::ChainAdjStep<T> ca{};
            for (int i = 0; i < 6; ++i) {
                for (int j = 0; j < 6; ++j) ca.a[i][j] = j <= i ? hstep * TA[i][j] : 0.0;
                const double t = tf - (i == 5 ? tau + hstep : tau + TC[i] * hstep);
                int64_t fi = (int64_t)(std::upper_bound(s->ts.begin(), s->ts.end(), t) - s->ts.begin()) - 1;
                fi = std::max<int64_t>(0, std::min<int64_t>(nsteps - 1, fi));
                const double dti = s->dts[fi];
                const double th = std::min(1.0, std::max(0.0, (t - s->ts[fi]) / dti));
                double c[7];
                interp_weights(th, c);
                ca.su_u[i] = (const T*)s->u(fi);
                for (int q = 0; q < 7; ++q) {
                    ca.su_k[i][q] = (const T*)s->k(fi, q + 1);
                    ca.su_c[i][q] = c[q] * dti;
                }
            }
            for (int j = 0; j < 7; ++j) ca.ec[j] = hstep * BT[j];
            ca.abstol = o.abstol;
            ca.reltol = o.reltol;
            ca.lam = (const T*)lam[lcur];
            ca.lam_out = (T*)lam[lcur ^ 1];
            ca.kl1 = (const T*)kl[0];
            ca.kl7 = (T*)kl[6];
            ca.want_error = o.adaptive ? 1 : 0;
            if (pend.on) {   // the stop's jump and kλ_1 / kμ_1 at τ (adj_rhs's dense output there)
                const double t = tf - tau;
                int64_t fi = (int64_t)(std::upper_bound(s->ts.begin(), s->ts.end(), t) - s->ts.begin()) - 1;
                fi = std::max<int64_t>(0, std::min<int64_t>(nsteps - 1, fi));
                const double dti = s->dts[fi];
                const double th = std::min(1.0, std::max(0.0, (t - s->ts[fi]) / dti));
                double c[7];
                interp_weights(th, c);
                ca.fsal = 1;
                ca.njump = pend.ng;
                for (int r = 0; r < pend.ng; ++r) ca.jump[r] = (const T*)pend.g[r];
                ca.j_u = (const T*)s->u(fi);
                for (int q = 0; q < 7; ++q) {
                    ca.j_k[q] = (const T*)s->k(fi, q + 1);
                    ca.j_c[q] = c[q] * dti;
                }
            }
            void* kms[7] = {km[1], km[2], km[3], km[4], km[5], km[6], km[0]};
            SOLVE_TRY(kanode_internal_chain_adjoint_step(h, p, &ca, kms, o.adaptive ? ctl(s) + 0 : nullptr, s->batch, st,
                                                         fused_step));
            if (pend.on && !fused_step) {   // (not launched after all: the stop's own stage, as take_stop would)
                double ones[8];
                void* g[8];
                for (int r = 0; r < pend.ng; ++r) {
                    ones[r] = 1.0;
                    g[r] = const_cast<void*>(pend.g[r]);
                }
                SOLVE_TRY(adj_rhs(tau, lam[lcur], pend.ng, g, ones, kl[0], km[0], lam[lcur ^ 1], nullptr, nullptr));
                lcur ^= 1;
                pend.on = false;
            }
        }
        for (int i = 0; i < 6 && !fused_step; ++i) {
            double lc[6];
            for (int j = 0; j <= i; ++j) lc[j] = hstep * TA[i][j];
            if (i == 5) {
                double ec[7];
                for (int j = 0; j < 7; ++j) ec[j] = hstep * BT[j];
                SOLVE_TRY(adj_rhs(tau + hstep, lam[lcur], 6, kl, lc, kl[6], km[6], lam[lcur ^ 1], o.adaptive ? ec : nullptr,
                                  ctl(s) + 0, true));
            } else {
                SOLVE_TRY(adj_rhs(tau + TC[i] * hstep, lam[lcur], i + 1, kl, lc, kl[i + 1], km[i + 1], nullptr,
                                  nullptr, nullptr, true));
            }
        }
        if (!fused_step) SOLVE_TRY(kanode_internal_vjp_flush(h, st));   // km[1..6] and the λ error
        nf += 6;
        double a6[6];
        for (int j = 0; j < 6; ++j) a6[j] = hstep * TA[5][j];
        int fin_blocks = 0;
        if (combined || finished) {
            // μ_new = μ + h a_61 km_1 + (the step's combined Σ_{j>=2} h a_6j km_j): formed by the step's
            // reduction launch (kanode_internal_fk_adjoint_step: AdjMuUpdate, or AdjAdaptiveFinish)
        } else if (o.adaptive) {
            // μ_new and the μ error partials in one launch (adj_step_finish_kernel)
            kan::AdjStepFinish<T> f{};
            for (int j = 0; j < 7; ++j) {
                f.km[j] = (const T*)km[j];
                f.b[j] = hstep * BT[j];
            }
            for (int j = 0; j < 6; ++j) f.a[j] = a6[j];
            f.abstol = o.abstol;
            f.reltol = o.reltol;
            SOLVE_HIP(h, kan::launch_adj_step_finish<T>((const T*)mu[mcur], (T*)mu[mcur ^ 1], f, ctl(s) + 16, P, &fin_blocks,
                                                        st));
        } else {
            SOLVE_TRY(lincomb<T>(h, mu[mcur], 6, km, a6, mu[mcur ^ 1], P, st));   // μ_new = μ + h Σ a_6j km_j
        }
        double hnew = hstep;
        if (o.adaptive) {
            double sumsq = 0.0;
            if (finished) {   // the λ sum and the P μ terms in one read, summed here in order
                if (s->mscal) SOLVE_TRY(wait_ctl(h, st, {{s->hscal + 8, (int)(1 + P)}}));
                else SOLVE_TRY(read_ctl(h, s, 8, (int)(1 + P), st));
                double mus = 0.0;
                for (int64_t q = 0; q < P; ++q) mus += s->hscal[9 + q];
                sumsq = s->hscal[8] + mus;
            } else if (lam_parts > 0) {   // the λ error partials (hparts) and the μ partials (slots 16..)
                SOLVE_TRY(wait_ctl(h, st, {{s->hparts, lam_parts}, {s->hscal + 16, fin_blocks}}));
                double ls = 0.0, mus = 0.0;
                for (int b = 0; b < lam_parts; ++b) ls += s->hparts[b];
                for (int b = 0; b < fin_blocks; ++b) mus += s->hscal[16 + b];
                arm_ctl(s->hparts, lam_parts);
                sumsq = ls + mus;
            } else {   // the λ total (slot 0) and the μ partials (slots 16..) in one read
                if (s->mscal) SOLVE_TRY(wait_ctl(h, st, {{s->hscal, 1}, {s->hscal + 16, fin_blocks}}));
                else SOLVE_TRY(read_ctl(h, s, 0, 16 + fin_blocks, st));
                double mus = 0.0;
                for (int b = 0; b < fin_blocks; ++b) mus += s->hscal[16 + b];
                sumsq = s->hscal[0] + mus;
            }
            const double EEst = std::sqrt(sumsq / (double)ntot);
            const double q11 = EEst > 0 ? std::pow(EEst, o.beta1) : 0.0;
            if (EEst > 1.0 && hstep > o.dtmin) {
                ++nreject;
                hstep = hstep / std::min(1.0 / o.qmin, q11 / o.gamma);
                continue;
            }
            double q = q11 / std::pow(qold, o.beta2);
            q = std::max(1.0 / o.qmax, std::min(1.0 / o.qmin, q / o.gamma));
            hnew = q > 0 ? hstep / q : hstep * o.qmax;
            qold = std::max(EEst, o.qoldinit);
        }
        tau = tau + hstep;
        lcur ^= 1;
        mcur ^= 1;
        pend.on = false;           // (the folded stop, if any, is part of this accepted step)
        std::swap(kl[0], kl[6]);   // FSAL
        std::swap(km[0], km[6]);
        if (hrec) hrec->push_back(hstep);
        ++naccept;
        if (std::fabs(tau - stops[si]) <= 1e-12 * std::max(1.0, TT)) {
            tau = stops[si];
            SOLVE_TRY(take_stop(kl[0], km[0]));
        }
        hstep = hnew;
    }
    SOLVE_TRY(kanode_internal_vjp_flush(h, st));   // (a deferred stage's last launch)
    if (pend.on) {   // (a stop no step followed: maxiters) its jump still belongs to λ
        for (int r = 0; r < pend.ng; ++r) {
            const double one = 1.0;
            SOLVE_TRY(lincomb<T>(h, lam[lcur], 1, &pend.g[r], &one, lam[lcur], n, st));
        }
    }
    if (it == o.maxiters && !(tau >= TT - 1e-14 * std::max(1.0, TT)))
        return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "adjoint Tsit5: maxiters reached");
    for (auto& jm : jumps)   // a saveat at t0 adds to dL/du0 only
        if (jm.live && std::fabs(jm.ts - t0) <= eps) SOLVE_TRY(add_jump(jm, lam[lcur]));
    if (du0) SOLVE_HIP(h, hipMemcpyAsync(du0, lam[lcur], sb, hipMemcpyDeviceToDevice, st));
    if (dp) SOLVE_HIP(h, hipMemcpyAsync(dp, mu[mcur], pb, hipMemcpyDeviceToDevice, st));
    if (stats) {
        stats->naccept = naccept;
        stats->nreject = nreject;
        stats->nf = nf;
    }
    return KANODE_OK;
}

// The stops, saveat jump groups and options of the one-launch adjoints (adjoint_t's semantics): the jump
// groups and stops go to the solution's adj_meta buffer, everything else into a (rec, k1_0, ts, dts and
// nsteps are the caller's).
kanode_status one_launch_adj_args(kanode_handle* h, kanode_solution* s, const void* dl_du, void* du0, void* dp,
                                  const kanode_solver_options& o, kan::ChainAdjointArgs& a, hipStream_t st) {
    if (!o.adaptive && !(o.dt > 0))
        return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "fixed-step adjoint needs opt->dt > 0");
    const double t0 = s->t0, tf = s->tf, TT = tf - t0;
    const double eps = 1e-12 * std::max(1.0, std::fabs(tf));
    // the jump groups of adjoint_t: distinct saveat values and their dl_du rows
    struct Jump { double ts; std::vector<int32_t> rows; };
    std::vector<Jump> jumps;
    for (int64_t jx = 0; jx < (int64_t)s->saveat.size(); ++jx) {
        auto f = std::find_if(jumps.begin(), jumps.end(), [&](const Jump& x) { return x.ts == s->saveat[jx]; });
        if (f == jumps.end()) jumps.push_back({s->saveat[jx], {(int32_t)jx}});
        else f->rows.push_back((int32_t)jx);
    }
    std::vector<std::pair<double, int>> st_j;   // (τ of the stop, jump)
    std::vector<int32_t> init_rows, final_rows;
    if (dl_du) {
        for (int q = 0; q < (int)jumps.size(); ++q) {
            const Jump& jm = jumps[q];
            if (jm.ts == tf) init_rows.insert(init_rows.end(), jm.rows.begin(), jm.rows.end());
            else if (t0 + eps < jm.ts && jm.ts < tf - eps) st_j.push_back({tf - jm.ts, q});
            else if (std::fabs(jm.ts - t0) <= eps) final_rows.insert(final_rows.end(), jm.rows.begin(), jm.rows.end());
        }
    }
    std::sort(st_j.begin(), st_j.end());
    std::vector<double> stops;
    std::vector<int32_t> rows(init_rows), off{0, (int32_t)init_rows.size()};
    for (auto& x : st_j) {
        stops.push_back(x.first);
        const Jump& jm = jumps[x.second];
        const bool hit = std::fabs(jm.ts - (tf - x.first)) <= eps;
        if (hit) rows.insert(rows.end(), jm.rows.begin(), jm.rows.end());
        off.push_back((int32_t)rows.size());
    }
    stops.push_back(TT);
    rows.insert(rows.end(), final_rows.begin(), final_rows.end());
    off.push_back((int32_t)rows.size());
    const int64_t ns = (int64_t)stops.size();
    // device copies: stops | joff | jrows
    const size_t bytes = ns * sizeof(double) + off.size() * sizeof(int32_t) + (rows.size() + 1) * sizeof(int32_t) + 64;
    auto& f = s->fused;
    if (f.adj_meta_bytes < bytes) {
        if (f.adj_meta) (void)hipFree(f.adj_meta);
        f.adj_meta = nullptr;
        f.adj_meta_bytes = 0;
        f.meta_last.clear();
        SOLVE_HIP(h, hipMalloc(&f.adj_meta, bytes));
        f.adj_meta_bytes = bytes;
    }
    std::vector<char> host(bytes, 0);
    double* dstops = (double*)f.adj_meta;
    int32_t* djoff = (int32_t*)((char*)f.adj_meta + ns * sizeof(double));
    int32_t* djrows = djoff + off.size();
    std::memcpy(host.data(), stops.data(), ns * sizeof(double));
    std::memcpy(host.data() + ns * sizeof(double), off.data(), off.size() * sizeof(int32_t));
    if (!rows.empty())
        std::memcpy(host.data() + ns * sizeof(double) + off.size() * sizeof(int32_t), rows.data(),
                    rows.size() * sizeof(int32_t));
    SOLVE_TRY(staged_upload(h, s, f.adj_meta, host.data(), bytes, st, &f.meta_last));
    if (!f.out) SOLVE_HIP(h, hipMalloc((void**)&f.out, 4 * sizeof(int64_t)));
    a = kan::ChainAdjointArgs{};
    a.t0 = t0;
    a.tf = tf;
    a.dt = o.dt;
    a.abstol = o.abstol;
    a.reltol = o.reltol;
    a.dtmin = o.dtmin;
    a.beta1 = o.beta1;
    a.beta2 = o.beta2;
    a.gamma = o.gamma;
    a.qmin = o.qmin;
    a.qmax = o.qmax;
    a.qoldinit = o.qoldinit;
    a.adaptive = o.adaptive ? 1 : 0;
    a.maxiters = o.maxiters;
    a.dl_du = dl_du;
    a.stops = dstops;
    a.nstops = ns;
    a.jrows = djrows;
    a.joff = djoff;
    a.du0 = du0;
    a.dp = dp;
    a.out = f.out;
    if (kanode_internal_adjoint_steps(h)) {
        const int64_t cap = 4 * (int64_t)s->ts.size() + 1024;
        if (s->hs_cap < cap) {
            if (s->hs_dev) SOLVE_HIP(h, hipFree(s->hs_dev));
            s->hs_dev = nullptr;
            s->hs_cap = 0;
            SOLVE_HIP(h, hipMalloc((void**)&s->hs_dev, (size_t)cap * sizeof(double)));
            s->hs_cap = cap;
        }
        a.hs = s->hs_dev;
        a.hs_cap = s->hs_cap;
    }
    return KANODE_OK;
}

// the step sizes a one-launch adjoint wrote (a.hs) into the handle's record
kanode_status fetch_adjoint_steps(kanode_handle* h, const kan::ChainAdjointArgs& a, int64_t naccept) {
    std::vector<double>* rec = kanode_internal_adjoint_steps(h);
    if (!rec || !a.hs) return KANODE_OK;
    rec->resize((size_t)std::min(naccept, a.hs_cap));
    if (!rec->empty()) SOLVE_HIP(h, hipMemcpy(rec->data(), a.hs, rec->size() * sizeof(double), hipMemcpyDeviceToHost));
    return KANODE_OK;
}

// ---- one-workgroup adjoint of a small chain (kd_chain_adjoint_kernel) ---------------------
// Needs the contiguous dense output of the one-workgroup forward solve; done = false when not
// covered (the host loop adjoint_t runs instead).
template <typename T>
kanode_status adjoint_fused_t(kanode_handle* h, const void* p, kanode_solution* s, const void* dl_du, void* du0,
                              void* dp, const kanode_solver_options& o, kanode_solve_stats* stats, hipStream_t st,
                              bool& done) {
    done = false;
    const int64_t nsteps = (int64_t)s->ts.size();
    if (o.control != 0 || capturing(st) || !s->slots_borrowed || nsteps < 1 ||
        !kanode_internal_chain_tsit5_ok(h, s->batch))
        return KANODE_OK;
    kan::ChainAdjointArgs a{};
    SOLVE_TRY(one_launch_adj_args(h, s, dl_du, du0, dp, o, a, st));
    auto& f = s->fused;
    a.rec = f.block;
    a.k1_0 = s->k1_0;
    a.ts = f.ts;
    a.dts = f.ts + f.cap;
    a.nsteps = nsteps;
    if (s->mscal) {   // (as solve_fused_t, spinning on the counters)
        a.out = (int64_t*)s->mscal;
        arm_ctl(s->hscal, 4);
    }
    bool launched = false;
    SOLVE_TRY(kanode_internal_chain_adjoint(h, p, s->batch, &a, st, launched));
    if (!launched) return KANODE_OK;
    if (!s->mscal) {
        SOLVE_HIP(h, hipMemcpyAsync(s->hscal, f.out, 4 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        SOLVE_HIP(h, hipStreamSynchronize(st));
    } else {
        SOLVE_TRY(wait_ctl(h, st, {{s->hscal, 4}}));
    }
    int64_t res[4];
    std::memcpy(res, s->hscal, sizeof(res));
    if (res[3] == 1) return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "adjoint Tsit5: maxiters reached");
    if (stats) {
        stats->naccept = res[0];
        stats->nreject = res[1];
        stats->nf = res[2];
    }
    SOLVE_TRY(fetch_adjoint_steps(h, a, res[0]));
    done = true;
    return KANODE_OK;
}

// ---- the persistent surrogate-pair adjoint (kd_pair_adjoint_kernel) --------------------------
// KANODE_OPT_PAIR_PERSIST: after a host-loop forward solve of an fp64 surrogate pair (K-form slots),
// the whole InterpolatingAdjoint is one launch; done = false when not covered (adjoint_t runs instead).
kanode_status adjoint_pair_t(kanode_handle* h, const void* p, kanode_solution* s, const void* dl_du, void* du0,
                             void* dp, const kanode_solver_options& o, kanode_solve_stats* stats, hipStream_t st,
                             bool& done) {
    done = false;
    const int64_t nsteps = (int64_t)s->ts.size();
    if (o.control != 0 || capturing(st) || s->slots_borrowed || s->qform || !s->record || nsteps < 1 ||
        s->dtype != KANODE_F64 || (int64_t)s->slots.size() < nsteps || !kanode_internal_pair_persist_ok(h))
        return KANODE_OK;
    const int nwg = kanode_internal_pair_adjoint_workgroups(h, s->batch);
    if (nwg < 1 || nwg > 256) return KANODE_OK;
    kan::PairAdjArgs pa{};
    SOLVE_TRY(one_launch_adj_args(h, s, dl_du, du0, dp, o, pa.c, st));
    const size_t tab = (size_t)nsteps * sizeof(double), off_tab = 256, off_ts = off_tab + tab, off_dts = off_ts + tab;
    const size_t off_x = (off_dts + tab + 255) / 256 * 256;
    const size_t need = off_x + (size_t)2 * nwg * kan::kPairAdjXW * sizeof(double);
    if (s->padj_bytes < need) {
        if (s->padj) SOLVE_HIP(h, hipFree(s->padj));
        s->padj = nullptr;
        s->padj_bytes = 0;
        SOLVE_HIP(h, hipMalloc(&s->padj, need));
        s->padj_bytes = need;
    }
    std::vector<char> host(3 * tab);
    static_assert(sizeof(void*) == sizeof(double), "slot table entries are 8 bytes");
    std::memcpy(host.data(), s->slots.data(), tab);
    std::memcpy(host.data() + tab, s->ts.data(), tab);
    std::memcpy(host.data() + 2 * tab, s->dts.data(), tab);
    char* base = (char*)s->padj;
    SOLVE_HIP(h, hipStreamSynchronize(st));   // the forward solve's kernels are done with nothing we upload
    SOLVE_HIP(h, hipMemcpy(base + off_tab, host.data(), 3 * tab, hipMemcpyHostToDevice));
    pa.c.rec = base + off_tab;
    pa.c.k1_0 = s->k1_0;
    pa.c.ts = (const double*)(base + off_ts);
    pa.c.dts = (const double*)(base + off_dts);
    pa.c.nsteps = nsteps;
    pa.ctr = (unsigned*)base;
    pa.abrt = pa.ctr + 1;
    pa.xbuf = (double*)(base + off_x);
    bool launched = false;
    SOLVE_TRY(kanode_internal_pair_adjoint(h, p, s->batch, &pa, st, launched));
    if (!launched) return KANODE_OK;
    auto& f = s->fused;
    SOLVE_HIP(h, hipMemcpyAsync(s->hscal, f.out, 4 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    unsigned abort_word = 0;
    SOLVE_HIP(h, hipMemcpyAsync(&abort_word, pa.abrt, sizeof(abort_word), hipMemcpyDeviceToHost, st));
    SOLVE_HIP(h, hipStreamSynchronize(st));
    int64_t res[4];
    std::memcpy(res, s->hscal, sizeof(res));
    if (res[3] == 3 || abort_word != 0) {
        // an exchange timed out (workgroups not co-resident: other work held CUs) and the grid drained:
        // the launch-per-stage path (adjoint_t) re-runs the adjoint and writes every output again
        kanode_internal_set_last_adjoint(h, KANODE_ADJ_PAIR_FALLBACK);
        return KANODE_OK;
    }
    if (res[3] == 1) return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "adjoint Tsit5: maxiters reached");
    if (stats) {
        stats->naccept = res[0];
        stats->nreject = res[1];
        stats->nf = res[2];
    }
    SOLVE_TRY(fetch_adjoint_steps(h, pa.c, res[0]));
    done = true;
    return KANODE_OK;
}

kanode_status check_opts(kanode_handle* h, const kanode_solver_options& o) {
    if (!(o.abstol >= 0) || !(o.reltol >= 0) || o.maxiters < 1 || !(o.qmin > 0) || !(o.qmax > 0) || !(o.gamma > 0))
        return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "solver options out of range");
    if (!o.adaptive && !(o.dt > 0)) return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "fixed-step Tsit5 needs dt > 0");
    if (o.control < 0 || o.control > 2 || o.graph_steps < 0)
        return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "control must be 0 (auto), 1 (host) or 2 (device)");
    return KANODE_OK;
}

// The solution object in *slot for a state of n entries (reused when its shape matches, else made anew): its
// k1_0, control scalars (mapped pinned where the platform allows) and error-partials staging.
kanode_status acquire_solution(kanode_handle* h, kanode_solution** slot, int64_t n, int dtype, bool record,
                               hipStream_t st, kanode_solution*& s) {
    s = *slot;
    if (s && (s->h != h || s->n != n || s->dtype != dtype || s->record != record)) {
        // storage of another shape: start over
        if (capturing(st)) return kanode_internal_fail(h, KANODE_ERR_CAPTURE, "dense output of another shape");
        SOLVE_HIP(h, hipStreamSynchronize(st));
        delete s;
        s = nullptr;
        *slot = nullptr;
    }
    if (!s) {
        if (capturing(st)) return kanode_internal_fail(h, KANODE_ERR_CAPTURE, "solve allocates its dense output");
        s = new (std::nothrow) kanode_solution();
        if (!s) return kanode_internal_fail(h, KANODE_ERR_ALLOC, "solution");
        s->h = h;
        s->dtype = dtype;
        s->esize = dtype == KANODE_F64 ? 8 : 4;
        s->n = n;
        s->record = record;
        if (hipMalloc(&s->k1_0, s->state_bytes()) != hipSuccess || hipMalloc(&s->dscal, kScalars * sizeof(double)) != hipSuccess ||
            hipHostMalloc((void**)&s->hscal, kScalars * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent) !=
                hipSuccess) {
            (void)hipGetLastError();
            delete s;
            return kanode_internal_fail(h, KANODE_ERR_ALLOC, "solve: out of device memory");
        }
        if (hipHostGetDevicePointer((void**)&s->mscal, s->hscal, 0) != hipSuccess) {
            (void)hipGetLastError();
            s->mscal = nullptr;   // copy path (read_ctl)
        }
        const size_t pb = (size_t)kanode_internal_max_parts() * sizeof(double);
        if (s->mscal && hipHostMalloc((void**)&s->hparts, pb, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
            hipHostGetDevicePointer((void**)&s->mparts, s->hparts, 0) != hipSuccess) {
            (void)hipHostFree(s->hparts);
            s->hparts = nullptr;
        }
        (void)hipGetLastError();
        if (!s->hparts) s->mparts = nullptr;   // the final-reduction launch then sums them
        else arm_ctl(s->hparts, kanode_internal_max_parts());
    }
    *slot = s;
    return KANODE_OK;
}

}  // namespace

extern "C" kanode_status kanode_solve_tsit5(kanode_handle* h, const void* p, const void* u0, int64_t batch, double t0,
                                            double tf, const double* saveat, int64_t n_save, void* u_save,
                                            const kanode_solver_options* opt, kanode_solution** dense,
                                            kanode_solve_stats* stats, void* stream) {
    SOLVE_TRY(kanode_internal_check(h));
    const kanode_solver_options o = resolved(opt);
    SOLVE_TRY(check_opts(h, o));
    if (!p || !u0 || batch < 1 || !(tf > t0) || n_save < 0 || (n_save > 0 && (!saveat || !u_save)))
        return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "solve: null pointer, batch < 1 or tf <= t0");
    if (!kanode_internal_square(h))
        return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "solve needs an RHS with N_in == N_out");
    for (int64_t j = 1; j < n_save; ++j)
        if (!(saveat[j] >= saveat[j - 1])) return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "saveat must ascend");
    // a stop past tf would never be reached and its rows of u_save would stay unwritten
    if (n_save > 0 && !(saveat[n_save - 1] <= tf + 1e-12 * std::max(1.0, std::fabs(tf))))
        return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "saveat must lie within [t0, tf]");
    hipStream_t st = (hipStream_t)stream;
    const int dtype = kanode_internal_dtype(h);
    const int64_t n = kanode_internal_state_length(h) * batch;
    // without a dense output the handle keeps the solve's storage (and any cached graph) for the next call
    const bool record = dense != nullptr;
    kanode_solution** slot = record ? dense : (kanode_solution**)kanode_internal_solution_cache(h);
    kanode_solution* s = nullptr;
    SOLVE_TRY(acquire_solution(h, slot, n, dtype, record, st, s));
    s->batch = batch;
    s->t0 = t0;
    s->tf = tf;
    s->saveat.assign(saveat, saveat + n_save);
    s->ts.clear();
    s->dts.clear();
    s->qform = false;   // K-form dense output unless the host loop takes the Fisher-KPP step path
    kanode_status r = ctl_begin(h, s, st);
    if (r == KANODE_OK) {
        TableHold hold(h);
        // auto = host: a replayed graph node costs the GPU what an eager launch does (ROCm 7.2,
        // tools/solve_modes.py), so device control only wins where the per-step norm read is a
        // large part of a step (adaptive, small states); it is opt-in
        const bool dev = o.control == 2;
        if (dev && capturing(st)) {
            r = kanode_internal_fail(h, KANODE_ERR_CAPTURE, "device step control cannot run inside a capture");
        } else if (dev) {
            r = dtype == KANODE_F64 ? solve_graph_t<double>(h, p, u0, t0, tf, saveat, n_save, u_save, o, s, stats, st)
                                    : solve_graph_t<float>(h, p, u0, t0, tf, saveat, n_save, u_save, o, s, stats, st);
        } else {
            // auto: a small chain (<= 16 trajectories) runs the whole solve in one workgroup
            bool done = false;
            r = KANODE_OK;
            if (o.control == 0)
                r = dtype == KANODE_F64
                        ? solve_fused_t<double>(h, p, u0, t0, tf, saveat, n_save, u_save, o, s, stats, st, done)
                        : solve_fused_t<float>(h, p, u0, t0, tf, saveat, n_save, u_save, o, s, stats, st, done);
            if (r == KANODE_OK && !done)   // auto: the adaptive Fisher-KPP table path with the control on the device
                r = solve_fk_loop(h, p, u0, t0, tf, saveat, n_save, u_save, o, s, stats, st, done);
            if (r == KANODE_OK && !done)
                r = dtype == KANODE_F64 ? solve_t<double>(h, p, u0, t0, tf, saveat, n_save, u_save, o, s, stats, st)
                                        : solve_t<float>(h, p, u0, t0, tf, saveat, n_save, u_save, o, s, stats, st);
        }
    }
    if (r != KANODE_OK) s->ctl_dirty = true;
    if (record || s->state_bytes() <= (size_t)64 << 20) {
        *slot = s;   // kept for the next solve (a large scratch solve gives its memory back)
    } else {
        if (hipStreamSynchronize(st) != hipSuccess) (void)hipGetLastError();
        delete s;
        *slot = nullptr;
    }
    return r;
}

extern "C" int64_t kanode_forward_sensitivity_step_sizes(kanode_handle* h, double* ts, double* dts, int64_t cap) {
    if (!h) return -1;
    const kanode_solution* s = *(kanode_solution**)kanode_internal_solution_cache(h);
    if (!s) return 0;
    const int64_t n = (int64_t)s->ts.size();
    const int64_t m = std::min(n, cap);
    if (ts && m > 0) std::memcpy(ts, s->ts.data(), (size_t)m * sizeof(double));
    if (dts && m > 0) std::memcpy(dts, s->dts.data(), (size_t)m * sizeof(double));
    return n;
}

extern "C" int32_t kanode_forward_sensitivity_supported(const kanode_handle* h, int64_t batch) {
    return h && batch >= 1 && kanode_internal_fsens_ok(h, batch) ? 1 : 0;
}

extern "C" kanode_status kanode_forward_sensitivity_tsit5(kanode_handle* h, const void* p, const void* u0,
                                                           int64_t batch, double t0, double tf, const double* saveat,
                                                           int64_t n_save, void* u_save, void* s_save,
                                                           const kanode_solver_options* opt, kanode_solve_stats* stats,
                                                           void* stream) {
    SOLVE_TRY(kanode_internal_check(h));
    const kanode_solver_options o = resolved(opt);
    SOLVE_TRY(check_opts(h, o));
    if (!p || !u0 || batch < 1 || !(tf > t0) || n_save < 0 || (n_save > 0 && !saveat))
        return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "forward sensitivities: null pointer, batch < 1 or tf <= t0");
    if (!kanode_internal_square(h))
        return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "forward sensitivities need an RHS with N_in == N_out");
    for (int64_t j = 1; j < n_save; ++j)
        if (!(saveat[j] >= saveat[j - 1])) return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "saveat must ascend");
    if (n_save > 0 && !(saveat[n_save - 1] <= tf + 1e-12 * std::max(1.0, std::fabs(tf))))
        return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "saveat must lie within [t0, tf]");
    if (!kanode_internal_fsens_ok(h, batch))
        return kanode_internal_fail(h, KANODE_ERR_UNSUPPORTED,
                                    "forward sensitivities: a Fisher-KPP (pointwise + periodic Laplacian) fp64 RHS with "
                                    "nx * batch <= 64, rbf basis, G = 5 or 10, base activation, softsign / tanh_fast");
    hipStream_t st = (hipStream_t)stream;
    if (capturing(st)) return kanode_internal_fail(h, KANODE_ERR_CAPTURE, "forward sensitivities read their counters");
    const int64_t n = kanode_internal_state_length(h) * batch;
    kanode_solution** slot = (kanode_solution**)kanode_internal_solution_cache(h);
    kanode_solution* s = nullptr;
    SOLVE_TRY(acquire_solution(h, slot, n, KANODE_F64, false, st, s));
    SOLVE_TRY(ctl_begin(h, s, st));
    auto& f = s->fused;
    if (f.saveat_cap < n_save) {
        if (f.saveat) (void)hipFree(f.saveat);
        f.saveat = nullptr;
        f.saveat_cap = 0;
        f.saveat_last.clear();
        SOLVE_HIP(h, hipMalloc((void**)&f.saveat, (size_t)n_save * sizeof(double)));
        f.saveat_cap = n_save;
    }
    if (!f.out) SOLVE_HIP(h, hipMalloc((void**)&f.out, 4 * sizeof(int64_t)));
    if (n_save > 0) SOLVE_TRY(staged_upload(h, s, f.saveat, saveat, (size_t)n_save * sizeof(double), st, &f.saveat_last));
    // the accepted step times / sizes (up to kFsensSteps), read back with the counters
    constexpr int64_t kFsensSteps = 4096;
    if (f.ts_cap < kFsensSteps) {
        if (f.ts) (void)hipFree(f.ts);
        f.ts = nullptr;
        f.ts_cap = 0;
        SOLVE_HIP(h, hipMalloc((void**)&f.ts, 2 * (size_t)kFsensSteps * sizeof(double)));
        f.ts_cap = kFsensSteps;
    }
    if (f.hts_cap < f.ts_cap) {
        if (f.hts) (void)hipHostFree(f.hts);
        f.hts = nullptr;
        f.mts = nullptr;
        f.hts_cap = 0;
        SOLVE_HIP(h, hipHostMalloc((void**)&f.hts, 2 * (size_t)f.ts_cap * sizeof(double)));
        f.hts_cap = f.ts_cap;
    }
    kan::ChainSolveArgs a{};
    a.cap = f.ts_cap;
    a.ts = f.ts;
    a.dts = f.ts + f.ts_cap;
    a.t0 = t0;
    a.tf = tf;
    a.dt = o.dt;
    a.abstol = o.abstol;
    a.reltol = o.reltol;
    a.dtmin = o.dtmin;
    a.beta1 = o.beta1;
    a.beta2 = o.beta2;
    a.gamma = o.gamma;
    a.qmin = o.qmin;
    a.qmax = o.qmax;
    a.qoldinit = o.qoldinit;
    a.adaptive = o.adaptive ? 1 : 0;
    a.maxiters = o.maxiters;
    a.n_save = n_save;
    a.saveat = f.saveat;
    a.u_save = n_save > 0 ? u_save : nullptr;
    a.out = f.out;
    kanode_status r = kanode_internal_fk_fsens(h, p, u0, batch, &a, n_save > 0 ? s_save : nullptr, st);
    if (r != KANODE_OK) {
        s->ctl_dirty = true;
        return r;
    }
    SOLVE_HIP(h, hipMemcpyAsync(s->hscal, f.out, 4 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    SOLVE_HIP(h, hipMemcpyAsync(f.hts, f.ts, 2 * (size_t)f.ts_cap * sizeof(double), hipMemcpyDeviceToHost, st));
    SOLVE_HIP(h, hipStreamSynchronize(st));
    int64_t res[4];
    std::memcpy(res, s->hscal, sizeof(res));
    if (res[3] == 1) return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "Tsit5: maxiters reached");
    const int64_t nrec = std::min<int64_t>(res[0], f.ts_cap);
    s->t0 = t0;
    s->tf = tf;
    s->ts.assign(f.hts, f.hts + nrec);
    s->dts.assign(f.hts + f.ts_cap, f.hts + f.ts_cap + nrec);
    if (stats) {
        stats->naccept = res[0];
        stats->nreject = res[1];
        stats->nf = res[2];
    }
    return KANODE_OK;
}

extern "C" kanode_status kanode_adjoint_tsit5(kanode_handle* h, const void* p, const kanode_solution* dense,
                                              const void* dl_du, void* du0, void* dp, const kanode_solver_options* opt,
                                              kanode_solve_stats* stats, void* stream) {
    SOLVE_TRY(kanode_internal_check(h));
    const kanode_solver_options o = resolved(opt);
    SOLVE_TRY(check_opts(h, o));
    if (!p || !dense) return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "adjoint: null p or dense output");
    kanode_solution* s = const_cast<kanode_solution*>(dense);   // scratch only; the dense output is not modified
    if (s->h != h || !s->record)
        return kanode_internal_fail(h, KANODE_ERR_INVALID_ARG, "adjoint: dense output of another handle or not recorded");
    hipStream_t st = (hipStream_t)stream;
    SOLVE_TRY(ctl_begin(h, s, st));
    TableHold hold(h);
    bool done = false;
    kanode_internal_set_last_adjoint(h, KANODE_ADJ_NONE);
    kanode_internal_clear_adjoint_steps(h);   // recorded or not: no stale sizes from an earlier adjoint
    kanode_status r = s->dtype == KANODE_F64 ? adjoint_fused_t<double>(h, p, s, dl_du, du0, dp, o, stats, st, done)
                                             : adjoint_fused_t<float>(h, p, s, dl_du, du0, dp, o, stats, st, done);
    if (r == KANODE_OK && done) kanode_internal_set_last_adjoint(h, KANODE_ADJ_CHAIN_WG);
    if (r == KANODE_OK && !done) {
        r = adjoint_pair_t(h, p, s, dl_du, du0, dp, o, stats, st, done);
        if (r == KANODE_OK && done) kanode_internal_set_last_adjoint(h, KANODE_ADJ_PAIR_PERSIST);
    }
    if (r == KANODE_OK && !done) {
        const bool fell_back = kanode_get_option(h, KANODE_OPT_LAST_ADJOINT) == KANODE_ADJ_PAIR_FALLBACK;
        r = s->dtype == KANODE_F64 ? adjoint_t<double>(h, p, s, dl_du, du0, dp, o, stats, st)
                                   : adjoint_t<float>(h, p, s, dl_du, du0, dp, o, stats, st);
        if (!fell_back) kanode_internal_set_last_adjoint(h, KANODE_ADJ_HOST_LOOP);
    }
    if (r != KANODE_OK) {
        // a failed adjoint may leave a deferred surrogate-pair stage (raw pointers into this solution and the
        // handle's workspace) and finish jobs pending on the handle: drop them, so no later call launches them
        kanode_internal_vjp_discard(h);
        s->ctl_dirty = true;
    }
    return r;
}
