// kan_pair_adj.hip — the whole InterpolatingAdjoint of a full-field surrogate pair in ONE launch (gfx950).
//
// The surrogate RHS du = KDense(H -> N)(KDense(N -> H)(u)) (PDE examples/Burgers_Surrogate.jl:85-97,
// Schrodinger_Surrogate.jl:93-104; KAN [N, 10, N]) couples the N grid points only through the H hidden
// activations.  So the grid splits over workgroups exactly as kanode/tp.py splits it over ranks:
// workgroup w owns the points [a_w, a_w + S) — its slice of the state, layer 1's input columns
// C1[:, :, a:a+S], W1[:, a:a+S] and layer 2's output rows C2[a:a+S, :], W2[a:a+S, :].  Every parameter
// cotangent of an adjoint stage is then local to one workgroup, and a stage needs only two exchanges of
// H·B values between the workgroups:
//   A: the partial pre-activations Σ_{i in slice} (C1 φ(y_i) + W1 swish(y_i))   -> h       (every workgroup)
//   B: the partial hidden cotangents Σ_{o in slice} λs_o ∂out_o/∂h              -> h̄       (every workgroup)
// μ and its seven stage vectors (the adjoint's parameter part) live in the owning workgroup's LDS for the
// whole solve; λ and its stage values likewise for the slice.  The backward Tsit5 over [λ; μ] is
// kanode_solve.cpp adjoint_t's (the statement kd_chain_adjoint_kernel runs in one workgroup for small
// chains): the same steps, stops, saveat jumps with FSAL re-evaluation, PI controller and initial step;
// each decision is taken by every workgroup from the same fixed-order sums, so all take the same path.
// The embedded-error norm over [λ; μ] is one more exchange per step.
//
// Exchanges follow the agent-scope hand-off of cdna_hip_programming.md Guideline 16 (MI355X_MICROARCH.md
// §visibility, Valid forms, first row): each workgroup stores its partials write-through (relaxed agent
// atomics = sc1 stores) into one of two ping-pong slots, every storing wave drains (s_waitcnt vmcnt(0)),
// the block synchronises and one lane adds 1 to the arrival counter (agent scope); a consumer lane polls
// the counter with relaxed agent loads (sc1) until all nwg arrivals of this exchange are in, the block
// synchronises, and every load of the partials is again a relaxed agent (sc1) load.  Two slots suffice:
// a workgroup can only write exchange e + 2's slot after every workgroup has arrived at exchange e + 1,
// i.e. after it has read exchange e.  The counter and the abort word are zeroed by a memset before every
// launch; every spin is bounded, and a time-out raises the abort word every other spin also watches, so
// the grid always drains.  Nothing depends on dispatch order or workgroup->XCD placement.
//
// Numerics: the layer formulas are kdense.jl:109-130 / utils.jl:8-21 (direct basis per knot, the NNlib
// rrules); the sums run in a fixed order (bitwise reproducible for a given S), which differs from the
// launch-per-stage path's order, so results agree with it and with the CPU oracle to rounding.
#include "kan_common.hpp"
#include "kan_kernels.hpp"

namespace kan {

namespace {

constexpr int kPA = 256;                // threads per workgroup
constexpr int kPAMaxXW = kPairAdjXW;    // exchange width cap (6·H·B of a step's forward halves)
constexpr int kPALd = 16;              // exchange loads in flight per thread
constexpr unsigned kPASpinMax = 1u << 22;   // a few seconds: far beyond any legitimate wait

// (st_agent / ld_agent: kan_common.hpp)

// All nwg workgroups publish `cnt` values (vals[0..cnt) in LDS) as exchange e, then every workgroup
// forms out[q] = Σ_{w = 0..nwg-1} partial_w[q] in that order (the same bits everywhere).
// Returns false when the exchange was abandoned (abort raised / time-out): the caller exits.
// The two halves of an exchange: pa_publish stores this workgroup's partials and arrives; work that does
// not need the exchange's result may run before pa_collect waits for the other workgroups and sums.
__device__ void pa_publish(const double* vals, int cnt, double* xbuf, unsigned* ctr, int nwg, unsigned e) {
    double* slot = xbuf + (size_t)(e & 1u) * nwg * kPAMaxXW;
    const int w = blockIdx.x;
    for (int q = threadIdx.x; q < cnt; q += kPA) st_agent(slot + (size_t)w * kPAMaxXW + q, vals[q]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ bool pa_collect(int cnt, double* out, double* xbuf, unsigned* ctr, unsigned* abrt, int nwg, unsigned e,
                           double* tmp /* LDS, >= max(kPA, cnt) */, int* flag /* LDS */) {
    double* slot = xbuf + (size_t)(e & 1u) * nwg * kPAMaxXW;
    if (threadIdx.x == 0) {
        const unsigned target = (unsigned)nwg * (e + 1u);
        int ok = 1;
        for (unsigned spins = 0;; ++spins) {
            if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
            if (__hip_atomic_load(abrt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u || spins > kPASpinMax) {
                __hip_atomic_store(abrt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        *flag = ok;
    }
    __syncthreads();
    if (!*flag) return false;
    // fixed-order sum: item (c, q) sums output q over the workgroup range of chunk c (up to kPALd loads in
    // flight at once); the chunk partials are then added in chunk order
    const int nch = cnt >= kPA ? 1 : (kPA / cnt < nwg ? kPA / cnt : nwg);
    const int per = (nwg + nch - 1) / nch;
    for (int item = threadIdx.x; item < nch * cnt; item += kPA) {
        const int q = item % cnt, c = item / cnt;
        const int w0 = c * per, w1 = w0 + per < nwg ? w0 + per : nwg;
        double s = 0.0;
        for (int wb = w0; wb < w1; wb += kPALd) {
            double v[kPALd];
#pragma unroll
            for (int r = 0; r < kPALd; ++r)
                v[r] = wb + r < w1 ? ld_agent(slot + (size_t)(wb + r) * kPAMaxXW + q) : 0.0;
#pragma unroll
            for (int r = 0; r < kPALd; ++r)
                if (wb + r < w1) s = wb + r == w0 ? v[r] : s + v[r];
        }
        tmp[item] = s;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < cnt; q += kPA) {
        double s = tmp[q];
        for (int c = 1; c < nch; ++c) s += tmp[c * cnt + q];
        out[q] = s;
    }
    __syncthreads();
    return true;
}
__device__ bool pa_exchange(const double* vals, int cnt, double* out, double* xbuf, unsigned* ctr, unsigned* abrt,
                            int nwg, unsigned e, double* tmp, int* flag) {
    pa_publish(vals, cnt, xbuf, ctr, nwg, e);
    return pa_collect(cnt, out, xbuf, ctr, abrt, nwg, e, tmp, flag);
}

#ifdef KAN_PA_PROF
// phase timing of workgroup 0 (variant builds only, tools/build_var.sh -DKAN_PA_PROF): wall-clock ticks
// accumulated per phase mark, read by kanode_debug_pair_profile
__device__ unsigned long long g_pa_prof[16];
#define PA_MARK(i)                                                       \
    do {                                                                 \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                       \
            const unsigned long long n_ = wall_clock64();                \
            prof_acc[i] += n_ - prof_last;                               \
            prof_last = n_;                                              \
        }                                                                \
    } while (0)
#else
#define PA_MARK(i) \
    do {           \
    } while (0)
#endif

// Σ of one value per thread over the block, in a fixed order; every thread gets the total
__device__ __forceinline__ double pa_bsum(double v, double* red) {
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = v;
    __syncthreads();
    double t = red[0];
    for (int q = 1; q < kPA / kWave; ++q) t += red[q];
    __syncthreads();
    return t;
}

}  // namespace

// LDS carve (doubles), S points per workgroup, B columns, H hidden, G1 / G2 knots, NS = 6 stage slots:
//   ps[Pw] | mu[2][Pw] | km[7][Pw] | dens[8][S·B] | lam[S·B] | kl[7][S·B] | yv[NS][S·B] | lsv[S·B] |
//   phi1[NS][S·B·G1] | dphi1[NS][S·B·G1] | sw1[NS][S·B] | dsw1[NS][S·B] | hid[NS][H·B] | hbar[2][H·B] |
//   psi[NS][H·B·G2] | dpsi[NS][H·B·G2] | sw2[NS][H·B] | dsw2[NS][H·B] | part[NS·H·B] |
//   tmp[max(kPA, NS·H·B)] | red[4] | exp table[256] | wsp[max(NS·H·B·S, H·B·(G2+1), S·B·(G1+1))]
//   (wsp: per-item terms of the contractions)
constexpr int kPANS = 6;
__host__ __device__ inline int64_t pair_adj_pw(int S, int H, int G1, int G2, int ub1, int ub2) {
    return (int64_t)H * G1 * S + (int64_t)H * S * ub1 + (int64_t)S * G2 * H + (int64_t)S * H * ub2;
}
__host__ __device__ inline int64_t pair_adj_wsp(int S, int B, int H, int G1, int G2) {
    const int64_t a = (int64_t)kPANS * H * B * S, b = (int64_t)H * B * (G2 + 1), c = (int64_t)S * B * (G1 + 1);
    return a > b ? (a > c ? a : c) : (b > c ? b : c);
}
__host__ __device__ inline int64_t pair_adj_lds_doubles(int S, int B, int H, int G1, int G2, int ub1, int ub2) {
    const int64_t Pw = pair_adj_pw(S, H, G1, G2, ub1, ub2), SB = (int64_t)S * B, HB = (int64_t)H * B;
    const int64_t nshb = (int64_t)kPANS * HB;
    return 10 * Pw + 8 * SB + 8 * SB + kPANS * SB + SB + kPANS * (2 * SB * G1 + 2 * SB + HB) + 2 * HB +
           kPANS * (2 * HB * G2 + 2 * HB) + nshb + (nshb > kPA ? nshb : kPA) + 4 + 256 + pair_adj_wsp(S, B, H, G1, G2);
}

// SC: the points per workgroup, a compile-time constant so the contractions over a slice unroll (their
// LDS loads issue together)
template <int SC>
__global__ void __launch_bounds__(kPA)
kd_pair_adjoint_kernel(const LayerConst* __restrict__ lcs, const double* __restrict__ p, int64_t B, PairAdjArgs pa) {
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
    constexpr double RI[7][4] = {
        {1.0, -2.763706197274826, 2.9132554618219126, -1.0530884977290216},
        {0.0, 0.13169999999999998, -0.2234, 0.1017},
        {0.0, 3.9302962368947516, -5.941033872131505, 2.490627285651253},
        {0.0, -12.411077166933676, 30.33818863028232, -16.548102889244902},
        {0.0, 37.50931341651104, -88.1789048947664, 47.37952196281928},
        {0.0, -27.896526289197286, 65.09189467479366, -34.87065786149661},
        {0.0, 1.5, -4.0, 2.5},
    };
    const ChainAdjointArgs& a = pa.c;
    const LayerConst& L1 = lcs[0];
    const LayerConst& L2 = lcs[1];
    const int N = L1.I, H = L1.O, G1 = L1.G, G2 = L2.G;
    const int ub1 = L1.use_base, ub2 = L2.use_base;
    constexpr int S = SC;
    const int nwg = (int)gridDim.x;
    const int a0 = (int)blockIdx.x * S;
    const int Sw = N - a0 < S ? N - a0 : S;          // points of this workgroup (the last may hold fewer)
    const int SB = S * (int)B, HB = H * (int)B;
    const int64_t n = (int64_t)N * B;
    const int64_t Pw = pair_adj_pw(S, H, G1, G2, ub1, ub2);
    // local parameter slice: C1 [j + H(g + G1 il)] | W1 [j + H il] | C2 [c + GH2 ol], c = g + G2 j | W2 [j + H ol]
    // (layer 2 row-transposed: the lanes of a wave then read consecutive entries)
    const int GH2 = G2 * H;
    const int64_t oC1 = 0, oW1 = (int64_t)H * G1 * S, oC2 = oW1 + (int64_t)H * S * ub1,
                  oW2 = oC2 + (int64_t)S * G2 * H;

#ifdef KAN_PA_PROF
    unsigned long long prof_acc[16] = {};
    unsigned long long prof_last = wall_clock64();
#endif
    extern __shared__ __attribute__((aligned(16))) double pa_lds[];
    double* ps = pa_lds;
    double* mu = ps + Pw;          // [2][Pw]
    double* km = mu + 2 * Pw;      // [7][Pw]
    double* dens = km + 7 * Pw;    // [8][SB]: u_i, k_1..k_7 of the cached forward step
    double* lam = dens + 8 * SB;   // [SB]
    double* kl = lam + SB;         // [7][SB]
    double* yv = kl + 7 * SB;                              // [NS][SB]
    double* lsv = yv + (int64_t)kPANS * SB;
    double* phi1 = lsv + SB;                              // [NS][SB][G1]
    double* dphi1 = phi1 + (int64_t)kPANS * SB * G1;       // [NS][SB][G1]
    double* sw1 = dphi1 + (int64_t)kPANS * SB * G1;        // [NS][SB]
    double* dsw1 = sw1 + (int64_t)kPANS * SB;              // [NS][SB]
    double* hid = dsw1 + (int64_t)kPANS * SB;              // [NS][HB]
    double* hbar = hid + (int64_t)kPANS * HB;              // [HB]
    double* hbar_p = hbar + HB;                            // [HB]: h̄ of the stage whose dC1 is pending
    double* psi = hbar_p + HB;                             // [NS][HB][G2]
    double* dpsi = psi + (int64_t)kPANS * HB * G2;         // [NS][HB][G2]
    double* sw2 = dpsi + (int64_t)kPANS * HB * G2;         // [NS][HB]
    double* dsw2 = sw2 + (int64_t)kPANS * HB;              // [NS][HB]
    double* part = dsw2 + (int64_t)kPANS * HB;             // [NS·HB] this workgroup's partials of an exchange
    double* tmp = part + (int64_t)kPANS * HB;              // [max(kPA, NS·HB)]
    double* red = tmp + (kPANS * HB > kPA ? kPANS * HB : kPA);   // [4]
    double* tab = red + 4;                                 // [256] exp table
    double* wsp = tab + 256;                               // per-item contraction terms
    __shared__ int xflag;
    for (int i = threadIdx.x; i < 256; i += kPA) tab[i] = kExp2Tab256[i];
    const Math<double> M{tab};
    const int t = threadIdx.x;
    const int N2 = L2.O;   // == N
    // the workgroup's parameter slice (ComponentArray layout, LV_driver_KANODE.jl:173-175)
    for (int64_t q = t; q < Pw; q += kPA) {
        int64_t g;
        if (q < oW1) g = L1.p_off + (int64_t)H * G1 * a0 + q;                           // C1[j, g + G1 i]
        else if (q < oC2) g = L1.w_off + (int64_t)H * a0 + (q - oW1);                     // W1[j, i]
        else if (q < oW2) {                                                               // C2[o, g + G2 j]
            const int64_t r = q - oC2, c = r % GH2, ol = r / GH2;
            g = L2.p_off + a0 + ol + (int64_t)N2 * c;
        } else {                                                                          // W2[o, j]
            const int64_t r = q - oW2, j = r % H, ol = r / H;
            g = L2.w_off + a0 + ol + (int64_t)N2 * j;
        }
        const bool live = (q < oC2) ? ((q < oW1 ? (q / (H * G1)) : ((q - oW1) / H)) < Sw)
                                    : ((q < oW2 ? (q - oC2) / GH2 : (q - oW2) / H) < Sw);
        ps[q] = live ? p[g] : 0.0;
        mu[q] = 0.0;
        mu[Pw + q] = 0.0;
        for (int m = 0; m < 7; ++m) km[m * Pw + q] = 0.0;
    }
    for (int q = t; q < 8 * SB + SB + 7 * SB; q += kPA) dens[q] = 0.0;   // dens, lam, kl
    __syncthreads();

    const void* const* slots = reinterpret_cast<const void* const*>(a.rec);
    const double* __restrict__ dl = reinterpret_cast<const double*>(a.dl_du);
    const double t0 = a.t0, tf = a.tf, TT = tf - t0;
    const double ntot = (double)(n + pa.P);
    unsigned ex = 0;            // exchanges so far (the same count in every workgroup)
    int64_t cur = a.nsteps - 1, cached = -1;
    bool alive = true;

    // λ entries of this workgroup: e = il + S·k  <->  global (a0 + il) + N·k
    auto gidx = [&](int e) -> int64_t { return (int64_t)(a0 + e % S) + (int64_t)N * (e / S); };
    auto act_e = [&](int e) -> bool { return (e % S) < Sw; };

    auto add_rows = [&](int gi) {   // λ += Σ dl_du[row] (rows in order), own entries
        for (int e = t; e < SB; e += kPA) {
            if (!act_e(e)) continue;
            double l = lam[e];
            for (int32_t q = a.joff[gi]; q < a.joff[gi + 1]; ++q) l = l + dl[(int64_t)a.jrows[q] * n + gidx(e)];
            lam[e] = l;
        }
        __syncthreads();
    };

    // The layer-1 parameter cotangents of the last back_stage (dC1[j, g + G1 i] = Σ_k h̄_jk φ_g(y_ik), dW1), left
    // pending because nothing on λ's path needs them: formed inside the next stage's exchange window, or
    // before anything reads kμ or overwrites that stage's forward half (fwd_stages, the μ update).
    int pend_st = -1, pend_m = 0;
    auto flush_pending = [&](bool sync) {
        if (pend_st < 0) return;
        const double* ph1 = phi1 + (int64_t)pend_st * SB * G1;
        const double* sw1s = sw1 + (int64_t)pend_st * SB;
        double* kmm = km + (int64_t)pend_m * Pw;
        for (int64_t q = t; q < (int64_t)H * G1 * S; q += kPA) {
            const int j = (int)(q % H), c = (int)(q / H), g = c % G1, il = c / G1;
            double sm = 0.0;
            for (int k = 0; k < (int)B; ++k) sm = ::fma(hbar_p[j + H * k], ph1[(il + S * k) * G1 + g], sm);
            kmm[oC1 + q] = sm;
        }
        if (ub1)
            for (int q = t; q < H * S; q += kPA) {
                const int j = q % H, il = q / H;
                double sm = 0.0;
                for (int k = 0; k < (int)B; ++k) sm = ::fma(hbar_p[j + H * k], sw1s[il + S * k], sm);
                kmm[oW1 + q] = sm;
            }
        pend_st = -1;
        if (sync) __syncthreads();
    };

    // The forward half of ns adjoint stages at the times taus[0..ns): the interpolated forward state
    // y(tf - τ) = u_i + Σ_m (dt b_m(θ)) k_m (stage_lincomb order) over this slice, layer 1's basis per
    // (point, column, knot) -> stage slot s, and the hidden pre-activations of every stage in ONE exchange
    // (they do not depend on λ, so all stages of a step share it) -> hid[s].
    auto fwd_stages = [&](const double* taus, int ns) -> bool {
        flush_pending(true);   // (its stage's forward half is about to be overwritten)
        PA_MARK(0);
        for (int st = 0; st < ns; ++st) {
            const double tt = tf - taus[st];
            while (cur > 0 && a.ts[cur] > tt) --cur;
            while (cur + 1 < a.nsteps && a.ts[cur + 1] <= tt) ++cur;
            if (cur != cached) {       // the forward step's u_i, k_1..k_7 over this slice
                __syncthreads();       // (earlier stages' y read the previous step's values)
                const double* base = reinterpret_cast<const double*>(slots[cur]);
                const double* k1 = cur == 0 ? reinterpret_cast<const double*>(a.k1_0)
                                            : reinterpret_cast<const double*>(slots[cur - 1]) + 6 * n;
                for (int q = t; q < 8 * SB; q += kPA) {
                    const int m = q / SB, e = q - m * SB;
                    double v = 0.0;
                    if (act_e(e)) {
                        const int64_t gi = gidx(e);
                        v = m == 0 ? base[gi] : (m == 1 ? k1[gi] : base[(int64_t)(m - 1) * n + gi]);
                    }
                    dens[q] = v;
                }
                cached = cur;
                __syncthreads();
                PA_MARK(1);
            }
            const double dti = a.dts[cur];
            const double th = ::fmin(1.0, ::fmax(0.0, (tt - a.ts[cur]) / dti));
            double cw[7];
#pragma unroll
            for (int m = 0; m < 7; ++m) {
                double sm = 0.0, tp = th;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    sm += RI[m][r] * tp;
                    tp *= th;
                }
                cw[m] = sm * dti;
            }
            for (int e = t; e < SB; e += kPA) {
                double y = dens[e];
#pragma unroll
                for (int m = 0; m < 7; ++m) y = ::fma(cw[m], dens[(m + 1) * SB + e], y);
                yv[st * SB + e] = y;
            }
        }
        __syncthreads();
        // layer 1's basis of every stage, per (stage, point, column, knot)
        for (int q = t; q < ns * SB * G1; q += kPA) {
            const int se = q / G1, g = q - se * G1, e = se % SB;
            const double y = yv[se];
            const double nn = normalize<NORM_RUNTIME, double>(M, L1.norm, y);
            const double z = (nn - (double)L1.grid[g]) * (double)L1.invh;
            double aux = 0.0;
            const double ph = basis_direct<double>(M, L1.basis, z, aux);
            phi1[q] = act_e(e) ? ph : 0.0;
            dphi1[q] = act_e(e) ? dnormalize<NORM_RUNTIME, double>(L1.norm, nn) *
                                      (basis_pull<double>(L1.basis, L1.iqf_quirk, z, ph, aux, 1.0) * (double)L1.invh)
                                : 0.0;
            if (g == 0) {
                double sw = 0.0, dsw = 0.0;
                if (ub1) swish_and_grad<double>(M, y, sw, dsw);
                sw1[se] = act_e(e) ? sw : 0.0;
                dsw1[se] = act_e(e) ? dsw : 0.0;
            }
        }
        __syncthreads();
        // partial pre-activations of every stage over this slice: item (st, jk, il) forms one input's
        // terms, then output (st, jk) sums its S items in order
        for (int q = t; q < ns * HB * S; q += kPA) {   // item (st, k, il, j), j fastest (consecutive C1 entries)
            const int j = q % H, r = q / H, il = r % S, sk = r / S, k = sk % (int)B, st = sk / (int)B;
            double sm = 0.0;
            if (il < Sw) {
                const int se = st * SB + il + S * k;
#pragma unroll 5
                for (int g = 0; g < G1; ++g) sm = ::fma(ps[oC1 + j + H * (g + G1 * il)], phi1[se * G1 + g], sm);
                if (ub1) sm = ::fma(ps[oW1 + j + H * il], sw1[se], sm);
            }
            wsp[((int64_t)st * HB + j + H * k) * S + il] = sm;
        }
        __syncthreads();
        for (int q = t; q < ns * HB; q += kPA) {
            double v[S];
#pragma unroll
            for (int il = 0; il < S; ++il) v[il] = wsp[q * S + il];
            double sm = v[0];
#pragma unroll
            for (int il = 1; il < S; ++il)
                if (il < Sw) sm += v[il];
            part[q] = sm;
        }
        __syncthreads();
        PA_MARK(2);
        if (!pa_exchange(part, ns * HB, hid, pa.xbuf, pa.ctr, pa.abrt, nwg, ex++, tmp, &xflag)) return false;
        PA_MARK(3);
        // layer 2 at every stage's hidden activations (every workgroup: the same values)
        for (int q = t; q < ns * HB * G2; q += kPA) {
            const int sjk = q / G2, g = q - sjk * G2;
            const double h = hid[sjk];
            const double mm = normalize<NORM_RUNTIME, double>(M, L2.norm, h);
            const double z = (mm - (double)L2.grid[g]) * (double)L2.invh;
            double aux = 0.0;
            const double ph = basis_direct<double>(M, L2.basis, z, aux);
            psi[q] = ph;
            dpsi[q] = dnormalize<NORM_RUNTIME, double>(L2.norm, mm) *
                      (basis_pull<double>(L2.basis, L2.iqf_quirk, z, ph, aux, 1.0) * (double)L2.invh);
            if (g == 0) {
                double sw = 0.0, dsw = 0.0;
                if (ub2) swish_and_grad<double>(M, h, sw, dsw);
                sw2[sjk] = sw;
                dsw2[sjk] = dsw;
            }
        }
        __syncthreads();
        PA_MARK(4);
        return true;
    };

    // Partial hidden cotangents of stage slot st over this slice's output rows (λs in lsv) -> outp[0..HB):
    // item (jk, g) (g = G2: the base term) contracts λs over the rows, output jk sums its G2 + 1 items
    auto part_b = [&](int st, double* outp) {
        const double* dpsis = dpsi + (int64_t)st * HB * G2;
        const double* dsw2s = dsw2 + (int64_t)st * HB;
        const int nC = (int)B * GH2, nW = ub2 ? HB : 0;
        for (int q = t; q < nC + nW; q += kPA) {
            double c = 0.0, f;
            if (q < nC) {                       // (k, c = g + G2 j)
                const int k = q / GH2, cc = q - k * GH2;
#pragma unroll
                for (int ol = 0; ol < S; ++ol)
                    if (ol < Sw) c = ::fma(lsv[ol + S * k], ps[oC2 + cc + GH2 * ol], c);
                f = dpsis[q];                   // dψ at (j + H k)·G2 + g == cc + GH2·k == q
            } else {                            // (k, j): the base term
                const int r = q - nC, k = r / H, j = r - k * H;
#pragma unroll
                for (int ol = 0; ol < S; ++ol)
                    if (ol < Sw) c = ::fma(lsv[ol + S * k], ps[oW2 + j + H * ol], c);
                f = dsw2s[r];
            }
            wsp[q] = f * c;
        }
        __syncthreads();
        for (int q = t; q < HB; q += kPA) {
            const int j = q % H, k = q / H;
            const double* w = wsp + (int64_t)k * GH2 + (int64_t)G2 * j;
            double sm = w[0];
            for (int g = 1; g < G2; ++g) sm += w[g];
            if (ub2) sm += wsp[nC + q];
            outp[q] = sm;
        }
        __syncthreads();
        PA_MARK(5);
    };
    // While the other workgroups arrive: the previous stage's layer-1 parameter cotangents and this stage's
    // layer-2 ones (own rows): dC2[o, g + G2 j] = Σ_k λs_ok ψ_g(h_jk) (neither is on λ's path)
    auto dc2 = [&](int st, int mslot) {
        flush_pending(false);
        const double* psis = psi + (int64_t)st * HB * G2;
        const double* sw2s = sw2 + (int64_t)st * HB;
        double* kmm = km + (int64_t)mslot * Pw;
        for (int64_t q = t; q < (int64_t)S * GH2; q += kPA) {
            const int cc = (int)(q % GH2), ol = (int)(q / GH2);
            double sm = 0.0;
            for (int k = 0; k < (int)B; ++k) sm = ::fma(lsv[ol + S * k], psis[cc + (int64_t)GH2 * k], sm);
            kmm[oC2 + q] = ol < Sw ? sm : 0.0;
        }
        if (ub2)
            for (int q = t; q < S * H; q += kPA) {
                const int j = q % H, ol = q / H;
                double sm = 0.0;
                for (int k = 0; k < (int)B; ++k) sm = ::fma(lsv[ol + S * k], sw2s[j + H * k], sm);
                kmm[oW2 + q] = ol < Sw ? sm : 0.0;
            }
    };
    // Layer 1's pullback on this slice with h̄ (hbar): kλ -> kl[kslot] (item (e, g), g = G1: the base term,
    // contracts h̄ over the hidden units; entry e sums its G1 + 1 items in order); the parameter cotangents
    // are left pending (flush_pending)
    auto xbar = [&](int st, int kslot, int mslot) {
        const double* dph1 = dphi1 + (int64_t)st * SB * G1;
        const double* dsw1s = dsw1 + (int64_t)st * SB;
        double* klo = kl + (int64_t)kslot * SB;
        // item (e, j): h̄_jk · (Σ_g dφ_g(y_e) C1[j, g, il] + swish'(y_e) W1[j, il]); entry e sums its H items
        for (int q = t; q < SB * H; q += kPA) {
            const int e = q / H, j = q - e * H, il = e % S, k = e / S;
            double c = 0.0;
            if (il < Sw) {
#pragma unroll 5
                for (int g = 0; g < G1; ++g) c = ::fma(dph1[e * G1 + g], ps[oC1 + j + H * (g + G1 * il)], c);
                if (ub1) c = ::fma(dsw1s[e], ps[oW1 + j + H * il], c);
            }
            wsp[q] = hbar[j + H * k] * c;
        }
        __syncthreads();
        for (int e = t; e < SB; e += kPA) {
            double sm = wsp[e * H];
            for (int j = 1; j < H; ++j) sm += wsp[e * H + j];
            klo[e] = sm;
        }
        for (int q = t; q < HB; q += kPA) hbar_p[q] = hbar[q];
        pend_st = st;
        pend_m = mslot;
        __syncthreads();
        PA_MARK(7);
    };
    // The backward half of the stage in slot st with the adjoint stage input λs (lsv): layer 2 at the hidden
    // activations hid[st], the hidden cotangents in one exchange, layer 1's pullback on this slice:
    // kλ -> kl[kslot], kμ -> km[mslot]
    auto back_stage = [&](int st, int kslot, int mslot) -> bool {
        part_b(st, part);
        const unsigned eB = ex++;
        pa_publish(part, HB, pa.xbuf, pa.ctr, nwg, eB);
        dc2(st, mslot);
        if (!pa_collect(HB, hbar, pa.xbuf, pa.ctr, pa.abrt, nwg, eB, tmp, &xflag)) return false;
        PA_MARK(6);
        xbar(st, kslot, mslot);
        return true;
    };

    auto set_ls = [&](const double* src) {   // lsv <- src (own entries)
        for (int e = t; e < SB; e += kPA) lsv[e] = src[e];
        __syncthreads();
    };

    int64_t naccept = 0, nreject = 0, nf = 0, it = 0, status = 0;
    double h = a.dt;
    int mc = 0;   // mu[mc] holds μ
    int k0 = 0;   // km / kl slot of the FSAL stage value
    int64_t si = 0;
    double tau = 0.0;
    double taus[kPANS];
    if (dl) add_rows(0);
    set_ls(lam);
    taus[0] = 0.0;
    alive = fwd_stages(taus, 1) && back_stage(0, 0, 0);
    flush_pending(true);
    nf = 1;
    if (alive && a.adaptive && !(a.dt > 0)) {   // Hairer-Wanner on [λ; μ]
        double s0 = 0.0, s1 = 0.0;
        for (int e = t; e < SB; e += kPA) {
            if (!act_e(e)) continue;
            const double sk = ::fma(a.reltol, kabs(lam[e]), a.abstol);
            const double r0 = lam[e] / sk, r1 = kl[e] / sk;
            s0 += r0 * r0;
            s1 += r1 * r1;
        }
        for (int64_t q = t; q < Pw; q += kPA) {
            const double m = mu[q];
            const double sk = ::fma(a.reltol, kabs(m), a.abstol);
            const double r0 = m / sk, r1 = km[q] / sk;
            s0 += r0 * r0;
            s1 += r1 * r1;
        }
        const double b0 = pa_bsum(s0, red), b1 = pa_bsum(s1, red);
        if (t == 0) {
            part[0] = b0;
            part[1] = b1;
        }
        __syncthreads();
        alive = pa_exchange(part, 2, hbar, pa.xbuf, pa.ctr, pa.abrt, nwg, ex++, tmp, &xflag);
        if (alive) {
            const double d0 = ::sqrt(hbar[0] / ntot), d1 = ::sqrt(hbar[1] / ntot);
            __syncthreads();
            double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
            h0 = ::fmin(h0, TT);
            for (int e = t; e < SB; e += kPA) lsv[e] = ::fma(h0, kl[e], lam[e]);
            __syncthreads();
            taus[0] = h0;
            alive = fwd_stages(taus, 1) && back_stage(0, 1, 1);
            flush_pending(true);
            ++nf;
            if (alive) {
                double s2 = 0.0;
                for (int e = t; e < SB; e += kPA) {
                    if (!act_e(e)) continue;
                    const double sk = ::fma(a.reltol, kabs(lam[e]), a.abstol);
                    const double ee = ::fma(-1.0, kl[e], kl[SB + e]) / sk;
                    s2 += ee * ee;
                }
                for (int64_t q = t; q < Pw; q += kPA) {
                    const double sk = ::fma(a.reltol, kabs(mu[q]), a.abstol);
                    const double ee = ::fma(-1.0, km[q], km[Pw + q]) / sk;
                    s2 += ee * ee;
                }
                const double b2 = pa_bsum(s2, red);
                if (t == 0) part[0] = b2;
                __syncthreads();
                alive = pa_exchange(part, 1, hbar, pa.xbuf, pa.ctr, pa.abrt, nwg, ex++, tmp, &xflag);
                if (alive) {
                    const double d2 = ::sqrt(hbar[0] / ntot) / h0;
                    __syncthreads();
                    const double mx = ::fmax(d1, d2);
                    const double h1 = mx <= 1e-15 ? ::fmax(1e-6, h0 * 1e-3) : ::pow(0.01 / mx, 1.0 / 5.0);
                    h = ::fmin(::fmin(100 * h0, h1), TT);
                }
            }
        }
    }
    double qold = a.qoldinit;
    for (; alive && it < a.maxiters; ++it) {
        if (tau >= TT - 1e-14 * ::fmax(1.0, TT)) break;
        h = ::fmin(h, a.stops[si] - tau);
        int ks[7];
        ks[0] = k0;
#pragma unroll
        for (int m = 1; m < 6; ++m) ks[m] = m;
        ks[6] = k0 == 0 ? 6 : 0;
#pragma unroll
        for (int i = 0; i < 6; ++i) taus[i] = i == 5 ? tau + h : tau + TC[i] * h;
        alive = fwd_stages(taus, 6);
        for (int i = 0; i < 6 && alive; ++i) {
            for (int e = t; e < SB; e += kPA) {
                double l = lam[e];
                for (int m = 0; m <= i; ++m) l = ::fma(h * TA[i][m], kl[(int64_t)ks[m] * SB + e], l);
                lsv[e] = l;
            }
            __syncthreads();
            alive = back_stage(i, ks[i + 1], ks[i + 1]);
        }
        if (!alive) break;
        flush_pending(true);
        nf += 6;
        // μ_new = μ + h Σ a_6j kμ_j and the error terms over this workgroup's λ and μ entries
        double* mu0 = mu + (int64_t)mc * Pw;
        double* mu1 = mu + (int64_t)(mc ^ 1) * Pw;
        double sacc = 0.0;
        for (int64_t q = t; q < Pw; q += kPA) {
            double v = mu0[q];
#pragma unroll
            for (int m = 0; m < 6; ++m) v = ::fma(h * TA[5][m], km[(int64_t)ks[m] * Pw + q], v);
            mu1[q] = v;
            if (a.adaptive) {
                double ev = 0.0;
#pragma unroll
                for (int m = 0; m < 6; ++m) ev = ::fma(h * BT[m], km[(int64_t)ks[m] * Pw + q], ev);
                const double ee = ::fma(h * BT[6], km[(int64_t)ks[6] * Pw + q], ev);
                const double sk = ::fma(a.reltol, ::fmax(kabs(mu0[q]), kabs(v)), a.abstol);
                sacc += (ee / sk) * (ee / sk);
            }
        }
        double hnew = h;
        if (a.adaptive) {
            for (int e = t; e < SB; e += kPA) {
                if (!act_e(e)) continue;
                double ev = 0.0;
#pragma unroll
                for (int m = 0; m < 6; ++m) ev = ::fma(h * BT[m], kl[(int64_t)ks[m] * SB + e], ev);
                const double ee = ::fma(h * BT[6], kl[(int64_t)ks[6] * SB + e], ev);
                const double sk = ::fma(a.reltol, ::fmax(kabs(lam[e]), kabs(lsv[e])), a.abstol);
                sacc += (ee / sk) * (ee / sk);
            }
            const double bs = pa_bsum(sacc, red);
            // A step that lands on a saveat stop re-evaluates the FSAL stage after the jump λ += ∂L/∂u (below).
            // Its partial hidden cotangents do not depend on the accept/reject decision, so they ride in the
            // error's exchange (speculatively: discarded when the step is rejected).  λs = λ_new + jump rows
            // (add_rows' order) overwrites lsv, which a rejected step recomputes anyway.
            const int64_t sj = si + 1;
            const bool spec = dl && ::fabs((tau + h) - a.stops[si]) <= 1e-12 * ::fmax(1.0, TT) && sj < a.nstops &&
                              a.joff[sj + 1] > a.joff[sj];
            if (spec) {
                for (int e = t; e < SB; e += kPA) {
                    if (!act_e(e)) continue;
                    double l = lsv[e];
                    for (int32_t q = a.joff[sj]; q < a.joff[sj + 1]; ++q) l = l + dl[(int64_t)a.jrows[q] * n + gidx(e)];
                    lsv[e] = l;
                }
                __syncthreads();
                part_b(5, part + 1);
            }
            if (t == 0) part[0] = bs;
            __syncthreads();
            PA_MARK(8);
            const unsigned eE = ex++;
            pa_publish(part, spec ? 1 + HB : 1, pa.xbuf, pa.ctr, nwg, eE);
            if (spec) dc2(5, ks[6]);   // kμ_7 of this step was consumed above (μ update, error terms)
            alive = pa_collect(spec ? 1 + HB : 1, wsp, pa.xbuf, pa.ctr, pa.abrt, nwg, eE, tmp, &xflag);
            PA_MARK(9);
            if (!alive) break;
            const double eest = ::sqrt(wsp[0] / ntot);
            const double q11 = eest > 0 ? ::pow(eest, a.beta1) : 0.0;
            if (eest > 1.0 && h > a.dtmin) {
                ++nreject;
                h = h / ::fmin(1.0 / a.qmin, q11 / a.gamma);
                __syncthreads();
                continue;
            }
            double q = q11 / ::pow(qold, a.beta2);
            q = ::fmax(1.0 / a.qmax, ::fmin(1.0 / a.qmin, q / a.gamma));
            if (1.0 <= q && q <= 1.0) q = 1.0;
            hnew = q > 0 ? h / q : h * a.qmax;
            qold = ::fmax(eest, a.qoldinit);
            if (spec) {
                for (int q2 = t; q2 < HB; q2 += kPA) hbar[q2] = wsp[1 + q2];
                __syncthreads();
                tau = a.stops[si];                                   // lands on the stop (checked above)
                for (int e = t; e < SB; e += kPA) lam[e] = lsv[e];   // λ <- λ_new + ∂L/∂u(t_j)
                mc ^= 1;
                k0 = ks[6];
                if (a.hs && blockIdx.x == 0 && t == 0 && naccept < a.hs_cap) a.hs[naccept] = h;
                ++naccept;
                xbar(5, k0, k0);   // u_modified!: FSAL re-evaluated at τ (stage slot 5's forward half)
                ++nf;
                si = sj < a.nstops ? sj : a.nstops - 1;
                h = hnew;
                continue;
            }
        }
        __syncthreads();   // mu1 complete
        tau = tau + h;
        for (int e = t; e < SB; e += kPA) lam[e] = lsv[e];   // λ <- the last stage input
        mc ^= 1;
        k0 = ks[6];        // FSAL: kλ_7, kμ_7 become the next step's first stage values
        __syncthreads();
        if (a.hs && blockIdx.x == 0 && t == 0 && naccept < a.hs_cap) a.hs[naccept] = h;
        ++naccept;
        if (::fabs(tau - a.stops[si]) <= 1e-12 * ::fmax(1.0, TT)) {
            tau = a.stops[si];
            if (si + 1 < a.nstops) {
                if (dl && a.joff[si + 2] > a.joff[si + 1]) {
                    add_rows((int)si + 1);               // callback: λ += ∂L/∂u(t_j)
                    set_ls(lam);
                    // u_modified!: FSAL re-evaluated at τ, the time of the last stage (slot 5: its forward
                    // half, hidden activations included, is still in place)
                    alive = back_stage(5, k0, k0);
                    ++nf;
                }
            }
            si = si + 1 < a.nstops ? si + 1 : a.nstops - 1;
        }
        h = hnew;
    }
    if (!alive) {
        if (blockIdx.x == 0 && t == 0) a.out[3] = 3;   // exchange abandoned (time-out)
        return;
    }
    if (it == a.maxiters && !(tau >= TT - 1e-14 * ::fmax(1.0, TT))) status = 1;
    if (dl) add_rows((int)a.nstops);
    if (a.du0)
        for (int e = t; e < SB; e += kPA)
            if (act_e(e)) reinterpret_cast<double*>(a.du0)[gidx(e)] = lam[e];
    if (a.dp) {
        double* dp = reinterpret_cast<double*>(a.dp);
        const double* m = mu + (int64_t)mc * Pw;
        for (int64_t q = t; q < Pw; q += kPA) {
            if (q < oW1) {
                if (q / (H * G1) < Sw) dp[L1.p_off + (int64_t)H * G1 * a0 + q] = m[q];
            } else if (q < oC2) {
                if ((q - oW1) / H < Sw) dp[L1.w_off + (int64_t)H * a0 + (q - oW1)] = m[q];
            } else if (q < oW2) {
                const int64_t r = q - oC2, c = r % GH2, ol = r / GH2;
                if (ol < Sw) dp[L2.p_off + a0 + ol + (int64_t)N2 * c] = m[q];
            } else {
                const int64_t r = q - oW2, j = r % H, ol = r / H;
                if (ol < Sw) dp[L2.w_off + a0 + ol + (int64_t)N2 * j] = m[q];
            }
        }
    }
#ifdef KAN_PA_PROF
    PA_MARK(10);
    if (blockIdx.x == 0 && t == 0)
        for (int i = 0; i < 16; ++i) g_pa_prof[i] = prof_acc[i];
#endif
    if (blockIdx.x == 0 && t == 0) {
        a.out[0] = naccept;
        a.out[1] = nreject;
        a.out[2] = nf;
        a.out[3] = status;
    }
}

// The persistent pair adjoint: fp64, one KDense(N -> H) + KDense(H -> N) pair with H·B <= 256, S points
// per workgroup (S = 0: the default 8), every workgroup resident at once (<= 256 of them, one per CU by
// their LDS), the LDS carve within 160 KB.  hipErrorNotSupported when the shape is not covered.
int pair_adjoint_workgroups(const LayerConst* hl, int64_t B, int S) {
    if (S <= 0) S = 8;
    return (hl[0].I + S - 1) / S;
}

hipError_t launch_kd_pair_adjoint(const LayerConst* hl, const LayerConst* dlc, const double* p, int64_t B,
                                  PairAdjArgs pa, hipStream_t st) {
    if (pa.S <= 0) pa.S = 8;
    const LayerConst &L1 = hl[0], &L2 = hl[1];
    if (L1.O != L2.I || L2.O != L1.I || L1.O > kWideOMax || B < 1 || (int64_t)kPANS * L1.O * B > kPAMaxXW || L1.G > kMaxGrid ||
        L2.G > kMaxGrid || (pa.S != 4 && pa.S != 8 && pa.S != 16))
        return hipErrorNotSupported;
    const int nwg = pair_adjoint_workgroups(hl, B, pa.S);
    const size_t lds = sizeof(double) * (size_t)pair_adj_lds_doubles(pa.S, (int)B, L1.O, L1.G, L2.G, L1.use_base,
                                                                        L2.use_base);
    if (nwg < 1 || nwg > 256 || lds > 158 * 1024) return hipErrorNotSupported;
    const void* fn = pa.S == 4    ? reinterpret_cast<const void*>(&kd_pair_adjoint_kernel<4>)
                     : pa.S == 8 ? reinterpret_cast<const void*>(&kd_pair_adjoint_kernel<8>)
                                 : reinterpret_cast<const void*>(&kd_pair_adjoint_kernel<16>);
    hipError_t e = ensure_dynamic_lds(fn, lds);
    if (e != hipSuccess) return e;
    // every workgroup spins on the others at each exchange, so all nwg must be resident at once: launch only
    // when the device's capacity for this kernel (workgroups per CU at this LDS carve x CUs) covers the grid
    // (a caller-set cap stands for a partitioned or shared device).  Otherwise the caller takes the
    // launch-per-stage path.  Work already running on the device can still hold CUs: the exchanges then
    // time out, the kernel reports it and the caller re-runs on that path too.
    int dev = 0, ncu = 0, per_cu = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    if ((e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kPA, lds)) != hipSuccess) return e;
    int64_t cap = (int64_t)per_cu * ncu;
    if (pa.max_wg > 0 && pa.max_wg < cap) cap = pa.max_wg;
    if (nwg > cap) return hipErrorNotSupported;
    e = hipMemsetAsync(pa.ctr, 0, 16, st);   // the arrival counter and the abort word
    if (e != hipSuccess) return e;
    if (pa.force_abort && (e = hipMemsetAsync(pa.abrt, 1, 1, st)) != hipSuccess) return e;
    if (pa.S == 4) hipLaunchKernelGGL(kd_pair_adjoint_kernel<4>, dim3(nwg), dim3(kPA), lds, st, dlc, p, B, pa);
    else if (pa.S == 8) hipLaunchKernelGGL(kd_pair_adjoint_kernel<8>, dim3(nwg), dim3(kPA), lds, st, dlc, p, B, pa);
    else hipLaunchKernelGGL(kd_pair_adjoint_kernel<16>, dim3(nwg), dim3(kPA), lds, st, dlc, p, B, pa);
    return hipGetLastError();
}

}  // namespace kan

#ifdef KAN_PA_PROF
// variant builds only: the phase ticks of the last launch (workgroup 0) in µs -> out[16]
extern "C" int kanode_debug_pair_profile(double* out) {
    unsigned long long v[16];
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(kan::g_pa_prof), sizeof(v)) != hipSuccess) return 1;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0) != hipSuccess || khz <= 0) return 2;
    for (int i = 0; i < 16; ++i) out[i] = (double)v[i] / (double)khz * 1e3;
    return 0;
}
#endif
