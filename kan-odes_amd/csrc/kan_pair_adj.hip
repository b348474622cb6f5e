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
constexpr int kPAMaxXW = 256;           // exchange width (H·B) cap
constexpr unsigned kPASpinMax = 1u << 22;   // a few seconds: far beyond any legitimate wait

__device__ __forceinline__ void st_agent(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// All nwg workgroups publish `cnt` values (vals[0..cnt) in LDS) as exchange e, then every workgroup
// forms out[q] = Σ_{w = 0..nwg-1} partial_w[q] in that order (the same bits everywhere).
// Returns false when the exchange was abandoned (abort raised / time-out): the caller exits.
__device__ bool pa_exchange(const double* vals, int cnt, double* out, double* xbuf, unsigned* ctr, unsigned* abrt,
                            int nwg, unsigned e, double* tmp /* LDS, >= kPA */, int* flag /* LDS */) {
    double* slot = xbuf + (size_t)(e & 1u) * nwg * kPAMaxXW;
    const int w = blockIdx.x;
    for (int q = threadIdx.x; q < cnt; q += kPA) st_agent(slot + (size_t)w * kPAMaxXW + q, vals[q]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    // fixed-order sum: thread t takes output q = t % cnt over the workgroup range of chunk t / cnt; the
    // chunk partials are then added in chunk order
    const int nch = cnt > 0 ? (kPA / cnt < nwg ? kPA / cnt : nwg) : 1;
    const int per = (nwg + nch - 1) / nch;
    if (threadIdx.x < nch * cnt) {
        const int q = threadIdx.x % cnt, c = threadIdx.x / cnt;
        const int w0 = c * per, w1 = w0 + per < nwg ? w0 + per : nwg;
        double s = 0.0;
        for (int ww = w0; ww < w1; ++ww) s = ww == w0 ? ld_agent(slot + (size_t)ww * kPAMaxXW + q)
                                                      : s + ld_agent(slot + (size_t)ww * kPAMaxXW + q);
        tmp[threadIdx.x] = s;
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

// LDS carve (doubles), S points per workgroup, B columns, H hidden, G1 / G2 knots:
//   ps[Pw] | mu[2][Pw] | km[7][Pw] | dens[8][S·B] | lam[S·B] | kl[7][S·B] | yv[S·B] | lsv[S·B] |
//   phi1[S·B·G1] | dphi1[S·B·G1] | sw1[S·B] | dsw1[S·B] | hid[H·B] | hbar[H·B] | psi[H·B·G2] |
//   dpsi[H·B·G2] | sw2[H·B] | dsw2[H·B] | part[H·B] | tmp[kPA] | red[4] | exp table[256]
__host__ __device__ inline int64_t pair_adj_pw(int S, int H, int G1, int G2, int ub1, int ub2) {
    return (int64_t)H * G1 * S + (int64_t)H * S * ub1 + (int64_t)S * G2 * H + (int64_t)S * H * ub2;
}
__host__ __device__ inline int64_t pair_adj_lds_doubles(int S, int B, int H, int G1, int G2, int ub1, int ub2) {
    const int64_t Pw = pair_adj_pw(S, H, G1, G2, ub1, ub2), SB = (int64_t)S * B, HB = (int64_t)H * B;
    return 10 * Pw + 8 * SB + 8 * SB + 2 * SB + 2 * SB * G1 + 2 * SB + 2 * HB + 2 * HB * G2 + 3 * HB + kPA + 4 + 256;
}

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
    const int S = pa.S, nwg = (int)gridDim.x;
    const int a0 = (int)blockIdx.x * S;
    const int Sw = N - a0 < S ? N - a0 : S;          // points of this workgroup (the last may hold fewer)
    const int SB = S * (int)B, HB = H * (int)B;
    const int64_t n = (int64_t)N * B;
    const int64_t Pw = pair_adj_pw(S, H, G1, G2, ub1, ub2);
    const int64_t oC1 = 0, oW1 = (int64_t)H * G1 * S, oC2 = oW1 + (int64_t)H * S * ub1,
                  oW2 = oC2 + (int64_t)S * G2 * H;

    extern __shared__ __attribute__((aligned(16))) double pa_lds[];
    double* ps = pa_lds;
    double* mu = ps + Pw;          // [2][Pw]
    double* km = mu + 2 * Pw;      // [7][Pw]
    double* dens = km + 7 * Pw;    // [8][SB]: u_i, k_1..k_7 of the cached forward step
    double* lam = dens + 8 * SB;   // [SB]
    double* kl = lam + SB;         // [7][SB]
    double* yv = kl + 7 * SB;
    double* lsv = yv + SB;
    double* phi1 = lsv + SB;       // [SB][G1]
    double* dphi1 = phi1 + (int64_t)SB * G1;
    double* sw1 = dphi1 + (int64_t)SB * G1;
    double* dsw1 = sw1 + SB;
    double* hid = dsw1 + SB;       // [HB]
    double* hbar = hid + HB;
    double* psi = hbar + HB;       // [HB][G2]
    double* dpsi = psi + (int64_t)HB * G2;
    double* sw2 = dpsi + (int64_t)HB * G2;
    double* dsw2 = sw2 + HB;
    double* part = dsw2 + HB;      // [HB] this workgroup's partials of an exchange
    double* tmp = part + HB;       // [kPA]
    double* red = tmp + kPA;       // [4]
    double* tab = red + 4;         // [256] exp table
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
            const int64_t r = q - oC2, ol = r % S, c = r / S;
            g = L2.p_off + a0 + ol + (int64_t)N2 * c;
        } else {                                                                          // W2[o, j]
            const int64_t r = q - oW2, ol = r % S, j = r / S;
            g = L2.w_off + a0 + ol + (int64_t)N2 * j;
        }
        const bool live = (q < oC2) ? ((q < oW1 ? (q / (H * G1)) : ((q - oW1) / H)) < Sw)
                                    : (((q < oW2 ? (q - oC2) : (q - oW2)) % S) < Sw);
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

    // adjoint RHS at τ with the stage input ls (lsv, LDS): kλ -> kl[kslot], kμ -> km[mslot]
    auto adj = [&](double tau, int kslot, int mslot) -> bool {
        const double tt = tf - tau;
        while (cur > 0 && a.ts[cur] > tt) --cur;
        while (cur + 1 < a.nsteps && a.ts[cur + 1] <= tt) ++cur;
        if (cur != cached) {       // the forward step's u_i, k_1..k_7 over this slice
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
        }
        const double dti = a.dts[cur];
        const double th = ::fmin(1.0, ::fmax(0.0, (tt - a.ts[cur]) / dti));
        double cw[7];
#pragma unroll
        for (int m = 0; m < 7; ++m) {
            double s = 0.0, tp = th;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                s += RI[m][r] * tp;
                tp *= th;
            }
            cw[m] = s * dti;
        }
        // y = u_i + Σ_m (dt b_m(θ)) k_m (stage_lincomb order), then layer 1's basis per (point, column, knot)
        for (int e = t; e < SB; e += kPA) {
            double y = dens[e];
#pragma unroll
            for (int m = 0; m < 7; ++m) y = ::fma(cw[m], dens[(m + 1) * SB + e], y);
            yv[e] = y;
        }
        __syncthreads();
        for (int q = t; q < SB * G1; q += kPA) {
            const int e = q / G1, g = q - e * G1;
            const double y = yv[e];
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
                sw1[e] = act_e(e) ? sw : 0.0;
                dsw1[e] = act_e(e) ? dsw : 0.0;
            }
        }
        __syncthreads();
        // exchange A: partial pre-activations over this slice
        for (int q = t; q < HB; q += kPA) {
            const int j = q % H, k = q / H;
            double s = 0.0;
            for (int il = 0; il < Sw; ++il) {
                const int e = il + S * k;
                for (int g = 0; g < G1; ++g) s = ::fma(ps[oC1 + j + H * (g + G1 * il)], phi1[e * G1 + g], s);
                if (ub1) s = ::fma(ps[oW1 + j + H * il], sw1[e], s);
            }
            part[q] = s;
        }
        __syncthreads();
        if (!pa_exchange(part, HB, hid, pa.xbuf, pa.ctr, pa.abrt, nwg, ex++, tmp, &xflag)) return false;
        // layer 2 at the hidden activations (every workgroup: the same values)
        for (int q = t; q < HB * G2; q += kPA) {
            const int jk = q / G2, g = q - jk * G2;
            const double h = hid[jk];
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
                sw2[jk] = sw;
                dsw2[jk] = dsw;
            }
        }
        __syncthreads();
        // exchange B: partial hidden cotangents over this slice's output rows
        for (int q = t; q < HB; q += kPA) {
            const int j = q % H, k = q / H;
            double s = 0.0;
            for (int g = 0; g < G2; ++g) {
                double c = 0.0;
                for (int ol = 0; ol < Sw; ++ol) c = ::fma(lsv[ol + S * k], ps[oC2 + ol + S * (g + G2 * j)], c);
                s = ::fma(dpsi[q * G2 + g], c, s);
            }
            if (ub2) {
                double c = 0.0;
                for (int ol = 0; ol < Sw; ++ol) c = ::fma(lsv[ol + S * k], ps[oW2 + ol + S * j], c);
                s = ::fma(dsw2[q], c, s);
            }
            part[q] = s;
        }
        // layer 2's parameter cotangents (own rows): dC2[o, g + G2 j] = Σ_k λs_ok ψ_g(h_jk)
        double* kmm = km + (int64_t)mslot * Pw;
        for (int64_t q = t; q < (int64_t)S * G2 * H; q += kPA) {
            const int ol = (int)(q % S), c = (int)(q / S), g = c % G2, j = c / G2;
            double s = 0.0;
            for (int k = 0; k < (int)B; ++k) s = ::fma(lsv[ol + S * k], psi[(j + H * k) * G2 + g], s);
            kmm[oC2 + q] = ol < Sw ? s : 0.0;
        }
        if (ub2)
            for (int q = t; q < S * H; q += kPA) {
                const int ol = q % S, j = q / S;
                double s = 0.0;
                for (int k = 0; k < (int)B; ++k) s = ::fma(lsv[ol + S * k], sw2[j + H * k], s);
                kmm[oW2 + q] = ol < Sw ? s : 0.0;
            }
        __syncthreads();
        if (!pa_exchange(part, HB, hbar, pa.xbuf, pa.ctr, pa.abrt, nwg, ex++, tmp, &xflag)) return false;
        // layer 1's pullback on this slice: kλ and the input-column parameter cotangents
        double* klo = kl + (int64_t)kslot * SB;
        for (int e = t; e < SB; e += kPA) {
            const int il = e % S, k = e / S;
            double s = 0.0;
            if (il < Sw) {
                for (int g = 0; g < G1; ++g) {
                    double c = 0.0;
                    for (int j = 0; j < H; ++j) c = ::fma(hbar[j + H * k], ps[oC1 + j + H * (g + G1 * il)], c);
                    s = ::fma(dphi1[e * G1 + g], c, s);
                }
                if (ub1) {
                    double c = 0.0;
                    for (int j = 0; j < H; ++j) c = ::fma(hbar[j + H * k], ps[oW1 + j + H * il], c);
                    s = ::fma(dsw1[e], c, s);
                }
            }
            klo[e] = s;
        }
        for (int64_t q = t; q < (int64_t)H * G1 * S; q += kPA) {
            const int j = (int)(q % H), c = (int)(q / H), g = c % G1, il = c / G1;
            double s = 0.0;
            for (int k = 0; k < (int)B; ++k) s = ::fma(hbar[j + H * k], phi1[(il + S * k) * G1 + g], s);
            kmm[oC1 + q] = s;
        }
        if (ub1)
            for (int q = t; q < H * S; q += kPA) {
                const int j = q % H, il = q / H;
                double s = 0.0;
                for (int k = 0; k < (int)B; ++k) s = ::fma(hbar[j + H * k], sw1[il + S * k], s);
                kmm[oW1 + q] = s;
            }
        __syncthreads();
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
    if (dl) add_rows(0);
    set_ls(lam);
    alive = adj(0.0, 0, 0);
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
        part[0] = pa_bsum(s0, red);
        part[1] = pa_bsum(s1, red);
        __syncthreads();
        double tot[2];
        alive = pa_exchange(part, 2, hid, pa.xbuf, pa.ctr, pa.abrt, nwg, ex++, tmp, &xflag);
        if (alive) {
            tot[0] = hid[0];
            tot[1] = hid[1];
            __syncthreads();
            const double d0 = ::sqrt(tot[0] / ntot), d1 = ::sqrt(tot[1] / ntot);
            double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
            h0 = ::fmin(h0, TT);
            for (int e = t; e < SB; e += kPA) lsv[e] = ::fma(h0, kl[e], lam[e]);
            __syncthreads();
            alive = adj(h0, 1, 1);
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
                part[0] = pa_bsum(s2, red);
                __syncthreads();
                alive = pa_exchange(part, 1, hid, pa.xbuf, pa.ctr, pa.abrt, nwg, ex++, tmp, &xflag);
                if (alive) {
                    const double d2 = ::sqrt(hid[0] / ntot) / h0;
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
        for (int i = 0; i < 6 && alive; ++i) {
            for (int e = t; e < SB; e += kPA) {
                double l = lam[e];
                for (int m = 0; m <= i; ++m) l = ::fma(h * TA[i][m], kl[(int64_t)ks[m] * SB + e], l);
                lsv[e] = l;
            }
            __syncthreads();
            alive = adj(i == 5 ? tau + h : tau + TC[i] * h, ks[i + 1], ks[i + 1]);
        }
        if (!alive) break;
        nf += 6;
        // μ_new = μ + h Σ a_6j kμ_j and the error terms over this workgroup's λ and μ entries
        double* mu0 = mu + (int64_t)mc * Pw;
        double* mu1 = mu + (int64_t)(mc ^ 1) * Pw;
        double s = 0.0;
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
                s += (ee / sk) * (ee / sk);
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
                s += (ee / sk) * (ee / sk);
            }
            part[0] = pa_bsum(s, red);
            __syncthreads();
            alive = pa_exchange(part, 1, hid, pa.xbuf, pa.ctr, pa.abrt, nwg, ex++, tmp, &xflag);
            if (!alive) break;
            const double eest = ::sqrt(hid[0] / ntot);
            __syncthreads();
            const double q11 = eest > 0 ? ::pow(eest, a.beta1) : 0.0;
            if (eest > 1.0 && h > a.dtmin) {
                ++nreject;
                h = h / ::fmin(1.0 / a.qmin, q11 / a.gamma);
                continue;
            }
            double q = q11 / ::pow(qold, a.beta2);
            q = ::fmax(1.0 / a.qmax, ::fmin(1.0 / a.qmin, q / a.gamma));
            if (1.0 <= q && q <= 1.0) q = 1.0;
            hnew = q > 0 ? h / q : h * a.qmax;
            qold = ::fmax(eest, a.qoldinit);
        }
        __syncthreads();   // mu1 complete
        tau = tau + h;
        for (int e = t; e < SB; e += kPA) lam[e] = lsv[e];   // λ <- the last stage input
        mc ^= 1;
        k0 = ks[6];        // FSAL: kλ_7, kμ_7 become the next step's first stage values
        __syncthreads();
        ++naccept;
        if (::fabs(tau - a.stops[si]) <= 1e-12 * ::fmax(1.0, TT)) {
            tau = a.stops[si];
            if (si + 1 < a.nstops) {
                if (dl && a.joff[si + 2] > a.joff[si + 1]) {
                    add_rows((int)si + 1);               // callback: λ += ∂L/∂u(t_j)
                    set_ls(lam);
                    alive = adj(tau, k0, k0);            // u_modified!: FSAL re-evaluated
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
                const int64_t r = q - oC2, ol = r % S, c = r / S;
                if (ol < Sw) dp[L2.p_off + a0 + ol + (int64_t)N2 * c] = m[q];
            } else {
                const int64_t r = q - oW2, ol = r % S, j = r / S;
                if (ol < Sw) dp[L2.w_off + a0 + ol + (int64_t)N2 * j] = m[q];
            }
        }
    }
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
    if (L1.O != L2.I || L2.O != L1.I || B < 1 || (int64_t)L1.O * B > kPAMaxXW || L1.G > kMaxGrid ||
        L2.G > kMaxGrid)
        return hipErrorNotSupported;
    const int nwg = pair_adjoint_workgroups(hl, B, pa.S);
    const size_t lds = sizeof(double) * (size_t)pair_adj_lds_doubles(pa.S, (int)B, L1.O, L1.G, L2.G, L1.use_base,
                                                                        L2.use_base);
    if (nwg < 1 || nwg > 256 || lds > 150 * 1024) return hipErrorNotSupported;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&kd_pair_adjoint_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(pa.ctr, 0, 16, st);   // the arrival counter and the abort word
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kd_pair_adjoint_kernel, dim3(nwg), dim3(kPA), lds, st, dlc, p, B, pa);
    return hipGetLastError();
}

}  // namespace kan
