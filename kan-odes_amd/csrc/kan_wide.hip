// kan_wide.hip — KDense kernels for the full-field surrogate shapes (gfx950).
//
// The surrogate drivers chain KDense(N, 10, G) -> KDense(10, N, G) on a few
// trajectories (PDE examples/Burgers_Surrogate.jl:85-88, Schrodinger_Surrogate.jl:93-96;
// KDense forward kdense.jl:109-130).  With B <= 8 columns the contraction is a
// parameter-streaming GEMV, not a GEMM: VALU + reductions, no MFMA.
//
// The batch is a handful of trajectories, so the kernels spread each column over many
// workgroups instead of looping over the columns in a few:
//   wide-in  (I·G large, O <= 16): grid (input chunk, column); the chunk's C and W blocks are
//            contiguous and read with coalesced loads (thread t meets output t mod O), the
//            chunk's basis values staged in LDS meanwhile; per-output partials (slab), then an
//            ordered reduction over the chunks.
//   wide-out (O large): grid (row chunk of 256, column tile of 8); the block stages the
//            small basis of its tile in LDS; C[o + O*c] reads are coalesced over o.
// Pullbacks: wide-out parameters -- thread o owns dC[o, :], dW[o, :] (no reduction);
// wide-out input cotangent -- one workgroup per (input i, basis row r, column tile) forms
// Σ_o C[o, r + G i] ȳ[o, k] (coalesced over o, ordered block sum) into a slab, then one
// thread per (i, k) turns the G + 1 sums into x̄[i, k];
// wide-in -- one block per input chunk owns the chunk's dC, dW entries (coalesced, columns summed
// in order), other blocks form x̄ per column (one thread per basis slot, then per input).  Every reduction runs in a fixed order (bitwise reproducible).
// Surrogate chain [wide-in, wide-out]: the wide-out kernels can take their input as the
// wide-in layer's chunk partials (`xslab`), each block summing what it needs in the order of
// kd_widein_reduce_kernel, so the chain RHS is two launches and its VJP four, bitwise equal to
// the layer-by-layer path.
#include "kan_common.hpp"
#include "kan_kernels.hpp"

namespace kan {


constexpr int kKT = 8;        // column tile (trajectories per pass)
constexpr int kOWide = 16;    // max out_dims of a wide-in layer

// basis value/argument/aux for (input value xi, knot g) — direct or recurrence
template <typename T, int PATH>
struct Basis1 {
    T n, z0, F, R, tau, invh;
    __device__ __forceinline__ void init(const Math<T>& M, const LayerConst& lc, T xi) {
        n = normalize<NORM_RUNTIME, T>(M, lc.norm, xi);
        invh = T(lc.invh);
        if constexpr (PATH != PATH_DIRECT) rec_anchor<T>(M, lc, n, z0, F, R, tau);
    }
    __device__ __forceinline__ T next(const Math<T>& M, const LayerConst& lc, int g, T& z, T& aux) {
        if constexpr (PATH == PATH_DIRECT) {
            z = (n - T(lc.grid[g])) * invh;
            aux = T(0);
            return basis_direct<T>(M, lc.basis, z, aux);
        } else {
            T kc = T(lc.K[g]);
            if constexpr (PATH == PATH_REC_CORR) {
                const T e = T(lc.e[g]);
                kc = kc * kfma<T>(tau, kfma<T>(tau, T(0.5) * e * e, e), T(1));
            }
            const T v = F * kc;
            z = z0 - T(lc.Dl[g]);
            aux = T(0);
            F = F * R;
            return v;
        }
    }
};

// ---------------------------------------------------------------------------
constexpr int kSW = 4;     // waves per wide-out workgroup splitting the inner loop (latency: more loads in flight)

// Element x[i, k] of a layer input [I, K]: from x, or (xslab != nullptr) the ordered sum over the
// nblk chunk partials of the wide-in layer that produced it, xslab[(b*K + k)*I + i] -- the order
// of kd_widein_reduce_kernel.
template <typename T>
__device__ __forceinline__ T layer_in(const T* __restrict__ x, const T* __restrict__ xslab, int nblk, int I, int64_t K,
                                      int i, int64_t k) {
    if (!xslab) return x[(int64_t)I * k + i];
    // 16 partials in flight per round (a plain loop would wait for each load before the next
    // add); the additions keep the reduce kernel's order
    constexpr int kR = 16;
    const T* __restrict__ src = xslab + k * I + i;
    const int64_t stride = K * I;
    T s = T(0);
    for (int b0 = 0; b0 < nblk; b0 += kR) {
        T v[kR];
#pragma unroll
        for (int j = 0; j < kR; ++j) v[j] = b0 + j < nblk ? src[(int64_t)(b0 + j) * stride] : T(0);
#pragma unroll
        for (int j = 0; j < kR; ++j)
            if (b0 + j < nblk) s += v[j];
    }
    return s;
}

// wide-in forward, coalesced: grid (chunks of cw inputs, columns), 256 threads.  The chunk's C
// block (O·G·cw doubles) and W block (O·cw) are contiguous in the ComponentArray vector
// (C[o + O(g + G i)], W[o + O i]); thread t takes the entries t + m·Tn, Tn = ⌊256/O⌋·O, so every
// load instruction reads a contiguous run and thread t always meets output o = t mod O.  The C
// and W loads are issued before the chunk's basis values are staged in LDS (by the first cw
// threads), so their latency overlaps the exponentials.  Per-thread partials are summed per
// output in thread order: slab[(chunk*K + k)*O + o].
// With stage_on the chunk's inputs are the stage input y = x + Σ su.c·su.k, formed by the first ni
// threads into LDS (and y_out), which also form λs over the same range (WideStageIn).
template <typename T>
__device__ __forceinline__ T wide_stage_comb(const T* __restrict__ base, const StageArgs<T>& sa, int64_t idx) {
    const double sc = stage_scale(sa.cscale);
    T kv[kMaxStages];
    stage_ld<T>(sa, base, idx, kv);
    T v = base[idx];
#pragma unroll
    for (int j = 0; j < kMaxStages; ++j)
        if (j < sa.nk) v = kfma<T>((T)(sa.c[j] * sc), kv[j], v);
    return v;
}
// the same combination with its last array's entry given (the value the fused pair step's block has
// just formed itself, kd_vjp_pair_ba_kernel): the same fma order, so the same bits
template <typename T>
__device__ __forceinline__ T wide_stage_comb_last(const T* __restrict__ base, const StageArgs<T>& sa, int64_t idx,
                                                  T last) {
    const double sc = stage_scale(sa.cscale);
    T kv[kMaxStages];
    stage_ld<T>(sa, base, idx, kv);
    T v = base[idx];
#pragma unroll
    for (int j = 0; j < kMaxStages; ++j)
        if (j < sa.nk) v = kfma<T>((T)(sa.c[j] * sc), j == sa.nk - 1 ? last : kv[j], v);
    return v;
}
// MV / MW: C / W load slots per thread (>= the chunk's entries / tn; the launch picks the smallest
// instantiation that covers the chunk -- unused predicated slots still cost instructions).
// The pair pullback's dot products, formed by the wide-in forward blocks (DOT): the chunk's input
// range [i0, i0 + ni) is also an output range of the wide-out layer (N_in == N_out), so the block
// that holds ȳ[i0 .. i0 + ni, k] (λs it formed, or λ) forms the partial sums
//     spart[(bx·IR + q)·K + k] = Σ_{o in chunk} row_q[o] ȳ[o, k],   row_q = C2[:, r + G2 i2] (r < G2) or
// W2[:, i2] (r = G2), q = i2·R2 + r, IR = I2·R2; the consumer sums the nblk chunk partials in order.
// The pair's forward blocks also store the wide-in layer's basis values (WideBasisG, kan_kernels.hpp),
// which the pullback's parameter and x̄ blocks would otherwise recompute (one exponential each, ten times
// over for the ten parameter blocks of a chunk).  Bitwise the values the recomputation gives.
template <typename T>
struct PairDot {
    const LayerConst* lc1;
    T* spart;
    const T* ybar;   // ȳ without a stage (λ); with a stage, λs as the block forms it
    WideBasisG<T> bg;   // basis store (bg.phi == nullptr: none)
};
template <typename T, bool STAGE, int MV, int MW, bool DOT = false>
__device__ __forceinline__ void widein_fwd_body(const LayerConst* __restrict__ lcp, const T* __restrict__ p,
                                                const T* __restrict__ x, T* __restrict__ slab, int64_t K,
                                                const WideStageIn<T>* si, int bx, int by, int gy,
                                                const PairDot<T>* pd = nullptr, const T* lastk = nullptr) {
    __shared__ T phiL[kWideInMaxInputs * kMaxGrid];
    __shared__ T swL[kWideInMaxInputs];
    __shared__ T xL[kWideInMaxInputs];
    __shared__ T lsL[DOT ? kWideInMaxInputs : 1];
    __shared__ T red[256];
    const Math<T> M{kExp2Tab256};
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;
    const int cw = widein_cw(O, G, I);
    const int i0 = bx * cw;
    const int ni = I - i0 < cw ? I - i0 : cw;
    const int tn = (256 / O) * O, t = threadIdx.x;
    const int nf = O * G * ni, nw = lc.use_base ? O * ni : 0;
    const T* __restrict__ Cb = p + lc.p_off + (int64_t)O * G * i0;
    const T* __restrict__ Wb = p + lc.w_off + (int64_t)O * i0;
    const int c0 = t / O, cs = tn / O;   // entry t + m·tn belongs to basis slot c0 + m·cs
    for (int64_t k = by; k < K; k += gy) {
        T cv[MV], wv[MW];
#pragma unroll
        for (int m = 0; m < MV; ++m) {
            const int f = t + m * tn;
            cv[m] = t < tn && f < nf ? Cb[f] : T(0);
        }
#pragma unroll
        for (int m = 0; m < MW; ++m) {
            const int f = t + m * tn;
            wv[m] = t < tn && f < nw ? Wb[f] : T(0);
        }
        if constexpr (STAGE) {
            // y by the first wave, λs by the second (ni <= 64): the two combinations' loads in flight
            // together (in one thread the y_out store, which may alias λ, kept them one round apart)
            if (t < ni) {
                const int64_t idx = (int64_t)I * k + i0 + t;
                const T v = wide_stage_comb<T>(x, si->su, idx);
                xL[t] = v;
                if (si->y_out) si->y_out[idx] = v;
            } else if (t >= kWideInMaxInputs && t - kWideInMaxInputs < ni && si->lam) {
                const int tl = t - kWideInMaxInputs;
                const int64_t idx = (int64_t)I * k + i0 + tl;
                const T l = lastk ? wide_stage_comb_last<T>(si->lam, si->sl, idx, lastk[tl])
                                  : wide_stage_comb<T>(si->lam, si->sl, idx);
                si->ls_out[idx] = l;
                if constexpr (DOT) lsL[tl] = l;
            }
            __syncthreads();
        } else if constexpr (DOT) {
            if (t < ni) lsL[t] = pd->ybar[(int64_t)I * k + i0 + t];
        }
        // one thread per basis slot c = g + G i (direct formula: no per-input knot chain)
        for (int c = t; c < ni * G; c += blockDim.x) {
            const int i = c / G, g = c - i * G;
            const T xi = STAGE ? xL[i] : x[(int64_t)I * k + i0 + i];
            const T n = normalize<NORM_RUNTIME, T>(M, lc.norm, xi);
            T aux = T(0);
            const T ph = basis_direct<T>(M, lc.basis, (n - T(lc.grid[g])) * T(lc.invh), aux);
            phiL[c] = ph;
            bool stored = false;
            if constexpr (DOT) {
                if (pd->bg.phi) {
                    pd->bg.phi[((int64_t)I * k + i0) * G + c] = ph;
                    if (g == 0) {
                        T sw = T(0), dsw = T(0);
                        if (lc.use_base) swish_and_grad<T>(M, xi, sw, dsw);
                        swL[i] = sw;
                        pd->bg.sw[(int64_t)I * k + i0 + i] = sw;
                        pd->bg.dsw[(int64_t)I * k + i0 + i] = dsw;
                    }
                    stored = true;
                }
            }
            if (g == 0 && !stored) swL[i] = lc.use_base ? swish<T>(M, xi) : T(0);
        }
        __syncthreads();
        T acc = T(0);
        if (t < tn) {
#pragma unroll
            for (int m = 0; m < MV; ++m)
                if (t + m * tn < nf) acc = kfma<T>(cv[m], phiL[c0 + m * cs], acc);
#pragma unroll
            for (int m = 0; m < MW; ++m)
                if (t + m * tn < nw) acc = kfma<T>(wv[m], swL[c0 + m * cs], acc);
        }
        red[t] = acc;
        __syncthreads();
        if (t < O) {
            T sum = red[t];
#pragma unroll 8
            for (int q = 1; q < cs; ++q) sum += red[t + q * O];
            slab[((int64_t)bx * K + k) * O + t] = sum;
        }
        __syncthreads();
        if constexpr (DOT) {
            // rows q of the wide-out layer against the chunk's ȳ: thread (q, s) sums entries t ≡ s
            // (mod ns) of the chunk, then the ns sub-sums of row q are added in order (LDS `red`)
            const LayerConst& l1 = *pd->lc1;
            const int R1 = l1.G + (l1.use_base ? 1 : 0), IR = l1.I * R1, O1 = l1.O;
            const int ns = IR >= 256 ? 1 : 256 / IR;
            for (int q0 = 0; q0 < IR; q0 += 256 / ns) {
                const int q = q0 + t / ns, sub = t - (t / ns) * ns;
                T a = T(0);
                if (q < IR && t / ns < 256 / ns) {
                    const int i2 = q / R1, r = q - i2 * R1;
                    const T* __restrict__ row =
                        r < l1.G ? p + l1.p_off + (int64_t)O1 * (r + (int64_t)l1.G * i2) : p + l1.w_off + (int64_t)O1 * i2;
                    // (eight row loads in flight before the fma chain measured slower: Burgers VJP
                    // 15.9 -> 17.1 us)
                    for (int e = sub; e < ni; e += ns) a = kfma<T>(row[i0 + e], lsL[e], a);
                }
                red[t] = a;
                __syncthreads();
                if (t < 256 / ns && q0 + t < IR) {
                    T sum = red[t * ns];
                    for (int s2 = 1; s2 < ns; ++s2) sum += red[t * ns + s2];
                    pd->spart[((int64_t)bx * IR + q0 + t) * K + k] = sum;
                }
                __syncthreads();
            }
        }
    }
}
// (two kernels: the plain forward keeps a small argument block, the stage form carries StageArgs)
template <typename T, int MV, int MW>
__global__ void __launch_bounds__(256)
kd_fwd_widein_co_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                        T* __restrict__ slab, int64_t K) {
    widein_fwd_body<T, false, MV, MW>(lcp, p, x, slab, K, nullptr, blockIdx.x, blockIdx.y, gridDim.y);
}
template <typename T, int MV, int MW>
__global__ void __launch_bounds__(256)
kd_fwd_widein_stage_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                           T* __restrict__ slab, int64_t K, WideStageIn<T> si) {
    widein_fwd_body<T, true, MV, MW>(lcp, p, x, slab, K, &si, blockIdx.x, blockIdx.y, gridDim.y);
}

// y[o + O*k] = Σ_b slab[(b*K + k)*O + o]   (ordered over b)
template <typename T>
__global__ void __launch_bounds__(kBlock)
kd_widein_reduce_kernel(const T* __restrict__ slab, int nblk, int O, int64_t K, T* __restrict__ y) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)O * K) return;
    const int64_t k = idx / O;
    const int o = (int)(idx - k * O);
    y[(int64_t)O * k + o] = layer_in<T>(nullptr, slab, nblk, O, K, o, k);
}

// Basis values of a column tile of the (short) input, staged in LDS:
// phiL[(g + G i)*kKT + kk], swL[i*kKT + kk] (zero outside the tile).
template <typename T, int PATH>
__device__ __forceinline__ void stage_tile_basis(const Math<T>& M, const LayerConst& lc, const T* __restrict__ x,
                                                 const T* __restrict__ xslab, int nblk, int64_t K, int64_t k0, int kt,
                                                 T* phiL, T* swL) {
    const int I = lc.I, G = lc.G;
    for (int t = threadIdx.x; t < I * kKT; t += blockDim.x) {
        const int i = t / kKT, kk = t - i * kKT;
        if (kk < kt) {
            const T xi = layer_in<T>(x, xslab, nblk, I, K, i, k0 + kk);
            Basis1<T, PATH> bs;
            bs.init(M, lc, xi);
            for (int g = 0; g < G; ++g) {
                T z, aux;
                phiL[(g + G * i) * kKT + kk] = bs.next(M, lc, g, z, aux);
            }
            swL[i * kKT + kk] = lc.use_base ? swish<T>(M, xi) : T(0);
        } else {
            for (int g = 0; g < G; ++g) phiL[(g + G * i) * kKT + kk] = T(0);
            swL[i * kKT + kk] = T(0);
        }
    }
}

// ---------------------------------------------------------------------------
// wide-out forward: grid (ceil(O/64), column tiles); lane o contracts its row of C against
// the tile's basis, the kSW waves of the workgroup splitting the G·I columns of C (the
// launch is latency bound at a few trajectories: more workgroups and more loads in flight
// beat longer per-lane loops); partials are summed in wave order through LDS.
constexpr int kWOB = 64;
template <typename T, int PATH>
__global__ void __launch_bounds__(kWOB * kSW)
kd_fwd_wideout_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                      const T* __restrict__ xslab, int nblk, T* __restrict__ y, int64_t K) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    __shared__ T red[kSW][kKT][kWOB];
    const Math<T> M{kExp2Tab256};   // exp table from global memory (L1): no staging round trip
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;
    const int GI = G * I;
    T* phiL = reinterpret_cast<T*>(smem_raw);       // [GI][kKT]
    T* swL = phiL + (int64_t)GI * kKT;              // [I][kKT]
    const T* __restrict__ C = p + lc.p_off;
    const T* __restrict__ W = p + lc.w_off;
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const int o = blockIdx.x * kWOB + lane;
    for (int64_t k0 = (int64_t)blockIdx.y * kKT; k0 < K; k0 += (int64_t)gridDim.y * kKT) {
        const int kt = (int)((K - k0) < kKT ? (K - k0) : kKT);
        __syncthreads();
        stage_tile_basis<T, PATH>(M, lc, x, xslab, nblk, K, k0, kt, phiL, swL);
        __syncthreads();
        T acc[kKT];
#pragma unroll
        for (int kk = 0; kk < kKT; ++kk) acc[kk] = T(0);
        if (o < O) {
#pragma unroll 4
            for (int c = w; c < GI; c += kSW) {
                const T cv = C[o + (int64_t)O * c];
#pragma unroll
                for (int kk = 0; kk < kKT; ++kk) acc[kk] = kfma<T>(cv, phiL[c * kKT + kk], acc[kk]);
            }
            if (lc.use_base) {
#pragma unroll 2
                for (int i = w; i < I; i += kSW) {
                    const T wv = W[o + (int64_t)O * i];
#pragma unroll
                    for (int kk = 0; kk < kKT; ++kk) acc[kk] = kfma<T>(wv, swL[i * kKT + kk], acc[kk]);
                }
            }
        }
#pragma unroll
        for (int kk = 0; kk < kKT; ++kk) red[w][kk][lane] = acc[kk];
        __syncthreads();
        if (w == 0 && o < O) {
#pragma unroll
            for (int kk = 0; kk < kKT; ++kk) {
                if (kk < kt) {
                    T sum = red[0][kk][lane];
#pragma unroll
                    for (int v = 1; v < kSW; ++v) sum += red[v][kk][lane];
                    y[(int64_t)O * (k0 + kk) + o] = sum;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// wide-out pullback, parameters: workgroup (row chunk, input i); lane o owns
// dC[o, g + G i] (g < G) and dW[o, i] in registers, the kSW waves taking every kSW-th
// column; the wave partials are summed in order through LDS and added to pbar once
// (coalesced over o).  The basis of input i is staged in LDS kWOPK columns at a time.
constexpr int kWOPK = 128;
// Ph: LDS of (kMaxGrid + 1)·wk entries, wk <= kWOPK the column tile (the caller's: a static array in
// the dot+param launch, a K-sized slice of the dynamic block in the pair pullback).
template <typename T, int PATH>
__device__ __forceinline__ void wideout_param_body(const Math<T>& M, const LayerConst* __restrict__ lcp,
                                                   const T* __restrict__ x, const T* __restrict__ xslab, int nblk,
                                                   const T* __restrict__ ybar, T* __restrict__ pbar, int64_t K,
                                                   int bx, int i, int assign, T* __restrict__ Ph, int wk) {
    __shared__ T red[kSW][kWOB];
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const int o = bx * kWOB + lane;
    const bool base = lc.use_base != 0;
    T acc[kMaxGrid + 1];
#pragma unroll
    for (int r = 0; r <= kMaxGrid; ++r) acc[r] = T(0);
    for (int64_t k0 = 0; k0 < K; k0 += wk) {
        const int kt = (int)((K - k0) < wk ? (K - k0) : wk);
        __syncthreads();
        for (int kk = threadIdx.x; kk < kt; kk += blockDim.x) {
            const T xi = layer_in<T>(x, xslab, nblk, I, K, i, k0 + kk);
            Basis1<T, PATH> bs;
            bs.init(M, lc, xi);
            for (int g = 0; g < G; ++g) {
                T z, aux;
                Ph[g * wk + kk] = bs.next(M, lc, g, z, aux);
            }
            Ph[kMaxGrid * wk + kk] = base ? swish<T>(M, xi) : T(0);
        }
        __syncthreads();
        if (o < O) {
#pragma unroll 2
            for (int kk = w; kk < kt; kk += kSW) {
                const T yb = ybar[(int64_t)O * (k0 + kk) + o];
#pragma unroll
                for (int r = 0; r < kMaxGrid; ++r)
                    if (r < G) acc[r] = kfma<T>(yb, Ph[r * wk + kk], acc[r]);
                acc[kMaxGrid] = kfma<T>(yb, Ph[kMaxGrid * wk + kk], acc[kMaxGrid]);
            }
        }
    }
    T* __restrict__ dC = pbar + lc.p_off + o + (int64_t)O * G * i;
#pragma unroll
    for (int r = 0; r <= kMaxGrid; ++r) {
        if (r < G || (r == kMaxGrid && base)) {
            __syncthreads();
            red[w][lane] = acc[r];
            __syncthreads();
            if (w == 0 && o < O) {
                T sum = red[0][lane];
#pragma unroll
                for (int v = 1; v < kSW; ++v) sum += red[v][lane];
                T* dst = r < G ? dC + (int64_t)O * r : pbar + lc.w_off + o + (int64_t)O * i;
                *dst = assign ? sum : *dst + sum;
            }
        }
    }
}

// wide-out pullback, input cotangent, in two passes:
//   dot:  workgroup (i·R + r, column tile), R = G + use_base: S[i, r, k] = Σ_o row[o] ȳ[o, k]
//         with row = C[:, r + G i] (r < G) or W[:, i] (r = G); threads stride over o
//         (coalesced), then an ordered block reduction per column;
//   fin:  thread (i, k): x̄[i, k] from S through the basis / normalizer / swish rrules
//         (utils.jl:15-21, NNlib).
constexpr int kWOX = 256;
static_assert(kWOX == kWOB * kSW, "the dot and parameter bodies share one launch");
// ls (nullable): ȳ is the adjoint stage input λs = ls->lam + Σ ls->sl.c·ls->sl.k, formed here in
// wide_stage_comb's order (bitwise the values the wide-in stage forward writes to ls_out)
template <typename T>
__device__ __forceinline__ void wideout_dot_body(const LayerConst* __restrict__ lcp, const T* __restrict__ p,
                                                 const T* __restrict__ ybar, T* __restrict__ S, int64_t K, int bx,
                                                 int by, int gy, const WideStageIn<T>* ls = nullptr) {
    __shared__ T red[kWOX / kWave][kKT];
    const LayerConst& lc = *lcp;
    const int O = lc.O, G = lc.G;
    const int R = G + (lc.use_base ? 1 : 0);
    const int i = bx / R, r = bx - i * R;
    const T* __restrict__ row = r < G ? p + lc.p_off + (int64_t)O * (r + (int64_t)G * i) : p + lc.w_off + (int64_t)O * i;
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    for (int64_t k0 = (int64_t)by * kKT; k0 < K; k0 += (int64_t)gy * kKT) {
        const int kt = (int)((K - k0) < kKT ? (K - k0) : kKT);
        T acc[kKT];
#pragma unroll
        for (int kk = 0; kk < kKT; ++kk) acc[kk] = T(0);
        if (ls) {
            // λs[o, k] formed here: every column's stage loads issued before the first combination
            for (int o = threadIdx.x; o < O; o += kWOX) {
                const T cv = row[o];
                T yv[kKT];
#pragma unroll
                for (int kk = 0; kk < kKT; ++kk)
                    yv[kk] = kk < kt ? wide_stage_comb<T>(ls->lam, ls->sl, (int64_t)O * (k0 + kk) + o) : T(0);
#pragma unroll
                for (int kk = 0; kk < kKT; ++kk)
                    if (kk < kt) acc[kk] = kfma<T>(cv, yv[kk], acc[kk]);
            }
        } else {
#pragma unroll 4
            for (int o = threadIdx.x; o < O; o += kWOX) {
                const T cv = row[o];
#pragma unroll
                for (int kk = 0; kk < kKT; ++kk)
                    if (kk < kt) acc[kk] = kfma<T>(cv, ybar[(int64_t)O * (k0 + kk) + o], acc[kk]);
            }
        }
#pragma unroll
        for (int kk = 0; kk < kKT; ++kk) {
            const T s = wave_sum(acc[kk]);
            if (lane == 0) red[wid][kk] = s;
        }
        __syncthreads();
        if (threadIdx.x < kt) {
            T s = red[0][threadIdx.x];
#pragma unroll
            for (int w = 1; w < kWOX / kWave; ++w) s += red[w][threadIdx.x];
            S[((int64_t)bx * K) + k0 + threadIdx.x] = s;
        }
        __syncthreads();
    }
}

// One launch for both independent parts of the wide-out pullback's first pass: blocks
// [0, nd) are the dot products (nd = I·R·tiles, laid out (i·R + r) + I·R·tile), the rest the
// parameter cotangents ((row chunk, input i) = (b % nrc, b / nrc)).
template <typename T, int PATH>
__global__ void __launch_bounds__(kWOX)
kd_vjp_wideout_dotparam_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                               const T* __restrict__ xslab, int nblk, const T* __restrict__ ybar, T* __restrict__ S,
                               T* __restrict__ pbar, int64_t K, int nd, int tiles, int nrc, int assign) {
    const Math<T> M{kExp2Tab256};   // exp table from global memory (L1): no staging round trip
    const int b = blockIdx.x;
    if (b < nd) {
        const int ir = lcp->I * (lcp->G + (lcp->use_base ? 1 : 0));
        wideout_dot_body<T>(lcp, p, ybar, S, K, b % ir, b / ir, tiles);
    } else {
        __shared__ T Ph[(kMaxGrid + 1) * kWOPK];
        const int q = b - nd;
        wideout_param_body<T, PATH>(M, lcp, x, xslab, nblk, ybar, pbar, K, q % nrc, q / nrc, assign, Ph, kWOPK);
    }
}

// x̄[i, k] of the wide-out layer from its dot products S (one element)
// S: nS partial slabs of I·R·K sums each (the pair's chunk partials, summed in order; nS = 1: the
// dot launch's complete sums)
template <typename T>
__device__ __forceinline__ T dot_sum(const T* __restrict__ Si, int nS, int64_t sstride) {
    if (nS == 1) return Si[0];
    constexpr int kR = 16;
    T s = T(0);
    for (int b0 = 0; b0 < nS; b0 += kR) {
        T v[kR];
#pragma unroll
        for (int j = 0; j < kR; ++j) v[j] = b0 + j < nS ? Si[(int64_t)(b0 + j) * sstride] : T(0);
#pragma unroll
        for (int j = 0; j < kR; ++j)
            if (b0 + j < nS) s += v[j];
    }
    return s;
}
template <typename T, int PATH>
__device__ __forceinline__ T wideout_xfin_one(const Math<T>& M, const LayerConst& lc, const T* __restrict__ x,
                                              const T* __restrict__ xslab, int nblk, const T* __restrict__ S,
                                              int64_t K, int i, int64_t k, int nS = 1) {
    const int I = lc.I, G = lc.G;
    const int R = G + (lc.use_base ? 1 : 0);
    const int64_t sstride = (int64_t)I * R * K;
    const T invh = T(lc.invh);
    const T* __restrict__ Si = S + (int64_t)i * R * K + k;
    const T xi = layer_in<T>(x, xslab, nblk, I, K, i, k);
    Basis1<T, PATH> bs;
    bs.init(M, lc, xi);
    T nbar = T(0);
    for (int g = 0; g < G; ++g) {
        T z, aux;
        const T phi = bs.next(M, lc, g, z, aux);
        nbar = nbar + basis_pull<T>(lc.basis, lc.iqf_quirk, z, phi, aux, dot_sum<T>(Si + (int64_t)g * K, nS, sstride)) *
                          invh;
    }
    T xb = nbar * dnormalize<NORM_RUNTIME, T>(lc.norm, bs.n);
    if (lc.use_base) {
        T sw, dsw;
        swish_and_grad<T>(M, xi, sw, dsw);
        xb = xb + dot_sum<T>(Si + (int64_t)G * K, nS, sstride) * dsw;
    }
    return xb;
}

template <typename T, int PATH>
__global__ void __launch_bounds__(kBlock)
kd_vjp_wideout_xfin_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ x, const T* __restrict__ xslab,
                           int nblk, const T* __restrict__ S, T* __restrict__ xbar, int64_t K) {
    KAN_EXP_TABLE_LDS(tab);   // G + 2 dependent exponentials per thread: the LDS copy pays here
    const Math<T> M{tab};
    const LayerConst& lc = *lcp;
    const int I = lc.I;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < (int64_t)I * K;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = idx / I;
        const int i = (int)(idx - k * I);
        xbar[idx] = wideout_xfin_one<T, PATH>(M, lc, x, xslab, nblk, S, K, i, k);
    }
}

// ---------------------------------------------------------------------------
// wide-in pullback, grid (chunks of cw inputs as the forward, np + nxg), 256 threads:
//   blockIdx.y <  np (np = O with pbar): output o = y's parameter cotangents of the chunk over all
//          columns, dC[o, c] += Σ_k ȳ[o, k] φ_c(x_k), dW[o, i] += Σ_k ȳ[o, k] swish(x_ik), one
//          thread per basis slot (direct formula), columns summed in order, pbar written once;
//   blockIdx.y >= np: x̄ of the columns k ≡ y - np (mod nxg): the chunk's basis values in LDS,
//          one thread per basis slot c = g + G i forms Σ_o C[o, c] ȳ[o, k] and its rrule term,
//          then one thread per input sums them over g (the order of the reference pullback).
// The body of the wide-in pullback for block (bx, by) of the grid above.  yb_at(o, k) gives
// ȳ[o, k]; prep_param(o) runs once, block-uniformly, before a parameter block's column loop (the
// pair pullback forms that output's ȳ row there); yb_col(ybL, t, k) fills ybL[0, O) for an x̄
// block's column k (thread t < O writes entry t).
template <typename T, typename YB, typename PREP, typename YCOL, typename XOUT>
__device__ __forceinline__ void widein_vjp_body(const LayerConst* __restrict__ lcp, const T* __restrict__ p,
                                                const T* __restrict__ x, YB yb_at, PREP prep_param, YCOL yb_col,
                                                XOUT on_xbar, T* __restrict__ xbar, T* __restrict__ pbar, int64_t K,
                                                int np, int nsub, int nxg, int cw, int assign, int bx, int by, T* L,
                                                const WideBasisG<T>* bg = nullptr) {
    const Math<T> M{kExp2Tab256};   // exp table from global memory (L1): no staging round trip
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;

    const int i0 = bx * cw;
    const int ni = I - i0 < cw ? I - i0 : cw;
    const int t = threadIdx.x;
    const bool base = lc.use_base != 0;
    const T invh = T(lc.invh);
    if (by < np * nsub) {
        // output o = by / nsub: dC[o, c] += Σ_k ȳ[o, k] φ_c(x_k) for the basis slots c of
        // sub-chunk by % nsub (spb consecutive slots of the chunk), basis by the direct
        // formula; dW[o, i] += Σ_k ȳ[o, k] swish(x_ik).  With spb <= 128 the block's threads are
        // nq = 256 / spb column lanes per slot (columns k ≡ q mod nq), summed over the lanes in order
        // through LDS; otherwise one lane, slots t, t + 256, ...  (nsub > 1 keeps spb <= 128 for a
        // wide chunk, so a thread evaluates ~K/nq bases instead of K·ncp/256.)
        const int o = by / nsub, sub = by - o * nsub;
        prep_param(o);
        const int ncp = cw * G, spb = (ncp + nsub - 1) / nsub;
        const int c0 = sub * spb, nc = ni * G;
        const int c1 = c0 + spb < nc ? c0 + spb : nc;
        const int nq = spb <= 128 ? 256 / spb : 1;
        constexpr int kS = (kWideInMaxInputs * kMaxGrid + 255) / 256;
        const int q = nq > 1 ? t / spb : 0;
        const int cb = nq > 1 ? t - q * spb : t;
        T dcv[kS], dwv[kS];
#pragma unroll
        for (int m = 0; m < kS; ++m) dcv[m] = dwv[m] = T(0);
        if (q < nq && bg) {
            // the basis values the pair's forward blocks stored (WideBasisG): per slot, eight columns'
            // loads in flight, accumulated in ascending k (the per-slot order of the loop below)
            const int64_t ps = (int64_t)I * G;
#pragma unroll
            for (int m = 0; m < kS; ++m) {
                const int c = c0 + cb + 256 * m;
                if ((nq == 1 || m == 0) && c < c1) {
                    const int i = c / G, g = c - i * G;
                    const bool wsl = base && g == 0;
                    const T* __restrict__ ph = bg->phi + (int64_t)i0 * G + c;
                    const T* __restrict__ sw = bg->sw + i0 + i;
                    for (int64_t k0 = q; k0 < K; k0 += 8 * nq) {
                        T pv[8], sv[8];
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const int64_t k = k0 + j * nq;
                            pv[j] = k < K ? ph[k * ps] : T(0);
                            sv[j] = k < K && wsl ? sw[k * I] : T(0);
                        }
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const int64_t k = k0 + j * nq;
                            if (k < K) {
                                const T yb = yb_at(o, k);
                                dcv[m] = kfma<T>(yb, pv[j], dcv[m]);
                                if (wsl) dwv[m] = kfma<T>(yb, sv[j], dwv[m]);
                            }
                        }
                    }
                }
            }
        } else if (q < nq) {
            for (int64_t k = q; k < K; k += nq) {
                const T yb = yb_at(o, k);
#pragma unroll
                for (int m = 0; m < kS; ++m) {
                    const int c = c0 + cb + 256 * m;
                    if ((nq == 1 || m == 0) && c < c1) {
                        const int i = c / G, g = c - i * G;
                        const T xi = x[(int64_t)I * k + i0 + i];
                        const T n = normalize<NORM_RUNTIME, T>(M, lc.norm, xi);
                        T aux = T(0);
                        dcv[m] = kfma<T>(yb, basis_direct<T>(M, lc.basis, (n - T(lc.grid[g])) * invh, aux), dcv[m]);
                        if (base && g == 0) dwv[m] = kfma<T>(yb, swish<T>(M, xi), dwv[m]);
                    }
                }
            }
        }
        T* __restrict__ dC = pbar + lc.p_off + (int64_t)O * G * i0 + o;
        if (nq == 1) {
#pragma unroll
            for (int m = 0; m < kS; ++m) {
                const int c = c0 + t + 256 * m;
                if (c < c1) {
                    T* d = dC + (int64_t)O * c;
                    *d = assign ? dcv[m] : *d + dcv[m];
                    if (base && c % G == 0) {
                        T* dw = pbar + lc.w_off + (int64_t)O * (i0 + c / G) + o;
                        *dw = assign ? dwv[m] : *dw + dwv[m];
                    }
                }
            }
        } else {
            T* red = L;                 // [nq][spb] slot partials
            T* redw = L + nq * spb;     // [nq][spb] swish partials (g = 0 slots)
            if (q < nq) {
                red[t] = dcv[0];
                if (c0 + cb < c1 && (c0 + cb) % G == 0) redw[t] = dwv[0];
            }
            __syncthreads();
            const int c = c0 + t;
            if (t < spb && c < c1) {
                T sum = red[t];
                for (int r = 1; r < nq; ++r) sum += red[r * spb + t];
                T* d = dC + (int64_t)O * c;
                *d = assign ? sum : *d + sum;
                if (base && c % G == 0) {
                    T sw = redw[t];
                    for (int r = 1; r < nq; ++r) sw += redw[r * spb + t];
                    T* dw = pbar + lc.w_off + (int64_t)O * (i0 + c / G) + o;
                    *dw = assign ? sw : *dw + sw;
                }
            }
        }
        return;
    }
    const int nc = ni * G;
    T* phL = L;                  // [cw·G] basis values, arguments, aux, rrule terms
    T* zL = phL + cw * G;
    T* auL = zL + cw * G;
    T* puL = auL + cw * G;
    T* ybL = puL + cw * G;       // [O]
    T* dnL = ybL + kOWide;       // [cw] N'(x_i)
    T* dsL = dnL + cw;           // [cw] swish'(x_i)
    const T* __restrict__ C = p + lc.p_off + (int64_t)O * G * i0;
    const T* __restrict__ W = p + lc.w_off + (int64_t)O * i0;
    for (int64_t k = (int64_t)by - np * nsub; k < K; k += nxg) {
        __syncthreads();
        const bool stored = bg && lc.basis == BASIS_RBF;   // the rbf rrule needs φ and z only
        for (int c = t; c < nc; c += blockDim.x) {
            const int i = c / G, g = c - i * G;
            const T pst = stored ? bg->phi[((int64_t)I * k + i0) * G + c] : T(0);
            const T dst = stored && base && g == 0 ? bg->dsw[(int64_t)I * k + i0 + i] : T(0);
            const T xi = x[(int64_t)I * k + i0 + i];
            const T n = normalize<NORM_RUNTIME, T>(M, lc.norm, xi);
            const T z = (n - T(lc.grid[g])) * invh;
            T aux = T(0);
            phL[c] = stored ? pst : basis_direct<T>(M, lc.basis, z, aux);
            zL[c] = z;
            auL[c] = aux;
            if (g == 0) {
                dnL[i] = dnormalize<NORM_RUNTIME, T>(lc.norm, n);
                if (base) {
                    if (stored) {
                        dsL[i] = dst;
                    } else {
                        T sw, dsw;
                        swish_and_grad<T>(M, xi, sw, dsw);
                        dsL[i] = dsw;
                    }
                }
            }
        }
        yb_col(ybL, t, k);
        __syncthreads();
        for (int c = t; c < nc; c += blockDim.x) {
            const T* __restrict__ Cc = C + (int64_t)O * c;
            T bb = T(0);
            for (int o = 0; o < O; ++o) bb = kfma<T>(Cc[o], ybL[o], bb);
            puL[c] = basis_pull<T>(lc.basis, lc.iqf_quirk, zL[c], phL[c], auL[c], bb) * invh;
        }
        __syncthreads();
        if (t < ni) {
            T nbar = T(0);
            for (int g = 0; g < G; ++g) nbar = nbar + puL[t * G + g];
            T xb = nbar * dnL[t];
            if (base) {
                T sb = T(0);
                for (int o = 0; o < O; ++o) sb = kfma<T>(W[(int64_t)O * t + o], ybL[o], sb);
                xb = xb + sb * dsL[t];
            }
            xbar[(int64_t)I * k + i0 + t] = xb;
            on_xbar((int64_t)I * k + i0 + t, xb);
        }
    }
}

template <typename T>
__global__ void __launch_bounds__(256)
kd_vjp_widein_co_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                        const T* __restrict__ ybar, T* __restrict__ xbar, T* __restrict__ pbar, int64_t K, int np,
                        int nsub, int nxg, int cw, int assign) {
    extern __shared__ __attribute__((aligned(16))) unsigned char wv_raw[];
    const int O = lcp->O;
    widein_vjp_body<T>(
        lcp, p, x, [&](int o, int64_t k) { return ybar[(int64_t)O * k + o]; }, [](int) {},
        [&](T* ybL, int t, int64_t k) {
            if (t < O) ybL[t] = ybar[(int64_t)O * k + t];
        },
        [](int64_t, T) {}, xbar, pbar, K, np, nsub, nxg, cw, assign, blockIdx.x, blockIdx.y,
        reinterpret_cast<T*>(wv_raw));
}

// ---------------------------------------------------------------------------
// The surrogate pair's pullback in two launches (kanode_vjp / kanode_vjp_stage of a KAN [N, H, N],
// Burgers_Surrogate.jl:85-97, Schrodinger_Surrogate.jl:93-104), instead of four:
//   A: the wide-in forward's chunk partials of the hidden layer h (with a stage: y and λs formed and
//      written, WideStageIn), and, in the same blocks, the chunk partials of the wide-out dot products
//      S[i, r, k] = Σ_o row_{i,r}[o] ȳ[o, k] over the block's o-range (PairDot: ȳ = λs as the block
//      formed it; the dot products need ȳ and the parameters only, not h);
//   B: blocks [0, nP) the wide-out parameter cotangents (h summed from its partials, ȳ); the rest the
//      wide-in pullback, whose cotangent (x̄ of the hidden layer) each block forms itself from the S
//      and h partials (wideout_xfin_one: a parameter block its output's K entries, an x̄ block its
//      column's H), which removes the x̄ pass and its launch.
// The results equal the four-launch path's up to the summation order of S (chunk partials summed in
// chunk order instead of one wave-ordered block sum): fixed, so bitwise reproducible.
template <typename T, int MV, int MW, bool STAGE>
__global__ void __launch_bounds__(256)
kd_vjp_pair_a_kernel(const LayerConst* __restrict__ lc0, const LayerConst* __restrict__ lc1, const T* __restrict__ p,
                     const T* __restrict__ x, T* __restrict__ pslab, const T* __restrict__ ybar, T* __restrict__ spart,
                     int64_t K, int nblk, int gyF, WideStageIn<T> si, WideBasisG<T> bg) {
    const PairDot<T> pd{lc1, spart, ybar, bg};
    widein_fwd_body<T, STAGE, MV, MW, true>(lc0, p, x, pslab, K, STAGE ? &si : nullptr, blockIdx.x % nblk,
                                            blockIdx.x / nblk, gyF, &pd);
}

// Wide-out parameter cotangents in the pair pullback: one wave per unit (row chunk bx, hidden input i),
// four units per block.  Lanes k < K stage the basis of input i for every column in the wave's LDS block
// Ph [(G + 1)][K] (the hidden value summed from the wide-in chunk partials), then lane o accumulates
// dC[o, g + G i] = Σ_k ȳ[o, k] φ_g(h_ik) and dW[o, i] = Σ_k ȳ[o, k] swish(h_ik) over the columns in
// ascending k (eight ȳ loads in flight) and writes them: no cross-wave partial sums, one barrier.
// (The four-launch path's wideout_param_body splits the columns over the block's four waves and sums
// their partials through LDS: eleven rounds of two barriers for G = 10.)
template <typename T, int PATH>
__device__ __forceinline__ void wideout_param_wave(const Math<T>& M, const LayerConst& lc, const T* __restrict__ xslab,
                                                   int nblk, const T* __restrict__ ybar, T* __restrict__ pbar,
                                                   int64_t K, int unit, int nunits, int nrc, int assign,
                                                   T* __restrict__ Ph) {
    const int I = lc.I, O = lc.O, G = lc.G;
    const int lane = threadIdx.x & (kWave - 1);
    const bool live = unit < nunits;
    const int bx = live ? unit % nrc : 0, i = live ? unit / nrc : 0;
    const bool base = lc.use_base != 0;
    if (live) {
        for (int64_t kk = lane; kk < K; kk += kWave) {
            const T xi = layer_in<T>(nullptr, xslab, nblk, I, K, i, kk);
            Basis1<T, PATH> bs;
            bs.init(M, lc, xi);
            for (int g = 0; g < G; ++g) {
                T z, aux;
                Ph[g * K + kk] = bs.next(M, lc, g, z, aux);
            }
            Ph[(int64_t)G * K + kk] = base ? swish<T>(M, xi) : T(0);
        }
    }
    __syncthreads();   // (every wave of the block is a parameter wave: uniform)
    const int o = bx * kWOB + lane;
    if (!live || o >= O) return;
    T acc[kMaxGrid + 1];
#pragma unroll
    for (int r = 0; r <= kMaxGrid; ++r) acc[r] = T(0);
    for (int64_t k0 = 0; k0 < K; k0 += 8) {
        T yv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) yv[j] = k0 + j < K ? ybar[(int64_t)O * (k0 + j) + o] : T(0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (k0 + j < K) {
                const int64_t k = k0 + j;
#pragma unroll
                for (int r = 0; r < kMaxGrid; ++r)
                    if (r < G) acc[r] = kfma<T>(yv[j], Ph[r * K + k], acc[r]);
                acc[kMaxGrid] = kfma<T>(yv[j], Ph[(int64_t)G * K + k], acc[kMaxGrid]);
            }
        }
    }
    T* __restrict__ dC = pbar + lc.p_off + o + (int64_t)O * G * i;
#pragma unroll
    for (int r = 0; r < kMaxGrid; ++r) {
        if (r < G) {
            T* d = dC + (int64_t)O * r;
            *d = assign ? acc[r] : *d + acc[r];
        }
    }
    if (base) {
        T* d = pbar + lc.w_off + o + (int64_t)O * i;
        *d = assign ? acc[kMaxGrid] : *d + acc[kMaxGrid];
    }
}

// x̄ of one wide-out input from its value xi and its dot products Sl[g·ss] (g < G; the swish row at G)
template <typename T, int PATH>
__device__ __forceinline__ T wideout_xfin_lds(const Math<T>& M, const LayerConst& lc, T xi, const T* Sl, int ss) {
    const int G = lc.G;
    const T invh = T(lc.invh);
    Basis1<T, PATH> bs;
    bs.init(M, lc, xi);
    T nbar = T(0);
    for (int g = 0; g < G; ++g) {
        T z, aux;
        const T phi = bs.next(M, lc, g, z, aux);
        nbar = nbar + basis_pull<T>(lc.basis, lc.iqf_quirk, z, phi, aux, Sl[g * ss]) * invh;
    }
    T xb = nbar * dnormalize<NORM_RUNTIME, T>(lc.norm, bs.n);
    if (lc.use_base) {
        T sw, dsw;
        swish_and_grad<T>(M, xi, sw, dsw);
        xb = xb + Sl[G * ss] * dsw;
    }
    return xb;
}

// dst[v] = Σ_{b < nS} src(v, b) for v < nt, by the whole block (every thread calls): thread t sums the
// terms b ≡ s (mod ns) of value t / ns in ascending b, then the ns sub-sums are added in order (fixed
// order: bitwise reproducible).  red: LDS of 256 entries.
template <typename T, typename F>
__device__ __forceinline__ void block_gather_sums(F src, int nt, int nS, T* red, T* dst) {
    const int t = threadIdx.x;
    for (int v0 = 0; v0 < nt; v0 += 256) {
        const int nv = nt - v0 < 256 ? nt - v0 : 256;
        const int ns = 256 / nv;
        const int v = t / ns, s = t - v * ns;
        T a = T(0);
        if (v < nv) {
#pragma unroll 4
            for (int b = s; b < nS; b += ns) a += src(v0 + v, b);
        }
        red[t] = a;
        __syncthreads();
        if (t < nv) {
            T sum = red[t * ns];
            for (int j = 1; j < ns; ++j) sum += red[t * ns + j];
            dst[v0 + t] = sum;
        }
        __syncthreads();
    }
}

// The second launch's body (every block type); true for an x̄ block, whose chunk and column are returned.
// xbst (nullable, LDS): an x̄ block also leaves its x̄ entries there (the fused step's next stage reads them).
template <typename T, int PATH>
__device__ __forceinline__ bool pair_b_body(const LayerConst* __restrict__ lc0, const LayerConst* __restrict__ lc1,
                                            const T* __restrict__ p, const PairBArgs<T>& a, T* xbst, int& chunk,
                                            int& col) {
    // err_slab (adjoint stage with the λ error, si given): each x̄ block adds, for its entries,
    // (e / sk)², e = Σ_j ec_j lk_j + ec_n·λsᵀJ, sk = abstol + reltol·max(|λ|, |λs|) (stage_error_kernel's
    // statement), into err_slab[its index]; the stage's final reduction sums the nbx·nxg rows
    // S: the nblk chunk partials of the wide-out dot products (kd_vjp_pair_a_kernel), [b][I1·R1][K]
    extern __shared__ __attribute__((aligned(16))) unsigned char pb_raw[];
    T* L = reinterpret_cast<T*>(pb_raw);
    const Math<T> M{kExp2Tab256};   // exp table from global memory (L1)
    const int b = blockIdx.x;
    const int64_t K = a.K;
    const int nbx = a.nbx, np = a.np, nblk = a.nblk;
    const T* __restrict__ pslab = a.pslab;
    const T* __restrict__ S = a.S;
    if (b < a.nP) {   // four wide-out parameter units per block, one per wave
        const int w = threadIdx.x / kWave;
        const int64_t ph = (int64_t)(lc1->G + 1) * K;
        wideout_param_wave<T, PATH>(M, *lc1, pslab, nblk, a.ybar, a.pbar, K, 4 * b + w, a.nrc * lc1->I, a.nrc,
                                    a.assign, L + w * ph);
        return false;
    }
    const int q = b - a.nP;
    const LayerConst& l1 = *lc1;
    const int H = l1.I, R = l1.G + (l1.use_base ? 1 : 0);
    const int64_t bs = (int64_t)H * R * K;     // stride of one chunk's partials
    T* hbL = L + a.hb_off;                     // [K]: a parameter block's cotangent row
    T* red = hbL + K;                          // [256]
    T* Sv = red + 256;                         // [max(R·K, H·R)] the block's dot products
    T* hv = Sv + (R * K > H * R ? R * K : H * R);   // [max(K, H)] the hidden values it needs
    double eacc = 0.0;
    const WideStageIn<T>& si = a.si;
    double* __restrict__ err_slab = a.err_slab;
    const int i0 = (q % nbx) * a.cw;
    widein_vjp_body<T>(
        lc0, p, a.x, [&](int, int64_t k) { return hbL[k]; },
        [&](int o) {   // hidden unit o over all columns: S[o, r, k] for r < R, k < K, and h[o, k]
            block_gather_sums<T>([&](int v, int c) { return S[c * bs + (int64_t)o * R * K + v]; }, R * (int)K, nblk,
                                 red, Sv);
            for (int64_t k = threadIdx.x; k < K; k += blockDim.x)
                hv[k] = layer_in<T>(nullptr, pslab, nblk, H, K, o, k);
            __syncthreads();
            for (int64_t k = threadIdx.x; k < K; k += blockDim.x)
                hbL[k] = wideout_xfin_lds<T, PATH>(M, l1, hv[k], Sv + k, (int)K);
            __syncthreads();
        },
        [&](T* ybL, int t, int64_t k) {   // column k over all hidden units: S[i, r, k] and h[i, k]
            block_gather_sums<T>(
                [&](int v, int c) { return S[c * bs + (int64_t)v * K + k]; }, H * R, nblk, red, Sv);
            if (t < H) hv[t] = layer_in<T>(nullptr, pslab, nblk, H, K, t, k);
            __syncthreads();
            if (t < H) ybL[t] = wideout_xfin_lds<T, PATH>(M, l1, hv[t], Sv + t * R, 1);
        },
        [&](int64_t idx, T xb) {
            if (xbst) xbst[idx % l1.O - i0] = xb;   // (l1.O = the state size: idx = N·k + i0 + t)
            if (!err_slab) return;
            const StageArgs<T>& sl = si.sl;
            const double sc = stage_scale(sl.cscale);
            T kv[kMaxStages];
            stage_ld<T>(sl, si.lam, idx, kv);
            double e = 0.0;
#pragma unroll
            for (int j = 0; j < kMaxStages; ++j)
                if (j < sl.nk) e = ::fma(sl.ec[j] * sc, (double)kv[j], e);
            e = ::fma(stage_ec_last(sl) * sc, (double)xb, e);
            const double sk = ::fma(sl.reltol, fmax(kabs((double)si.lam[idx]), kabs((double)si.ls_out[idx])), sl.abstol);
            const double r = e / sk;
            eacc = ::fma(r, r, eacc);
        },
        a.xbar, a.pbar, K, np, 1, a.nxg, a.cw, a.assign, q % nbx, q / nbx, L, a.bg.phi ? &a.bg : nullptr);
    if (q / nbx < np) return false;
    if (err_slab) {   // an x̄ block: its error partial
        __shared__ double ered[256 / kWave];
        const double v[1] = {eacc};
        block_sum_to<double, 1>(v, 1, ered, err_slab + (q / nbx - np) * nbx + q % nbx);
    }
    chunk = q % nbx;
    col = q / nbx - np;
    return true;
}

template <typename T, int PATH>
__global__ void __launch_bounds__(256)
kd_vjp_pair_b_kernel(const LayerConst* __restrict__ lc0, const LayerConst* __restrict__ lc1, const T* __restrict__ p,
                     PairBArgs<T> a) {
    int chunk, col;
    (void)pair_b_body<T, PATH>(lc0, lc1, p, a, nullptr, chunk, col);
}

// The fused pair step (the solver's deferred adjoint stages, kanode_abi.cpp): stage s's second launch
// and stage s+1's first in one.  Stage s+1's first-launch block for (chunk, column) needs, beyond data
// earlier launches wrote, only the λᵀJ of stage s over that chunk and column (the last term of its λs
// combination) -- exactly what stage s's x̄ block for (chunk, column) forms.  So every x̄ block, after its
// pullback, runs the next stage's wide-in forward body for its own chunk and column, taking that term
// from LDS; the parameter blocks run beside them as in kd_vjp_pair_b_kernel.  The next stage's outputs
// (hidden and dot-product partials, basis store, y, λs) go to the other buffer of a ping-pong pair, since
// this launch's parameter blocks still read stage s's.  Same statements in the same order as the two
// launches: bitwise equal results.
template <typename T, int PATH, int MV, int MW>
__global__ void __launch_bounds__(256)
kd_vjp_pair_ba_kernel(const LayerConst* __restrict__ lc0, const LayerConst* __restrict__ lc1, const T* __restrict__ p,
                      PairBArgs<T> a, PairAArgs<T> n) {
    __shared__ T xbst[kWideInMaxInputs];
    int chunk, col;
    if (!pair_b_body<T, PATH>(lc0, lc1, p, a, xbst, chunk, col)) return;
    __syncthreads();   // this block's x̄ entries are in xbst
    const PairDot<T> pd{lc1, n.spart, n.si.ls_out, n.bg};
    widein_fwd_body<T, true, MV, MW, true>(lc0, p, n.x, n.pslab, a.K, &n.si, chunk, col, (int)a.K, &pd, xbst);
}

// ---------------------------------------------------------------------------
// launchers
static inline size_t wideout_lds(const LayerConst& h, size_t es) { return es * (size_t)(h.G * h.I + h.I) * kKT; }
static inline unsigned col_tiles(int64_t K) {
    const int64_t t = (K + kKT - 1) / kKT;
    return (unsigned)(t < 65535 ? t : 65535);
}

template <typename T>
hipError_t launch_kd_fwd_widein(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, T* y, T* slab,
                                int64_t K, hipStream_t st, const WideStageIn<T>* si) {
    const int nblk = widein_chunks(h);
    const dim3 grid(nblk, (unsigned)(K < 65535 ? K : 65535));
    const int cw = widein_cw(h.O, h.G, h.I), tn = (256 / h.O) * h.O;
    const int nv = (h.O * h.G * cw + tn - 1) / tn, nw = (h.O * cw + tn - 1) / tn;   // load slots needed
#define KAN_WIN(MV, MW)                                                                                          \
    do {                                                                                                         \
        if (si) hipLaunchKernelGGL((kd_fwd_widein_stage_kernel<T, MV, MW>), grid, dim3(256), 0, st, lc, p, x, slab, K, *si); \
        else hipLaunchKernelGGL((kd_fwd_widein_co_kernel<T, MV, MW>), grid, dim3(256), 0, st, lc, p, x, slab, K); \
    } while (0)
    if (nv <= 8 && nw <= 2) KAN_WIN(8, 2);
    else if (nv <= 16 && nw <= 4) KAN_WIN(16, 4);
    else KAN_WIN(kWIMaxV, kWIMaxW);
#undef KAN_WIN
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !y) return e;   // y == nullptr: the consumer sums the slab itself
    const int64_t n = (int64_t)h.O * K;
    hipLaunchKernelGGL((kd_widein_reduce_kernel<T>), dim3(grid_for(n, kBlock, 1 << 30)), dim3(kBlock), 0, st, slab,
                       nblk, h.O, K, y);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_kd_fwd_wideout(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, T* y, int64_t K,
                                 hipStream_t st, const T* xslab, int xnblk) {
    const dim3 grid((h.O + kWOB - 1) / kWOB, col_tiles(K));
    const size_t lds = wideout_lds(h, sizeof(T));
#define KAN_WO(PATH)                                                                                               \
    hipLaunchKernelGGL((kd_fwd_wideout_kernel<T, PATH>), grid, dim3(kWOB * kSW), lds, st, lc, p, x, xslab, xnblk, y, K)
    switch (h.path) {
    case PATH_REC_CORR: KAN_WO(PATH_REC_CORR); break;
    case PATH_REC: KAN_WO(PATH_REC); break;
    default: KAN_WO(PATH_DIRECT);
    }
#undef KAN_WO
    return hipGetLastError();
}

template <typename T>
hipError_t launch_kd_vjp_wideout(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, const T* yb,
                                 T* xb, T* pbar, T* slab, int64_t K, hipStream_t st, const T* xslab, int xnblk,
                                 bool assign) {
    const int R = h.G + (h.use_base ? 1 : 0);
    const int tiles = (int)col_tiles(K), nrc = (h.O + kWOB - 1) / kWOB;
    const int nd = xb ? h.I * R * tiles : 0, np = pbar ? nrc * h.I : 0;
    const unsigned gf = grid_for((int64_t)h.I * K, kBlock, kGridCap);
#define KAN_WOV(PATH)                                                                                              \
    do {                                                                                                           \
        if (nd + np > 0)                                                                                           \
            hipLaunchKernelGGL((kd_vjp_wideout_dotparam_kernel<T, PATH>), dim3(nd + np), dim3(kWOX), 0, st, lc, p, x, \
                               xslab, xnblk, yb, slab, pbar, K, nd, tiles, nrc, assign ? 1 : 0);                  \
        if (xb) hipLaunchKernelGGL((kd_vjp_wideout_xfin_kernel<T, PATH>), dim3(gf), dim3(kBlock), 0, st, lc, x, xslab, \
                                   xnblk, slab, xb, K);                                                           \
    } while (0)
    switch (h.path) {
    case PATH_REC_CORR: KAN_WOV(PATH_REC_CORR); break;
    case PATH_REC: KAN_WOV(PATH_REC); break;
    default: KAN_WOV(PATH_DIRECT);
    }
#undef KAN_WOV
    return hipGetLastError();
}

template <typename T>
hipError_t launch_kd_vjp_widein(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, const T* yb, T* xb,
                                T* pbar, int64_t K, hipStream_t st, bool assign) {
    // few columns: the forward's chunks; many: chunks of <= 64 basis slots, so the parameter blocks
    // spread the columns over 256 / (cw·G) >= 4 lanes per slot
#ifndef KAN_VJP_WIDEIN_SMALL_CW
#define KAN_VJP_WIDEIN_SMALL_CW 0
#endif
#ifndef KAN_VJP_WIDEIN_SUBCHUNKS
#define KAN_VJP_WIDEIN_SUBCHUNKS 0   // measured neutral (Schrodinger VJP 44.0-45.1 vs 44.8-46.2 us): off
#endif
    const int cw = (K > 8 || KAN_VJP_WIDEIN_SMALL_CW) ? (64 / h.G > 1 ? 64 / h.G : 1) : widein_cw(h.O, h.G, h.I);
    const int nblk = (h.I + cw - 1) / cw;
    const int np = pbar ? h.O : 0;
    const int nxg = xb ? (int)(K < 4096 ? K : 4096) : 0;
    if (np + nxg == 0) return hipSuccess;
    // parameter blocks: a chunk of more than 128 basis slots is split into sub-chunks of <= 128, so
    // every slot gets >= 2 column lanes (Schrodinger [2048 -> 10], G = 10: 640 slots, 5 sub-chunks)
    const int ncp = cw * h.G;
    const int nsub = np > 0 && ncp > 128 && KAN_VJP_WIDEIN_SUBCHUNKS ? (ncp + 127) / 128 : 1;
    const dim3 grid(nblk, np * nsub + nxg);
    size_t lds = (size_t)4 * cw * h.G + kOWide + 2 * (size_t)cw;   // x̄ blocks
    lds = sizeof(T) * (lds > 512 ? lds : 512);                         // parameter blocks' lane sums
    hipLaunchKernelGGL((kd_vjp_widein_co_kernel<T>), grid, dim3(256), lds, st, lc, p, x, yb, xb, pbar, K, np, nsub,
                       nxg, cw, assign ? 1 : 0);
    return hipGetLastError();
}

template <typename T>
hipError_t plan_kd_vjp_pair(const LayerConst& h0, const LayerConst& h1, const LayerConst* lc, const T* p, const T* x,
                            const WideStageIn<T>* si, const T* ybar, const T* xvjp, T* pslab, T* S, T* xb, T* pbar,
                            int64_t K, bool assign, double* err_slab, int err_rows, double* err_out, T* bas,
                            PairPlan<T>* out) {
    if (K < 1 || K > kPairMaxK || !xb) return hipErrorNotSupported;
    PairPlan<T> pl{};
    pl.lc = lc;
    pl.p = p;
    pl.path = h1.path;
    pl.stage = si != nullptr;
    // the wide-in basis store (WideBasisG): phi [K][I][G], sw [K][I], dsw [K][I]
    WideBasisG<T> bg{};
    if (bas) {
        bg.phi = bas;
        bg.sw = bas + K * h0.I * h0.G;
        bg.dsw = bg.sw + K * h0.I;
    }
    const int nrc = (h1.O + kWOB - 1) / kWOB;
    // B's LDS: the wide-in pullback's dynamic block (+ the K-row) beside the wide-out parameter
    // body's static arrays; beyond 64 KB the four-launch path runs instead
    const int cw = K > 8 ? (64 / h0.G > 1 ? 64 / h0.G : 1) : widein_cw(h0.O, h0.G, h0.I);
    size_t lw = (size_t)4 * cw * h0.G + kOWide + 2 * (size_t)cw;
    lw = lw > 512 ? lw : 512;
    const size_t R1 = (size_t)h1.G + (h1.use_base ? 1 : 0), H = (size_t)h1.I, R1w = (size_t)h1.G + 1;
    const size_t lds_w = lw + (size_t)K + 256 + (R1 * K > H * R1 ? R1 * K : H * R1) + ((size_t)K > H ? (size_t)K : H);
    const size_t lds_p = 4 * R1w * (size_t)K;   // wideout_param_wave: four waves' [(G + 1)][K] blocks
    const size_t lds_b = sizeof(T) * (lds_w > lds_p ? lds_w : lds_p);
    if (lds_b > 65536) return hipErrorNotSupported;
    // A
    const int nblk = widein_chunks(h0);
    const int gyF = (int)(K < 65535 ? K : 65535);
    const int tn = (256 / h0.O) * h0.O, cwf = widein_cw(h0.O, h0.G, h0.I);
    const int nv = (h0.O * h0.G * cwf + tn - 1) / tn, nw = (h0.O * cwf + tn - 1) / tn;
    pl.a.x = x;
    pl.a.pslab = pslab;
    pl.a.spart = S;
    pl.a.si = si ? *si : WideStageIn<T>{};
    pl.a.bg = bg;
    pl.ybar_a = ybar;
    pl.nF = nblk * gyF;
    pl.nblk = nblk;
    pl.mv = nv <= 8 && nw <= 2 ? 0 : (nv <= 16 && nw <= 4 ? 1 : 2);
    // B
    const int nbx = (h0.I + cw - 1) / cw;
    const int np = pbar ? h0.O : 0;
    const int nxg = (int)(K < 4096 ? K : 4096);
    const bool err = si && err_out && err_slab && nbx * nxg <= err_rows;
    if (si && err_out && !err) return hipErrorNotSupported;
    PairBArgs<T>& b = pl.b;
    b.x = xvjp;
    b.pslab = pslab;
    b.nblk = nblk;
    b.ybar = si ? si->ls_out : ybar;   // ȳ of the wide-out parameter blocks: λs as A wrote it
    b.S = S;
    b.xbar = xb;
    b.pbar = pbar;
    b.K = K;
    b.nP = pbar ? (nrc * h1.I + 3) / 4 : 0;   // wide-out parameter blocks, four units each
    b.nrc = nrc;
    b.np = np;
    b.nxg = nxg;
    b.cw = cw;
    b.nbx = nbx;
    b.hb_off = (int)lw;
    b.assign = assign ? 1 : 0;
    b.si = pl.a.si;
    b.err_slab = err ? err_slab : nullptr;
    b.bg = bg;
    pl.gridB = b.nP + nbx * (np + nxg);
    pl.ldsB = lds_b;
    pl.err_out = err ? err_out : nullptr;
    pl.err_rows = nbx * nxg;
    // the next stage's first launch fits this plan's x̄ blocks: one block per (chunk, column) on both
    // sides, and the small load-slot instantiation (the fused kernel's registers stay at the second
    // launch's occupancy)
    pl.fuse_ok = pl.stage && nbx == nblk && cw == cwf && nxg == K && gyF == K && pl.mv == 0;
    *out = pl;
    return hipSuccess;
}

template <typename T>
hipError_t launch_pair_first(const PairPlan<T>& pl, hipStream_t st) {
    const LayerConst* lc = pl.lc;
    const int64_t K = pl.b.K;
    const int gyF = (int)(K < 65535 ? K : 65535);
#define KAN_PA(MV, MW)                                                                                             \
    do {                                                                                                           \
        if (pl.stage) hipLaunchKernelGGL((kd_vjp_pair_a_kernel<T, MV, MW, true>), dim3(pl.nF), dim3(256), 0, st, lc, \
                                         lc + 1, pl.p, pl.a.x, pl.a.pslab, pl.ybar_a, pl.a.spart, K, pl.nblk, gyF,  \
                                         pl.a.si, pl.a.bg);                                                        \
        else hipLaunchKernelGGL((kd_vjp_pair_a_kernel<T, MV, MW, false>), dim3(pl.nF), dim3(256), 0, st, lc,        \
                                lc + 1, pl.p, pl.a.x, pl.a.pslab, pl.ybar_a, pl.a.spart, K, pl.nblk, gyF,           \
                                pl.a.si, pl.a.bg);                                                                 \
    } while (0)
    if (pl.mv == 0) KAN_PA(8, 2);
    else if (pl.mv == 1) KAN_PA(16, 4);
    else KAN_PA(kWIMaxV, kWIMaxW);
#undef KAN_PA
    return hipGetLastError();
}

template <typename T>
hipError_t launch_pair_second(const PairPlan<T>& pl, const PairPlan<T>* next, hipStream_t st, bool* fused) {
    const LayerConst* lc = pl.lc;
    bool fuse = false;
    if (next && pl.fuse_ok && next->fuse_ok && next->lc == pl.lc && next->p == pl.p && next->b.K == pl.b.K &&
        next->mv == 0) {
        const StageArgs<T>& sl = next->a.si.sl;
        fuse = sl.nk >= 1 && sl.k[sl.nk - 1] == pl.b.xbar;
    }
    if (fused) *fused = fuse;
#define KAN_PB(PATH)                                                                                               \
    do {                                                                                                           \
        if (fuse) hipLaunchKernelGGL((kd_vjp_pair_ba_kernel<T, PATH, 8, 2>), dim3(pl.gridB), dim3(256), pl.ldsB, st, \
                                     lc, lc + 1, pl.p, pl.b, next->a);                                             \
        else hipLaunchKernelGGL((kd_vjp_pair_b_kernel<T, PATH>), dim3(pl.gridB), dim3(256), pl.ldsB, st, lc, lc + 1, \
                                pl.p, pl.b);                                                                       \
    } while (0)
    switch (pl.path) {
    case PATH_REC_CORR: KAN_PB(PATH_REC_CORR); break;
    case PATH_REC: KAN_PB(PATH_REC); break;
    default: KAN_PB(PATH_DIRECT);
    }
#undef KAN_PB
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (pl.err_out && (e = launch_stage_error_final(pl.b.err_slab, pl.err_rows, pl.err_out, st)) != hipSuccess) return e;
    if (next && !fuse) return launch_pair_first(*next, st);
    return hipSuccess;
}

template <typename T>
hipError_t launch_kd_vjp_pair(const LayerConst& h0, const LayerConst& h1, const LayerConst* lc, const T* p,
                              const T* x, const WideStageIn<T>* si, const T* ybar, const T* xvjp, T* pslab, T* S,
                              T* xb, T* pbar, int64_t K, hipStream_t st, bool assign, double* err_slab,
                              int err_rows, double* err_out, T* bas) {
    PairPlan<T> pl;
    hipError_t e = plan_kd_vjp_pair<T>(h0, h1, lc, p, x, si, ybar, xvjp, pslab, S, xb, pbar, K, assign, err_slab,
                                       err_rows, err_out, bas, &pl);
    if (e != hipSuccess) return e;
    if ((e = launch_pair_first<T>(pl, st)) != hipSuccess) return e;
    return launch_pair_second<T>(pl, nullptr, st);
}

#define KAN_WIDE_INST(T)                                                                                       \
    template hipError_t launch_kd_fwd_widein<T>(const LayerConst&, const LayerConst*, const T*, const T*, T*, T*, \
                                                int64_t, hipStream_t, const WideStageIn<T>*);                   \
    template hipError_t launch_kd_fwd_wideout<T>(const LayerConst&, const LayerConst*, const T*, const T*, T*,   \
                                                 int64_t, hipStream_t, const T*, int);                          \
    template hipError_t launch_kd_vjp_wideout<T>(const LayerConst&, const LayerConst*, const T*, const T*,       \
                                                 const T*, T*, T*, T*, int64_t, hipStream_t, const T*, int, bool); \
    template hipError_t launch_kd_vjp_widein<T>(const LayerConst&, const LayerConst*, const T*, const T*,        \
                                                const T*, T*, T*, int64_t, hipStream_t, bool);                  \
    template hipError_t launch_kd_vjp_pair<T>(const LayerConst&, const LayerConst&, const LayerConst*, const T*,  \
                                              const T*, const WideStageIn<T>*, const T*, const T*, T*, T*, T*, T*, \
                                              int64_t, hipStream_t, bool, double*, int, double*, T*);              \
    template hipError_t plan_kd_vjp_pair<T>(const LayerConst&, const LayerConst&, const LayerConst*, const T*,    \
                                            const T*, const WideStageIn<T>*, const T*, const T*, T*, T*, T*, T*,   \
                                            int64_t, bool, double*, int, double*, T*, PairPlan<T>*);               \
    template hipError_t launch_pair_first<T>(const PairPlan<T>&, hipStream_t);                                     \
    template hipError_t launch_pair_second<T>(const PairPlan<T>&, const PairPlan<T>*, hipStream_t, bool*);
KAN_WIDE_INST(double)
KAN_WIDE_INST(float)
#undef KAN_WIDE_INST

}  // namespace kan
