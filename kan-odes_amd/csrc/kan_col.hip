// kan_col.hip — generic KDense layer kernels, "column" form (gfx950).
//
// One thread per column k of x [I, K] (a trajectory of a batched NeuralODE RHS,
// e.g. Lotka-Volterra KAN [2,10,2]: LV_driver_KANODE.jl:139-142); O <= OMAX
// output accumulators live in registers; C/W reads are wave-uniform (scalar
// loads).  Reference: KDense forward kdense.jl:109-130, pullback = Zygote over it
// with rrule(_rbf) (utils.jl:15-21), per-edge activations Activation_getter.jl.
// Parameter gradients: per-block LDS-staged tile products into a slab, then the
// ordered slab reduction (bitwise reproducible; no float atomics).
#include "kan_common.hpp"
#include "kan_kernels.hpp"
#include "kan_onewg.hpp"

namespace kan {

template <typename T>
__global__ void __launch_bounds__(kBlock) slab_reduce_kernel(const T* __restrict__ slab, int64_t nblk, int64_t P,
                                                             T* __restrict__ dp) {
    __shared__ T red[kBlock / kWave];
    const int64_t q = blockIdx.x;
    T s = T(0);
    s = strided_rows_sum(slab + q, nblk, P, s);
    s = wave_sum(s);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        T t = red[0];
        for (int w = 1; w < (int)(blockDim.x / kWave); ++w) t += red[w];
        dp[q] += t;
    }
}

template <typename T>
hipError_t launch_slab_reduce(const T* slab, int64_t nblk, int64_t P, T* dp, hipStream_t st) {
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL((slab_reduce_kernel<T>), dim3((unsigned)P), dim3(kBlock), 0, st, slab, nblk, P, dp);
    return hipGetLastError();
}

// Sequential basis generator for one normalised input: direct (per-knot formula)
// or the Gaussian recurrence.
template <typename T, int PATH>
struct BasisStream {
    T n, F, R, z0, tau, invh;
    __device__ __forceinline__ void init(const Math<T>& M, const LayerConst& lc, T nn) {
        n = nn;
        invh = T(lc.invh);
        if constexpr (PATH != PATH_DIRECT) rec_anchor<T>(M, lc, n, z0, F, R, tau);   // tau = τ - τ_c
    }
    // returns φ_g, z_g (the scaled argument), aux (tanh for rswaf)
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

template <typename T, int NORM, int PATH, int OMAX>
__global__ void __launch_bounds__(kBlock)
kd_fwd_col_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                  T* __restrict__ y, int64_t K) {
    KAN_EXP_TABLE_LDS(tab);
    const Math<T> M{tab};
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;
    const T* __restrict__ C = p + lc.p_off;
    const T* __restrict__ W = p + lc.w_off;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < K; k += stride) {
        T acc[OMAX], bas[OMAX];
#pragma unroll
        for (int o = 0; o < OMAX; ++o) { acc[o] = T(0); bas[o] = T(0); }
        for (int i = 0; i < I; ++i) {
            const T xi = x[(int64_t)I * k + i];
            BasisStream<T, PATH> bs;
            bs.init(M, lc, normalize<NORM, T>(M, lc.norm, xi));
            for (int g = 0; g < G; ++g) {
                T z, aux;
                const T phi = bs.next(M, lc, g, z, aux);
                const T* Cc = C + (int64_t)O * (g + (int64_t)G * i);
#pragma unroll
                for (int o = 0; o < OMAX; ++o)
                    if (o < O) acc[o] = kfma<T>(Cc[o], phi, acc[o]);
            }
            if (lc.use_base) {
                const T sw = swish<T>(M, xi);
                const T* Wi = W + (int64_t)O * i;
#pragma unroll
                for (int o = 0; o < OMAX; ++o)
                    if (o < O) bas[o] = kfma<T>(Wi[o], sw, bas[o]);
            }
        }
#pragma unroll
        for (int o = 0; o < OMAX; ++o)
            if (o < O) y[(int64_t)O * k + o] = lc.use_base ? acc[o] + bas[o] : acc[o];
    }
}

// A whole small chain in one launch (every layer I, O <= 16; the NeuralODE dudt of
// LV_driver_KANODE.jl:139-143, KAN [2,10,2]).  A group of 16 lanes owns one column and lane
// j holds activation j, so a layer's inputs are spread over lanes: lane i evaluates the G
// basis values and swish of its input and its partial sums for every output o, the group
// sums them with butterfly shuffles, and lane o keeps output o as the next layer's input.
// 16x the waves of a thread-per-column kernel, each with 1/I of the serial work: at 4096
// columns the per-column latency chain, not launch count, bounds it.  The parameter vector
// and the layers' constants are staged in LDS once per block (wave-uniform LDS reads).
// Layer dimensions of a small chain: read from the layer constants (ChainShapeAny) or fixed at
// compile time for the Lotka-Volterra KAN [2,10,2], G = 5 (LV_driver_KANODE.jl:139-142), where
// the loops over outputs and knots then unroll to exactly the live iterations (the generic code
// runs all 16 output slots per layer: ~3x the instructions on a latency-bound single wave).
#ifndef KAN_CHAIN_OUTMAJOR
#define KAN_CHAIN_OUTMAJOR 1
#endif
struct ChainShapeAny {
    static constexpr int NL = 0;
    static constexpr int dim(int) { return 0; }
    static constexpr int GG = 0;
};
template <int D0, int D1, int D2, int G_>
struct ChainShape2 {
    static constexpr int NL = 2;
    static constexpr int dim(int l) { return l == 0 ? D0 : (l == 1 ? D1 : D2); }
    static constexpr int GG = G_;
};
using ChainShapeLV = ChainShape2<2, 10, 2, 5>;
template <class S> __device__ __forceinline__ int sh_nl(int nl) {
    if constexpr (S::NL > 0) return S::NL;
    else return nl;
}
template <class S> __device__ __forceinline__ int sh_I(const LayerConst& lc, int l) {
    if constexpr (S::NL > 0) return S::dim(l);
    else return lc.I;
}
template <class S> __device__ __forceinline__ int sh_O(const LayerConst& lc, int l) {
    if constexpr (S::NL > 0) return S::dim(l + 1);
    else return lc.O;
}
template <class S> __device__ __forceinline__ int sh_G(const LayerConst& lc) {
    if constexpr (S::NL > 0) return S::GG;
    else return lc.G;
}
static bool chain_is_lv(const LayerConst* hlcs, int nl) {
    return nl == 2 && hlcs[0].I == 2 && hlcs[0].O == 10 && hlcs[1].I == 10 && hlcs[1].O == 2 && hlcs[0].G == 5 &&
           hlcs[1].G == 5;
}

// The forward of a whole small chain for one column group (16 lanes, lane j holds entry j of the
// activation): lane i evaluates the basis and swish of input i and its partial sums for every
// output o, butterfly shuffles sum them over the group, lane o keeps output o.
template <typename T, int NORM, int PATH, class S = ChainShapeAny>
__device__ __forceinline__ T chain_forward(const Math<T>& M, const LayerConst* lcl, int nl, const T* ps, int j, T a);

constexpr int kChainBlock = 256;
constexpr int kChainDim = 16;    // lanes per column = max layer width

// Output-major evaluation of a fixed-shape layer with a few inputs and more outputs (the LV layer
// [2 -> 10]): the I inputs are broadcast from lanes 0..I-1 of the row, every lane evaluates their
// bases, and lane o < O forms output o itself -- no cross-lane sums (input-major, each of the O
// outputs costs two 16-lane row sums: 20 of them for the LV layer).
constexpr int kOutMajorMaxI = 4;
constexpr int kOutMajorMaxG = 8;
template <class S> __host__ __device__ constexpr bool out_major(int l) {
    return S::NL > 0 && S::dim(l) <= kOutMajorMaxI && S::dim(l + 1) > 2 * S::dim(l) && S::GG <= kOutMajorMaxG;
}
// The bases of an output-major layer's inputs as its forward evaluated them, for its pullback in the
// same chain_pullback call (one wave per column: the registers are there; saves the normalizer,
// anchor exponentials and basis recurrence of every input a second time)
template <typename T>
struct OMCache {
    T n[kOutMajorMaxI], sw[kOutMajorMaxI], dsw[kOutMajorMaxI];
    T phi[kOutMajorMaxI][kOutMajorMaxG], z[kOutMajorMaxI][kOutMajorMaxG], aux[kOutMajorMaxI][kOutMajorMaxG];
};
template <typename T, int NORM, int PATH>
__device__ __forceinline__ T layer_fwd_outmajor(const Math<T>& M, const LayerConst& lc, const T* ps, int I, int O,
                                                int G, int j, T a, OMCache<T>* cache = nullptr) {
    const T* __restrict__ C = ps + lc.p_off;
    const T* __restrict__ W = ps + lc.w_off;
    const int o = j < O ? j : 0;   // lanes >= O evaluate output 0 and discard it
    T acc = T(0), bas = T(0);
#pragma unroll
    for (int i = 0; i < kOutMajorMaxI; ++i) {
        if (i < I) {
            const T xi = row16_bcast(a, i);
            const T n = normalize<NORM, T>(M, lc.norm, xi);
            BasisStream<T, PATH> bs;
            bs.init(M, lc, n);
            if (cache) cache->n[i] = n;
#pragma unroll
            for (int g = 0; g < kOutMajorMaxG; ++g) {
                if (g < G) {
                    T z, aux;
                    const T phi = bs.next(M, lc, g, z, aux);
                    acc = kfma<T>(C[o + O * (g + G * i)], phi, acc);
                    if (cache) {
                        cache->phi[i][g] = phi;
                        cache->z[i][g] = z;
                        cache->aux[i][g] = aux;
                    }
                }
            }
            if (lc.use_base) {
                T sw;
                if (cache) {
                    swish_and_grad<T>(M, xi, cache->sw[i], cache->dsw[i]);   // (the same Ω as swish)
                    sw = cache->sw[i];
                } else {
                    sw = swish<T>(M, xi);
                }
                bas = kfma<T>(W[o + O * i], sw, bas);
            }
        }
    }
    return j < O ? (lc.use_base ? acc + bas : acc) : T(0);
}
// Its pullback: lane o holds ȳ_o; it adds ȳ_o φ_c(x) and ȳ_o swish(x_i) into its own entries of the
// group's gradient row and its terms of x̄_i, which the row sums over o; lane i keeps x̄_i.
template <typename T, int NORM, int PATH>
__device__ __forceinline__ T layer_pull_outmajor(const Math<T>& M, const LayerConst& lc, const T* ps,
                                                 T* __restrict__ row, int I, int O, int G, int j, T a, T ybar,
                                                 const OMCache<T>* cache = nullptr) {
    const T* __restrict__ C = ps + lc.p_off;
    const T* __restrict__ W = ps + lc.w_off;
    const bool live = j < O;
    const int o = live ? j : 0;
    const T yb = live ? ybar : T(0);
    const T invh = T(lc.invh);
    T xb = T(0);
#pragma unroll
    for (int i = 0; i < kOutMajorMaxI; ++i) {
        if (i < I) {
            const T xi = cache ? T(0) : row16_bcast(a, i);
            const T n = cache ? cache->n[i] : normalize<NORM, T>(M, lc.norm, xi);
            BasisStream<T, PATH> bs;
            if (!cache) bs.init(M, lc, n);
            T sc = T(0);
#pragma unroll
            for (int g = 0; g < kOutMajorMaxG; ++g) {
                if (g < G) {
                    T z, aux, phi;
                    if (cache) {
                        phi = cache->phi[i][g];
                        z = cache->z[i][g];
                        aux = cache->aux[i][g];
                    } else {
                        phi = bs.next(M, lc, g, z, aux);
                    }
                    const int c = g + G * i;
                    if (live) row[lc.p_off + O * c + o] = kfma<T>(yb, phi, row[lc.p_off + O * c + o]);
                    sc = sc + basis_pull<T>(lc.basis, lc.iqf_quirk, z, phi, aux, C[o + O * c] * yb) * invh;
                }
            }
            T v = row16_sum(sc) * dnormalize<NORM, T>(lc.norm, n);
            if (lc.use_base) {
                T sw, dsw;
                if (cache) {
                    sw = cache->sw[i];
                    dsw = cache->dsw[i];
                } else {
                    swish_and_grad<T>(M, xi, sw, dsw);
                }
                if (live) row[lc.w_off + O * i + o] = kfma<T>(yb, sw, row[lc.w_off + O * i + o]);
                v = v + row16_sum(W[o + O * i] * yb) * dsw;
            }
            if (j == i) xb = v;
        }
    }
    return xb;
}

template <typename T, int NORM, int PATH, class S>
__device__ __forceinline__ T chain_forward(const Math<T>& M, const LayerConst* lcl, int nl, const T* ps, int j, T a) {
    auto layer = [&](int l) {
        const LayerConst& lc = lcl[l];
        const int I = sh_I<S>(lc, l), O = sh_O<S>(lc, l), G = sh_G<S>(lc);
        if (KAN_CHAIN_OUTMAJOR && out_major<S>(l)) {
            a = layer_fwd_outmajor<T, NORM, PATH>(M, lc, ps, I, O, G, j, a);
            return;
        }
        const T* __restrict__ C = ps + lc.p_off;
        const T* __restrict__ W = ps + lc.w_off;
        T acc[kChainDim], bas[kChainDim];
#pragma unroll
        for (int o = 0; o < kChainDim; ++o) { acc[o] = T(0); bas[o] = T(0); }
        if (j < I) {
            BasisStream<T, PATH> bs;
            bs.init(M, lc, normalize<NORM, T>(M, lc.norm, a));
            for (int g = 0; g < G; ++g) {
                T z, aux;
                const T phi = bs.next(M, lc, g, z, aux);
                const T* Cc = C + O * (g + G * j);
#pragma unroll
                for (int o = 0; o < kChainDim; ++o)
                    if (o < O) acc[o] = kfma<T>(Cc[o], phi, acc[o]);
            }
            if (lc.use_base) {
                const T sw = swish<T>(M, a);
                const T* Wj = W + O * j;
#pragma unroll
                for (int o = 0; o < kChainDim; ++o)
                    if (o < O) bas[o] = Wj[o] * sw;
            }
        }
        T out = T(0);
#pragma unroll
        for (int o = 0; o < kChainDim; ++o) {
            if (o < O) {
                const T s = row16_sum(acc[o]);
                const T bsum = lc.use_base ? row16_sum(bas[o]) : T(0);   // (DPP: every lane of the row takes part)
                if (o == j) out = lc.use_base ? s + bsum : s;
            }
        }
        a = out;
    };
    if constexpr (S::NL > 0) {   // fixed shape: unrolled, every layer's loops folded
#pragma unroll
        for (int l = 0; l < S::NL; ++l) layer(l);
    } else {
        for (int l = 0; l < nl; ++l) layer(l);
    }
    return a;
}

// The layer constants (nw words) and the parameters (P) into LDS with every thread's loads in flight before its
// first store (the plain strided loops wait for each load: at 64 threads and P = 240 that was eight dependent round
// trips at every block's start)
template <typename T>
__device__ __forceinline__ void stage_chain_consts(int32_t* __restrict__ dst, const int32_t* __restrict__ src, int nw,
                                                   T* __restrict__ ps, const T* __restrict__ p, int P) {
    constexpr int R = 4;
    const int nt = blockDim.x, n = nw > P ? nw : P;
    for (int b = threadIdx.x; b < n; b += R * nt) {
        int32_t w[R];
        T v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = b + r * nt;
            if (i < nw) w[r] = src[i];
            if (i < P) v[r] = p[i];
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = b + r * nt;
            if (i < nw) dst[i] = w[r];
            if (i < P) ps[i] = v[r];
        }
    }
}

template <typename T, int NORM, int PATH, class S>
__global__ void __launch_bounds__(kChainBlock)
kd_chain_col_kernel(const LayerConst* __restrict__ lcs, int nl, const T* __restrict__ p, int P,
                    const T* __restrict__ x, T* __restrict__ y, int64_t K, StageArgs<T> sa, T* __restrict__ y_out,
                    double* __restrict__ err_slab, double* __restrict__ err_direct) {
    extern __shared__ __attribute__((aligned(16))) unsigned char chain_raw[];
    LayerConst* lcl = reinterpret_cast<LayerConst*>(chain_raw);
    T* ps = reinterpret_cast<T*>(chain_raw + nl * sizeof(LayerConst));
    {
        const int nw = nl * (int)(sizeof(LayerConst) / sizeof(int32_t));
        const int32_t* src = reinterpret_cast<const int32_t*>(lcs);
        int32_t* dst = reinterpret_cast<int32_t*>(chain_raw);
        stage_chain_consts(dst, src, nw, ps, p, P);
    }
    KAN_EXP_TABLE_LDS(tab);   // (its __syncthreads also publishes lcl, ps)
    const Math<T> M{tab};
    const int I0 = lcl[0].I, OL = lcl[nl - 1].O;
    const int j = threadIdx.x & (kChainDim - 1);
    // Runge-Kutta stage (kanode_rhs_stage): input y = x + Σ sa.c k formed here, optional y_out and
    // the embedded-error partial Σ (e/sk)² (block total -> err_slab[block], or err_direct with one block)
    const double sc = stage_scale(sa.cscale);
    const bool want_err = err_slab != nullptr || err_direct != nullptr;
    double eacc = 0.0;
    const int64_t stride = ((int64_t)gridDim.x * blockDim.x) / kChainDim;
    for (int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kChainDim; k < K; k += stride) {
        const int64_t idx = (int64_t)I0 * k + j;
        T a = T(0), x0 = T(0);
        double ev = 0.0;
        if (j < I0) {
            T kv[kMaxStages];
            stage_ld<T>(sa, x, idx, kv);
            a = x0 = x[idx];
#pragma unroll
            for (int m = 0; m < kMaxStages; ++m) {
                if (m < sa.nk) {
                    const T km = kv[m];
                    a = kfma<T>((T)(sa.c[m] * sc), km, a);
                    if (want_err) ev = ::fma(sa.ec[m] * sc, (double)km, ev);
                }
            }
            if (y_out) y_out[idx] = a;
        }
        const T yin = a;
        a = chain_forward<T, NORM, PATH, S>(M, lcl, nl, ps, j, a);
        if (j < OL) {
            y[(int64_t)OL * k + j] = a;
            if (want_err) {
                const double e = ::fma(stage_ec_last(sa) * sc, (double)a, ev);
                const double sk = ::fma(sa.reltol, fmax(kabs((double)x0), kabs((double)yin)), sa.abstol);
                const double r = e / sk;
                eacc = ::fma(r, r, eacc);
            }
        }
    }
    if (want_err) {
        __shared__ double red[kChainBlock / kWave];
        const double v[1] = {eacc};
        block_sum_to<double, 1>(v, 1, red, err_direct ? err_direct : err_slab + blockIdx.x);
    }
}

// The whole Tsit5 solve of a small chain in ONE workgroup (kanode_solve_tsit5 for the
// Lotka-Volterra shape, LV_driver_KANODE.jl:180-184, a batch of <= 16 trajectories): column
// group g (16 lanes) owns trajectory g, lane j < N holds u_j and its seven stage values in
// registers, every stage is chain_forward, and the embedded-error norm over the whole state
// is a block sum that every lane receives, so every lane takes the same step-control decision
// (the arithmetic and order of kanode_solve.cpp solve_t / tsit5_post_kernel: Hairer-Wanner
// initial step, PI controller, saveat from the dense output, FSAL).  No launch or host
// round trip per stage or step: the host loop pays ~6 launches + one 8-byte read per step.
template <typename T, int NORM, int PATH, class S>
__device__ __forceinline__ T chain_pullback(const Math<T>& M, const LayerConst* lcl, int nl, const T* ps,
                                            T* __restrict__ row, int j, T yj, T lj);

// The small-chain right-hand side for the one-workgroup drivers (kan_onewg.hpp): column group g of 16
// lanes holds trajectory g, lane j entry j; f is chain_forward, the VJP chain_pullback with the group
// gradient rows summed into kμ in the order of kd_chain_vjp_stage_kernel + chain_vjp_finish_kernel (4
// groups per block, then the blocks).
template <typename T, int NORM, int PATH, class S>
struct ChainModel {
    const Math<T>& M;
    const LayerConst* lcl;
    int nl;
    const T* ps;
    T* rows;     // [NG][P] group gradient rows (LDS, zero between calls)
    int P, j, NGa;
    bool act;
    int64_t idx, n;
    __device__ T rhs(T y) { return chain_forward<T, NORM, PATH, S>(M, lcl, nl, ps, j, y); }
    __device__ T vjp(T y, T ls, T* __restrict__ km) {
        const T lj = chain_pullback<T, NORM, PATH, S>(M, lcl, nl, ps, rows + (size_t)(threadIdx.x / kChainDim) * P, j,
                                                       y, ls);
        __syncthreads();
        // kμ = Σ of the group rows: 4 groups per block-equivalent, then across them, in order.  The rows of
        // groups without a trajectory (g >= B) stay zero, so they are left out of the sum
        for (int q = threadIdx.x; q < P; q += blockDim.x) {
            T tot = T(0);
            for (int g0 = 0; g0 < NGa; g0 += 4) {
                T sblk = rows[(size_t)g0 * P + q];
                for (int g = g0 + 1; g < g0 + 4 && g < NGa; ++g) sblk = sblk + rows[(size_t)g * P + q];
                tot = g0 == 0 ? sblk : tot + sblk;
            }
            km[q] = tot;
            for (int g = 0; g < NGa; ++g) rows[(size_t)g * P + q] = T(0);
        }
        __syncthreads();
        return act ? lj : T(0);
    }
};

// A whole Tsit5 solve of a small chain in one workgroup: column group g owns trajectory g, lane j holds
// u_j and its seven stage values in registers, every stage is chain_forward, and the embedded-error norm
// over the whole state is a block sum that every lane receives (onewg_tsit5).  No launch or host round
// trip per stage or step: the host loop pays ~6 launches + one 8-byte read per step.
template <typename T, int NORM, int PATH, class S>
__global__ void __launch_bounds__(kChainBlock)
kd_chain_tsit5_kernel(const LayerConst* __restrict__ lcs, int nl, const T* __restrict__ p, int P,
                      const T* __restrict__ u0, int64_t B, ChainSolveArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char cs_raw[];
    LayerConst* lcl = reinterpret_cast<LayerConst*>(cs_raw);
    T* ps = reinterpret_cast<T*>(cs_raw + nl * sizeof(LayerConst));
    {
        const int nw = nl * (int)(sizeof(LayerConst) / sizeof(int32_t));
        const int32_t* src = reinterpret_cast<const int32_t*>(lcs);
        int32_t* dst = reinterpret_cast<int32_t*>(cs_raw);
        stage_chain_consts(dst, src, nw, ps, p, P);
    }
    KAN_EXP_TABLE_LDS(tab);
    __shared__ double red[kChainBlock / kWave];
    const Math<T> M{tab};
    const int N = lcl[0].I;
    const int j = threadIdx.x & (kChainDim - 1);
    const int64_t col = threadIdx.x / kChainDim;
    ChainModel<T, NORM, PATH, S> m{M, lcl, nl, ps, nullptr, P, j, 0, col < B && j < N, (int64_t)N * col + j,
                                   (int64_t)N * B};
    onewg_tsit5<T>(m, u0, a, red);
}

// The adjoint stage of a small chain in one launch (kanode_vjp_stage for the LV [2,10,2]
// shape): 16 lanes per column as in kd_chain_col_kernel.  Lane j forms the forward dense output
// y_j = u_j + Σ su.c k_j and the adjoint stage input λs_j = λ_j + Σ sl.c lk_j, the forward pass
// keeps each layer's input activation in registers, and the backward pass walks the layers in
// reverse: the group broadcasts ȳ_o, lane i (input i) forms x̄_i exactly as kd_vjp_col_kernel
// does and adds ȳ_o φ_g(x_i), ȳ_o swish(x_i) into its own entries of the group's LDS gradient
// row (disjoint per lane, so no atomics).  The block sums its group rows in a fixed order into
// its slab row; chain_vjp_finish_kernel reduces the slab rows (dp) and the λ error partials.
constexpr int kChainVjpBlock = 64;               // 4 columns per block
constexpr int kChainMaxLayers = 4;
// The pullback of a whole small chain for one column group (lane j holds entry j): the forward
// keeps each layer's input activation in registers, the backward walks the layers in reverse;
// ȳ of the last layer is lj, lane i of layer l turns it into x̄_i and adds ȳ_o φ_g(x_i),
// ȳ_o swish(x_i) into its own entries of the group's LDS gradient row (disjoint per lane).
// Returns λᵀ∂f/∂u (lane j: entry j).
template <typename T, int NORM, int PATH, class S = ChainShapeAny>
__device__ __forceinline__ T chain_pullback(const Math<T>& M, const LayerConst* lcl, int nl, const T* ps,
                                            T* __restrict__ row, int j, T yj, T lj) {
    // layer 0's basis cache (omc0) is filled by the forward loop below only when layer 0 is not the
    // last layer: a one-layer output-major shape would read it uninitialised
    static_assert(!(S::NL == 1 && out_major<S>(0)), "an output-major layer must not be the only layer");
    // forward: the input activation of every layer (lane j holds entry j)
    T act[kChainMaxLayers];
    act[0] = yj;
    OMCache<T> omc0;   // layer 0's bases when it is output-major (the only such layer of a fixed shape)
#pragma unroll
    for (int l = 0; l + 1 < kChainMaxLayers; ++l) {
        act[l + 1] = T(0);
        if (l + 1 < sh_nl<S>(nl) && KAN_CHAIN_OUTMAJOR && out_major<S>(l)) {
            const LayerConst& lc = lcl[l];
            act[l + 1] = layer_fwd_outmajor<T, NORM, PATH>(M, lc, ps, sh_I<S>(lc, l), sh_O<S>(lc, l), sh_G<S>(lc), j,
                                                           act[l], l == 0 ? &omc0 : nullptr);
        } else if (l + 1 < sh_nl<S>(nl)) {
            const LayerConst& lc = lcl[l];
            const int I = sh_I<S>(lc, l), O = sh_O<S>(lc, l), G = sh_G<S>(lc);
            const T* __restrict__ C = ps + lc.p_off;
            const T* __restrict__ W = ps + lc.w_off;
            T acc[kChainDim], bas[kChainDim];
#pragma unroll
            for (int o = 0; o < kChainDim; ++o) { acc[o] = T(0); bas[o] = T(0); }
            if (j < I) {
                const T a = act[l];
                BasisStream<T, PATH> bs;
                bs.init(M, lc, normalize<NORM, T>(M, lc.norm, a));
                for (int g = 0; g < G; ++g) {
                    T z, aux;
                    const T phi = bs.next(M, lc, g, z, aux);
                    const T* Cc = C + O * (g + G * j);
#pragma unroll
                    for (int o = 0; o < kChainDim; ++o)
                        if (o < O) acc[o] = kfma<T>(Cc[o], phi, acc[o]);
                }
                if (lc.use_base) {
                    const T sw = swish<T>(M, a);
#pragma unroll
                    for (int o = 0; o < kChainDim; ++o)
                        if (o < O) bas[o] = W[O * j + o] * sw;
                }
            }
            T out = T(0);
#pragma unroll
            for (int o = 0; o < kChainDim; ++o) {
                if (o < O) {
                    const T s = row16_sum(acc[o]);
                    const T bsum = lc.use_base ? row16_sum(bas[o]) : T(0);
                    if (o == j) out = lc.use_base ? s + bsum : s;
                }
            }
            act[l + 1] = out;
        }
    }
    // backward: ȳ of the last layer is λs; lane i of layer l turns it into x̄_i
    T ybar = lj;
#pragma unroll
    for (int l = kChainMaxLayers - 1; l >= 0; --l) {
        if (l < sh_nl<S>(nl) && KAN_CHAIN_OUTMAJOR && out_major<S>(l)) {
            const LayerConst& lc = lcl[l];
            ybar = layer_pull_outmajor<T, NORM, PATH>(M, lc, ps, row, sh_I<S>(lc, l), sh_O<S>(lc, l), sh_G<S>(lc), j,
                                                      act[l], ybar, l == 0 ? &omc0 : nullptr);
        } else if (l < sh_nl<S>(nl)) {
            const LayerConst& lc = lcl[l];
            const int I = sh_I<S>(lc, l), O = sh_O<S>(lc, l), G = sh_G<S>(lc);
            const T* __restrict__ C = ps + lc.p_off;
            const T* __restrict__ W = ps + lc.w_off;
            T yb[kChainDim];
#pragma unroll
            for (int o = 0; o < kChainDim; ++o) yb[o] = o < O ? row16_bcast(ybar, o) : T(0);
            T xb = T(0);
            if (j < I) {
                const T a = act[l];
                const T n = normalize<NORM, T>(M, lc.norm, a);
                BasisStream<T, PATH> bs;
                bs.init(M, lc, n);
                const T invh = T(lc.invh);
                T nbar = T(0);
                for (int g = 0; g < G; ++g) {
                    T z, aux;
                    const T phi = bs.next(M, lc, g, z, aux);
                    const int c = g + G * j;
                    const T* Cc = C + O * c;
                    T* __restrict__ rc = row + lc.p_off + O * c;
                    T bb = T(0);
#pragma unroll
                    for (int o = 0; o < kChainDim; ++o) {
                        if (o < O) {
                            bb = kfma<T>(Cc[o], yb[o], bb);
                            rc[o] = kfma<T>(yb[o], phi, rc[o]);
                        }
                    }
                    const T zb = basis_pull<T>(lc.basis, lc.iqf_quirk, z, phi, aux, bb);
                    nbar = nbar + zb * invh;
                }
                xb = nbar * dnormalize<NORM, T>(lc.norm, n);
                if (lc.use_base) {
                    T sw, dsw;
                    swish_and_grad<T>(M, a, sw, dsw);
                    const T* Wj = W + O * j;
                    T* __restrict__ rw = row + lc.w_off + O * j;
                    T sb = T(0);
#pragma unroll
                    for (int o = 0; o < kChainDim; ++o) {
                        if (o < O) {
                            sb = kfma<T>(Wj[o], yb[o], sb);
                            rw[o] = kfma<T>(yb[o], sw, rw[o]);
                        }
                    }
                    xb = xb + sb * dsw;
                }
            }
            ybar = xb;
        }
    }
    return ybar;
}

template <typename T, int NORM, int PATH, class S>
__global__ void __launch_bounds__(kChainVjpBlock)
kd_chain_vjp_stage_kernel(const LayerConst* __restrict__ lcs, int nl, const T* __restrict__ p, int P,
                          const T* __restrict__ u, StageArgs<T> su, const T* __restrict__ lam, StageArgs<T> sl,
                          T* __restrict__ lam_out, T* __restrict__ lamJ, T* __restrict__ slab,
                          double* __restrict__ err_slab, int64_t K, T* __restrict__ dp_direct, int assign,
                          double* __restrict__ err_direct) {
    extern __shared__ __attribute__((aligned(16))) unsigned char cv_raw[];
    constexpr int NG = kChainVjpBlock / kChainDim;
    LayerConst* lcl = reinterpret_cast<LayerConst*>(cv_raw);
    T* ps = reinterpret_cast<T*>(cv_raw + nl * sizeof(LayerConst));
    T* rows = ps + P;                                 // [NG][P] gradient rows
    {
        const int nw = nl * (int)(sizeof(LayerConst) / sizeof(int32_t));
        const int32_t* src = reinterpret_cast<const int32_t*>(lcs);
        int32_t* dst = reinterpret_cast<int32_t*>(cv_raw);
        stage_chain_consts(dst, src, nw, ps, p, P);
        for (int i = threadIdx.x; i < NG * P; i += blockDim.x) rows[i] = T(0);
    }
    KAN_EXP_TABLE_LDS(tab);   // (its __syncthreads also publishes lcl, ps, rows)
    const Math<T> M{tab};
    const int N0 = lcl[0].I;
    const int j = threadIdx.x & (kChainDim - 1);
    T* __restrict__ row = rows + (threadIdx.x / kChainDim) * P;
    const double suc = stage_scale(su.cscale), slc = stage_scale(sl.cscale);
    const bool want_err = err_slab != nullptr || err_direct != nullptr;
    double eacc = 0.0;
    const int64_t stride = ((int64_t)gridDim.x * blockDim.x) / kChainDim;
    for (int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kChainDim; k < K; k += stride) {
        const int64_t idx = (int64_t)N0 * k + j;
        T yj = T(0), lj = T(0), l0 = T(0);
        double ev = 0.0;
        if (j < N0) {
            T kv[kMaxStages], kw[kMaxStages];
            stage_ld<T>(su, u, idx, kv);
            stage_ld<T>(sl, lam, idx, kw);
            yj = u[idx];
#pragma unroll
            for (int m = 0; m < kMaxStages; ++m)
                if (m < su.nk) yj = kfma<T>((T)(su.c[m] * suc), kv[m], yj);
            lj = lam[idx];
            l0 = lj;
#pragma unroll
            for (int m = 0; m < kMaxStages; ++m) {
                if (m < sl.nk) {
                    const T km = kw[m];
                    lj = kfma<T>((T)(sl.c[m] * slc), km, lj);
                    if (want_err) ev = ::fma(sl.ec[m] * slc, (double)km, ev);
                }
            }
            if (lam_out) lam_out[idx] = lj;
        }
        const T ybar = chain_pullback<T, NORM, PATH, S>(M, lcl, nl, ps, row, j, yj, lj);
        if (j < N0) {
            lamJ[idx] = ybar;
            if (want_err) {
                const double e = ::fma(stage_ec_last(sl) * slc, (double)ybar, ev);
                const double sk = ::fma(sl.reltol, fmax(kabs((double)l0), kabs((double)lj)), sl.abstol);
                const double r = e / sk;
                eacc = ::fma(r, r, eacc);
            }
        }
    }
    __syncthreads();
    // one block (a few columns, e.g. the single LV trajectory): the block's sums are the totals
    for (int q = threadIdx.x; q < P; q += blockDim.x) {
        T s = rows[q];
#pragma unroll
        for (int g = 1; g < NG; ++g) s = s + rows[g * P + q];
        if (dp_direct) dp_direct[q] = assign ? s : dp_direct[q] + s;
        else if (slab) slab[(int64_t)blockIdx.x * P + q] = s;
    }
    if (want_err) {
        __shared__ double red[kChainVjpBlock / kWave];
        const double v[1] = {eacc};
        block_sum_to<double, 1>(v, 1, red, err_direct ? err_direct : err_slab + blockIdx.x);
    }
}

// (the generic shapes' stage loop is not unrolled; only the fixed LV shape needs it to be)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wpass-failed"
// The six adjoint stages of one InterpolatingAdjoint step in one launch (ChainAdjStep, kan_kernels.hpp): per
// column, stage s forms the forward dense output and λs exactly as kd_chain_vjp_stage_kernel does from the
// integrator's stage arrays, but kλ_1..kλ_6 stay in registers; the stage's parameter cotangents go to the group's
// LDS row of that stage and the block's per-stage sums to slab region s.  Only λ_new and kλ_7 are written.
template <typename T, int NORM, int PATH, class S>
__global__ void __launch_bounds__(kChainVjpBlock)
kd_chain_vjp_step_kernel(const LayerConst* __restrict__ lcs, int nl, const T* __restrict__ p, int P, int64_t K,
                         ChainAdjStep<T> a, T* __restrict__ slab, int64_t region, double* __restrict__ err_slab) {
    extern __shared__ __attribute__((aligned(16))) unsigned char cs_raw[];
    constexpr int NG = kChainVjpBlock / kChainDim;
    LayerConst* lcl = reinterpret_cast<LayerConst*>(cs_raw);
    T* ps = reinterpret_cast<T*>(cs_raw + nl * sizeof(LayerConst));
    T* rows = ps + P;                                 // [6 (+1 with fsal)][NG][P] gradient rows
    const int nreg = a.fsal ? 7 : 6;
    {
        const int nw = nl * (int)(sizeof(LayerConst) / sizeof(int32_t));
        const int32_t* src = reinterpret_cast<const int32_t*>(lcs);
        int32_t* dst = reinterpret_cast<int32_t*>(cs_raw);
        stage_chain_consts(dst, src, nw, ps, p, P);
        for (int i = threadIdx.x; i < nreg * NG * P; i += blockDim.x) rows[i] = T(0);
    }
    KAN_EXP_TABLE_LDS(tab);   // (its __syncthreads also publishes lcl, ps, rows)
    const Math<T> M{tab};
    const int N0 = lcl[0].I;
    const int j = threadIdx.x & (kChainDim - 1);
    const int g = threadIdx.x / kChainDim;
    double eacc = 0.0;
    const int64_t stride = ((int64_t)gridDim.x * blockDim.x) / kChainDim;
    for (int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kChainDim; k < K; k += stride) {
        const int64_t idx = (int64_t)N0 * k + j;
        const bool live = j < N0;
        T kl[7];
        T l0 = live ? a.lam[idx] : T(0);
        if (a.fsal) {   // the stop's jump and FSAL re-evaluation (the stage kernel's arithmetic for that call)
            T yj = T(0);
            if (live) {
                T kv[7];
#pragma unroll
                for (int q = 0; q < 7; ++q) kv[q] = a.j_k[q][idx];
                yj = a.j_u[idx];
#pragma unroll
                for (int q = 0; q < 7; ++q) yj = kfma<T>((T)a.j_c[q], kv[q], yj);
                for (int r = 0; r < a.njump; ++r) l0 = kfma<T>(T(1), a.jump[r][idx], l0);
            }
            kl[0] = chain_pullback<T, NORM, PATH, S>(M, lcl, nl, ps, rows + ((size_t)6 * NG + g) * P, j, yj, l0);
        } else {
            kl[0] = live ? a.kl1[idx] : T(0);
        }
        T ls = l0;
        double ev = 0.0;
#pragma unroll
        for (int s = 0; s < 6; ++s) {
            T yj = T(0);
            if (live) {
                T kv[7];
#pragma unroll
                for (int q = 0; q < 7; ++q) kv[q] = a.su_k[s][q][idx];   // (all loads first)
                yj = a.su_u[s][idx];
#pragma unroll
                for (int q = 0; q < 7; ++q) yj = kfma<T>((T)a.su_c[s][q], kv[q], yj);
                ls = l0;
#pragma unroll
                for (int q = 0; q <= s; ++q) {
                    ls = kfma<T>((T)a.a[s][q], kl[q], ls);
                    if (s == 5) ev = ::fma(a.ec[q], (double)kl[q], ev);
                }
            }
            kl[s + 1] = chain_pullback<T, NORM, PATH, S>(M, lcl, nl, ps, rows + ((size_t)s * NG + g) * P, j, yj, ls);
        }
        if (live) {
            a.lam_out[idx] = ls;
            a.kl7[idx] = kl[6];
            if (a.want_error) {
                const double e = ::fma(a.ec[6], (double)kl[6], ev);
                const double sk = ::fma(a.reltol, fmax(kabs((double)l0), kabs((double)ls)), a.abstol);
                const double r = e / sk;
                eacc = ::fma(r, r, eacc);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nreg * P; i += blockDim.x) {   // each stage's block sums, the stage kernel's order
        const int s = i / P, q = i - s * P;
        const T* r0 = rows + (size_t)s * NG * P;
        T v = r0[q];
#pragma unroll
        for (int gg = 1; gg < NG; ++gg) v = v + r0[gg * P + q];
        slab[s * region + (int64_t)q * gridDim.x + blockIdx.x] = v;   // parameter-major: the finish reads rows
    }
    if (a.want_error) {
        __shared__ double red[kChainVjpBlock / kWave];
        const double v[1] = {eacc};
        block_sum_to<double, 1>(v, 1, red, err_slab + blockIdx.x);
    }
}

#pragma clang diagnostic pop

// km_out[s][q] = Σ_b slab[s·region + q·nblk + b] (block (q, s), q < P) and err_out[0] = Σ_b err_slab[b] (block (P, 0)):
// chain_vjp_finish_kernel's sums for the six stages of a step in one launch
template <typename T>
__global__ void __launch_bounds__(kBlock)
chain_vjp_step_finish_kernel(const T* __restrict__ slab, int64_t region, int64_t nblk, int64_t P, ChainKmOut<T> km,
                             const double* __restrict__ err_slab, double* __restrict__ err_out) {
    __shared__ double red[kBlock / kWave];
    const int64_t q = blockIdx.x;
    const int s = blockIdx.y;
    if (q == P && (s != 0 || !err_out)) return;
    double acc = 0.0;
    if (q < P) {
        acc = strided_rows_sum(slab + s * region + q * nblk, nblk, 1, acc);   // (the same order as a stride-P walk)
    } else {
        acc = strided_rows_sum(err_slab, nblk, 1, acc);
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = red[0];
        for (int w = 1; w < (int)(blockDim.x / kWave); ++w) t += red[w];
        T* const out = s == 0 ? km.k[0] : s == 1 ? km.k[1] : s == 2 ? km.k[2] : s == 3 ? km.k[3] : s == 4 ? km.k[4]
                     : s == 5 ? km.k[5] : km.k[6];
        if (q < P) out[q] = (T)t;
        else err_out[0] = t;
    }
}

// dp[q] (= or +=) Σ_b slab[b·P + q] (block q < P) and err_out[0] = Σ_b err_slab[b] (block P)
template <typename T>
__global__ void __launch_bounds__(kBlock)
chain_vjp_finish_kernel(const T* __restrict__ slab, int64_t nblk, int64_t P, T* __restrict__ dp, int assign,
                        const double* __restrict__ err_slab, double* __restrict__ err_out) {
    __shared__ double red[kBlock / kWave];
    const int64_t q = blockIdx.x;
    double s = 0.0;
    if (q < P) {
        s = strided_rows_sum(slab + q, nblk, P, s);
    } else {
        s = strided_rows_sum(err_slab, nblk, 1, s);
    }
    s = wave_sum(s);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = red[0];
        for (int w = 1; w < (int)(blockDim.x / kWave); ++w) t += red[w];
        if (q < P) dp[q] = assign ? (T)t : dp[q] + (T)t;
        else err_out[0] = t;
    }
}

// Column VJP with LDS staging: per tile of TILE columns every thread stages its
// basis values φ[c][t], ȳ[o][t], swish(x)[i][t] in LDS (rows padded to TILE+1),
// then the block computes the tile's dC = ȳ·φᵀ, dW = ȳ·swish(x)ᵀ with each
// thread owning <= NPT parameters (accumulated in registers across tiles).
template <typename T, int NORM, int PATH, int OMAX, int TILE, int NPT>
__global__ void __launch_bounds__(TILE)
kd_vjp_col_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                  const T* __restrict__ ybar, T* __restrict__ xbar, T* __restrict__ slab, int64_t K) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    KAN_EXP_TABLE_LDS(tab);
    const Math<T> M{tab};
    T* smem = reinterpret_cast<T*>(smem_raw);
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;
    const int GI = G * I;
    const int nC = O * GI;
    const int P = nC + (lc.use_base ? O * I : 0);
    constexpr int LD = TILE + 1;
    T* phiL = smem;                        // [GI][LD]
    T* ybL = phiL + (int64_t)GI * LD;      // [O][LD]
    T* swL = ybL + (int64_t)O * LD;        // [I][LD]
    const T* __restrict__ C = p + lc.p_off;
    const T* __restrict__ W = p + lc.w_off;
    const int t = threadIdx.x;
    T dacc[NPT];
#pragma unroll
    for (int q = 0; q < NPT; ++q) dacc[q] = T(0);
    const T invh = T(lc.invh);
    for (int64_t tile = blockIdx.x; tile * TILE < K; tile += gridDim.x) {
        const int64_t k = tile * TILE + t;
        const bool valid = k < K;
        T yb[OMAX];
#pragma unroll
        for (int o = 0; o < OMAX; ++o) yb[o] = (o < O && valid) ? ybar[(int64_t)O * k + o] : T(0);
#pragma unroll
        for (int o = 0; o < OMAX; ++o)
            if (o < O) ybL[o * LD + t] = yb[o];
        for (int i = 0; i < I; ++i) {
            const T xi = valid ? x[(int64_t)I * k + i] : T(0);
            const T n = normalize<NORM, T>(M, lc.norm, xi);
            BasisStream<T, PATH> bs;
            bs.init(M, lc, n);
            T nbar = T(0);
            for (int g = 0; g < G; ++g) {
                T z, aux;
                const T phi = bs.next(M, lc, g, z, aux);
                const int c = g + G * i;
                const T* Cc = C + (int64_t)O * c;
                T bb = T(0);
#pragma unroll
                for (int o = 0; o < OMAX; ++o)
                    if (o < O) bb = kfma<T>(Cc[o], yb[o], bb);
                const T zb = basis_pull<T>(lc.basis, lc.iqf_quirk, z, phi, aux, bb);
                nbar = nbar + zb * invh;
                phiL[c * LD + t] = valid ? phi : T(0);
            }
            T xb = nbar * dnormalize<NORM, T>(lc.norm, n);
            if (lc.use_base) {
                T sw, dsw;
                swish_and_grad<T>(M, xi, sw, dsw);
                const T* Wi = W + (int64_t)O * i;
                T sb = T(0);
#pragma unroll
                for (int o = 0; o < OMAX; ++o)
                    if (o < O) sb = kfma<T>(Wi[o], yb[o], sb);
                xb = xb + sb * dsw;
                swL[i * LD + t] = valid ? sw : T(0);
            }
            if (valid) xbar[(int64_t)I * k + i] = xb;
        }
        __syncthreads();
        const int nt = (int)((K - tile * TILE) < TILE ? (K - tile * TILE) : TILE);
#pragma unroll
        for (int qq = 0; qq < NPT; ++qq) {
            const int q = t + qq * TILE;
            if (q < P) {
                const T* a;
                const T* b;
                if (q < nC) { a = ybL + (q % O) * LD; b = phiL + (q / O) * LD; }
                else { const int r = q - nC; a = ybL + (r % O) * LD; b = swL + (r / O) * LD; }
                T s = T(0);
                for (int tt = 0; tt < nt; ++tt) s = kfma<T>(a[tt], b[tt], s);
                dacc[qq] += s;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int qq = 0; qq < NPT; ++qq) {
        const int q = t + qq * TILE;
        if (q < P) slab[(int64_t)blockIdx.x * P + q] = dacc[qq];
    }
}

// Per-edge activations act[o + O*(i + I*k)] (Activation_getter.jl:28-31,48-53).
template <typename T, int NORM, int PATH, int OMAX>
__global__ void __launch_bounds__(kBlock)
kd_edge_act_kernel(const LayerConst* __restrict__ lcp, const T* __restrict__ p, const T* __restrict__ x,
                   T* __restrict__ act, int64_t K) {
    KAN_EXP_TABLE_LDS(tab);
    const Math<T> M{tab};
    const LayerConst& lc = *lcp;
    const int I = lc.I, O = lc.O, G = lc.G;
    const T* __restrict__ C = p + lc.p_off;
    const T* __restrict__ W = p + lc.w_off;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < K; k += stride) {
        for (int i = 0; i < I; ++i) {
            const T xi = x[(int64_t)I * k + i];
            T acc[OMAX];
#pragma unroll
            for (int o = 0; o < OMAX; ++o) acc[o] = T(0);
            BasisStream<T, PATH> bs;
            bs.init(M, lc, normalize<NORM, T>(M, lc.norm, xi));
            for (int g = 0; g < G; ++g) {
                T z, aux;
                const T phi = bs.next(M, lc, g, z, aux);
                const T* Cc = C + (int64_t)O * (g + (int64_t)G * i);
#pragma unroll
                for (int o = 0; o < OMAX; ++o)
                    if (o < O) acc[o] = kfma<T>(phi, Cc[o], acc[o]);
            }
            const T sw = lc.use_base ? swish<T>(M, xi) : T(0);
#pragma unroll
            for (int o = 0; o < OMAX; ++o)
                if (o < O)
                    act[(int64_t)O * ((int64_t)I * k + i) + o] =
                        lc.use_base ? kfma<T>(sw, W[(int64_t)O * i + o], acc[o]) : acc[o];
        }
    }
}

// ---------------------------------------------------------------------------
// launchers: the LV configuration (tanh_fast, exact G=5 grid) is specialised;
// every other layer runs the runtime-normalizer kernels.
template <typename T, int NORM, int PATH>
static hipError_t col_fwd_go(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, T* y, int64_t K,
                             hipStream_t st) {
    const int g = grid_for(K, kBlock, kGridCap);
    if (hlc.O <= 16)
        hipLaunchKernelGGL((kd_fwd_col_kernel<T, NORM, PATH, 16>), dim3(g), dim3(kBlock), 0, st, lc, p, x, y, K);
    else
        hipLaunchKernelGGL((kd_fwd_col_kernel<T, NORM, PATH, 64>), dim3(g), dim3(kBlock), 0, st, lc, p, x, y, K);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_kd_fwd_col(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, T* y, int64_t K,
                             hipStream_t st) {
    if (hlc.norm == NORM_TANH_FAST && hlc.path == PATH_REC) return col_fwd_go<T, NORM_TANH_FAST, PATH_REC>(hlc, lc, p, x, y, K, st);
    switch (hlc.path) {
    case PATH_REC_CORR: return col_fwd_go<T, NORM_RUNTIME, PATH_REC_CORR>(hlc, lc, p, x, y, K, st);
    case PATH_REC: return col_fwd_go<T, NORM_RUNTIME, PATH_REC>(hlc, lc, p, x, y, K, st);
    default: return col_fwd_go<T, NORM_RUNTIME, PATH_DIRECT>(hlc, lc, p, x, y, K, st);
    }
}

template <typename T, int NORM, int PATH, int TILE, int NPT>
static hipError_t col_vjp_go2(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, const T* yb,
                              T* xb, T* pbar, T* slab, int slab_blocks, int64_t K, hipStream_t st) {
    const int GI = hlc.G * hlc.I;
    const size_t lds = sizeof(T) * (size_t)(GI + hlc.O + hlc.I) * (TILE + 1);
    const int P = hlc.O * GI + (hlc.use_base ? hlc.O * hlc.I : 0);
    const int nb = grid_for(K, TILE, slab_blocks);
    hipLaunchKernelGGL((kd_vjp_col_kernel<T, NORM, PATH, 16, TILE, NPT>), dim3(nb), dim3(TILE), lds, st, lc, p, x,
                       yb, xb, slab, K);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !pbar) return e;
    return launch_slab_reduce<T>(slab, nb, P, pbar + hlc.p_off, st);
}

template <typename T, int NORM, int PATH>
static hipError_t col_vjp_go(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, const T* yb, T* xb,
                             T* pbar, T* slab, int slab_blocks, int64_t K, hipStream_t st) {
    const int GI = hlc.G * hlc.I;
    const int P = hlc.O * GI + (hlc.use_base ? hlc.O * hlc.I : 0);
    const size_t rows = (size_t)(GI + hlc.O + hlc.I);
    if (rows * 257 * sizeof(T) <= 150 * 1024 && P <= 256 * 8)
        return col_vjp_go2<T, NORM, PATH, 256, 8>(hlc, lc, p, x, yb, xb, pbar, slab, slab_blocks, K, st);
    // narrow tile (64 columns, one wave) for wider layers
    return col_vjp_go2<T, NORM, PATH, 64, 32>(hlc, lc, p, x, yb, xb, pbar, slab, slab_blocks, K, st);
}

template <typename T>
hipError_t launch_kd_vjp_col(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, const T* yb,
                             T* xb, T* pbar, T* slab, int slab_blocks, int64_t K, hipStream_t st) {
    if (hlc.norm == NORM_TANH_FAST && hlc.path == PATH_REC)
        return col_vjp_go<T, NORM_TANH_FAST, PATH_REC>(hlc, lc, p, x, yb, xb, pbar, slab, slab_blocks, K, st);
    switch (hlc.path) {
    case PATH_REC_CORR:
        return col_vjp_go<T, NORM_RUNTIME, PATH_REC_CORR>(hlc, lc, p, x, yb, xb, pbar, slab, slab_blocks, K, st);
    case PATH_REC:
        return col_vjp_go<T, NORM_RUNTIME, PATH_REC>(hlc, lc, p, x, yb, xb, pbar, slab, slab_blocks, K, st);
    default:
        return col_vjp_go<T, NORM_RUNTIME, PATH_DIRECT>(hlc, lc, p, x, yb, xb, pbar, slab, slab_blocks, K, st);
    }
}

template <typename T, int PATH>
static hipError_t edge_go(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, T* act, int64_t K,
                          hipStream_t st) {
    const int g = grid_for(K, kBlock, kGridCap);
    if (hlc.O <= 16)
        hipLaunchKernelGGL((kd_edge_act_kernel<T, NORM_RUNTIME, PATH, 16>), dim3(g), dim3(kBlock), 0, st, lc, p, x,
                           act, K);
    else
        hipLaunchKernelGGL((kd_edge_act_kernel<T, NORM_RUNTIME, PATH, 64>), dim3(g), dim3(kBlock), 0, st, lc, p, x,
                           act, K);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_kd_edge_act(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, T* act, int64_t K,
                              hipStream_t st) {
    switch (hlc.path) {
    case PATH_REC_CORR: return edge_go<T, PATH_REC_CORR>(hlc, lc, p, x, act, K, st);
    case PATH_REC: return edge_go<T, PATH_REC>(hlc, lc, p, x, act, K, st);
    default: return edge_go<T, PATH_DIRECT>(hlc, lc, p, x, act, K, st);
    }
}

static bool I_ne_O(const LayerConst* hlcs, int nl) { return hlcs[0].I != hlcs[nl - 1].O; }

// One launch for the whole chain when every layer is small (I, O <= 16), shares the
// normalizer/path specialisation, the parameters fit in LDS and the batch is small enough
// to be latency-bound; else returns hipErrorNotSupported and the caller runs one launch
// per layer.
template <typename T>
hipError_t launch_kd_chain_col(const LayerConst* hlcs, int nl, const LayerConst* lcs, const T* p, int64_t P,
                               const T* x, T* y, int64_t K, hipStream_t st, const StageArgs<T>* sa, T* y_out,
                               double* err_slab, int slab_rows, double* err_out) {
    // 16 lanes per column pays while the batch leaves the chip latency-bound (<= 32 columns
    // per CU); beyond that the per-layer thread-per-column kernels keep every lane busy
    if (nl < 1 || nl > 8 || K > 32768) return hipErrorNotSupported;
    for (int l = 0; l < nl; ++l) {
        const LayerConst& h = hlcs[l];
        if (h.I > kChainDim || h.O > kChainDim || h.path != hlcs[0].path || h.norm != hlcs[0].norm)
            return hipErrorNotSupported;
        if (l > 0 && h.I != hlcs[l - 1].O) return hipErrorNotSupported;
    }
    const size_t lds = nl * sizeof(LayerConst) + (size_t)P * sizeof(T);
    if (lds > 48 * 1024) return hipErrorNotSupported;
    if (sa && I_ne_O(hlcs, nl)) return hipErrorNotSupported;
    const StageArgs<T> none{};
    const StageArgs<T>& s = sa ? *sa : none;
    const int g = grid_for(K * kChainDim, kChainBlock, err_out ? (slab_rows < kGridCap ? slab_rows : kGridCap) : kGridCap);
    const bool one = g == 1;
    double* es = err_out && !one ? err_slab : nullptr;
    double* ed = err_out && one ? err_out : nullptr;
    const LayerConst& h = hlcs[0];
#define KAN_CHAIN_S(NORM, PATH, S)                                                                                    \
    hipLaunchKernelGGL((kd_chain_col_kernel<T, NORM, PATH, S>), dim3(g), dim3(kChainBlock), lds, st, lcs, nl, p,     \
                       (int)P, x, y, K, s, y_out, es, ed)
    if (h.norm == NORM_TANH_FAST && h.path == PATH_REC && chain_is_lv(hlcs, nl))
        KAN_CHAIN_S(NORM_TANH_FAST, PATH_REC, ChainShapeLV);
    else if (h.norm == NORM_TANH_FAST && h.path == PATH_REC) KAN_CHAIN_S(NORM_TANH_FAST, PATH_REC, ChainShapeAny);
    else if (h.path == PATH_REC_CORR) KAN_CHAIN_S(NORM_RUNTIME, PATH_REC_CORR, ChainShapeAny);
    else if (h.path == PATH_REC) KAN_CHAIN_S(NORM_RUNTIME, PATH_REC, ChainShapeAny);
    else KAN_CHAIN_S(NORM_RUNTIME, PATH_DIRECT, ChainShapeAny);
#undef KAN_CHAIN_S
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !es) return e;
    return launch_stage_error_final(err_slab, g, err_out, st);
}

// The InterpolatingAdjoint of a small chain in ONE workgroup (kanode_adjoint_tsit5 after a
// kd_chain_tsit5_kernel forward): the backward Tsit5 over [λ; μ] with the steps, stops, jumps,
// FSAL re-evaluation and controller of kanode_solve.cpp adjoint_t.  Column group g holds λ of
// trajectory g and its seven stage values in registers; every adjoint stage interpolates the
// forward dense output u(tf - τ), forms λs = λ + h Σ a_sj kλ_j, runs chain_pullback (each group
// adds into its own LDS gradient row) and reduces the rows into the stage's kμ (LDS), in the
// order kd_chain_vjp_stage_kernel + chain_vjp_finish_kernel use (4 groups per block, then the
// blocks).  μ and its seven stage vectors live in LDS; the error norm covers λ and μ.
// A whole Tsit5 step of a small chain per trajectory column, in one launch (kanode_solve_tsit5's
// host loop for batches the one-workgroup solve does not take): column group g keeps u, k_1..k_7
// of its column in registers through the six stages (chain_forward each), writes k_2..k_7 and
// u_new once, and adds its embedded-error partial to the block's slab row.  Same arithmetic as
// six kd_chain_col_kernel stage launches.
template <typename T, int NORM, int PATH, class S>
__global__ void __launch_bounds__(kChainBlock)
kd_chain_step_kernel(const LayerConst* __restrict__ lcs, int nl, const T* __restrict__ p, int P, int64_t K,
                     ChainStepArgs a, double* __restrict__ err_slab) {
    extern __shared__ __attribute__((aligned(16))) unsigned char cst_raw[];
    LayerConst* lcl = reinterpret_cast<LayerConst*>(cst_raw);
    T* ps = reinterpret_cast<T*>(cst_raw + nl * sizeof(LayerConst));
    {
        const int nw = nl * (int)(sizeof(LayerConst) / sizeof(int32_t));
        const int32_t* src = reinterpret_cast<const int32_t*>(lcs);
        int32_t* dst = reinterpret_cast<int32_t*>(cst_raw);
        stage_chain_consts(dst, src, nw, ps, p, P);
    }
    KAN_EXP_TABLE_LDS(tab);
    const Math<T> M{tab};
    const int N = lcl[0].I;
    const int j = threadIdx.x & (kChainDim - 1);
    const T* __restrict__ u = reinterpret_cast<const T*>(a.u);
    const T* __restrict__ k1 = reinterpret_cast<const T*>(a.k1);
    double eacc = 0.0;
    const int64_t stride = ((int64_t)gridDim.x * blockDim.x) / kChainDim;
    for (int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kChainDim; k < K; k += stride) {
        const bool act = j < N;
        const int64_t idx = (int64_t)N * k + j;
        const T uv = act ? u[idx] : T(0);
        T kk[7];
        kk[0] = act ? k1[idx] : T(0);
        T y = uv;
#pragma unroll
        for (int s = 0; s < 6; ++s) {
            y = uv;
#pragma unroll
            for (int m = 0; m <= s; ++m) y = kfma<T>((T)a.a[s][m], kk[m], y);
            kk[s + 1] = chain_forward<T, NORM, PATH, S>(M, lcl, nl, ps, j, y);
            if (act) reinterpret_cast<T*>(a.k[s])[idx] = kk[s + 1];
        }
        if (act) {
            reinterpret_cast<T*>(a.u_new)[idx] = y;
            if (err_slab) {
                double ev = 0.0;
#pragma unroll
                for (int m = 0; m < 6; ++m) ev = ::fma(a.e[m], (double)kk[m], ev);
                const double e = ::fma(a.e[6], (double)kk[6], ev);
                const double sk = ::fma(a.reltol, fmax(kabs((double)uv), kabs((double)y)), a.abstol);
                const double r = e / sk;
                eacc = ::fma(r, r, eacc);
            }
        }
    }
    if (err_slab) {
        __shared__ double red[kChainBlock / kWave];
        const double v[1] = {eacc};
        block_sum_to<double, 1>(v, 1, red, err_slab + blockIdx.x);
    }
}

// (the generic-shape instantiations are too large for the stage loop to be unrolled; their
// stage values then live in scratch, which only the non-LV small chains pay for)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wpass-failed"
// The whole InterpolatingAdjoint of a small chain in one workgroup (onewg_adjoint), after a
// kd_chain_tsit5_kernel forward: column group g holds λ of trajectory g and its seven stage values in
// registers; μ, its seven stage vectors and the group gradient rows in LDS.
template <typename T, int NORM, int PATH, class S>
__global__ void __launch_bounds__(kChainBlock)
kd_chain_adjoint_kernel(const LayerConst* __restrict__ lcs, int nl, const T* __restrict__ p, int P, int64_t B,
                        ChainAdjointArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char ca_raw[];
    const int NG = blockDim.x / kChainDim;
    const int NGa = B < NG ? (int)B : NG;   // groups holding a trajectory
    LayerConst* lcl = reinterpret_cast<LayerConst*>(ca_raw);
    T* ps = reinterpret_cast<T*>(ca_raw + nl * sizeof(LayerConst));
    T* rows = ps + P;                        // [NG][P] gradient rows
    T* mu = rows + (size_t)NG * P;           // [2][P]
    T* km = mu + 2 * (size_t)P;              // [7][P]
    double* tsl = reinterpret_cast<double*>(km + 7 * (size_t)P);   // [nsteps] (8-byte aligned: P·sizeof(T) offsets)
    double* dtsl = tsl + a.nsteps;
    {
        const int nw = nl * (int)(sizeof(LayerConst) / sizeof(int32_t));
        const int32_t* src = reinterpret_cast<const int32_t*>(lcs);
        int32_t* dst = reinterpret_cast<int32_t*>(ca_raw);
        stage_chain_consts(dst, src, nw, ps, p, P);
        for (int i = threadIdx.x; i < NG * P + 9 * P; i += blockDim.x) rows[i] = T(0);
        for (int64_t i = threadIdx.x; i < a.nsteps; i += blockDim.x) {
            tsl[i] = a.ts[i];
            dtsl[i] = a.dts[i];
        }
    }
    KAN_EXP_TABLE_LDS(tab);
    __shared__ double red[kChainBlock / kWave];
    const Math<T> M{tab};
    const int N = lcl[0].I;
    const int j = threadIdx.x & (kChainDim - 1);
    const int64_t col = threadIdx.x / kChainDim;
    ChainModel<T, NORM, PATH, S> m{M, lcl, nl, ps, rows, P, j, NGa, col < B && j < N, (int64_t)N * col + j,
                                   (int64_t)N * B};
    onewg_adjoint<T>(m, a, mu, km, tsl, dtsl, red);
}
#pragma clang diagnostic pop

// ---- one trajectory over a whole workgroup (LV_driver_KANODE.jl:180-184,279-291) ------------
// At B = 1 the group model above runs every adjoint stage as one 16-lane group's serial chain (~1,900
// dependent VALU per stage, one wave, the other 240 lanes idle).  Here the four waves split the pullback of a
// two-layer chain [I -> H -> O] by (output, basis feature): row r (16 lanes) of the block owns hidden unit r of
// layer 1 and lane c its feature c = (input i, knot g | swish); wave o owns output o of layer 2 and lane c its
// feature c.  Every lane evaluates ONE basis function (the reference formula, utils.jl:8-13, one exp), the
// sums over features are DPP row / wave sums and LDS gathers, and every parameter cotangent (∂f/∂p)ᵀλ is
// one lane's single product: kμ needs no reduction at all.  Seven block barriers per adjoint stage.
constexpr int kWideF1 = 16;   // layer-1 features per hidden unit (one DPP row)
constexpr int kWideF2 = 64;   // layer-2 features per output (one wave)
struct WideShape {
    int I, H, O, G1, G2;
};
__host__ __device__ inline bool wide_fits(const WideShape& w) {
    return w.I >= 1 && w.O >= 1 && w.I == w.O && w.H <= kChainBlock / kWideF1 && w.I * (w.G1 + 1) <= kWideF1 &&
           w.H * (w.G2 + 1) <= kWideF2 && w.O <= kChainBlock / kWave;
}

// One feature of a layer at input value x: c < G -> basis g = c of N(x), c == G -> swish(x).  feat, and the
// rrule factors: for a basis the pullback factor -2·y·φ (times φ̄·invh later), for swish swish'(x).
template <typename T, int NORM>
__device__ __forceinline__ void wide_feature(const Math<T>& M, const LayerConst& lc, int g, T x, T& feat, T& pull,
                                             T& dnorm) {
    const T n = normalize<NORM, T>(M, lc.norm, x);
    dnorm = dnormalize<NORM, T>(lc.norm, n);
    if (g < lc.G) {
        const T y = (n - (T)lc.grid[g]) * (T)lc.invh;
        const T phi = M.exp_neg(-(y * y));
        feat = phi;
        pull = T(-2) * y * phi;   // basis_pull(BASIS_RBF, ·, y, φ, ·, 1)
    } else {
        T om, d;
        swish_and_grad<T>(M, x, om, d);
        feat = om;
        pull = d;
    }
}

template <typename T, int NORM>
struct WideModel {
    const Math<T>& M;
    const LayerConst* lcl;   // [2] (LDS)
    const T* ps;             // parameters (LDS)
    T* sx;                   // LDS scratch (kWideScratch T)
    int P;
    bool act;
    int64_t idx, n;
    static constexpr int kX = 0, kYb = 16, kH = 32, kHb = 48, kY = 64, kCb2 = 80, kV2 = kCb2 + 4 * kWideF2,
                         kCb1 = kV2 + kWideF2, kV1 = kCb1 + 16 * kWideF1, kEnd = kV1 + kWideF1;

    // layer 1 row r, lane c: its feature of the inputs in sx[kX..]; returns the row sum h_r (all lanes)
    __device__ T layer1(int r, int c, T& feat, T& pull, T& dnorm, T& coef) const {
        const LayerConst& L1 = lcl[0];
        const int per = L1.G + 1, H = L1.O;
        const bool on = r < H && c < L1.I * per;
        const int i = on ? c / per : 0, g = on ? c % per : 0;
        wide_feature<T, NORM>(M, L1, g, sx[kX + i], feat, pull, dnorm);
        coef = on ? (g < L1.G ? ps[L1.p_off + r + H * (g + L1.G * i)] : ps[L1.w_off + r + H * i]) : T(0);
        return row16_sum(coef * feat);
    }
    __device__ T rhs(T y) {
        const LayerConst &L1 = lcl[0], &L2 = lcl[1];
        const int t = threadIdx.x, lane = t & (kWave - 1), r = t / kWideF1, c = t & (kWideF1 - 1), w = t / kWave;
        if (act) sx[kX + idx] = y;
        __syncthreads();
        T f1, p1, d1, k1;
        const T h = layer1(r, c, f1, p1, d1, k1);
        if (c == 0 && r < L1.O) sx[kH + r] = h;
        __syncthreads();
        const int per = L2.G + 1, O = L2.O;
        const bool on = w < O && lane < L2.I * per;
        const int i = on ? lane / per : 0, g = on ? lane % per : 0;
        T f2, p2, d2;
        wide_feature<T, NORM>(M, L2, g, sx[kH + i], f2, p2, d2);
        const T coef = on ? (g < L2.G ? ps[L2.p_off + w + O * (g + L2.G * i)] : ps[L2.w_off + w + O * i]) : T(0);
        const T yo = wave_sum(coef * f2);
        if (lane == 0 && w < O) sx[kY + w] = yo;
        __syncthreads();
        return act ? sx[kY + idx] : T(0);
    }
    __device__ T vjp(T y, T ls, T* __restrict__ km) {
        const LayerConst &L1 = lcl[0], &L2 = lcl[1];
        const int t = threadIdx.x, lane = t & (kWave - 1), r = t / kWideF1, c = t & (kWideF1 - 1), w = t / kWave;
        if (act) {
            sx[kX + idx] = y;
            sx[kYb + idx] = ls;
        }
        __syncthreads();
        // layer 1 forward: h_r, this lane's feature kept for its cotangent and the pullback
        T f1, p1, d1, k1;
        const T h = layer1(r, c, f1, p1, d1, k1);
        if (c == 0 && r < L1.O) sx[kH + r] = h;
        __syncthreads();
        // layer 2: wave o lane c: dC2 / dW2 = ȳ_o·feature, and the feature's share of φ̄ = C2ᵀȳ
        const int per2 = L2.G + 1, O = L2.O, H = L2.I;
        {
            const bool on = w < O && lane < H * per2;
            const int i = on ? lane / per2 : 0, g = on ? lane % per2 : 0;
            T f2, p2, d2;
            wide_feature<T, NORM>(M, L2, g, sx[kH + i], f2, p2, d2);
            if (on) {
                const T yb = sx[kYb + w];
                const int64_t q = g < L2.G ? L2.p_off + w + O * (g + L2.G * i) : L2.w_off + w + O * i;
                km[q] = yb * f2;
                sx[kCb2 + w * kWideF2 + lane] = ps[q] * yb;
            }
            __syncthreads();
            // φ̄ of feature `lane` (Σ_o in order) and its rrule term: basis z̄·invh, swish swish'·φ̄
            if (t < H * per2) {   // (waves >= O left their rows at zero: adding them is exact)
                T pb = sx[kCb2 + t];
#pragma unroll
                for (int o = 1; o < kChainBlock / kWave; ++o) pb = pb + sx[kCb2 + o * kWideF2 + t];
                sx[kV2 + t] = g < L2.G ? p2 * pb * (T)L2.invh : p2 * pb;
                if (g == 0) sx[kHb + i] = d2;   // N'(h_i) (every basis lane of input i holds it)
            }
            __syncthreads();
            // h̄_i = N'(h_i)·Σ_g z̄_g·invh + swish'(h_i)·φ̄_sw
            if (t < H) {
                T sb = T(0);
#pragma unroll
                for (int gg = 0; gg < kWideF1; ++gg)
                    if (gg < L2.G) sb = sb + sx[kV2 + t * per2 + gg];
                sx[kHb + t] = sx[kHb + t] * sb + sx[kV2 + t * per2 + L2.G];
            }
            __syncthreads();
        }
        // layer 1 backward: row r lane c: dC1 / dW1 = h̄_r·feature, and its share of φ̄ = C1ᵀh̄
        const int per1 = L1.G + 1, I = L1.I;
        {
            const bool on = r < H && c < I * per1;
            if (on) {
                const int i = c / per1, g = c % per1;
                const T hb = sx[kHb + r];
                const int64_t q = g < L1.G ? L1.p_off + r + H * (g + L1.G * i) : L1.w_off + r + H * i;
                km[q] = hb * f1;
                sx[kCb1 + r * kWideF1 + c] = k1 * hb;
            }
            __syncthreads();
            if (t < I * per1) {   // (rows >= H left their entries at zero: adding them is exact)
                const int g = t % per1;
                T pb = sx[kCb1 + t];
#pragma unroll
                for (int rr = 1; rr < kChainBlock / kWideF1; ++rr) pb = pb + sx[kCb1 + rr * kWideF1 + t];
                sx[kV1 + t] = g < L1.G ? p1 * pb * (T)L1.invh : p1 * pb;
            }
            __syncthreads();
        }
        T xb = T(0);
        if (act) {   // x̄_i = N'(x_i)·Σ_g z̄_g·invh + swish'(x_i)·φ̄_sw  (thread i = input i)
            T sb = T(0);
#pragma unroll
            for (int gg = 0; gg < kWideF1; ++gg)
                if (gg < L1.G) sb = sb + sx[kV1 + idx * per1 + gg];
            // N'(x_i): lane c = i·per1 of row 0 evaluated it; recompute (one normalizer) rather than gather
            const T nn = normalize<NORM, T>(M, L1.norm, y);
            xb = dnormalize<NORM, T>(L1.norm, nn) * sb + sx[kV1 + idx * per1 + L1.G];
        }
        __syncthreads();   // (sx and km complete before the next stage / the caller's reads)
        return xb;
    }
};

// The adjoint of one trajectory of a two-layer chain over the whole workgroup (WideModel): the forward's dense
// output is staged in LDS too (a single trajectory's is a few KB).
template <typename T, int NORM>
__global__ void __launch_bounds__(kChainBlock)
kd_chain_adjoint_wide_kernel(const LayerConst* __restrict__ lcs, const T* __restrict__ p, int P, ChainAdjointArgs a,
                             int stage_rec) {
    extern __shared__ __attribute__((aligned(16))) unsigned char cw_raw[];
    LayerConst* lcl = reinterpret_cast<LayerConst*>(cw_raw);
    T* ps = reinterpret_cast<T*>(cw_raw + 2 * sizeof(LayerConst));
    T* sx = ps + P;                                  // WideModel scratch
    T* mu = sx + WideModel<T, NORM>::kEnd;           // [2][P]
    T* km = mu + 2 * (size_t)P;                      // [7][P]
    double* tsl = reinterpret_cast<double*>(km + 7 * (size_t)P);
    double* dtsl = tsl + a.nsteps;
    {
        const int nw = 2 * (int)(sizeof(LayerConst) / sizeof(int32_t));
        const int32_t* src = reinterpret_cast<const int32_t*>(lcs);
        int32_t* dst = reinterpret_cast<int32_t*>(cw_raw);
        stage_chain_consts(dst, src, nw, ps, p, P);
        for (int i = threadIdx.x; i < WideModel<T, NORM>::kEnd + 9 * P; i += blockDim.x) sx[i] = T(0);
        for (int64_t i = threadIdx.x; i < a.nsteps; i += blockDim.x) {
            tsl[i] = a.ts[i];
            dtsl[i] = a.dts[i];
        }
    }
    KAN_EXP_TABLE_LDS(tab);
    __shared__ double red[kChainBlock / kWave];
    const Math<T> M{tab};
    const int N = lcl[0].I;
    T* recl = nullptr;
    if (stage_rec) {
        recl = reinterpret_cast<T*>(dtsl + a.nsteps);
        onewg_stage_rec<T>(recl, a, N);
    }
    WideModel<T, NORM> m{M, lcl, ps, sx, P, (int)threadIdx.x < N, (int64_t)threadIdx.x, (int64_t)N};
    onewg_adjoint<T>(m, a, mu, km, tsl, dtsl, red, recl);
}

// One trajectory of the Lotka-Volterra chain [2 -> 10 -> 2] (G = 5, base activations; LV_driver_KANODE.jl:
// 139-143) on ONE wave: no barriers at all.  A lane evaluates one basis feature of a layer (the reference formula,
// utils.jl:8-13, as WideModel): layer 1's 12 features of (x_0, x_1) on lanes 0..11, layer 2's 60 features of
// (h_0..h_9) on lanes 0..59; every cross-lane value is a readlane (uniform) or a ds_bpermute.  Each lane keeps
// the layer coefficients it multiplies in registers for the whole adjoint (C1 row r on lane r, C1 column c on
// lane c, C2 column c on lane c).  kμ: the parameter cotangents go straight to km (one product each).
template <typename T>
__device__ __forceinline__ T lane_read(T v, int l) {   // v of lane l (l uniform)
    if constexpr (sizeof(T) == 8) {
        const long long x = __double_as_longlong((double)v);
        const int lo = __builtin_amdgcn_readlane((int)x, l), hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
        return (T)__longlong_as_double(((long long)hi << 32) | (unsigned)lo);
    } else {
        return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
    }
}
template <typename T>
__device__ __forceinline__ T wave_sum_rows(T v) {   // Σ over the wave (all lanes): DPP row sums, then the rows
    v = row16_sum(v);
    return (lane_read(v, 0) + lane_read(v, 16)) + (lane_read(v, 32) + lane_read(v, 48));
}
struct LvWaveShape {
    static constexpr int I = 2, H = 10, O = 2, G = 5, per = G + 1, F1 = I * per, F2 = H * per;
};
// LDSC: the coefficients are read from the LDS parameters at each use instead of held in registers (the
// stage-parallel adjoint, whose waves have half the register file each)
template <typename T, int NORM, bool LDSC = false>
struct LvWaveModel {
    using S = LvWaveShape;
    const Math<T>& M;
    const LayerConst* lcl;   // [2] (LDS)
    int P;
    bool act;
    int64_t idx, n;
    int lane;
    const T* ps;                     // the parameters (LDS)
    T c1r[LDSC ? 1 : S::F1];   // lane r < H: C1[r][c], c < F1 (feature c = input c / per, knot c % per)
    T c1c[LDSC ? 1 : S::H];    // lane c < F1: C1[r][c], r < H
    T c2c[LDSC ? 1 : S::O];    // lane c < F2: C2[o][c]
    __device__ T C1r(int c) const {
        if constexpr (LDSC) return lane < S::H ? ps[q1(lcl[0], lane, c)] : T(0);
        else return c1r[c];
    }
    __device__ T C1c(int r) const {
        if constexpr (LDSC) return lane < S::F1 ? ps[q1(lcl[0], r, lane)] : T(0);
        else return c1c[r];
    }
    __device__ T C2c(int o) const {
        if constexpr (LDSC) return lane < S::F2 ? ps[q2(lcl[1], o, lane)] : T(0);
        else return c2c[o];
    }

    __device__ static int64_t q1(const LayerConst& L, int r, int c) {
        const int i = c / S::per, g = c % S::per;
        return g < S::G ? L.p_off + r + S::H * (g + S::G * i) : L.w_off + r + S::H * i;
    }
    __device__ static int64_t q2(const LayerConst& L, int o, int c) {
        const int i = c / S::per, g = c % S::per;
        return g < S::G ? L.p_off + o + S::O * (g + S::G * i) : L.w_off + o + S::O * i;
    }
    __device__ LvWaveModel(const Math<T>& M_, const LayerConst* lcl_, const T* ps_, int P_)
        : M(M_), lcl(lcl_), P(P_), act((int)(threadIdx.x & (kWave - 1)) < S::I), idx(threadIdx.x & (kWave - 1)),
          n(S::I), lane(threadIdx.x & (kWave - 1)), ps(ps_) {
        if constexpr (!LDSC) {
            const LayerConst &L1 = lcl[0], &L2 = lcl[1];
#pragma unroll
            for (int c = 0; c < S::F1; ++c) c1r[c] = lane < S::H ? ps[q1(L1, lane, c)] : T(0);
#pragma unroll
            for (int r = 0; r < S::H; ++r) c1c[r] = lane < S::F1 ? ps[q1(L1, r, lane)] : T(0);
#pragma unroll
            for (int o = 0; o < S::O; ++o) c2c[o] = lane < S::F2 ? ps[q2(L2, o, lane)] : T(0);
        }
    }
    // layer 1: this lane's feature of (x_0, x_1) (lanes < F1) and h_r on lane r < H
    __device__ T layer1(T y, T& f1, T& p1, T& d1) const {
        const T x0 = lane_read(y, 0), x1 = lane_read(y, 1);
        const int c = lane < S::F1 ? lane : 0;
        wide_feature<T, NORM>(M, lcl[0], c % S::per, c / S::per == 0 ? x0 : x1, f1, p1, d1);
        T h = T(0);
#pragma unroll
        for (int k = 0; k < S::F1; ++k) h = kfma<T>(C1r(k), lane_read(f1, k), h);
        return h;
    }
    // layer 2: this lane's feature of h_{lane / per} (lanes < F2)
    __device__ void layer2(T h, T& f2, T& p2, T& d2) const {
        const int c = lane < S::F2 ? lane : 0;
        const T hi = __shfl(h, c / S::per, kWave);
        wide_feature<T, NORM>(M, lcl[1], c % S::per, hi, f2, p2, d2);
        if (lane >= S::F2) f2 = T(0);
    }
    __device__ T rhs(T y) {
        T f1, p1, d1, f2, p2, d2;
        const T h = layer1(y, f1, p1, d1);
        layer2(h, f2, p2, d2);
        const T y0 = wave_sum_rows(C2c(0) * f2), y1 = wave_sum_rows(C2c(1) * f2);
        return lane == 0 ? y0 : (lane == 1 ? y1 : T(0));
    }
    __device__ T vjp(T y, T ls, T* __restrict__ km) {
        const LayerConst &L1 = lcl[0], &L2 = lcl[1];
        T f1, p1, d1, f2, p2, d2;
        const T h = layer1(y, f1, p1, d1);
        layer2(h, f2, p2, d2);
        // layer 2: dC2[o][c] = ȳ_o·f2_c, φ̄2_c = Σ_o C2[o][c]·ȳ_o, z̄ = rrule factor·φ̄2
        const T yb0 = lane_read(ls, 0), yb1 = lane_read(ls, 1);
        const int g2 = lane % S::per;
        T z2 = T(0);
        if (lane < S::F2) {
            km[q2(L2, 0, lane)] = yb0 * f2;
            km[q2(L2, 1, lane)] = yb1 * f2;
            const T pb = C2c(0) * yb0 + C2c(1) * yb1;
            z2 = g2 < S::G ? p2 * pb * (T)L2.invh : p2 * pb;
        }
        // h̄_r = N'(h_r)·Σ_g z̄_(r,g) + z̄_(r,swish) on lane r < H (the group's lanes per·r .. per·r + G)
        const int r = lane < S::H ? lane : 0;
        T sb = T(0);
#pragma unroll
        for (int g = 0; g < S::G; ++g) sb = sb + __shfl(z2, S::per * r + g, kWave);
        const T zsw = __shfl(z2, S::per * r + S::G, kWave);
        const T dn = __shfl(d2, S::per * r, kWave);
        const T hb = lane < S::H ? dn * sb + zsw : T(0);
        // layer 1: dC1[r][c] = h̄_r·f1_c, φ̄1_c = Σ_r C1[r][c]·h̄_r on lane c < F1
        const int g1 = lane % S::per;
        T pb1 = T(0);
#pragma unroll
        for (int rr = 0; rr < S::H; ++rr) {
            const T hbr = lane_read(hb, rr);
            if (lane < S::F1) km[q1(L1, rr, lane)] = hbr * f1;
            pb1 = kfma<T>(C1c(rr), hbr, pb1);
        }
        const T z1 = lane < S::F1 ? (g1 < S::G ? p1 * pb1 * (T)L1.invh : p1 * pb1) : T(0);
        // x̄_i = N'(x_i)·Σ_g z̄_(i,g) + z̄_(i,swish) on lane i < I
        const int i = lane < S::I ? lane : 0;
        T sx = T(0);
#pragma unroll
        for (int g = 0; g < S::G; ++g) sx = sx + __shfl(z1, S::per * i + g, kWave);
        const T xsw = __shfl(z1, S::per * i + S::G, kWave);
        const T dx = __shfl(d1, S::per * i, kWave);
        __syncthreads();   // (one wave: km complete before the driver reads it)
        return act ? dx * sx + xsw : T(0);
    }
    // vjp at λs = e_0 and e_1 at once (one forward, the two pullbacks interleaved): the rows G_0, G_1 of ∂f/∂p
    // into g0, g1 (no barrier: the caller's) and J_0, J_1 of ∂f/∂u on lanes < I.  Each product is vjp's with
    // λs = e_k (its x·1 and + x·0 are exact).
    __device__ void vjp2(T y, T* __restrict__ g0, T* __restrict__ g1, T& j0, T& j1) const {
        const LayerConst &L1 = lcl[0], &L2 = lcl[1];
        T f1, p1, d1, f2, p2, d2;
        const T h = layer1(y, f1, p1, d1);
        layer2(h, f2, p2, d2);
        const int g2 = lane % S::per;
        T za = T(0), zb = T(0);
        if (lane < S::F2) {
            g0[q2(L2, 0, lane)] = f2;
            g0[q2(L2, 1, lane)] = T(0);
            g1[q2(L2, 0, lane)] = T(0);
            g1[q2(L2, 1, lane)] = f2;
            const T ca = C2c(0), cb = C2c(1);
            za = g2 < S::G ? p2 * ca * (T)L2.invh : p2 * ca;
            zb = g2 < S::G ? p2 * cb * (T)L2.invh : p2 * cb;
        }
        const int r = lane < S::H ? lane : 0;
        T sa = T(0), sb = T(0);
#pragma unroll
        for (int g = 0; g < S::G; ++g) {
            sa = sa + __shfl(za, S::per * r + g, kWave);
            sb = sb + __shfl(zb, S::per * r + g, kWave);
        }
        const T swa = __shfl(za, S::per * r + S::G, kWave), swb = __shfl(zb, S::per * r + S::G, kWave);
        const T dn = __shfl(d2, S::per * r, kWave);
        const T ha = lane < S::H ? dn * sa + swa : T(0), hb = lane < S::H ? dn * sb + swb : T(0);
        const int g1i = lane % S::per;
        T pa = T(0), pb = T(0);
#pragma unroll
        for (int rr = 0; rr < S::H; ++rr) {
            const T hra = lane_read(ha, rr), hrb = lane_read(hb, rr);
            if (lane < S::F1) {
                g0[q1(L1, rr, lane)] = hra * f1;
                g1[q1(L1, rr, lane)] = hrb * f1;
            }
            const T cc = C1c(rr);
            pa = kfma<T>(cc, hra, pa);
            pb = kfma<T>(cc, hrb, pb);
        }
        const T z1a = lane < S::F1 ? (g1i < S::G ? p1 * pa * (T)L1.invh : p1 * pa) : T(0);
        const T z1b = lane < S::F1 ? (g1i < S::G ? p1 * pb * (T)L1.invh : p1 * pb) : T(0);
        const int i = lane < S::I ? lane : 0;
        T xa = T(0), xb = T(0);
#pragma unroll
        for (int g = 0; g < S::G; ++g) {
            xa = xa + __shfl(z1a, S::per * i + g, kWave);
            xb = xb + __shfl(z1b, S::per * i + g, kWave);
        }
        const T xwa = __shfl(z1a, S::per * i + S::G, kWave), xwb = __shfl(z1b, S::per * i + S::G, kWave);
        const T dx = __shfl(d1, S::per * i, kWave);
        j0 = act ? dx * xa + xwa : T(0);
        j1 = act ? dx * xb + xwb : T(0);
    }
};

template <typename T, int NORM>
__global__ void __launch_bounds__(kWave)
kd_chain_adjoint_lvwave_kernel(const LayerConst* __restrict__ lcs, const T* __restrict__ p, int P, ChainAdjointArgs a,
                               int stage_rec) {
    extern __shared__ __attribute__((aligned(16))) unsigned char cv_raw[];
    LayerConst* lcl = reinterpret_cast<LayerConst*>(cv_raw);
    T* ps = reinterpret_cast<T*>(cv_raw + 2 * sizeof(LayerConst));
    T* mu = ps + P;                                  // [2][P]
    T* km = mu + 2 * (size_t)P;                      // [7][P]
    double* tsl = reinterpret_cast<double*>(km + 7 * (size_t)P);
    double* dtsl = tsl + a.nsteps;
    {
        const int nw = 2 * (int)(sizeof(LayerConst) / sizeof(int32_t));
        const int32_t* src = reinterpret_cast<const int32_t*>(lcs);
        int32_t* dst = reinterpret_cast<int32_t*>(cv_raw);
        stage_chain_consts(dst, src, nw, ps, p, P);
        for (int i = threadIdx.x; i < 9 * P; i += blockDim.x) mu[i] = T(0);
        for (int64_t i = threadIdx.x; i < a.nsteps; i += blockDim.x) {
            tsl[i] = a.ts[i];
            dtsl[i] = a.dts[i];
        }
    }
    KAN_EXP_TABLE_LDS(tab);
    __shared__ double red[1];
    const Math<T> M{tab};
    T* recl = nullptr;
    if (stage_rec) {
        recl = reinterpret_cast<T*>(dtsl + a.nsteps);
        onewg_stage_rec<T>(recl, a, LvWaveShape::I);
    }
    LvWaveModel<T, NORM> m(M, lcl, ps, P);
    onewg_adjoint<T>(m, a, mu, km, tsl, dtsl, red, recl);
}

// One Lotka-Volterra trajectory's adjoint with its stage evaluations in parallel (fp64; the idea of
// kan_small.hip's fk_small_adjoint_sp_kernel).  The pullback is linear in the stage input: kλ = λsᵀJ(u),
// kμ = λsᵀG(u), with J = ∂f/∂u (2 × 2) and G = ∂f/∂p (2 × 240) at the stage's point u(t) of the forward dense
// output, which does not depend on λ.  So the rows of J and G at the six stage points of a step are evaluated
// at once, wave i taking stage i (LvWaveModel::vjp2: both rows, λs = e_0 and e_1), into LDS; the stage
// recurrence is then two-vector algebra, and lane l keeps the μ entries l, l + 64, .. (no sums over lanes but
// the error norm's).  Every wave runs the recurrence and the step control on the same LDS values.  FSAL: the
// accepted step's last point is the next step's first (its rows carry over; after a saveat jump kλ_1 is
// re-formed from them).  Same step control as onewg_adjoint; rounding-level differences from its order.
#ifndef KAN_LV_SP
#define KAN_LV_SP 1
#endif
constexpr int kLvSpWaves = 6;   // the stage waves; one more takes the controller's qold^β2 during the stage phase
constexpr int kLvP = LvWaveShape::F1 * LvWaveShape::H + LvWaveShape::F2 * LvWaveShape::O;   // 240
constexpr int kLvPL = (kLvP + kWave - 1) / kWave;                                               // μ entries per lane
template <int NORM>
__global__ void __launch_bounds__((kLvSpWaves + 1) * kWave)
kd_chain_adjoint_lvsp_kernel(const LayerConst* __restrict__ lcs, const double* __restrict__ p, ChainAdjointArgs a,
                             int stage_rec) {
    using K = Tsit5Tab;
#define KAN_LVSP_POW(x, y) KAN_ONEWG_POW(x, y)
    constexpr int N = LvWaveShape::I, P = kLvP, RW = P + N;   // a row: G_k (P), then J_k (N)
    extern __shared__ __attribute__((aligned(16))) unsigned char cv_raw[];
    LayerConst* lcl = reinterpret_cast<LayerConst*>(cv_raw);
    double* ps = reinterpret_cast<double*>(cv_raw + 2 * sizeof(LayerConst));
    double* tsl = ps + P;
    double* dtsl = tsl + a.nsteps;
    __shared__ double jst[6][N][RW];   // this step's stage points: row k of [G | J] at stage i
    __shared__ double jfs[2][N][RW];   // the step's first point (FSAL), by parity
    __shared__ double pqs;             // qold^β2 of this step (the last wave)
    // the tableau in LDS (a_ij [6][6], b̃ [7], the interpolant's r_qm [7][4]): as compile-time literals the 71
    // fp64 constants were materialised once and held (then spilled) across the step loop; LDS reads of a
    // uniform address are broadcasts, re-issued after each barrier
    __shared__ double kt[71];
    for (int q = threadIdx.x; q < 71; q += blockDim.x)
        kt[q] = q < 36 ? K::TA[q / 6][q % 6] : (q < 43 ? K::BT[q - 36] : K::RI[(q - 43) / 4][(q - 43) % 4]);
    {
        const int nw = 2 * (int)(sizeof(LayerConst) / sizeof(int32_t));
        const int32_t* src = reinterpret_cast<const int32_t*>(lcs);
        int32_t* dst = reinterpret_cast<int32_t*>(cv_raw);
        stage_chain_consts(dst, src, nw, ps, p, P);
        for (int64_t i = threadIdx.x; i < a.nsteps; i += blockDim.x) {
            tsl[i] = a.ts[i];
            dtsl[i] = a.dts[i];
        }
    }
    KAN_EXP_TABLE_LDS(tab);
    const Math<double> M{tab};
    const double* rec = reinterpret_cast<const double*>(a.rec);
    const double* rk1 = reinterpret_cast<const double*>(a.k1_0);
    if (stage_rec) {
        double* recl = dtsl + a.nsteps;
        onewg_stage_rec<double>(recl, a, N);
        rec = recl;
        rk1 = recl + a.nsteps * 7 * N;
    }
    LvWaveModel<double, NORM, true> m(M, lcl, ps, P);
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const double* dl = reinterpret_cast<const double*>(a.dl_du);
    const double t0 = a.t0, tf = a.tf, TT = tf - t0;
    const double ntot = (double)(N + P);
    int64_t cur = a.nsteps - 1;   // this wave's forward interval
    auto interp = [&](double tau) -> double {   // u(tf - τ) on lanes < N (onewg_adjoint's adj)
        const double t = tf - tau;
        while (cur > 0 && tsl[cur] > t) --cur;
        while (cur + 1 < a.nsteps && tsl[cur + 1] <= t) ++cur;
        const double dti = dtsl[cur];
        const double th = ::fmin(1.0, ::fmax(0.0, (t - tsl[cur]) / dti));
        const int c = lane < N ? lane : 0;
        const double* __restrict__ r = rec + cur * 7 * N;
        const double* __restrict__ k1 = cur == 0 ? rk1 : rec + (cur - 1) * 7 * N + 6 * N;
        double kv[7];
        kv[0] = k1[c];
#pragma unroll
        for (int q = 1; q < 7; ++q) kv[q] = r[q * N + c];
        double y = r[c];
#pragma unroll
        for (int q = 0; q < 7; ++q) {
            const double* ri = kt + 43 + 4 * q;
            const double b = th * (ri[0] + th * (ri[1] + th * (ri[2] + th * ri[3])));
            y = ::fma(b * dti, kv[q], y);
        }
        return lane < N ? y : 0.0;
    };
    auto rows = [&](double tau, double (*R)[RW]) {   // both rows of [G | J] at τ into R[0], R[1]
        // (the lane made opaque per call: the model's lane-derived indices are then recomputed here, a few
        // integer ops, instead of hoisted out of the step loop and spilled)
        int ln = lane;
        asm volatile("" : "+v"(ln));
        m.lane = ln;
        const double y = interp(tau);
        double j0, j1;
        m.vjp2(y, R[0], R[1], j0, j1);
        if (lane < N) {
            R[0][P + lane] = j0;
            R[1][P + lane] = j1;
        }
    };
    auto jump = [&](int gidx, double& l0, double& l1) {   // λ += Σ ∂L/∂u rows (in order)
        for (int32_t q = a.joff[gidx]; q < a.joff[gidx + 1]; ++q) {
            l0 = l0 + dl[(int64_t)a.jrows[q] * N];
            l1 = l1 + dl[(int64_t)a.jrows[q] * N + 1];
        }
    };
    // kλ = λsᵀJ and this lane's kμ entries λsᵀG from rows R[0], R[1]
    auto kl_of = [&](const double (*R)[RW], double s0, double s1, double& k0, double& k1) {
        k0 = ::fma(s1, R[1][P], s0 * R[0][P]);
        k1 = ::fma(s1, R[1][P + 1], s0 * R[0][P + 1]);
    };
    auto km_of = [&](const double (*R)[RW], double s0, double s1, int r) -> double {
        const int q = lane + kWave * r;
        return q < P ? ::fma(s1, R[1][q], s0 * R[0][q]) : 0.0;
    };
    double l0 = 0.0, l1 = 0.0;
    if (dl) jump(0, l0, l1);
    int fp = 0;
    if (w < kLvSpWaves) rows(0.0, w == 0 ? jfs[0] : jst[w]);   // (waves > 0: a scratch copy)
    __syncthreads();
    double k10, k11;   // kλ_1
    kl_of(jfs[0], l0, l1, k10, k11);
    int64_t nf = 1;
    double mu[kLvPL];
#pragma unroll
    for (int r = 0; r < kLvPL; ++r) mu[r] = 0.0;
    double h = a.dt;
    if (a.adaptive && !(a.dt > 0)) {   // Hairer-Wanner on [λ; μ] (μ = 0)
        double sm1 = 0.0;
#pragma unroll
        for (int r = 0; r < kLvPL; ++r) {
            const double v = km_of(jfs[0], l0, l1, r) / a.abstol;
            sm1 = ::fma(v, v, sm1);
        }
        const double sk0 = ::fma(a.reltol, kabs(l0), a.abstol), sk1 = ::fma(a.reltol, kabs(l1), a.abstol);
        const double d0 = ::sqrt(((l0 / sk0) * (l0 / sk0) + (l1 / sk1) * (l1 / sk1)) / ntot);
        const double d1 = ::sqrt(((k10 / sk0) * (k10 / sk0) + (k11 / sk1) * (k11 / sk1) + wave_sum(sm1)) / ntot);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        h0 = ::fmin(h0, TT);
        if (w < kLvSpWaves) rows(h0, jst[w]);
        __syncthreads();
        const double s0 = ::fma(h0, k10, l0), s1 = ::fma(h0, k11, l1);
        double kh0, kh1;
        kl_of(jst[0], s0, s1, kh0, kh1);
        ++nf;
        double sm2 = 0.0;
#pragma unroll
        for (int r = 0; r < kLvPL; ++r) {
            const double v = (km_of(jst[0], s0, s1, r) - km_of(jfs[0], l0, l1, r)) / a.abstol;
            sm2 = ::fma(v, v, sm2);
        }
        const double e0 = (kh0 - k10) / sk0, e1 = (kh1 - k11) / sk1;
        const double d2 = ::sqrt((e0 * e0 + e1 * e1 + wave_sum(sm2)) / ntot) / h0;
        const double mx = ::fmax(d1, d2);
        const double h1 = mx <= 1e-15 ? ::fmax(1e-6, h0 * 1e-3) : ::pow(0.01 / mx, 1.0 / 5.0);
        h = ::fmin(::fmin(100 * h0, h1), TT);
        __syncthreads();   // jst is rewritten by the first step
    }
    double qold = a.qoldinit, tau = 0.0;
    int64_t si = 0, naccept = 0, nreject = 0, it = 0, status = 0;
    double wc = 1.0;   // c of this wave's stage (selects: no runtime index into the tableau)
#pragma unroll
    for (int i = 0; i < 5; ++i) wc = w == i ? K::TC[i] : wc;
    for (; it < a.maxiters; ++it) {
        if (tau >= TT - 1e-14 * ::fmax(1.0, TT)) break;
        h = ::fmin(h, a.stops[si] - tau);
#ifndef KAN_LVSP_NOPH1   // timing experiment only: the stage points left at their first values (wrong results)
        if (w < kLvSpWaves) rows(w == 5 ? tau + h : tau + wc * h, jst[w]);
#endif
        if (w == kLvSpWaves && lane == 0 && a.adaptive) pqs = KAN_LVSP_POW(qold, a.beta2);
        __syncthreads();
        double cA[kLvPL], cE[kLvPL];
#pragma unroll
        for (int r = 0; r < kLvPL; ++r) {
            const double m1 = km_of(jfs[fp], l0, l1, r);
            cA[r] = (h * kt[30]) * m1;
            cE[r] = (h * kt[36]) * m1;
        }
        double k0[7], k1[7];
        k0[0] = k10;
        k1[0] = k11;
        double s0 = l0, s1 = l1;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            s0 = l0;
            s1 = l1;
#pragma unroll
            for (int q = 0; q <= i; ++q) {
                const double c = h * kt[6 * i + q];
                s0 = ::fma(c, k0[q], s0);
                s1 = ::fma(c, k1[q], s1);
            }
            kl_of(jst[i], s0, s1, k0[i + 1], k1[i + 1]);
#pragma unroll
            for (int r = 0; r < kLvPL; ++r) {
                const double mm = km_of(jst[i], s0, s1, r);
                if (i < 5) cA[r] = ::fma(h * kt[30 + i + 1], mm, cA[r]);
                cE[r] = ::fma(h * kt[36 + i + 1], mm, cE[r]);
            }
        }
        nf += 6;
        double hnew = h;
        if (a.adaptive) {
            double ev0 = 0.0, ev1 = 0.0;
#pragma unroll
            for (int r = 0; r < 6; ++r) {
                ev0 = ::fma(h * kt[36 + r], k0[r], ev0);
                ev1 = ::fma(h * kt[36 + r], k1[r], ev1);
            }
            const double e0 = ::fma(h * kt[42], k0[6], ev0), e1 = ::fma(h * kt[42], k1[6], ev1);
            const double sk0 = ::fma(a.reltol, ::fmax(kabs(l0), kabs(s0)), a.abstol);
            const double sk1 = ::fma(a.reltol, ::fmax(kabs(l1), kabs(s1)), a.abstol);
            double sm = 0.0;
#pragma unroll
            for (int r = 0; r < kLvPL; ++r) {
                const double sk = ::fma(a.reltol, ::fmax(kabs(mu[r]), kabs(mu[r] + cA[r])), a.abstol);
                sm = ::fma(cE[r] / sk, cE[r] / sk, sm);
            }
            const double eest = ::sqrt(((e0 / sk0) * (e0 / sk0) + (e1 / sk1) * (e1 / sk1) + wave_sum(sm)) / ntot);
            const double q11 = eest > 0 ? KAN_LVSP_POW(eest, a.beta1) : 0.0;
            if (eest > 1.0 && h > a.dtmin) {
                ++nreject;
                h = h / ::fmin(1.0 / a.qmin, q11 / a.gamma);
                __syncthreads();   // every wave is done with jst
                continue;
            }
            double q = q11 / pqs;   // (= pow(qold, β2); read after the stage phase's barrier)
            q = ::fmax(1.0 / a.qmax, ::fmin(1.0 / a.qmin, q / a.gamma));
            if (1.0 <= q && q <= 1.0) q = 1.0;
            hnew = q > 0 ? h / q : h * a.qmax;
            qold = ::fmax(eest, a.qoldinit);
        }
        // the accepted step's last point becomes the next step's first (wave 5 wrote it)
        if (w == 5)
            for (int q = lane; q < RW; q += kWave) {
                jfs[fp ^ 1][0][q] = jst[5][0][q];
                jfs[fp ^ 1][1][q] = jst[5][1][q];
            }
        __syncthreads();   // every wave is done with jst, and jfs[fp ^ 1] is complete
        fp ^= 1;
        tau = tau + h;
        l0 = s0;
        l1 = s1;
#pragma unroll
        for (int r = 0; r < kLvPL; ++r) mu[r] = mu[r] + cA[r];
        k10 = k0[6];
        k11 = k1[6];
        if (a.hs && threadIdx.x == 0 && naccept < a.hs_cap) a.hs[naccept] = h;
        ++naccept;
        if (::fabs(tau - a.stops[si]) <= 1e-12 * ::fmax(1.0, TT)) {
            tau = a.stops[si];
            if (si + 1 < a.nstops) {
                if (dl && a.joff[si + 2] > a.joff[si + 1]) {
                    jump((int)si + 1, l0, l1);
                    kl_of(jfs[fp], l0, l1, k10, k11);   // u_modified!: kλ_1 re-formed
                    ++nf;
                }
            }
            si = si + 1 < a.nstops ? si + 1 : a.nstops - 1;
        }
        h = hnew;
    }
#undef KAN_LVSP_POW
    if (it == a.maxiters && !(tau >= TT - 1e-14 * ::fmax(1.0, TT))) status = 1;
    if (dl) jump((int)a.nstops, l0, l1);
    if (w == 0) {
        if (a.du0 && lane < N) reinterpret_cast<double*>(a.du0)[lane] = lane == 0 ? l0 : l1;
        if (a.dp) {
#pragma unroll
            for (int r = 0; r < kLvPL; ++r)
                if (lane + kWave * r < P) reinterpret_cast<double*>(a.dp)[lane + kWave * r] = mu[r];
        }
        if (lane == 0) {
            a.out[0] = naccept;
            a.out[1] = nreject;
            a.out[2] = nf;
            a.out[3] = status;
        }
    }
}

// The one-workgroup adjoint (kd_chain_adjoint_kernel): the small-chain conditions of
// launch_kd_chain_tsit5 plus nsteps <= kChainAdjointMaxSteps and the LDS budget.
template <typename T>
hipError_t launch_kd_chain_adjoint(const LayerConst* hlcs, int nl, const LayerConst* lcs, const T* p, int64_t P,
                                   int64_t B, const ChainAdjointArgs& a, hipStream_t st, bool wide) {
    if (nl < 1 || nl > kChainMaxLayers || B < 1 || B > kChainSolveMaxBatch || I_ne_O(hlcs, nl) || a.nsteps < 1 ||
        a.nsteps > kChainAdjointMaxSteps)
        return hipErrorNotSupported;
    // one Lotka-Volterra trajectory: the chain on one wave (LvWaveModel)
    if (wide && B == 1 && nl == 2 && hlcs[0].use_base && hlcs[1].use_base && hlcs[0].norm == hlcs[1].norm &&
        hlcs[0].I == LvWaveShape::I && hlcs[0].O == LvWaveShape::H && hlcs[1].I == LvWaveShape::H &&
        hlcs[1].O == LvWaveShape::O && hlcs[0].G == LvWaveShape::G && hlcs[1].G == LvWaveShape::G &&
        hlcs[0].basis == BASIS_RBF && hlcs[1].basis == BASIS_RBF &&
        (hlcs[0].norm == NORM_TANH_FAST || hlcs[0].norm == NORM_SOFTSIGN)) {
        const size_t pre = 2 * sizeof(LayerConst) + sizeof(T) * (size_t)P * 10;   // ps, μ [2], kμ [7]
        size_t lds = pre + 2 * sizeof(double) * a.nsteps;
        const size_t rec = sizeof(T) * ((size_t)a.nsteps * 7 + 1) * LvWaveShape::I;
        const int stage_rec = lds + rec <= 60 * 1024 ? 1 : 0;
        if (stage_rec) lds += rec;
        if constexpr (std::is_same<T, double>::value) {   // the stage-parallel form (kd_chain_adjoint_lvsp_kernel)
            const size_t jst = sizeof(double) * 8 * LvWaveShape::I * (kLvP + LvWaveShape::I);
            size_t lsp = 2 * sizeof(LayerConst) + sizeof(double) * (kLvP + 2 * (size_t)a.nsteps);
            const int sp_rec = lsp + rec + jst <= 140 * 1024 ? 1 : 0;
            if (sp_rec) lsp += rec;
            if (KAN_LV_SP && P == kLvP && lsp + jst <= 140 * 1024) {
                const void* fn = hlcs[0].norm == NORM_TANH_FAST
                                     ? reinterpret_cast<const void*>(&kd_chain_adjoint_lvsp_kernel<NORM_TANH_FAST>)
                                     : reinterpret_cast<const void*>(&kd_chain_adjoint_lvsp_kernel<NORM_SOFTSIGN>);
                {
                    const hipError_t e = ensure_dynamic_lds(fn, lsp);
                    if (e != hipSuccess) return e;
                }
                if (hlcs[0].norm == NORM_TANH_FAST)
                    hipLaunchKernelGGL((kd_chain_adjoint_lvsp_kernel<NORM_TANH_FAST>), dim3(1), dim3((kLvSpWaves + 1) * kWave),
                                       lsp, st, lcs, p, a, sp_rec);
                else
                    hipLaunchKernelGGL((kd_chain_adjoint_lvsp_kernel<NORM_SOFTSIGN>), dim3(1), dim3((kLvSpWaves + 1) * kWave),
                                       lsp, st, lcs, p, a, sp_rec);
                return hipGetLastError();
            }
        }
        if (pre % 8 == 0 && lds <= 60 * 1024) {
            if (hlcs[0].norm == NORM_TANH_FAST)
                hipLaunchKernelGGL((kd_chain_adjoint_lvwave_kernel<T, NORM_TANH_FAST>), dim3(1), dim3(kWave), lds, st,
                                   lcs, p, (int)P, a, stage_rec);
            else
                hipLaunchKernelGGL((kd_chain_adjoint_lvwave_kernel<T, NORM_SOFTSIGN>), dim3(1), dim3(kWave), lds, st,
                                   lcs, p, (int)P, a, stage_rec);
            return hipGetLastError();
        }
    }
    // one trajectory of a two-layer chain with base activations: the whole workgroup on it (WideModel)
    if (wide && B == 1 && nl == 2 && hlcs[0].use_base && hlcs[1].use_base && hlcs[0].norm == hlcs[1].norm &&
        hlcs[1].I == hlcs[0].O && wide_fits(WideShape{hlcs[0].I, hlcs[0].O, hlcs[1].O, hlcs[0].G, hlcs[1].G}) &&
        (hlcs[0].norm == NORM_TANH_FAST || hlcs[0].norm == NORM_SOFTSIGN)) {
        const size_t pre = 2 * sizeof(LayerConst) + sizeof(T) * ((size_t)P * 10 + WideModel<T, NORM_SOFTSIGN>::kEnd);
        size_t lds = pre + 2 * sizeof(double) * a.nsteps;
        const size_t rec = sizeof(T) * ((size_t)a.nsteps * 7 + 1) * hlcs[0].I;   // the dense output, staged
        const int stage_rec = lds + rec <= 60 * 1024 ? 1 : 0;
        if (stage_rec) lds += rec;
        if (pre % 8 == 0 && lds <= 60 * 1024) {
            if (hlcs[0].norm == NORM_TANH_FAST)
                hipLaunchKernelGGL((kd_chain_adjoint_wide_kernel<T, NORM_TANH_FAST>), dim3(1), dim3(kChainBlock), lds, st,
                                   lcs, p, (int)P, a, stage_rec);
            else
                hipLaunchKernelGGL((kd_chain_adjoint_wide_kernel<T, NORM_SOFTSIGN>), dim3(1), dim3(kChainBlock), lds, st,
                                   lcs, p, (int)P, a, stage_rec);
            return hipGetLastError();
        }
    }
    for (int l = 0; l < nl; ++l) {
        const LayerConst& h = hlcs[l];
        if (h.I > kChainDim || h.O > kChainDim || h.path != hlcs[0].path || h.norm != hlcs[0].norm)
            return hipErrorNotSupported;
        if (l > 0 && h.I != hlcs[l - 1].O) return hipErrorNotSupported;
    }
    const int threads = (int)((B * kChainDim + kWave - 1) / kWave) * kWave;
    const int NG = threads / kChainDim;
    const size_t lds = nl * sizeof(LayerConst) + (size_t)P * sizeof(T) * (1 + NG + 9) + 2 * sizeof(double) * a.nsteps + 16;
    if (lds > 60 * 1024 || (P * sizeof(T)) % 8) return hipErrorNotSupported;
    const LayerConst& h = hlcs[0];
#define KAN_CADJ_S(NORM, PATH, S)                                                                                     \
    hipLaunchKernelGGL((kd_chain_adjoint_kernel<T, NORM, PATH, S>), dim3(1), dim3(threads), lds, st, lcs, nl, p,     \
                       (int)P, B, a)
    if (h.norm == NORM_TANH_FAST && h.path == PATH_REC && chain_is_lv(hlcs, nl))
        KAN_CADJ_S(NORM_TANH_FAST, PATH_REC, ChainShapeLV);
    else if (h.norm == NORM_TANH_FAST && h.path == PATH_REC) KAN_CADJ_S(NORM_TANH_FAST, PATH_REC, ChainShapeAny);
    else if (h.path == PATH_REC_CORR) KAN_CADJ_S(NORM_RUNTIME, PATH_REC_CORR, ChainShapeAny);
    else if (h.path == PATH_REC) KAN_CADJ_S(NORM_RUNTIME, PATH_REC, ChainShapeAny);
    else KAN_CADJ_S(NORM_RUNTIME, PATH_DIRECT, ChainShapeAny);
#undef KAN_CADJ_S
    return hipGetLastError();
}

// The one-workgroup solve (kd_chain_tsit5_kernel): every layer small, one normalizer/path
// specialisation, N_in == N_out, B <= kChainSolveMaxBatch; hipErrorNotSupported otherwise.
template <typename T>
hipError_t launch_kd_chain_tsit5(const LayerConst* hlcs, int nl, const LayerConst* lcs, const T* p, int64_t P,
                                 const T* u0, int64_t B, const ChainSolveArgs& a, hipStream_t st) {
    if (nl < 1 || nl > 8 || B < 1 || B > kChainSolveMaxBatch || I_ne_O(hlcs, nl)) return hipErrorNotSupported;
    for (int l = 0; l < nl; ++l) {
        const LayerConst& h = hlcs[l];
        if (h.I > kChainDim || h.O > kChainDim || h.path != hlcs[0].path || h.norm != hlcs[0].norm)
            return hipErrorNotSupported;
        if (l > 0 && h.I != hlcs[l - 1].O) return hipErrorNotSupported;
    }
    const size_t lds = nl * sizeof(LayerConst) + (size_t)P * sizeof(T);
    if (lds > 48 * 1024) return hipErrorNotSupported;
    const int threads = (int)((B * kChainDim + kWave - 1) / kWave) * kWave;
    const LayerConst& h = hlcs[0];
#define KAN_CSOLVE_S(NORM, PATH, S)                                                                                   \
    hipLaunchKernelGGL((kd_chain_tsit5_kernel<T, NORM, PATH, S>), dim3(1), dim3(threads), lds, st, lcs, nl, p, (int)P, \
                       u0, B, a)
    if (h.norm == NORM_TANH_FAST && h.path == PATH_REC && chain_is_lv(hlcs, nl))
        KAN_CSOLVE_S(NORM_TANH_FAST, PATH_REC, ChainShapeLV);
    else if (h.norm == NORM_TANH_FAST && h.path == PATH_REC) KAN_CSOLVE_S(NORM_TANH_FAST, PATH_REC, ChainShapeAny);
    else if (h.path == PATH_REC_CORR) KAN_CSOLVE_S(NORM_RUNTIME, PATH_REC_CORR, ChainShapeAny);
    else if (h.path == PATH_REC) KAN_CSOLVE_S(NORM_RUNTIME, PATH_REC, ChainShapeAny);
    else KAN_CSOLVE_S(NORM_RUNTIME, PATH_DIRECT, ChainShapeAny);
#undef KAN_CSOLVE_S
    return hipGetLastError();
}

// One Tsit5 step of a small chain per column (kd_chain_step_kernel); err_out (with err_slab of
// slab_rows rows) receives Σ (e/sk)².  hipErrorNotSupported outside the small-chain shapes.
template <typename T>
hipError_t launch_kd_chain_step(const LayerConst* hlcs, int nl, const LayerConst* lcs, const T* p, int64_t P,
                                int64_t K, const ChainStepArgs& a, double* err_slab, int slab_rows, double* err_out,
                                hipStream_t st) {
    if (nl < 1 || nl > 8 || K > 32768 || I_ne_O(hlcs, nl)) return hipErrorNotSupported;
    for (int l = 0; l < nl; ++l) {
        const LayerConst& h = hlcs[l];
        if (h.I > kChainDim || h.O > kChainDim || h.path != hlcs[0].path || h.norm != hlcs[0].norm)
            return hipErrorNotSupported;
        if (l > 0 && h.I != hlcs[l - 1].O) return hipErrorNotSupported;
    }
    const size_t lds = nl * sizeof(LayerConst) + (size_t)P * sizeof(T);
    if (lds > 48 * 1024) return hipErrorNotSupported;
    const int g = grid_for(K * kChainDim, kChainBlock, slab_rows < kGridCap ? slab_rows : kGridCap);
    double* es = err_out ? err_slab : nullptr;
    const LayerConst& h = hlcs[0];
#define KAN_CSTEP(NORM, PATH, S)                                                                                 \
    hipLaunchKernelGGL((kd_chain_step_kernel<T, NORM, PATH, S>), dim3(g), dim3(kChainBlock), lds, st, lcs, nl, p,  \
                       (int)P, K, a, es)
    if (h.norm == NORM_TANH_FAST && h.path == PATH_REC && chain_is_lv(hlcs, nl))
        KAN_CSTEP(NORM_TANH_FAST, PATH_REC, ChainShapeLV);
    else if (h.norm == NORM_TANH_FAST && h.path == PATH_REC) KAN_CSTEP(NORM_TANH_FAST, PATH_REC, ChainShapeAny);
    else if (h.path == PATH_REC_CORR) KAN_CSTEP(NORM_RUNTIME, PATH_REC_CORR, ChainShapeAny);
    else if (h.path == PATH_REC) KAN_CSTEP(NORM_RUNTIME, PATH_REC, ChainShapeAny);
    else KAN_CSTEP(NORM_RUNTIME, PATH_DIRECT, ChainShapeAny);
#undef KAN_CSTEP
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !es) return e;
    return launch_stage_error_final(err_slab, g, err_out, st);
}

// The fused adjoint stage of a small chain (kd_chain_vjp_stage_kernel) when every layer is
// small (I, O <= 16), the layers share the normalizer/path specialisation, nl <= 4 and the
// parameter vector plus the gradient rows fit in LDS; hipErrorNotSupported otherwise.
size_t chain_vjp_step_slab_bytes(int64_t P, int64_t K, size_t esize, int grid_cap) {
    const int grid = grid_for(K, kChainVjpBlock / kChainDim, grid_cap);
    return 7 * (((size_t)grid * P * esize + 255) & ~(size_t)255) + (size_t)grid * sizeof(double) + 256;
}
bool chain_vjp_step_supported(const LayerConst* hlcs, int nl, int64_t P, size_t esize) {
    if (nl < 1 || nl > kChainMaxLayers) return false;
    for (int l = 0; l < nl; ++l) {
        const LayerConst& h = hlcs[l];
        if (h.I > kChainDim || h.O > kChainDim || h.path != hlcs[0].path || h.norm != hlcs[0].norm) return false;
        if (l > 0 && h.I != hlcs[l - 1].O) return false;
    }
    if (hlcs[nl - 1].O != hlcs[0].I) return false;
    return nl * sizeof(LayerConst) + (size_t)P * esize * (1 + 7 * (kChainVjpBlock / kChainDim)) <= 64 * 1024;
}

template <typename T>
hipError_t launch_kd_chain_vjp_step(const LayerConst* hlcs, int nl, const LayerConst* lcs, const T* p, int64_t P,
                                    int64_t K, const ChainAdjStep<T>& a, int grid_cap, void* slab, size_t slab_bytes,
                                    T* const* km_out, double* err_out, hipStream_t st) {
    if (K < 1 || grid_cap < 1 || !chain_vjp_step_supported(hlcs, nl, P, sizeof(T)) || a.njump > 8)
        return hipErrorNotSupported;
    const int ng = kChainVjpBlock / kChainDim;
    const size_t lds = nl * sizeof(LayerConst) + (size_t)P * sizeof(T) * (1 + (a.fsal ? 7 : 6) * ng);
    // the stage kernel's grid (grid_cap: its slab's row capacity, <= 1024): the same blocks sum the same columns,
    // so the per-block sums and the reduction order are the stage kernel's
    const int grid = grid_for(K, ng, grid_cap);
    if (chain_vjp_step_slab_bytes(P, K, sizeof(T), grid_cap) > slab_bytes) return hipErrorNotSupported;
    const int64_t region = (int64_t)((((size_t)grid * P * sizeof(T) + 255) & ~(size_t)255) / sizeof(T));
    T* tslab = (T*)slab;
    double* eslab = (double*)((char*)slab + 7 * region * sizeof(T));
    const LayerConst& h = hlcs[0];
#define KAN_CVSTEP(NORM, PATH, S)                                                                                 \
    hipLaunchKernelGGL((kd_chain_vjp_step_kernel<T, NORM, PATH, S>), dim3(grid), dim3(kChainVjpBlock), lds, st,  \
                       lcs, nl, p, (int)P, K, a, tslab, region, eslab)
    if (h.norm == NORM_TANH_FAST && h.path == PATH_REC && chain_is_lv(hlcs, nl))
        KAN_CVSTEP(NORM_TANH_FAST, PATH_REC, ChainShapeLV);
    else if (h.norm == NORM_TANH_FAST && h.path == PATH_REC) KAN_CVSTEP(NORM_TANH_FAST, PATH_REC, ChainShapeAny);
    else if (h.path == PATH_REC_CORR) KAN_CVSTEP(NORM_RUNTIME, PATH_REC_CORR, ChainShapeAny);
    else if (h.path == PATH_REC) KAN_CVSTEP(NORM_RUNTIME, PATH_REC, ChainShapeAny);
    else KAN_CVSTEP(NORM_RUNTIME, PATH_DIRECT, ChainShapeAny);
#undef KAN_CVSTEP
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    ChainKmOut<T> km{};
    for (int s = 0; s < (a.fsal ? 7 : 6); ++s) km.k[s] = km_out[s];
    hipLaunchKernelGGL((chain_vjp_step_finish_kernel<T>), dim3((unsigned)P + 1, a.fsal ? 7 : 6), dim3(kBlock), 0, st,
                       tslab, region,
                       (int64_t)grid, (int64_t)P, km, eslab, a.want_error ? err_out : nullptr);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_kd_chain_vjp_stage(const LayerConst* hlcs, int nl, const LayerConst* lcs, const T* p, int64_t P,
                                     const T* u, const StageArgs<T>& su, const T* lam, const StageArgs<T>& sl,
                                     T* lam_out, T* lamJ, T* dp, bool dp_assign, double* err_out, void* slab,
                                     size_t slab_bytes, int64_t K, hipStream_t st) {
    if (nl < 1 || nl > kChainMaxLayers || K < 1) return hipErrorNotSupported;
    for (int l = 0; l < nl; ++l) {
        const LayerConst& h = hlcs[l];
        if (h.I > kChainDim || h.O > kChainDim || h.path != hlcs[0].path || h.norm != hlcs[0].norm)
            return hipErrorNotSupported;
        if (l > 0 && h.I != hlcs[l - 1].O) return hipErrorNotSupported;
    }
    if (hlcs[nl - 1].O != hlcs[0].I) return hipErrorNotSupported;
    const int ng = kChainVjpBlock / kChainDim;
    const size_t lds = nl * sizeof(LayerConst) + (size_t)P * sizeof(T) * (1 + ng);
    if (lds > 60 * 1024) return hipErrorNotSupported;
    // slab: [grid][P] T rows, then [grid] double error partials
    int64_t cap = (int64_t)(slab_bytes / (P * sizeof(T) + sizeof(double))) - 1;
    if (cap > 1024) cap = 1024;
    if (cap < 1) return hipErrorNotSupported;
    const int grid = grid_for(K, ng, (int)cap);
    T* tslab = (T*)slab;
    double* eslab = err_out ? (double*)((char*)slab + (((size_t)grid * P * sizeof(T) + 255) & ~(size_t)255)) : nullptr;
    const LayerConst& h = hlcs[0];
    const bool one = grid == 1;   // a single block writes dp and the error total itself
#define KAN_CVJP(NORM, PATH, S)                                                                                  \
    hipLaunchKernelGGL((kd_chain_vjp_stage_kernel<T, NORM, PATH, S>), dim3(grid), dim3(kChainVjpBlock), lds, st, \
                       lcs, nl, p, (int)P, u, su, lam, sl, lam_out, lamJ, one ? nullptr : tslab,                  \
                       one ? nullptr : eslab, K, one ? dp : nullptr, dp_assign ? 1 : 0, one ? err_out : nullptr)
    if (h.norm == NORM_TANH_FAST && h.path == PATH_REC && chain_is_lv(hlcs, nl))
        KAN_CVJP(NORM_TANH_FAST, PATH_REC, ChainShapeLV);
    else if (h.norm == NORM_TANH_FAST && h.path == PATH_REC) KAN_CVJP(NORM_TANH_FAST, PATH_REC, ChainShapeAny);
    else if (h.path == PATH_REC_CORR) KAN_CVJP(NORM_RUNTIME, PATH_REC_CORR, ChainShapeAny);
    else if (h.path == PATH_REC) KAN_CVJP(NORM_RUNTIME, PATH_REC, ChainShapeAny);
    else KAN_CVJP(NORM_RUNTIME, PATH_DIRECT, ChainShapeAny);
#undef KAN_CVJP
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || one || (!dp && !err_out)) return e;
    hipLaunchKernelGGL((chain_vjp_finish_kernel<T>), dim3((unsigned)(dp ? P : 0) + (err_out ? 1 : 0)), dim3(kBlock), 0,
                       st, tslab, (int64_t)grid, (int64_t)P, dp, dp_assign ? 1 : 0, eslab, err_out);
    return hipGetLastError();
}

#define KAN_COL_INST(T)                                                                                          \
    template hipError_t launch_kd_chain_vjp_step<T>(const LayerConst*, int, const LayerConst*, const T*, int64_t,  \
                                                    int64_t, const ChainAdjStep<T>&, int, void*, size_t,        \
                                                    T* const*,                                                  \
                                                    double*, hipStream_t);                                        \
    template hipError_t launch_kd_chain_vjp_stage<T>(const LayerConst*, int, const LayerConst*, const T*, int64_t, \
                                                     const T*, const StageArgs<T>&, const T*, const StageArgs<T>&, \
                                                     T*, T*, T*, bool, double*, void*, size_t, int64_t,          \
                                                     hipStream_t);                                                \
    template hipError_t launch_kd_chain_col<T>(const LayerConst*, int, const LayerConst*, const T*, int64_t,     \
                                               const T*, T*, int64_t, hipStream_t, const StageArgs<T>*, T*,       \
                                               double*, int, double*);                                            \
    template hipError_t launch_slab_reduce<T>(const T*, int64_t, int64_t, T*, hipStream_t);                       \
    template hipError_t launch_kd_chain_step<T>(const LayerConst*, int, const LayerConst*, const T*, int64_t,    \
                                                int64_t, const ChainStepArgs&, double*, int, double*, hipStream_t); \
    template hipError_t launch_kd_chain_tsit5<T>(const LayerConst*, int, const LayerConst*, const T*, int64_t,   \
                                                 const T*, int64_t, const ChainSolveArgs&, hipStream_t);         \
    template hipError_t launch_kd_chain_adjoint<T>(const LayerConst*, int, const LayerConst*, const T*, int64_t, \
                                                   int64_t, const ChainAdjointArgs&, hipStream_t, bool);         \
    template hipError_t launch_kd_fwd_col<T>(const LayerConst&, const LayerConst*, const T*, const T*, T*,        \
                                             int64_t, hipStream_t);                                               \
    template hipError_t launch_kd_vjp_col<T>(const LayerConst&, const LayerConst*, const T*, const T*, const T*,  \
                                             T*, T*, T*, int, int64_t, hipStream_t);                              \
    template hipError_t launch_kd_edge_act<T>(const LayerConst&, const LayerConst*, const T*, const T*, T*,       \
                                              int64_t, hipStream_t);
KAN_COL_INST(double)
KAN_COL_INST(float)
#undef KAN_COL_INST

}  // namespace kan
