// kan_common.hpp — shared device helpers for the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

#include "kan_device.hpp"

namespace kan {

// Raise a kernel's dynamic-LDS limit (hipFuncAttributeMaxDynamicSharedMemorySize) on the CURRENT device to
// at least `lds` bytes.  HIP applies the attribute per device, so the raised sizes are remembered per
// (kernel, device) under a lock: a second GPU driven from the same process, or two threads, still raise it.
inline hipError_t ensure_dynamic_lds(const void* fn, size_t lds) {
    static std::mutex mu;
    static std::map<std::pair<const void*, int>, size_t> raised;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(mu);
    size_t& cap = raised[{fn, dev}];
    if (lds <= cap) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e == hipSuccess) cap = lds;
    return e;
}

constexpr int kBlock = 256;
constexpr int kWave = 64;
constexpr int kGridCap = 256 * 16;   // 16 blocks per CU over 256 CUs; grid-stride beyond

// DPP lane permutations (VALU, no LDS round trip) of a 32/64-bit value
template <int CTRL> __device__ __forceinline__ double dpp_mov(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
template <int CTRL> __device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// Sum over the 16 lanes of a DPP row, received by every lane of the row: quad_perm [1,0,3,2],
// quad_perm [2,3,0,1], row_half_mirror, row_mirror (each step adds a partner, so all lanes
// end with the same bits)
template <typename T> __device__ __forceinline__ T row16_sum(T v) {
    v += dpp_mov<0xB1>(v);
    v += dpp_mov<0x4E>(v);
    v += dpp_mov<0x141>(v);
    v += dpp_mov<0x140>(v);
    return v;
}
// Lane o of each 16-lane row broadcast to the row (row_newbcast, gfx90a+); o is a constant
// after unrolling, so the switch folds away
template <typename T> __device__ __forceinline__ T row16_bcast(T v, int o) {
    switch (o) {
    case 0: return dpp_mov<0x150>(v);
    case 1: return dpp_mov<0x151>(v);
    case 2: return dpp_mov<0x152>(v);
    case 3: return dpp_mov<0x153>(v);
    case 4: return dpp_mov<0x154>(v);
    case 5: return dpp_mov<0x155>(v);
    case 6: return dpp_mov<0x156>(v);
    case 7: return dpp_mov<0x157>(v);
    case 8: return dpp_mov<0x158>(v);
    case 9: return dpp_mov<0x159>(v);
    case 10: return dpp_mov<0x15A>(v);
    case 11: return dpp_mov<0x15B>(v);
    case 12: return dpp_mov<0x15C>(v);
    case 13: return dpp_mov<0x15D>(v);
    case 14: return dpp_mov<0x15E>(v);
    default: return dpp_mov<0x15F>(v);
    }
}

template <typename T> __device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

// Wave reduce-scatter of M values per lane (recursive halving): at lane offset OFF the lanes with
// that bit set keep the upper half of their slots and the others the lower half, each adding its
// partner's copy, so the exchange count halves with every step (N = 11: 14 exchanges instead of
// 6 x 11 shuffles).  Lane-local (base, cnt): the lane's slots hold the global values
// [base, base + cnt).  Once one slot is left, the remaining offsets are a plain butterfly (a + b and
// b + a: the same bits on both lanes).  No LDS: OFF = 32 / 16 exchange halves / rows with
// v_permlane32_swap / v_permlane16_swap (gfx950), which also do the keep/send selection; OFF = 8, 4,
// 2, 1 pair lanes inside a 16-lane row with DPP row_mirror, row_half_mirror and quad perms (each an
// involution that pairs lanes differing in bit OFF).
__device__ __forceinline__ void perm_swap32(double& x, double& y) {
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(y), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(y), false, false);
    x = __hiloint2double((int)hi[0], (int)lo[0]);
    y = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void perm_swap16(double& x, double& y) {
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(y), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(y), false, false);
    x = __hiloint2double((int)hi[0], (int)lo[0]);
    y = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void perm_swap32(float& x, float& y) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(x), __float_as_int(y), false, false);
    x = __int_as_float((int)r[0]);
    y = __int_as_float((int)r[1]);
}
__device__ __forceinline__ void perm_swap16(float& x, float& y) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(x), __float_as_int(y), false, false);
    x = __int_as_float((int)r[0]);
    y = __int_as_float((int)r[1]);
}
template <int OFF, typename T> __device__ __forceinline__ T row_partner(T v) {
    static_assert(OFF == 8 || OFF == 4 || OFF == 2 || OFF == 1, "row-local partner");
    return dpp_mov<OFF == 8 ? 0x140 : OFF == 4 ? 0x141 : OFF == 2 ? 0x4E : 0xB1>(v);
}
template <typename T, int M, int OFF>
__device__ __forceinline__ void rs_step(T (&w)[16], int lane, int& base, int& cnt) {
    if constexpr (OFF > 0) {
        if constexpr (M == 1) {
            static_assert(OFF <= 8, "N >= 3 keeps two slots past the cross-row steps");
            w[0] = w[0] + row_partner<OFF>(w[0]);
            rs_step<T, 1, OFF / 2>(w, lane, base, cnt);
        } else {
            constexpr int H = (M + 1) / 2;
            const bool hi = (lane & OFF) != 0;
#pragma unroll
            for (int i = 0; i < H; ++i) {
                T a = w[i];
                T b = i + H < M ? w[i + H] : T(0);
                if constexpr (OFF >= 16) {
                    // x = [own a | partner's b], y = [partner's a | own b] on the lower / upper lanes
                    if constexpr (OFF == 32) perm_swap32(a, b);
                    else perm_swap16(a, b);
                    w[i] = hi ? b + a : a + b;   // own + partner on both sides
                } else {
                    const T keep = hi ? b : a, send = hi ? a : b;
                    w[i] = keep + row_partner<OFF>(send);
                }
            }
            if (hi) {
                base += H;
                cnt = cnt > H ? cnt - H : 0;
            } else {
                cnt = cnt < H ? cnt : H;
            }
            rs_step<T, H, OFF / 2>(w, lane, base, cnt);
        }
    }
}

#ifndef KAN_BLOCK_RS
#define KAN_BLOCK_RS 1
#endif
// Sum `n` (<= N) per-thread values across the block into out[0..n): a wave reduce-scatter
// (3 <= N <= 16; wave_sum per value otherwise), then the wave partials summed in wave order (fixed
// order, so the result is bitwise reproducible).  `red` is LDS of >= (blockDim/64)*N elements.
// Agent-scope relaxed 64-bit store / load (sc1: visible across the XCDs' L2s without a cache flush), for
// hand-offs between workgroups of one launch (cdna_hip_programming.md Guideline 16)
__device__ __forceinline__ void st_agent(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// s + Σ x[b·stride] over this thread's rows b = threadIdx.x + k·blockDim.x < n, in increasing b (the adds in
// the order of the one-row loop, so the same bits), four rows' loads in flight per pass: the finish and
// reduction kernels are load-latency bound (round 4: adj_finish_kernel 5.71 -> 5.37 us per adaptive step)
template <typename A, typename T>
__device__ __forceinline__ A strided_rows_sum(const T* x, int64_t n, int64_t stride, A s) {
    const int64_t bs = blockDim.x;
    int64_t b = threadIdx.x;
    for (; b + 3 * bs < n; b += 4 * bs) {
        T v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = x[(b + r * bs) * stride];
#pragma unroll
        for (int r = 0; r < 4; ++r) s += (A)v[r];
    }
    for (; b < n; b += bs) s += (A)x[b * stride];
    return s;
}

// Global -> LDS copy of n 16-byte elements by direct-to-LDS loads (global_load_lds_dwordx4: the destination is the
// wave-uniform base + lane·16, so each wave copies 64 consecutive elements per instruction).  No VGPR holds the data
// and no load waits for the one before it: a strided register copy loop waits for each load before its ds_write,
// one memory round trip per 16·blockDim bytes at every block's start.  The caller's next __syncthreads waits for
// the copies (hipcc emits vmcnt(0) there while they are outstanding).
template <typename V>
__device__ __forceinline__ void lds_copy16(V* lds, const V* g, int n) {
    static_assert(sizeof(V) == 16, "16-byte elements");
    typedef __attribute__((address_space(1))) void gvoid;
    typedef __attribute__((address_space(3))) void lvoid;
    const int lane = threadIdx.x & (kWave - 1);
    for (int base = threadIdx.x & ~(kWave - 1); base < n; base += blockDim.x)
        if (base + lane < n)
            __builtin_amdgcn_global_load_lds((gvoid*)(g + base + lane), (lvoid*)(lds + base), 16, 0, 0);
}

// AGENT: the sums are stored with st_agent (another workgroup of the same launch reads them); sum q goes
// to out[q·ostride]
template <typename T, int N, bool AGENT = false>
__device__ __forceinline__ void block_sum_to(const T (&v)[N], int n, T* red, T* out, int64_t ostride = 1) {
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    const int nw = blockDim.x / kWave;
    if constexpr (KAN_BLOCK_RS && N >= 3 && N <= 16) {
        T w[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) w[q] = q < N ? v[q] : T(0);
        int base = 0, cnt = N;
        rs_step<T, N, 32>(w, lane, base, cnt);
        if ((lane & 3) == 0 && cnt >= 1 && base < n) red[wid * n + base] = w[0];
    } else {
#pragma unroll
        for (int q = 0; q < N; ++q) {
            if (q < n) {
                const T s = wave_sum(v[q]);
                if (lane == 0) red[wid * n + q] = s;
            }
        }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < n; q += blockDim.x) {
        T s = red[q];
        for (int w = 1; w < nw; ++w) s += red[w * n + q];
        if constexpr (AGENT) st_agent(out + q * ostride, s);
        else out[q * ostride] = s;
    }
    __syncthreads();
}

inline int grid_for(int64_t work, int per_block, int cap) {
    int64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    return (int)(g < cap ? g : cap);
}

inline int ceil_log2(int v) {
    int l = 0;
    while ((1 << l) < v) ++l;
    return l;
}

template <typename T> struct Vec2;
template <> struct Vec2<double> { using type = double2; };
template <> struct Vec2<float> { using type = float2; };

// dp[q] += Σ_b slab[b*P + q] (ordered): defined in kan_col.hip
template <typename T>
hipError_t launch_slab_reduce(const T* slab, int64_t nblk, int64_t P, T* dp, hipStream_t st);

}  // namespace kan
