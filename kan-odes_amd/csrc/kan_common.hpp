// kan_common.hpp — shared device helpers for the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "kan_device.hpp"

namespace kan {

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

// Sum `n` (<= N) per-thread values across the block into out[0..n): wave
// shuffles, then the wave partials summed in wave order (fixed order, so the
// result is bitwise reproducible).  `red` is LDS of >= (blockDim/64)*N elements.
template <typename T, int N>
__device__ __forceinline__ void block_sum_to(const T (&v)[N], int n, T* red, T* out) {
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    const int nw = blockDim.x / kWave;
#pragma unroll
    for (int q = 0; q < N; ++q) {
        if (q < n) {
            const T s = wave_sum(v[q]);
            if (lane == 0) red[wid * n + q] = s;
        }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < n; q += blockDim.x) {
        T s = red[q];
        for (int w = 1; w < nw; ++w) s += red[w * n + q];
        out[q] = s;
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
