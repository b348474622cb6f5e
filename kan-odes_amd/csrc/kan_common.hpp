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
