// streambench.hip — HBM ceiling of the Fisher-KPP RHS access pattern (development tool,
// not part of libkanode.so).  B rows of Nx=256 doubles in, B rows out; each variant
// moves the same 2·8·B·Nx bytes and reports GB/s.
//   copy_rows    thread per point pair, 128 threads per row, grid-stride over rows (the RHS mapping)
//   stencil_rows same + the two neighbour loads and a 3-point combination
//   copy_flat    flat dwordx4 grid-stride copy (no row structure)
//   copy_nt      copy_rows with nontemporal loads/stores
//   copy_rows4   4 rows per thread per iteration (loads first)
//   wave_nt      one wave per row, 2 x 16 B per lane (the fk_rhs_pp_wave_kernel access), nontemporal
//   wave_nt_r2   the same with two rows per wave in flight
//   wave_dflt    wave_nt with default-policy loads and stores
//   wave_ntld    nontemporal loads, default-policy stores
//   flat_nt_u4   flat copy, 4 independent 1 KB wave loads per iteration, nontemporal
// argv: [B rows] [grid list, comma separated; 0 = one wave per row, no grid stride]
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/streambench tools/streambench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

constexpr int NX = 256;

__global__ void __launch_bounds__(256) copy_rows(const double* __restrict__ u, double* __restrict__ d, long B) {
    const int lt = threadIdx.x & 127;
    for (long b = blockIdx.x * 2 + (threadIdx.x >> 7); b < B; b += gridDim.x * 2) {
        const double2 v = *reinterpret_cast<const double2*>(u + b * NX + 2 * lt);
        *reinterpret_cast<double2*>(d + b * NX + 2 * lt) = v;
    }
}

__global__ void __launch_bounds__(256) stencil_rows(const double* __restrict__ u, double* __restrict__ d, long B) {
    const int lt = threadIdx.x & 127;
    const int i = 2 * lt, im = i ? i - 1 : NX - 1, ip = i + 2 < NX ? i + 2 : 0;
    for (long b = blockIdx.x * 2 + (threadIdx.x >> 7); b < B; b += gridDim.x * 2) {
        const double* ub = u + b * NX;
        const double2 v = *reinterpret_cast<const double2*>(ub + i);
        const double um = ub[im], up = ub[ip];
        double2 o;
        o.x = um + v.y - 2.0 * v.x;
        o.y = v.x + up - 2.0 * v.y;
        *reinterpret_cast<double2*>(d + b * NX + i) = o;
    }
}

__global__ void __launch_bounds__(256) copy_flat(const double2* __restrict__ u, double2* __restrict__ d, long n2) {
    for (long k = blockIdx.x * 256L + threadIdx.x; k < n2; k += (long)gridDim.x * 256) d[k] = u[k];
}

__global__ void __launch_bounds__(256) copy_nt(const double* __restrict__ u, double* __restrict__ d, long B) {
    const int lt = threadIdx.x & 127;
    for (long b = blockIdx.x * 2 + (threadIdx.x >> 7); b < B; b += gridDim.x * 2) {
        const double2* src = reinterpret_cast<const double2*>(u + b * NX + 2 * lt);
        double2* dst = reinterpret_cast<double2*>(d + b * NX + 2 * lt);
        double2 v;
        v.x = __builtin_nontemporal_load(&src->x);
        v.y = __builtin_nontemporal_load(&src->y);
        __builtin_nontemporal_store(v.x, &dst->x);
        __builtin_nontemporal_store(v.y, &dst->y);
    }
}

__global__ void __launch_bounds__(256) copy_rows4(const double* __restrict__ u, double* __restrict__ d, long B) {
    const int lt = threadIdx.x & 127;
    const long st = gridDim.x * 2L;
    long b = blockIdx.x * 2 + (threadIdx.x >> 7);
    for (; b + 3 * st < B; b += 4 * st) {
        double2 v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = *reinterpret_cast<const double2*>(u + (b + r * st) * NX + 2 * lt);
#pragma unroll
        for (int r = 0; r < 4; ++r) *reinterpret_cast<double2*>(d + (b + r * st) * NX + 2 * lt) = v[r];
    }
    for (; b < B; b += st) *reinterpret_cast<double2*>(d + b * NX + 2 * lt) = *reinterpret_cast<const double2*>(u + b * NX + 2 * lt);
}

typedef double kd2 __attribute__((ext_vector_type(2)));

template <int R, int LD, int ST>   // LD/ST: 1 = nontemporal
__global__ void __launch_bounds__(256) wave_rows(const double* __restrict__ u, double* __restrict__ d, long B) {
    const int lane = threadIdx.x & 63;
    const long rs = (long)gridDim.x * 4;
    for (long b = blockIdx.x * 4L + (threadIdx.x >> 6); b < B; b += R * rs) {
        kd2 v[R][2];
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (b + r * rs < B)
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const kd2* src = reinterpret_cast<const kd2*>(u + (b + r * rs) * NX + 128 * k + 2 * lane);
                    v[r][k] = LD ? __builtin_nontemporal_load(src) : *src;
                }
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (b + r * rs < B)
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    kd2* dst = reinterpret_cast<kd2*>(d + (b + r * rs) * NX + 128 * k + 2 * lane);
                    if (ST) __builtin_nontemporal_store(v[r][k], dst);
                    else *dst = v[r][k];
                }
    }
}

__global__ void __launch_bounds__(256) flat_nt_u4(const kd2* __restrict__ u, kd2* __restrict__ d, long n2) {
    const long step = (long)gridDim.x * 256;
    long k = blockIdx.x * 256L + threadIdx.x;
    for (; k + 3 * step < n2; k += 4 * step) {
        kd2 v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = __builtin_nontemporal_load(u + k + r * step);
#pragma unroll
        for (int r = 0; r < 4; ++r) __builtin_nontemporal_store(v[r], d + k + r * step);
    }
    for (; k < n2; k += step) __builtin_nontemporal_store(__builtin_nontemporal_load(u + k), d + k);
}

int main(int argc, char** argv) {
    const long B = argc > 1 ? atol(argv[1]) : 131072;
    const int reps = B > 262144 ? 20 : 50;
    const size_t n = (size_t)B * NX;
    double *u, *d;
    CK(hipMalloc(&u, n * 8));
    CK(hipMalloc(&d, n * 8));
    CK(hipMemset(u, 0, n * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = 2.0 * 8.0 * n;
    std::vector<int> grids;
    {
        const char* gl = argc > 2 ? argv[2] : "1024,2048,4096,8192,0";
        for (const char* c = gl; *c;) {
            grids.push_back(atoi(c));
            while (*c && *c != ',') ++c;
            if (*c == ',') ++c;
        }
    }
    static const char* names[] = {"copy_rows", "stencil_rows", "copy_flat", "copy_nt", "copy_rows4", "wave_nt",
                                  "wave_nt_r2", "wave_dflt", "wave_ntld", "flat_nt_u4"};
    for (int v = 0; v < 10; ++v) {
        for (int g0 : grids) {
            const int g = g0 > 0 ? g0 : (int)((B + 3) / 4);
            auto launch = [&]() {
                switch (v) {
                case 0: hipLaunchKernelGGL(copy_rows, dim3(g), dim3(256), 0, 0, u, d, B); break;
                case 1: hipLaunchKernelGGL(stencil_rows, dim3(g), dim3(256), 0, 0, u, d, B); break;
                case 2: hipLaunchKernelGGL(copy_flat, dim3(g), dim3(256), 0, 0, (const double2*)u, (double2*)d, (long)(n / 2)); break;
                case 3: hipLaunchKernelGGL(copy_nt, dim3(g), dim3(256), 0, 0, u, d, B); break;
                case 4: hipLaunchKernelGGL(copy_rows4, dim3(g), dim3(256), 0, 0, u, d, B); break;
                case 5: hipLaunchKernelGGL((wave_rows<1, 1, 1>), dim3(g), dim3(256), 0, 0, u, d, B); break;
                case 6: hipLaunchKernelGGL((wave_rows<2, 1, 1>), dim3(g), dim3(256), 0, 0, u, d, B); break;
                case 7: hipLaunchKernelGGL((wave_rows<1, 0, 0>), dim3(g), dim3(256), 0, 0, u, d, B); break;
                case 8: hipLaunchKernelGGL((wave_rows<1, 1, 0>), dim3(g), dim3(256), 0, 0, u, d, B); break;
                case 9: hipLaunchKernelGGL(flat_nt_u4, dim3(g), dim3(256), 0, 0, (const kd2*)u, (kd2*)d, (long)(n / 2)); break;
                }
            };
            for (int r = 0; r < 5; ++r) launch();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            for (int r = 0; r < reps; ++r) launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / reps;
            std::printf("%-13s grid %7d  %8.1f us  %7.0f GB/s\n", names[v], g, us, bytes / (us * 1e-6) / 1e9);
            std::fflush(stdout);
        }
    }
    return 0;
}
