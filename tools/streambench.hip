// streambench.hip — HBM ceiling of the Fisher-KPP RHS access pattern (development tool,
// not part of libkanode.so).  B rows of Nx=256 doubles in, B rows out; each variant
// moves the same 2·8·B·Nx bytes and reports GB/s.
//   copy_rows    thread per point pair, 128 threads per row, grid-stride over rows (the RHS mapping)
//   stencil_rows same + the two neighbour loads and a 3-point combination
//   copy_flat    flat dwordx4 grid-stride copy (no row structure)
//   copy_nt      copy_rows with nontemporal loads/stores
//   copy_rows4   4 rows per thread per iteration (loads first)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/streambench tools/streambench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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

int main(int argc, char** argv) {
    const long B = argc > 1 ? atol(argv[1]) : 131072;
    const int reps = 50;
    const size_t n = (size_t)B * NX;
    double *u, *d;
    CK(hipMalloc(&u, n * 8));
    CK(hipMalloc(&d, n * 8));
    CK(hipMemset(u, 0, n * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = 2.0 * 8.0 * n;
    const int grids[] = {1024, 1792, 2048, 4096, 8192, 16384};
    for (int v = 0; v < 5; ++v) {
        for (int g : grids) {
            auto launch = [&]() {
                switch (v) {
                case 0: hipLaunchKernelGGL(copy_rows, dim3(g), dim3(256), 0, 0, u, d, B); break;
                case 1: hipLaunchKernelGGL(stencil_rows, dim3(g), dim3(256), 0, 0, u, d, B); break;
                case 2: hipLaunchKernelGGL(copy_flat, dim3(g), dim3(256), 0, 0, (const double2*)u, (double2*)d, (long)(n / 2)); break;
                case 3: hipLaunchKernelGGL(copy_nt, dim3(g), dim3(256), 0, 0, u, d, B); break;
                case 4: hipLaunchKernelGGL(copy_rows4, dim3(g), dim3(256), 0, 0, u, d, B); break;
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
            static const char* names[] = {"copy_rows", "stencil_rows", "copy_flat", "copy_nt", "copy_rows4"};
            std::printf("%-13s grid %6d  %8.1f us  %7.0f GB/s\n", names[v], g, us, bytes / (us * 1e-6) / 1e9);
        }
    }
    return 0;
}
