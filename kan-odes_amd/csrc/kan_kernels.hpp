// kan_kernels.hpp — internal launcher declarations (C++ linkage, not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kan_device.hpp"

namespace kan {

// `hlc` is the host copy of the layer constants (selects the kernel variant),
// `lc` the device copy the kernels read.  All pointers are device pointers.
template <typename T>
hipError_t launch_fk_rhs(const LayerConst& hlc, const LayerConst* lc, const T* p, T cd, T co, int Nx,
                         const T* u, T* du, int64_t B, hipStream_t st);
template <typename T>
hipError_t launch_fk_vjp(const LayerConst& hlc, const LayerConst* lc, const T* p, T cd, T co, int Nx,
                         const T* u, const T* lam, T* lamJ, T* dp, T* slab, int slab_blocks, int64_t B,
                         hipStream_t st);
// piecewise-polynomial Fisher-KPP RHS / VJP (kan_pp.hip).  `tables` holds
// kPPMaxFns slots of kPPCoef·ni doubles (slot = PPFn id); the build fills the listed
// functions from p, the RHS then reads slot PP_PHI (fp64, Nx even).
hipError_t launch_fk_pp_build(const PPConst& hpc, const LayerConst* lc, const PPConst* pc, const double* p,
                              double* tables, const int* fns, int nfn, hipStream_t st);
hipError_t launch_fk_rhs_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc, const double* p,
                            double* table, double cd, double co, int Nx, const double* u, double* du, int64_t B,
                            hipStream_t st);
bool fk_vjp_pp_supported(const LayerConst& hlc, int Nx);
hipError_t launch_fk_vjp_pp(const PPConst& hpc, const LayerConst& hlc, const LayerConst* lc, const PPConst* pc,
                            const double* p, double* tables, double cd, double co, int Nx, const double* u,
                            const double* lam, double* lamJ, double* dp, double* slab, int slab_blocks, int64_t B,
                            hipStream_t st);
template <typename T>
hipError_t launch_kd_fwd_col(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, T* y, int64_t K,
                             hipStream_t st);
template <typename T>
hipError_t launch_kd_vjp_col(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, const T* yb,
                             T* xb, T* pbar, T* slab, int slab_blocks, int64_t K, hipStream_t st);
template <typename T>
hipError_t launch_kd_edge_act(const LayerConst& hlc, const LayerConst* lc, const T* p, const T* x, T* act, int64_t K,
                              hipStream_t st);

// surrogate shapes (kan_wide.hip)
constexpr int kWideKT = 8;       // column tile of the wide-out kernels
constexpr int kWideOMax = 16;    // max out_dims of a wide-in layer
template <typename T>
hipError_t launch_kd_fwd_widein(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, T* y, T* slab,
                                int64_t K, hipStream_t st);
template <typename T>
hipError_t launch_kd_fwd_wideout(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, T* y, int64_t K,
                                 hipStream_t st);
template <typename T>
hipError_t launch_kd_vjp_wideout(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, const T* yb,
                                 T* xb, T* pbar, T* slab, int64_t K, hipStream_t st);
template <typename T>
hipError_t launch_kd_vjp_widein(const LayerConst& h, const LayerConst* lc, const T* p, const T* x, const T* yb, T* xb,
                                T* pbar, int64_t K, hipStream_t st);

}  // namespace kan
