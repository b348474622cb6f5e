// kan_lap.hpp — rows of the reference's periodic Laplacian (D*lap)*u, in the dense
// matvec's ascending-column order (PDE examples/Fisher-KPP_Source.jl:55-59,97).
#pragma once
#include <hip/hip_runtime.h>

namespace kan {

// (D*lap)*u row i: the reference matrix's nonzeros in ascending column order,
// no FMA contraction (the dense gemv adds exact zeros elsewhere).  um/up are
// the periodic neighbours (already wrapped).
template <typename T>
__device__ __forceinline__ T lap3(T um, T u0, T up, int i, int Nx, T cd, T co) {
#pragma clang fp contract(off)
    if (Nx >= 3) {
        if (i == 0) { T s = cd * u0; s = s + co * up; s = s + co * um; return s; }
        if (i == Nx - 1) { T s = co * up; s = s + co * um; s = s + cd * u0; return s; }
        T s = co * um; s = s + cd * u0; s = s + co * up; return s;
    }
    if (Nx == 2) {
        if (i == 0) { T s = cd * u0; s = s + co * up; return s; }
        T s = co * um; s = s + cd * u0; return s;
    }
    return co * u0;  // Nx == 1: lap[1,end] overwrote the diagonal
}

// Rows i and i+1 (i even, Nx even >= 4) branch-free: the same per-row ascending-
// column orders as lap3, the boundary orders picked by selects.
template <typename T>
__device__ __forceinline__ void lap_pair(T um, T u0, T u1, T up, int i, int Nx, T cd, T co, T& r0, T& r1) {
#pragma clang fp contract(off)
    const bool first = i == 0;
    const bool last = i + 2 == Nx;
    {
        const T a = co * um, b = cd * u0, c = co * u1;   // row i: middle (a+b)+c, row 0 (b+c)+a
        const T f1 = first ? b : a, f2 = first ? c : b, f3 = first ? a : c;
        r0 = (f1 + f2) + f3;
    }
    {
        const T a = co * u0, b = cd * u1, c = co * up;   // row i+1: middle (a+b)+c, row Nx-1 (c+a)+b
        const T f1 = last ? c : a, f2 = last ? a : b, f3 = last ? b : c;
        r1 = (f1 + f2) + f3;
    }
}

}  // namespace kan
