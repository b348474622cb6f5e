/*
 * kanode_ref.c — CPU ORACLE (test infrastructure only; see kanode_ref.h).
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off: no silent FMA contraction,
 * so the restated evaluation order is the one executed).
 */
#include "kanode_ref.h"
#include <math.h>
#include <stdlib.h>

#define KREF_MAX_G 64
#define KREF_STACK 256

/* kdense.jl:98-107 */
int64_t kref_layer_param_length(const kref_layer* L) {
    int64_t n = (int64_t)L->in_dims * L->grid_len * L->out_dims;
    if (L->use_base_act) n += (int64_t)L->in_dims * L->out_dims;
    return n;
}

/* kdense.jl:88-92: grid = collect(LinRange(grid_lims..., G)) with Float32 lims.
 * Julia's LinRange getindex is lerpi(j, G-1, a, b) = T((1-t)*a + t*b) with
 * t = j/(G-1) evaluated in Float64, then rounded to Float32 (T). */
void kref_knots(const kref_layer* L, float* grid) {
    const int32_t G = L->grid_len;
    const double a = (double)L->grid_lo, b = (double)L->grid_hi;
    for (int32_t j = 0; j < G; ++j) {
        double t = (double)j / (double)(G - 1);
        grid[j] = (float)((1.0 - t) * a + t * b);
    }
}

/* kdense.jl:27: denominator = Float32(2 / (grid_len - 1)) (independent of grid_lims) */
float kref_default_denominator(int32_t grid_len) { return (float)(2.0 / (double)(grid_len - 1)); }

/* utils.jl:9: (1/h) with h::Float32 is a Float32 division */
float kref_inv_h(const kref_layer* L) {
    volatile float h = L->denominator;
    return 1.0f / h;
}

#define KREF_IS_F64 1
#define R double
#define SFX(name) name##_f64
#define RF(fn) fn
#include "kanode_ref_impl.inc"
#undef KREF_IS_F64
#undef R
#undef SFX
#undef RF

#define KREF_IS_F64 0
#define R float
#define SFX(name) name##_f32
#define RF(fn) fn##f
#include "kanode_ref_impl.inc"
#undef KREF_IS_F64
#undef R
#undef SFX
#undef RF
