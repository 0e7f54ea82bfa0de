// fp16-pair arithmetic shared by the precision-mode-2 GEMM kernels (gemm_x6.hip, wgrad.hip):
// the exact power-of-two scaled split of f32 values into fp16 (hi, lo) pairs and the
// 32x32x16 f16 MFMA (gemm_x6.hip's header comment has the error analysis).
#pragma once
#include "gemm.hpp"

namespace nerf {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_f16(float a, float b) {
    f32x2 v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2v));   // RNE
}

// (a, b) scaled by 2^e -> packed fp16 pairs hi, lo with a 2^e = hi.x + lo.x (+ <= 2^-22 |a| 2^e).
// The residual a 2^e - hi is exact in f32; one v_fma_mix_f32 per value forms it from the fp16
// half in place (-hi x 1 + a), instead of a conversion back to f32 and a subtraction
__device__ __forceinline__ void split2h(float a, float b, int e, uint32_t& h, uint32_t& l) {
    a = __builtin_amdgcn_ldexpf(a, e);
    b = __builtin_amdgcn_ldexpf(b, e);
    h = pk_f16(a, b);
    float ra, rb;
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(ra) : "v"(h), "v"(a));
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(rb) : "v"(h), "v"(b));
    l = pk_f16(ra, rb);
}

__device__ __forceinline__ f32x16 mfma_f16(const uint4& a, const uint4& b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                  0, 0, 0);
}

// max over the 128-row groups of rows [s0, s0 + rows) of a column-max array cm[group][ld]
// (eight groups' loads in flight at a time: a split of 1024 rows is one round trip, not eight)
__device__ __forceinline__ float tn_colmax(const float* cm, int ld, size_t s0, int rows, int col) {
    float m = 0.f;
    int g = (int)(s0 / 128);
    const int g1 = (int)((s0 + rows) / 128);
    for (; g + 8 <= g1; g += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = cm[(size_t)(g + u) * ld + col];
#pragma unroll
        for (int u = 0; u < 8; ++u) m = fmaxf(m, v[u]);
    }
    for (; g < g1; ++g) m = fmaxf(m, cm[(size_t)g * ld + col]);
    return m;
}

}  // namespace nerf
