// 4x4 row-major helpers shared by the ray prologue (rays.hip) and the pair terms (pair.hip).
#pragma once
#include "common.hpp"

namespace nerf {

// 4x4 helpers (row-major)
__device__ __forceinline__ void load4(const float* __restrict__ p, float a[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = p[i];
}
__device__ __forceinline__ void store4(float* __restrict__ p, const float a[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) p[i] = a[i];
}
__device__ __forceinline__ void matmul4(const float a[16], const float b[16], float c[16]) {
#pragma clang fp contract(off)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float s = a[4 * i] * b[j];
#pragma unroll
            for (int k = 1; k < 4; ++k) s = s + a[4 * i + k] * b[4 * k + j];
            c[4 * i + j] = s;
        }
}

// Gauss-Jordan elimination with partial pivoting (first maximal |pivot|, as getrf picks)
__device__ inline void inverse4(const float in[16], float out[16]) {
#pragma clang fp contract(off)
    float a[4][4], b[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            a[i][j] = in[4 * i + j];
            b[i][j] = i == j ? 1.f : 0.f;
        }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        int p = c;
        float best = fabsf(a[c][c]);
#pragma unroll
        for (int r = c + 1; r < 4; ++r)
            if (fabsf(a[r][c]) > best) { best = fabsf(a[r][c]); p = r; }
        if (p != c) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float t = a[c][j]; a[c][j] = a[p][j]; a[p][j] = t;
                t = b[c][j]; b[c][j] = b[p][j]; b[p][j] = t;
            }
        }
        const float piv = a[c][c];
#pragma unroll
        for (int j = 0; j < 4; ++j) { a[c][j] = a[c][j] / piv; b[c][j] = b[c][j] / piv; }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (r == c) continue;
            const float f = a[r][c];
#pragma unroll
            for (int j = 0; j < 4; ++j) { a[r][j] = a[r][j] - f * a[c][j]; b[r][j] = b[r][j] - f * b[c][j]; }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) out[4 * i + j] = b[i][j];
}

}  // namespace nerf
