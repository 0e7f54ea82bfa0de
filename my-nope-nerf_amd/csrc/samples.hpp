// Per-sample device helpers shared by the render kernels (render.hip) and the fused
// per-ray eval kernel (chain.hip): sample positions, positional encoding, the density /
// colour activations of the composite.
//
// Reference semantics: model/rendering.py:113-198, model/official_nerf.py:66-119.
#pragma once
#include "common.hpp"

namespace nerf {

constexpr int ENC_P = 64;  // 63 used + 1 zero pad (L = 10)
constexpr int ENC_D = 64;  // 27 used + 37 zero pad (L = 4); 64 wide so every GEMM K tile is whole

// Sample positions are rounded exactly as eager torch rounds them (separate multiply and
// add, never fused).  HIP's __fmul_rn/__fadd_rn are plain operators inside the header, where
// -ffp-contract=fast still fuses them, so these helpers use plain operators under
// `#pragma clang fp contract(off)` instead.

// torch.linspace(0, 1, S) element i (CUDA kernel: halfway split, float step)
__device__ __forceinline__ float linspace01(int i, int S) {
#pragma clang fp contract(off)
    if (S == 1) return 0.f;
    const float step = 1.0f / (float)(S - 1);
    return (i < S / 2) ? step * (float)i : 1.0f - step * (float)(S - 1 - i);
}
// depth_range[0] * (1 - t) + depth_range[1] * t   (rendering.py:186)
__device__ __forceinline__ float lerp_z(float t, float nz, float fz) {
#pragma clang fp contract(off)
    return nz * (1.0f - t) + fz * t;
}
// stratified jitter inside the bin (rendering.py:187-191)
__device__ __forceinline__ float jitter_z(float z, float zp, float zn, bool first, bool last, float u) {
#pragma clang fp contract(off)
    const float lo = first ? z : 0.5f * (z + zp);
    const float hi = last ? z : 0.5f * (zn + z);
    return lo + (hi - lo) * u;
}
__device__ __forceinline__ float ray_point(float o, float d, float z) {
#pragma clang fp contract(off)
    return o + d * z;
}

enum { F_DIST_ALPHA = 1, F_WHITE_BKGD = 2, F_RELU = 4 };
constexpr float kEps = 1e-6f;  // rendering.py:9

__device__ __forceinline__ float f_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float f_sigmoid(float x) { return f_rcp(1.f + __expf(-x)); }
// torch softplus(beta=1, threshold=20) and its derivative z / (z + 1)
__device__ __forceinline__ float f_softplus(float x) { return x > 20.f ? x : __logf(1.f + __expf(x)); }
__device__ __forceinline__ float f_softplus_grad(float x) {
    if (x > 20.f) return 1.f;
    const float z = __expf(x);
    return z * f_rcp(z + 1.f);
}
__device__ __forceinline__ float f_density(float raw, int flags) {
    return (flags & F_RELU) ? fmaxf(raw, 0.f) : f_softplus(raw);
}

// DPP row (16-lane) scans and sums of the composite kernels: a DPP row is one ray
template <int CTRL>
__device__ __forceinline__ float dpp_f(float old, float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                                                  CTRL, 0xF, 0xF, false));
}
// inclusive product scan over each 16-lane row (row_shr n; lanes without a source keep 1)
__device__ __forceinline__ float row_scan_mul(float v) {
    v *= dpp_f<0x111>(1.f, v);
    v *= dpp_f<0x112>(1.f, v);
    v *= dpp_f<0x114>(1.f, v);
    v *= dpp_f<0x118>(1.f, v);
    return v;
}
// inclusive suffix sum over each 16-lane row (row_shl n)
__device__ __forceinline__ float row_suffix_add(float v) {
    v += dpp_f<0x101>(0.f, v);
    v += dpp_f<0x102>(0.f, v);
    v += dpp_f<0x104>(0.f, v);
    v += dpp_f<0x108>(0.f, v);
    return v;
}
// sum over each 16-lane row, in every lane (quad_perm [1,0,3,2], [2,3,0,1], half-mirror, mirror)
__device__ __forceinline__ float row_sum(float v) {
    v += dpp_f<0xB1>(0.f, v);
    v += dpp_f<0x4E>(0.f, v);
    v += dpp_f<0x141>(0.f, v);
    v += dpp_f<0x140>(0.f, v);
    return v;
}


}  // namespace nerf
