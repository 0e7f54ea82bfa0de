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

// Streams an encoding row to global memory 16 bytes at a time (keeps few values live).
template <int W>
struct RowWriter {
    float4* dst;
    float buf[4];
    int n;
    float amax;   // max |v| of the row (row scale of GEMM precision mode 2)
    __device__ __forceinline__ void put(float v) {
        amax = fmaxf(amax, fabsf(v));
        buf[n & 3] = v;
        ++n;
        if ((n & 3) == 0) dst[(n >> 2) - 1] = make_float4(buf[0], buf[1], buf[2], buf[3]);
    }
    __device__ __forceinline__ void finish() {
        while (n < W) put(0.f);
    }
};

// encode_position (official_nerf.py:99-119): [x, sin(2^0 x), cos(2^0 x), ...], zero padded to W
template <int L, int W>
__device__ __forceinline__ float encode3(const float x[3], float* row) {
    RowWriter<W> w{reinterpret_cast<float4*>(row), {0.f, 0.f, 0.f, 0.f}, 0, 0.f};
#pragma unroll
    for (int c = 0; c < 3; ++c) w.put(x[c]);
#pragma unroll
    for (int i = 0; i < L; ++i) {
        const float f = (float)(1 << i);
        float s[3], co[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) sincosf(f * x[c], &s[c], &co[c]);
#pragma unroll
        for (int c = 0; c < 3; ++c) w.put(s[c]);
#pragma unroll
        for (int c = 0; c < 3; ++c) w.put(co[c]);
    }
    w.finish();
    return w.amax;
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

}  // namespace nerf
