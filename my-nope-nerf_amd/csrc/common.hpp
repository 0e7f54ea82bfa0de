// Shared helpers for the nerf_hip C-ABI (error reporting, argument checks, wave utilities).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdarg>

#include "../../include/nerf_hip.h"

namespace nerf {

// thread-local last error message (nerf_hip_last_error)
void set_error(const char* fmt, ...);

#define NERF_CHECK(cond, ...)                     \
    do {                                          \
        if (!(cond)) {                            \
            ::nerf::set_error(__VA_ARGS__);       \
            return NERF_EINVAL;                   \
        }                                         \
    } while (0)

#define NERF_CHECK_PTR(p) NERF_CHECK((p) != nullptr, "%s: null pointer '%s'", __func__, #p)
#define NERF_CHECK_ALIGN16(p) \
    NERF_CHECK((((uintptr_t)(p)) & 15u) == 0, "%s: pointer '%s' not 16-byte aligned", __func__, #p)

inline int check_launch(const char* fn) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", fn, hipGetErrorString(e));
        return NERF_ELAUNCH;
    }
    return NERF_OK;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// GEMM timing hooks (capi.cpp): kind = NERF_PROF_FWD / _DX / _DW; flops and bytes are the
// launch's algorithmic f32 FLOPs and HBM bytes; products = MFMA products per f32 product
// (1 exact f32, 6 bf16x6, 3 f16x3) -- it prices the launch against its MFMA peak
// prof_next: set by the C-ABI entry before it dispatches (kind, algorithmic bytes)
void prof_next(int kind, double bytes);
void prof_begin(hipStream_t s);
void prof_end(hipStream_t s, double flops, int products);

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// row max -> the power-of-two exponent e with max 2^e in [2^14, 2^15) (0 for a zero row):
// the row scale of GEMM precision mode 2 (fp16 pair operands)
__device__ __forceinline__ int row_exp(float rmax) {
    const int ex = (int)((__float_as_uint(rmax) >> 23) & 0xff);
    return rmax == 0.f ? 0 : (ex ? 141 - ex : 140);
}

// the chain images' K order (nerf_pack_weights dst_cs / dst_cts): image column c of a 32-wide
// k-step holds feature chain_perm(c) -- lane group g's eight k (c = 8 g + i) are features 4 g
// + i (i < 4) and 16 + 4 g + i - 4 of the step, the tile layout of the 16x16x32 accumulators
__host__ __device__ constexpr int chain_perm(int c) {
    const int t = c >> 5, q = c & 31, g = q >> 3, i = q & 7;
    return 32 * t + 4 * g + (i & 3) + (i >= 4 ? 16 : 0);
}

// GEMM arithmetic mode (nerf_gemm_set_precision), host side
int gemm_precision();
// several split-K slab reduces (nerf_slab_reduce without accumulate) in one launch
constexpr int kSlabJobsMax = 12;   // ten layers + the two head-weight reduces
struct SlabJobDesc {
    const float* slab;
    int splits, nout, ldslab, nout_ref, kin_ref;
    const float* bslab;
    float* gw;
    float* gb;
};
int slab_reduce_jobs(const SlabJobDesc* d, int n, hipStream_t s);
// the chain backward's head-weight partials (render.hip k_heads_part: hidden 256, colour 128) into
// `part` (heads_part_blocks(n) x 644 floats) and the two slab-reduce jobs that finish them
int heads_part_blocks(int n);
int heads_partials(const float* graw4, const float* h8, int ld8, const float* hr, int ldr, int n, float* part,
                   float* gwd, float* gbd, float* gwc, float* gbc, SlabJobDesc (&jobs)[2], hipStream_t s);
constexpr int kWgradPairsMax = 8;
constexpr int kWgradJobsMax = 8;   // jobs of one k_wgrad_jobs launch
// two 256 x 64 weight gradients over the position encoding in one launch (l4's enc_p segment and
// l0, nerf_linear_bwd_weight's arguments each): a's splits first, then b's, on the 4-wave kernel
int wgrad_narrow_pair(const float* dy_a, int lddy_a, const float* x_a, int ldx_a, int splits_a, float* slab_a,
                      int ldslab_a, int col0_a, float* bslab_a, const float* dcm_a, const float* xcm_a,
                      const float* dy_b, int lddy_b, const float* x_b, int ldx_b, int splits_b, float* slab_b,
                      int ldslab_b, int col0_b, float* bslab_b, const float* dcm_b, const float* xcm_b, int m,
                      hipStream_t s);

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// torch.nn.functional.softplus(x, beta=1, threshold=20)
__device__ __forceinline__ float softplus_f(float x) { return x > 20.f ? x : log1pf(expf(x)); }
// its derivative as torch computes it (z = exp(x); z / (z + 1)), 1 above the threshold
__device__ __forceinline__ float softplus_grad_f(float x) {
    if (x > 20.f) return 1.f;
    float z = expf(x);
    return z / (z + 1.f);
}
__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + expf(-x)); }

}  // namespace nerf
