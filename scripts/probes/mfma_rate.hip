// Calibration probe: sustained v_mfma_f32_32x32x16_bf16 rate on the whole chip.
//   mode 0: operands in registers, 16 independent accumulators per wave
//   mode 1: + 1 ds_read_b128 per 4 MFMAs (fragment re-read from LDS, conflict-free)
//   mode 2: 6-deep dependent chains per accumulator (the split-bf16 product order)
// Grid: 1024 blocks x 256 threads (4 waves/CU resident = 1 per SIMD), random operands.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int MODE>
__global__ __launch_bounds__(256) void k_probe(const uint4* __restrict__ src, float* out, int iters) {
    __shared__ uint4 lds[4096];
    for (int i = threadIdx.x; i < 4096; i += 256) lds[i] = src[(blockIdx.x * 4096 + i) & 65535];
    __syncthreads();
    uint4 a = src[threadIdx.x], b = src[threadIdx.x + 256];
    f32x16 acc[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint4 ai = a;
            if (MODE == 1) ai = lds[(w * 1024 + (it & 7) * 128 + i * 64 + lane) & 4095];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (MODE == 2) {
#pragma unroll
                    for (int q = 0; q < 6; ++q)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ai),
                                                                            __builtin_bit_cast(bf16x8, b), acc[i][j], 0, 0, 0);
                } else {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ai),
                                                                        __builtin_bit_cast(bf16x8, b), acc[i][j], 0, 0, 0);
                }
            }
        }
    }
    float t = 0.f;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            for (int r = 0; r < 16; ++r) t += acc[i][j][r];
    out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int MODE>
static void run(const uint4* src, float* out, int iters) {
    const int blocks = 1024;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_probe<MODE>, dim3(blocks), dim3(256), 0, 0, src, out, iters);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_probe<MODE>, dim3(blocks), dim3(256), 0, 0, src, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double mfma = (double)blocks * 4 * iters * 16 * (MODE == 2 ? 6 : 1);
        const double tf = mfma * 32768.0 / (ms * 1e-3) / 1e12;
        printf("mode %d: %.3f ms  %.0f TF/s bf16 (%.1f%% of 2516.6)\n", MODE, ms, tf, 100 * tf / 2516.6);
    }
}

int main() {
    uint4* src;
    float* out;
    hipMalloc(&src, 65536 * 16);
    hipMalloc(&out, 1024 * 256 * 4);
    uint32_t* h = (uint32_t*)malloc(65536 * 16);
    uint32_t x = 12345;
    for (int i = 0; i < 65536 * 4; ++i) {   // random bf16 pairs in [-1, 1)
        x = x * 1664525u + 1013904223u;
        const uint32_t lo = 0x3f00u | ((x >> 9) & 0x7f) | ((x & 1) << 15);
        const uint32_t hi = 0x3e80u | ((x >> 17) & 0x7f) | ((x & 2) << 14);
        h[i] = lo | (hi << 16);
    }
    hipMemcpy(src, h, 65536 * 16, hipMemcpyHostToDevice);
    run<0>(src, out, 2000);
    run<1>(src, out, 2000);
    run<2>(src, out, 400);
    return 0;
}
