// Per-sample and per-ray kernels of the render path: stratified samples +
// positional encoding, output heads, fused sigma->alpha->transmittance compositing
// (forward/backward) and the gradient back to the ray inputs.
//
// Reference semantics: model/rendering.py:36-198, model/official_nerf.py:66-119.
#include "samples.hpp"

namespace nerf {

// Four threads per sample, 128 samples (one 128-row group) per block.  Each row is built in
// LDS (65-float stride: the per-thread scalar writes are conflict-free) and then copied out
// as whole 256-byte rows, 16 lanes x float4 per row: a thread-per-row float4 store touches 64
// rows' lines per wave instruction, which held the 67 MB of encodings at ~1.5 TB/s.
constexpr int ENC_ROWS = 128, ENC_LD = 65, ENC_THREADS = 4 * ENC_ROWS;

// encode_position (official_nerf.py:99-119) of one sample into its LDS row; returns max |.|
template <int L, int W>
__device__ __forceinline__ float encode3_lds(const float x[3], float* row) {
    float m = 0.f;
    int k = 0;
    auto put = [&](float v) { row[k++] = v; m = fmaxf(m, fabsf(v)); };
#pragma unroll
    for (int c = 0; c < 3; ++c) put(x[c]);
#pragma unroll
    for (int i = 0; i < L; ++i) {
        const float f = (float)(1 << i);
        float sn[3], co[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) sincosf(f * x[c], &sn[c], &co[c]);
#pragma unroll
        for (int c = 0; c < 3; ++c) put(sn[c]);
#pragma unroll
        for (int c = 0; c < 3; ++c) put(co[c]);
    }
#pragma unroll
    for (int c = 3 + 6 * L; c < W; ++c) row[c] = 0.f;
    return m;
}

// (plain stores: the forward chain reads the encodings next; non-temporal ones made it slower,
// 538-543 vs 526-530 us, profiles/r05/nt_loads_ab.txt)
__device__ __forceinline__ void enc_st4(float* d, const float4& v) {
    *reinterpret_cast<float4*>(d) = v;
}
// the block's 128 LDS rows -> rows m0 .. m0 + 127 of a [n][64] encoding, coalesced
__device__ __forceinline__ void enc_copy_out(const float* lds, float* dst, size_t m0) {
#pragma unroll
    for (int it = 0; it < ENC_ROWS * 16 / ENC_THREADS; ++it) {
        const int idx = it * ENC_THREADS + threadIdx.x;
        const int row = idx >> 4, c4 = (idx & 15) * 4;
        const float* src = lds + row * ENC_LD + c4;
        enc_st4(dst + (m0 + row) * 64 + c4, make_float4(src[0], src[1], src[2], src[3]));
    }
}

// the view-direction encodings of the block's rays (one LDS record per ray, slot r - r0) ->
// rows m0 .. m0 + 127 of the [n][64] enc_d: every sample row repeats its ray's record, rows
// past the last sample are zeros
__device__ __forceinline__ void enc_copy_out_rays(const float* rec, float* dst, size_t m0, int S, int r0,
                                                  int total) {
#pragma unroll
    for (int it = 0; it < ENC_ROWS * 16 / ENC_THREADS; ++it) {
        const int idx = it * ENC_THREADS + threadIdx.x;
        const int row = idx >> 4, c4 = (idx & 15) * 4;
        const int s = (int)m0 + row;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (s < total) {
            const float* src = rec + (s / S - r0) * ENC_LD + c4;
            v = make_float4(src[0], src[1], src[2], src[3]);
        }
        enc_st4(dst + (m0 + row) * 64 + c4, v);
    }
}

// 128 samples per block, four threads per sample (part = threadIdx.x >> 7, wave-uniform): part 0
// the coordinates and frequencies 0-2, part 1 3-5, part 2 6-7, part 3 8-9 of the position
// encoding (official_nerf.py:99-119) -- the per-thread sincosf chain a quarter as long and four
// times the waves to hide it (one thread per sample: ~32 us per cfg2 step)
__global__ __launch_bounds__(ENC_THREADS) void k_encode_samples(const float* __restrict__ po, const float* __restrict__ pd,
                                 const float* __restrict__ view, const float* __restrict__ noise,
                                 int R, int S, int n_pad, float nz, float fz,
                                 float* __restrict__ z_out, float* __restrict__ enc_p,
                                 float* __restrict__ enc_d, float* __restrict__ rmax_p,
                                 float* __restrict__ rmax_d, float* __restrict__ cmax_p,
                                 float* __restrict__ cmax_d) {
    static_assert(ENC_P == 64 && ENC_D == 64, "row copies assume 64-wide encodings");
    __shared__ float rows[ENC_ROWS * ENC_LD];
    __shared__ float wm[2][6];
    __shared__ uint32_t lmdu[ENC_ROWS];   // max |enc_d| per ray slot (float bits)
    __shared__ float lmp[4][ENC_ROWS];   // max |enc_p| per part and row
    const size_t m0 = (size_t)blockIdx.x * ENC_ROWS;
    const int row = threadIdx.x & (ENC_ROWS - 1), part = threadIdx.x >> 7;
    const int s = (int)m0 + row;
    const int total = R * S;
    float* lrow = rows + row * ENC_LD;
    float ax[3] = {0.f, 0.f, 0.f}, av[3] = {0.f, 0.f, 0.f};   // |coordinates| (column bounds)
    float x[3] = {0.f, 0.f, 0.f}, v[3] = {0.f, 0.f, 0.f};
    const bool live = s < total;
    float z = 0.f;
    if (live) {
        const int r = s / S, i = s - r * S;
        z = lerp_z(linspace01(i, S), nz, fz);
        if (noise != nullptr) {  // rendering.py:187-191
            const float zp = i > 0 ? lerp_z(linspace01(i - 1, S), nz, fz) : z;
            const float zn = i < S - 1 ? lerp_z(linspace01(i + 1, S), nz, fz) : z;
            z = jitter_z(z, zp, zn, i == 0, i == S - 1, noise[s]);
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            x[c] = ray_point(po[3 * r + c], pd[3 * r + c], z);  // rendering.py:193-194
            v[c] = view[3 * r + c];
            ax[c] = fabsf(x[c]);
            av[c] = fabsf(v[c]);
        }
    }
    // this part's columns of the position encoding row (padding rows: zeros, max 0)
    float mp = 0.f;
    const int lv0 = part == 0 ? 0 : part == 1 ? 3 : part == 2 ? 6 : 8;
    const int lv1 = part == 0 ? 3 : part == 1 ? 6 : part == 2 ? 8 : 10;
    if (part == 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) { lrow[c] = x[c]; mp = fmaxf(mp, fabsf(x[c])); }
    }
    if (part == 3) lrow[63] = 0.f;
    for (int lv = lv0; lv < lv1; ++lv) {
        const float f = (float)(1 << lv);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float sn = 0.f, co = 0.f;
            if (live) sincosf(f * x[c], &sn, &co);
            lrow[3 + 6 * lv + c] = sn;
            lrow[6 + 6 * lv + c] = co;
            mp = fmaxf(mp, fmaxf(fabsf(sn), fabsf(co)));
        }
    }
    lmp[part][row] = mp;
    if (part == 0) lmdu[row] = 0u;
    if (part == 0 && s < n_pad) z_out[s] = z;
    __syncthreads();
    if (part == 0 && s < n_pad && rmax_p)
        rmax_p[s] = fmaxf(fmaxf(lmp[0][row], lmp[1][row]), fmaxf(lmp[2][row], lmp[3][row]));
    enc_copy_out(rows, enc_p, m0);
    __syncthreads();
    // the view-direction encoding is per ray (official_nerf.py:87 encodes the ray's direction,
    // repeated over its samples): the block's first sample of each ray encodes it once into
    // that ray's LDS record (slot r - r0 < 128), the copy-out repeats it per sample row --
    // the same sincosf on the same input, so enc_d is bit-identical to a per-sample encode
    // one thread per (ray slot, column), so the slot's sincosf run side by side: the values of
    // encode3_lds<4, ENC_D> (the same sincosf on the same input), its max by an LDS max on the
    // bits (non-negative floats order like their bits)
    const int r0 = (int)(m0 / (size_t)S);
    const int nslot = (int)m0 < total ? min((int)((m0 + ENC_ROWS - 1) / (size_t)S), R - 1) - r0 + 1 : 0;
    for (int idx = threadIdx.x; idx < nslot * 64; idx += ENC_THREADS) {
        const int slot = idx >> 6, col = idx & 63;
        float val = 0.f;
        if (col < 3) {
            val = view[3 * (size_t)(r0 + slot) + col];
        } else if (col < 3 + 6 * 4) {
            const int lv = (col - 3) / 6, w = (col - 3) % 6, c = w % 3;
            float sn, co;
            sincosf((float)(1 << lv) * view[3 * (size_t)(r0 + slot) + c], &sn, &co);
            val = w < 3 ? sn : co;
        }
        rows[slot * ENC_LD + col] = val;
        atomicMax(&lmdu[slot], __float_as_uint(fabsf(val)));
    }
    __syncthreads();
    if (part == 0) {
        const float md = live ? __uint_as_float(lmdu[s / S - r0]) : 0.f;
        if (s < n_pad && rmax_d) rmax_d[s] = md;
    }
    enc_copy_out_rays(rows, enc_d, m0, S, r0, total);
    if (cmax_p != nullptr) {
        // per 128-row group (this block): exact max of the coordinate columns (wave max over the
        // part-0 waves, then the two waves in LDS), 1 for the sin / cos columns (|sin|, |cos| <=
        // 1), 0 for the pad
        const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
        if (part == 0) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    ax[c] = fmaxf(ax[c], __shfl_xor(ax[c], off, 64));
                    av[c] = fmaxf(av[c], __shfl_xor(av[c], off, 64));
                }
            }
            if (l == 0)
#pragma unroll
                for (int c = 0; c < 3; ++c) { wm[w][c] = ax[c]; wm[w][3 + c] = av[c]; }
        }
        __syncthreads();
        if (w == 0) {
            float vp, vd;
            if (l < 3) {
                vp = fmaxf(wm[0][l], wm[1][l]);
                vd = fmaxf(wm[0][3 + l], wm[1][3 + l]);
            } else {
                vp = l < 63 ? 1.f : 0.f;
                vd = l < 27 ? 1.f : 0.f;
            }
            cmax_p[blockIdx.x * ENC_P + l] = vp;
            cmax_d[blockIdx.x * ENC_D + l] = vd;
        }
    }
}

// ---------------------------------------------------------------------------
// Output heads.  A wave processes 16 consecutive samples; lane l owns features
// l, l+64, ...; the 16 per-sample partial dots are reduced across the wave by a
// halving butterfly (17 shuffles for 16 samples) that leaves the total of sample
// (lane >> 2) in every lane.
// ---------------------------------------------------------------------------
template <bool MAX = false>
__device__ __forceinline__ float reduce16(float (&v)[16]) {
    auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : a + b; };
    const int lane = lane_id();
    float w8[8], w4[4], w2[2];
    {
        const bool h = (lane >> 5) & 1;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float keep = h ? v[j + 8] : v[j];
            const float send = h ? v[j] : v[j + 8];
            w8[j] = op(keep, __shfl_xor(send, 32, 64));
        }
    }
    {
        const bool h = (lane >> 4) & 1;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float keep = h ? w8[j + 4] : w8[j];
            const float send = h ? w8[j] : w8[j + 4];
            w4[j] = op(keep, __shfl_xor(send, 16, 64));
        }
    }
    {
        const bool h = (lane >> 3) & 1;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float keep = h ? w4[j + 2] : w4[j];
            const float send = h ? w4[j] : w4[j + 2];
            w2[j] = op(keep, __shfl_xor(send, 8, 64));
        }
    }
    const bool h = (lane >> 2) & 1;
    float w = op(h ? w2[1] : w2[0], __shfl_xor(h ? w2[0] : w2[1], 4, 64));
    w = op(w, __shfl_xor(w, 2, 64));
    w = op(w, __shfl_xor(w, 1, 64));
    return w;
}

template <int NH, int NR>  // NH = hidden/64, NR = rgb-hidden/64
__global__ __launch_bounds__(256) void k_heads_fwd(const float* __restrict__ h8, int ld8,
                                                   const float* __restrict__ hr, int ldr,
                                                   const float* __restrict__ wd, const float* __restrict__ bd,
                                                   const float* __restrict__ wc, const float* __restrict__ bc,
                                                   float* __restrict__ raw4, int n_pad) {
    const int lane = lane_id();
    const int gwave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nwaves = (gridDim.x * blockDim.x) >> 6;
    float wdr[NH], wcr[3][NR];
#pragma unroll
    for (int q = 0; q < NH; ++q) wdr[q] = wd[lane + 64 * q];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int q = 0; q < NR; ++q) wcr[c][q] = wc[c * NR * 64 + lane + 64 * q];
    const float b_d = bd[0];
    const float b_c[3] = {bc[0], bc[1], bc[2]};

    for (int g = gwave; g * 16 < n_pad; g += nwaves) {
        const size_t s0 = (size_t)g * 16;
        float pd[16], pc0[16], pc1[16], pc2[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            float a = 0.f;
#pragma unroll
            for (int q = 0; q < NH; ++q) a += h8[(s0 + t) * ld8 + lane + 64 * q] * wdr[q];
            pd[t] = a;
            float c0 = 0.f, c1 = 0.f, c2 = 0.f;
#pragma unroll
            for (int q = 0; q < NR; ++q) {
                const float x = hr[(s0 + t) * ldr + lane + 64 * q];
                c0 += x * wcr[0][q];
                c1 += x * wcr[1][q];
                c2 += x * wcr[2][q];
            }
            pc0[t] = c0; pc1[t] = c1; pc2[t] = c2;
        }
        const float sd = reduce16(pd);
        const float s0c = reduce16(pc0);
        const float s1c = reduce16(pc1);
        const float s2c = reduce16(pc2);
        if ((lane & 3) == 0) {
            const size_t s = s0 + (lane >> 2);
            *reinterpret_cast<float4*>(raw4 + 4 * s) =
                make_float4(sd + b_d, s0c + b_c[0], s1c + b_c[1], s2c + b_c[2]);
        }
    }
}

// the head partials' h8 / hr loads are non-temporal: cfg2 step 2.021 vs 2.035 ms in three
// interleaved rounds, profiles/r05/nt_loads_ab.txt (the same hint on the weight-gradient stage
// loads made those 9-27 % slower)
__device__ __forceinline__ float heads_ld(const float* a) {
    return __builtin_nontemporal_load(a);
}
// part layout per block: [wd: 64*NH][wc: 3*64*NR][bd, bc0, bc1, bc2]
// MODE bit 0: dyr and its row / column maxima (the input-gradient chain waits for these);
// bit 1: the head-weight / bias partials (read h8 and hr; nothing downstream waits for them
// until the optimizer, so the backward runs them on a side stream)
// MB (mode 1 only): the ReLU gate of dyr from the colour layer's mask bits [n][ldm] (bit =
// hr > 0, written by its forward) instead of re-reading hr
template <int NH, int NR, int MODE = 3, bool MB = false>
__global__ __launch_bounds__(256) void k_heads_bwd(const float* __restrict__ graw4,
                                                   const float* __restrict__ h8, int ld8,
                                                   const float* __restrict__ hr, int ldr,
                                                   const uint32_t* __restrict__ hmask, int ldm,
                                                   const float* __restrict__ wc,
                                                   float* __restrict__ dyr, int lddyr,
                                                   float* __restrict__ part, int n_pad,
                                                   float* __restrict__ dyr_rmax, float* __restrict__ dyr_cmax) {
    constexpr int H = 64 * NH, HR = 64 * NR, PART = H + 3 * HR + 4;
    __shared__ float red[4][PART];
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    const int gwave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nwaves = (gridDim.x * blockDim.x) >> 6;
    float wcr[3][NR];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int q = 0; q < NR; ++q) wcr[c][q] = wc[c * HR + lane + 64 * q];
    float awd[NH], awc[3][NR], abd = 0.f, abc[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NH; ++q) awd[q] = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int q = 0; q < NR; ++q) awc[c][q] = 0.f;

    // each wave walks whole 128-row chunks (8 groups of 16 samples) so that the column
    // maxima of dyr (mode 2 scales) come out per chunk without atomics
    for (int ch = gwave; ch * 128 < n_pad; ch += nwaves) {
      float cm[NR];
#pragma unroll
      for (int q = 0; q < NR; ++q) cm[q] = 0.f;
      for (int g = ch * 8; g < ch * 8 + 8 && g * 16 < n_pad; ++g) {
        const size_t s0 = (size_t)g * 16;
        float dm[16];   // this lane's max |dyr| per sample of the group
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const size_t s = s0 + t;
            const float4 gr = *reinterpret_cast<const float4*>(graw4 + 4 * s);
            if constexpr (MODE & 2) {
#pragma unroll
                for (int q = 0; q < NH; ++q) awd[q] = fmaf(gr.x, heads_ld(h8 + s * ld8 + lane + 64 * q), awd[q]);
            }
            float dmax = 0.f;
#pragma unroll
            for (int q = 0; q < NR; ++q) {
                static_assert(!MB || MODE == 1, "mask-bit gate: dyr-only mode");
                const float x = MB ? 0.f : heads_ld(hr + s * ldr + lane + 64 * q);
                const bool on = MB ? ((hmask[s * ldm + ((lane + 64 * q) >> 5)] >> (lane & 31)) & 1u) != 0 : x > 0.f;
                if constexpr (MODE & 1) {
                    // explicit fmas: every MODE instantiation rounds identically
                    float d = fmaf(gr.w, wcr[2][q], fmaf(gr.z, wcr[1][q], gr.y * wcr[0][q]));
                    d = on ? d : 0.f;
                    dyr[s * lddyr + lane + 64 * q] = d;
                    dmax = fmaxf(dmax, fabsf(d));
                    cm[q] = fmaxf(cm[q], fabsf(d));
                }
                if constexpr (MODE & 2) {
                    awc[0][q] = fmaf(gr.y, x, awc[0][q]);
                    awc[1][q] = fmaf(gr.z, x, awc[1][q]);
                    awc[2][q] = fmaf(gr.w, x, awc[2][q]);
                }
            }
            dm[t] = dmax;
            if constexpr (MODE & 2) {
                abd += gr.x;
                abc[0] += gr.y; abc[1] += gr.z; abc[2] += gr.w;
            }
        }
        if ((MODE & 1) && dyr_rmax) {   // row maxima of dyr (row scales of GEMM precision mode 2): one butterfly per group
            const float m = reduce16<true>(dm);
            if ((lane & 3) == 0) dyr_rmax[s0 + (lane >> 2)] = m;
        }
      }
      if ((MODE & 1) && dyr_cmax)
#pragma unroll
        for (int q = 0; q < NR; ++q) dyr_cmax[(size_t)ch * HR + lane + 64 * q] = cm[q];
    }
    if constexpr (!(MODE & 2)) return;
    float* rw = red[wave];
#pragma unroll
    for (int q = 0; q < NH; ++q) rw[lane + 64 * q] = awd[q];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int q = 0; q < NR; ++q) rw[H + c * HR + lane + 64 * q] = awc[c][q];
    if (lane == 0) {
        rw[H + 3 * HR + 0] = abd;
        rw[H + 3 * HR + 1] = abc[0];
        rw[H + 3 * HR + 2] = abc[1];
        rw[H + 3 * HR + 3] = abc[2];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < PART; e += blockDim.x)
        part[(size_t)blockIdx.x * PART + e] = red[0][e] + red[1][e] + red[2][e] + red[3][e];
}

// MODE 1 alone (dyr + its maxima, on the input-gradient chain): one block per 128-row chunk,
// each wave two 16-sample groups, the chunk's column maxima combined over the 4 waves in LDS.
// k_heads_bwd<.., 1, ..> gives a wave a whole chunk (1024 waves at cfg2, one per SIMD): its
// store stream then waits on one load latency per group; here 4x the waves are resident.  The
// arithmetic is k_heads_bwd's (same fmas, maxima are order-free), so dyr is bit-identical.
template <int NR, bool MB>
__global__ __launch_bounds__(256) void k_heads_dyr(const float* __restrict__ graw4,
                                                   const float* __restrict__ hr, int ldr,
                                                   const uint32_t* __restrict__ hmask, int ldm,
                                                   const float* __restrict__ wc,
                                                   float* __restrict__ dyr, int lddyr,
                                                   float* __restrict__ dyr_rmax, float* __restrict__ dyr_cmax) {
    constexpr int HR = 64 * NR;
    __shared__ float lcm[4][HR];
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    const size_t ch = blockIdx.x;
    float wcr[3][NR], cm[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q) {
        wcr[0][q] = wc[lane + 64 * q];
        wcr[1][q] = wc[HR + lane + 64 * q];
        wcr[2][q] = wc[2 * HR + lane + 64 * q];
        cm[q] = 0.f;
    }
#pragma unroll
    for (int gg = 0; gg < 2; ++gg) {
        const size_t s0 = (ch * 8 + 2 * wave + gg) * 16;
        float dm[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const size_t s = s0 + t;
            const float4 gr = *reinterpret_cast<const float4*>(graw4 + 4 * s);
            float dmax = 0.f;
#pragma unroll
            for (int q = 0; q < NR; ++q) {
                const bool on = MB ? ((hmask[s * ldm + ((lane + 64 * q) >> 5)] >> (lane & 31)) & 1u) != 0
                                   : hr[s * ldr + lane + 64 * q] > 0.f;
                float d = fmaf(gr.w, wcr[2][q], fmaf(gr.z, wcr[1][q], gr.y * wcr[0][q]));
                d = on ? d : 0.f;
                dyr[s * lddyr + lane + 64 * q] = d;
                dmax = fmaxf(dmax, fabsf(d));
                cm[q] = fmaxf(cm[q], fabsf(d));
            }
            dm[t] = dmax;
        }
        if (dyr_rmax) {
            const float m = reduce16<true>(dm);
            if ((lane & 3) == 0) dyr_rmax[s0 + (lane >> 2)] = m;
        }
    }
    if (dyr_cmax) {
#pragma unroll
        for (int q = 0; q < NR; ++q) lcm[wave][lane + 64 * q] = cm[q];
        __syncthreads();
        for (int e = threadIdx.x; e < HR; e += blockDim.x)
            dyr_cmax[ch * HR + e] = fmaxf(fmaxf(lcm[0][e], lcm[1][e]), fmaxf(lcm[2][e], lcm[3][e]));
    }
}

// sum the per-block partials: a block per 64 partial elements, its 4 waves split the block
// range and combine through LDS
__global__ __launch_bounds__(256) void k_heads_reduce(const float* __restrict__ part, int nblocks, int H, int HR,
                                                      float* __restrict__ gwd, float* __restrict__ gbd,
                                                      float* __restrict__ gwc, float* __restrict__ gbc,
                                                      int accumulate) {
    __shared__ float red[4][64];
    const int PART = H + 3 * HR + 4;
    const int e = blockIdx.x * 64 + (threadIdx.x & 63);
    const int w = threadIdx.x >> 6;
    float a0 = 0.f, a1 = 0.f;
    if (e < PART) {
        int b = w;
        for (; b + 4 < nblocks; b += 8) {
            a0 += part[(size_t)b * PART + e];
            a1 += part[(size_t)(b + 4) * PART + e];
        }
        for (; b < nblocks; b += 4) a0 += part[(size_t)b * PART + e];
    }
    red[w][threadIdx.x & 63] = a0 + a1;
    __syncthreads();
    if (w == 0 && e < PART) {
        const float acc = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
        float* dst;
        if (e < H) dst = gwd + e;
        else if (e < H + 3 * HR) dst = gwc + (e - H);
        else if (e == H + 3 * HR) dst = gbd;
        else dst = gbc + (e - H - 3 * HR - 1);
        *dst = accumulate ? *dst + acc : acc;
    }
}

// ---------------------------------------------------------------------------
// Compositing: one wavefront per ray, lane l owns samples [l*J, l*J + J).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float density_act(float raw, int flags) {
    return (flags & F_RELU) ? fmaxf(raw, 0.f) : softplus_f(raw);
}

// inclusive multiplicative scan across the wave
__device__ __forceinline__ float wave_scan_mul(float v) {
    const int lane = lane_id();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const float o = __shfl_up(v, off, 64);
        if (lane >= off) v *= o;
    }
    return v;
}
// inclusive additive scan from the top lane down (suffix sums)
__device__ __forceinline__ float wave_suffix_add(float v) {
    const int lane = lane_id();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const float o = __shfl_down(v, off, 64);
        if (lane + off < 64) v += o;
    }
    return v;
}

template <int J>
struct RaySamples {
    float alpha[J], f[J], T[J], w[J], c[J][3], z[J];
    bool valid[J];
};

// alpha_i (rendering.py:113-122 / official_nerf.py:77-83), colour sigmoid, transmittance
template <int J>
__device__ __forceinline__ void load_ray(const float* __restrict__ raw4, const float* __restrict__ zv,
                                         int ray, int S, int flags, RaySamples<J>& rs) {
    const int lane = lane_id();
    const size_t base = (size_t)ray * S;
    float pl = 1.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int i = lane * J + j;
        rs.valid[j] = i < S;
        float a = 0.f, zz = 0.f;
        float c0 = 0.f, c1 = 0.f, c2 = 0.f;
        if (rs.valid[j]) {
            const float4 r = *reinterpret_cast<const float4*>(raw4 + 4 * (base + i));
            zz = zv[base + i];
            const float sig = density_act(r.x, flags);
            if (flags & F_DIST_ALPHA) {
                if (i == S - 1) {
                    a = 1.f;  // rendering.py:121 (delta_last = 1e10 then alpha forced to 1)
                } else {
                    const float delta = zv[base + i + 1] - zz;
                    a = 1.f - expf(-1.0f * sig * delta);
                }
            } else {
                a = 1.f - expf(-1.0f * sig);
            }
            c0 = sigmoid_f(r.y); c1 = sigmoid_f(r.z); c2 = sigmoid_f(r.w);
        }
        rs.alpha[j] = a;
        rs.z[j] = zz;
        rs.c[j][0] = c0; rs.c[j][1] = c1; rs.c[j][2] = c2;
        const float f = rs.valid[j] ? (1.f - a + kEps) : 1.f;
        rs.f[j] = f;
        rs.T[j] = pl;  // exclusive within the lane
        pl *= f;
    }
    // exclusive prefix of the lane products
    const float incl = wave_scan_mul(pl);
    float excl = __shfl_up(incl, 1, 64);
    if (lane == 0) excl = 1.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        rs.T[j] *= excl;
        rs.w[j] = rs.alpha[j] * rs.T[j];
    }
}

template <int J>
__global__ __launch_bounds__(256) void k_composite_fwd(const float* __restrict__ raw4,
                                                       const float* __restrict__ zv, int R, int S,
                                                       int flags, float* __restrict__ rgb,
                                                       float* __restrict__ dist,
                                                       float* __restrict__ alpha_out) {
    const int ray = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (ray >= R) return;
    const int lane = lane_id();
    RaySamples<J> rs;
    load_ray<J>(raw4, zv, ray, S, flags, rs);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, sd = 0.f, sw = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        if (!rs.valid[j]) continue;
        s0 += rs.w[j] * rs.c[j][0];
        s1 += rs.w[j] * rs.c[j][1];
        s2 += rs.w[j] * rs.c[j][2];
        sd += rs.w[j] * rs.z[j];
        sw += rs.w[j];
        alpha_out[(size_t)ray * S + lane * J + j] = rs.alpha[j];
    }
    s0 = wave_sum(s0); s1 = wave_sum(s1); s2 = wave_sum(s2); sd = wave_sum(sd);
    if (flags & F_WHITE_BKGD) sw = wave_sum(sw);
    if (lane == 0) {
        if (flags & F_WHITE_BKGD) {  // rendering.py:139-141
            const float bg = 1.f - sw;
            s0 += bg; s1 += bg; s2 += bg;
        }
        rgb[3 * ray + 0] = s0;
        rgb[3 * ray + 1] = s1;
        rgb[3 * ray + 2] = s2;
        dist[ray] = sd;
    }
}

template <int J>
__global__ __launch_bounds__(256) void k_composite_bwd(const float* __restrict__ raw4,
                                                       const float* __restrict__ zv, int R, int S,
                                                       int flags, const float* __restrict__ g_rgb,
                                                       const float* __restrict__ g_dist,
                                                       float* __restrict__ graw4, int n_pad) {
    const int gtid = blockIdx.x * blockDim.x + threadIdx.x;
    const int ray = gtid >> 6;
    // zero the padded sample rows (grid-stride over the tail)
    for (size_t s = (size_t)R * S + gtid; s < (size_t)n_pad; s += (size_t)gridDim.x * blockDim.x)
        *reinterpret_cast<float4*>(graw4 + 4 * s) = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ray >= R) return;
    const int lane = lane_id();
    RaySamples<J> rs;
    load_ray<J>(raw4, zv, ray, S, flags, rs);
    const float gc0 = g_rgb[3 * ray], gc1 = g_rgb[3 * ray + 1], gc2 = g_rgb[3 * ray + 2];
    const float gd = g_dist[ray];
    const float gbg = (flags & F_WHITE_BKGD) ? -(gc0 + gc1 + gc2) : 0.f;
    // g_w_i and the suffix sums S_i = sum_{k>i} g_w_k w_k
    float gw[J], lsum = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        gw[j] = rs.valid[j] ? (gc0 * rs.c[j][0] + gc1 * rs.c[j][1] + gc2 * rs.c[j][2] + gd * rs.z[j] + gbg) : 0.f;
        lsum += gw[j] * rs.w[j];
    }
    const float incl = wave_suffix_add(lsum);
    float after = __shfl_down(incl, 1, 64);  // sum over lanes > this one
    if (lane == 63) after = 0.f;
    float suffix = after;
#pragma unroll
    for (int j = J - 1; j >= 0; --j) {
        if (!rs.valid[j]) continue;
        const int i = lane * J + j;
        const size_t s = (size_t)ray * S + i;
        // d alpha_i = T_i g_w_i - S_i / (1 - alpha_i + eps)
        const float ga = rs.T[j] * gw[j] - suffix / rs.f[j];
        suffix += gw[j] * rs.w[j];
        const float4 r = *reinterpret_cast<const float4*>(raw4 + 4 * s);
        float graw;
        const float sig = density_act(r.x, flags);
        const float dact = (flags & F_RELU) ? (sig > 0.f ? 1.f : 0.f) : softplus_grad_f(r.x);
        if (flags & F_DIST_ALPHA) {
            if (i == S - 1) {
                graw = 0.f;
            } else {
                const float delta = zv[s + 1] - rs.z[j];
                graw = ga * expf(-1.0f * sig * delta) * delta * dact;
            }
        } else {
            graw = ga * expf(-1.0f * sig) * dact;
        }
        const float gcw = rs.w[j];
        float4 o;
        o.x = graw;
        o.y = gcw * gc0 * (1.f - rs.c[j][0]) * rs.c[j][0];
        o.z = gcw * gc1 * (1.f - rs.c[j][1]) * rs.c[j][1];
        o.w = gcw * gc2 * (1.f - rs.c[j][2]) * rs.c[j][2];
        *reinterpret_cast<float4*>(graw4 + 4 * s) = o;
    }
}

// ---------------------------------------------------------------------------
// Compositing, 16 lanes per ray (4 rays per wave), lane l owns samples [l*J, l*J + J)
// (S <= 256).  Scans and sums over a ray are 4-step DPP row operations (a DPP row is
// exactly one ray), amortised over J samples per lane, and the activations use the
// hardware transcendentals (v_exp_f32 / v_log_f32 / v_rcp_f32, a few ulp): with the
// wave-per-ray kernels above the kernel was VALU-bound (~40 % of the HBM roofline at
// 2^20 rays); these keep it on HBM.
// ---------------------------------------------------------------------------
// (dpp_f, row_scan_mul, row_suffix_add, row_sum: samples.hpp)

template <int J>
struct Ray16 {
    float alpha[J], f[J], T[J], w[J], c[J][3], z[J], sig[J], raw[J];
    bool valid[J];
};

// alpha, colour sigmoid, exclusive transmittance of this lane's J samples
// The block's raw4 rows (16 rays) staged in LDS with one 16-byte pad after every lane's
// J samples: global loads stay fully coalesced and a lane's J consecutive samples sit at
// a 16(J+1)-byte lane stride, conflict-free for ds_read_b128.
template <int J>
__device__ __forceinline__ int stage_slot(int r_local, int i) { return (r_local * 16 + i / J) * (J + 1) + i % J; }

// ray-local (row, sample) of the c-th staged element; shifts when S is a power of two
__device__ __forceinline__ void split_rs(int c, int S, int lgS, int& r, int& i) {
    if (lgS >= 0) { r = c >> lgS; i = c & (S - 1); }
    else { r = c / S; i = c - r * S; }
}

template <int J>
__device__ __forceinline__ void stage_raw(const float* __restrict__ raw4, float4* lds, int ray0, int R, int S,
                                          int lgS) {
    const int nr = min(16, R - ray0);
    if (nr <= 0) return;
    const float4* src = reinterpret_cast<const float4*>(raw4) + (size_t)ray0 * S;
    if (nr == 16 && S == 16 * J) {
        // whole block, S = 16 J: each thread's J loads are issued back to back (J 16-byte
        // loads in flight per lane instead of one)
        float4 v[J];
#pragma unroll
        for (int q = 0; q < J; ++q) v[q] = src[threadIdx.x + q * 256];
#pragma unroll
        for (int q = 0; q < J; ++q) {
            const int c = threadIdx.x + q * 256;
            lds[stage_slot<J>(c / S, c % S)] = v[q];
        }
        return;
    }
    for (int c = threadIdx.x; c < nr * S; c += blockDim.x) {
        int r, i;
        split_rs(c, S, lgS, r, i);
        lds[stage_slot<J>(r, i)] = src[c];
    }
}

template <int J>
__device__ __forceinline__ void load_ray16(const float4* __restrict__ lraw, const float* __restrict__ zv, int ray,
                                           bool active, int S, int flags, Ray16<J>& rs) {
    const int l16 = threadIdx.x & 15;
    const size_t base = (size_t)ray * S;
    const int i0 = l16 * J;
    // z of this lane's samples (float4 when aligned), and of the next lane's first sample
    if (J % 4 == 0 && (S & 3) == 0 && active && i0 + J <= S) {
#pragma unroll
        for (int q = 0; q < J / 4; ++q) {
            const float4 v = *reinterpret_cast<const float4*>(zv + base + i0 + 4 * q);
            rs.z[4 * q] = v.x; rs.z[4 * q + 1] = v.y; rs.z[4 * q + 2] = v.z; rs.z[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < J; ++j) rs.z[j] = (active && i0 + j < S) ? zv[base + i0 + j] : 0.f;
    }
    const float z_next = dpp_f<0x101>(0.f, rs.z[0]);   // lane l+1's first sample (row_shl 1)
    float pl = 1.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int i = i0 + j;
        rs.valid[j] = active && i < S;
        float a = 0.f, c0 = 0.f, c1 = 0.f, c2 = 0.f, sg = 0.f, r0 = 0.f;
        if (rs.valid[j]) {
            const float4 r = lraw[((threadIdx.x >> 4) * 16 + l16) * (J + 1) + j];
            r0 = r.x;
            sg = f_density(r.x, flags);
            if (flags & F_DIST_ALPHA) {
                if (i == S - 1) {
                    a = 1.f;   // rendering.py:121
                } else {
                    const float zn = (j + 1 < J) ? rs.z[j + 1 < J ? j + 1 : 0] : z_next;
                    a = 1.f - __expf(-1.0f * sg * (zn - rs.z[j]));
                }
            } else {
                a = 1.f - __expf(-1.0f * sg);
            }
            c0 = f_sigmoid(r.y); c1 = f_sigmoid(r.z); c2 = f_sigmoid(r.w);
        }
        rs.sig[j] = sg;
        rs.raw[j] = r0;
        rs.alpha[j] = a;
        rs.c[j][0] = c0; rs.c[j][1] = c1; rs.c[j][2] = c2;
        const float f = rs.valid[j] ? (1.f - a + kEps) : 1.f;
        rs.f[j] = f;
        rs.T[j] = pl;
        pl *= f;
    }
    const float excl = dpp_f<0x111>(1.f, row_scan_mul(pl));   // product over the lanes before this one
#pragma unroll
    for (int j = 0; j < J; ++j) {
        rs.T[j] *= excl;
        rs.w[j] = rs.alpha[j] * rs.T[j];
    }
}

template <int J>
__global__ __launch_bounds__(256) void k_composite16_fwd(const float* __restrict__ raw4, const float* __restrict__ zv,
                                                         int R, int S, int flags, float* __restrict__ rgb,
                                                         float* __restrict__ dist, float* __restrict__ alpha_out) {
    __shared__ float4 lraw[256 * (J + 1)];
    const int ray = (blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const bool active = ray < R;       // a 16-lane DPP row is one ray: whole rows are (in)active
    const int l16 = threadIdx.x & 15;
    const int lgS = (S & (S - 1)) == 0 ? __builtin_ctz(S) : -1;
    stage_raw<J>(raw4, lraw, blockIdx.x * 16, R, S, lgS);
    __syncthreads();
    Ray16<J> rs;
    load_ray16<J>(lraw, zv, ray, active, S, flags, rs);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, sd = 0.f, sw = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        s0 += rs.w[j] * rs.c[j][0];
        s1 += rs.w[j] * rs.c[j][1];
        s2 += rs.w[j] * rs.c[j][2];
        sd += rs.w[j] * rs.z[j];
        sw += rs.w[j];
    }
    const size_t a0 = (size_t)ray * S + l16 * J;
    if (J % 4 == 0 && (S & 3) == 0 && active && l16 * J + J <= S) {
#pragma unroll
        for (int q = 0; q < J / 4; ++q)
            *reinterpret_cast<float4*>(alpha_out + a0 + 4 * q) =
                make_float4(rs.alpha[4 * q], rs.alpha[4 * q + 1], rs.alpha[4 * q + 2], rs.alpha[4 * q + 3]);
    } else {
#pragma unroll
        for (int j = 0; j < J; ++j)
            if (rs.valid[j]) alpha_out[a0 + j] = rs.alpha[j];
    }
    s0 = row_sum(s0); s1 = row_sum(s1); s2 = row_sum(s2); sd = row_sum(sd);
    if (flags & F_WHITE_BKGD) sw = row_sum(sw);
    if (active && l16 == 0) {
        if (flags & F_WHITE_BKGD) {   // rendering.py:139-141
            const float bg = 1.f - sw;
            s0 += bg; s1 += bg; s2 += bg;
        }
        rgb[3 * ray + 0] = s0;
        rgb[3 * ray + 1] = s1;
        rgb[3 * ray + 2] = s2;
        dist[ray] = sd;
    }
}

template <int J>
__global__ __launch_bounds__(256) void k_composite16_bwd(const float* __restrict__ raw4, const float* __restrict__ zv,
                                                         int R, int S, int flags, const float* __restrict__ g_rgb,
                                                         const float* __restrict__ g_dist,
                                                         float* __restrict__ graw4, int n_pad) {
    const int gtid = blockIdx.x * blockDim.x + threadIdx.x;
    for (size_t s = (size_t)R * S + gtid; s < (size_t)n_pad; s += (size_t)gridDim.x * blockDim.x)
        *reinterpret_cast<float4*>(graw4 + 4 * s) = make_float4(0.f, 0.f, 0.f, 0.f);
    __shared__ float4 lraw[256 * (J + 1)];
    const int ray = gtid >> 4;
    const bool active = ray < R;
    const int l16 = threadIdx.x & 15;
    const int lgS = (S & (S - 1)) == 0 ? __builtin_ctz(S) : -1;
    stage_raw<J>(raw4, lraw, blockIdx.x * 16, R, S, lgS);
    __syncthreads();
    Ray16<J> rs;
    load_ray16<J>(lraw, zv, ray, active, S, flags, rs);
    __syncthreads();   // lraw is reused for the gradient rows below
    const float gc0 = active ? g_rgb[3 * ray] : 0.f, gc1 = active ? g_rgb[3 * ray + 1] : 0.f;
    const float gc2 = active ? g_rgb[3 * ray + 2] : 0.f, gd = active ? g_dist[ray] : 0.f;
    const float gbg = (flags & F_WHITE_BKGD) ? -(gc0 + gc1 + gc2) : 0.f;
    float gw[J], lsum = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        gw[j] = rs.valid[j] ? (gc0 * rs.c[j][0] + gc1 * rs.c[j][1] + gc2 * rs.c[j][2] + gd * rs.z[j] + gbg) : 0.f;
        lsum += gw[j] * rs.w[j];
    }
    // suffix sums S_i = sum_{k>i} g_w_k w_k: lanes after this one, then this lane's samples
    float suffix = dpp_f<0x101>(0.f, row_suffix_add(lsum));
    const float z_next = dpp_f<0x101>(0.f, rs.z[0]);
#pragma unroll
    for (int j = J - 1; j >= 0; --j) {
        if (!rs.valid[j]) continue;
        const int i = l16 * J + j;
        const size_t s = (size_t)ray * S + i;
        const float ga = rs.T[j] * gw[j] - suffix * f_rcp(rs.f[j]);   // d alpha_i
        suffix += gw[j] * rs.w[j];
        const float sig = rs.sig[j];
        const float dact = (flags & F_RELU) ? (sig > 0.f ? 1.f : 0.f) : f_softplus_grad(rs.raw[j]);
        float graw;
        if (flags & F_DIST_ALPHA) {
            if (i == S - 1) {
                graw = 0.f;
            } else {
                const float delta = ((j + 1 < J) ? rs.z[j + 1 < J ? j + 1 : 0] : z_next) - rs.z[j];
                graw = ga * __expf(-1.0f * sig * delta) * delta * dact;
            }
        } else {
            graw = ga * __expf(-1.0f * sig) * dact;
        }
        const float gcw = rs.w[j];
        float4 o;
        o.x = graw;
        o.y = gcw * gc0 * (1.f - rs.c[j][0]) * rs.c[j][0];
        o.z = gcw * gc1 * (1.f - rs.c[j][1]) * rs.c[j][1];
        o.w = gcw * gc2 * (1.f - rs.c[j][2]) * rs.c[j][2];
        (void)s;
        lraw[((threadIdx.x >> 4) * 16 + l16) * (J + 1) + j] = o;
    }
    __syncthreads();
    const int ray0 = blockIdx.x * 16, nr = min(16, R - ray0);
    float4* dst = reinterpret_cast<float4*>(graw4) + (size_t)ray0 * S;
    if (nr == 16 && S == 16 * J) {
#pragma unroll
        for (int q = 0; q < J; ++q) {
            const int c = threadIdx.x + q * 256;
            dst[c] = lraw[stage_slot<J>(c / S, c % S)];
        }
        return;
    }
    for (int c = threadIdx.x; c < nr * S; c += blockDim.x) {
        int r, i;
        split_rs(c, S, lgS, r, i);
        dst[c] = lraw[stage_slot<J>(r, i)];
    }
}

// ---------------------------------------------------------------------------
// gradient back to the ray inputs (pose / ray learning)
// ---------------------------------------------------------------------------
// One workgroup per ray, EB_WAVES waves over its samples, lane = encoding column: every load of
// a gradient row is one coalesced 256-byte wave access (a lane-per-sample layout reads 64
// lines per instruction).  Column k of encode_position (official_nerf.py:99-119) is x_c
// (k < 3) or sin / cos(2^i x_c) (k = 3 + 6 i + c, + 3 for cos); its derivative w.r.t. x_c
// is 1, 2^i cos, -2^i sin.  A lane accumulates G[s][k] d_k(x(s)) over its samples (and the
// same times z_s for the direction gradient, x = o + d z); the view encoding is constant per
// ray, so its columns are summed first and scaled once.  The per-component sums meet in LDS.
constexpr int EB_WAVES = 16;   // waves per ray (8 samples each at S = 128: 4 waves of 32 ran ~31 us per cfg3 step)
struct EncCol {
    int c;        // input component, -1 for a padding column
    float f;      // 2^i (1 for the identity columns)
    int kind;     // 0 identity, 1 sin column, 2 cos column
};
__device__ __forceinline__ EncCol enc_col(int k, int L) {
    EncCol e{-1, 0.f, 0};
    if (k < 3) { e.c = k; e.f = 1.f; e.kind = 0; return e; }
    const int q = k - 3;
    if (q >= 6 * L) return e;
    const int i = q / 6, r = q - 6 * i;
    e.c = r % 3; e.f = (float)(1 << i); e.kind = r < 3 ? 1 : 2;
    return e;
}
__device__ __forceinline__ float enc_dfac(const EncCol& e, float x) {
    if (e.c < 0) return 0.f;
    if (e.kind == 0) return 1.f;
    float sn, cs;
    sincosf(e.f * x, &sn, &cs);
    return e.kind == 1 ? e.f * cs : -e.f * sn;
}

__global__ __launch_bounds__(64 * EB_WAVES) void k_encode_bwd(const float* __restrict__ po, const float* __restrict__ pd,
                                                    const float* __restrict__ view, const float* __restrict__ zv,
                                                    const float* __restrict__ gp, const float* __restrict__ gp2,
                                                    const float* __restrict__ gd,
                                                    int R, int S, float* __restrict__ g_po,
                                                    float* __restrict__ g_pd, float* __restrict__ g_view) {
    __shared__ float red[EB_WAVES][3][3];   // [wave][o / d / view][component]
    const int ray = blockIdx.x;
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const EncCol ep = enc_col(lane, 10), ed = enc_col(lane, 4);
    const float o = ep.c >= 0 ? po[3 * ray + ep.c] : 0.f;
    const float d = ep.c >= 0 ? pd[3 * ray + ep.c] : 0.f;
    float ao = 0.f, ad = 0.f, sv = 0.f;
    const size_t base = (size_t)ray * S;
#pragma unroll 4
    for (int i = w; i < S; i += EB_WAVES) {
        const size_t s = base + i;
        const float z = zv[s];
        float g = gp[s * ENC_P + lane];
        if (gp2) g += gp2[s * ENC_P + lane];
        sv += gd[s * ENC_D + lane];
        const float t = g * enc_dfac(ep, ray_point(o, d, z));
        ao += t;
        ad += t * z;
    }
    const float av = ed.c >= 0 ? sv * enc_dfac(ed, view[3 * ray + ed.c]) : 0.f;
    // per-component sums over the wave's lanes
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float so = wave_sum(ep.c == c ? ao : 0.f);
        const float sd = wave_sum(ep.c == c ? ad : 0.f);
        const float s2 = wave_sum(ed.c == c ? av : 0.f);
        if (lane == 0) { red[w][0][c] = so; red[w][1][c] = sd; red[w][2][c] = s2; }
    }
    __syncthreads();
    if (threadIdx.x < 9) {
        const int k = threadIdx.x / 3, c = threadIdx.x % 3;
        float v = red[0][k][c];
#pragma unroll
        for (int q = 1; q < EB_WAVES; ++q) v += red[q][k][c];   // waves in order
        (k == 0 ? g_po : k == 1 ? g_pd : g_view)[3 * ray + c] = v;
    }
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_encode_samples(const float* pts_o, const float* pts_d, const float* view,
                                   const float* noise, int n_rays, int n_samples, int n_pad,
                                   float near_z, float far_z, float* z, float* enc_p, float* enc_d,
                                   float* enc_p_rmax, float* enc_d_rmax, float* enc_p_cmax, float* enc_d_cmax,
                                   void* stream) {
    NERF_CHECK_PTR(pts_o); NERF_CHECK_PTR(pts_d); NERF_CHECK_PTR(view);
    NERF_CHECK_PTR(z); NERF_CHECK_PTR(enc_p); NERF_CHECK_PTR(enc_d);
    NERF_CHECK((enc_p_cmax == nullptr) == (enc_d_cmax == nullptr) && (enc_p_cmax == nullptr || n_pad % 128 == 0),
               "%s: enc_p_cmax / enc_d_cmax go together and need n_pad %% 128 == 0", __func__);
    NERF_CHECK_ALIGN16(enc_p); NERF_CHECK_ALIGN16(enc_d);
    NERF_CHECK(n_rays > 0 && n_samples > 0 && (int64_t)n_rays * n_samples <= n_pad,
               "%s: n_pad=%d < R*S=%lld", __func__, n_pad, (long long)n_rays * n_samples);
    NERF_CHECK(n_pad % ENC_ROWS == 0, "%s: n_pad=%d must be a multiple of %d", __func__, n_pad, ENC_ROWS);
    hipLaunchKernelGGL(k_encode_samples, dim3(n_pad / ENC_ROWS), dim3(ENC_THREADS), 0, as_stream(stream), pts_o, pts_d,
                       view, noise, n_rays, n_samples, n_pad, near_z, far_z, z, enc_p, enc_d, enc_p_rmax,
                       enc_d_rmax, enc_p_cmax, enc_d_cmax);
    return check_launch(__func__);
}

static int heads_blocks(int n_pad) {
    const int groups = n_pad / 16;
    int b = (groups + 3) / 4;
    return b > 256 ? 256 : (b < 1 ? 1 : b);
}

extern "C" int nerf_heads_fwd(const float* h8, int ld8, const float* hr, int ldr, int hidden,
                              const float* wd, const float* bd, const float* wc, const float* bc,
                              float* raw4, int n_pad, void* stream) {
    NERF_CHECK_PTR(h8); NERF_CHECK_PTR(hr); NERF_CHECK_PTR(wd); NERF_CHECK_PTR(bd);
    NERF_CHECK_PTR(wc); NERF_CHECK_PTR(bc); NERF_CHECK_PTR(raw4);
    NERF_CHECK_ALIGN16(raw4);
    NERF_CHECK(n_pad % 16 == 0, "%s: n_pad %% 16 != 0", __func__);
    const int hrw = hidden / 2 < 64 ? 64 : hidden / 2;  // colour hidden is padded to >= 64
    hipStream_t s = as_stream(stream);
    dim3 g(heads_blocks(n_pad)), b(256);
    if (hidden == 256 && hrw == 128)
        hipLaunchKernelGGL((k_heads_fwd<4, 2>), g, b, 0, s, h8, ld8, hr, ldr, wd, bd, wc, bc, raw4, n_pad);
    else if (hidden == 128 && hrw == 64)
        hipLaunchKernelGGL((k_heads_fwd<2, 1>), g, b, 0, s, h8, ld8, hr, ldr, wd, bd, wc, bc, raw4, n_pad);
    else if (hidden == 64 && hrw == 64)
        hipLaunchKernelGGL((k_heads_fwd<1, 1>), g, b, 0, s, h8, ld8, hr, ldr, wd, bd, wc, bc, raw4, n_pad);
    else if (hidden == 512 && hrw == 256)
        hipLaunchKernelGGL((k_heads_fwd<8, 4>), g, b, 0, s, h8, ld8, hr, ldr, wd, bd, wc, bc, raw4, n_pad);
    else
        NERF_CHECK(false, "%s: unsupported hidden width %d (64/128/256/512)", __func__, hidden);
    return check_launch(__func__);
}

extern "C" int nerf_heads_part_size(int hidden, int n_pad) {
    const int hrw = hidden / 2 < 64 ? 64 : hidden / 2;
    return heads_blocks(n_pad) * (hidden + 3 * hrw + 4);
}

template <int MODE, bool MB = false>
static int heads_bwd(const float* graw4, const float* h8, int ld8, const float* hr, int ldr, const uint32_t* hmask,
                     int ldm, int hidden, const float* wc, float* dyr, int lddyr, float* part, int n_pad,
                     float* dyr_rmax, float* dyr_cmax, hipStream_t s) {
    const int hrw = hidden / 2 < 64 ? 64 : hidden / 2;
    if (MODE == 1 && n_pad % 128 == 0) {   // dyr only: a block per 128-row chunk
#define NERF_HEADS_DYR(NR) \
        hipLaunchKernelGGL((k_heads_dyr<NR, MB>), dim3(n_pad / 128), dim3(256), 0, s, graw4, hr, ldr, hmask, ldm, wc, \
                           dyr, lddyr, dyr_rmax, dyr_cmax)
        if (hrw == 128) NERF_HEADS_DYR(2);
        else if (hrw == 64) NERF_HEADS_DYR(1);
        else if (hrw == 256) NERF_HEADS_DYR(4);
        else NERF_CHECK(false, "heads_bwd: unsupported hidden width %d (64/128/256/512)", hidden);
#undef NERF_HEADS_DYR
        return check_launch("nerf_heads_bwd (dyr)");
    }
    dim3 g(heads_blocks(n_pad)), b(256);
#define NERF_HEADS_BWD(NH, NR) \
    hipLaunchKernelGGL((k_heads_bwd<NH, NR, MODE, MB>), g, b, 0, s, graw4, h8, ld8, hr, ldr, hmask, ldm, wc, dyr, \
                       lddyr, part, n_pad, dyr_rmax, dyr_cmax)
    if (hidden == 256 && hrw == 128) NERF_HEADS_BWD(4, 2);
    else if (hidden == 128 && hrw == 64) NERF_HEADS_BWD(2, 1);
    else if (hidden == 64 && hrw == 64) NERF_HEADS_BWD(1, 1);
    else if (hidden == 512 && hrw == 256) NERF_HEADS_BWD(8, 4);
    else NERF_CHECK(false, "heads_bwd: unsupported hidden width %d (64/128/256/512)", hidden);
#undef NERF_HEADS_BWD
    return check_launch("nerf_heads_bwd");
}

extern "C" int nerf_heads_bwd_mode(int mode, const float* graw4, const float* h8, int ld8, const float* hr, int ldr,
                                   const uint32_t* hr_mask, int ldm, int hidden, const float* wc, float* dyr,
                                   int lddyr, float* part, int n_pad, float* dyr_rmax, float* dyr_cmax,
                                   void* stream) {
    NERF_CHECK(mode >= 1 && mode <= 3, "%s: mode %d (1: dyr, 2: head-weight partials, 3: both)", __func__, mode);
    NERF_CHECK(hr_mask == nullptr || mode == 1, "%s: the mask-bit gate (hr_mask) is for mode 1", __func__);
    NERF_CHECK(hr_mask == nullptr || ldm * 32 >= (hidden / 2 < 64 ? 64 : hidden / 2), "%s: ldm %d too small",
               __func__, ldm);
    NERF_CHECK_PTR(graw4); NERF_CHECK_PTR(wc);
    if (hr_mask == nullptr) NERF_CHECK_PTR(hr);
    if (mode & 1) NERF_CHECK_PTR(dyr);
    if (mode & 2) { NERF_CHECK_PTR(h8); NERF_CHECK_PTR(part); }
    NERF_CHECK_ALIGN16(graw4);
    NERF_CHECK(n_pad % 16 == 0, "%s: n_pad %% 16 != 0", __func__);
    NERF_CHECK(dyr_cmax == nullptr || n_pad % 128 == 0, "%s: dyr_cmax needs n_pad %% 128 == 0", __func__);
    hipStream_t s = as_stream(stream);
    if (mode == 1 && hr_mask)
        return heads_bwd<1, true>(graw4, h8, ld8, hr, ldr, hr_mask, ldm, hidden, wc, dyr, lddyr, part, n_pad, dyr_rmax,
                                  dyr_cmax, s);
    if (mode == 1)
        return heads_bwd<1>(graw4, h8, ld8, hr, ldr, nullptr, 0, hidden, wc, dyr, lddyr, part, n_pad, dyr_rmax,
                            dyr_cmax, s);
    if (mode == 2)
        return heads_bwd<2>(graw4, h8, ld8, hr, ldr, nullptr, 0, hidden, wc, dyr, lddyr, part, n_pad, dyr_rmax,
                            dyr_cmax, s);
    return heads_bwd<3>(graw4, h8, ld8, hr, ldr, nullptr, 0, hidden, wc, dyr, lddyr, part, n_pad, dyr_rmax, dyr_cmax,
                        s);
}

extern "C" int nerf_heads_bwd(const float* graw4, const float* h8, int ld8, const float* hr, int ldr,
                              int hidden, const float* wc, float* dyr, int lddyr, float* part,
                              int n_pad, float* dyr_rmax, float* dyr_cmax, void* stream) {
    return nerf_heads_bwd_mode(3, graw4, h8, ld8, hr, ldr, nullptr, 0, hidden, wc, dyr, lddyr, part, n_pad, dyr_rmax,
                               dyr_cmax, stream);
}

// The head-weight partials of the chain backward (hidden 256, colour width 128): per 128-row
// block, the density head's sum_s graw4[s].x h8[s][:] (256), the colour head's sum_s graw4[s].c
// hr[s][:] (3 x 128) and the bias sums sum_s graw4[s] (4) -- k_heads_bwd mode 2's sums in another
// order, laid out as slabs for nerf::slab_reduce_jobs (the reduce then rides in the weight
// gradients' batch).  Each wave walks 32 rows with 16-byte loads: an h8 row per wave instruction
// (lane: columns 4 lane .. + 3), two hr rows per instruction (half-wave h: the rows of parity h);
// 1024 blocks x 4 waves at cfg2 (the mode-2 kernel's 1024 waves of 4-byte loads ran at ~2.8 TB/s
// in-step).  Sums in a fixed order: the gradients are the same bits on every run.
constexpr int HP_RPW = 32;                    // rows per wave
constexpr int HP_ROWS = 4 * HP_RPW;           // rows per block
__global__ __launch_bounds__(256, 4) void k_heads_part(const float* __restrict__ graw4, const float* __restrict__ h8,
                                                    int ld8, const float* __restrict__ hr, int ldr, int n,
                                                    float* __restrict__ wdp, float* __restrict__ wcp,
                                                    float* __restrict__ bdp, float* __restrict__ bcp) {
    __shared__ float4 red[4][4][64];   // [wave][wd, wc r, wc g, wc b][lane]
    __shared__ float4 rb[4];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int half = lane >> 5, l32 = lane & 31;
    const int r0 = blockIdx.x * HP_ROWS + wave * HP_RPW;
    float4 awd = make_float4(0.f, 0.f, 0.f, 0.f), ac[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) ac[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    auto fma4 = [](float g, const float4& v, float4& a) {
        a.x = fmaf(g, v.x, a.x); a.y = fmaf(g, v.y, a.y); a.z = fmaf(g, v.z, a.z); a.w = fmaf(g, v.w, a.w);
    };
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    // the wave's rows as buffer resources: row offsets in SGPRs, the lane's column (and for hr
    // its row parity) in one VGPR each -- few address registers, so every load of a batch can be
    // in flight at once
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc((void*)(h8 + (size_t)r0 * ld8), (short)0,
                                                                        HP_RPW * ld8 * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)(hr + (size_t)r0 * ldr), (short)0,
                                                                        HP_RPW * ldr * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)(graw4 + 4 * (size_t)r0), (short)0,
                                                                        HP_RPW * 16, 0x00020000);
    const int vh = 16 * lane, vr = half * ldr * 4 + 16 * l32, vg = half * 16;
    auto ld4 = [](const __amdgpu_buffer_rsrc_t& r, int v, int so) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        const u4 t = __builtin_amdgcn_raw_buffer_load_b128(r, v, so, 0);
        return make_float4(__uint_as_float(t.x), __uint_as_float(t.y), __uint_as_float(t.z), __uint_as_float(t.w));
    };
#pragma unroll 1
    for (int t = 0; t < HP_RPW; t += 8) {
        float4 hv[8], rv[4], gc[4];
        float gh[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            hv[u] = ld4(rh, vh, (t + u) * ld8 * 4);
            gh[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rg, 0, (t + u) * 16, 0));
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            rv[u] = ld4(rr, vr, (t + 2 * u) * ldr * 4);
            gc[u] = ld4(rg, vg, (t + 2 * u) * 16);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) fma4(gh[u], hv[u], awd);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            fma4(gc[u].y, rv[u], ac[0]);
            fma4(gc[u].z, rv[u], ac[1]);
            fma4(gc[u].w, rv[u], ac[2]);
        }
    }
    // the colour sums of the two row parities (lanes l32 and l32 + 32), then the bias sums (lane
    // l: row r0 + l of the wave's 32; a butterfly in a fixed order)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        ac[c].x += __shfl_xor(ac[c].x, 32, 64); ac[c].y += __shfl_xor(ac[c].y, 32, 64);
        ac[c].z += __shfl_xor(ac[c].z, 32, 64); ac[c].w += __shfl_xor(ac[c].w, 32, 64);
    }
    float4 b = lane < HP_RPW ? *reinterpret_cast<const float4*>(graw4 + 4 * (size_t)(r0 + lane)) : z4;
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) {
        b.x += __shfl_xor(b.x, o, 64); b.y += __shfl_xor(b.y, o, 64);
        b.z += __shfl_xor(b.z, o, 64); b.w += __shfl_xor(b.w, o, 64);
    }
    red[wave][0][lane] = awd;
    red[wave][1][lane] = ac[0];
    red[wave][2][lane] = ac[1];
    red[wave][3][lane] = ac[2];
    if (lane == 0) rb[wave] = b;
    __syncthreads();
    const int k = threadIdx.x >> 6, e = lane;   // thread: section k (wd, r, g, b), lane e
    float4 v = red[0][k][e];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
        const float4 q = red[w][k][e];
        v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
    }
    const size_t blk = blockIdx.x;
    if (k == 0) *reinterpret_cast<float4*>(wdp + blk * 256 + 4 * e) = v;
    else if (e < 32) *reinterpret_cast<float4*>(wcp + blk * 384 + (k - 1) * 128 + 4 * e) = v;
    if (threadIdx.x == 0) {
        float4 q = rb[0];
#pragma unroll
        for (int w = 1; w < 4; ++w) { q.x += rb[w].x; q.y += rb[w].y; q.z += rb[w].z; q.w += rb[w].w; }
        bdp[blk] = q.x;
        bcp[blk * 3 + 0] = q.y; bcp[blk * 3 + 1] = q.z; bcp[blk * 3 + 2] = q.w;
    }
}

namespace nerf {
int heads_part_blocks(int n) { return (n + HP_ROWS - 1) / HP_ROWS; }   // (the kernel takes n % HP_ROWS == 0)
// the partial slabs of k_heads_part and the two slab-reduce jobs that finish them (gw / gb: the
// density head's [1][256] + [1], the colour head's [3][128] + [3])
int heads_partials(const float* graw4, const float* h8, int ld8, const float* hr, int ldr, int n, float* part,
                   float* gwd, float* gbd, float* gwc, float* gbc, SlabJobDesc (&jobs)[2], hipStream_t s) {
    NERF_CHECK_PTR(graw4); NERF_CHECK_PTR(h8); NERF_CHECK_PTR(hr); NERF_CHECK_PTR(part);
    NERF_CHECK(n > 0 && n % HP_ROWS == 0 && ld8 % 4 == 0 && ldr % 4 == 0 && ld8 >= 256 && ldr >= 128,
               "%s: n %d (a multiple of %d), ld8 %d, ldr %d", __func__, n, HP_ROWS, ld8, ldr);
    NERF_CHECK_ALIGN16(graw4); NERF_CHECK_ALIGN16(h8); NERF_CHECK_ALIGN16(hr); NERF_CHECK_ALIGN16(part);
    const int nb = heads_part_blocks(n);
    float* wdp = part;
    float* wcp = wdp + (size_t)nb * 256;
    float* bdp = wcp + (size_t)nb * 384;
    float* bcp = bdp + nb;
    hipLaunchKernelGGL(k_heads_part, dim3(nb), dim3(256), 0, s, graw4, h8, ld8, hr, ldr, n, wdp, wcp, bdp, bcp);
    jobs[0] = SlabJobDesc{wdp, nb, 1, 256, 1, 256, bdp, gwd, gbd};
    jobs[1] = SlabJobDesc{wcp, nb, 3, 128, 3, 128, bcp, gwc, gbc};
    return check_launch(__func__);
}
}  // namespace nerf

extern "C" int nerf_heads_reduce(const float* part, int hidden, int n_pad, float* gwd, float* gbd,
                                 float* gwc, float* gbc, int accumulate, void* stream) {
    NERF_CHECK_PTR(part); NERF_CHECK_PTR(gwd); NERF_CHECK_PTR(gbd); NERF_CHECK_PTR(gwc); NERF_CHECK_PTR(gbc);
    const int hrw = hidden / 2 < 64 ? 64 : hidden / 2;
    const int PART = hidden + 3 * hrw + 4;
    hipLaunchKernelGGL(k_heads_reduce, dim3((PART + 63) / 64), dim3(256), 0, as_stream(stream), part,
                       heads_blocks(n_pad), hidden, hrw, gwd, gbd, gwc, gbc, accumulate);
    return check_launch(__func__);
}

#define NERF_J_DISPATCH(KERNEL, S, ...)                                            \
    do {                                                                           \
        const int J_ = ((S) + 63) / 64;                                            \
        if (J_ <= 1) hipLaunchKernelGGL((KERNEL<1>), __VA_ARGS__);                 \
        else if (J_ == 2) hipLaunchKernelGGL((KERNEL<2>), __VA_ARGS__);            \
        else if (J_ <= 4) hipLaunchKernelGGL((KERNEL<4>), __VA_ARGS__);            \
        else if (J_ <= 8) hipLaunchKernelGGL((KERNEL<8>), __VA_ARGS__);            \
        else if (J_ <= 16) hipLaunchKernelGGL((KERNEL<16>), __VA_ARGS__);          \
        else NERF_CHECK(false, "%s: n_samples=%d > 1024", __func__, (int)(S));     \
    } while (0)

#define NERF_J16_DISPATCH(KERNEL, S, ...)                                          \
    do {                                                                           \
        const int J_ = ((S) + 15) / 16;                                            \
        if (J_ <= 1) hipLaunchKernelGGL((KERNEL<1>), __VA_ARGS__);                 \
        else if (J_ == 2) hipLaunchKernelGGL((KERNEL<2>), __VA_ARGS__);            \
        else if (J_ <= 4) hipLaunchKernelGGL((KERNEL<4>), __VA_ARGS__);            \
        else if (J_ <= 8) hipLaunchKernelGGL((KERNEL<8>), __VA_ARGS__);            \
        else hipLaunchKernelGGL((KERNEL<16>), __VA_ARGS__);                        \
    } while (0)

extern "C" int nerf_composite_fwd(const float* raw4, const float* z, int n_rays, int n_samples, int flags,
                                  float* rgb, float* dist, float* alpha, void* stream) {
    NERF_CHECK_PTR(raw4); NERF_CHECK_PTR(z); NERF_CHECK_PTR(rgb); NERF_CHECK_PTR(dist); NERF_CHECK_PTR(alpha);
    NERF_CHECK_ALIGN16(raw4);
    NERF_CHECK(n_rays > 0 && n_samples > 0, "%s: empty input", __func__);
    if (n_samples <= 256) {   // 16 lanes per ray
        NERF_J16_DISPATCH(k_composite16_fwd, n_samples, dim3((n_rays + 15) / 16), dim3(256), 0, as_stream(stream), raw4,
                          z, n_rays, n_samples, flags, rgb, dist, alpha);
        return check_launch(__func__);
    }
    const int blocks = (n_rays + 3) / 4;
    NERF_J_DISPATCH(k_composite_fwd, n_samples, dim3(blocks), dim3(256), 0, as_stream(stream), raw4, z,
                    n_rays, n_samples, flags, rgb, dist, alpha);
    return check_launch(__func__);
}

extern "C" int nerf_composite_bwd(const float* raw4, const float* z, int n_rays, int n_samples, int flags,
                                  const float* grad_rgb, const float* grad_dist, float* graw4, int n_pad,
                                  void* stream) {
    NERF_CHECK_PTR(raw4); NERF_CHECK_PTR(z); NERF_CHECK_PTR(grad_rgb); NERF_CHECK_PTR(grad_dist);
    NERF_CHECK_PTR(graw4);
    NERF_CHECK_ALIGN16(raw4); NERF_CHECK_ALIGN16(graw4);
    NERF_CHECK(n_rays > 0 && n_samples > 0 && (int64_t)n_rays * n_samples <= n_pad, "%s: bad sizes", __func__);
    if (n_samples <= 256) {
        NERF_J16_DISPATCH(k_composite16_bwd, n_samples, dim3((n_rays + 15) / 16), dim3(256), 0, as_stream(stream), raw4,
                          z, n_rays, n_samples, flags, grad_rgb, grad_dist, graw4, n_pad);
        return check_launch(__func__);
    }
    const int blocks = (n_rays + 3) / 4;
    NERF_J_DISPATCH(k_composite_bwd, n_samples, dim3(blocks), dim3(256), 0, as_stream(stream), raw4, z,
                    n_rays, n_samples, flags, grad_rgb, grad_dist, graw4, n_pad);
    return check_launch(__func__);
}

extern "C" int nerf_encode_bwd(const float* pts_o, const float* pts_d, const float* view, const float* z,
                               const float* genc_p, const float* genc_p2, const float* genc_d, int n_rays, int n_samples,
                               float* g_pts_o, float* g_pts_d, float* g_view, void* stream) {
    NERF_CHECK_PTR(pts_o); NERF_CHECK_PTR(pts_d); NERF_CHECK_PTR(view); NERF_CHECK_PTR(z);
    NERF_CHECK_PTR(genc_p); NERF_CHECK_PTR(genc_d);
    NERF_CHECK_PTR(g_pts_o); NERF_CHECK_PTR(g_pts_d); NERF_CHECK_PTR(g_view);
    NERF_CHECK(n_rays > 0 && n_samples > 0, "%s: empty input", __func__);
    hipLaunchKernelGGL(k_encode_bwd, dim3(n_rays), dim3(64 * EB_WAVES), 0, as_stream(stream), pts_o, pts_d, view, z,
                       genc_p, genc_p2, genc_d, n_rays, n_samples, g_pts_o, g_pts_d, g_view);
    return check_launch(__func__);
}
