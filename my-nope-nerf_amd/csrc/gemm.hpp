// Shared pieces of the field-MLP GEMMs: launch arguments, the gfx950 32x32 MFMA C/D map
// and the fused epilogues.  Two K-loop bodies use them:
//   gemm_f32.hip  exact-f32 v_mfma_f32_32x32x2_f32 (64 FLOP/clk/SIMD);
//   gemm_x6.hip   f32 emulated on v_mfma_f32_32x32x16_bf16: every f32 operand is split
//                 into three bf16 words and the six significant cross products are
//                 accumulated in f32 (1024 FLOP/clk/SIMD / 6).
// The 32x32 C/D layout is dtype-independent on gfx950, so the epilogues are shared.
#pragma once
#include "common.hpp"

namespace nerf {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// accumulator register r of a 32x32 tile -> row offset inside the tile (gfx950 C/D map)
__device__ __forceinline__ int acc_row(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }

template <int TM, int TN>
__device__ __forceinline__ void zero_acc(f32x16 (&acc)[TM][TN]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
}

// NT GEMM: C[m][n] = epi( sum_k A[m][k] B[n][k] ), A from up to two K segments.
struct NTArgs {
    const float* a1; int lda1; int k1;
    const float* a2; int lda2; int k2;
    const float* b;  int ldb;           // [n][k1+k2]
    const uint16_t* bs; int bs_rows;    // optional bf16x3 image of b (split-bf16 kernels only)
    const float* bias;                  // fwd
    const float* u;  const float* v;    // bwd-data rank-1 term u[m*ldu] v[n]
    int ldu;
    const uint32_t* mask; int ldmask;   // bwd-data ReLU mask bits [m][n/32] (bit = x > 0)
    uint32_t* mask_out; int ldmo;       // fwd: write the ReLU mask bits of the output
    float* c; int ldc;
    int m, n;
    int relu;
    unsigned long long* stamps;   // diagnostics (nerf_gemm_debug_stamps): per-block phase clocks or NULL
    int ablate;   // diagnostics only (nerf_gemm_debug_ablate): 1 = no epilogue stores, 2 = no K-loop loads
                  // (f32 kernels; the split-bf16 kernels honour 1 only)
    // precision mode 2 (fp16 pair): max |a| per row of each A segment (ar2 may be NULL),
    // and (optional) the row max of the output written by the epilogue; c_cmax (optional):
    // column maxima of the output per 128-row group, [m/128][ldcm]
    const float* ar1; const float* ar2;
    float* c_rmax;
    float* c_cmax; int ldcm;
    // fused output heads (nerf_linear_fwd_heads, precision mode 2, one column block): raw4[m][raw_col + c]
    // = sum_f y[m][f] head_w[c][f] + head_b[c] for c < n_heads (official_nerf.py:66, 91)
    const float* head_w; const float* head_b; float* raw4;
    int n_heads; int raw_col;
};

__device__ __forceinline__ void store_out4(float* dst, const float4& x) { *reinterpret_cast<float4*>(dst) = x; }

// max |a| over row m of the (one or two segment) A operand
__device__ __forceinline__ float a_rowmax(const NTArgs& p, int m) {
    const float r1 = p.ar1[m];
    return p.ar2 ? fmaxf(r1, p.ar2[m]) : r1;
}

enum { EPI_FWD = 0, EPI_BWD = 1 };

// TN GEMM (weight gradient): slab[split][o][col0+j] = sum_s dy[s][o] x[s][j]
struct TNArgs {
    const float* dy; int lddy;   // A[m=o][k=s] = dy[s][o]
    const float* x;  int ldx;    // B[k=s][n=j] = x[s][j]
    int rows_per_split;
    float* slab; int ldslab; int col0; size_t slab_stride;
    float* bslab; int nout;
    int ablate;   // diagnostics: 1 = no slab stores, 2 = no K-loop loads, 4 = no bias column sums
    // precision mode 2: column maxima of dy and x per 128-row group ([m/128][ld]); the
    // fp16 pair kernel scales each split's columns by them
    const float* cm_dy; int ldcm_dy;
    const float* cm_x; int ldcm_x;
    unsigned long long* stamps;   // unused (the round-3 TN phase stamps were a diagnostic build)
};

// Backward-data epilogue operands (ReLU bits, rank-1 column), prefetched into registers
// with coalesced loads while the last K tile computes, parked in LDS by nt_epilogue.
template <int BM, int BN, int NT, int EPI>
struct NTEpiPrefetch {
    static constexpr int MW = BN / 32;                    // mask words per row of the tile
    static constexpr int M_PF = (BM * MW + NT - 1) / NT;  // mask words prefetched per thread
    uint32_t mpf[M_PF];
    float upf = 0.f;
    __device__ __forceinline__ void load(const NTArgs& p, int m0, int n0) {
        if (EPI != EPI_BWD) return;
        const int tid = threadIdx.x;
#pragma unroll
        for (int q = 0; q < M_PF; ++q) {
            const int e = tid + NT * q;
            mpf[q] = (p.mask && e < BM * MW) ? p.mask[(size_t)(m0 + e / MW) * p.ldmask + (n0 >> 5) + e % MW]
                                             : 0xffffffffu;
        }
        if (tid < BM) upf = p.u ? p.u[(size_t)(m0 + tid) * p.ldu] : 0.f;
    }
};

// Fused NT epilogue.  smem: at least BM*(BN/32) words + BM floats, free (after the last
// K-loop barrier).  FWD: +bias, ReLU, ReLU bit mask via ballot.  BWD: + u[m] v[n], masked.
template <int BM, int BN, int NT, int TM, int TN, int EPI>
__device__ __forceinline__ void nt_epilogue(const NTArgs& p, f32x16 (&acc)[TM][TN], float* smem, int m0, int n0,
                                            int wm0, int wn0, const NTEpiPrefetch<BM, BN, NT, EPI>& pf) {
    constexpr int MW = BN / 32;
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int l32 = lane & 31, hi = lane >> 5;
    if (p.ablate & 1) {   // keep the accumulators live, store one value per thread
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) t += acc[i][j][r];
        p.c[(size_t)(m0 + (tid & 127)) * p.ldc + n0 + (tid >> 7)] = t;
        return;
    }
    if (EPI == EPI_FWD) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn0 + 32 * j + l32;
            const int cword = (n0 + wn0 + 32 * j) >> 5;
            const float bcol = p.bias ? p.bias[col] : 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m0 + wm0 + 32 * i + acc_row(r, hi);
                    float x = acc[i][j][r] + bcol;
                    if (p.relu) x = fmaxf(x, 0.f);
                    p.c[(size_t)row * p.ldc + col] = x;
                    if (p.mask_out) {
                        // bits 0-31: the 32 columns of this register's row held by lanes 0-31,
                        // bits 32-63: the row held by lanes 32-63
                        const uint64_t bits = __ballot(x > 0.f);
                        if (l32 == 0)
                            p.mask_out[(size_t)row * p.ldmo + cword] = (uint32_t)(hi ? (bits >> 32) : bits);
                    }
                }
        }
    } else {
        uint32_t* lmask = reinterpret_cast<uint32_t*>(smem);
        float* lu = smem + BM * MW;
#pragma unroll
        for (int q = 0; q < NTEpiPrefetch<BM, BN, NT, EPI>::M_PF; ++q) {
            const int e = tid + NT * q;
            if (e < BM * MW) lmask[e] = pf.mpf[q];
        }
        if (tid < BM) lu[tid] = pf.upf;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn0 + 32 * j + l32;
            const int cw = (wn0 + 32 * j) >> 5;
            const float vcol = p.u ? p.v[col] : 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int lr = wm0 + 32 * i + acc_row(r, hi);
                    float x = acc[i][j][r] + lu[lr] * vcol;
                    x = ((lmask[lr * MW + cw] >> l32) & 1u) ? x : 0.f;
                    p.c[(size_t)(m0 + lr) * p.ldc + col] = x;
                }
        }
    }
}

// TN epilogue: this split's partial weight gradient tile into its slab
template <int TM, int TN>
__device__ __forceinline__ void tn_store(const TNArgs& p, f32x16 (&acc)[TM][TN], int split, int o0, int j0,
                                         int wm0, int wn0) {
    float* slab = p.slab + (size_t)split * p.slab_stride;
    const int lane = lane_id();
    const int l32 = lane & 31, hi = lane >> 5;
    if (p.ablate & 1) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) t += acc[i][j][r];
        slab[threadIdx.x] = t;
        return;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = o0 + wm0 + 32 * i + acc_row(r, hi);
                const int c = p.col0 + j0 + wn0 + 32 * j + l32;
                slab[(size_t)o * p.ldslab + c] = acc[i][j][r];
            }
}

// diagnostics: wave 0 of each block records (s_memtime, s_memrealtime) at phase
// boundaries into stamps[block][phase][2]
constexpr int kStampPhases = 10;
__device__ __forceinline__ void stamp(unsigned long long* st, int phase) {
    if (st == nullptr) return;
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    const unsigned long long r = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        const size_t b = (size_t)blockIdx.x + (size_t)gridDim.x * (blockIdx.y + (size_t)gridDim.y * blockIdx.z);
        st[(b * kStampPhases + phase) * 2] = t;
        st[(b * kStampPhases + phase) * 2 + 1] = r;
    }
    __builtin_amdgcn_sched_barrier(0);
}

// ---------------------------------------------------------------------------
// LDS-transposed tile writer (split-bf16 kernels).  The 32x32 C/D layout gives each
// lane one column of 16 rows, so storing from registers takes one 4-byte store per
// element (256 per wave at a 128x128 wave tile) and the store issue dominates the
// epilogue.  Instead each wave writes its tile, 64 rows per pass, into a private LDS
// region (rows padded to WTN + 8 floats: the column writes of lanes 0-31 and 32-63
// land on disjoint banks) and reads it back as row-contiguous float4s: emit(row, col,
// v) is called for WTN/4 lanes per row, 64*4/WTN rows per wave-instruction.
// ---------------------------------------------------------------------------
template <int TN>
struct TileLds {
    static constexpr int WTN = 32 * TN;
    static constexpr int LD = WTN + 8;              // floats per LDS row
    static constexpr int BYTES = 64 * LD * 4;       // per wave
    static constexpr int LPR = WTN / 4;             // lanes per row (read phase)
    static constexpr int RPI = 64 / LPR;            // rows per read instruction
};

template <int TM, int TN, typename Emit>
__device__ __forceinline__ void write_tile_lds(f32x16 (&acc)[TM][TN], float* wlds, Emit&& emit) {
    using T = TileLds<TN>;
    const int lane = lane_id();
    const int l32 = lane & 31, hi = lane >> 5;
#pragma unroll
    for (int h = 0; h < TM; h += 2) {
        constexpr int NT2 = TM >= 2 ? 2 : 1;
#pragma unroll
        for (int ii = 0; ii < NT2; ++ii)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    wlds[(32 * ii + acc_row(r, hi)) * T::LD + 32 * j + l32] = acc[h + ii][j][r];
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int q = 0; q < 32 * NT2 / T::RPI; ++q) {
            const int rl = q * T::RPI + lane / T::LPR;
            const int c4 = (lane % T::LPR) * 4;
            const float4 v = *reinterpret_cast<const float4*>(wlds + rl * T::LD + c4);
            emit(32 * h + rl, c4, v);
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
}

// ReLU mask word of 32 columns from 8 lanes holding 4 consecutive columns each (lane
// groups of 8 aligned to the word): valid in the lane with (lane & 7) == 0.  The OR over
// the 8 lanes runs on DPP (quad_perm xor 1, xor 2, then row_half_mirror), not on
// ds_bpermute round trips.
__device__ __forceinline__ uint32_t mask_word8(float4 v) {
    const uint32_t nib = (v.x > 0.f ? 1u : 0u) | (v.y > 0.f ? 2u : 0u) | (v.z > 0.f ? 4u : 0u) | (v.w > 0.f ? 8u : 0u);
    int w = (int)(nib << (4 * (lane_id() & 7)));
    w |= __builtin_amdgcn_mov_dpp(w, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    w |= __builtin_amdgcn_mov_dpp(w, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    w |= __builtin_amdgcn_mov_dpp(w, 0x141, 0xF, 0xF, false);   // row_half_mirror
    return (uint32_t)w;
}

// Fused NT epilogue through the LDS writer.  smem layout: [4 waves][TileLds::BYTES],
// then (BWD) the parked mask words and u column.
template <int BM, int BN, int NT, int TM, int TN, int EPI>
__device__ __forceinline__ void nt_epilogue_lds(const NTArgs& p, f32x16 (&acc)[TM][TN], char* smem, int m0,
                                                int n0, int wm0, int wn0,
                                                const NTEpiPrefetch<BM, BN, NT, EPI>& pf) {
    using T = TileLds<TN>;
    constexpr int MW = BN / 32;
    constexpr int NW = NT / 64;
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    if (p.ablate & 1) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) t += acc[i][j][r];
        p.c[(size_t)(m0 + (tid & 127)) * p.ldc + n0 + (tid >> 7)] = t;
        return;
    }
    float* wlds = reinterpret_cast<float*>(smem + wave * T::BYTES);
    const int c4l = (lane_id() % T::LPR) * 4;          // this lane's 4 columns (read phase)
    const int col = n0 + wn0 + c4l;
    if (EPI == EPI_FWD) {
        // ReLU mask words are gathered in LDS and written as the block's contiguous rows
        // at the end (per-wave 16-byte pieces at a 32-byte row stride are partial-line
        // HBM writes)
        uint32_t* lmask = reinterpret_cast<uint32_t*>(smem + NW * T::BYTES);
        const float4 b4 = p.bias ? *reinterpret_cast<const float4*>(p.bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
        const int cw = (wn0 + c4l) >> 5;
        write_tile_lds<TM, TN>(acc, wlds, [&](int rl, int c4, float4 v) {
            const int row = m0 + wm0 + rl;
            float4 x = make_float4(v.x + b4.x, v.y + b4.y, v.z + b4.z, v.w + b4.w);
            if (p.relu) x = make_float4(fmaxf(x.x, 0.f), fmaxf(x.y, 0.f), fmaxf(x.z, 0.f), fmaxf(x.w, 0.f));
            *reinterpret_cast<float4*>(p.c + (size_t)row * p.ldc + col) = x;
            if (p.mask_out) {
                const uint32_t w = mask_word8(x);
                if ((lane_id() & 7) == 0) lmask[(wm0 + rl) * MW + cw] = w;
            }
        });
        if (p.mask_out) {
            __syncthreads();
            for (int e = tid; e < BM * MW; e += NT)
                p.mask_out[(size_t)(m0 + e / MW) * p.ldmo + (n0 >> 5) + e % MW] = lmask[e];
        }
    } else {
        uint32_t* lmask = reinterpret_cast<uint32_t*>(smem + NW * T::BYTES);
        float* lu = reinterpret_cast<float*>(lmask + BM * MW);
#pragma unroll
        for (int q = 0; q < NTEpiPrefetch<BM, BN, NT, EPI>::M_PF; ++q) {
            const int e = tid + NT * q;
            if (e < BM * MW) lmask[e] = pf.mpf[q];
        }
        if (tid < BM) lu[tid] = pf.upf;
        __syncthreads();
        const float4 v4 = p.u ? *reinterpret_cast<const float4*>(p.v + col) : make_float4(0.f, 0.f, 0.f, 0.f);
        const int cw = (wn0 + c4l) >> 5, sh = (wn0 + c4l) & 31;
        write_tile_lds<TM, TN>(acc, wlds, [&](int rl, int c4, float4 v) {
            const int lr = wm0 + rl;
            const float u = lu[lr];
            const uint32_t bits = lmask[lr * MW + cw] >> sh;
            float4 x = make_float4(v.x + u * v4.x, v.y + u * v4.y, v.z + u * v4.z, v.w + u * v4.w);
            x.x = (bits & 1u) ? x.x : 0.f;
            x.y = (bits & 2u) ? x.y : 0.f;
            x.z = (bits & 4u) ? x.z : 0.f;
            x.w = (bits & 8u) ? x.w : 0.f;
            *reinterpret_cast<float4*>(p.c + (size_t)(m0 + lr) * p.ldc + col) = x;
        });
    }
}

// One halving step of a max-butterfly over the lanes of a half-wave: lanes whose STEP bit is
// set keep the upper HALF values, the rest the lower, each merged with its partner's copy;
// base tracks the first feature index kept.  HALF = 0: no halving, plain exchange.
template <int HALF, int STEP, int NV>
__device__ __forceinline__ void bfly_max(float (&v)[NV], int sl, int& base) {
    const bool bit = (sl & STEP) != 0;
    if constexpr (HALF >= 1) {
#pragma unroll
        for (int t = 0; t < HALF; ++t) {
            const float keep = bit ? v[t + HALF] : v[t];
            const float send = bit ? v[t] : v[t + HALF];
            v[t] = fmaxf(keep, __shfl_xor(send, STEP, 64));
        }
        base += bit ? HALF : 0;
    } else {
        v[0] = fmaxf(v[0], __shfl_xor(v[0], STEP, 64));
    }
}

// The same halving step with the partner lane read by DPP instead of ds_bpermute (no LDS
// round trip; the move folds into the max).  CTRL pairs every lane with one that differs in
// the STEP bit: row_mirror (r <-> 15 - r) for 8, row_half_mirror for 4, quad_perm [3,2,1,0]
// for 2, [1,0,3,2] for 1.  A mirror also flips the lower bits, so the steps must run from the
// high bit down (each partner then agrees on every bit already reduced, hence on the kept
// feature set); xor 16 keeps the shuffle and can run anywhere.
template <int HALF, int STEP, int NV>
__device__ __forceinline__ void bfly_max_dpp(float (&v)[NV], int sl, int& base) {
    constexpr int CTRL = STEP == 8 ? 0x140 : STEP == 4 ? 0x141 : STEP == 2 ? 0x1B : 0xB1;
    static_assert(STEP == 8 || STEP == 4 || STEP == 2 || STEP == 1, "DPP pairing for bits 0-3 only");
    const bool bit = (sl & STEP) != 0;
#pragma unroll
    for (int t = 0; t < HALF; ++t) {
        const float keep = bit ? v[t + HALF] : v[t];
        const float send = bit ? v[t] : v[t + HALF];
        const float part = __builtin_bit_cast(
            float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, send), CTRL, 0xF, 0xF, false));
        v[t] = fmaxf(keep, part);
    }
    base += bit ? HALF : 0;
}

// Direct NT epilogue for the operand-swapped K loop (the MFMAs compute C^T tiles, so each
// lane holds one sample row and, per register quad 4q..4q+3, four consecutive output
// features 8q + 4*(lane>>5) + 0..3): float4 stores straight from the accumulators, no
// LDS round trip and no block barrier.  A wave's four quads of a 32x32 tile cover 128 B
// of each of its 32 rows; L2 merges them into full lines.
//   FWD: + bias, ReLU, ReLU mask word per (row, 32 features) from the nibbles of the
//        lane pair (lane, lane ^ 32).
//   BWD: + u[row] v[feature], masked by the input layer's ReLU bits.
//   H (precision mode 2): the accumulators carry the row scales 2^(ea[row] + eb[feature])
//        (LDS arrays lea / leb, block-local indices), undone first; the row max of the
//        stored values is max-accumulated into lrm (LDS, float bits) for NTArgs::c_rmax.
//   lvb (optional): the column block's bias (FWD) / v (BWD) staged in LDS by the kernel; a global load
//        issued between the stores would make its wait retire every earlier store first.

template <int TM, int TN, int EPI, bool H = false, bool HD = false>
__device__ __forceinline__ void nt_epilogue_direct(const NTArgs& p, f32x16 (&acc)[TM][TN], int m0, int n0, int wm0,
                                                   int wn0, uint32_t* lmask = nullptr, int mw = 0,
                                                   const int* leb = nullptr, const int* lea = nullptr,
                                                   uint32_t* lrm = nullptr, uint32_t* lcm = nullptr, int lcm_ld = 0,
                                                   float* lhs = nullptr, const float* lhw = nullptr, int lhw_ld = 0,
                                                   const float* lvb = nullptr) {
    const int lane = lane_id();
    const int sl = lane & 31, hf = lane >> 5;
    int er[TM];
    float rmx[TM];
    constexpr int NV = 16 * TN;       // this lane's features (j, q, c) -> index 16 j + 4 q + c
    float cmx[NV];
#pragma unroll
    for (int f = 0; f < NV; ++f) cmx[f] = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        er[i] = H ? lea[wm0 + 32 * i + sl] : 0;
        rmx[i] = 0.f;
    }
    // undo the operand scales of register quad q (features fl .. fl+3, block-local)
    auto unscale = [&](int i, int j, int q) {
        if constexpr (H) {
            const int4 eb = *reinterpret_cast<const int4*>(leb + wn0 + 32 * j + 4 * hf + 8 * q);
            acc[i][j][4 * q + 0] = __builtin_amdgcn_ldexpf(acc[i][j][4 * q + 0], -(er[i] + eb.x));
            acc[i][j][4 * q + 1] = __builtin_amdgcn_ldexpf(acc[i][j][4 * q + 1], -(er[i] + eb.y));
            acc[i][j][4 * q + 2] = __builtin_amdgcn_ldexpf(acc[i][j][4 * q + 2], -(er[i] + eb.z));
            acc[i][j][4 * q + 3] = __builtin_amdgcn_ldexpf(acc[i][j][4 * q + 3], -(er[i] + eb.w));
        }
    };
    auto out4 = [&](float* dst, const float4& x) { store_out4(dst, x); };
    auto track = [&](int i, int j, int q, const float4& x) {
        if constexpr (H) {
            rmx[i] = fmaxf(rmx[i], fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
            if (lcm) {
#pragma unroll
                for (int jj = 0; jj < TN; ++jj)
#pragma unroll
                    for (int qq = 0; qq < 4; ++qq)
                        if (jj == j && qq == q) {
                            cmx[16 * jj + 4 * qq + 0] = fmaxf(cmx[16 * jj + 4 * qq + 0], fabsf(x.x));
                            cmx[16 * jj + 4 * qq + 1] = fmaxf(cmx[16 * jj + 4 * qq + 1], fabsf(x.y));
                            cmx[16 * jj + 4 * qq + 2] = fmaxf(cmx[16 * jj + 4 * qq + 2], fabsf(x.z));
                            cmx[16 * jj + 4 * qq + 3] = fmaxf(cmx[16 * jj + 4 * qq + 3], fabsf(x.w));
                        }
            }
        }
    };
    if (p.ablate & 1) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) t += acc[i][j][r];
        p.c[(size_t)(m0 + (threadIdx.x & 127)) * p.ldc + n0 + (threadIdx.x >> 7)] = t;
        return;
    }
    const int cw0 = (n0 + wn0) >> 5;
    // fused heads (FWD, H only): this lane's partial dots over its features, per row tile
    const int nh = (EPI == EPI_FWD && H && HD) ? p.n_heads : 0;   // HD: instantiated for the head layers only
    float hp[3][TM];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int i = 0; i < TM; ++i) hp[c][i] = 0.f;
    if (EPI == EPI_FWD) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int fb = n0 + wn0 + 32 * j + 4 * hf;
            float4 b4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                b4[q] = lvb ? *reinterpret_cast<const float4*>(lvb + (fb - n0) + 8 * q)
                      : p.bias ? *reinterpret_cast<const float4*>(p.bias + fb + 8 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const size_t row = (size_t)(m0 + wm0 + 32 * i + sl);
                uint32_t w = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    unscale(i, j, q);
                    float4 x = make_float4(acc[i][j][4 * q] + b4[q].x, acc[i][j][4 * q + 1] + b4[q].y,
                                           acc[i][j][4 * q + 2] + b4[q].z, acc[i][j][4 * q + 3] + b4[q].w);
                    if (p.relu) x = make_float4(fmaxf(x.x, 0.f), fmaxf(x.y, 0.f), fmaxf(x.z, 0.f), fmaxf(x.w, 0.f));
                    if constexpr (EPI == EPI_FWD && H && HD) {
#pragma unroll
                        for (int c = 0; c < 3; ++c)
                            if (c < nh) {
                                // head weights staged in LDS (block-local features)
                                const float4 hw = *reinterpret_cast<const float4*>(lhw + c * lhw_ld + (fb - n0) + 8 * q);
                                hp[c][i] += x.x * hw.x + x.y * hw.y + x.z * hw.z + x.w * hw.w;
                            }
                    }
                    track(i, j, q, x);
                    out4(p.c + row * p.ldc + fb + 8 * q, x);
                    const uint32_t nib = (x.x > 0.f ? 1u : 0u) | (x.y > 0.f ? 2u : 0u) | (x.z > 0.f ? 4u : 0u) |
                                         (x.w > 0.f ? 8u : 0u);
                    w |= nib << (8 * q + 4 * hf);
                }
                if (p.mask_out) {
                    w |= (uint32_t)__shfl_xor((int)w, 32, 64);
                    // gathered in LDS and stored as the block's contiguous mask rows by the
                    // caller (4-byte stores at a 32-byte row stride are partial-line writes)
                    if (hf == 0) {
                        if (lmask) lmask[(wm0 + 32 * i + sl) * mw + (wn0 >> 5) + j] = w;
                        else p.mask_out[row * p.ldmo + cw0 + j] = w;
                    }
                }
            }
        }
    } else {
        float u[TM];
        uint32_t mw[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const size_t row = (size_t)(m0 + wm0 + 32 * i + sl);
            u[i] = p.u ? p.u[row * p.ldu] : 0.f;
#pragma unroll
            for (int j = 0; j < TN; ++j) mw[i][j] = p.mask ? p.mask[row * p.ldmask + cw0 + j] : 0xffffffffu;
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int fb = n0 + wn0 + 32 * j + 4 * hf;
            float4 v4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                v4[q] = lvb ? *reinterpret_cast<const float4*>(lvb + (fb - n0) + 8 * q)
                      : p.u ? *reinterpret_cast<const float4*>(p.v + fb + 8 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const size_t row = (size_t)(m0 + wm0 + 32 * i + sl);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    unscale(i, j, q);
                    const uint32_t bits = mw[i][j] >> (8 * q + 4 * hf);
                    float4 x = make_float4(acc[i][j][4 * q] + u[i] * v4[q].x, acc[i][j][4 * q + 1] + u[i] * v4[q].y,
                                           acc[i][j][4 * q + 2] + u[i] * v4[q].z, acc[i][j][4 * q + 3] + u[i] * v4[q].w);
                    x.x = (bits & 1u) ? x.x : 0.f;
                    x.y = (bits & 2u) ? x.y : 0.f;
                    x.z = (bits & 4u) ? x.z : 0.f;
                    x.w = (bits & 8u) ? x.w : 0.f;
                    track(i, j, q, x);
                    out4(p.c + row * p.ldc + fb + 8 * q, x);
                }
            }
        }
    }
    if (HD && nh) {
        // head partials: the lane pair (lane, lane ^ 32) holds one row's features of this wave;
        // lhs is this wave's [BM][3] slot (one per wave along N), summed in wave order by the
        // kernel (deterministic)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int c = 0; c < 3; ++c)
                if (c < nh) {
                    const float v = hp[c][i] + __shfl_xor(hp[c][i], 32, 64);
                    if (hf == 0) lhs[(wm0 + 32 * i + sl) * 3 + c] = v;
                }
    }
    if constexpr (H) {
        // the lane pair (lane, lane ^ 32) holds one row's features of this wave; the other
        // waves along N meet in LDS (non-negative floats order like their bits)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const float m = fmaxf(rmx[i], __shfl_xor(rmx[i], 32, 64));
            if (hf == 0) atomicMax(lrm + wm0 + 32 * i + sl, __float_as_uint(m));
        }
        if (lcm) {
            // column maxima over this wave's rows: a halving butterfly over the 32 lanes of each
            // half-wave (xor 16 .. 1) leaves lane sl with features base + t; the waves along M
            // of one 128-row group meet in LDS
            // (bits 3..0 by DPP, high bit first; bit 4 by shuffle once 2 values are left)
            int base = 0;
            bfly_max_dpp<NV / 2, 8>(cmx, sl, base);
            bfly_max_dpp<NV / 4, 4>(cmx, sl, base);
            bfly_max_dpp<NV / 8, 2>(cmx, sl, base);
            bfly_max_dpp<NV / 16, 1>(cmx, sl, base);
            bfly_max<NV / 32, 16>(cmx, sl, base);
            constexpr int n = NV / 32 > 1 ? NV / 32 : 1;   // features left per lane
            uint32_t* g = lcm + (wm0 / 128) * lcm_ld;
#pragma unroll
            for (int t = 0; t < n; ++t) {
                const int f = base + t;
                atomicMax(g + wn0 + 32 * (f >> 4) + 4 * hf + 8 * ((f >> 2) & 3) + (f & 3), __float_as_uint(cmx[t]));
            }
        }
    }
}

// TN epilogue through the LDS writer: float4 slab stores.  H: undo the scales 2^(ea[row] +
// eb[col]) of the fp16 pair kernel (block-local exponent arrays in LDS).
template <int TM, int TN, bool H = false>
__device__ __forceinline__ void tn_store_lds(const TNArgs& p, f32x16 (&acc)[TM][TN], char* smem, int split, int o0,
                                             int j0, int wm0, int wn0, const int* lea = nullptr,
                                             const int* leb = nullptr) {
    using T = TileLds<TN>;
    if (p.ablate & 1) {
        tn_store(p, acc, split, o0, j0, wm0, wn0);
        return;
    }
    float* slab = p.slab + (size_t)split * p.slab_stride;
    float* wlds = reinterpret_cast<float*>(smem + (threadIdx.x >> 6) * T::BYTES);
    write_tile_lds<TM, TN>(acc, wlds, [&](int rl, int c4, float4 v) {
        if constexpr (H) {
            const int ea = lea[wm0 + rl];
            const int4 eb = *reinterpret_cast<const int4*>(leb + wn0 + c4);
            v.x = __builtin_amdgcn_ldexpf(v.x, -(ea + eb.x));
            v.y = __builtin_amdgcn_ldexpf(v.y, -(ea + eb.y));
            v.z = __builtin_amdgcn_ldexpf(v.z, -(ea + eb.z));
            v.w = __builtin_amdgcn_ldexpf(v.w, -(ea + eb.w));
        }
        float* d = slab + (size_t)(o0 + wm0 + rl) * p.ldslab + p.col0 + j0 + wn0 + c4;
        {   // (plain stores: non-temporal slab stores made the weight gradients slower, 368-373 vs
            // 329-333 us per launch, profiles/r05/chain_nt_ab.txt)
            store_out4(d, v);
        }
    });
}

// TN policies 7 and 8 (8 the default, nerf_gemm_set_policy): a 256 x 256 weight gradient in the split
// modes runs as XCD-paired 256 x 128 column tiles of eight waves (k_gemm_tn_x6 CT = 2), twice the rows
// per split at the same block count; needs a split count that is a multiple of 8
inline int tn_xcd_group(int policy, int nout, int kin, int splits) {
    return (policy >= 7 && nout == 256 && kin == 256 && splits % 8 == 0) ? 2 : 0;
}

// split-bf16 launchers (gemm_x6.hip); policy as nerf_gemm_set_policy
int dispatch_nt_x6(const NTArgs& a, int epi, int policy, hipStream_t s, double flops, bool h16 = false);
int dispatch_tn_x6(const TNArgs& a, int nout, int kin, int splits, int policy, hipStream_t s, double flops,
                   bool h16 = false);
// the two-segment weight gradient in one launch (fp16 pair, TN policy 7 shapes only)
bool tn_seg_supported(int nout, int k1, int k2, int splits);
int dispatch_tn_x6_seg(const TNArgs& pm, const TNArgs& ps, int nout, int splits, int policy, hipStream_t s,
                       double flops);
// the 4-wave weight-gradient kernels (wgrad.hip): which shapes they cover, and their launchers
bool wgrad_supported(int nout, int kin, int splits, int rows_per_split);
bool wgrad_seg_supported(int nout, int k1, int k2, int splits, int rows_per_split);
void launch_wgrad(const TNArgs& a, int nout, int kin, int splits, hipStream_t s);
void launch_wgrad_seg(const TNArgs& pm, const TNArgs& ps, int nout, int splits, hipStream_t s);
// several 256 x 256 layers of the same split count in one launch (k_wgrad_pairs)
struct TNPairs {
    TNArgs a[kWgradPairsMax];
    int n;
};
void launch_wgrad_pairs(const TNPairs& m, int splits, hipStream_t s);
// a job list of weight-gradient tiles of several shapes in one launch (k_wgrad_jobs)
enum WgradJobKind : int { WJ_PAIR = 0, WJ_WIDE = 1, WJ_ENC = 2, WJ_ENC_HALF = 3, WJ_ENC128 = 4 };
struct TNJobs {
    TNArgs a[kWgradJobsMax];
    int kind[kWgradJobsMax];
    int grp[kWgradJobsMax];   // the block group that runs job i (0 .. ngroups - 1)
    int n;
    int ngroups;              // the launch is ngroups x 2 S blocks, each group walking its own jobs
};
void launch_wgrad_jobs(const TNJobs& m, int splits, hipStream_t s);
void launch_wgrad_two(const TNArgs& a, int na, const TNArgs& b, int nb, hipStream_t s);

}  // namespace nerf
