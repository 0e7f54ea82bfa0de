// FP32 MFMA GEMMs for the NeRF field MLP (forward, backward-data, backward-weight).
//
// Replaces the cuBLAS SGEMM (addmm) + ReLU + torch.cat work of
// OfficialStaticNerf.infer_occ/forward (official_nerf.py:60-96) and its autograd
// backward (training.py:92), SURVEY.md section 2.1 K4/K12.
//
// Design (gfx950):
//  * exact-f32 v_mfma_f32_32x32x2_f32 (64 FLOP/clk/SIMD, the f32 peak; no xf32 on
//    CDNA4) so results stay an f32 fma chain -> 1e-4 parity with the fp32 reference;
//  * 256-thread workgroups (4 waves), block tile BM x BN, BK = 32, LDS k-major
//    images As[k][m], Bs[k][n] double-buffered, register-staged global loads issued
//    before the MFMA block of the current tile (one barrier per K tile);
//  * K-contiguous operands (activations [m][k], weights [n][k]) are transposed while
//    staging: 16-B global loads, 4 ds_write_b32 into rows padded to BM+1 floats,
//    which keeps both the stores and the per-lane MFMA operand reads conflict-free;
//  * sample-major operands of the weight gradient (dy[s][o], x[s][j]) are already
//    k-major: 16-B loads and ds_write_b128 into rows padded to BM+4 floats;
//  * fused epilogues: +bias/ReLU (forward), rank-1 add + ReLU-mask (backward-data),
//    split-K slab + bias-gradient column sums (backward-weight).
#include "gemm.hpp"

#include <cstdlib>

namespace nerf {

constexpr int BK = 32;

// ---------------------------------------------------------------------------
// shared MFMA block: acc[TM][TN] += As[k][wm0..] x Bs[k][wn0..] over BK
// ---------------------------------------------------------------------------
// SWAP: the weight fragment is the MFMA's A operand, so acc[i][j] holds the transposed tile
// (lanes along samples, registers along features: nt_epilogue_direct's float4 row stores)
template <int TM, int TN, int LDA, int LDB, bool SWAP = false>
__device__ __forceinline__ void mfma_tile(const float* __restrict__ As, const float* __restrict__ Bs,
                                          int wm0, int wn0, f32x16 (&acc)[TM][TN]) {
    // operands of k-pair kp+1 are read from LDS before the MFMAs of kp issue, so the
    // ds_read latency hides behind 64-cycle MFMAs instead of stalling every group
    const int lane = lane_id();
    const int l32 = lane & 31;
    const int hi = lane >> 5;
    // two NAMED operand sets (a runtime-indexed a[cur] would live in scratch, guide rule 20)
    float a0[TM], b0[TN], a1[TM], b1[TN];
    auto rd = [&](int kp, float (&ra)[TM], float (&rb)[TN]) {
        const int k = 2 * kp + hi;
#pragma unroll
        for (int i = 0; i < TM; ++i) ra[i] = As[k * LDA + wm0 + 32 * i + l32];
#pragma unroll
        for (int j = 0; j < TN; ++j) rb[j] = Bs[k * LDB + wn0 + 32 * j + l32];
    };
    auto mm = [&](const float (&ra)[TM], const float (&rb)[TN]) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                acc[i][j] = SWAP ? __builtin_amdgcn_mfma_f32_32x32x2f32(rb[j], ra[i], acc[i][j], 0, 0, 0)
                                 : __builtin_amdgcn_mfma_f32_32x32x2f32(ra[i], rb[j], acc[i][j], 0, 0, 0);
    };
    rd(0, a0, b0);
#pragma unroll
    for (int kp = 0; kp < BK / 2; kp += 2) {
        rd(kp + 1, a1, b1);
        // pin the order: hipcc otherwise sinks the reads below the MFMAs and reuses one
        // operand register set, exposing the LDS latency before every MFMA group
        __builtin_amdgcn_sched_barrier(0);
        mm(a0, b0);
        if (kp + 2 < BK / 2) rd(kp + 2, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        mm(a1, b1);
    }
}

// ---------------------------------------------------------------------------
// NT GEMM: C[m][n] = epi( sum_k A[m][k] B[n][k] ), A from up to two K segments.
// WM x WN waves; each wave owns a (BM/WM) x (BN/WN) output tile of 32x32 MFMA blocks.
// ---------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_nt(NTArgs p) {
    constexpr int NT = 64 * WM * WN;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int LDA = BM + 1, LDB = BN + 1;     // odd strides: conflict-free transposing stores
    constexpr int A_F4 = BM * BK / 4 / NT;
    constexpr int B_F4 = BN * BK / 4 / NT;
    static_assert(A_F4 >= 1 && B_F4 >= 1 && TM >= 1 && TN >= 1, "bad tile");

    __shared__ __attribute__((aligned(16))) float smem[2 * BK * (LDA + LDB)];
    auto As = [&](int buf) { return smem + buf * BK * LDA; };
    auto Bs = [&](int buf) { return smem + 2 * BK * LDA + buf * BK * LDB; };

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int wm0 = (wave / WN) * WTM;
    const int wn0 = (wave % WN) * WTN;
    const int m0 = blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const int nkt = (p.k1 + p.k2) / BK;

    // staging addresses: a wave-uniform base (SGPRs) + a 32-bit per-thread offset that is
    // the same for every K tile (keeps VGPR use and 64-bit address math out of the loop)
    const float* __restrict__ a1b = p.a1 + (size_t)m0 * p.lda1;
    const float* __restrict__ a2b = p.a2 ? p.a2 + (size_t)m0 * p.lda2 : nullptr;
    const float* __restrict__ bb = p.b + (size_t)n0 * p.ldb;
    const int r0 = tid >> 3, kc4 = 4 * (tid & 7);
    const int ao1 = r0 * p.lda1 + kc4, ao2 = r0 * p.lda2 + kc4, bo = r0 * p.ldb + kc4;
    constexpr int RSTEP = NT / 8;   // rows covered by one pass of the block
    float4 ra[A_F4], rb[B_F4];
    auto load_tile = [&](int kt) {
        const int kk = kt * BK;
        const bool seg1 = kk < p.k1;
        const float* abase = seg1 ? a1b + kk : a2b + (kk - p.k1);
        const int lda = seg1 ? p.lda1 : p.lda2;
        const int ao = seg1 ? ao1 : ao2;
#pragma unroll
        for (int i = 0; i < A_F4; ++i)
            ra[i] = *reinterpret_cast<const float4*>(abase + ao + i * RSTEP * lda);
#pragma unroll
        for (int i = 0; i < B_F4; ++i)
            rb[i] = *reinterpret_cast<const float4*>(bb + kk + bo + i * RSTEP * p.ldb);
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int i = 0; i < A_F4; ++i) {
            const int idx = tid + NT * i;
            const int row = idx >> 3, kc = idx & 7;
            float* d = As(buf) + (4 * kc) * LDA + row;
            d[0] = ra[i].x; d[LDA] = ra[i].y; d[2 * LDA] = ra[i].z; d[3 * LDA] = ra[i].w;
        }
#pragma unroll
        for (int i = 0; i < B_F4; ++i) {
            const int idx = tid + NT * i;
            const int row = idx >> 3, kc = idx & 7;
            float* d = Bs(buf) + (4 * kc) * LDB + row;
            d[0] = rb[i].x; d[LDB] = rb[i].y; d[2 * LDB] = rb[i].z; d[3 * LDB] = rb[i].w;
        }
    };

    f32x16 acc[TM][TN];
    zero_acc(acc);

    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nkt && !(p.ablate & 2)) load_tile(kt + 1);
        mfma_tile<TM, TN, LDA, LDB, true>(As(cur), Bs(cur), wm0, wn0, acc);
        if (kt + 1 < nkt) store_tile(cur ^ 1);
        __syncthreads();
    }

    // operand-swapped accumulators: every lane owns one sample row, four consecutive features
    // per register quad -> one float4 store each (4x fewer store instructions than one float
    // per accumulator register; the row-per-lane store tail is issue-bound).  The column
    // block's bias (FWD) / rank-1 v (BWD) is staged in LDS first (after the last barrier the
    // image buffers are free): a global load between the stores would wait for all of them.
    float* lvb = smem;
    const float* vb = EPI == EPI_FWD ? p.bias : (p.u ? p.v : nullptr);
    if (vb) {
        for (int e = tid; e < BN; e += NT) lvb[e] = vb[n0 + e];
        __syncthreads();
    }
    nt_epilogue_direct<TM, TN, EPI>(p, acc, m0, n0, wm0, wn0, nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0,
                                    nullptr, nullptr, 0, vb ? lvb : nullptr);
}

// ---------------------------------------------------------------------------
// TN GEMM (weight gradient): slab[split][o][col0+j] = sum_s dy[s][o] x[s][j]
// ---------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_tn(TNArgs p) {
    constexpr int NT = 64 * WM * WN;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int LDA = BM + 4, LDB = BN + 4;   // 16-B aligned rows for ds_write_b128
    constexpr int A_F4 = BM * BK / 4 / NT;
    constexpr int B_F4 = BN * BK / 4 / NT;
    constexpr int A_C4 = BM / 4, B_C4 = BN / 4;
    static_assert(A_F4 >= 1 && B_F4 >= 1, "bad tile");

    __shared__ __attribute__((aligned(16))) float smem[2 * BK * (LDA + LDB)];
    auto As = [&](int buf) { return smem + buf * BK * LDA; };
    auto Bs = [&](int buf) { return smem + 2 * BK * LDA + buf * BK * LDB; };

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int wm0 = (wave / WN) * WTM;
    const int wn0 = (wave % WN) * WTN;
    const int o0 = blockIdx.x * BM;
    const int j0 = blockIdx.y * BN;
    const int split = blockIdx.z;
    const size_t s0 = (size_t)split * p.rows_per_split;
    const int nkt = p.rows_per_split / BK;
    const bool do_bias = (p.bslab != nullptr) && (blockIdx.y == 0) && !(p.ablate & 4);

    // wave-uniform bases + constant 32-bit per-thread offsets (see k_gemm_nt)
    const float* __restrict__ dyb = p.dy + s0 * p.lddy + o0;
    const float* __restrict__ xb = p.x + s0 * p.ldx + j0;
    const int ao = (tid / A_C4) * p.lddy + 4 * (tid % A_C4);
    const int bo = (tid / B_C4) * p.ldx + 4 * (tid % B_C4);
    constexpr int ARSTEP = NT / A_C4, BRSTEP = NT / B_C4;
    float4 ra[A_F4], rb[B_F4];
    auto load_tile = [&](int kt) {
        const float* da = dyb + (size_t)kt * BK * p.lddy;
        const float* db = xb + (size_t)kt * BK * p.ldx;
#pragma unroll
        for (int i = 0; i < A_F4; ++i)
            ra[i] = *reinterpret_cast<const float4*>(da + ao + i * ARSTEP * p.lddy);
#pragma unroll
        for (int i = 0; i < B_F4; ++i)
            rb[i] = *reinterpret_cast<const float4*>(db + bo + i * BRSTEP * p.ldx);
    };
    auto store_tile = [&](int buf) {
        // component-wise copies: a whole-float4 aggregate store made hipcc keep ra/rb in
        // a scratch (stack) array instead of registers
#pragma unroll
        for (int i = 0; i < A_F4; ++i) {
            const int idx = tid + NT * i;
            const int row = idx / A_C4, c4 = idx % A_C4;
            *reinterpret_cast<float4*>(As(buf) + row * LDA + 4 * c4) = make_float4(ra[i].x, ra[i].y, ra[i].z, ra[i].w);
        }
#pragma unroll
        for (int i = 0; i < B_F4; ++i) {
            const int idx = tid + NT * i;
            const int row = idx / B_C4, c4 = idx % B_C4;
            *reinterpret_cast<float4*>(Bs(buf) + row * LDB + 4 * c4) = make_float4(rb[i].x, rb[i].y, rb[i].z, rb[i].w);
        }
    };

    f32x16 acc[TM][TN];
    zero_acc(acc);
    float bsum = 0.f;

    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nkt && !(p.ablate & 2)) load_tile(kt + 1);
        mfma_tile<TM, TN, LDA, LDB>(As(cur), Bs(cur), wm0, wn0, acc);
        if (do_bias && tid < BM) {
#pragma unroll 8
            for (int k = 0; k < BK; ++k) bsum += As(cur)[k * LDA + tid];
        }
        if (kt + 1 < nkt) store_tile(cur ^ 1);
        __syncthreads();
    }

    tn_store(p, acc, split, o0, j0, wm0, wn0);
    if (do_bias && tid < BM && !(p.ablate & 1)) p.bslab[(size_t)split * p.nout + o0 + tid] = bsum;
}

// sum split-K slabs into the reference-layout gradient.  A block owns 64 consecutive
// slab columns of one output row: 16 lane groups (4 per wave) of 16 lanes x float4 each
// sum the splits of one residue class mod 16 (8 float4 loads in flight per lane, 256 B
// contiguous per group), then the 16 partials are combined through LDS in group order
// (deterministic).  ~4 blocks per CU at the production shapes: enough loads in flight to
// stream the 64 MB of a 256-split slab while the GEMMs run beside it.  Bias partials
// (bslab) ride along in the last row of blocks.
constexpr int SR_COLS = 64;
constexpr int SR_GROUPS = 16;
struct SlabJob {
    const float* slab;
    int splits, nout, ldslab, nout_ref, kin_ref;
    const float* bslab;
    float* gw;
    float* gb;
    int accumulate;
};
// the slab reduce's loads are non-temporal (the slabs are read once; cfg2 step 2.020 vs 2.030
// ms, per round -0.5 / -1.9 / -14 us, profiles/r05/reduce_nt_ab.txt)
// one block of the reduce: block `blk` of job j (weight blocks, then bias blocks)
__device__ __forceinline__ void slab_reduce_block(const SlabJob& j, int blk, float4 (&part)[SR_GROUPS][16]) {
    const int l16 = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const int cblocks = (j.kin_ref + SR_COLS - 1) / SR_COLS;
    const int wblocks = j.nout_ref * cblocks;          // then ceil(nout_ref / SR_COLS) bias blocks
    const bool bias_row = blk >= wblocks;
    const int o = bias_row ? j.nout_ref : blk / cblocks;
    const int c0 = (bias_row ? blk - wblocks : blk % cblocks) * SR_COLS + 4 * l16;
    if (bias_row && (j.bslab == nullptr || j.gb == nullptr)) return;   // block-uniform
    const float* src;
    size_t st;
    int ncol;
    if (!bias_row) { src = j.slab + (size_t)o * j.ldslab; st = (size_t)j.nout * j.ldslab; ncol = j.kin_ref; }
    else { src = j.bslab; st = j.nout; ncol = j.nout_ref; }
    const int splits = j.splits;
    const bool vec = (c0 + 4 <= ncol) && ((st & 3) == 0) && ((((uintptr_t)(src + c0)) & 15) == 0);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c0 < ncol) {
        if (vec) {
            int q = grp;
            for (; q + 7 * SR_GROUPS < splits; q += 8 * SR_GROUPS) {      // 8 loads in flight per lane
                float4 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const float* a = src + (size_t)(q + SR_GROUPS * u) * st + c0;
                    {
                        typedef float sr_f4 __attribute__((ext_vector_type(4)));
                        const sr_f4 t = __builtin_nontemporal_load(reinterpret_cast<const sr_f4*>(a));
                        v[u] = make_float4(t.x, t.y, t.z, t.w);
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
                }
            }
            // (the grouped weight gradients' 64-split slabs leave 4 splits per lane group: in flight
            // together, not one dependent load at a time; the same summation order)
            for (; q + 3 * SR_GROUPS < splits; q += 4 * SR_GROUPS) {
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    typedef float sr_f4 __attribute__((ext_vector_type(4)));
                    const sr_f4 t = __builtin_nontemporal_load(
                        reinterpret_cast<const sr_f4*>(src + (size_t)(q + SR_GROUPS * u) * st + c0));
                    v[u] = make_float4(t.x, t.y, t.z, t.w);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
                }
            }
            for (; q < splits; q += SR_GROUPS) {
                const float4 v = *reinterpret_cast<const float4*>(src + (size_t)q * st + c0);
                acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
            }
        } else {
            float a[4] = {0.f, 0.f, 0.f, 0.f};
            for (int q = grp; q < splits; q += SR_GROUPS)
                for (int t = 0; t < 4; ++t)
                    if (c0 + t < ncol) a[t] += src[(size_t)q * st + c0 + t];
            acc = make_float4(a[0], a[1], a[2], a[3]);
        }
    }
    part[grp][l16] = acc;
    __syncthreads();
    if (grp != 0 || c0 >= ncol) return;
    float4 r = part[0][l16];
#pragma unroll
    for (int w = 1; w < SR_GROUPS; ++w) {
        const float4 v = part[w][l16];
        r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    }
    float* dst = bias_row ? j.gb + c0 : j.gw + (size_t)o * j.kin_ref + c0;
    const float rv[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int t = 0; t < 4; ++t)
        if (c0 + t < ncol) dst[t] = j.accumulate ? dst[t] + rv[t] : rv[t];
}

__global__ __launch_bounds__(256) void k_slab_reduce(SlabJob j) {
    __shared__ float4 part[SR_GROUPS][16];
    slab_reduce_block(j, blockIdx.x, part);
}

// several layers' reduces in one launch (the field backward's weight gradients, one launch per
// group of layers instead of one per layer): job k owns blocks first[k] .. first[k + 1]; each
// block runs k_slab_reduce's arithmetic, so the gradients are the same bits
struct SlabJobs {
    SlabJob j[kSlabJobsMax];
    int first[kSlabJobsMax + 1];
    int n;
};
__global__ __launch_bounds__(256) void k_slab_reduce_jobs(SlabJobs js) {
    __shared__ float4 part[SR_GROUPS][16];
    const int b = blockIdx.x;
    int k = 0;
    while (k + 1 < js.n && b >= js.first[k + 1]) ++k;
    slab_reduce_block(js.j[k], b - js.first[k], part);
}

}  // namespace nerf

using namespace nerf;

static int g_ablate = 0;   // nerf_gemm_debug_ablate
static unsigned long long* g_stamps = nullptr;   // nerf_gemm_debug_stamps

template <int BM, int BN, int WM, int WN, int EPI>
static int launch_nt(const NTArgs& a, hipStream_t s, double flops) {
    dim3 grid(a.m / BM, a.n / BN);
    NTArgs b = a;
    b.ablate = g_ablate;
    prof_begin(s);
    hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, EPI>), grid, dim3(64 * WM * WN), 0, s, b);
    prof_end(s, flops, 1);
    return check_launch("k_gemm_nt");
}

// tile policy (nerf_gemm_set_policy): NT 0 = default, 1 = 128x128/4 waves, 2 = 128x256/8 waves,
// 3 = 256x256/8 waves (exact-f32 kernels; the split kernels: 128x256 fp16 pair, 256x256 bf16x3)
static int g_nt_policy = 0;
static int g_tn_policy = 0;
// TN policy 7 -- a 256 x 256 weight gradient in the split modes as
// XCD-paired 256 x 128 column tiles of eight waves (128 splits, half the slab bytes), the
// 64-wide inputs' 256 x 64 tile and the colour layer's 128 x 256 tile with eight waves (one
// column tile: each split reads its dy rows once); 87 vs 104 us per 131072 x 256 x 256 layer
// with its slab reduce, 37 vs 44 us per 256 x 64 one (profiles/r02/dw_xcd_group_ab.txt).
// Policy 3 is the round-2 256 x 256 tile at one wave per SIMD (also the fallback when a split
// count is not a multiple of 8).  Policy 8 (the default since round 4): the splits and tiles
// of 7 on the 4-wave kernels of wgrad.hip in precision mode 2, bit-identical slabs.
static const int kTnDefault = 8;

// f32 arithmetic (nerf_gemm_set_precision): 0 = exact-f32 MFMA, 1 = split-bf16 emulation
// (6 products), 2 = row-scaled fp16 pair (3 products; the library default since ABI 9 -- the
// benchmarked path and the one the fused eval kernel needs; f32-accurate: DESIGN.md section 4.1)
static int g_precision = 2;

template <int EPI>
static int dispatch_nt(const NTArgs& a, hipStream_t s, double flops) {
    const int pol = g_nt_policy ? g_nt_policy : 3;
    if (g_precision >= 1 && a.bs != nullptr) {   // the split paths need the weight image
        NTArgs b = a;
        b.ablate = g_ablate;
        b.stamps = g_stamps;
        if (g_precision == 2) {
            NERF_CHECK(a.ar1 != nullptr && (a.a2 == nullptr || a.ar2 != nullptr),
                       "GEMM precision mode 2 needs the row max of every A segment (x_rmax / dy_rmax)");
            return dispatch_nt_x6(b, EPI, pol, s, flops, true);
        }
        return dispatch_nt_x6(b, EPI, pol, s, flops);
    }
    if (pol == 3 && a.m % 256 == 0 && a.n % 256 == 0) return launch_nt<256, 256, 2, 4, EPI>(a, s, flops);
    if (pol >= 2 && a.n % 256 == 0) return launch_nt<128, 256, 2, 4, EPI>(a, s, flops);
    if (a.n % 128 == 0) return launch_nt<128, 128, 2, 2, EPI>(a, s, flops);
    return launch_nt<128, 64, 4, 1, EPI>(a, s, flops);
}

static int check_nt(const NTArgs& a, const char* fn) {
    NERF_CHECK(a.a1 && a.b && a.c, "%s: null operand", fn);
    NERF_CHECK(a.m > 0 && a.m % 128 == 0, "%s: m=%d must be a positive multiple of 128", fn, a.m);
    NERF_CHECK(a.n > 0 && a.n % 64 == 0, "%s: n=%d must be a positive multiple of 64", fn, a.n);
    NERF_CHECK(a.k1 > 0 && a.k1 % 32 == 0 && a.k2 % 32 == 0 && a.k2 >= 0,
               "%s: k1=%d k2=%d must be multiples of 32", fn, a.k1, a.k2);
    NERF_CHECK(a.k2 == 0 || a.a2 != nullptr, "%s: k2>0 needs x2", fn);
    NERF_CHECK(a.lda1 % 4 == 0 && a.lda2 % 4 == 0 && a.ldb % 4 == 0 && a.ldc >= a.n,
               "%s: leading dimensions must be multiples of 4", fn);
    NERF_CHECK(a.lda1 >= a.k1 && (a.k2 == 0 || a.lda2 >= a.k2) && a.ldb >= a.k1 + a.k2,
               "%s: leading dimension smaller than K", fn);
    NERF_CHECK((((uintptr_t)a.a1 | (uintptr_t)a.b | (uintptr_t)(a.a2 ? a.a2 : a.a1)) & 15u) == 0,
               "%s: operands must be 16-byte aligned", fn);
    NERF_CHECK(a.bs == nullptr || ((((uintptr_t)a.bs) & 15u) == 0 && a.bs_rows >= a.n),
               "%s: split weight image must be 16-byte aligned with at least n rows", fn);
    return NERF_OK;
}

static int linear_fwd(const float* x1, int ldx1, int k1, const float* x2, int ldx2, int k2, const float* w,
                      const uint16_t* w_split, int w_split_rows, const float* bias, float* y, int ldy, int m, int n,
                      int relu, uint32_t* mask_out, int ldmo, const float* x1_rmax, const float* x2_rmax,
                      float* y_rmax, float* y_cmax, const float* head_w, int n_heads, const float* head_b,
                      float* raw4, int raw_col, void* stream) {
    NTArgs a{};
    a.head_w = head_w; a.n_heads = n_heads; a.head_b = head_b; a.raw4 = raw4; a.raw_col = raw_col;
    a.a1 = x1; a.lda1 = ldx1; a.k1 = k1;
    a.a2 = x2; a.lda2 = x2 ? ldx2 : 0; a.k2 = x2 ? k2 : 0;
    a.b = w; a.ldb = k1 + a.k2;
    a.bs = w_split; a.bs_rows = w_split_rows;
    a.bias = bias; a.c = y; a.ldc = ldy; a.m = m; a.n = n; a.relu = relu;
    a.mask_out = mask_out; a.ldmo = ldmo;
    a.ar1 = x1_rmax; a.ar2 = x2 ? x2_rmax : nullptr; a.c_rmax = y_rmax;
    a.c_cmax = y_cmax; a.ldcm = n;
    int rc = check_nt(a, __func__);
    if (rc) return rc;
    NERF_CHECK(mask_out == nullptr || ldmo >= n / 32, "%s: ldmo=%d < n/32", __func__, ldmo);
    const double fl = 2.0 * m * n * (double)(k1 + a.k2);
    // algorithmic bytes: x1 (+ x2), W, y, ReLU bits
    prof_next(NERF_PROF_FWD, 4.0 * m * (double)(k1 + a.k2) + 4.0 * n * (double)(k1 + a.k2) + 4.0 * m * (double)n +
                                 (mask_out ? m * (double)n / 8 : 0.0));
    return dispatch_nt<EPI_FWD>(a, as_stream(stream), fl);
}

extern "C" int nerf_linear_fwd(const float* x1, int ldx1, int k1, const float* x2, int ldx2, int k2,
                               const float* w, const uint16_t* w_split, int w_split_rows, const float* bias,
                               float* y, int ldy, int m, int n, int relu, uint32_t* mask_out, int ldmo,
                               const float* x1_rmax, const float* x2_rmax, float* y_rmax, float* y_cmax,
                               void* stream) {
    return linear_fwd(x1, ldx1, k1, x2, ldx2, k2, w, w_split, w_split_rows, bias, y, ldy, m, n, relu, mask_out, ldmo,
                      x1_rmax, x2_rmax, y_rmax, y_cmax, nullptr, 0, nullptr, nullptr, 0, stream);
}

extern "C" int nerf_linear_fwd_heads(const float* x1, int ldx1, int k1, const float* x2, int ldx2, int k2,
                                     const float* w, const uint16_t* w_split, int w_split_rows, const float* bias,
                                     float* y, int ldy, int m, int n, int relu, uint32_t* mask_out, int ldmo,
                                     const float* x1_rmax, const float* x2_rmax, float* y_rmax, float* y_cmax,
                                     const float* head_w, int n_heads, const float* head_b, float* raw4,
                                     int raw_col, void* stream) {
    NERF_CHECK_PTR(head_w); NERF_CHECK_PTR(head_b); NERF_CHECK_PTR(raw4);
    NERF_CHECK(n_heads >= 1 && n_heads <= 3 && raw_col >= 0 && raw_col + n_heads <= 4,
               "%s: n_heads=%d raw_col=%d (raw4 rows have 4 columns)", __func__, n_heads, raw_col);
    NERF_CHECK(g_precision == 2 && w_split != nullptr && (n == 256 || n == 128),
               "%s: fused heads need GEMM precision mode 2, the weight image and one column block (n = 128 or 256)",
               __func__);
    NERF_CHECK((((uintptr_t)head_w) & 15u) == 0, "%s: head_w must be 16-byte aligned", __func__);
    return linear_fwd(x1, ldx1, k1, x2, ldx2, k2, w, w_split, w_split_rows, bias, y, ldy, m, n, relu, mask_out, ldmo,
                      x1_rmax, x2_rmax, y_rmax, y_cmax, head_w, n_heads, head_b, raw4, raw_col, stream);
}

extern "C" int nerf_linear_bwd_data(const float* dy, int lddy, int k, const float* wt,
                                    const uint16_t* wt_split, int wt_split_rows, const float* u, int ldu,
                                    const float* v, const uint32_t* mask, int ldmask, float* dx, int lddx,
                                    int m, int n, const float* dy_rmax, float* dx_rmax, float* dx_cmax,
                                    void* stream) {
    NTArgs a{};
    a.a1 = dy; a.lda1 = lddy; a.k1 = k;
    a.a2 = nullptr; a.lda2 = 0; a.k2 = 0;
    a.b = wt; a.ldb = k;
    a.bs = wt_split; a.bs_rows = wt_split_rows;
    a.u = u; a.ldu = ldu; a.v = v; a.mask = mask; a.ldmask = ldmask;
    a.ar1 = dy_rmax; a.c_rmax = dx_rmax;
    a.c_cmax = dx_cmax; a.ldcm = n;
    a.c = dx; a.ldc = lddx; a.m = m; a.n = n;
    int rc = check_nt(a, __func__);
    if (rc) return rc;
    NERF_CHECK(u == nullptr || v != nullptr, "%s: u without v", __func__);
    NERF_CHECK(mask == nullptr || ldmask >= n / 32, "%s: ldmask=%d < n/32 words", __func__, ldmask);
    const double fl = 2.0 * m * n * (double)k;
    // algorithmic bytes: dy, W^T, dx, the input layer's ReLU bits, the rank-1 term's u / v
    prof_next(NERF_PROF_DX, 4.0 * m * (double)k + 4.0 * n * (double)k + 4.0 * m * (double)n +
                                (mask ? m * (double)n / 8 : 0.0) + (u ? 4.0 * m + 4.0 * n : 0.0));
    return dispatch_nt<EPI_BWD>(a, as_stream(stream), fl);
}

// argument checks + the kernel arguments of one weight-gradient segment
static int tn_args(const char* fn, const float* dy, int lddy, int nout, const float* x, int ldx, int kin, int m,
                   int splits, float* slab, int ldslab, int col0, float* bslab, const float* dy_cmax,
                   const float* x_cmax, TNArgs& a) {
    NERF_CHECK(dy && x && slab, "%s: null operand", fn);
    NERF_CHECK(nout > 0 && nout % 64 == 0, "%s: nout=%d must be a multiple of 64", fn, nout);
    NERF_CHECK(kin > 0 && kin % 64 == 0, "%s: kin=%d must be a multiple of 64", fn, kin);
    NERF_CHECK(splits > 0 && m % splits == 0 && (m / splits) % BK == 0,
               "%s: m=%d not divisible into %d splits of a multiple of %d rows", fn, m, splits, BK);
    NERF_CHECK(lddy % 4 == 0 && ldx % 4 == 0 && ldslab >= col0 + kin, "%s: bad leading dims", fn);
    NERF_CHECK((((uintptr_t)dy | (uintptr_t)x) & 15u) == 0, "%s: dy / x must be 16-byte aligned", fn);
    // the split kernels address a split's rows through 32-bit buffer descriptors (byte offsets)
    NERF_CHECK((int64_t)(m / splits) * (lddy > ldx ? lddy : ldx) * 4 < ((int64_t)1 << 31),
               "%s: %d rows per split x leading dimension %d exceed the 2 GB buffer range; use more splits",
               fn, m / splits, lddy > ldx ? lddy : ldx);
    a = TNArgs{};
    a.dy = dy; a.lddy = lddy; a.x = x; a.ldx = ldx;
    a.rows_per_split = m / splits;
    a.slab = slab; a.ldslab = ldslab; a.col0 = col0; a.slab_stride = (size_t)nout * ldslab;
    a.bslab = bslab; a.nout = nout;
    a.ablate = g_ablate >> 4;
    a.cm_dy = dy_cmax; a.ldcm_dy = nout; a.cm_x = x_cmax; a.ldcm_x = kin;
    a.stamps = g_stamps;
    return NERF_OK;
}

extern "C" int nerf_linear_bwd_weight(const float* dy, int lddy, int nout, const float* x, int ldx,
                                      int kin, int m, int splits, float* slab, int ldslab, int col0,
                                      float* bslab, const float* dy_cmax, const float* x_cmax, void* stream) {
    TNArgs a;
    int rc = tn_args(__func__, dy, lddy, nout, x, ldx, kin, m, splits, slab, ldslab, col0, bslab, dy_cmax, x_cmax, a);
    if (rc) return rc;
    // mode 2 runs the fp16 pair kernel when the column maxima are there and every split is
    // whole 128-row groups; otherwise the bf16x3 kernel (it needs no scales)
    const bool h16 = g_precision == 2 && dy_cmax && x_cmax && (m / splits) % 128 == 0;
    hipStream_t s = as_stream(stream);
    const double fl = 2.0 * m * nout * (double)kin;
    // algorithmic bytes: the dy and x panels and one nout x kin gradient (+ bias); the
    // split-K slabs are structural traffic of this design, not algorithmic
    prof_next(nout % 256 == 0 && kin % 256 == 0 ? NERF_PROF_DW : NERF_PROF_DW_NARROW,
              4.0 * m * (double)(nout + kin) + 4.0 * nout * (double)kin + (bslab ? 4.0 * nout : 0.0));
    const int pol = g_tn_policy ? g_tn_policy : kTnDefault;
    if (g_precision >= 1) return dispatch_tn_x6(a, nout, kin, splits, pol, s, fl, h16);
    prof_begin(s);
    if (pol >= 3 && nout % 256 == 0 && kin % 256 == 0) {
        dim3 grid(nout / 256, kin / 256, splits);
        hipLaunchKernelGGL((k_gemm_tn<256, 256, 2, 4>), grid, dim3(512), 0, s, a);
    } else if (nout % 128 == 0 && kin % 128 == 0) {
        dim3 grid(nout / 128, kin / 128, splits);
        hipLaunchKernelGGL((k_gemm_tn<128, 128, 2, 2>), grid, dim3(256), 0, s, a);
    } else if (nout % 128 == 0) {
        dim3 grid(nout / 128, kin / 64, splits);
        hipLaunchKernelGGL((k_gemm_tn<128, 64, 4, 1>), grid, dim3(256), 0, s, a);
    } else if (kin % 128 == 0) {
        dim3 grid(nout / 64, kin / 128, splits);
        hipLaunchKernelGGL((k_gemm_tn<64, 128, 2, 2>), grid, dim3(256), 0, s, a);
    } else {
        dim3 grid(nout / 64, kin / 64, splits);
        hipLaunchKernelGGL((k_gemm_tn<64, 64, 2, 2>), grid, dim3(256), 0, s, a);
    }
    prof_end(s, fl, 1);
    return check_launch(__func__);
}

// several 256 x 256 weight gradients of one split count (the field backward's consecutive
// 256-wide layers) in one launch of k_wgrad_pairs when the fp16-pair 4-wave kernels cover them;
// otherwise one nerf_linear_bwd_weight per layer (the same slabs either way)
extern "C" int nerf_linear_bwd_weight_multi(const nerf_wgrad_job* j, int n, int m, int splits, void* stream) {
    NERF_CHECK_PTR(j);
    hipStream_t s = as_stream(stream);
    NERF_CHECK(n >= 1 && n <= kWgradPairsMax, "%s: %d layers (1..%d)", __func__, n, kWgradPairsMax);
    const int pol = g_tn_policy ? g_tn_policy : kTnDefault;
    bool fused = n > 1 && g_precision == 2 && pol == 8 && splits > 0 && m % splits == 0 && (m / splits) % 128 == 0 &&
                 wgrad_supported(256, 256, splits, m / splits);
    TNPairs tp{};
    for (int i = 0; i < n && fused; ++i) {
        fused = j[i].dy_cmax && j[i].x_cmax;
        int rc = tn_args(__func__, j[i].dy, j[i].lddy, 256, j[i].x, j[i].ldx, 256, m, splits, j[i].slab, j[i].ldslab, 0,
                         j[i].bslab, j[i].dy_cmax, j[i].x_cmax, tp.a[i]);
        if (rc) return rc;
    }
    if (!fused) {
        for (int i = 0; i < n; ++i) {
            int rc = nerf_linear_bwd_weight(j[i].dy, j[i].lddy, 256, j[i].x, j[i].ldx, 256, m, splits, j[i].slab,
                                            j[i].ldslab, 0, j[i].bslab, j[i].dy_cmax, j[i].x_cmax, s);
            if (rc) return rc;
        }
        return NERF_OK;
    }
    tp.n = n;
    prof_next(NERF_PROF_DW, n * (4.0 * m * 512.0 + 4.0 * 256 * 256 + 4.0 * 256));
    prof_begin(s);
    launch_wgrad_pairs(tp, splits, s);
    prof_end(s, n * 2.0 * m * 256.0 * 256.0, 3);
    return check_launch("k_wgrad_pairs");
}

// weight gradients of several shapes in one launch (k_wgrad_jobs): each job's shape and split
// count against the launch's S (2 S blocks) pick its tile kind; anything else runs per job
extern "C" int nerf_linear_bwd_weight_job_groups(const nerf_wgrad_tile_job* j, const int* group, int n, int m,
                                                 int splits, int n_groups, void* stream) {
    NERF_CHECK_PTR(j);
    hipStream_t s = as_stream(stream);
    NERF_CHECK(n >= 1 && n <= kWgradJobsMax, "%s: %d jobs (1..%d)", __func__, n, kWgradJobsMax);
    NERF_CHECK(n_groups >= 1 && n_groups <= 4, "%s: n_groups %d (1..4)", __func__, n_groups);
    for (int i = 0; i < n; ++i)
        NERF_CHECK(group == nullptr ? n_groups == 1 : (group[i] >= 0 && group[i] < n_groups),
                   "%s: job %d: group %d of %d", __func__, i, group ? group[i] : 0, n_groups);
    const int pol = g_tn_policy ? g_tn_policy : kTnDefault;
    bool fused = g_precision == 2 && pol == 8 && splits > 0 && splits % 8 == 0;
    TNJobs tj{};
    tj.ngroups = n_groups;
    double bytes = 0.0, flops = 0.0;
    for (int i = 0; i < n && fused; ++i) {
        const nerf_wgrad_tile_job& q = j[i];
        const bool twice = q.splits == 2 * splits, once = q.splits == splits;
        int kind = -1;
        if (q.nout == 256 && q.kin == 256 && once) kind = WJ_PAIR;
        else if (q.nout == 128 && q.kin == 256 && twice) kind = WJ_WIDE;
        else if (q.nout == 256 && q.kin == 64 && twice) kind = WJ_ENC;
        else if (q.nout == 256 && q.kin == 64 && once) kind = WJ_ENC_HALF;
        else if (q.nout == 128 && q.kin == 64 && twice) kind = WJ_ENC128;
        fused = kind >= 0 && q.dy_cmax && q.x_cmax && m % q.splits == 0 && (m / q.splits) % 128 == 0 &&
                wgrad_supported(q.nout, q.kin, q.splits, m / q.splits);
        if (!fused) break;
        int rc = tn_args(__func__, q.dy, q.lddy, q.nout, q.x, q.ldx, q.kin, m, q.splits, q.slab, q.ldslab, q.col0,
                         q.bslab, q.dy_cmax, q.x_cmax, tj.a[i]);
        if (rc) return rc;
        tj.kind[i] = kind;
        tj.grp[i] = group ? group[i] : 0;
        // dy counted once per layer: a second segment over the same dy (col0 > 0) adds its x only
        bytes += 4.0 * m * (q.kin + (q.col0 == 0 ? q.nout : 0)) + 4.0 * q.nout * q.kin + (q.bslab ? 4.0 * q.nout : 0.0);
        flops += 2.0 * m * q.nout * q.kin;
    }
    if (!fused) {
        for (int i = 0; i < n; ++i) {
            const nerf_wgrad_tile_job& q = j[i];
            int rc = nerf_linear_bwd_weight(q.dy, q.lddy, q.nout, q.x, q.ldx, q.kin, m, q.splits, q.slab, q.ldslab,
                                            q.col0, q.bslab, q.dy_cmax, q.x_cmax, s);
            if (rc) return rc;
        }
        return NERF_OK;
    }
    tj.n = n;
    prof_next(NERF_PROF_DW, bytes);
    prof_begin(s);
    launch_wgrad_jobs(tj, splits, s);
    prof_end(s, flops, 3);
    return check_launch("k_wgrad_jobs");
}

extern "C" int nerf_linear_bwd_weight_jobs(const nerf_wgrad_tile_job* j, int n, int m, int splits, void* stream) {
    return nerf_linear_bwd_weight_job_groups(j, nullptr, n, m, splits, 1, stream);
}

namespace nerf {
int wgrad_narrow_pair(const float* dy_a, int lddy_a, const float* x_a, int ldx_a, int splits_a, float* slab_a,
                      int ldslab_a, int col0_a, float* bslab_a, const float* dcm_a, const float* xcm_a,
                      const float* dy_b, int lddy_b, const float* x_b, int ldx_b, int splits_b, float* slab_b,
                      int ldslab_b, int col0_b, float* bslab_b, const float* dcm_b, const float* xcm_b, int m,
                      hipStream_t s) {
    const int pol = g_tn_policy ? g_tn_policy : kTnDefault;
    const bool fused = g_precision == 2 && pol == 8 && dcm_a && xcm_a && dcm_b && xcm_b && m % splits_a == 0 &&
                       m % splits_b == 0 && (m / splits_a) % 128 == 0 && (m / splits_b) % 128 == 0 &&
                       wgrad_supported(256, 64, splits_a, m / splits_a) && wgrad_supported(256, 64, splits_b, m / splits_b);
    if (!fused) {
        int rc = nerf_linear_bwd_weight(dy_a, lddy_a, 256, x_a, ldx_a, 64, m, splits_a, slab_a, ldslab_a, col0_a, bslab_a,
                                        dcm_a, xcm_a, s);
        if (rc) return rc;
        return nerf_linear_bwd_weight(dy_b, lddy_b, 256, x_b, ldx_b, 64, m, splits_b, slab_b, ldslab_b, col0_b, bslab_b,
                                      dcm_b, xcm_b, s);
    }
    TNArgs a, b;
    int rc = tn_args(__func__, dy_a, lddy_a, 256, x_a, ldx_a, 64, m, splits_a, slab_a, ldslab_a, col0_a, bslab_a, dcm_a,
                     xcm_a, a);
    if (rc) return rc;
    rc = tn_args(__func__, dy_b, lddy_b, 256, x_b, ldx_b, 64, m, splits_b, slab_b, ldslab_b, col0_b, bslab_b, dcm_b, xcm_b,
                 b);
    if (rc) return rc;
    prof_next(NERF_PROF_DW_NARROW, 2 * (4.0 * m * 320.0 + 4.0 * 256 * 64) + (bslab_a ? 1024.0 : 0.0) + (bslab_b ? 1024.0 : 0.0));
    prof_begin(s);
    launch_wgrad_two(a, splits_a, b, splits_b, s);
    prof_end(s, 2 * 2.0 * m * 256.0 * 64.0, 3);
    return check_launch("k_wgrad_two");
}
}  // namespace nerf

extern "C" int nerf_linear_bwd_weight_seg(const float* dy, int lddy, int nout, const float* x1, int ldx1, int k1,
                                          const float* x2, int ldx2, int k2, int m, int splits, float* slab,
                                          int ldslab, float* bslab, const float* dy_cmax, const float* x1_cmax,
                                          const float* x2_cmax, void* stream) {
    TNArgs pm, ps;
    int rc = tn_args(__func__, dy, lddy, nout, x1, ldx1, k1, m, splits, slab, ldslab, 0, bslab, dy_cmax, x1_cmax, pm);
    if (rc) return rc;
    rc = tn_args(__func__, dy, lddy, nout, x2, ldx2, k2, m, splits, slab, ldslab, k1, nullptr, dy_cmax, x2_cmax, ps);
    if (rc) return rc;
    const int pol = g_tn_policy ? g_tn_policy : kTnDefault;
    const bool one = g_precision == 2 && pol >= 7 && dy_cmax && x1_cmax && x2_cmax && (m / splits) % 128 == 0 &&
                     tn_seg_supported(nout, k1, k2, splits);
    if (!one) {   // the same slab from two launches
        rc = nerf_linear_bwd_weight(dy, lddy, nout, x1, ldx1, k1, m, splits, slab, ldslab, 0, bslab, dy_cmax, x1_cmax,
                                    stream);
        if (rc) return rc;
        return nerf_linear_bwd_weight(dy, lddy, nout, x2, ldx2, k2, m, splits, slab, ldslab, k1, nullptr, dy_cmax,
                                      x2_cmax, stream);
    }
    const double fl = 2.0 * m * nout * (double)(k1 + k2);
    prof_next(nout % 256 == 0 ? NERF_PROF_DW : NERF_PROF_DW_NARROW,
              4.0 * m * (double)(nout + k1 + k2) + 4.0 * nout * (double)(k1 + k2) + (bslab ? 4.0 * nout : 0.0));
    return dispatch_tn_x6_seg(pm, ps, nout, splits, pol, as_stream(stream), fl);
}

static int slab_job_check(const char* fn, const SlabJob& j) {
    NERF_CHECK(j.slab && j.gw, "%s: null slab / gradient", fn);
    NERF_CHECK(j.splits > 0 && j.nout > 0 && j.kin_ref > 0 && j.ldslab >= j.kin_ref && j.nout_ref <= j.nout &&
                   j.nout_ref > 0,
               "%s: bad sizes", fn);
    return NERF_OK;
}
// one block per (output row, 64 columns), then the bias row's blocks
static int slab_job_blocks(const SlabJob& j) {
    const int cblocks = (j.kin_ref + SR_COLS - 1) / SR_COLS;
    const int bias_blocks = (j.bslab && j.gb) ? (j.nout_ref + SR_COLS - 1) / SR_COLS : 0;
    return j.nout_ref * cblocks + bias_blocks;
}

extern "C" int nerf_slab_reduce(const float* slab, int splits, int nout, int ldslab, int nout_ref,
                                int kin_ref, const float* bslab, float* gw, float* gb, int accumulate,
                                void* stream) {
    const SlabJob j{slab, splits, nout, ldslab, nout_ref, kin_ref, bslab, gw, gb, accumulate};
    int rc = slab_job_check(__func__, j);
    if (rc) return rc;
    hipLaunchKernelGGL(k_slab_reduce, dim3(slab_job_blocks(j)), dim3(256), 0, as_stream(stream), j);
    return check_launch(__func__);
}

namespace nerf {
int slab_reduce_jobs(const SlabJobDesc* d, int n, hipStream_t s) {
    NERF_CHECK(n >= 1 && n <= kSlabJobsMax, "%s: %d jobs (1..%d)", __func__, n, kSlabJobsMax);
    SlabJobs js{};
    js.n = n;
    js.first[0] = 0;
    for (int k = 0; k < n; ++k) {
        js.j[k] = SlabJob{d[k].slab, d[k].splits, d[k].nout, d[k].ldslab, d[k].nout_ref, d[k].kin_ref,
                          d[k].bslab, d[k].gw, d[k].gb, 0};
        int rc = slab_job_check(__func__, js.j[k]);
        if (rc) return rc;
        js.first[k + 1] = js.first[k] + slab_job_blocks(js.j[k]);
    }
    hipLaunchKernelGGL(k_slab_reduce_jobs, dim3(js.first[n]), dim3(256), 0, s, js);
    return check_launch(__func__);
}
}  // namespace nerf

extern "C" int nerf_gemm_set_policy(int nt_policy, int tn_policy) {
    NERF_CHECK(nt_policy >= 0 && nt_policy <= 3 && (tn_policy == 0 || tn_policy == 3 || tn_policy == 7 || tn_policy == 8),
               "%s: policies are 0..3 (NT) and 0, 3, 7, 8 (TN)", __func__);
    g_nt_policy = nt_policy;
    g_tn_policy = tn_policy;
    return NERF_OK;
}

// split-K factor for nerf_linear_bwd_weight under the current tile policy: about one
// resident wave of blocks (256-tiles: 1 block per CU, 128-tiles: 2), each split a whole
// number of 32-row K tiles and at least 256 rows
extern "C" int nerf_linear_bwd_weight_splits(int nout, int kin, int m) {
    const int pol = g_tn_policy ? g_tn_policy : kTnDefault;
    int tiles, target;
    if (pol >= 7 && g_precision >= 1 && nout == 256 && kin == 256) { tiles = 2; target = 256; }   // XCD pairs
    else if (pol >= 7 && g_precision >= 1 && nout == 128 && kin % 256 == 0) { tiles = kin / 256; target = 256; }
    else if (pol >= 3 && nout % 256 == 0 && kin % 256 == 0) { tiles = (nout / 256) * (kin / 256); target = 256; }
    else if (pol >= 3 && nout % 256 == 0 && kin == 64 && g_precision >= 1) { tiles = nout / 256; target = 256; }
    else { tiles = ((nout + 127) / 128) * ((kin + 127) / 128); target = 512; }
    int splits = 1;
    while (splits * 2 * tiles <= target && m % (splits * 2 * BK) == 0 && m / (splits * 2) >= 256) splits *= 2;
    return splits;
}

extern "C" int nerf_gemm_set_precision(int mode) {
    NERF_CHECK(mode >= 0 && mode <= 2, "%s: mode must be 0 (f32 MFMA), 1 (split-bf16) or 2 (fp16 pair)", __func__);
    g_precision = mode;
    return NERF_OK;
}

namespace nerf {
int gemm_precision() { return g_precision; }
}

extern "C" int nerf_gemm_get_precision(void) { return g_precision; }

// diagnostics: per-block phase clocks of the split-bf16 NT kernel into a device buffer
// of grid * 4 * 2 uint64 (NULL switches it off); not for production
extern "C" int nerf_gemm_debug_stamps(void* buf) {
    g_stamps = reinterpret_cast<unsigned long long*>(buf);
    return NERF_OK;
}

// diagnostics: ablate parts of the NT GEMM (results are wrong while set); not for production
extern "C" int nerf_gemm_debug_ablate(int mask) {
    g_ablate = mask;
    return NERF_OK;
}
