// Weight gradients of the field MLP in GEMM precision mode 2 (fp16 pairs):
//   slab[split][o][col0 + j] = sum over the split's rows s of dy[s][o] x[s][j]
// -- the autograd of every nn.Linear in official_nerf.py:60-96 as training.py:92 runs it,
// for the D = 256 field at the training batch (131 072 rows; 128 splits of 1024 rows).
//
// Same arithmetic as gemm_x6.hip's TN kernels, bit for bit: each split's columns scaled by
// the power of two of their maximum over the split (from the producers' per-128-row-group
// column maxima), split into RNE fp16 (hi, lo) pairs, and hi.lo + lo.hi + hi.hi accumulated
// on v_mfma_f32_32x32x16_f16 over 16-row k-steps in row order.  What differs is the work
// split inside a block: 8 waves, two per SIMD, in two roles (MI355X_MICROARCH.md "Two waves
// per SIMD": a matrix wave beside a load wave on each SIMD):
//   * waves 0-3 (MFMA): 2 x 2 wave tiles of 128 x 64 (or 64 x 128) outputs, accumulators in
//     AGPRs, 24 MFMAs per 16-row k-step between LDS fragment reads, 48 per 32-row stage;
//   * waves 4-7 (load + split): each thread owns an 8-row strip of CA + CB columns per
//     stage, loaded straight to registers as dwordx4 / dwordx2 row pieces (one 1 KB / 512 B
//     row of the tile per wave instruction) two stages ahead, split into fp16 pairs and
//     written as one 16-byte fragment chunk per column and plane (gemm_x6.hip's XImg layout);
// one block barrier per 32-row stage, so a SIMD's split VALU runs beside its MFMAs instead
// of between them.
// The 256-output layers run as two XCD-paired 256 x 128 column tiles per split (workgroups
// w and w + 8 share an XCD, so the second read of each dy stage is an L2 hit); the layers with
// a 64-wide second input segment (l4 over [h3 | enc_p], the colour layer over [f | enc_d],
// official_nerf.py:63, 89) put every column tile of a split on one XCD the same way.
#include "gemm.hpp"
#include "x16.hpp"

#include <utility>

namespace nerf {
namespace wg {

constexpr int NTH = 512;   // 8 waves, two per SIMD: 4 MFMA waves + 4 load / split waves
constexpr int KS = 32;     // rows per pipeline stage: two 16-row MFMA k-steps
constexpr int NS = 3;      // register stages of a load wave: loads issued three stages ahead of their split
                           // (k_wgrad_jobs<3>: four)

template <int BO, int BK>
struct Cfg {
    static constexpr int CA = BO / 64, CB = BK / 64;   // columns per thread (dy, x)
    static constexpr int WO = BO / 2, WK = BK / 2;     // wave tile (2 x 2 waves)
    static constexpr int TM = WO / 32, TN = WK / 32;
    // the images of one 16-row k-step: [plane][k-half][column][8 fp16], k-halves 128 B apart
    static constexpr int AH = BO * 16 + 128, BH = BK * 16 + 128;
    static constexpr int AP = 2 * AH, BP = 2 * BH;
    static constexpr int KSTEP = 2 * AP + 2 * BP;
    static constexpr int BUF = 2 * KSTEP;              // one 32-row stage
    static constexpr int LOOP = 2 * BUF;               // double-buffered
    static constexpr int EPI = 4 * TileLds<TN>::BYTES;
    static constexpr int MAIN = LOOP > EPI ? LOOP : EPI;
    // + column exponents (two sets: consecutive layers of one launch alternate), bias partials
    static constexpr int BYTES = MAIN + 2 * (BO + BK) * 4 + 4 * BO * 4;
    static_assert(TM >= 1 && TN >= 1 && CA >= 1 && CB >= 1 && CA <= 4 && CB <= 4, "tile");
};

// f(integral_constant<0>), ..., f(integral_constant<N - 1>), in order
template <class F, int... I>
__device__ __forceinline__ void unroll_seq(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void unroll(F&& f) {
    unroll_seq(f, std::make_integer_sequence<int, N>{});
}

typedef unsigned wg_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned wg_u32x2 __attribute__((ext_vector_type(2)));
// (named components: subscripting the builtin's vector with an unrolled index miscompiles to
// one dword load on this toolchain)
// POL: the buffer instruction's cache-policy bits (2 = nt)
template <int C, int POL = 0>
__device__ __forceinline__ void load_row(float (&v)[C], const __amdgpu_buffer_rsrc_t& r, int voff, int soff) {
    if constexpr (C == 4) {
        const wg_u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, POL);
        v[0] = __uint_as_float(t.x); v[1] = __uint_as_float(t.y);
        v[2] = __uint_as_float(t.z); v[3] = __uint_as_float(t.w);
    } else if constexpr (C == 2) {
        const wg_u32x2 t = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, POL);
        v[0] = __uint_as_float(t.x); v[1] = __uint_as_float(t.y);
    } else {
        v[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, POL));
    }
}
// (the stage loads keep the default cache policy: nt on x made a launch 9 % slower, on dy and x
// 27 %, profiles/r05/nt_loads_ab.txt)

// The operand images hold one 16-byte fragment chunk (8 k values) per column; column col's chunk
// sits at swz(col) (a permutation within aligned groups of 4 columns).  A load wave's column c of
// lane l is CA l + c (CB l + c): unswizzled, the 8 lanes of a ds_write_b128 group land CA x 16 bytes
// apart -- 4-way bank conflicts at CA = 4, more than half the kernel's LDS cycles (SQ_LDS_BANK_CONFLICT,
// profiles/r06/wgrad_sq_r06cc.json); swizzled they cover 8 distinct 4-bank groups, and the MFMA waves'
// reads of 32 consecutive columns stay a permutation of the same chunks (the same banks per lane group)
__device__ __forceinline__ int swz(int col) { return col ^ ((col >> 3) & 3); }

// 8 rows of one column, scaled by 2^e -> one 16-byte fragment chunk per plane
__device__ __forceinline__ void put_strip(char* d, int plane_bytes, const float (&v)[8], int e) {
    uint32_t h[4], l[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) split2h(v[2 * t], v[2 * t + 1], e, h[t], l[t]);
    *reinterpret_cast<uint4*>(d) = make_uint4(h[0], h[1], h[2], h[3]);
    *reinterpret_cast<uint4*>(d + plane_bytes) = make_uint4(l[0], l[1], l[2], l[3]);
}

// one block: output rows o0 .. o0 + BO (dy columns), column tile jt (x columns jt BK ..), split;
// BIAS: the load waves also sum the dy columns (the bias gradient; one column tile per split)
// par: which exponent set (consecutive layers of one launch alternate, so a layer's exponents
// can be written while the previous layer's epilogue still reads its own)
// AUX: the LDS offset of the column exponents and bias partials (a kernel that runs tiles of
// several shapes puts them past the largest main region, so one shape's exponents never land in
// the region another shape's epilogue is still staging its slab through)
// SET: ints per exponent set.  A kernel that runs tiles of several shapes passes one stride for
// all of them (JOBS_SET): the next job's exponents() writes its set while the previous job's
// epilogue may still read the other set's lea / leb, so the two sets must not overlap whatever
// the two jobs' shapes (with a per-shape stride BO + BK, a 128 x 64 job's set 1 overlapped a
// 256 x 128 job's set 0)
template <int BO, int BK, bool BIAS, int AUX = Cfg<BO, BK>::MAIN, int SET = BO + BK, int NS = wg::NS>
__device__ __forceinline__ void block(const TNArgs& p, char* smem, int o0, int jt, int split, int par) {
    using C = Cfg<BO, BK>;
    constexpr int CA = C::CA, CB = C::CB, TM = C::TM, TN = C::TN;
    // an opaque copy: nothing derived from the thread index is hoisted out of a kernel's job loop
    // (k_wgrad_jobs: the shapes' hoisted lane offsets would stay live together and spill)
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j0 = jt * BK;
    const size_t s0 = (size_t)split * p.rows_per_split;
    const int nst = p.rows_per_split / KS;
    static_assert(AUX >= C::MAIN, "aux region");
    static_assert(SET >= BO + BK, "an exponent set holds BO + BK ints");
    int* lea = reinterpret_cast<int*>(smem + AUX) + par * SET;   // the tile's column exponents
    int* leb = lea + BO;
    float* lbias = reinterpret_cast<float*>(smem + AUX) + 2 * SET;   // [4 load waves][BO] bias partials
    // the column exponents: every thread its share (one round trip to the producers' group
    // maxima), in both roles -- the load waves issue their first NS stages before theirs
    auto exponents = [&]() {
        for (int e = tid; e < BO; e += NTH) lea[e] = row_exp(tn_colmax(p.cm_dy, p.ldcm_dy, s0, p.rows_per_split, o0 + e));
        for (int e = tid; e < BK; e += NTH) leb[e] = row_exp(tn_colmax(p.cm_x, p.ldcm_x, s0, p.rows_per_split, j0 + e));
        __syncthreads();
    };

    if (wave >= 4) {
        // ---- load / split waves: rows 8 lw .. 8 lw + 7 of every stage, CA + CB columns ----
        const int lw = wave - 4;
        // the split's rows as buffer resources: the lane's column offset in a VGPR, the row
        // offset (stage, strip, row) wave-uniform in an SGPR
        const __amdgpu_buffer_rsrc_t rdy = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(p.dy + s0 * p.lddy + o0), (short)0, (p.rows_per_split * p.lddy - o0) * 4, 0x00020000);
        const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(p.x + s0 * p.ldx + j0), (short)0, (p.rows_per_split * p.ldx - j0) * 4, 0x00020000);
        const int va_off = 4 * CA * lane, vb_off = 4 * CB * lane;
        float va[NS][8][CA], vb[NS][8][CB];
        auto load = [&](auto uc, int t) {
            constexpr int U = decltype(uc)::value;
            t = t < nst ? t : nst - 1;   // the tail re-loads the last stage: every iteration is alike
            const int r0 = KS * t + 8 * lw;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                load_row<CA>(va[U][i], rdy, va_off, (r0 + i) * p.lddy * 4);
                load_row<CB>(vb[U][i], rx, vb_off, (r0 + i) * p.ldx * 4);
            }
        };
        unroll<NS>([&](auto u) { load(u, decltype(u)::value); });
        exponents();
        int ea[CA], eb[CB];
#pragma unroll
        for (int c = 0; c < CA; ++c) ea[c] = lea[CA * lane + c];
#pragma unroll
        for (int c = 0; c < CB; ++c) eb[c] = leb[CB * lane + c];
        float bsum[CA];
#pragma unroll
        for (int c = 0; c < CA; ++c) bsum[c] = 0.f;
        // stage in register set U -> image buffer `buf` (k-step lw >> 1, k-half lw & 1);
        // `real` false: the tail's clamped re-split, left out of the bias sums
        auto put = [&](auto uc, char* buf, bool real) {
            constexpr int U = decltype(uc)::value;
            char* ks = buf + (lw >> 1) * C::KSTEP;
            // one column at a time (scheduling barriers): hoisting every column's scaling ahead
            // of the conversions runs out of registers and reuses in-flight load destinations
#pragma unroll
            for (int c = 0; c < CA; ++c) {
                __builtin_amdgcn_sched_barrier(0);
                float v[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = va[U][i][c];
                put_strip(ks + (lw & 1) * C::AH + swz(CA * lane + c) * 16, C::AP, v, ea[c]);
                if constexpr (BIAS) {
                    float sm = 0.f;
#pragma unroll
                    for (int i = 0; i < 8; ++i) sm += v[i];
                    bsum[c] += real ? sm : 0.f;
                }
            }
#pragma unroll
            for (int c = 0; c < CB; ++c) {
                __builtin_amdgcn_sched_barrier(0);
                float v[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = vb[U][i][c];
                put_strip(ks + 2 * C::AP + (lw & 1) * C::BH + swz(CB * lane + c) * 16, C::BP, v, eb[c]);
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        // prologue (stages 0 .. NS - 1 in flight): stage 0 split into buffer 0, stage NS's
        // loads into the set it freed
        put(std::integral_constant<int, 0>{}, smem, true);
        load(std::integral_constant<int, 0>{}, NS);
        __syncthreads();
        // iteration s: stage s + 1 (register set (s + 1) % NS, loaded NS iterations ago) into
        // buffer (s + 1) & 1, then the loads of stage s + 1 + NS into the set it freed
        // The bias partials are final after iteration nst - 2 (stage nst - 1); they go to LDS in
        // the last iteration, before its barrier, so the MFMA waves (past that barrier) sum them
        // and no barrier follows the loop: the load waves go straight on to a next layer
        auto iter = [&](int s, auto uc) {
            put(uc, smem + ((s + 1) & 1) * C::BUF, s + 1 < nst);
            load(uc, s + 1 + NS);
            if constexpr (BIAS) {
                if (s == nst - 1) {
#pragma unroll
                    for (int c = 0; c < CA; ++c) lbias[lw * BO + CA * lane + c] = bsum[c];
                }
            }
            __syncthreads();
        };
        // trips of NS straight-line iterations, so that every set index is a constant and the
        // vmcnt waits count the loads issued since (a loop-carried set would wait for all)
        int s = 0;
        for (; s + NS <= nst; s += NS)
            unroll<NS>([&](auto r) {
                constexpr int R = decltype(r)::value;
                iter(s + R, std::integral_constant<int, (R + 1) % NS>{});
            });
        unroll<NS - 1>([&](auto r) {
            constexpr int R = decltype(r)::value;
            if (s + R < nst) iter(s + R, std::integral_constant<int, (R + 1) % NS>{});
        });
    } else {
        // ---- MFMA waves: a 2 x 2 grid of WO x WK wave tiles ----
        exponents();
        const int l32 = lane & 31, hi = lane >> 5;
        const int wm0 = (wave >> 1) * C::WO, wn0 = (wave & 1) * C::WK;
        f32x16 acc[TM][TN];
        zero_acc(acc);
        // the fragments of a stage's two k-steps in two register sets: each set is read one
        // k-step (24 MFMAs) before its MFMAs, so no LDS latency sits between MFMAs; the block
        // barrier sits between the two k-steps (stage s + 1's images are complete there, and
        // stage s's second k-step is already in registers)
        uint4 fa[2][TM][2], fb[2][TN][2];
        auto frag = [&](auto kc, const char* ks) {
            constexpr int K = decltype(kc)::value;
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    fb[K][j][q] = *reinterpret_cast<const uint4*>(ks + 2 * C::AP + q * C::BP + hi * C::BH + swz(wn0 + 32 * j + l32) * 16);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    fa[K][i][q] = *reinterpret_cast<const uint4*>(ks + q * C::AP + hi * C::AH + swz(wm0 + 32 * i + l32) * 16);
        };
        auto mma = [&](auto kc) {
            constexpr int K = decltype(kc)::value;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    f32x16 c = acc[i][j];
                    c = mfma_f16(fa[K][i][0], fb[K][j][1], c);   // hi.lo
                    c = mfma_f16(fa[K][i][1], fb[K][j][0], c);   // lo.hi
                    c = mfma_f16(fa[K][i][0], fb[K][j][0], c);   // hi.hi
                    acc[i][j] = c;
                }
        };
        constexpr std::integral_constant<int, 0> k0{};
        constexpr std::integral_constant<int, 1> k1{};
        __syncthreads();
        frag(k0, smem);
        for (int s = 0; s < nst; ++s) {
            const char* cur = smem + (s & 1) * C::BUF;
            frag(k1, cur + C::KSTEP);
            __builtin_amdgcn_sched_barrier(0);
            mma(k0);
            __syncthreads();
            // (the last iteration reads buffer nst & 1 to no use: straight-line waits)
            frag(k0, smem + ((s + 1) & 1) * C::BUF);
            __builtin_amdgcn_sched_barrier(0);
            mma(k1);
        }
        if constexpr (BIAS) {
            // the load waves' strip sums -> column sums, added in strip order: deterministic
            for (int c = tid; c < BO; c += NTH / 2)
                p.bslab[(size_t)split * p.nout + o0 + c] =
                    ((lbias[c] + lbias[BO + c]) + lbias[2 * BO + c]) + lbias[3 * BO + c];
        }
        tn_store_lds<TM, TN, true>(p, acc, smem, split, o0, j0, wm0, wn0, lea, leb);
    }
}

// the block of column tile jt, with the bias sums where the layer wants them (column tile 0)
template <int BO, int BK, int AUX = Cfg<BO, BK>::MAIN, int SET = BO + BK, int NS = wg::NS>
__device__ __forceinline__ void block_any(const TNArgs& p, char* smem, int o0, int jt, int split, int par = 0) {
    if (jt == 0 && p.bslab != nullptr) block<BO, BK, true, AUX, SET, NS>(p, smem, o0, jt, split, par);
    else block<BO, BK, false, AUX, SET, NS>(p, smem, o0, jt, split, par);
}

// the LDS of a kernel that runs tiles of every shape (k_wgrad_jobs): the main regions, then two
// exponent sets of JOBS_SET ints (the widest shape's BO + BK) and the bias partials
constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int JOBS_AUX = cmax(cmax(Cfg<256, 128>::MAIN, Cfg<128, 256>::MAIN), cmax(Cfg<256, 64>::MAIN, Cfg<128, 64>::MAIN));
constexpr int JOBS_SET = cmax(cmax(256 + 128, 128 + 256), cmax(256 + 64, 128 + 64));
constexpr int JOBS_BYTES = JOBS_AUX + 2 * JOBS_SET * 4 + 4 * 256 * 4;
static_assert(JOBS_SET == 384, "exponent sets");

}  // namespace wg

// a 256 x 256 layer: two XCD-paired 256 x 128 column tiles per split (splits % 8 == 0)
__global__ __launch_bounds__(wg::NTH, 2) void k_wgrad_pair(TNArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[wg::Cfg<256, 128>::BYTES];
    const int w = blockIdx.x, slot = w >> 3;
    wg::block_any<256, 128>(p, smem, 0, slot & 1, (slot >> 1) * 8 + (w & 7));
}

// several consecutive 256 x 256 layers in one launch (l_f .. l5, l3 .. l1 of the field backward):
// a block walks the layers in order, its load waves issuing a layer's first stages while its
// MFMA waves still store the previous layer's slab -- one prologue ramp and one launch per
// group instead of per layer; each layer's slabs are those of its own k_wgrad_pair launch
__global__ __launch_bounds__(wg::NTH, 2) void k_wgrad_pairs(TNPairs m) {
    __shared__ __attribute__((aligned(16))) char smem[wg::Cfg<256, 128>::BYTES];
    const int w = blockIdx.x, slot = w >> 3;
    // LDS across the layer boundary: nothing here orders layer i + 1's first LDS write after
    // layer i's last LDS reads.  It is the __syncthreads() inside layer i + 1's exponents()
    // (block(), before any stage is put into the operand image) that keeps the load waves'
    // stage-0 put out of the region the MFMA waves' tn_store_lds is still using for layer i's
    // slab; a change that writes LDS before that barrier (hoisting the put, or the exponents'
    // reads after the loads) must add a barrier here.  test_wgrad_multi_matches_single
    // (n = 1 .. 4 and 8, tests/test_gpu_kernels.py) checks the slabs against one launch per layer.
    for (int i = 0; i < m.n; ++i)
        wg::block_any<256, 128>(m.a[i], smem, 0, slot & 1, (slot >> 1) * 8 + (w & 7), i & 1);
}

// every weight gradient of a backward group in one launch (TN schedule 3, field_bwd.cpp): a job
// list walked in order by 2 S blocks (S = the 256 x 256 layers' split count, a multiple of 8),
// block w on XCD w % 8 with column tile jt = (w >> 3) & 1 of split sp = (w >> 4) * 8 + w % 8:
//   WJ_PAIR      256 x 256 over S splits: column tile jt of split sp (k_wgrad_pair's tiles);
//   WJ_WIDE      128 x 256 over 2 S splits (the colour layer over f): the whole tile of split 2 sp + jt;
//   WJ_ENC       256 x 64 over 2 S splits (l0 over enc_p): split 2 sp + jt;
//   WJ_ENC_HALF  256 x 64 over S splits (l4 over enc_p): output rows 128 jt .. + 127 of split sp
//                (the XCD pair shares the split's enc_p rows through L2);
//   WJ_ENC128    128 x 64 over 2 S splits (the colour layer over enc_d): split 2 sp + jt.
// The jobs run grouped by shape (see the kernel for the order), each group in list order.  The splits and slab columns are those of the per-layer launches, so are the slabs, bit
// for bit.
// Each job's exponents alternate between the two sets of one aux region past every shape's main
// region (JOBS_AUX), at one stride for every shape (JOBS_SET), so a job's exponents never land
// on the set the previous job's epilogue still reads, and the barrier in a job's exponents()
// orders the rest of it after that epilogue as in k_wgrad_pairs.
// SH: the shapes compiled in (bit 0 128 x 256, bit 1 128 x 64, bit 2 256 x 64; 256 x 256 always):
// with all four in one kernel the register allocation spills, with any three it does not.
// Block groups (m.ngroups > 1): the grid is ngroups consecutive ranges of 2 S blocks, range g
// running the jobs with grp == g -- two job lists side by side on half the chip each, at half
// the split count of one list on the whole chip: the same work per launch, half the split-K
// slab bytes (written here, read back by the slab reduce).  2 S is a multiple of 8, so a block's
// XCD pairing within its range is the single-group one.
template <int SH>
__global__ __launch_bounds__(wg::NTH, 2) void k_wgrad_jobs(TNJobs m) {
    __shared__ __attribute__((aligned(16))) char smem[wg::JOBS_BYTES];
    constexpr int A = wg::JOBS_AUX;
    // the load waves' stages in flight: 4 in the colour .. l5 launch (shape set 3; 1.8653 vs 1.8702
    // ms per cfg2 step, profiles/r06/wgrad_ns4_ab.txt), 3 elsewhere (shape set 6 spills at 4)
    constexpr int NSJ = SH == 3 ? 4 : wg::NS;
    const int per = gridDim.x / m.ngroups;
    const int gsel = blockIdx.x / per;
    const int w = blockIdx.x - gsel * per, q = w >> 3;
    const int jt = q & 1, sp = (q >> 1) * 8 + (w & 7);
    // one loop per tile shape, each group in list order; the exponent set alternates per job run
    // (c).  The order keeps a layer's second segment right behind its first (the same dy rows;
    // measured: 20 of l4's 134 MB dy re-read come from the MALL, gpurun_out/r05q): with a 128 x 256
    // job (the colour layer)
    // 128 x 256, 128 x 64, 256 x 256; otherwise 256 x 256 (l4's h3 job last in the list), 128 x 64
    // (l4's enc_p), 256 x 64
    int c = 0;
    auto pairs = [&]() {
        for (int i = 0; i < m.n; ++i)
            if (m.kind[i] == WJ_PAIR && m.grp[i] == gsel)
                wg::block_any<256, 128, A, wg::JOBS_SET, NSJ>(m.a[i], smem, 0, jt, sp, c++ & 1);
    };
    auto narrow = [&]() {
        for (int i = 0; i < m.n; ++i) {
            const int k = m.kind[i];
            if ((k == WJ_ENC128 || k == WJ_ENC_HALF) && m.grp[i] == gsel)
                wg::block_any<128, 64, A, wg::JOBS_SET, NSJ>(m.a[i], smem, k == WJ_ENC_HALF ? 128 * jt : 0, 0,
                                          k == WJ_ENC_HALF ? sp : 2 * sp + jt, c++ & 1);
        }
    };
    if constexpr (SH & 1) {
        for (int i = 0; i < m.n; ++i)
            if (m.kind[i] == WJ_WIDE && m.grp[i] == gsel)
                wg::block_any<128, 256, A, wg::JOBS_SET, NSJ>(m.a[i], smem, 0, 0, 2 * sp + jt, c++ & 1);
        if constexpr (SH & 2) narrow();
        pairs();
    } else if (m.ngroups > 1) {
        // block groups: a group's narrow jobs first, so l4's enc_p job (group 1) reads l4's dy
        // beside its h3 job (group 0's first) instead of after it
        if constexpr (SH & 2) narrow();
        pairs();
    } else {
        pairs();
        if constexpr (SH & 2) narrow();
    }
    if constexpr (SH & 4)
        for (int i = 0; i < m.n; ++i)
            if (m.kind[i] == WJ_ENC && m.grp[i] == gsel)
                wg::block_any<256, 64, A, wg::JOBS_SET, NSJ>(m.a[i], smem, 0, 0, 2 * sp + jt, c++ & 1);
}

// two layers' 256 x 64 tiles in one launch: a's splits (blocks 0 .. na - 1), then b's (l4's
// enc_p segment at 1024 rows per split, then l0 at 512: the long blocks are dispatched first,
// the short ones fill in behind them -- one full-chip wave instead of two half-empty launches)
__global__ __launch_bounds__(wg::NTH, 2) void k_wgrad_two(TNArgs a, int na, TNArgs b) {
    __shared__ __attribute__((aligned(16))) char smem[wg::Cfg<256, 64>::BYTES];
    const int w = blockIdx.x;
    if (w < na) wg::block_any<256, 64>(a, smem, 0, 0, w);
    else wg::block_any<256, 64>(b, smem, 0, 0, w - na);
}

// one BO x BK tile per split (l0: 256 outputs over the 64 encoding columns)
template <int BO, int BK>
__global__ __launch_bounds__(wg::NTH, 2) void k_wgrad_one(TNArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[wg::Cfg<BO, BK>::BYTES];
    wg::block_any<BO, BK>(p, smem, 0, 0, blockIdx.x);
}

// two input segments, all tiles of a split on one XCD in consecutive dispatch slots: l4 (256
// outputs: two 256 x 128 tiles over h3 + a 256 x 64 tile over enc_p) and the colour layer (128
// outputs: a 128 x 256 tile over f + a 128 x 64 tile over enc_d)
template <int BO, int BK, int CT, int BK2>
__global__ __launch_bounds__(wg::NTH, 2) void k_wgrad_seg(TNArgs pm, TNArgs ps) {
    constexpr int B1 = wg::Cfg<BO, BK>::BYTES, B2 = wg::Cfg<BO, BK2>::BYTES;
    __shared__ __attribute__((aligned(16))) char smem[B1 > B2 ? B1 : B2];
    const int w = blockIdx.x, slot = w >> 3;
    const int jt = slot % (CT + 1), split = (slot / (CT + 1)) * 8 + (w & 7);
    if (jt < CT) wg::block_any<BO, BK>(pm, smem, 0, jt, split);
    else wg::block_any<BO, BK2>(ps, smem, 0, 0, split);
}

// which shapes the 4-wave kernels cover (the rest stay on gemm_x6.hip's TN kernels)
bool wgrad_supported(int nout, int kin, int splits, int rows_per_split) {
    if (rows_per_split % wg::KS != 0 || rows_per_split < 3 * wg::KS) return false;
    return (nout == 256 && kin == 256 && splits % 8 == 0) || (nout == 256 && kin == 64) ||
           (nout == 128 && (kin == 256 || kin == 64));
}
bool wgrad_seg_supported(int nout, int k1, int k2, int splits, int rows_per_split) {
    return rows_per_split % wg::KS == 0 && rows_per_split >= 3 * wg::KS && k1 == 256 && k2 == 64 &&
           (nout == 256 || nout == 128) && splits % 8 == 0;
}

void launch_wgrad(const TNArgs& a, int nout, int kin, int splits, hipStream_t s) {
    if (nout == 256 && kin == 256)
        hipLaunchKernelGGL(k_wgrad_pair, dim3(2 * splits), dim3(wg::NTH), 0, s, a);
    else if (nout == 256)
        hipLaunchKernelGGL((k_wgrad_one<256, 64>), dim3(splits), dim3(wg::NTH), 0, s, a);
    else if (kin == 256)
        hipLaunchKernelGGL((k_wgrad_one<128, 256>), dim3(splits), dim3(wg::NTH), 0, s, a);
    else
        hipLaunchKernelGGL((k_wgrad_one<128, 64>), dim3(splits), dim3(wg::NTH), 0, s, a);
}

void launch_wgrad_two(const TNArgs& a, int na, const TNArgs& b, int nb, hipStream_t s) {
    hipLaunchKernelGGL(k_wgrad_two, dim3(na + nb), dim3(wg::NTH), 0, s, a, na, b);
}

void launch_wgrad_pairs(const TNPairs& m, int splits, hipStream_t s) {
    hipLaunchKernelGGL(k_wgrad_pairs, dim3(2 * splits), dim3(wg::NTH), 0, s, m);
}

void launch_wgrad_jobs(const TNJobs& m, int splits, hipStream_t s) {
    int sh = 0;
    for (int i = 0; i < m.n; ++i)
        sh |= m.kind[i] == WJ_WIDE ? 1 : m.kind[i] == WJ_ENC128 || m.kind[i] == WJ_ENC_HALF ? 2 : m.kind[i] == WJ_ENC ? 4 : 0;
    const dim3 g(2 * splits * m.ngroups), b(wg::NTH);
    switch (sh) {
    case 0: hipLaunchKernelGGL(k_wgrad_jobs<0>, g, b, 0, s, m); break;
    case 1: hipLaunchKernelGGL(k_wgrad_jobs<1>, g, b, 0, s, m); break;
    case 2: hipLaunchKernelGGL(k_wgrad_jobs<2>, g, b, 0, s, m); break;
    case 3: hipLaunchKernelGGL(k_wgrad_jobs<3>, g, b, 0, s, m); break;
    case 4: hipLaunchKernelGGL(k_wgrad_jobs<4>, g, b, 0, s, m); break;
    case 5: hipLaunchKernelGGL(k_wgrad_jobs<5>, g, b, 0, s, m); break;
    case 6: hipLaunchKernelGGL(k_wgrad_jobs<6>, g, b, 0, s, m); break;
    default: hipLaunchKernelGGL(k_wgrad_jobs<7>, g, b, 0, s, m); break;   // (spills; no schedule uses it)
    }
}

void launch_wgrad_seg(const TNArgs& pm, const TNArgs& ps, int nout, int splits, hipStream_t s) {
    if (nout == 256)
        hipLaunchKernelGGL((k_wgrad_seg<256, 128, 2, 64>), dim3(3 * splits), dim3(wg::NTH), 0, s, pm, ps);
    else
        hipLaunchKernelGGL((k_wgrad_seg<128, 256, 1, 64>), dim3(2 * splits), dim3(wg::NTH), 0, s, pm, ps);
}

}  // namespace nerf
