// f32 GEMMs of the field MLP emulated on the bf16 matrix cores (gfx950).
//
// Same launches, arguments and epilogues as gemm_f32.hip (forward, backward-data,
// backward-weight of OfficialStaticNerf's linears, official_nerf.py:60-96), different
// K loop:
//  * every f32 operand x is split while it is staged into LDS into three bf16 words,
//    x = hi + mid + lo, each the round-to-nearest-even bf16 of what the previous words
//    leave (8 + 8 + 8 significand bits: exact for normal f32 x);
//  * a.b = sum over the six cross products whose magnitude is >= 2^-16 |a||b| (hi.hi,
//    hi.mid, mid.hi, hi.lo, mid.mid, lo.hi), issued smallest first into ONE f32
//    accumulator with v_mfma_f32_32x32x16_bf16; the dropped ones (mid.lo, lo.mid, lo.lo)
//    are <= 2^-26 |a||b| each, below the f32 rounding of the sum.  Per product this is
//    within ~2^-24 of the exact-f32 v_mfma_f32_32x32x2_f32 result, at 6/16 of its cost:
//    1024 FLOP/clk/SIMD bf16 vs 64 FLOP/clk/SIMD f32.
//  * LDS images per operand and buffer: 3 planes (hi/mid/lo) x 2 k-halves of
//    [row][8 bf16]; a lane's MFMA fragment (row r, k = 8h..8h+7) is one ds_read_b128,
//    and the half images are offset by 128 B so a wave's staging ds_write_b64 covers
//    all 64 banks.  K tile = 16 (one MFMA K step), double-buffered: ~99 KB at 256x256.
//  * K-contiguous operands ([m][k], [n][k]) load as float4 along k; sample-major ones
//    (dy[s][o], x[s][j]) load as 8-row column strips so each thread owns 8 consecutive
//    k of one column and writes its fragment chunk with one ds_write_b128 per plane.
//
// Precision mode 2 (H = true, the NT kernels only) replaces the bf16 triple by an fp16
// pair: every operand row is scaled by a power of two 2^e (row max -> [2^14, 2^15),
// exact), split into x 2^e = hi + lo (RNE fp16 each: 11 + 11 significand bits, the
// remainder <= 2^-22 |x|), and a.b = hi.lo + lo.hi + hi.hi on v_mfma_f32_32x32x16_f16
// (the dropped lo.lo <= 2^-22 |a||b|) -- three products instead of six, two LDS planes
// instead of three.  The epilogue undoes the scales (2^-(e_row + e_feature), exact).
// Row scales come from the producers: every kernel that writes an A operand also writes
// its row max (max |x| over the row), read here as NTArgs::ar1 / ar2; the weight image's
// per-row exponents sit in plane 2 of the image (nerf_pack_weights).
#include "gemm.hpp"
#include "x16.hpp"

#include <cstdlib>

namespace nerf {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

constexpr int XK = 16;   // K per LDS tile


__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    f32x2 v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));   // v_cvt_pk_bf16_f32 (RNE)
}

// (a, b) -> packed bf16 pairs hi, mid, lo with a = hi.x + mid.x + lo.x (same for b)
__device__ __forceinline__ void split2(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
    h = pk_bf16(a, b);
    const float ra = a - __uint_as_float(h << 16);
    const float rb = b - __uint_as_float(h & 0xffff0000u);
    m = pk_bf16(ra, rb);
    l = pk_bf16(ra - __uint_as_float(m << 16), rb - __uint_as_float(m & 0xffff0000u));
}


// bytes of one k-half image of ROWS rows (+128 B bank offset between the halves);
// NP planes (3: bf16 hi/mid/lo, 2: fp16 hi/lo)
template <int ROWS, int NP = 3>
struct XImg {
    static constexpr int HALF = ROWS * 16 + 128;
    static constexpr int PLANE = 2 * HALF;
    static constexpr int BYTES = NP * PLANE;
};

__device__ __forceinline__ f32x16 mfma_bf16(const uint4& a, const uint4& b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
}

// float4 along k at (row, k = 4q) -> the three planes' 8-byte pieces of that row's chunk
template <int ROWS>
__device__ __forceinline__ void put_row4(char* img, int row, int q, float4 v) {
    using I = XImg<ROWS>;
    uint32_t h0, m0, l0, h1, m1, l1;
    split2(v.x, v.y, h0, m0, l0);
    split2(v.z, v.w, h1, m1, l1);
    char* d = img + (q >> 1) * I::HALF + row * 16 + (q & 1) * 8;
    *reinterpret_cast<uint2*>(d) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(d + I::PLANE) = make_uint2(m0, m1);
    *reinterpret_cast<uint2*>(d + 2 * I::PLANE) = make_uint2(l0, l1);
}

// fp16 pair form of put_row4 (row scale 2^e)
template <int ROWS>
__device__ __forceinline__ void put_row4h(char* img, int row, int q, float4 v, int e) {
    using I = XImg<ROWS, 2>;
    uint32_t h0, l0, h1, l1;
    split2h(v.x, v.y, e, h0, l0);
    split2h(v.z, v.w, e, h1, l1);
    char* d = img + (q >> 1) * I::HALF + row * 16 + (q & 1) * 8;
    *reinterpret_cast<uint2*>(d) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(d + I::PLANE) = make_uint2(l0, l1);
}

// 8 consecutive k of column c (k-half g) -> one 16-byte chunk per plane
template <int ROWS>
__device__ __forceinline__ void put_col8(char* img, int c, int g, const float (&v)[8]) {
    using I = XImg<ROWS>;
    uint32_t h[4], m[4], l[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) split2(v[2 * t], v[2 * t + 1], h[t], m[t], l[t]);
    char* d = img + g * I::HALF + c * 16;
    *reinterpret_cast<uint4*>(d) = make_uint4(h[0], h[1], h[2], h[3]);
    *reinterpret_cast<uint4*>(d + I::PLANE) = make_uint4(m[0], m[1], m[2], m[3]);
    *reinterpret_cast<uint4*>(d + 2 * I::PLANE) = make_uint4(l[0], l[1], l[2], l[3]);
}

// fp16 pair form of put_col8 (column scale 2^e)
template <int ROWS>
__device__ __forceinline__ void put_col8h(char* img, int c, int g, const float (&v)[8], int e) {
    using I = XImg<ROWS, 2>;
    uint32_t h[4], l[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) split2h(v[2 * t], v[2 * t + 1], e, h[t], l[t]);
    char* d = img + g * I::HALF + c * 16;
    *reinterpret_cast<uint4*>(d) = make_uint4(h[0], h[1], h[2], h[3]);
    *reinterpret_cast<uint4*>(d + I::PLANE) = make_uint4(l[0], l[1], l[2], l[3]);
}

// R consecutive k of column c (sub-strip q of the 16-row tile, R = 8 / 4 / 2) -> the pieces of
// put_col8h's layout: k-half q / (8 / R), byte offset 2 R (q % (8 / R)) inside the column's chunk
template <int ROWS, int R>
__device__ __forceinline__ void put_colRh(char* img, int c, int q, const float (&v)[8], int e) {
    using I = XImg<ROWS, 2>;
    constexpr int PER_HALF = 8 / R;
    char* d = img + (q / PER_HALF) * I::HALF + c * 16 + (q % PER_HALF) * (2 * R);
    if constexpr (R == 4) {
        uint32_t h[2], l[2];
        split2h(v[0], v[1], e, h[0], l[0]);
        split2h(v[2], v[3], e, h[1], l[1]);
        *reinterpret_cast<uint2*>(d) = make_uint2(h[0], h[1]);
        *reinterpret_cast<uint2*>(d + I::PLANE) = make_uint2(l[0], l[1]);
    } else {
        static_assert(R == 2, "sub-strips of 4 or 2 rows");
        uint32_t h, l;
        split2h(v[0], v[1], e, h, l);
        *reinterpret_cast<uint32_t*>(d) = h;
        *reinterpret_cast<uint32_t*>(d + I::PLANE) = l;
    }
}


typedef __attribute__((address_space(3))) void lds_void_t;

// 16 bytes per lane global -> LDS (global_load_lds_dwordx4): lane l lands at
// lds_wave_base + 16 l; the base must be wave-uniform.  Issued from inline asm so the
// compiler does not treat the in-flight DMA as a pending write of every later ds_read
// (it would drain it with vmcnt(0) at the next fragment read); the stager waits for
// its DMAs itself (dma_wait) before the barrier that publishes them.
__device__ __forceinline__ void dma16(const void* gsrc, char* lds_wave_base) {
    const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t*)lds_wave_base);
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(l) : "memory", "m0");
}
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------------------
// Main loop of the NT kernel: every fragment double-buffered in registers, every
// global operand moved by LDS-DMA (invisible to the compiler's wait counting, so no
// hidden vmcnt drains; the waits are counted here).
//
// Iteration kt: the fragments of tile kt are in registers (set `c`); its MFMAs run
// while the fragments of tile kt+1 are read from image buffer (kt+1)&1 (set `n`).
// Image buffer kt&1 -- read into registers during iteration kt-1 -- receives tile
// kt+2: its B part by DMA from the pre-split weight image, its A part split from the
// raw ring (VALU spread over row tile 0's MFMAs).  Raw A of tile kt+4 is DMA'd into
// the ring slot freed by iteration kt-1's split.  At the end `vmcnt(A_F4)` retires
// every DMA but this iteration's raw A, which gets a second iteration to land.
// ---------------------------------------------------------------------------
template <int TM, int TN, int BM, int BN, bool SWAP, typename Stager>
__device__ __forceinline__ void x6_mainloop_pf(char* smem, int nkt, int wm0, int wn0, f32x16 (&acc)[TM][TN],
                                               Stager& st, unsigned long long* stamps = nullptr) {
    constexpr bool H = Stager::H;          // fp16 pair (3 products) instead of bf16 triple (6)
    constexpr int NP = H ? 2 : 3;
    constexpr int NPROD = H ? 3 : 6;
    using IA = XImg<BM, NP>;
    using IB = XImg<BN, NP>;
    constexpr int BUF = IA::BYTES + IB::BYTES;
    const int lane = lane_id();
    const int l32 = lane & 31, hi = lane >> 5;
    const int aoff = hi * IA::HALF + (wm0 + l32) * 16;
    const int boff = IA::BYTES + hi * IB::HALF + (wn0 + l32) * 16;
    auto rd = [&](const char* q, int plane, uint4 (&f)[NP]) {
#pragma unroll
        for (int p = 0; p < NP; ++p) f[p] = *reinterpret_cast<const uint4*>(q + p * plane);
    };
    auto rdA = [&](const char* buf, uint4 (&a)[TM][NP], int i0, int i1) {
#pragma unroll
        for (int i = i0; i < i1; ++i) rd(buf + aoff + 32 * 16 * i, IA::PLANE, a[i]);
    };
    auto rdB = [&](const char* buf, uint4 (&b)[TN][NP]) {
#pragma unroll
        for (int j = 0; j < TN; ++j) rd(buf + boff + 32 * 16 * j, IB::PLANE, b[j]);
    };
    // SWAP: the MFMA's A operand is the weight fragment, so acc[i][j] holds the transposed
    // tile (lanes along samples, registers along features) for nt_epilogue_direct
    auto mf = [&](const uint4& a, const uint4& b, const f32x16& c) {
        if constexpr (H) return SWAP ? mfma_f16(b, a, c) : mfma_f16(a, b, c);
        else return SWAP ? mfma_bf16(b, a, c) : mfma_bf16(a, b, c);
    };
    auto mm = [&](int i, const uint4 (&a)[NP], const uint4 (&b)[TN][NP]) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            f32x16 c = acc[i][j];
            if constexpr (H) {
                c = mf(a[0], b[j][1], c);            // hi.lo
                c = mf(a[1], b[j][0], c);            // lo.hi
                c = mf(a[0], b[j][0], c);            // hi.hi
            } else {
                c = mf(a[1], b[j][1], c);            // mid.mid
                c = mf(a[0], b[j][2], c);            // hi.lo
                c = mf(a[2], b[j][0], c);            // lo.hi
                c = mf(a[0], b[j][1], c);            // hi.mid
                c = mf(a[1], b[j][0], c);            // mid.hi
                c = mf(a[0], b[j][0], c);            // hi.hi
            }
            acc[i][j] = c;
        }
    };
    uint4 aX[TM][NP], bX[TN][NP], aY[TM][NP], bY[TN][NP];

    st.prologue3(smem, nkt);        // tiles 0, 1 in image buffers 0, 1; raw tiles 2, 3 in the ring
    rdA(smem, aX, 0, TM);
    rdB(smem, bX);
    __syncthreads();                // buffer 0 is restaged in iteration 0
    stamp(stamps, 1);

    auto iter = [&](int kt, uint4 (&ac)[TM][NP], uint4 (&bc)[TN][NP], uint4 (&an)[TM][NP], uint4 (&bn)[TN][NP]) {
        char* wimg = smem + (kt & 1) * BUF;
        const char* nbuf = smem + ((kt + 1) & 1) * BUF;
        constexpr int HT = (TM + 1) / 2;
        // row tiles whose MFMAs carry the split VALU: 6 products per tile leave room for it
        // in row tile 0's gaps, 3 products need two row tiles
        constexpr int R0 = (H && TM >= 2) ? 2 : 1;
        st.dma3(kt, nkt, wimg + IA::BYTES);   // B image of tile kt+2, then raw A of tile kt+4
        float4 raw[Stager::A_F4];
        st.read_raw3(kt, raw);                 // raw A of tile kt+2
        rdB(nbuf, bn);
        rdA(nbuf, an, 0, HT);
        st.split_raw(raw, wimg);
#pragma unroll
        for (int i = 0; i < R0; ++i) mm(i, ac[i], bc);
#pragma unroll
        for (int q = 0; q < NPROD * TN * R0; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = R0; i < HT; ++i) mm(i, ac[i], bc);
        __builtin_amdgcn_sched_barrier(0);
        rdA(nbuf, an, HT, TM);
#pragma unroll
        for (int i = (HT > R0 ? HT : R0); i < TM; ++i) mm(i, ac[i], bc);
        if (kt == 5) stamp(stamps, 6);
        st.wait3();
        if (kt == 5) stamp(stamps, 7);
        __syncthreads();
        if (kt == 5) stamp(stamps, 8);
    };
    for (int kt = 0; kt < nkt; kt += 2) {
        iter(kt, aX, bX, aY, bY);
        iter(kt + 1, aY, bY, aX, bX);
    }
}


// ---------------------------------------------------------------------------
// NT: C[m][n] = epi( sum_k A[m][k] B[n][k] ).
// A (activations, f32 [m][k]): LDS-DMA into a 2-slot raw ring, 16 B per lane (a wave
// moves 16 rows x 64 B), split from there into the A image.  B: fragments loaded
// straight from the pre-split weight image (p.bs, L2-resident).  No staging registers.
// ---------------------------------------------------------------------------
template <int BM, int BN, int NT, bool HH = false>
struct NTStager {
    static constexpr bool H = HH;                   // fp16 pair images (precision mode 2)
    static constexpr int NP = H ? 2 : 3;
    static constexpr int A_F4 = BM * XK / 4 / NT;   // raw A float4 (= DMA instructions) per thread and tile
    static constexpr int RSTEP = NT / 4;            // rows per pass of the block
    static constexpr int RAW = BM * XK * 4;         // bytes of one raw A slot
    static constexpr int NSLOT = 3;
    static constexpr int B_CH = 2 * NP * BN;        // 16-B chunks of a tile's B image
    static constexpr int B_C = (B_CH + NT - 1) / NT;
    static_assert(A_F4 >= 1 && BN % 64 == 0, "bad tile");
    const float* a1b; const float* a2b; const uint16_t* bsb;
    int lda1, lda2, k1, bs_rows, Kc;
    int r0, q0;
    int ea[A_F4];                                   // H: row scale exponents of this thread's rows
    char* raw;
    const int* lea;                                 // H: the block's row exponents (LDS)

    __device__ __forceinline__ void init(const NTArgs& p, int m0, int n0, int K, char* raw_ring, const int* lds_ea) {
        lda1 = p.lda1; lda2 = p.lda2; k1 = p.k1; bs_rows = p.bs_rows; Kc = K / 8;
        a1b = p.a1 + (size_t)m0 * lda1;
        a2b = p.a2 ? p.a2 + (size_t)m0 * lda2 : p.a1;
        bsb = p.bs + (size_t)n0 * 8;
        r0 = threadIdx.x >> 2; q0 = threadIdx.x & 3;
        raw = raw_ring;
        lea = lds_ea;   // read after the prologue's first barrier (the kernel fills it)
    }
    __device__ __forceinline__ void dma_a_piece(int kt, int slot, int i) {
        const int kk = kt * XK;
        const bool seg1 = kk < k1;
        const float* abase = seg1 ? a1b + kk : a2b + (kk - k1);
        const int lda = seg1 ? lda1 : lda2;
        const int wrow = (threadIdx.x >> 6) * 16;   // first row of this wave's lanes
        dma16(abase + (size_t)(r0 + i * RSTEP) * lda + 4 * q0, raw + slot * RAW + (wrow + i * RSTEP) * 64);
    }
    __device__ __forceinline__ void dma_a(int kt, int slot) {
#pragma unroll
        for (int i = 0; i < A_F4; ++i) dma_a_piece(kt, slot, i);
    }
    __device__ __forceinline__ void dma_b_piece(int kt, char* Bimg, int i) {
        const uint16_t* bt = bsb + (size_t)kt * 16 * bs_rows;
        const int lane = threadIdx.x & 63;
        const int idx = threadIdx.x + NT * i;
        const int n = idx % BN, pk = idx / BN;
        dma16(bt + (((size_t)(pk >> 1) * Kc + (pk & 1)) * bs_rows + n) * 8,
              Bimg + (pk >> 1) * XImg<BN, NP>::PLANE + (pk & 1) * XImg<BN, NP>::HALF + (n - lane) * 16);
    }
    __device__ __forceinline__ void dma_b(int kt, char* Bimg) {
#pragma unroll
        for (int i = 0; i < B_C; ++i) {
            if (B_C * NT != B_CH && (int)(threadIdx.x & ~63) + NT * i >= B_CH) break;   // wave-uniform
            dma_b_piece(kt, Bimg, i);
        }
    }
    __device__ __forceinline__ void read_slot(int slot, float4 (&v)[A_F4]) {
#pragma unroll
        for (int i = 0; i < A_F4; ++i)
            v[i] = *reinterpret_cast<const float4*>(raw + slot * RAW + (r0 + i * RSTEP) * 64 + q0 * 16);
    }
    __device__ __forceinline__ void put(const float4 (&v)[A_F4], char* Aimg) {
#pragma unroll
        for (int i = 0; i < A_F4; ++i) {
            if constexpr (H) put_row4h<BM>(Aimg, r0 + i * RSTEP, q0, v[i], ea[i]);
            else put_row4<BM>(Aimg, r0 + i * RSTEP, q0, v[i]);
        }
    }
    __device__ __forceinline__ int clamp(int t, int nkt) const { return t < nkt ? t : nkt - 1; }
    // tiles 0, 1 in image buffers 0, 1 (raw tile t lives in slot t % 3); raw tiles 2 (landed)
    // and 3 (in flight) in the ring
    __device__ __forceinline__ void prologue3(char* smem, int nkt) {
        constexpr int BUF = XImg<BM, NP>::BYTES + XImg<BN, NP>::BYTES;
        dma_a(0, 0);
        dma_a(clamp(1, nkt), 1);
        dma_a(clamp(2, nkt), 2);
        dma_b(0, smem + XImg<BM, NP>::BYTES);
        dma_b(clamp(1, nkt), smem + BUF + XImg<BM, NP>::BYTES);
        dma_wait();
        __syncthreads();
        if (H) {
#pragma unroll
            for (int i = 0; i < A_F4; ++i) ea[i] = lea[r0 + i * RSTEP];
        }
        float4 v[A_F4];
        read_slot(0, v);
        put(v, smem);
        read_slot(1, v);
        put(v, smem + BUF);
        __syncthreads();            // slot 0 is refilled below (tile 3)
        dma_a(clamp(3, nkt), 0);
    }
    // iteration kt: B image of tile kt+2 into buffer kt&1 (lands this iteration), then raw A
    // of tile kt+4 into slot (kt+4)%3 = (kt+1)%3 (lands next iteration)
    __device__ __forceinline__ void dma3(int kt, int nkt, char* Bimg) {
        dma_b(clamp(kt + 2, nkt), Bimg);
        dma_a(clamp(kt + 4, nkt), (kt + 1) % NSLOT);
    }
    __device__ __forceinline__ void read_raw3(int kt, float4 (&v)[A_F4]) { read_slot((kt + 2) % NSLOT, v); }
    __device__ __forceinline__ void split_raw(const float4 (&v)[A_F4], char* Aimg) {
        put(v, Aimg);
    }
    // one float4 of the split (NERF_NT_SPREAD schedule)
    __device__ __forceinline__ void split_piece(const float4 (&v)[A_F4], char* Aimg, int i) {
        if constexpr (H) put_row4h<BM>(Aimg, r0 + i * RSTEP, q0, v[i], ea[i]);
        else put_row4<BM>(Aimg, r0 + i * RSTEP, q0, v[i]);
    }
    // everything but this iteration's raw-A DMA (the last A_F4 VM instructions) has landed
    __device__ __forceinline__ void wait3() {
        static_assert(A_F4 <= 63, "vmcnt field");
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_F4) : "memory");
    }
};

// OCC: waves per SIMD the kernel is compiled for (2: two co-resident blocks per CU, one
// block's epilogue store burst beside the other's MFMAs; <= 256 registers per lane)
template <int BM, int BN, int WM, int WN, int EPI, bool DIRECT, bool H = false, int OCC = 1, bool HD = false>
__global__ __launch_bounds__(64 * WM * WN, OCC) void k_gemm_nt_x6(NTArgs p) {
    constexpr int NT = 64 * WM * WN;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int NP = H ? 2 : 3;
    using St = NTStager<BM, BN, NT, H>;
    static_assert(TM >= 1 && TN >= 1, "bad tile");
    static_assert(!H || DIRECT, "the fp16 pair kernels use the direct epilogue");
    constexpr int IMG_BYTES = 2 * (XImg<BM, NP>::BYTES + XImg<BN, NP>::BYTES);
    constexpr int LOOP_BYTES = IMG_BYTES + St::NSLOT * St::RAW;
    constexpr int EPI_BYTES = DIRECT ? BM * (BN / 32) * 4 : (NT / 64) * TileLds<TN>::BYTES + (BM * (BN / 32) + BM) * 4;
    constexpr int MAIN_BYTES = LOOP_BYTES > EPI_BYTES ? LOOP_BYTES : EPI_BYTES;
    constexpr int NG = BM >= 128 ? BM / 128 : 1;                // 128-row groups of the tile
    // leb[BN], lea[BM], lrm[BM], lcm[NG][BN], lvb[BN] (the epilogue's bias / rank-1 v of this column block)
    constexpr int SCALE_BYTES = H ? (2 * BN + 2 * BM + NG * BN) * 4 : 0;
    __shared__ __attribute__((aligned(16))) char smem[MAIN_BYTES + SCALE_BYTES];
    const int wave = threadIdx.x >> 6;
    const int wm0 = (wave / WN) * WTM;
    const int wn0 = (wave % WN) * WTN;
    const int m0 = blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const int K = p.k1 + p.k2;
    int* leb = reinterpret_cast<int*>(smem + MAIN_BYTES);
    int* lea = leb + BN;
    uint32_t* lrm = reinterpret_cast<uint32_t*>(lea + BM);
    uint32_t* lcm = lrm + BM;
    float* lvb = H ? reinterpret_cast<float*>(lcm + NG * BN) : nullptr;

    stamp(p.stamps, 0);
    if (H) {
        // Block constants in LDS, published by the prologue's first barrier: weight row
        // exponents (plane 2 of the image, one int per 16-byte row chunk), bias (forward) / v
        // (input gradient), row exponents of A, zeroed row / column max accumulators.  bias
        // and v live here because a global load between the epilogue's stores would wait
        // for them (loads and stores retire through one vmcnt in order).  All loads are
        // issued (clamped indices, no per-element branches) before the first LDS write, so
        // the block pays one load latency here, not one per array.
        const float* vb = EPI == EPI_FWD ? p.bias : (p.u ? p.v : nullptr);
        const int* eimg = reinterpret_cast<const int*>(p.bs + (size_t)2 * (K / 8) * p.bs_rows * 8);
        constexpr int IB = (BN + NT - 1) / NT, IA = (BM + NT - 1) / NT;
        int ev[IB];
        float vv[IB], av[IA];
#pragma unroll
        for (int i = 0; i < IB; ++i) {
            const int e = threadIdx.x + i * NT, ec = e < BN ? e : BN - 1;
            ev[i] = eimg[(size_t)(n0 + ec) * 4];
            vv[i] = vb ? vb[n0 + ec] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < IA; ++i) {
            const int e = threadIdx.x + i * NT;
            av[i] = a_rowmax(p, m0 + (e < BM ? e : BM - 1));
        }
#pragma unroll
        for (int i = 0; i < IB; ++i) {
            const int e = threadIdx.x + i * NT;
            if (e < BN) {
                leb[e] = ev[i];
                lvb[e] = vv[i];
            }
        }
#pragma unroll
        for (int i = 0; i < IA; ++i) {
            const int e = threadIdx.x + i * NT;
            if (e < BM) {
                lea[e] = row_exp(av[i]);
                lrm[e] = 0u;
            }
        }
        for (int e = threadIdx.x; e < NG * BN; e += NT) lcm[e] = 0u;
        // vmcnt(0) as the builtin, which the compiler's wait insertion sees (an asm wait it
        // cannot: it would then re-wait before reusing a load's register -- after the first
        // operand DMA, which that wait would also drain)
        __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    St st;
    st.init(p, m0, n0, K, smem + IMG_BYTES, lea);
    f32x16 acc[TM][TN];
    zero_acc(acc);
    if (DIRECT) {
        x6_mainloop_pf<TM, TN, BM, BN, true>(smem, K / XK, wm0, wn0, acc, st, p.stamps);
        stamp(p.stamps, 2);
        constexpr int MW = BN / 32;
        const bool gather = EPI == EPI_FWD && p.mask_out != nullptr && !(p.ablate & 1);
        // fused heads: per-wave row partials in LDS after the mask rows (one column block only)
        const bool heads = HD && EPI == EPI_FWD && H && p.n_heads > 0 && !(p.ablate & 1);
        static_assert(BM * MW * 4 + WN * BM * 3 * 4 + 3 * BN * 4 <= MAIN_BYTES, "heads overflow the staging LDS");
        float* lhs = heads ? reinterpret_cast<float*>(smem + BM * MW * 4) + (wave % WN) * BM * 3 : nullptr;
        float* lhw = heads ? reinterpret_cast<float*>(smem + BM * MW * 4 + WN * BM * 3 * 4) : nullptr;
        uint32_t* lmask = nullptr;
        if (gather || heads) {    // the mask rows / head partials reuse the staging LDS once the last DMA landed
            dma_wait();
            __syncthreads();
            if (gather) lmask = reinterpret_cast<uint32_t*>(smem);
            if (heads) {          // head weights [n_heads][BN] of this column block, one pass of the block
                for (int e = threadIdx.x; e < p.n_heads * BN; e += NT)
                    lhw[e] = p.head_w[(size_t)(e / BN) * p.n + n0 + e % BN];
                __syncthreads();
            }
        }
        nt_epilogue_direct<TM, TN, EPI, H, HD>(p, acc, m0, n0, wm0, wn0, lmask, MW, leb, lea, lrm,
                                               (H && p.c_cmax) ? lcm : nullptr, BN, lhs, lhw, BN, lvb);
        if (gather || heads || (H && (p.c_rmax || p.c_cmax))) {
            __syncthreads();
            if (heads) {
                const float* part = reinterpret_cast<const float*>(smem + BM * MW * 4);
                for (int e = threadIdx.x; e < BM * 3; e += NT) {
                    const int r = e / 3, c = e - 3 * r;
                    if (c >= p.n_heads) continue;
                    float v = 0.f;
#pragma unroll
                    for (int w = 0; w < WN; ++w) v += part[w * BM * 3 + e];
                    p.raw4[(size_t)(m0 + r) * 4 + p.raw_col + c] = v + p.head_b[c];
                }
            }
            if (gather)
                for (int e = threadIdx.x; e < BM * MW; e += NT)
                    p.mask_out[(size_t)(m0 + e / MW) * p.ldmo + (n0 >> 5) + e % MW] = lmask[e];
            if (H && p.c_rmax) {
                // one column block: plain stores; several: max-accumulate (caller zeroes c_rmax)
                for (int e = threadIdx.x; e < BM; e += NT) {
                    if (gridDim.y == 1) p.c_rmax[m0 + e] = __uint_as_float(lrm[e]);
                    else atomicMax(reinterpret_cast<uint32_t*>(p.c_rmax) + m0 + e, lrm[e]);
                }
            }
            if (H && p.c_cmax)   // every (128-row group, column) pair belongs to one block
                for (int e = threadIdx.x; e < NG * BN; e += NT)
                    p.c_cmax[(size_t)(m0 / 128 + e / BN) * p.ldcm + n0 + e % BN] = __uint_as_float(lcm[e]);
        }
        dma_wait();      // the last (clamped) raw-A DMA lands before the workgroup's LDS is released
    } else {
        NTEpiPrefetch<BM, BN, NT, EPI> pf;
        pf.load(p, m0, n0);
        x6_mainloop_pf<TM, TN, BM, BN, false>(smem, K / XK, wm0, wn0, acc, st, p.stamps);
        dma_wait();      // the last (clamped) raw-A DMA must land before the epilogue reuses LDS
        __syncthreads();
        stamp(p.stamps, 2);
        nt_epilogue_lds<BM, BN, NT, TM, TN, EPI>(p, acc, smem, m0, n0, wm0, wn0, pf);
    }
    if (p.stamps) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stamp(p.stamps, 3);
    }
}

// ---------------------------------------------------------------------------
// TN (weight gradient): slab[split][o][col0+j] = sum_s dy[s][o] x[s][j].  Both operands
// are sample-major: 8-row column strips, split in the kernel; the bias gradient (column
// sums of dy) is accumulated from the same registers.
// ---------------------------------------------------------------------------
// The strips of a k-tile can be loaded NS tiles ahead of the split that consumes them (NS
// register sets; dispatch_tn_x6 picks the depth).

template <int BM, int BN, int NT, bool HH = false, int NSET = 1>
struct TNStager {
    static constexpr bool H = HH;       // fp16 pair images with per-column scales (mode 2)
    static constexpr int NP = H ? 2 : 3;
    static constexpr int NS = NSET;     // register sets (tiles in flight)
    static constexpr int SA = (2 * BM + NT - 1) / NT;
    // RB: rows per x strip.  With fewer than NT / 2 columns the 8-row strips would go to part of
    // the threads only; as RB-row sub-strips (RB = 16 BN / NT: 4 for 128 columns, 2 for 64 at
    // eight waves) every thread takes one and every wave loads and splits the same share instead
    // of some waves waiting at each barrier for the others
    static constexpr int RB = (HH && NT % BN == 0 && (NT / BN == 4 || NT / BN == 8)) ? 16 * BN / NT : 8;
    static constexpr bool BQ = RB < 8;
    static constexpr int SB = BQ ? 1 : (2 * BN + NT - 1) / NT;
    const float* dyb; const float* xb;
    int lddy, ldx;
    int offa[SA], offb[SB];
    int ea[SA], eb[SB];                 // H: scale exponents of this thread's columns
    float va[NS][SA][8], vb[NS][SB][8];
    float bsum[SA];
    bool do_bias;
    __device__ __forceinline__ bool a_ok(int i) const { return SA * NT == 2 * BM || (int)threadIdx.x + NT * i < 2 * BM; }
    __device__ __forceinline__ bool b_ok(int i) const {
        return BQ || SB * NT == 2 * BN || (int)threadIdx.x + NT * i < 2 * BN;
    }

    // buffer descriptors over this split's dy / x rows: one 32-bit lane offset per strip
    // (VGPR) and the row offset of each of its 8 loads in an SGPR, instead of 16 + 16
    // per-load 64-bit addresses
    __amdgpu_buffer_rsrc_t rdy, rx;
    __device__ __forceinline__ void init(const TNArgs& p, size_t s0, int o0, int j0, bool bias) {
        lddy = p.lddy; ldx = p.ldx;
        dyb = p.dy + s0 * lddy + o0;
        xb = p.x + s0 * ldx + j0;
        rdy = __builtin_amdgcn_make_buffer_rsrc((void*)dyb, (short)0, (p.rows_per_split * lddy - o0) * 4, 0x00020000);
        rx = __builtin_amdgcn_make_buffer_rsrc((void*)xb, (short)0, (p.rows_per_split * ldx - j0) * 4, 0x00020000);
#pragma unroll
        for (int i = 0; i < SA; ++i) {
            const int idx = threadIdx.x + NT * i;
            offa[i] = 4 * (8 * (idx / BM) * lddy + idx % BM);
            bsum[i] = 0.f;
            if (H) ea[i] = row_exp(tn_colmax(p.cm_dy, p.ldcm_dy, s0, p.rows_per_split, o0 + idx % BM));
        }
#pragma unroll
        for (int i = 0; i < SB; ++i) {
            const int idx = threadIdx.x + NT * i;
            offb[i] = 4 * (RB * (idx / BN) * ldx + idx % BN);
            if (H) eb[i] = row_exp(tn_colmax(p.cm_x, p.ldcm_x, s0, p.rows_per_split, j0 + idx % BN));
        }
        do_bias = bias;
    }
    template <int U>
    __device__ __forceinline__ void load(int kt) {
        const int sa = kt * XK * lddy * 4, sb = kt * XK * ldx * 4;
#pragma unroll
        for (int i = 0; i < SA; ++i)
            if (a_ok(i)) {
#pragma unroll
                for (int t = 0; t < 8; ++t)
                    va[U][i][t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rdy, offa[i], sa + t * lddy * 4, 0));
            }
#pragma unroll
        for (int i = 0; i < SB; ++i)
            if (b_ok(i)) {
#pragma unroll
                for (int t = 0; t < RB; ++t)
                    vb[U][i][t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, offb[i], sb + t * ldx * 4, 0));
            }
    }
    // bias sums are taken here, once per real tile (`count` false for the clamped
    // re-stage of the last tile at the end of the main loop)
    template <int U>
    __device__ __forceinline__ void put(char* Aimg, char* Bimg, bool count) {
#pragma unroll
        for (int i = 0; i < SA; ++i)
            if (a_ok(i)) {
                const int idx = threadIdx.x + NT * i;
                if constexpr (H) put_col8h<BM>(Aimg, idx % BM, idx / BM, va[U][i], ea[i]);
                else put_col8<BM>(Aimg, idx % BM, idx / BM, va[U][i]);
                if (do_bias && count) {
                    float s = 0.f;
#pragma unroll
                    for (int t = 0; t < 8; ++t) s += va[U][i][t];
                    bsum[i] += s;
                }
            }
#pragma unroll
        for (int i = 0; i < SB; ++i)
            if (b_ok(i)) {
                const int idx = threadIdx.x + NT * i;
                if constexpr (BQ) put_colRh<BN, RB>(Bimg, idx % BN, idx / BN, vb[U][i], eb[i]);
                else if constexpr (H) put_col8h<BN>(Bimg, idx % BN, idx / BN, vb[U][i], eb[i]);
                else put_col8<BN>(Bimg, idx % BN, idx / BN, vb[U][i]);
            }
    }
    template <int U>
    __device__ __forceinline__ void prologue_load(int nkt) {
        if constexpr (U < NS) {
            if (U < nkt) load<U>(U);
            prologue_load<U + 1>(nkt);
        }
    }
    // register pipeline: tile 0 in image buffer 0, raw tiles 1 .. NS-1 in flight (tile t
    // lives in register set t % NS)
    __device__ __forceinline__ void prologue(char* smem, int nkt) {
        prologue_load<0>(nkt);
        put<0>(smem, smem + XImg<BM, NP>::BYTES, true);
        if constexpr (NS == 1) {
            if (1 < nkt) load<0>(1);
        }
        __syncthreads();
    }
};

// Main loop of the TN kernel (split-bf16 / fp16 pair images, register-staged column strips):
// iteration kt reads the fragments of tile kt from buffer kt&1, splits tile kt+1 (register
// set (kt+1) % NS) into the other buffer, issues the loads of tile kt+NS into the set tile kt
// used (NS == 1: tile kt+2 into the one set, as before), then the MFMAs (VALU of the split
// interleaved, 3 per MFMA gap) and one barrier.
// phase-clock hooks of the TN main loop (the round-3 stamp build is retired: no-ops)
struct TnClock {
    __device__ __forceinline__ void begin() {}
    __device__ __forceinline__ void tick(int) {}
    __device__ __forceinline__ void write(unsigned long long*) {}
};

template <int TM, int TN, int BM, int BN, typename Stager>
__device__ __forceinline__ void tn_mainloop(char* smem, int nkt, int wm0, int wn0, f32x16 (&acc)[TM][TN],
                                            Stager& st, TnClock& clk) {
    constexpr bool H = Stager::H;
    constexpr int NP = H ? 2 : 3;
    constexpr int NS = Stager::NS;
    using IA = XImg<BM, NP>;
    using IB = XImg<BN, NP>;
    constexpr int BUF = IA::BYTES + IB::BYTES;
    const int lane = lane_id();
    const int l32 = lane & 31, hi = lane >> 5;
    const int aoff = hi * IA::HALF + (wm0 + l32) * 16;
    const int boff = IA::BYTES + hi * IB::HALF + (wn0 + l32) * 16;
    auto rd = [&](const char* q, int plane, uint4 (&f)[NP]) {
#pragma unroll
        for (int p = 0; p < NP; ++p) f[p] = *reinterpret_cast<const uint4*>(q + p * plane);
    };
    auto mm = [&](int i, const uint4 (&a)[NP], const uint4 (&b)[TN][NP]) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            f32x16 c = acc[i][j];
            if constexpr (H) {
                c = mfma_f16(a[0], b[j][1], c);    // hi.lo
                c = mfma_f16(a[1], b[j][0], c);    // lo.hi
                c = mfma_f16(a[0], b[j][0], c);    // hi.hi
            } else {
                c = mfma_bf16(a[1], b[j][1], c);   // mid.mid
                c = mfma_bf16(a[0], b[j][2], c);   // hi.lo
                c = mfma_bf16(a[2], b[j][0], c);   // lo.hi
                c = mfma_bf16(a[0], b[j][1], c);   // hi.mid
                c = mfma_bf16(a[1], b[j][0], c);   // mid.hi
                c = mfma_bf16(a[0], b[j][0], c);   // hi.hi
            }
            acc[i][j] = c;
        }
    };
    constexpr int NPROD = H ? 3 : 6;
    st.prologue(smem, nkt);
    clk.tick(5);
    auto iter = [&](int kt, auto uc) {
        constexpr int U = decltype(uc)::value;
        const char* cur = smem + (kt & 1) * BUF;
        char* wimg = smem + ((kt + 1) & 1) * BUF;
        uint4 b[TN][NP], a[TM][NP];
#pragma unroll
        for (int j = 0; j < TN; ++j) rd(cur + boff + 32 * 16 * j, IB::PLANE, b[j]);
#pragma unroll
        for (int i = 0; i < TM; ++i) rd(cur + aoff + 32 * 16 * i, IA::PLANE, a[i]);
        clk.tick(0);
        if (kt + 1 < nkt) st.template put<(U + 1) % NS>(wimg, wimg + IA::BYTES, true);
        clk.tick(1);
        if constexpr (NS == 1) {
            if (kt + 2 < nkt) st.template load<0>(kt + 2);
        } else {
            if (kt + NS < nkt) st.template load<U>(kt + NS);
        }
        clk.tick(2);
#pragma unroll
        for (int i = 0; i < TM; ++i) mm(i, a[i], b);
#pragma unroll
        for (int q = 0; q < NPROD * TN * TM; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        clk.tick(3);
        __syncthreads();
        clk.tick(4);
    };
    for (int kt0 = 0; kt0 < nkt; kt0 += NS) {
        iter(kt0, std::integral_constant<int, 0>{});
        if constexpr (NS > 1) { if (kt0 + 1 < nkt) iter(kt0 + 1, std::integral_constant<int, 1 % NS>{}); }
        if constexpr (NS > 2) { if (kt0 + 2 < nkt) iter(kt0 + 2, std::integral_constant<int, 2 % NS>{}); }
        if constexpr (NS > 3) { if (kt0 + 3 < nkt) iter(kt0 + 3, std::integral_constant<int, 3 % NS>{}); }
    }
}

// CT > 0: XCD-paired column tiles.  One output row tile (nout == BM) and CT column tiles of
// BN; a 1-D grid of splits * CT workgroups in which the CT column tiles of one split sit on
// the same XCD in consecutive dispatch slots (workgroups go round-robin over the 8 XCDs, so
// w and w + 8 share one), so they stream the same dy rows at about the same time and the
// second read of a dy k-tile hits that XCD's L2.  With BN = kin / 2 this halves the split-K
// slab bytes of a 256 x 256 layer (twice the rows per split at the same block count)
// without a second HBM read of dy.  Needs splits % 8 == 0.
// LDS of one TN block: two operand image buffers (the epilogue's per-wave tiles reuse them),
// + H: the tile's row / column scale exponents
template <int BM, int BN, int WM, int WN, bool H>
struct TNSmem {
    static constexpr int NT = 64 * WM * WN;
    static constexpr int TN = BN / WN / 32;
    static constexpr int NP = H ? 2 : 3;
    static constexpr int BUF = XImg<BM, NP>::BYTES + XImg<BN, NP>::BYTES;
    static constexpr int LOOP = 2 * BUF;
    static constexpr int EPI = (NT / 64) * TileLds<TN>::BYTES;
    static constexpr int MAIN = LOOP > EPI ? LOOP : EPI;
    static constexpr int BYTES = MAIN + (H ? (BM + BN) * 4 : 0);
};

// one TN block: output rows o0 .. o0 + BM, column tile jt (x columns jt BN ..), split `split`
template <int BM, int BN, int WM, int WN, bool H, int NS>
__device__ __forceinline__ void tn_block(const TNArgs& p, char* smem, int o0, int jt, int split) {
    constexpr int NT = 64 * WM * WN;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    static_assert(TM >= 1 && TN >= 1, "bad tile");
    static_assert(TNSmem<BM, BN, WM, WN, H>::LOOP >= 2 * BM * 4, "bias scratch");
    constexpr int MAIN_BYTES = TNSmem<BM, BN, WM, WN, H>::MAIN;
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int wm0 = (wave / WN) * WTM;
    const int wn0 = (wave % WN) * WTN;
    const int j0 = jt * BN;
    const size_t s0 = (size_t)split * p.rows_per_split;
    const int nkt = p.rows_per_split / XK;
    const bool do_bias = (p.bslab != nullptr) && (jt == 0) && !(p.ablate & 4);

    int* lea = reinterpret_cast<int*>(smem + MAIN_BYTES);   // H: scale exponents of the tile's rows / columns
    int* leb = lea + BM;
    if (H) {   // published by the prologue's barrier
        for (int e = tid; e < BM; e += NT) lea[e] = row_exp(tn_colmax(p.cm_dy, p.ldcm_dy, s0, p.rows_per_split, o0 + e));
        for (int e = tid; e < BN; e += NT) leb[e] = row_exp(tn_colmax(p.cm_x, p.ldcm_x, s0, p.rows_per_split, j0 + e));
    }
    TnClock clk;
    clk.begin();
    TNStager<BM, BN, NT, H, NS> st;
    st.init(p, s0, o0, j0, do_bias);
    f32x16 acc[TM][TN];
    zero_acc(acc);
    tn_mainloop<TM, TN, BM, BN>(smem, nkt, wm0, wn0, acc, st, clk);

    if constexpr (H) tn_store_lds<TM, TN, true>(p, acc, smem, split, o0, j0, wm0, wn0, lea, leb);
    else tn_store_lds(p, acc, smem, split, o0, j0, wm0, wn0);
    if (do_bias && !(p.ablate & 1)) {
        // strip (c, g) partial sums -> column sums, added in g order (deterministic)
        __syncthreads();
        float* lb = reinterpret_cast<float*>(smem);
#pragma unroll
        for (int i = 0; i < TNStager<BM, BN, NT>::SA; ++i)
            if (st.a_ok(i)) lb[tid + NT * i] = st.bsum[i];
        __syncthreads();
        for (int c = tid; c < BM; c += NT) p.bslab[(size_t)split * p.nout + o0 + c] = lb[c] + lb[BM + c];
    }
    clk.tick(6);
    clk.write(p.stamps);
}

template <int BM, int BN, int WM, int WN, bool H = false, int NS = 1, int CT = 0>
__global__ __launch_bounds__(64 * WM * WN, WM * WN >= 8 ? 2 : 1) void k_gemm_tn_x6(TNArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[TNSmem<BM, BN, WM, WN, H>::BYTES];
    int o0, jt, split;
    if constexpr (CT > 0) {
        const int w = blockIdx.x, slot = w >> 3;
        o0 = 0;
        jt = slot % CT;
        split = (slot / CT) * 8 + (w & 7);
    } else {
        o0 = blockIdx.x * BM;
        jt = blockIdx.y;
        split = blockIdx.z;
    }
    tn_block<BM, BN, WM, WN, H, NS>(p, smem, o0, jt, split);
}

// A layer with a 64-wide second input segment (l4's skip input enc_p, the colour layer's
// view encoding enc_d) in ONE launch (nerf_linear_bwd_weight_seg): per split, CT column tiles
// of BN over the first segment (pm) and one BN2 tile over the second (ps: its x, col0 = k1),
// all CT + 1 on one XCD in consecutive dispatch slots (workgroups go round-robin over the 8
// XCDs), so the split's dy rows come from HBM once and from that XCD's L2 for the other tiles
// -- as two launches, the 64-wide one re-read all of dy for a quarter of the columns.
template <int BM, int BN, int WM, int WN, int BN2, int WM2, int WN2, int CT, int NS>
__global__ __launch_bounds__(64 * WM * WN, 2) void k_gemm_tn_x6_seg(TNArgs pm, TNArgs ps) {
    static_assert(WM * WN == WM2 * WN2 && WM * WN == 8, "both tiles at eight waves");
    constexpr int B1 = TNSmem<BM, BN, WM, WN, true>::BYTES, B2 = TNSmem<BM, BN2, WM2, WN2, true>::BYTES;
    __shared__ __attribute__((aligned(16))) char smem[B1 > B2 ? B1 : B2];
    const int w = blockIdx.x, slot = w >> 3;
    const int jt = slot % (CT + 1);
    const int split = (slot / (CT + 1)) * 8 + (w & 7);
    if (jt < CT) tn_block<BM, BN, WM, WN, true, NS>(pm, smem, 0, jt, split);
    else tn_block<BM, BN2, WM2, WN2, true, NS>(ps, smem, 0, 0, split);
}

template <int BM, int BN, int WM, int WN, int EPI>
static void launch_nt_x6(const NTArgs& a, hipStream_t s, bool h16) {
    constexpr bool co = BM == 128 && BN == 256;   // fits two co-resident blocks per CU (fp16 pair)
    if constexpr (EPI == EPI_FWD) {
        if (h16 && a.n_heads > 0) {   // fused output heads: their own instantiation (registers)
            hipLaunchKernelGGL((k_gemm_nt_x6<BM, BN, WM, WN, EPI, true, true, co ? 2 : 1, true>),
                               dim3(a.m / BM, a.n / BN), dim3(64 * WM * WN), 0, s, a);
            return;
        }
    }
    if (h16 && co)
        hipLaunchKernelGGL((k_gemm_nt_x6<BM, BN, WM, WN, EPI, true, true, co ? 2 : 1>), dim3(a.m / BM, a.n / BN),
                           dim3(64 * WM * WN), 0, s, a);
    else if (h16)
        hipLaunchKernelGGL((k_gemm_nt_x6<BM, BN, WM, WN, EPI, true, true>), dim3(a.m / BM, a.n / BN),
                           dim3(64 * WM * WN), 0, s, a);
    else
        hipLaunchKernelGGL((k_gemm_nt_x6<BM, BN, WM, WN, EPI, true>), dim3(a.m / BM, a.n / BN), dim3(64 * WM * WN), 0,
                           s, a);
}

// default policy (3): 256x256 tiles for the bf16x3 kernels; the fp16 pair kernels at 128x256
// with two co-resident blocks per CU (one block's epilogue stores beside the other's MFMAs:
// 96 -> 83 us for a 131072 x 256 x 256 forward, profiles/r01/gemm_policy_h16.txt)
template <int EPI>
static void pick_nt_x6(const NTArgs& a, int pol, hipStream_t s, bool h16) {
    // fused output heads: one column block holds the whole output row (its head dot products
    // are complete per block), whatever the policy
    if (EPI == EPI_FWD && h16 && a.n_heads > 0) {
        if (a.n == 256) launch_nt_x6<128, 256, 2, 2, EPI>(a, s, h16);
        else launch_nt_x6<128, 128, 2, 2, EPI>(a, s, h16);
        return;
    }
    if (h16 && pol == 3 && a.n % 256 == 0) launch_nt_x6<128, 256, 2, 2, EPI>(a, s, h16);
    else if (pol == 3 && a.m % 256 == 0 && a.n % 256 == 0) launch_nt_x6<256, 256, 2, 2, EPI>(a, s, h16);
    else if (pol >= 2 && a.n % 256 == 0) launch_nt_x6<128, 256, 2, 2, EPI>(a, s, h16);
    else if (a.n % 128 == 0) launch_nt_x6<128, 128, 2, 2, EPI>(a, s, h16);
    else launch_nt_x6<128, 64, 2, 2, EPI>(a, s, h16);
}

int dispatch_nt_x6(const NTArgs& a, int epi, int policy, hipStream_t s, double flops, bool h16) {
    prof_begin(s);
    if (epi == EPI_FWD) pick_nt_x6<EPI_FWD>(a, policy, s, h16);
    else pick_nt_x6<EPI_BWD>(a, policy, s, h16);
    prof_end(s, flops, h16 ? 3 : 6);
    return check_launch(h16 ? "k_gemm_nt_x6 (fp16 pair)" : "k_gemm_nt_x6");
}

// one register set for the eight-wave TN tiles too: loads issued two and three iterations
// ahead (register sets 3 / 4) ran the same, 90.3 / 90.8 / 90.6 us per 131072 x 256 x 256
// weight gradient (profiles/r03/tn_ns_ab.txt) -- the loop is not waiting on load latency
constexpr int kTnNs8 = 1;

template <bool H>
static void pick_tn_x6(const TNArgs& a, int nout, int kin, int splits, int policy, hipStream_t s) {
    constexpr int NS = 1;   // the 4-wave tiles: loaded 3 ahead ran the same (profiles/r02/tn_pipeline_ab.txt)
    if (tn_xcd_group(policy, nout, kin, splits) == 2)   // eight waves (two per SIMD), 64 x 64 per wave
        hipLaunchKernelGGL((k_gemm_tn_x6<256, 128, 4, 2, H, kTnNs8, 2>), dim3(2 * splits), dim3(512), 0, s, a);
    else if (policy >= 3 && nout % 256 == 0 && kin % 256 == 0)
        hipLaunchKernelGGL((k_gemm_tn_x6<256, 256, 2, 2, H, NS>), dim3(nout / 256, kin / 256, splits), dim3(256), 0,
                           s, a);
    else if (policy >= 7 && nout == 128 && kin % 256 == 0)
        // the colour layer (128 outputs, 256 feature columns): one column tile per 256 inputs, so
        // each split reads its dy rows once (two 128 x 128 column tiles read them twice)
        hipLaunchKernelGGL((k_gemm_tn_x6<128, 256, 2, 4, H, kTnNs8>), dim3(1, kin / 256, splits), dim3(512), 0, s, a);
    else if (nout % 128 == 0 && kin % 128 == 0)
        hipLaunchKernelGGL((k_gemm_tn_x6<128, 128, 2, 2, H, NS>), dim3(nout / 128, kin / 128, splits), dim3(256), 0,
                           s, a);
    else if (policy >= 7 && nout % 256 == 0 && kin == 64)   // eight waves, 64 x 32 per wave
        hipLaunchKernelGGL((k_gemm_tn_x6<256, 64, 4, 2, H, kTnNs8>), dim3(nout / 256, 1, splits), dim3(512), 0, s, a);
    else if (policy >= 3 && nout % 256 == 0 && kin == 64)
        // a 64-wide input (the encodings: l0, the skip segment of l4) against all 256 outputs in
        // one tile, so each split's dy rows are read once (128 x 64 tiles read them twice)
        hipLaunchKernelGGL((k_gemm_tn_x6<256, 64, 2, 2, H, NS>), dim3(nout / 256, 1, splits), dim3(256), 0, s, a);
    else if (nout % 128 == 0)
        hipLaunchKernelGGL((k_gemm_tn_x6<128, 64, 2, 2, H, NS>), dim3(nout / 128, kin / 64, splits), dim3(256), 0, s,
                           a);
    else if (kin % 128 == 0)
        hipLaunchKernelGGL((k_gemm_tn_x6<64, 128, 1, 4, H, NS>), dim3(nout / 64, kin / 128, splits), dim3(256), 0, s,
                           a);
    else
        hipLaunchKernelGGL((k_gemm_tn_x6<64, 64, 1, 2, H, NS>), dim3(nout / 64, kin / 64, splits), dim3(128), 0, s, a);
}

int dispatch_tn_x6(const TNArgs& a, int nout, int kin, int splits, int policy, hipStream_t s, double flops,
                   bool h16) {
    prof_begin(s);
    if (h16 && policy == 8 && wgrad_supported(nout, kin, splits, a.rows_per_split))
        launch_wgrad(a, nout, kin, splits, s);
    else if (h16) pick_tn_x6<true>(a, nout, kin, splits, policy, s);
    else pick_tn_x6<false>(a, nout, kin, splits, policy, s);
    prof_end(s, flops, h16 ? 3 : 6);
    return check_launch(h16 ? "k_gemm_tn_x6 (fp16 pair)" : "k_gemm_tn_x6");
}

bool tn_seg_supported(int nout, int k1, int k2, int splits) {
    return k2 == 64 && k1 == 256 && (nout == 256 || nout == 128) && splits % 8 == 0;
}

int dispatch_tn_x6_seg(const TNArgs& pm, const TNArgs& ps, int nout, int splits, int policy, hipStream_t s,
                       double flops) {
    prof_begin(s);
    if (policy == 8 && wgrad_seg_supported(nout, 256, 64, splits, pm.rows_per_split))
        launch_wgrad_seg(pm, ps, nout, splits, s);
    else if (nout == 256)   // l4: two XCD-paired 256 x 128 tiles over h3 + the 256 x 64 tile over enc_p
        hipLaunchKernelGGL((k_gemm_tn_x6_seg<256, 128, 4, 2, 64, 4, 2, 2, kTnNs8>), dim3(3 * splits), dim3(512), 0, s, pm,
                           ps);
    else               // colour layer: the 128 x 256 tile over f + the 128 x 64 tile over enc_d
        hipLaunchKernelGGL((k_gemm_tn_x6_seg<128, 256, 2, 4, 64, 4, 2, 1, kTnNs8>), dim3(2 * splits), dim3(512), 0, s, pm,
                           ps);
    prof_end(s, flops, 3);
    return check_launch("k_gemm_tn_x6_seg (fp16 pair)");
}

}  // namespace nerf
