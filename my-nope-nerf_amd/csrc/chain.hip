// Fused forward chain of the field MLP (GEMM precision mode 2, hidden width 256).
//
// OfficialStaticNerf's ten linears (official_nerf.py:20-37, 60-91) run in ONE launch: a
// block owns 128 sample rows (4 waves x 32 rows) and walks them through
//   l0 [enc_p] -> l1 -> l2 -> l3 -> l4 [h3, enc_p] -> l5 -> l6 -> l7 -> lf -> lr [f, enc_d]
// with the activation tile resident in registers between layers.  Per layer a wave holds
//   * its A operand: 32 rows x K as row-scaled fp16 pairs (x 2^e = hi + lo, the split of
//     gemm_x6.hip precision mode 2), 4 VGPRs per plane and 16-deep k-step;
//   * the accumulators: 32 rows x 256 outputs in AGPRs (operand-swapped MFMAs, so a lane
//     owns one sample row and 16 features per 32x32 tile, gemm.hpp nt_epilogue_direct).
// The weights stream through a 5-slot LDS ring by LDS-DMA (pre-split fp16 pair images of
// nerf_pack_weights, 16 KB per k-step); their schedule does not depend on the activations,
// so the ring runs ahead across layer boundaries and the next layer's first k-steps land
// during the epilogue.  The epilogue undoes the scales, adds the bias, applies the ReLU,
// stores the f32 activation (the backward's saved tensor; skipped when `out` is NULL, as in
// eval renders), the ReLU bits and the per-feature column maxima of the 128-row group (the
// weight-gradient GEMM's scales), then re-splits the tile as the next layer's A operand:
// the row max over both half-wave lanes sets the new exponent and one v_permlane32_swap per
// VGPR pair turns the accumulator layout (lane halves hold alternating feature quads) into
// the fragment layout (lane halves hold 8 consecutive features).
//
// Against one launch per layer (gemm_x6.hip) this removes the read of every layer input
// (134 MB per 256-wide layer at 1024 x 128 samples), every per-layer prologue, launch gap
// and tail, and keeps the weight stream off the critical path.
#include "gemm.hpp"
#include "samples.hpp"

#include <cstdlib>
#include <type_traits>

namespace nerf {
namespace {

typedef _Float16 ch16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 ch16x2 __attribute__((ext_vector_type(2)));
typedef float cf32x2 __attribute__((ext_vector_type(2)));

constexpr int CNL = 10;                     // layers
constexpr int CROWS = 128;                  // rows per block (4 waves x 32)
constexpr int NSLOT = 5;                    // weight ring slots
constexpr int SHALF = 256 * 16 + 128;       // one k-half of a 256-row slot (+ bank offset)
constexpr int SPLANE = 2 * SHALF;
constexpr int SBYTES = 2 * SPLANE;          // two planes (fp16 hi / lo)
constexpr int DMA_PER_STEP = 4;             // LDS-DMA instructions per wave and k-step
constexpr int STG_LD = 36;                  // floats per row of a wave's epilogue staging tile (32 + pad)

// topology (hidden width 256, colour width 128): k-steps of each layer's weight image,
// k-steps taken from the register tile, from an encoding, output width
constexpr int L_KS[CNL] = {4, 16, 16, 16, 20, 16, 16, 16, 16, 20};
constexpr int L_OUT[CNL] = {256, 256, 256, 256, 256, 256, 256, 256, 256, 128};

__device__ __forceinline__ f32x16 cmfma(const uint4& w, const uint4& a, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(ch16x8, w), __builtin_bit_cast(ch16x8, a), c,
                                                  0, 0, 0);
}
__device__ __forceinline__ uint32_t cpk(float a, float b) {
    cf32x2 v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, ch16x2));   // RNE
}
// already scaled (a, b) -> fp16 pair words (hi, lo)
// MIX: the residual a - hi (exact in f32) by one v_fma_mix_f32 per value, -hi x 1 + a reading
// the fp16 half in place, instead of a conversion back to f32 and a subtraction -- the same
// bits at two thirds of the VALU (the training chain keeps the conversions: the mix form
// costs it a register it does not have)
template <bool MIX = true>
__device__ __forceinline__ void csplit(float a, float b, uint32_t& h, uint32_t& l) {
    h = cpk(a, b);
    if constexpr (MIX) {
        float ra, rb;
        asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(ra) : "v"(h), "v"(a));
        asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(rb) : "v"(h), "v"(b));
        l = cpk(ra, rb);
    } else {
        const ch16x2 hv = __builtin_bit_cast(ch16x2, h);
        l = cpk(a - (float)hv[0], b - (float)hv[1]);
    }
}

typedef __attribute__((address_space(3))) void clds_t;
// 16 bytes per lane from sbase + voff (wave-uniform base in SGPRs, 32-bit lane offset: no
// 64-bit per-lane addresses to keep live) into LDS at lds_wave_base + 16 lane
__device__ __forceinline__ void cdma16(const void* sbase, uint32_t voff, char* lds_wave_base) {
    const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(clds_t*)lds_wave_base);
    asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(l) : "memory", "m0");
}

// 8 consecutive f32 (k = 8 hf .. 8 hf + 7 of one k-step) scaled by 2^e -> fragment planes
__device__ __forceinline__ void frag_from8(const float4& u, const float4& v, int e, uint4& hi, uint4& lo) {
    const float s0 = __builtin_amdgcn_ldexpf(u.x, e), s1 = __builtin_amdgcn_ldexpf(u.y, e);
    const float s2 = __builtin_amdgcn_ldexpf(u.z, e), s3 = __builtin_amdgcn_ldexpf(u.w, e);
    const float s4 = __builtin_amdgcn_ldexpf(v.x, e), s5 = __builtin_amdgcn_ldexpf(v.y, e);
    const float s6 = __builtin_amdgcn_ldexpf(v.z, e), s7 = __builtin_amdgcn_ldexpf(v.w, e);
    csplit<false>(s0, s1, hi.x, lo.x);
    csplit<false>(s2, s3, hi.y, lo.y);
    csplit<false>(s4, s5, hi.z, lo.z);
    csplit<false>(s6, s7, hi.w, lo.w);
}

}  // namespace

struct ChainFwdArgs {
    const float* enc_p; const float* enc_d;   // [n_pad][64]
    const float* rp; const float* rd;         // row maxima of enc_p / enc_d
    int n_pad;
    nerf_chain_layer L[CNL];
    unsigned long long* stamps;   // diagnostics (nerf_chain_debug_stamps): per-block phase cycles or NULL
    // the fused per-ray eval render (nerf_render_eval_fused): samples + encodings in the
    // prologue, density / colour heads in the l7 / colour-layer epilogues, sigma -> alpha ->
    // composite of the block's rays at the end
    const float* po; const float* pd; const float* view;   // [R][3]
    int R, S, flags;
    float near_z, far_z;
    const float* wd; const float* bd;   // fc_density weight [256], bias [1]
    const float* wc; const float* bc;   // fc_rgb weight padded [3][128], bias [3]
    float* rgb; float* dist; float* alpha; float* z;   // [R][3], [R], [R][S], [R*S]
    float* raw4;                                       // training chain: [n_pad][4] head outputs
};

constexpr int kbase(int l) { return l == 0 ? 0 : kbase(l - 1) + L_KS[l - 1]; }
constexpr int CT = kbase(CNL);   // k-steps of the whole chain

// per-block state of the chain (all register arrays statically indexed after inlining)
struct ChainState {
    char* ring; char* leb16; float* lbias; uint32_t* lcm;   // leb16: [2][256 rows][16 B], exponent in word 0
    char* lenc; float* lrp; float* lrd;                      // encoding tile [128][64], row maxima [128] x 2
    float* stage;                                            // this wave's [32][STG_LD] epilogue tile
    float* fx;                                               // fused eval: wd [256], wc [3][128], raw [128][4], z [128]
    int tid, lane, sl, hf;
    size_t m0, row;
    int er;                          // row exponent of the current A operand
    uint4 act_hi[16], act_lo[16];    // register tile: 16 k-steps of the 256 activations
    uint4 enc_hi[4], enc_lo[4];      // encoding segment of the current layer
    f32x16 acc[8];
    unsigned long long t_wait, t_bar, t_mma, t_epi, t_last;   // diagnostics (stamps)
};

__device__ __forceinline__ void chain_tick(const ChainFwdArgs& p, ChainState& st, unsigned long long& bucket) {
    if (p.stamps == nullptr) return;
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    bucket += t - st.t_last;
    st.t_last = t;
    __builtin_amdgcn_sched_barrier(0);
}

constexpr bool first_step(int tt) {
    for (int l = 0; l < CNL; ++l)
        if (kbase(l) == tt) return true;
    return false;
}
constexpr int ENC_D_STEP = 4 + 16 * 3 + 20;   // kbase(5): the enc_d tile replaces enc_p once l4 is done
// LDS-DMA instructions every wave issues with global k-step tt (uniform across waves):
// 4 for the weight ring, +2 at a layer's first step (weight-row exponents, biases), +10 at
// step 0 (enc_p tile 8, enc_p / enc_d row maxima 1 + 1), +8 at ENC_D_STEP (enc_d tile)
// (fused eval: the encodings are computed in-kernel, so step 0 and ENC_D_STEP carry no extras)
constexpr int dma_count(int tt, bool fused = false) {
    return tt >= CT ? 0
                    : DMA_PER_STEP + (first_step(tt) ? 2 : 0) + (tt == 0 && !fused ? 10 : 0) +
                          (tt == ENC_D_STEP && !fused ? 8 : 0);
}
// DMAs issued after those of step tt by the time step tt is consumed (steps tt+1 .. tt+NSLOT-2)
constexpr int dma_after(int tt, bool fused = false) {
    int n = 0;
    for (int u = tt + 1; u <= tt + NSLOT - 2; ++u) n += dma_count(u, fused);
    return n;
}

// the 128-row x 64 encoding tile of the block into LDS: wave w moves rows 32 w .. 32 w + 31,
// four 256-byte rows per instruction
__device__ __forceinline__ void chain_dma_enc(const float* enc, ChainState& st) {
    const int w = st.tid >> 6;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int r = 32 * w + 4 * i + (st.lane >> 4);
        cdma16(enc + st.m0 * 64, (uint32_t)(r * 256 + (st.lane & 15) * 16), st.lenc + (32 * w + 4 * i) * 256);
    }
}

// global k-step TT -> ring slot TT % NSLOT, plus the extras of dma_count(TT)
template <int TT, bool F>
__device__ __forceinline__ void chain_dma(const ChainFwdArgs& p, ChainState& st) {
    if constexpr (TT < CT) {
        constexpr int l = [] { int i = 0; while (kbase(i + 1) <= TT) ++i; return i; }();
        constexpr int s = TT - kbase(l);
        constexpr int ks = L_KS[l];
        const nerf_chain_layer& L = p.L[l];
        const int w = st.tid >> 6;
        char* slot = st.ring + (TT % NSLOT) * SBYTES;
#pragma unroll
        for (int i = 0; i < DMA_PER_STEP; ++i) {
            int n, ph;   // image row, plane * 2 + k-half
            if (L_OUT[l] == 256) { n = st.tid; ph = i; }
            else { n = st.tid & 127; ph = ((st.tid >> 7) + 2 * i) & 3; }   // 128 rows: i = 2, 3 repeat i = 0, 1
            const uint32_t off = (uint32_t)(((ph >> 1) * (2 * ks) + 2 * s + (ph & 1)) * L.img_rows + n) * 16;
            cdma16(L.img, off, slot + (ph >> 1) * SPLANE + (ph & 1) * SHALF + (n - st.lane) * 16);
        }
        if constexpr (s == 0) {
            // this layer's weight-row exponents (the 16-byte plane-2 chunk 0 of each image row,
            // exponent in its first word) and biases, into the layer's LDS parity buffers
            const int wr = L_OUT[l] == 256 ? w : (w & 1);
            const int n = 64 * wr + st.lane;
            cdma16(L.img, (uint32_t)((2 * (2 * ks) * L.img_rows + n) * 16), st.leb16 + (l & 1) * 4096 + 64 * wr * 16);
            // one instruction with lanes 0-15 active (lane l lands at base + 16 l): 64 biases
            if (st.lane < 16)
                cdma16(L.bias, (uint32_t)((64 * wr + 4 * st.lane) * 4), reinterpret_cast<char*>(st.lbias + (l & 1) * 256 + 64 * wr));
        }
        if constexpr (TT == 0 && !F) {
            chain_dma_enc(p.enc_p, st);
            if (st.lane < 8) {   // 32 row maxima per wave
                cdma16(p.rp + st.m0, (uint32_t)((32 * w + 4 * st.lane) * 4), reinterpret_cast<char*>(st.lrp + 32 * w));
                cdma16(p.rd + st.m0, (uint32_t)((32 * w + 4 * st.lane) * 4), reinterpret_cast<char*>(st.lrd + 32 * w));
            }
        }
        if constexpr (TT == ENC_D_STEP && !F) chain_dma_enc(p.enc_d, st);
    }
}

// one k-step of layer l: wait for its slot, publish, refill the ring, MFMAs
template <int l, int s, bool F>
__device__ __forceinline__ void chain_kstep(const ChainFwdArgs& p, ChainState& st) {
    constexpr int TT = kbase(l) + s;
    constexpr int nreg = l == 0 ? 0 : 16;
    constexpr int ntj = L_OUT[l] / 32;
    chain_tick(p, st, st.t_mma);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(dma_after(TT, F)) : "memory");   // this step's DMAs landed
    chain_tick(p, st, st.t_wait);
    __syncthreads();
    chain_tick(p, st, st.t_bar);
    chain_dma<TT + NSLOT - 1, F>(p, st);
    if constexpr (s == 0) {
        // layer prologue (behind a barrier): the previous layer's column maxima out, this
        // layer's column-max accumulators zeroed (its exponents and biases arrived by DMA)
        if constexpr (l > 0) {
            if (p.L[l - 1].cmax)
                p.L[l - 1].cmax[(st.m0 / 128) * L_OUT[l - 1] + st.tid] =
                    __uint_as_float(st.lcm[((l - 1) & 1) * 256 + st.tid]);
        }
        st.lcm[(l & 1) * 256 + st.tid] = 0u;
    }
    const char* slot = st.ring + (TT % NSLOT) * SBYTES;
    const uint4& ah = s < nreg ? st.act_hi[s < nreg ? s : 0] : st.enc_hi[s < nreg ? 0 : s - nreg];
    const uint4& al = s < nreg ? st.act_lo[s < nreg ? s : 0] : st.enc_lo[s < nreg ? 0 : s - nreg];
    // weight fragments two tiles ahead of their MFMAs (3 rotating pairs); the scheduling
    // barriers pin the order so every LDS read has two MFMA groups (~190 cycles) to land
    const char* bbase = slot + st.hf * SHALF + st.sl * 16;
    uint4 bh[3], bl[3];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        bh[j] = *reinterpret_cast<const uint4*>(bbase + 32 * 16 * j);
        bl[j] = *reinterpret_cast<const uint4*>(bbase + 32 * 16 * j + SPLANE);
    }
#pragma unroll
    for (int j = 0; j < ntj; ++j) {
        if (j + 2 < ntj) {
            bh[(j + 2) % 3] = *reinterpret_cast<const uint4*>(bbase + 32 * 16 * (j + 2));
            bl[(j + 2) % 3] = *reinterpret_cast<const uint4*>(bbase + 32 * 16 * (j + 2) + SPLANE);
        }
        __builtin_amdgcn_sched_barrier(0);
        st.acc[j] = cmfma(bh[j % 3], al, st.acc[j]);   // hi . lo
        st.acc[j] = cmfma(bl[j % 3], ah, st.acc[j]);   // lo . hi
        st.acc[j] = cmfma(bh[j % 3], ah, st.acc[j]);   // hi . hi
        if constexpr (l > 0 && s < nreg && !F) {
            if (j == 1 && p.L[l - 1].out) {
                // the previous layer's output, stored beside this layer's MFMAs instead of in a
                // burst at its epilogue: this k-step's 8 features of the row, rebuilt from the
                // fp16 pair (hi + lo) 2^-e -- the value the next layer consumed, within 2^-22
                // relative of the f32 epilogue result
                const ch16x2* h = reinterpret_cast<const ch16x2*>(&ah);
                const ch16x2* o = reinterpret_cast<const ch16x2*>(&al);
                float v[8];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    v[2 * t] = __builtin_amdgcn_ldexpf((float)h[t][0] + (float)o[t][0], -st.er);
                    v[2 * t + 1] = __builtin_amdgcn_ldexpf((float)h[t][1] + (float)o[t][1], -st.er);
                }
                float* dst = p.L[l - 1].out + st.row * p.L[l - 1].ldo + 16 * s + 8 * st.hf;
                *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
                *reinterpret_cast<float4*>(dst + 4) = make_float4(v[4], v[5], v[6], v[7]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int l, int s, bool F>
__device__ __forceinline__ void chain_ksteps(const ChainFwdArgs& p, ChainState& st) {
    if constexpr (s < L_KS[l]) {
        chain_kstep<l, s, F>(p, st);
        chain_ksteps<l, s + 1, F>(p, st);
    }
}

// this lane's 8-feature chunks of the encoding row (LDS tile) -> the 4 encoding k-steps of
// the current A operand at exponent st.er
__device__ __forceinline__ void enc_frags(ChainState& st, int rl) {
    const float4* src = reinterpret_cast<const float4*>(st.lenc + rl * 256);
#pragma unroll
    for (int s = 0; s < 4; ++s)
        frag_from8(src[4 * s + 2 * st.hf], src[4 * s + 2 * st.hf + 1], st.er, st.enc_hi[s], st.enc_lo[s]);
}

// fused eval: the view-direction encodings of the block's rays (27 values of
// encode_position L = 4, official_nerf.py:87, 99-119, zero padded to 32) and their maxima
// live in LDS, one 36-float record per ray (fx + FX_ENCD): the view direction is per ray,
// so 128 / S records serve the block's 128 rows
constexpr int FX_RAW = 640, FX_Z = 1152, FX_ENCD = 1280, ENCD_REC = 36;
__device__ __forceinline__ void fused_encode_d(const ChainFwdArgs& p, float* fx, int tid, size_t m0) {
    const int nr = CROWS / p.S;
    if (tid >= nr) return;
    const size_t ray = m0 / (size_t)p.S + tid;
    float d[3] = {0.f, 0.f, 0.f};
    if (ray < (size_t)p.R) {
#pragma unroll
        for (int c = 0; c < 3; ++c) d[c] = p.view[3 * ray + c];
    }
    float* rec = fx + FX_ENCD + ENCD_REC * tid;
    float m = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) { rec[c] = d[c]; m = fmaxf(m, fabsf(d[c])); }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float f = (float)(1 << i);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float sn, cs;
            sincosf(f * d[c], &sn, &cs);
            rec[3 + 6 * i + c] = sn;
            rec[6 + 6 * i + c] = cs;
            m = fmaxf(m, fmaxf(fabsf(sn), fabsf(cs)));
        }
    }
#pragma unroll
    for (int c = 27; c < 32; ++c) rec[c] = 0.f;
    rec[32] = m;
}
// the same records spread over threads t0 .. t0 + nt - 1 (nt a multiple of 64): sixteen lanes
// (one DPP row) per ray, lane i < 12 one (level i / 3, coordinate i % 3) sin / cos pair, lane 12
// the direction itself, the record's max by a row reduction -- the same values as
// fused_encode_d, 12 sincosf deep on one thread there, one here
// the direction of the ray whose record lane u of the range works on in pass rb (zero past the
// rays): loaded before the prologue's LDS-DMAs for pass 0
__device__ __forceinline__ void encd_load(const ChainFwdArgs& p, int u, int nt, size_t m0, int rb, float (&d)[3]) {
    const int nr = CROWS / p.S;
    const int r = rb + (u >> 4);
    const size_t ray = m0 / (size_t)p.S + r;
    const bool live = u >= 0 && u < nt && r < nr && ray < (size_t)p.R;
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] = live ? p.view[3 * ray + c] : 0.f;
}
__device__ __forceinline__ void fused_encode_d_rows(const ChainFwdArgs& p, float* fx, int tid, int t0, int nt,
                                                    size_t m0, const float (&d0)[3]) {
    const int nr = CROWS / p.S;
    const int u = tid - t0;
    if (u < 0 || u >= nt) return;
    const int i = u & 15;
    for (int rb = 0; rb < nr; rb += nt / 16) {   // block-uniform trip count: the row shuffles stay converged
        const int r = rb + (u >> 4);
        float dv[3] = {d0[0], d0[1], d0[2]};
        if (rb > 0) encd_load(p, u, nt, m0, rb, dv);
        float m = 0.f;
        if (r < nr) {
            float* rec = fx + FX_ENCD + ENCD_REC * r;
            if (i < 12) {
                const int lv = i / 3, c = i % 3;
                const float d = c == 0 ? dv[0] : c == 1 ? dv[1] : dv[2];
                float sn, cs;
                sincosf((float)(1 << lv) * d, &sn, &cs);
                rec[3 + 6 * lv + c] = sn;
                rec[6 + 6 * lv + c] = cs;
                m = fmaxf(fabsf(sn), fabsf(cs));
            } else if (i == 12) {
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    rec[c] = dv[c];
                    m = fmaxf(m, fabsf(dv[c]));
                }
            } else if (i == 13) {
#pragma unroll
                for (int c = 27; c < 32; ++c) rec[c] = 0.f;
            }
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        if (r < nr && i == 0) fx[FX_ENCD + ENCD_REC * r + 32] = m;
    }
}
// this lane's 4 encoding k-steps (8-feature chunks 16 s + 8 hf .. + 7; columns >= 32 zero)
__device__ __forceinline__ void enc_d_frags(ChainState& st, const float* rec) {
    const float4* src = reinterpret_cast<const float4*>(rec);
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const float4 u = s < 2 ? src[4 * s + 2 * st.hf] : z4;
        const float4 v = s < 2 ? src[4 * s + 2 * st.hf + 1] : z4;
        frag_from8(u, v, st.er, st.enc_hi[s], st.enc_lo[s]);
    }
}

// layer l: k-loop, epilogue (features f = 32 j + 8 q + 4 hf + c of row st.row), next A
template <int l, bool F>
__device__ __forceinline__ void chain_layer(const ChainFwdArgs& p, ChainState& st) {
    constexpr int ntj = L_OUT[l] / 32;
    constexpr bool relu = l != 8;
    const nerf_chain_layer& L = p.L[l];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) st.acc[j][r] = 0.f;
    chain_ksteps<l, 0, F>(p, st);
    chain_tick(p, st, st.t_mma);
    // fused eval heads: sigma_raw = fc_density(h8) in l7's epilogue, the colour logits
    // fc_rgb(hr) in the colour layer's (official_nerf.py:66, 91), partial dots over this
    // lane's features, the lane halves summed below
    constexpr bool head_d = F && l == 7, head_c = F && l == CNL - 1;
    float hs0 = 0.f, hs1 = 0.f, hs2 = 0.f;

    // the colour layer stores its output here; every other layer's output is stored by the
    // next layer's k-steps (chain_kstep)
    const bool store_here = l == CNL - 1 && L.out != nullptr;
    const char* eb = st.leb16 + (l & 1) * 4096;
    const float* bb = st.lbias + (l & 1) * 256;
    float rmx = 0.f;
#pragma unroll
    for (int j = 0; j < ntj; ++j) {
        uint32_t w = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int f0 = 32 * j + 8 * q + 4 * st.hf;
            const int4 e4 = make_int4(*reinterpret_cast<const int*>(eb + 16 * f0), *reinterpret_cast<const int*>(eb + 16 * (f0 + 1)),
                                      *reinterpret_cast<const int*>(eb + 16 * (f0 + 2)), *reinterpret_cast<const int*>(eb + 16 * (f0 + 3)));
            const float4 b4 = *reinterpret_cast<const float4*>(bb + f0);
            float4 x;
            x.x = __builtin_amdgcn_ldexpf(st.acc[j][4 * q + 0], -(st.er + e4.x)) + b4.x;
            x.y = __builtin_amdgcn_ldexpf(st.acc[j][4 * q + 1], -(st.er + e4.y)) + b4.y;
            x.z = __builtin_amdgcn_ldexpf(st.acc[j][4 * q + 2], -(st.er + e4.z)) + b4.z;
            x.w = __builtin_amdgcn_ldexpf(st.acc[j][4 * q + 3], -(st.er + e4.w)) + b4.w;
            if (relu) x = make_float4(fmaxf(x.x, 0.f), fmaxf(x.y, 0.f), fmaxf(x.z, 0.f), fmaxf(x.w, 0.f));

            st.acc[j][4 * q + 0] = x.x; st.acc[j][4 * q + 1] = x.y;
            st.acc[j][4 * q + 2] = x.z; st.acc[j][4 * q + 3] = x.w;
            w |= ((x.x > 0.f ? 1u : 0u) | (x.y > 0.f ? 2u : 0u) | (x.z > 0.f ? 4u : 0u) | (x.w > 0.f ? 8u : 0u))
                 << (8 * q + 4 * st.hf);
            rmx = fmaxf(rmx, fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
            if (store_here || L.cmax)   // this lane's quad into the wave's staging tile (row sl, 32 features)
                *reinterpret_cast<float4*>(st.stage + st.sl * STG_LD + 8 * q + 4 * st.hf) = x;
        }
        if (L.mask) {
            w |= (uint32_t)__shfl_xor((int)w, 32, 64);
            if (st.hf == 0) L.mask[st.row * L.ldmask + j] = w;
        }
        if (store_here || L.cmax) {
            // read the tile back row-contiguous: lane l holds rows 8 r + (l >> 3) and features
            // 4 (l & 7) .. + 3, so each store covers 8 whole 128-byte row pieces (the
            // accumulator layout would scatter 64 16-byte pieces over 32 rows); the column
            // maxima reduce over 4 rows in-lane and over the 8 lanes of equal (l & 7)
            const int rr = st.lane >> 3, cq = st.lane & 7;
            float4 cmx = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float4 v = *reinterpret_cast<const float4*>(st.stage + (8 * r + rr) * STG_LD + 4 * cq);
                if (store_here)
                    *reinterpret_cast<float4*>(L.out + (st.m0 + 32 * (st.tid >> 6) + 8 * r + rr) * L.ldo + 32 * j + 4 * cq) = v;
                cmx = make_float4(fmaxf(cmx.x, fabsf(v.x)), fmaxf(cmx.y, fabsf(v.y)), fmaxf(cmx.z, fabsf(v.z)),
                                  fmaxf(cmx.w, fabsf(v.w)));
            }
            if (L.cmax) {
#pragma unroll
                for (int off = 8; off <= 32; off <<= 1) {
                    cmx.x = fmaxf(cmx.x, __shfl_xor(cmx.x, off, 64));
                    cmx.y = fmaxf(cmx.y, __shfl_xor(cmx.y, off, 64));
                    cmx.z = fmaxf(cmx.z, __shfl_xor(cmx.z, off, 64));
                    cmx.w = fmaxf(cmx.w, __shfl_xor(cmx.w, off, 64));
                }
                if (st.lane < 8) {
                    uint32_t* g = st.lcm + (l & 1) * 256 + 32 * j + 4 * cq;
                    atomicMax(g + 0, __float_as_uint(cmx.x));
                    atomicMax(g + 1, __float_as_uint(cmx.y));
                    atomicMax(g + 2, __float_as_uint(cmx.z));
                    atomicMax(g + 3, __float_as_uint(cmx.w));
                }
            }
        }
    }
    if constexpr (head_d || head_c) {
        // the head dots over the epilogue's results (acc now holds the layer output), one
        // feature quad at a time: the scheduling barriers keep the weight reads from being
        // hoisted into one 128-register burst
#pragma unroll
        for (int j = 0; j < ntj; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                __builtin_amdgcn_sched_barrier(0);
                const int f0 = 32 * j + 8 * q + 4 * st.hf;
                const float x0 = st.acc[j][4 * q], x1 = st.acc[j][4 * q + 1];
                const float x2 = st.acc[j][4 * q + 2], x3 = st.acc[j][4 * q + 3];
                if constexpr (head_d) {
                    const float4 wv = *reinterpret_cast<const float4*>(st.fx + f0);
                    hs0 += x0 * wv.x + x1 * wv.y + x2 * wv.z + x3 * wv.w;
                } else {
                    const float4 w0 = *reinterpret_cast<const float4*>(st.fx + 256 + f0);
                    const float4 w1 = *reinterpret_cast<const float4*>(st.fx + 384 + f0);
                    const float4 w2 = *reinterpret_cast<const float4*>(st.fx + 512 + f0);
                    hs0 += x0 * w0.x + x1 * w0.y + x2 * w0.z + x3 * w0.w;
                    hs1 += x0 * w1.x + x1 * w1.y + x2 * w1.z + x3 * w1.w;
                    hs2 += x0 * w2.x + x1 * w2.y + x2 * w2.z + x3 * w2.w;
                }
            }
        __builtin_amdgcn_sched_barrier(0);
        // raw4 row (sigma_raw, rgb logits) of this sample into the block's LDS rows
        float* raw = st.fx + FX_RAW + 4 * ((st.tid >> 6) * 32 + st.sl);
        hs0 += __shfl_xor(hs0, 32, 64);
        if constexpr (head_d) {
            if (st.hf == 0) raw[0] = hs0 + p.bd[0];
        } else {
            hs1 += __shfl_xor(hs1, 32, 64);
            hs2 += __shfl_xor(hs2, 32, 64);
            if (st.hf == 0) {
                raw[1] = hs0 + p.bc[0];
                raw[2] = hs1 + p.bc[1];
                raw[3] = hs2 + p.bc[2];
            }
        }
    }
    chain_tick(p, st, st.t_epi);
    if constexpr (l < CNL - 1) {
        // next layer's A operand: row exponent over the row's 256 features (and the encoding
        // joined in the next layer), fp16 pairs, quad exchange between the lane halves
        float m = fmaxf(rmx, __shfl_xor(rmx, 32, 64));
        const int rl = (st.tid >> 6) * 32 + st.sl;   // row inside the block
        const float* drec = F ? st.fx + FX_ENCD + ENCD_REC * (rl / (F ? p.S : 1)) : nullptr;
        if constexpr (l == 3) m = fmaxf(m, F ? fmaxf(st.lrp[rl], st.lrd[rl]) : st.lrp[rl]);
        if constexpr (l == 8) m = fmaxf(m, F ? drec[32] : st.lrd[rl]);
        st.er = row_exp(m);
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const int j = s >> 1, qa = 2 * (s & 1), qb = qa + 1;
            const int e = st.er;
            uint32_t ha0, la0, ha1, la1, hb0, lb0, hb1, lb1;
            csplit(__builtin_amdgcn_ldexpf(st.acc[j][4 * qa + 0], e), __builtin_amdgcn_ldexpf(st.acc[j][4 * qa + 1], e),
                   ha0, la0);
            csplit(__builtin_amdgcn_ldexpf(st.acc[j][4 * qa + 2], e), __builtin_amdgcn_ldexpf(st.acc[j][4 * qa + 3], e),
                   ha1, la1);
            csplit(__builtin_amdgcn_ldexpf(st.acc[j][4 * qb + 0], e), __builtin_amdgcn_ldexpf(st.acc[j][4 * qb + 1], e),
                   hb0, lb0);
            csplit(__builtin_amdgcn_ldexpf(st.acc[j][4 * qb + 2], e), __builtin_amdgcn_ldexpf(st.acc[j][4 * qb + 3], e),
                   hb1, lb1);
            // low lanes keep quad a and take the high lanes' quad a; high lanes take the low
            // lanes' quad b and keep quad b: v_permlane32_swap(vdst = a, vsrc = b) gives both
            const auto h0 = __builtin_amdgcn_permlane32_swap(ha0, hb0, false, false);
            const auto h1 = __builtin_amdgcn_permlane32_swap(ha1, hb1, false, false);
            const auto l0 = __builtin_amdgcn_permlane32_swap(la0, lb0, false, false);
            const auto l1 = __builtin_amdgcn_permlane32_swap(la1, lb1, false, false);
            st.act_hi[s] = make_uint4(h0[0], h1[0], h0[1], h1[1]);
            st.act_lo[s] = make_uint4(l0[0], l1[0], l0[1], l1[1]);
        }
        if constexpr (l == 3 || (l == 8 && !F)) enc_frags(st, rl);   // the enc_p / enc_d tile in LDS
        if constexpr (l == 8 && F) enc_d_frags(st, drec);
        chain_tick(p, st, st.t_epi);
    }
}

// fused eval prologue: samples (rendering.py:183-198, no jitter) and the position encoding
// (official_nerf.py:61, 99-119) of the block's 128 rows into the LDS tile the chain reads
// (the layout nerf_encode_samples writes), with row maxima and z.  Waves 0-1 write columns
// 0..32 (x, levels 0-4), waves 2-3 columns 33..63 (levels 5-9, zero pad): no divergence.
__device__ __forceinline__ void fused_encode_p(const ChainFwdArgs& p, ChainState& st) {
    const int row = st.tid & 127, half = st.tid >> 7;
    const size_t g = st.m0 + row;
    float* dst = reinterpret_cast<float*>(st.lenc + row * 256);
    float x[3] = {0.f, 0.f, 0.f}, z = 0.f;
    const bool live = g < (size_t)p.R * p.S;
    if (live) {
        const size_t ray = g / (size_t)p.S;
        const int i = (int)(g - ray * (size_t)p.S);
        z = lerp_z(linspace01(i, p.S), p.near_z, p.far_z);
#pragma unroll
        for (int c = 0; c < 3; ++c) x[c] = ray_point(p.po[3 * ray + c], p.pd[3 * ray + c], z);
    }
    float m = 0.f;
    if (half == 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) { dst[c] = x[c]; m = fmaxf(m, fabsf(x[c])); }
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const float f = (float)(1 << i);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                float sn, cs;
                sincosf(f * x[c], &sn, &cs);
                dst[3 + 6 * i + c] = sn;
                dst[6 + 6 * i + c] = cs;
                m = fmaxf(m, fmaxf(fabsf(sn), fabsf(cs)));
            }
        }
        st.fx[FX_Z + row] = z;
        if (live) p.z[g] = z;
    } else {
#pragma unroll
        for (int i = 5; i < 10; ++i) {
            const float f = (float)(1 << i);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                float sn, cs;
                sincosf(f * x[c], &sn, &cs);
                dst[3 + 6 * i + c] = sn;
                dst[6 + 6 * i + c] = cs;
                m = fmaxf(m, fmaxf(fabsf(sn), fabsf(cs)));
            }
        }
        dst[63] = 0.f;
    }
    // the two halves' maxima of a row: lrp (columns 0..32) and lrd (33..63; lrd holds no
    // enc_d maxima in the fused kernel); readers take the max of both
    (half == 0 ? st.lrp : st.lrd)[row] = m;
}

// fused eval epilogue: sigma -> alpha -> exclusive-product compositing of the block's
// 128 / S rays (rendering.py:113-141), from the raw4 / z rows in LDS, with the arithmetic of
// k_composite16_fwd (so the fused and the unfused render agree bit for bit): one 16-lane DPP
// row per ray, lane l owning samples [l J, l J + J) (J = max(1, S / 16)); transmittance by a
// row prefix-product scan, the sums by row butterflies; each lane stores its J alphas as
// contiguous float4s (a ray's S alphas are one contiguous run across its row)
template <int J, int NTH>
__device__ __forceinline__ void fused_composite16(const ChainFwdArgs& p, const float* fx, int tid, size_t m0) {
    const int S = p.S;
    const int nr = CROWS / S;
    const int l16 = tid & 15;
    for (int rb = 0; rb < nr; rb += NTH / 16) {    // NTH / 16 rays per pass of the block
        const int rloc = rb + (tid >> 4);
        const size_t ray = m0 / (size_t)S + rloc;
        const bool active = rloc < nr && ray < (size_t)p.R;   // whole 16-lane rows are (in)active
        const int i0 = l16 * J;
        float al[J], T[J], c[J][3], z[J];
        bool valid[J];
        float pl = 1.f;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int i = i0 + j;
            valid[j] = active && i < S;
            float a = 0.f, c0 = 0.f, c1 = 0.f, c2 = 0.f, zz = 0.f;
            if (valid[j]) {
                const int e = rloc * S + i;
                const float4 r = *reinterpret_cast<const float4*>(fx + FX_RAW + 4 * e);
                zz = fx[FX_Z + e];
                const float sg = f_density(r.x, p.flags);
                if (p.flags & F_DIST_ALPHA)
                    a = i == S - 1 ? 1.f : 1.f - __expf(-1.0f * sg * (fx[FX_Z + e + 1] - zz));   // rendering.py:116-122
                else
                    a = 1.f - __expf(-1.0f * sg);
                c0 = f_sigmoid(r.y); c1 = f_sigmoid(r.z); c2 = f_sigmoid(r.w);
            }
            al[j] = a; z[j] = zz;
            c[j][0] = c0; c[j][1] = c1; c[j][2] = c2;
            T[j] = pl;
            pl *= valid[j] ? (1.f - a + kEps) : 1.f;
        }
        const float excl = dpp_f<0x111>(1.f, row_scan_mul(pl));   // product over the lanes before this one
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, sd = 0.f, sw = 0.f;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const float w = al[j] * (T[j] * excl);
            s0 += w * c[j][0];
            s1 += w * c[j][1];
            s2 += w * c[j][2];
            sd += w * z[j];
            sw += w;
        }
        float* ao = p.alpha + ray * (size_t)S + i0;
        if (J % 4 == 0 && active) {
#pragma unroll
            for (int q = 0; q < J / 4; ++q)
                *reinterpret_cast<float4*>(ao + 4 * q) = make_float4(al[4 * q], al[4 * q + 1], al[4 * q + 2], al[4 * q + 3]);
        } else {
#pragma unroll
            for (int j = 0; j < J; ++j)
                if (valid[j]) ao[j] = al[j];
        }
        s0 = row_sum(s0); s1 = row_sum(s1); s2 = row_sum(s2); sd = row_sum(sd);
        if (p.flags & F_WHITE_BKGD) sw = row_sum(sw);
        if (active && l16 == 0) {
            if (p.flags & F_WHITE_BKGD) {          // rendering.py:139-141
                const float bg = 1.f - sw;
                s0 += bg; s1 += bg; s2 += bg;
            }
            p.rgb[3 * ray + 0] = s0;
            p.rgb[3 * ray + 1] = s1;
            p.rgb[3 * ray + 2] = s2;
            p.dist[ray] = sd;
        }
    }
}

template <int NTH>
__device__ __forceinline__ void fused_composite(const ChainFwdArgs& p, const float* fx, int tid, size_t m0) {
    if (p.S >= 128) fused_composite16<8, NTH>(p, fx, tid, m0);
    else if (p.S >= 64) fused_composite16<4, NTH>(p, fx, tid, m0);
    else if (p.S >= 32) fused_composite16<2, NTH>(p, fx, tid, m0);
    else fused_composite16<1, NTH>(p, fx, tid, m0);
}

template <bool F>
__global__ __launch_bounds__(256) void k_mlp_chain_fwd(ChainFwdArgs p) {
    constexpr int RING = NSLOT * SBYTES, LEB = 2 * 4096, LBIAS = 2 * 256 * 4, LCM = 2 * 256 * 4, LENC = 128 * 256;
    constexpr int LSTG = 4 * 32 * STG_LD * 4;
    static_assert(LSTG >= (FX_ENCD + ENCD_REC * 64) * 4, "the fused eval buffers live in the staging region");
    __shared__ __attribute__((aligned(16))) char smem[RING + LEB + LBIAS + LCM + LENC + 2 * 512 + LSTG];
    ChainState st;
    st.ring = smem;
    st.leb16 = smem + RING;
    st.lbias = reinterpret_cast<float*>(smem + RING + LEB);
    st.lcm = reinterpret_cast<uint32_t*>(smem + RING + LEB + LBIAS);
    st.lenc = smem + RING + LEB + LBIAS + LCM;
    st.lrp = reinterpret_cast<float*>(st.lenc + LENC);
    st.lrd = st.lrp + 128;
    st.stage = reinterpret_cast<float*>(st.lenc + LENC + 2 * 512) + (threadIdx.x >> 6) * 32 * STG_LD;
    st.fx = reinterpret_cast<float*>(st.lenc + LENC + 2 * 512);
    st.tid = threadIdx.x;
    st.lane = st.tid & 63; st.sl = st.lane & 31; st.hf = st.lane >> 5;
    st.m0 = (size_t)blockIdx.x * CROWS;
    st.row = st.m0 + 32 * (st.tid >> 6) + st.sl;
    st.t_wait = st.t_bar = st.t_mma = st.t_epi = 0;
    st.t_last = __builtin_amdgcn_s_memtime();
    const unsigned long long t_start = st.t_last;

    chain_dma<0, F>(p, st);
    chain_dma<1, F>(p, st);
    chain_dma<2, F>(p, st);
    chain_dma<3, F>(p, st);
    static_assert(NSLOT == 5, "prologue issues NSLOT - 1 k-steps");
    if constexpr (F) {
        // head weights into LDS, then the samples and position encodings (beside the DMAs)
        st.fx[st.tid] = p.wd[st.tid];
        for (int e = st.tid; e < 384; e += 256) st.fx[256 + e] = p.wc[e];
        fused_encode_p(p, st);
        fused_encode_d(p, st.fx, st.tid, st.m0);
    }
    // step 0's group (with the enc_p tile and the row maxima) landed, published to the block
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(dma_count(1, F) + dma_count(2, F) + dma_count(3, F)) : "memory");
    __syncthreads();
    const int rl = (st.tid >> 6) * 32 + st.sl;
    st.er = row_exp(F ? fmaxf(st.lrp[rl], st.lrd[rl]) : st.lrp[rl]);
    enc_frags(st, rl);

    chain_layer<0, F>(p, st);
    chain_layer<1, F>(p, st);
    chain_layer<2, F>(p, st);
    chain_layer<3, F>(p, st);
    chain_layer<4, F>(p, st);
    chain_layer<5, F>(p, st);
    chain_layer<6, F>(p, st);
    chain_layer<7, F>(p, st);
    chain_layer<8, F>(p, st);
    chain_layer<9, F>(p, st);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every DMA landed before the LDS is released
    if constexpr (F) {
        __syncthreads();   // every row's raw4 in LDS
        fused_composite<256>(p, st.fx, st.tid, st.m0);
    }
    if (p.stamps && st.tid == 0) {
        unsigned long long* o = p.stamps + (size_t)blockIdx.x * 6;
        o[0] = st.t_wait; o[1] = st.t_bar; o[2] = st.t_mma; o[3] = st.t_epi;
        o[4] = __builtin_amdgcn_s_memtime() - t_start; o[5] = __builtin_amdgcn_s_memrealtime();
    }
}

// ---------------------------------------------------------------------------
// The chains at two waves per SIMD: the fused per-ray eval kernel (k_render_fused2, the
// default of nerf_render_eval_fused), the training forward (k_mlp_chain_train2) and the
// input-gradient chain (k_mlp_chain_bwd).  Same per-ray path as k_mlp_chain_fwd -- the ten
// linears with the activations resident in registers, the weights streaming through an LDS
// ring -- but a block's 128 rows are 8 waves x 16 rows on v_mfma_f32_16x16x32_f16: a wave's
// accumulators (16 rows x 256 outputs) and its A operand (16 rows x 256 as fp16 pairs) are 64
// + 64 registers, so the kernels fit 256 registers and two waves share each SIMD.
//
// Operand-swapped 16x16x32 MFMAs: A = a weight fragment (lane l: image row l & 15, k = 8 (l >>
// 4) .. + 7), B = an activation fragment (sample l & 15, the same k), so D[feature][sample]
// puts sample l & 15 in lane l with features 16 j + 4 (l >> 4) .. + 3 of tile j (the "tile
// layout").  The next layer's k-step t takes tiles 2t and 2t + 1 AS THEY LIE: lane (g, n)'s
// eight k are features 32 t + 4 g + 0..3 and 32 t + 16 + 4 g + 0..3, and the weight images of
// these kernels (nerf_pack_weights' chain images, dst_cs / dst_cts) hold their K columns in
// that order (chain_perm).  No data moves between lanes to form an A fragment.
//
// Per value of an A operand: two v_fma_mix{lo,hi}_f16 (the fp16 pair hi = RNE(x 2^e), lo =
// RNE(x 2^e - hi), read from the f32 epilogue value and the scale 2^e in place, msplit).  The
// training kernels save what the next GEMMs need beside their MFMAs, from the same registers:
// the f32 epilogue value (two float4 stores per tile pair), its column maxima over the
// wave's 16 rows (two DPP steps per value with |.| modifiers, one LDS atomic max per lane
// quad) and, in the forward, the ReLU words (from the fp16 hi words: two bits per
// v_pk_min_u16 + v_dot2_u32_u16, one LDS atomic or per lane and k-step).
// ---------------------------------------------------------------------------
#ifndef NERF_CHAIN_STAMPS
#define NERF_CHAIN_STAMPS 0   // diagnostic builds only (make EXTRA=-DNERF_CHAIN_STAMPS=1): phase stamps
#endif
namespace f2 {
constexpr int NW = 8;                   // waves per block, two per SIMD
constexpr int NTH = 64 * NW;            // threads
constexpr int SHALF = 256 * 16;         // one k-half of a slot: 256 image rows x 16 B, unpadded (the
                                        // 16x16x32 fragment reads are conflict-free without a pad)
constexpr int SPLANE = 2 * SHALF;
constexpr int SBYTES = 2 * SPLANE;      // 16 KB per 16-k step (fp16 hi / lo planes)
constexpr int FX_WD = 0, FX_WC = 256;   // fc_density weight [256], fc_rgb weight [3][128]

// LDS map.  Eval: a 6-slot weight ring (two 32-k steps in flight) and the position-encoding
// tile the prologue computes.  Training (TR): the encodings come from HBM, so their 32 KB go
// to two more ring slots (three 32-k steps in flight: a store issued beside a k-step's
// MFMAs has three k-steps to complete before a wait counts it, see wait_n), the column
// maxima of the block's 128-row group ([2 parities][256] uint, LDS atomic max) and its ReLU
// words ([2 parities][128 rows][8] uint, LDS atomic or)
// Column maxima in LDS: CMQ copies of the [2 parities][256] array.  CMQ = 1: the max over the
// 16-lane row by four DPP steps, one LDS atomic per row; CMQ = 2 / 4: over 8 / 4 lanes by three /
// two DPP steps, one atomic per 8 / 4 lanes into copy n >> 3 / n >> 2 -- copies CMS words apart, so
// the leaders' atomics of one instruction hit distinct banks -- and the copies are combined when the
// maxima leave LDS
// (forward: 1 -- 4 copies ran within noise, profiles/r06/fwd_colmax_relu_ab.txt; input-gradient
// chain: 4 -- 469-472 vs 494-506 us, profiles/r06/colmax_copies_ab.txt)
constexpr int CMQ_FWD = 1, CMQ_BWD = 4;
constexpr int CMS = 513;                                     // words per copy (both parities + 1)
constexpr int cm_words(int q) { return q == 1 ? 512 : q * CMS; }
// the max of word w (parity * 256 + feature) over the q copies
template <int Q>
__device__ __forceinline__ uint32_t cm_read(const uint32_t* cm, int w) {
    uint32_t m = cm[w];
#pragma unroll
    for (int c = 1; c < Q; ++c) m = max(m, cm[c * CMS + w]);
    return m;
}
template <int Q>
__device__ __forceinline__ void cm_clear(uint32_t* cm, int w) {
#pragma unroll
    for (int c = 0; c < Q; ++c) cm[c * CMS + w] = 0u;
}

// words per row of the training forward's ReLU-word array (rows padded to 9 words against the
// OR atomics' 4-way bank conflicts ran slower: profiles/r06/fwd_colmax_relu_ab.txt)
constexpr int MSKW = 8;

template <bool TR>
struct LY {
    static constexpr int NSLOT = TR ? 8 : 6;
    static constexpr int D = NSLOT / 2 - 1;                   // 32-k steps in flight
    static constexpr int O_RING = 0;
    static constexpr int O_LEB = NSLOT * SBYTES;              // [2][256] int weight-row exponents (compact array)
    static constexpr int O_EXP = O_LEB + 2 * 256 * 4;         // [2][256] float: 2^-(weight-row exponent)
    static constexpr int O_BIAS = O_EXP + 2 * 256 * 4;        // [2][256] float
    static constexpr int O_ENC = O_BIAS + 2 * 256 * 4;        // eval: [128][64] float position encodings
    static constexpr int O_CMX = O_ENC;                       // training: [2][256] uint column maxima
    static constexpr int O_MSK = O_CMX + cm_words(CMQ_FWD) * 4;   // training: [2][128][MSKW] uint ReLU words
    static constexpr int O_RMX = O_ENC + 128 * 64 * 4;        // eval: [4][128] row maxima
    static constexpr int O_FX = TR ? O_MSK + 2 * 128 * MSKW * 4 : O_RMX + 4 * 128 * 4;   // head weights, raw4, ...
    static constexpr int FX_FLOATS = TR ? FX_ENCD : FX_ENCD + (CROWS / 2) * ENCD_REC;
    static constexpr int BYTES = O_FX + FX_FLOATS * 4;
    static_assert(BYTES <= 160 * 1024, "LDS");
};

constexpr int layer_of(int tt) { int i = 0; while (i + 1 < CNL && kbase(i + 1) <= tt) ++i; return i; }
constexpr int dma_count(int tt) {
    return tt >= CT ? 0 : (L_OUT[layer_of(tt)] == 256 ? 2 : 1) + (kbase(layer_of(tt)) == tt ? 1 : 0);
}

// The barrier of a 32-k step sits in the middle of the step before it.  32-k step k (global
// over the chain, slot pair k % NPAIR) is published by barrier B_k, which every wave passes at
// tile tb(k - 1) of step k - 1 (B_0 in the prologue) after waiting (vmcnt) for its own share of
// step k's DMAs; right behind B_k a wave issues the DMAs of step k - 1 + NPAIR - 1 = k + NPAIR - 2
// (the pair step k - 2 used: every wave is past it), and from tile tb + 1 on it reads step k's
// first weight fragments while step k - 1's last MFMAs run.  A step therefore starts without a
// barrier, without LDS latency and without DMA issue, and a layer's epilogue sits between two
// barriers: the two waves of a SIMD leave it at their own pace (the older one first) and the
// one ahead starts the next layer's MFMAs beside the other's epilogue VALU.
constexpr int nks(int l) { return L_KS[l] / 2; }
constexpr int kfirst(int l) { return l == 0 ? 0 : kfirst(l - 1) + nks(l - 1); }
constexpr int layer_of_k(int k) { int l = 0; while (l + 1 < CNL && kfirst(l + 1) <= k) ++l; return l; }
constexpr int tt_of_k(int k) { return kbase(layer_of_k(k)) + 2 * (k - kfirst(layer_of_k(k))); }
constexpr int NK = kfirst(CNL);             // 32-k steps of the chain
template <bool TR>
constexpr int npair() { return LY<TR>::NSLOT / 2; }
// weight fragments are read PF tiles ahead of their MFMAs (a ring of PF + 1 fragment pairs that
// runs on across steps and layers): 2 in the training forward (3 measured no faster,
// profiles/r05/chain_variants_ab.txt), 3 in the eval kernel.  NERF_CHAIN_PF_EVAL (diagnostic
// builds) sets the eval depth; the ring holds at most PF_MAX + 1 entries (State::wh / wl), and a
// step of 8 tiles must keep its barrier tile tb >= 0 (static_asserts below): round 5's PF 4
// eval build indexed wh[4] of a 4-entry ring -- a register array read out of bounds, hence
// its non-finite frame (profiles/r06/pf_eval4.txt)
#ifndef NERF_CHAIN_PF_EVAL
#define NERF_CHAIN_PF_EVAL 3
#endif
template <bool TR>
constexpr int pf_tiles() { return TR ? 2 : NERF_CHAIN_PF_EVAL; }
constexpr int PF_BWD = 3;                   // the input-gradient chain (b2::PF; 2 measured no change)
constexpr int PF_MAX = 4;                   // fragment-ring entries - 1 (State::wh / wl)
static_assert(pf_tiles<true>() >= 1 && pf_tiles<true>() <= PF_MAX && pf_tiles<false>() >= 1 &&
                  pf_tiles<false>() <= PF_MAX && PF_BWD <= PF_MAX,
              "the weight-fragment ring holds PF_MAX + 1 entries");
constexpr int ntj_k(int k) { return L_OUT[layer_of_k(k)] / 16; }
// step -> first global tile and tile -> step, tabulated once (the templates ask per tile)
struct TileMap {
    int first[NK + 1];
    int step[16 * NK];
    constexpr TileMap() : first{}, step{} {
        int g = 0;
        for (int k = 0; k < NK; ++k) {
            first[k] = g;
            for (int j = 0; j < ntj_k(k); ++j) step[g + j] = k;
            g += ntj_k(k);
        }
        first[NK] = g;
    }
};
constexpr TileMap kTiles{};
constexpr int gtile(int k) { return kTiles.first[k]; }
constexpr int NG = gtile(NK);               // MFMA tiles of the chain
constexpr int step_of_tile(int G) { return kTiles.step[G]; }
// the tile of step k behind whose MFMAs (and save pieces) the wave waits, passes B_{k+1} and
// issues DMAs: the last tile before the first read of step k + 1's fragments
template <bool TR>
constexpr int tb(int k) { return ntj_k(k) - pf_tiles<TR>() - 1; }
// every step's barrier tile exists (the 8-tile colour-layer steps bound PF at 6), and in the
// training forward the save stores (issued no later than tb: piece_tile) precede it
constexpr bool tb_ok() {
    for (int k = 0; k < NK; ++k)
        if (tb<true>(k) < 0 || tb<false>(k) < 0) return false;
    return true;
}
static_assert(tb_ok(), "a step's barrier tile tb = ntj - PF - 1 must exist");
// vector-memory ops of the DMAs of 32-k step m (two 16-k steps), and of those issued in step j
constexpr int dma_step(int m) { return m >= NK ? 0 : dma_count(tt_of_k(m)) + dma_count(tt_of_k(m) + 1); }
template <bool TR>
constexpr int dma_in(int j) { return dma_step(j + npair<TR>() - 1); }
// training, layer l >= 1, step u: the previous layer's output is saved two float4 stores per
// tile pair (pairs 0 and 1 at u = 0, pair u + 1 at u = 1..6); at u = 0 of l >= 2 layer l - 2's
// column maxima and ReLU words leave LDS (one store each).  All before the step's barrier
template <bool TR>
constexpr int pre_st(int k) {
    const int l = layer_of_k(k), u = k - kfirst(l);
    if (!TR || l == 0) return 0;
    return u == 0 ? 4 + (l >= 2 ? 2 : 0) : (u <= 6 ? 2 : 0);
}
// the counted wait before B_{k+1} (at tile tb(k) of step k) for the DMAs of step k + 1, issued
// behind B_{k + 3 - NPAIR} in step j0 = k + 2 - NPAIR (the prologue when negative): vmcnt counts
// loads, stores and LDS-DMA together in issue order, so the count is every vector-memory op the
// wave issued after them.  Ops left out of the count only make a wait stricter
template <bool TR>
constexpr int wait_n(int k) {
    constexpr int P = npair<TR>();
    const int j0 = k + 2 - P;
    int n = 0;
    if (j0 < 0)
        for (int m = k + 2; m <= P - 2; ++m) n += dma_step(m);
    for (int j = (j0 + 1 > 0 ? j0 + 1 : 0); j < k; ++j) n += pre_st<TR>(j) + dma_in<TR>(j);
    return n + pre_st<TR>(k);
}
// the prologue's wait for step 0 (it issues the DMAs of steps 0 .. NPAIR - 2)
template <bool TR>
constexpr int wait_prologue() {
    int n = 0;
    for (int m = 1; m <= npair<TR>() - 2; ++m) n += dma_step(m);
    return n;
}
static_assert(wait_n<true>(0) == dma_step(2) && wait_n<true>(1) == dma_in<true>(0), "training waits");
static_assert(wait_n<true>(5) == pre_st<true>(4) + dma_in<true>(4) + pre_st<true>(5), "training waits");
static_assert(wait_n<false>(0) == 0 && wait_n<false>(7) == 0, "eval waits");

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float pf2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x4 mfma16(const uint4& w, const uint4& a, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(ch16x8, w), __builtin_bit_cast(ch16x8, a), c,
                                                  0, 0, 0);
}
// pins a value's computation here (the compiler may not sink it past the LDS-DMA issue)
__device__ __forceinline__ void opaque(uint4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }
// OR over the four 16-lane rows
__device__ __forceinline__ uint32_t rows_or(uint32_t v) {
    const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    const uint32_t r = a[0] | a[1];
    const auto b = __builtin_amdgcn_permlane32_swap(r, r, false, false);
    return b[0] | b[1];
}
// max / sum over the four 16-lane rows (lanes n, n + 16, n + 32, n + 48) by permlane swaps: no
// ds_bpermute and no lane-address registers (which the compiler would keep -- or spill --
// across the chain).  rows_max takes non-negative floats (ordered as their bits)
__device__ __forceinline__ float rows_max(float v) {
    const uint32_t x = __float_as_uint(v);
    const auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    const uint32_t r = max((uint32_t)a[0], (uint32_t)a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(r, r, false, false);
    return __uint_as_float(max((uint32_t)b[0], (uint32_t)b[1]));
}
__device__ __forceinline__ float rows_sum(float v) {
    const uint32_t x = __float_as_uint(v);
    const auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    const float r = __uint_as_float(a[0]) + __uint_as_float(a[1]);   // own + the partner row's, as a shuffle sum
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(r), __float_as_uint(r), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
// max(m, |a|, |b|) in one v_max3_f32 with |.| source modifiers (the compiler forms ~2.3
// instructions per value from fmaxf / fabsf chains); max is exact, so the same bits
__device__ __forceinline__ float max3abs(float m, float a, float b) {
    float r;
    asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}
// a fresh copy of a lane value the compiler may not keep live (or spill) across the chain:
// derived addresses are rebuilt from it where they are used
__device__ __forceinline__ int fresh(int v) {
    asm volatile("" : "+v"(v));
    return v;
}
// the chains' row exponent: row_exp capped at 127 so that 2^e is an f32 (rows below 2^-113
// keep a smaller scale; nothing overflows)
__device__ __forceinline__ int chain_exp(float m) {
    const int e = row_exp(m);
    return e > 127 ? 127 : e;
}

// fp16 pair words of (x0, x1) at scale s = 2^e (exact): hi = RNE(x s) per half (two
// v_fma_mix{lo,hi}_f16 x s + 0), lo = RNE(x s - hi) (x s - hi is exact in f32; the fp16 half
// of hi is read in place) -- the bits of ldexp + v_cvt_pk_f16_f32 + residual + convert at half
// the VALU
__device__ __forceinline__ uint32_t mhi(float x0, float x1, float s) {
    uint32_t h;
    asm("v_fma_mixlo_f16 %0, %1, %2, 0\n\t"
        "v_fma_mixhi_f16 %0, %3, %2, 0"
        : "=&v"(h) : "v"(x0), "v"(s), "v"(x1));
    return h;
}
__device__ __forceinline__ uint32_t mlo(float x0, float x1, float s, uint32_t h) {
    uint32_t l;
    asm("v_fma_mixlo_f16 %0, %1, %2, -%4 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %0, %3, %2, -%4 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(l) : "v"(x0), "v"(s), "v"(x1), "v"(h));
    return l;
}
// 16 bytes per lane from (g + voff) into LDS at lds + 16 lane; g and lds wave-uniform (SGPRs:
// the address arithmetic is scalar), voff the lane's 16-byte offset
// (the nt hint on these loads made both training chains ~20 % slower, profiles/r05/nt_loads_ab.txt)
__device__ __forceinline__ void dma16(const void* g, uint32_t voff, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(g), "s"(lds) : "memory", "m0");
}

struct State {
    char* lds;
    uint32_t lds0;                      // LDS address of the block's buffer (wave-uniform)
    float* fx;
    int tid, wave, lane, n, g;          // n = lane & 15 (the lane's sample in the wave), g = lane >> 4
    size_t m0;
    int rl;                             // the lane's row in the block (16 wave + n)
    uint32_t voff16;                    // 16 lane: the lane's offset in a 16-byte-per-lane LDS-DMA
    int vrow;                           // (rl 256 + 4 g) 4: the lane's byte offset in a [128][256] f32 tile
    int er;                             // row exponent of the current A operand
    float ser;                          // 2^er
    uint32_t mk0, mk1;                  // training: the colour layer's ReLU words
    u16x2 rk0, rk1;                     // ReLU-bit weights {1, 2} << 4 g, {4, 8} << 4 g (relu_word)
    unsigned long long t_wait, t_bar, t_epi, t_pro, t_last, t_start;   // diagnostics (stamps): cycles in the
                                                       // k-step waits, barriers, layer epilogues, prologue
    int fr;                             // the lane's weight-fragment offset in a ring slot pair: slot
                                        // g >> 1 of the pair, k-half g & 1, image row n (+ 16 j per tile)
    uint4 act_hi[8], act_lo[8];         // A operand: 8 k-steps of 32 (the 256 activations)
    uint4 enc_hi[2], enc_lo[2];         // encoding segment (64 columns) of the current layer
    f32x4 acc[16];                      // 16 rows x 256 outputs
    f32x4 xs[16];                       // the previous epilogue's outputs (tile layout), split into act
                                        // and saved during the next layer's k-steps
    uint4 wh[PF_MAX + 1], wl[PF_MAX + 1];   // weight-fragment ring (hi / lo planes), PF + 1 tiles
};

// diagnostics (nerf_chain_debug_stamps, NERF_CHAIN_STAMPS builds): cycles since the last tick
__device__ __forceinline__ void tick(const ChainFwdArgs& p, State& st, unsigned long long* bucket) {
    if constexpr (NERF_CHAIN_STAMPS) {
        if (p.stamps == nullptr) return;
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        if (bucket) *bucket += t - st.t_last;
        st.t_last = t;
        __builtin_amdgcn_sched_barrier(0);
    }
}

// per block (wave 0): k-step waits, barriers, prologue, layer epilogues, total, and the tail
// (from the last epilogue to here)
__device__ __forceinline__ void write_stamps(const ChainFwdArgs& p, State& st) {
    if constexpr (NERF_CHAIN_STAMPS) {
        if (p.stamps && threadIdx.x == 0) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            unsigned long long* o = p.stamps + (size_t)blockIdx.x * 6;
            o[0] = st.t_wait; o[1] = st.t_bar; o[2] = st.t_pro; o[3] = st.t_epi;
            o[4] = t - st.t_start; o[5] = t - st.t_last;
        }
    }
}

// global 16-k step TT -> ring slot TT % NSLOT (2 pieces per wave; 1 for the 128-row colour
// layer) + at a layer's first step one piece per wave: waves 0-3 the weight-row exponents
// (64 image rows each), waves 4-7 the biases (16 lanes x 4 floats each); the 128-wide layer's
// extra waves repeat the first ones (same bytes to the same place), so every wave issues the
// same count (its vmcnt waits are compile-time).  A wave's piece is 64 consecutive image rows
// of one plane and k-half: everything but the lane's 16-byte offset is wave-uniform
template <int TT, bool TR>
__device__ __forceinline__ void dma(const ChainFwdArgs& p, State& st) {
    using Y = LY<TR>;
    if constexpr (TT < CT) {
        constexpr int l = layer_of(TT);
        constexpr int s = TT - kbase(l);
        constexpr int ks = L_KS[l];
        constexpr int NO = L_OUT[l];
        const nerf_chain_layer& L = p.L[l];
        const char* img = reinterpret_cast<const char*>(L.img);
        const uint32_t slot = st.lds0 + Y::O_RING + (TT % Y::NSLOT) * SBYTES;
#pragma unroll
        for (int i = 0; i < (NO == 256 ? 2 : 1); ++i) {
            const int ph = NO == 256 ? (st.wave >> 2) + 2 * i : (st.wave >> 1);   // plane * 2 + k-half
            const int n0 = NO == 256 ? 64 * (st.wave & 3) : 64 * (st.wave & 1);   // first image row
            const int chunk = (ph >> 1) * (2 * ks) + 2 * s + (ph & 1);
            dma16(img + (chunk * NO + n0) * 16, st.voff16, slot + ph * SHALF + n0 * 16);
        }
        if constexpr (s == 0) {
            if (st.wave < 4) {
                // the layer's weight-row exponents: the compact int array of the chain image
                // (plane 2, chunk 1), 1 KB, the same bytes from each of waves 0-3 (one vmcnt op
                // per wave); 128-row layers take the first 512 B of it
                dma16(img + ((2 * (2 * ks) + 1) * NO) * 16, st.voff16, st.lds0 + Y::O_LEB + (l & 1) * 1024);
            } else if (st.lane < 16) {                   // one instruction, lanes 0-15 active
                const int wb = NO == 256 ? st.wave - 4 : ((st.wave - 4) & 1);
                dma16(reinterpret_cast<const char*>(L.bias) + 64 * wb * 4, st.voff16,
                      st.lds0 + Y::O_BIAS + ((l & 1) * 256 + 64 * wb) * 4);
            } else {
                // the other lanes of the bias instruction: masked off (the instruction is one
                // vmcnt op for the wave either way)
            }
        }
    }
}

template <int T0, int N, bool TR>
__device__ __forceinline__ void dma_n(const ChainFwdArgs& p, State& st) {
    if constexpr (N > 0) {
        dma<T0, TR>(p, st);
        dma_n<T0 + 1, N - 1, TR>(p, st);
    }
}

// the 8 consecutive encoding columns 32 t + 8 g .. + 7 of a row (the encoding segments of the
// chain images keep their natural column order) at scale s -> fragment planes
__device__ __forceinline__ void enc_frag(const float* row, int t, int g, float s, uint4& hi, uint4& lo) {
    const float4* src = reinterpret_cast<const float4*>(row + 32 * t + 8 * g);
    const float4 a = src[0], b = src[1];
    hi = make_uint4(mhi(a.x, a.y, s), mhi(a.z, a.w, s), mhi(b.x, b.y, s), mhi(b.z, b.w, s));
    lo = make_uint4(mlo(a.x, a.y, s, hi.x), mlo(a.z, a.w, s, hi.y), mlo(b.x, b.y, s, hi.z), mlo(b.z, b.w, s, hi.w));
}

// the eval kernel's encoding tile in LDS ([128 rows][64] floats): row's float4 chunk q at
// q ^ (row & 15), so the prologue's per-row scalar writes (64 consecutive rows per instruction,
// 256 bytes apart) spread over the banks instead of all landing on one, and a 16-lane group of
// enc_frag_lds's 16-byte reads (16 rows) covers 16 distinct chunks
__device__ __forceinline__ int enc_swz(int row, int k) { return (((k >> 2) ^ (row & 15)) << 2) | (k & 3); }
__device__ __forceinline__ void enc_frag_lds(const float* tile, int rl, int t, int g, float s, uint4& hi, uint4& lo) {
    const float* row = tile + rl * 64;
    const int c0 = 8 * t + 2 * g, sw = rl & 15;
    const float4 a = *reinterpret_cast<const float4*>(row + 4 * (c0 ^ sw));
    const float4 b = *reinterpret_cast<const float4*>(row + 4 * ((c0 + 1) ^ sw));
    hi = make_uint4(mhi(a.x, a.y, s), mhi(a.z, a.w, s), mhi(b.x, b.y, s), mhi(b.z, b.w, s));
    lo = make_uint4(mlo(a.x, a.y, s, hi.x), mlo(a.z, a.w, s, hi.y), mlo(b.x, b.y, s, hi.z), mlo(b.z, b.w, s, hi.w));
}

// k-step t's A fragment from tiles 2t, 2t + 1 of xs, in two halves (hi words, lo words)
template <int t>
__device__ __forceinline__ void split_hi(State& st) {
    const f32x4 A = st.xs[2 * t], B = st.xs[2 * t + 1];
    const float s = st.ser;
    st.act_hi[t] = make_uint4(mhi(A[0], A[1], s), mhi(A[2], A[3], s), mhi(B[0], B[1], s), mhi(B[2], B[3], s));
}
template <int t>
__device__ __forceinline__ void split_lo(State& st) {
    const f32x4 A = st.xs[2 * t], B = st.xs[2 * t + 1];
    const float s = st.ser;
    const uint4 h = st.act_hi[t];
    st.act_lo[t] = make_uint4(mlo(A[0], A[1], s, h.x), mlo(A[2], A[3], s, h.y), mlo(B[0], B[1], s, h.z),
                              mlo(B[2], B[3], s, h.w));
}

typedef unsigned cu32x4 __attribute__((ext_vector_type(4)));
// the training chains' saved-output stores are non-temporal (cache-policy bits 2): forward
// chain 525-536 vs 550-554 us, input-gradient chain 493-498 vs 507-510 us, cfg2 step 1.999 vs
// 2.047 ms in three interleaved rounds (profiles/r05/chain_nt_ab.txt) -- the 1.3 GB each chain
// writes no longer displaces the weight stream every block re-reads
constexpr int ST_POL = 2;
// a float4 into a row-major [128 rows][W] f32 tile of one block through a buffer resource: the
// lane's row / column byte offset in one VGPR, the block base in SGPRs, the column offset an
// immediate -- no 64-bit per-lane address arithmetic per store
template <int W>
__device__ __forceinline__ void tile_store4(float* block_base, int voff, int imm_bytes, const f32x4& x) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)block_base, (short)0, 128 * W * 4, 0x00020000);
    const cu32x4 v = {__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]), __float_as_uint(x[3])};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, imm_bytes, ST_POL);
}

// column maxima of tile x's four features over the wave's 16 rows: max |x| over the lane
// quad by two v_max_f32_dpp steps with |.| source modifiers (non-negative floats order as
// their bits), the quads combined by two row_ror steps, then one LDS atomic max per row
// leader (lane n == 0) -- against one atomic per quad: forward chain 556-558 vs 563-565 us,
// input-gradient chain 504 vs 510 us, cfg2 step 2.076 vs 2.091 ms in three interleaved rounds
// (profiles/r05/colmax_row_ab.txt).  The asm keeps the DPP hazard explicit (a DPP source
// written by VALU needs two wait states: the s_nop; the later steps' sources are four
// instructions old) and the maxima out of the leaders' branch
template <int Q = 1>
__device__ __forceinline__ void colmax4(const f32x4& x, uint32_t* cm, bool leader) {
    float a0, a1, a2, a3;
    asm volatile(
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, |%4|, |%4| quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_max_f32_dpp %1, |%5|, |%5| quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_max_f32_dpp %2, |%6|, |%6| quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_max_f32_dpp %3, |%7|, |%7| quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_max_f32_dpp %1, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_max_f32_dpp %2, %2, %2 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_max_f32_dpp %3, %3, %3 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf"
        : "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3)
        : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]));
    if constexpr (Q == 2) {
        asm volatile(
            "v_max_f32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
            "v_max_f32_dpp %1, %1, %1 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
            "v_max_f32_dpp %2, %2, %2 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
            "v_max_f32_dpp %3, %3, %3 row_ror:4 row_mask:0xf bank_mask:0xf"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    }
    if constexpr (Q == 1) {
        // the max over all 16 lanes of the row (quads combined by row_ror 4, 8): one atomic per
        // row and feature, no address conflicts
        asm volatile(
            "v_max_f32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
            "v_max_f32_dpp %1, %1, %1 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
            "v_max_f32_dpp %2, %2, %2 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
            "v_max_f32_dpp %3, %3, %3 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
            "v_max_f32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
            "v_max_f32_dpp %1, %1, %1 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
            "v_max_f32_dpp %2, %2, %2 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
            "v_max_f32_dpp %3, %3, %3 row_ror:8 row_mask:0xf bank_mask:0xf"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    }
    if (leader) {
        atomicMax(cm + 0, __float_as_uint(a0));
        atomicMax(cm + 1, __float_as_uint(a1));
        atomicMax(cm + 2, __float_as_uint(a2));
        atomicMax(cm + 3, __float_as_uint(a3));
    }
}

// the lane's ReLU bits of k-step t (features 32 t + 4 g + c -> bit 4 g + c, 32 t + 16 + 4 g +
// c -> bit 16 + 4 g + c of word t) from the fp16 hi words of the pair: a value is kept by the
// ReLU iff its hi half is non-zero (x >= +0, and hi = 0 exactly when x 2^e < 2^-25, i.e. when
// the pair is (0, 0): the value the next layer consumed) -- v_pk_min_u16 gives two bits per
// word, v_dot2_u32_u16 places them
__device__ __forceinline__ uint32_t relu_word(const uint4& h, const State& st) {
    uint32_t m0, m1, m2, m3;   // v_pk_min_u16 (the compiler would form min(x, 1) by compare + select)
    asm("v_pk_min_u16 %0, %4, 1 op_sel_hi:[1,0]\n\t"
        "v_pk_min_u16 %1, %5, 1 op_sel_hi:[1,0]\n\t"
        "v_pk_min_u16 %2, %6, 1 op_sel_hi:[1,0]\n\t"
        "v_pk_min_u16 %3, %7, 1 op_sel_hi:[1,0]"
        : "=v"(m0), "=v"(m1), "=v"(m2), "=v"(m3) : "v"(h.x), "v"(h.y), "v"(h.z), "v"(h.w));
    const u16x2 b0 = __builtin_bit_cast(u16x2, m0), b1 = __builtin_bit_cast(u16x2, m1);
    const u16x2 b2 = __builtin_bit_cast(u16x2, m2), b3 = __builtin_bit_cast(u16x2, m3);
    const uint32_t lo = __builtin_amdgcn_udot2(b1, st.rk1, __builtin_amdgcn_udot2(b0, st.rk0, 0u, false), false);
    const uint32_t hi = __builtin_amdgcn_udot2(b3, st.rk1, __builtin_amdgcn_udot2(b2, st.rk0, 0u, false), false);
    return lo | (hi << 16);
}

// a row's ReLU word of k-step t into LDS: an atomic OR from each of the row's four lanes (the
// OR over the four 16-lane rows by permlane swaps and one plain store per row was slower:
// forward chain 557-559 vs 546-550 us, profiles/r05/chain_variants_ab.txt)
__device__ __forceinline__ void relu_put(uint32_t* a, uint32_t w, const State&) {
    atomicOr(a, w);
}

// Save pieces of the training kernels: tile pair t of xs (the previous epilogue's values,
// features 32 t .. 32 t + 31) -- two float4 stores, the column maxima of each tile, the ReLU
// word -- spread over the MFMA tiles of a k-step.  The placement (tile of each piece) for a
// k-step of ntj tiles: pair 0 rides on k-step 0's first tiles, pair u + 1 on k-step u's later
// tiles, behind its split (which it shares the xs registers with)
enum Piece { P_SPLIT_HI_A, P_SPLIT_HI_B, P_SPLIT_LO_A, P_SPLIT_LO_B, P_STORE, P_CMAX_A, P_CMAX_B, P_RELU,
             P0_STORE, P0_CMAX_A, P0_CMAX_B, P0_RELU, P_STORE_B, P0_STORE_B };
// the second 16-k step's DMAs one tile after the barrier tile (two tiles: within noise; the two
// stores of a pair on different tiles: +10 us per chain, profiles/r06/chain_store_dma_spread_ab.txt)
constexpr int DMA2 = 1;
// (a staggered table for waves 4-7, their pieces at the tiles waves 0-3 leave free, ran 4 %
// slower: profiles/r05/chain_variants_ab.txt)
template <int ntj>
constexpr int piece_tile(int piece) {
    if constexpr (ntj == 16) {
        constexpr int T[14] = {6, 7, 8, 9, 10, 11, 12, 13, 1, 2, 3, 4, 10, 1};
        return T[piece];
    } else {
        constexpr int T[14] = {3, 3, 4, 4, 5, 6, 7, 7, 0, 1, 2, 2, 5, 0};
        return T[piece];
    }
}
// the pieces that store (vector memory) run no later than the tile of the step's barrier, tb =
// ntj - PF - 1 (the wait counts take every store of a step as issued before it): PF 2 in the
// training forward (16- and 8-tile steps), 3 in the backward (16)
static_assert(piece_tile<16>(P_STORE) <= 16 - 3 - 1 && piece_tile<16>(P0_STORE) <= 16 - 3 - 1 &&
                  piece_tile<8>(P_STORE) <= 8 - 2 - 1 && piece_tile<8>(P0_STORE) <= 8 - 2 - 1 &&
                  piece_tile<16>(P_STORE_B) <= 16 - 3 - 1 && piece_tile<16>(P0_STORE_B) <= 16 - 3 - 1 &&
                  piece_tile<8>(P_STORE_B) <= 8 - 2 - 1 && piece_tile<8>(P0_STORE_B) <= 8 - 2 - 1,
              "stores before the barrier");
// training: the save work of layer l's k-step u (the previous layer's output, P = p.L[l - 1]),
// piece j of ntj
template <int l, int u, int j, int ntj>
__device__ __forceinline__ void save_pieces(const ChainFwdArgs& p, State& st) {
    using Y = LY<true>;
    if constexpr (l >= 1 && u < 8) {
        const nerf_chain_layer& P = p.L[l - 1];
        constexpr bool relu = l - 1 != 8;           // lf has no ReLU
        constexpr int par = (l - 1) & 1;
        // a per-piece opaque copy of the lane's LDS offsets (the compiler would otherwise keep
        // every piece's address live across the chain)
        // (the LDS offsets of the arrays are beyond a ds_* immediate: they ride in the base)
        constexpr int Q = CMQ_FWD;
        auto cm_at = [&](int t, int half) {
            int o = Y::O_CMX + 16 * st.g + (Q == 1 ? 0 : 4 * CMS * (st.n >> (Q == 2 ? 3 : 2)));
            asm volatile("" : "+v"(o));
            return reinterpret_cast<uint32_t*>(st.lds + o) + par * 256 + 32 * t + 16 * half;
        };
        auto msk_at = [&](int t) {
            int o = Y::O_MSK + 4 * MSKW * st.rl;
            asm volatile("" : "+v"(o));
            return reinterpret_cast<uint32_t*>(st.lds + o) + par * 128 * MSKW + t;
        };
        const bool leader = (st.n & (16 / Q - 1)) == 0;
        float* ob = P.out + st.m0 * 256;
        constexpr bool CM = true, RW = relu, SV = true;
        if constexpr (u == 0) {
            if constexpr (SV && j == piece_tile<ntj>(P0_STORE)) tile_store4<256>(ob, st.vrow, 0, st.xs[0]);
            if constexpr (SV && j == piece_tile<ntj>(P0_STORE_B)) tile_store4<256>(ob, st.vrow, 64, st.xs[1]);
            if constexpr (CM && j == piece_tile<ntj>(P0_CMAX_A)) colmax4<Q>(st.xs[0], cm_at(0, 0), leader);
            if constexpr (CM && j == piece_tile<ntj>(P0_CMAX_B)) colmax4<Q>(st.xs[1], cm_at(0, 1), leader);
            if constexpr (RW && j == piece_tile<ntj>(P0_RELU)) relu_put(msk_at(0), relu_word(st.act_hi[0], st), st);
        }
        if constexpr (u + 1 < 8) {
            constexpr int t = u + 1;
            if constexpr (SV && j == piece_tile<ntj>(P_STORE)) tile_store4<256>(ob, st.vrow, 128 * t, st.xs[2 * t]);
            if constexpr (SV && j == piece_tile<ntj>(P_STORE_B))
                tile_store4<256>(ob, st.vrow, 128 * t + 64, st.xs[2 * t + 1]);
            if constexpr (CM && j == piece_tile<ntj>(P_CMAX_A)) colmax4<Q>(st.xs[2 * t], cm_at(t, 0), leader);
            if constexpr (CM && j == piece_tile<ntj>(P_CMAX_B)) colmax4<Q>(st.xs[2 * t + 1], cm_at(t, 1), leader);
            if constexpr (RW && j == piece_tile<ntj>(P_RELU)) relu_put(msk_at(t), relu_word(st.act_hi[t], st), st);
        }
    }
}

// the next k-step's A fragment (tiles 2 (u + 1), 2 (u + 1) + 1 of the previous epilogue), in
// four pieces
template <int l, int u, int j, int ntj>
__device__ __forceinline__ void split_pieces(State& st) {
    if constexpr (l > 0 && u + 1 < 8) {
        constexpr int t = u + 1;
        const f32x4 A = st.xs[2 * t], B = st.xs[2 * t + 1];
        const float s = st.ser;
        if constexpr (j == piece_tile<ntj>(P_SPLIT_HI_A)) {
            st.act_hi[t].x = mhi(A[0], A[1], s);
            st.act_hi[t].y = mhi(A[2], A[3], s);
        }
        if constexpr (j == piece_tile<ntj>(P_SPLIT_HI_B)) {
            st.act_hi[t].z = mhi(B[0], B[1], s);
            st.act_hi[t].w = mhi(B[2], B[3], s);
        }
        if constexpr (j == piece_tile<ntj>(P_SPLIT_LO_A)) {
            st.act_lo[t].x = mlo(A[0], A[1], s, st.act_hi[t].x);
            st.act_lo[t].y = mlo(A[2], A[3], s, st.act_hi[t].y);
        }
        if constexpr (j == piece_tile<ntj>(P_SPLIT_LO_B)) {
            st.act_lo[t].z = mlo(B[0], B[1], s, st.act_hi[t].z);
            st.act_lo[t].w = mlo(B[2], B[3], s, st.act_hi[t].w);
        }
    }
}

// global tile G's weight fragments (hi, lo) into ring entry G % (PF + 1): lane (g, n) reads
// k-chunk g -- slot g >> 1 of the step's pair, k-half g & 1, image row 16 j + n -- one
// ds_read_b128 per plane from the lane's base (two bases: slot pairs 0-1 and 2-3 of the ring)
// with the rest an immediate offset
template <int G, bool TR>
__device__ __forceinline__ void frag_read(State& st) {
    if constexpr (G < NG) {
        using Y = LY<TR>;
        constexpr int R = pf_tiles<TR>() + 1;
        constexpr int k = step_of_tile(G), j = G - gtile(k), slot = tt_of_k(k) % Y::NSLOT;
        static_assert(slot % 2 == 0, "a 32-k step's two slots are consecutive");
        constexpr int off = Y::O_RING + (slot & 3) * SBYTES + 256 * j;
        const char* b = st.lds + st.fr + (slot >= 4 ? 4 * SBYTES : 0);
        st.wh[G % R] = *reinterpret_cast<const uint4*>(b + off);
        st.wl[G % R] = *reinterpret_cast<const uint4*>(b + off + SPLANE);
    }
}
template <int G0, int N, bool TR>
__device__ __forceinline__ void frag_reads(State& st) {
    if constexpr (N > 0) {
        frag_read<G0, TR>(st);
        frag_reads<G0 + 1, N - 1, TR>(st);
    }
}

// the work at the start of a layer's first step (behind its first tile's MFMAs): the layer's
// weight-row exponents (landed with the step, published by its barrier) into the compact
// array for the epilogue; training: layer l - 2's column maxima over the block's 128 rows
// (its 128-row group) and its ReLU words, complete since layer l - 1's last step, leave LDS
// -- wave w stores features 32 w .. + 31, lane (g, n) its row's words 2 g, 2 g + 1 -- and are
// cleared for layer l's saves
template <int l, bool TR>
__device__ __forceinline__ void layer_start(const ChainFwdArgs& p, State& st) {
    using Y = LY<TR>;
    const int tid = fresh(st.tid);
    if (tid < L_OUT[l])   // as the scale 2^-e of the weight row (exact)
        reinterpret_cast<float*>(st.lds + Y::O_EXP)[(l & 1) * 256 + tid] = __builtin_amdgcn_ldexpf(
            1.f, -reinterpret_cast<const int*>(st.lds + Y::O_LEB + (l & 1) * 1024)[tid]);
    if constexpr (TR && l >= 2) {
        const int lane = tid & 63;
        if (lane < 32) {
            uint32_t* cm = reinterpret_cast<uint32_t*>(st.lds + Y::O_CMX);
            const int cw = (l & 1) * 256 + 32 * st.wave + lane;
            p.L[l - 2].cmax[(st.m0 / CROWS) * L_OUT[l - 2] + 32 * st.wave + lane] =
                __uint_as_float(cm_read<CMQ_FWD>(cm, cw));
            cm_clear<CMQ_FWD>(cm, cw);
        }
        const int rl = 16 * st.wave + (lane & 15), g = lane >> 4;
        const nerf_chain_layer& Q = p.L[l - 2];
        uint2* mw = reinterpret_cast<uint2*>(st.lds + Y::O_MSK + (l & 1) * 4096 + 32 * rl + 8 * g);
        *reinterpret_cast<uint2*>(Q.mask + (st.m0 + rl) * Q.ldmask + 2 * g) = *mw;
        *mw = make_uint2(0u, 0u);
    }
}

// tile j of 32-k step u of layer l: the read of tile j + PF's fragments, this tile's three
// MFMA products, the pieces placed behind it, and at tile tb the wait, barrier B_{k+1} and the
// DMAs of step k + NPAIR - 1 (one 16-k step at tb, the other at tb + 1)
template <int l, int u, bool TR, int j, int ntj>
__device__ __forceinline__ void mstep_tiles(const ChainFwdArgs& p, State& st, const uint4& ah, const uint4& al) {
    constexpr int PF = pf_tiles<TR>(), R = PF + 1;
    constexpr int k = kfirst(l) + u, G = gtile(k) + j, T = tb<TR>(k);
    if constexpr (j < ntj) {
        // the next layer's first tiles are read after this layer's epilogue (kstep): the ring
        // is not live across the epilogue's registers
        if constexpr (G + PF < NG && layer_of_k(step_of_tile(G + PF)) == l) frag_read<G + PF, TR>(st);
        __builtin_amdgcn_sched_barrier(0);
        st.acc[j] = mfma16(st.wh[G % R], al, st.acc[j]);   // hi . lo
        st.acc[j] = mfma16(st.wl[G % R], ah, st.acc[j]);   // lo . hi
        st.acc[j] = mfma16(st.wh[G % R], ah, st.acc[j]);   // hi . hi
        if constexpr (u == 0 && j == 0) layer_start<l, TR>(p, st);
        split_pieces<l, u, j, ntj>(st);
        if constexpr (TR) save_pieces<l, u, j, ntj>(p, st);
        if constexpr (k + 1 < NK && j == T) {
            tick(p, st, nullptr);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(wait_n<TR>(k)) : "memory");
            tick(p, st, &st.t_wait);
            __syncthreads();
            tick(p, st, &st.t_bar);
            dma<tt_of_k(k + npair<TR>() - 1), TR>(p, st);
        }
        if constexpr (k + 1 < NK && j == T + DMA2) dma<tt_of_k(k + npair<TR>() - 1) + 1, TR>(p, st);
        __builtin_amdgcn_sched_barrier(0);
        mstep_tiles<l, u, TR, j + 1, ntj>(p, st, ah, al);
    }
}

// one 32-k MFMA step u of layer l (16-k steps TT, TT + 1): 16 or 8 feature tiles x 3 products
// over the fragments the ring already holds; the steps from the register tile split the next
// step's A fragment and (training) save the previous layer's output beside the MFMAs
template <int l, int u, bool TR>
__device__ __forceinline__ void kstep(const ChainFwdArgs& p, State& st) {
    constexpr int nact = l == 0 ? 0 : 8;         // k-steps from the register tile, then the encoding
    constexpr int ntj = L_OUT[l] / 16;
    if constexpr (u == 0) frag_reads<gtile(kfirst(l)), pf_tiles<TR>(), TR>(st);   // published by B_k
    const uint4& ah = u < nact ? st.act_hi[u < nact ? u : 0] : st.enc_hi[u < nact ? 0 : u - nact];
    const uint4& al = u < nact ? st.act_lo[u < nact ? u : 0] : st.enc_lo[u < nact ? 0 : u - nact];
    mstep_tiles<l, u, TR, 0, ntj>(p, st, ah, al);
}

template <int l, int u, bool TR>
__device__ __forceinline__ void ksteps(const ChainFwdArgs& p, State& st) {
    if constexpr (2 * u < L_KS[l]) {
        kstep<l, u, TR>(p, st);
        ksteps<l, u + 1, TR>(p, st);
    }
}

// layer l: k-loop, epilogue (feature f = 16 j + 4 g + i of the lane's sample), heads, next A.
// Training: the colour layer stores its f32 output and ReLU words here (no later layer
// consumes it; every other layer's are saved by the next layer's k-steps)
template <int l, bool TR>
__device__ __forceinline__ void layer(const ChainFwdArgs& p, State& st) {
    using Y = LY<TR>;
    constexpr int ntj = L_OUT[l] / 16;
    constexpr bool relu = l != 8;
    constexpr bool head_d = l == 7, head_c = l == CNL - 1;
    constexpr bool last_tr = TR && l == CNL - 1;
#pragma unroll
    for (int j = 0; j < 16; ++j) st.acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    ksteps<l, 0, TR>(p, st);
    tick(p, st, nullptr);
    // the lane's feature offset, opaque per layer: otherwise the exponent / bias addresses of
    // the even (odd) layers are computed once and kept live -- spilled -- across the chain
    int g4 = 4 * st.g;
    asm volatile("" : "+v"(g4));
    const float* le = reinterpret_cast<const float*>(st.lds + Y::O_EXP) + (l & 1) * 256 + g4;
    const float* lb = reinterpret_cast<const float*>(st.lds + Y::O_BIAS) + (l & 1) * 256 + g4;
    // unscale as (acc 2^-er) 2^-ew + b on packed-f32 ops: both scalings exact (powers of two
    // in range), one rounding, as ldexp(acc, -(er + ew)) + b
    const float sr = __builtin_amdgcn_ldexpf(1.f, -st.er);
    const pf2 sr2 = {sr, sr};
    float rmx = 0.f, rmx1 = 0.f, hs0 = 0.f, hs1 = 0.f, hs2 = 0.f;
    uint32_t mw = 0;
#pragma unroll
    for (int j = 0; j < ntj; ++j) {
        // one tile at a time: the barrier keeps the exponent / bias / head-weight reads from
        // being hoisted into one register burst (two waves per SIMD leave 256 registers)
        __builtin_amdgcn_sched_barrier(0);
        const int f0 = 16 * j + g4;
        const float4 s4 = *reinterpret_cast<const float4*>(le + 16 * j);
        const float4 b4 = *reinterpret_cast<const float4*>(lb + 16 * j);
        const pf2 x01 = __builtin_elementwise_fma(pf2{st.acc[j][0], st.acc[j][1]} * sr2, pf2{s4.x, s4.y},
                                                  pf2{b4.x, b4.y});
        const pf2 x23 = __builtin_elementwise_fma(pf2{st.acc[j][2], st.acc[j][3]} * sr2, pf2{s4.z, s4.w},
                                                  pf2{b4.z, b4.w});
        f32x4 x;
        x[0] = x01[0]; x[1] = x01[1]; x[2] = x23[0]; x[3] = x23[1];
        if (relu) {   // as an integer max: every non-positive value (-0 included) becomes +0
#pragma unroll
            for (int c = 0; c < 4; ++c) x[c] = __int_as_float(max(__float_as_int(x[c]), 0));
        }
        st.xs[j] = x;
        {   // v_max3 with |.| operands, two accumulators (even / odd tiles): half the dependent chain
            // (forward chain -2 us, eval -0.17 ms per frame: profiles/r06/max3_ab.txt)
            float& r = (j & 1) ? rmx1 : rmx;
            r = max3abs(max3abs(r, x[0], x[1]), x[2], x[3]);
        }
        if constexpr (last_tr) {   // hr (the f32 epilogue value, as the per-layer kernel) and its ReLU words
            const nerf_chain_layer& L = p.L[l];
            tile_store4<128>(L.out + st.m0 * 128, (fresh(st.rl) * 128 + g4) * 4, 64 * j, x);
            mw |= ((x[0] > 0.f ? 1u : 0u) | (x[1] > 0.f ? 2u : 0u) | (x[2] > 0.f ? 4u : 0u) | (x[3] > 0.f ? 8u : 0u))
                  << ((j & 1) * 16 + g4);
            if (j & 1) {
                const uint32_t w = rows_or(mw);          // word j / 2 of the row, in every row of lanes
                if ((j >> 1) & 1) st.mk1 = st.g == (j >> 2) ? w : st.mk1;
                else st.mk0 = st.g == (j >> 2) ? w : st.mk0;
                mw = 0;
            }
        }
        if constexpr (head_d) {              // sigma_raw = fc_density(h8) (official_nerf.py:66)
            const float4 w = *reinterpret_cast<const float4*>(st.fx + FX_WD + f0);
            hs0 += x[0] * w.x + x[1] * w.y + x[2] * w.z + x[3] * w.w;
        }
        if constexpr (head_c) {              // rgb logits = fc_rgb(hr) (official_nerf.py:91)
            const float4 w0 = *reinterpret_cast<const float4*>(st.fx + FX_WC + f0);
            const float4 w1 = *reinterpret_cast<const float4*>(st.fx + FX_WC + 128 + f0);
            const float4 w2 = *reinterpret_cast<const float4*>(st.fx + FX_WC + 256 + f0);
            hs0 += x[0] * w0.x + x[1] * w0.y + x[2] * w0.z + x[3] * w0.w;
            hs1 += x[0] * w1.x + x[1] * w1.y + x[2] * w1.z + x[3] * w1.w;
            hs2 += x[0] * w2.x + x[1] * w2.y + x[2] * w2.z + x[3] * w2.w;
        }
    }
    if constexpr (last_tr) {
        const nerf_chain_layer& L = p.L[l];
        const int rl = fresh(st.rl);
        if (2 * st.g < L_OUT[l] / 32)
            *reinterpret_cast<uint2*>(L.mask + (st.m0 + rl) * L.ldmask + 2 * st.g) = make_uint2(st.mk0, st.mk1);
    }
    // the four 16-lane rows hold one sample's features: reduce across them (lanes n, n + 16,
    // n + 32, n + 48)
    if constexpr (head_d || head_c) {
        float* raw = st.fx + FX_RAW + 4 * st.rl;
        hs0 = rows_sum(hs0);
        if constexpr (head_d) {
            if (st.g == 0) raw[0] = hs0 + p.bd[0];
        } else {
            hs1 = rows_sum(hs1);
            hs2 = rows_sum(hs2);
            if (st.g == 0) {
                raw[1] = hs0 + p.bc[0];
                raw[2] = hs1 + p.bc[1];
                raw[3] = hs2 + p.bc[2];
            }
        }
    }
    if constexpr (l < CNL - 1) {
        // next layer's A operand: row exponent over the row's 256 features (and the encoding
        // the next layer joins), k-step 0's fp16 pairs now, the others during the next layer's
        // k-steps (split_pieces)
        float m = rows_max(fmaxf(rmx, rmx1));
        const float* drec = st.fx + FX_ENCD + ENCD_REC * (st.rl / p.S);
        if constexpr (l == 3) {
            if constexpr (TR) {
                m = fmaxf(m, p.rp[st.m0 + st.rl]);
            } else {
                const float* rp = reinterpret_cast<const float*>(st.lds + Y::O_RMX);
                m = fmaxf(m, fmaxf(fmaxf(rp[st.rl], rp[128 + st.rl]), fmaxf(rp[256 + st.rl], rp[384 + st.rl])));
            }
        }
        if constexpr (l == 8) m = fmaxf(m, TR ? p.rd[st.m0 + st.rl] : drec[32]);
        st.er = chain_exp(m);
        st.ser = __builtin_amdgcn_ldexpf(1.f, st.er);
        split_hi<0>(st);
        split_lo<0>(st);
        if constexpr (l == 3) {   // training: the encodings in HBM
            if constexpr (TR) {
                const float* er_row = p.enc_p + (st.m0 + st.rl) * 64;
                enc_frag(er_row, 0, st.g, st.ser, st.enc_hi[0], st.enc_lo[0]);
                enc_frag(er_row, 1, st.g, st.ser, st.enc_hi[1], st.enc_lo[1]);
            } else {
                const float* tile = reinterpret_cast<const float*>(st.lds + Y::O_ENC);
                enc_frag_lds(tile, st.rl, 0, st.g, st.ser, st.enc_hi[0], st.enc_lo[0]);
                enc_frag_lds(tile, st.rl, 1, st.g, st.ser, st.enc_hi[1], st.enc_lo[1]);
            }
        }
        if constexpr (l == 8) {   // the view-direction encoding (27 columns + zeros)
            enc_frag(TR ? p.enc_d + (st.m0 + st.rl) * 64 : drec, 0, st.g, st.ser, st.enc_hi[0], st.enc_lo[0]);
            st.enc_hi[1] = make_uint4(0u, 0u, 0u, 0u);
            st.enc_lo[1] = make_uint4(0u, 0u, 0u, 0u);
        }
    }
    tick(p, st, &st.t_epi);
}

// prologue: samples (rendering.py:183-198, no jitter) and the position encoding
// (official_nerf.py:61, 99-119) of the block's 128 rows into the LDS tile, four threads per
// row (x and levels 0-2 | 3-5 | 6-7 | 8-9 and the zero pad), with a row max per part and z
// the row's sample depth and point (its ray's origin / direction loaded from HBM)
__device__ __forceinline__ void encode_p_load(const ChainFwdArgs& p, const State& st, float (&x)[3], float& z) {
    const int row = st.tid & 127;
    const size_t g = st.m0 + row;
    x[0] = x[1] = x[2] = 0.f;
    z = 0.f;
    if (g < (size_t)p.R * p.S) {
        const size_t ray = g / (size_t)p.S;
        const int i = (int)(g - ray * (size_t)p.S);
        z = lerp_z(linspace01(i, p.S), p.near_z, p.far_z);
#pragma unroll
        for (int c = 0; c < 3; ++c) x[c] = ray_point(p.po[3 * ray + c], p.pd[3 * ray + c], z);
    }
}
__device__ __forceinline__ void encode_p(const ChainFwdArgs& p, State& st, const float (&x)[3], float z) {
    using Y = LY<false>;
    const int row = st.tid & 127, part = st.tid >> 7;
    float* dst = reinterpret_cast<float*>(st.lds + Y::O_ENC) + row * 64;   // (chunks swizzled: enc_swz)
    float m = 0.f;
    const int lv0 = part == 0 ? 0 : part == 1 ? 3 : part == 2 ? 6 : 8;
    const int lv1 = part == 0 ? 3 : part == 1 ? 6 : part == 2 ? 8 : 10;
    if (part == 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) { dst[enc_swz(row, c)] = x[c]; m = fmaxf(m, fabsf(x[c])); }
        st.fx[FX_Z + row] = z;   // (to HBM in the kernel's tail: a store here would sit in the prologue's vmcnt wait)
    }
    if (part == 3) dst[enc_swz(row, 63)] = 0.f;
    for (int lv = lv0; lv < lv1; ++lv) {
        const float f = (float)(1 << lv);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float sn, cs;
            sincosf(f * x[c], &sn, &cs);
            dst[enc_swz(row, 3 + 6 * lv + c)] = sn;
            dst[enc_swz(row, 6 + 6 * lv + c)] = cs;
            m = fmaxf(m, fmaxf(fabsf(sn), fabsf(cs)));
        }
    }
    reinterpret_cast<float*>(st.lds + Y::O_RMX)[part * 128 + row] = m;
}

// waves 4-7 (the second-dispatched half, the arbitration loser) at s_setprio 1 for the whole
// chain (MI355X_MICROARCH.md "Two waves per SIMD" item 4): -0.5 % per cfg2 step in two
// interleaved library A/Bs (profiles/r05/chain_variants_ab.txt)
template <bool TR>
__device__ __forceinline__ void init_state(State& st, char* smem) {
    st.lds = smem;
    st.lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(clds_t*)smem);
    st.fx = reinterpret_cast<float*>(smem + LY<TR>::O_FX);
    st.tid = threadIdx.x;
    st.wave = __builtin_amdgcn_readfirstlane(st.tid >> 6);
    st.lane = st.tid & 63; st.n = st.lane & 15; st.g = st.lane >> 4;
    st.m0 = (size_t)blockIdx.x * CROWS;
    st.rl = 16 * st.wave + st.n;
    st.voff16 = 16u * st.lane;
    st.vrow = (st.rl * 256 + 4 * st.g) * 4;
    st.fr = (st.g >> 1) * SBYTES + (st.g & 1) * SHALF + st.n * 16;
    st.mk0 = st.mk1 = 0u;
    st.rk0 = u16x2{(unsigned short)(1u << (4 * st.g)), (unsigned short)(2u << (4 * st.g))};
    st.rk1 = u16x2{(unsigned short)(4u << (4 * st.g)), (unsigned short)(8u << (4 * st.g))};
    st.t_wait = st.t_bar = st.t_epi = st.t_pro = 0;
    st.t_last = st.t_start = NERF_CHAIN_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    if (st.wave >= 4) __builtin_amdgcn_s_setprio(1);
}

template <bool TR>
__device__ __forceinline__ void chain_layers(const ChainFwdArgs& p, State& st) {
    layer<0, TR>(p, st);
    layer<1, TR>(p, st);
    layer<2, TR>(p, st);
    layer<3, TR>(p, st);
    layer<4, TR>(p, st);
    layer<5, TR>(p, st);
    layer<6, TR>(p, st);
    layer<7, TR>(p, st);
    layer<8, TR>(p, st);
    layer<9, TR>(p, st);
}

}  // namespace f2

__global__ __launch_bounds__(512, 2) void k_render_fused2(ChainFwdArgs p) {
    using namespace f2;
    using Y = LY<false>;
    __shared__ __attribute__((aligned(16))) char smem[Y::BYTES];
    State st;
    init_state<false>(st, smem);
    // the prologue's HBM loads (head weights, the rows' rays, the view directions) BEFORE the
    // LDS-DMAs: vmcnt retires in issue order, so a load behind the DMAs would wait for them and
    // the encodings' sincos could not overlap the weights' flight
    const float wdv = st.tid < 256 ? p.wd[st.tid] : 0.f;
    const float wcv = st.tid < 384 ? p.wc[st.tid] : 0.f;
    float x[3], z, dv[3];
    encode_p_load(p, st, x, z);
    encd_load(p, st.tid - 256, 256, st.m0, 0, dv);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (st.tid < 256) st.fx[FX_WD + st.tid] = wdv;
    if (st.tid < 384) st.fx[FX_WC + st.tid] = wcv;
    dma_n<0, 2 * (npair<false>() - 1), false>(p, st);   // steps 0 .. NPAIR - 2
    // the samples and both encodings beside the DMAs; the view records on waves 4-7 (the encode_p
    // parts with 6 sincos, not 9): no wave carries 12 sincos more than the others into B_0
    encode_p(p, st, x, z);
    fused_encode_d_rows(p, st.fx, st.tid, 256, 256, st.m0, dv);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(wait_prologue<false>()) : "memory");
    __syncthreads();   // B_0 (and the encodings in LDS)
    {
        const float* rp = reinterpret_cast<const float*>(smem + Y::O_RMX);
        st.er = chain_exp(fmaxf(fmaxf(rp[st.rl], rp[128 + st.rl]), fmaxf(rp[256 + st.rl], rp[384 + st.rl])));
        st.ser = __builtin_amdgcn_ldexpf(1.f, st.er);
        const float* tile = reinterpret_cast<const float*>(smem + Y::O_ENC);
        enc_frag_lds(tile, st.rl, 0, st.g, st.ser, st.enc_hi[0], st.enc_lo[0]);
        enc_frag_lds(tile, st.rl, 1, st.g, st.ser, st.enc_hi[1], st.enc_lo[1]);
    }
    tick(p, st, &st.t_pro);
    chain_layers<false>(p, st);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every DMA landed before the LDS is released
    __syncthreads();   // every row's raw4 in LDS
    {
        const int t = fresh(threadIdx.x);
        const size_t g = (size_t)blockIdx.x * CROWS + t;
        if (t < CROWS && g < (size_t)p.R * p.S) p.z[g] = st.fx[FX_Z + t];
    }
    fused_composite<NTH>(p, st.fx, st.tid, st.m0);
    write_stamps(p, st);
}

// The training forward chain at two waves per SIMD (nerf_mlp_chain_train): the layer walk of
// k_render_fused2 over the encodings nerf_encode_samples wrote (the backward needs them in
// HBM anyway), saving what the per-layer kernels save -- every layer's output, the ReLU
// words, the per-128-row-group column maxima -- and raw4 from the in-epilogue heads.  The
// stores ride beside the MFMAs and are counted in the k-steps' vmcnt waits (wait_n).
__global__ __launch_bounds__(512, 2) void k_mlp_chain_train2(ChainFwdArgs p) {
    using namespace f2;
    using Y = LY<true>;
    __shared__ __attribute__((aligned(16))) char smem[Y::BYTES];
    State st;
    init_state<true>(st, smem);
    // l0's A operand straight from HBM, before any LDS-DMA is in flight (the compiler waits
    // for ordinary loads with vmcnt(0))
    st.er = chain_exp(p.rp[st.m0 + st.rl]);
    st.ser = __builtin_amdgcn_ldexpf(1.f, st.er);
    {
        const float* row = p.enc_p + (st.m0 + st.rl) * 64;
        enc_frag(row, 0, st.g, st.ser, st.enc_hi[0], st.enc_lo[0]);
        enc_frag(row, 1, st.g, st.ser, st.enc_hi[1], st.enc_lo[1]);
        opaque(st.enc_hi[0]); opaque(st.enc_lo[0]); opaque(st.enc_hi[1]); opaque(st.enc_lo[1]);
    }
    if (st.tid < 256) st.fx[FX_WD + st.tid] = p.wd[st.tid];
    for (int e = st.tid; e < 384; e += NTH) st.fx[FX_WC + e] = p.wc[e];
    // both column-max parities (512 words) and both ReLU-word parities (2048 words) cleared
    for (int e = st.tid; e < cm_words(CMQ_FWD); e += NTH) reinterpret_cast<uint32_t*>(smem + Y::O_CMX)[e] = 0u;
    static_assert(2 * 128 * MSKW == 4 * NTH, "one uint4 per thread");
    reinterpret_cast<uint4*>(smem + Y::O_MSK)[st.tid] = make_uint4(0u, 0u, 0u, 0u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    dma_n<0, 2 * (npair<true>() - 1), true>(p, st);   // steps 0 .. NPAIR - 2
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(wait_prologue<true>()) : "memory");
    __syncthreads();   // B_0
    tick(p, st, &st.t_pro);
    chain_layers<true>(p, st);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // every row's raw4 in LDS, lf's column maxima complete
    write_stamps(p, st);
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));   // re-derived here: nothing of the prologue stays live to the end
    const size_t m0 = (size_t)blockIdx.x * CROWS;
    if (tid < CROWS)
        *reinterpret_cast<float4*>(p.raw4 + (m0 + tid) * 4) = *reinterpret_cast<const float4*>(st.fx + FX_RAW + 4 * tid);
    else if (tid < CROWS + 256)
        p.L[8].cmax[(m0 / CROWS) * L_OUT[8] + tid - CROWS] =
            __uint_as_float(cm_read<CMQ_FWD>(reinterpret_cast<const uint32_t*>(smem + Y::O_CMX), (8 & 1) * 256 + tid - CROWS));
}

// ---------------------------------------------------------------------------
// The input-gradient chain (nerf_mlp_chain_bwd): the backward mirror of k_mlp_chain_train2.
// The autograd of official_nerf.py:60-96 under training.py:92 walks the layers from the
// colour layer down; each layer's input gradient dx = dy W (+ the density head's rank-one
// term d sigma_raw x w_density at the feature layer, official_nerf.py:66), masked by the
// ReLU bits of the layer's input, is the next layer's dy.  A block keeps its 128 rows' dy
// resident in registers as row-scaled fp16 pairs through all nine input gradients -- the
// layer loop of k_mlp_chain_train2 with the weight-transpose chain images (rows = input
// features, K in chain_perm order) streaming through the LDS ring -- and saves every dy beside
// the next layer's MFMAs for the weight gradients: the f32 value, per-128-row-group column
// maxima and row maxima.  Against nine input-gradient launches this removes the read of every
// dy (134 MB per 256-wide layer at 1024 x 128 samples), the in-kernel split of every A
// operand, eight launch gaps and k_heads_dyr: the first dy (the colour layer's, dyr) is
// computed in the prologue from graw4, fc_rgb and the colour layer's ReLU words (k_heads_dyr's
// arithmetic, render.hip).
// Layer order i = 0..8: the colour layer (K = 128), lf, l7, ..., l1.  D_i is layer i's A
// operand: D_0 = dyr, D_{i+1} = layer i's output; D_9 (the gradient at l0's output) is
// stored by the last epilogue.
// ---------------------------------------------------------------------------
struct ChainBwdArgs {
    nerf_chain_bwd a;
};

namespace b2 {
using f2::NTH;
using f2::SBYTES;
using f2::SHALF;
using f2::SPLANE;
using f2::piece_tile;
constexpr int NL = 9;
constexpr int KS_[NL] = {8, 16, 16, 16, 16, 16, 16, 16, 16};   // 16-k steps: the layer's output width / 16
constexpr int KPB[NL] = {320, 256, 256, 256, 256, 320, 256, 256, 256};   // W^T image rows (the layer's padded K)
constexpr int kb(int i) { return i == 0 ? 0 : kb(i - 1) + KS_[i - 1]; }
constexpr int CTB = kb(NL);
constexpr int layer_of(int tt) { int i = 0; while (i + 1 < NL && kb(i + 1) <= tt) ++i; return i; }
constexpr bool first_step(int tt) { return tt < CTB && kb(layer_of(tt)) == tt; }
// LDS-DMA instructions per wave at 16-k step tt: 2 ring pieces, +1 at a layer's first step
// (waves 0-3 the weight-row exponents, waves 4-7 the block's ReLU words of the layer input)
constexpr int dma_count(int tt) { return tt >= CTB ? 0 : 2 + (first_step(tt) ? 1 : 0); }
constexpr int NSLOT = 8, NPAIR = NSLOT / 2;   // ring slots (16-k), slot pairs (32-k steps)
constexpr int nks(int i) { return KS_[i] / 2; }
constexpr int kfirst(int i) { return i == 0 ? 0 : kfirst(i - 1) + nks(i - 1); }
constexpr int layer_of_k(int k) { int i = 0; while (i + 1 < NL && kfirst(i + 1) <= k) ++i; return i; }
constexpr int tt_of_k(int k) { return kb(layer_of_k(k)) + 2 * (k - kfirst(layer_of_k(k))); }
constexpr int NK = kfirst(NL);
constexpr int PF = f2::PF_BWD;   // weight fragments read PF tiles ahead of their MFMAs (the ring runs across steps)
constexpr int NG = 16 * NK;                  // MFMA tiles (16 per step)
constexpr int TB = 16 - PF - 1;              // the barrier tile of a step (f2::tb)
constexpr int dma_step(int m) { return m >= NK ? 0 : dma_count(tt_of_k(m)) + dma_count(tt_of_k(m) + 1); }
constexpr int dma_in(int j) { return dma_step(j + NPAIR - 1); }
// stores of step k before its barrier: the D_i pair stores (pairs 0 and 1 at u = 0, pair u + 1
// at u = 1 .. nks - 2), at a layer's first step the previous dy's column maxima; behind its
// DMAs (post): at a layer's last step the epilogue's row-max store
constexpr int pre_st(int k) {
    const int i = layer_of_k(k), u = k - kfirst(i);
    return (u == 0 ? 4 : (u + 1 < nks(i) ? 2 : 0)) + (u == 0 && i >= 1 ? 1 : 0);
}
constexpr int post_st(int k) {
    const int i = layer_of_k(k), u = k - kfirst(i);
    return u == nks(i) - 1 && i < NL - 1 ? 1 : 0;
}
// the counted wait before B_{k+1} for step k + 1's DMAs, issued behind the barrier of step j0 =
// k + 2 - NPAIR (f2::wait_n, plus the post stores)
constexpr int wait_n(int k) {
    const int j0 = k + 2 - NPAIR;
    int n = 0;
    if (j0 < 0)
        for (int m = k + 2; m <= NPAIR - 2; ++m) n += dma_step(m);
    else
        n += post_st(j0);
    for (int j = (j0 + 1 > 0 ? j0 + 1 : 0); j < k; ++j) n += pre_st(j) + dma_in(j) + post_st(j);
    return n + pre_st(k);
}
constexpr int wait_prologue() {
    int n = 0;
    for (int m = 1; m <= NPAIR - 2; ++m) n += dma_step(m);
    return n;
}
static_assert(wait_n(0) == dma_step(2) + pre_st(0) && wait_prologue() == dma_step(1) + dma_step(2), "prologue waits");
static_assert(wait_n(4) == post_st(2) + pre_st(3) + dma_in(3) + post_st(3) + pre_st(4), "waits");
static_assert(f2::piece_tile<16>(f2::P_STORE) <= TB && f2::piece_tile<16>(f2::P0_STORE) <= TB &&
                  f2::piece_tile<16>(f2::P_STORE_B) <= TB && f2::piece_tile<16>(f2::P0_STORE_B) <= TB,
              "stores before B");

constexpr int O_RING = 0;
constexpr int O_LEB = NSLOT * SBYTES;            // [2][256] int weight-row exponents (compact array)
constexpr int O_EXP = O_LEB + 2 * 256 * 4;       // [2][256] float 2^-e of the weight rows
constexpr int O_MASK = O_EXP + 2 * 256 * 4;      // [2][128 rows][8 words] ReLU words of the layer input
constexpr int O_CMX = O_MASK + 2 * 128 * 32;     // [2][256] uint column maxima (LDS atomics)
constexpr int CMQ = f2::CMQ_BWD;                // column-max copies (f2::cm_words)
constexpr int O_FX = O_CMX + f2::cm_words(CMQ) * 4;   // fc_density [256], fc_rgb [3][128]
constexpr int BYTES = O_FX + (256 + 384) * 4;
static_assert(BYTES <= 160 * 1024, "LDS");

struct State : f2::State {
    float gr0;   // d sigma_raw of the lane's row (the feature layer's rank-one term)
};

template <int TT>
__device__ __forceinline__ void dma(const nerf_chain_bwd& p, State& st) {
    if constexpr (TT < CTB) {
        constexpr int i = layer_of(TT);
        constexpr int s = TT - kb(i);
        constexpr int ks = KS_[i];
        const char* img = reinterpret_cast<const char*>(p.wt_img[i]);
        constexpr int rows = KPB[i];   // image rows (checked by the host entry)
        const uint32_t slot = st.lds0 + O_RING + (TT % NSLOT) * SBYTES;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int ph = (st.wave >> 2) + 2 * q;      // plane * 2 + k-half
            const int n0 = 64 * (st.wave & 3);          // first image row of the wave's piece
            const int chunk = (ph >> 1) * (2 * ks) + 2 * s + (ph & 1);
            f2::dma16(img + (chunk * rows + n0) * 16, st.voff16, slot + ph * SHALF + n0 * 16);
        }
        if constexpr (s == 0) {
            if (st.wave < 4 || i == 0) {
                // the weight-row exponents of image rows 0..255 (the layer's input features the
                // chain produces gradients for): the compact int array in plane 2, chunk 1, 1 KB,
                // the same bytes from each of these waves (the colour layer -- its input f has no
                // ReLU -- repeats them on waves 4-7)
                f2::dma16(img + ((2 * (2 * ks) + 1) * rows) * 16, st.voff16, st.lds0 + O_LEB + (i & 1) * 1024);
            } else {
                // the block's ReLU words of the layer input: wave 4 + w rows 32 w .. 32 w + 31
                // (two lanes per row, 16 bytes each)
                const int w = st.wave - 4;
                const int ld = p.ld_in_mask[i];
                const int lane = f2::fresh(st.lane);
                f2::dma16(reinterpret_cast<const char*>(p.in_mask[i] + (st.m0 + 32 * w) * ld),
                          (uint32_t)(((lane >> 1) * ld + 4 * (lane & 1)) * 4),
                          st.lds0 + O_MASK + (i & 1) * 4096 + 32 * w * 32);
            }
        }
    }
}
template <int T0, int N>
__device__ __forceinline__ void dma_n(const nerf_chain_bwd& p, State& st) {
    if constexpr (N > 0) {
        dma<T0>(p, st);
        dma_n<T0 + 1, N - 1>(p, st);
    }
}

// D_i's save work at layer i's k-step u, piece j: pair stores and the column maxima (parity
// i & 1) of tiles 2t, 2t + 1 (pair 0 and 1 at u = 0, pair u + 1 later)
template <int i, int u, int j>
__device__ __forceinline__ void save_pieces(const nerf_chain_bwd& p, State& st) {
    using f2::Piece;
    constexpr int W = i == 0 ? 128 : 256;   // D_0 = dyr is 128 wide
    constexpr int npair = W / 32;
    auto cm_at = [&](int t, int half) {
        int o = O_CMX + 16 * st.g + (CMQ == 1 ? 0 : 4 * f2::CMS * (st.n >> (CMQ == 2 ? 3 : 2)));
        asm volatile("" : "+v"(o));
        return reinterpret_cast<uint32_t*>(st.lds + o) + (i & 1) * 256 + 32 * t + 16 * half;
    };
    const bool leader = (st.n & (16 / CMQ - 1)) == 0;
    float* ob = p.dy[i] + st.m0 * W;
    int vrow = st.vrow;
    if constexpr (W != 256) vrow = (st.rl * W + 4 * st.g) * 4;
    if constexpr (u == 0) {
        if constexpr (j == piece_tile<16>(f2::P0_STORE)) f2::tile_store4<W>(ob, vrow, 0, st.xs[0]);
        if constexpr (j == piece_tile<16>(f2::P0_STORE_B)) f2::tile_store4<W>(ob, vrow, 64, st.xs[1]);
        if constexpr (j == piece_tile<16>(f2::P0_CMAX_A)) f2::colmax4<CMQ>(st.xs[0], cm_at(0, 0), leader);
        if constexpr (j == piece_tile<16>(f2::P0_CMAX_B)) f2::colmax4<CMQ>(st.xs[1], cm_at(0, 1), leader);
    }
    if constexpr (u + 1 < npair) {
        constexpr int t = u + 1;
        if constexpr (j == piece_tile<16>(f2::P_STORE)) f2::tile_store4<W>(ob, vrow, 128 * t, st.xs[2 * t]);
        if constexpr (j == piece_tile<16>(f2::P_STORE_B)) f2::tile_store4<W>(ob, vrow, 128 * t + 64, st.xs[2 * t + 1]);
        if constexpr (j == piece_tile<16>(f2::P_CMAX_A)) f2::colmax4<CMQ>(st.xs[2 * t], cm_at(t, 0), leader);
        if constexpr (j == piece_tile<16>(f2::P_CMAX_B)) f2::colmax4<CMQ>(st.xs[2 * t + 1], cm_at(t, 1), leader);
    }
}

template <int i, int u, int j>
__device__ __forceinline__ void split_pieces(State& st) {
    if constexpr (u + 1 < nks(i)) {
        constexpr int t = u + 1;
        const f2::f32x4 A = st.xs[2 * t], B = st.xs[2 * t + 1];
        const float s = st.ser;
        if constexpr (j == piece_tile<16>(f2::P_SPLIT_HI_A)) {
            st.act_hi[t].x = f2::mhi(A[0], A[1], s);
            st.act_hi[t].y = f2::mhi(A[2], A[3], s);
        }
        if constexpr (j == piece_tile<16>(f2::P_SPLIT_HI_B)) {
            st.act_hi[t].z = f2::mhi(B[0], B[1], s);
            st.act_hi[t].w = f2::mhi(B[2], B[3], s);
        }
        if constexpr (j == piece_tile<16>(f2::P_SPLIT_LO_A)) {
            st.act_lo[t].x = f2::mlo(A[0], A[1], s, st.act_hi[t].x);
            st.act_lo[t].y = f2::mlo(A[2], A[3], s, st.act_hi[t].y);
        }
        if constexpr (j == piece_tile<16>(f2::P_SPLIT_LO_B)) {
            st.act_lo[t].z = f2::mlo(B[0], B[1], s, st.act_hi[t].z);
            st.act_lo[t].w = f2::mlo(B[2], B[3], s, st.act_hi[t].w);
        }
    }
}

// global tile G's weight fragments into ring entry G % (PF + 1) (f2::frag_read)
template <int G>
__device__ __forceinline__ void frag_read(State& st) {
    if constexpr (G < NG) {
        constexpr int R = PF + 1;
        constexpr int k = G / 16, j = G % 16, slot = tt_of_k(k) % NSLOT;
        static_assert(slot % 2 == 0, "a 32-k step's two slots are consecutive");
        constexpr int off = O_RING + (slot & 3) * SBYTES + 256 * j;
        const char* b = st.lds + st.fr + (slot >= 4 ? 4 * SBYTES : 0);
        st.wh[G % R] = *reinterpret_cast<const uint4*>(b + off);
        st.wl[G % R] = *reinterpret_cast<const uint4*>(b + off + SPLANE);
    }
}
template <int G0, int N>
__device__ __forceinline__ void frag_reads(State& st) {
    if constexpr (N > 0) {
        frag_read<G0>(st);
        frag_reads<G0 + 1, N - 1>(st);
    }
}

// behind layer i's first tile: its weight-row exponents (landed with the step) as the scales
// 2^-e for its epilogue; D_{i-1}'s column maxima (complete since layer i-1's last step) out and
// cleared -- D_0 is 128 wide: waves 4-7 store theirs to the scratch row (one store op per wave)
template <int i>
__device__ __forceinline__ void layer_start(const nerf_chain_bwd& p, State& st) {
    const int tid = f2::fresh(st.tid);
    if (tid < 256)
        reinterpret_cast<float*>(st.lds + O_EXP)[(i & 1) * 256 + tid] = __builtin_amdgcn_ldexpf(
            1.f, -reinterpret_cast<const int*>(st.lds + O_LEB + (i & 1) * 1024)[tid]);
    if constexpr (i >= 1) {
        constexpr int W = i - 1 == 0 ? 128 : 256;
        const int lane = tid & 63;
        if (lane < 32) {
            uint32_t* cm = reinterpret_cast<uint32_t*>(st.lds + O_CMX);
            const int cw = ((i - 1) & 1) * 256 + 32 * st.wave + lane;
            float* dst = 32 * st.wave < W ? p.dy_cmax[i - 1] + (st.m0 / CROWS) * W + 32 * st.wave + lane
                                          : p.scratch + 64 * st.wave + lane;
            *dst = __uint_as_float(f2::cm_read<CMQ>(cm, cw));
            f2::cm_clear<CMQ>(cm, cw);
        }
    }
}

template <int i, int u, int j>
__device__ __forceinline__ void tiles(const nerf_chain_bwd& p, State& st, const uint4& ah, const uint4& al) {
    constexpr int R = PF + 1;
    constexpr int k = kfirst(i) + u, G = 16 * k + j;
    if constexpr (j < 16) {
        if constexpr (G + PF < NG && layer_of_k((G + PF) / 16) == i) frag_read<G + PF>(st);   // (f2::mstep_tiles)
        __builtin_amdgcn_sched_barrier(0);
        st.acc[j] = f2::mfma16(st.wh[G % R], al, st.acc[j]);   // hi . lo
        st.acc[j] = f2::mfma16(st.wl[G % R], ah, st.acc[j]);   // lo . hi
        st.acc[j] = f2::mfma16(st.wh[G % R], ah, st.acc[j]);   // hi . hi
        if constexpr (u == 0 && j == 0) layer_start<i>(p, st);
        split_pieces<i, u, j>(st);
        save_pieces<i, u, j>(p, st);
        if constexpr (k + 1 < NK && j == TB) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(wait_n(k)) : "memory");
            __syncthreads();   // B_{k+1}
            dma<tt_of_k(k + NPAIR - 1)>(p, st);
        }
        if constexpr (k + 1 < NK && j == TB + f2::DMA2) dma<tt_of_k(k + NPAIR - 1) + 1>(p, st);
        __builtin_amdgcn_sched_barrier(0);
        tiles<i, u, j + 1>(p, st, ah, al);
    }
}

template <int i, int u>
__device__ __forceinline__ void kstep(const nerf_chain_bwd& p, State& st) {
    if constexpr (u == 0) frag_reads<16 * kfirst(i), PF>(st);
    tiles<i, u, 0>(p, st, st.act_hi[u], st.act_lo[u]);
}

template <int i, int u>
__device__ __forceinline__ void ksteps(const nerf_chain_bwd& p, State& st) {
    if constexpr (u < nks(i)) {
        kstep<i, u>(p, st);
        ksteps<i, u + 1>(p, st);
    }
}

// layer i: k-loop, then the epilogue -- unscale, the feature layer's rank-one term, the
// input's ReLU mask -> D_{i+1} (features 16 j + 4 g + c of the lane's row, tile layout), its
// row max and k-step 0's A fragment (the rest during the next layer's k-steps); the last
// layer stores D_9 and its column maxima here
template <int i>
__device__ __forceinline__ void layer(const nerf_chain_bwd& p, State& st) {
    constexpr bool last = i == NL - 1;
#pragma unroll
    for (int j = 0; j < 16; ++j) st.acc[j] = f2::f32x4{0.f, 0.f, 0.f, 0.f};
    ksteps<i, 0>(p, st);
    int g4 = 4 * st.g;
    asm volatile("" : "+v"(g4));
    const float* le = reinterpret_cast<const float*>(st.lds + O_EXP) + (i & 1) * 256 + g4;
    const float sr = __builtin_amdgcn_ldexpf(1.f, -st.er);
    const f2::pf2 sr2 = {sr, sr};
    uint32_t mw[8];
    if constexpr (i >= 1) {
        const uint4* mrow = reinterpret_cast<const uint4*>(st.lds + O_MASK + (i & 1) * 4096 + st.rl * 32);
        const uint4 a = mrow[0], b = mrow[1];
        mw[0] = a.x; mw[1] = a.y; mw[2] = a.z; mw[3] = a.w;
        mw[4] = b.x; mw[5] = b.y; mw[6] = b.z; mw[7] = b.w;
    }
    float rmx = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        __builtin_amdgcn_sched_barrier(0);
        const int f0 = 16 * j + g4;
        const float4 s4 = *reinterpret_cast<const float4*>(le + 16 * j);
        const f2::pf2 x01 = (f2::pf2{st.acc[j][0], st.acc[j][1]} * sr2) * f2::pf2{s4.x, s4.y};
        const f2::pf2 x23 = (f2::pf2{st.acc[j][2], st.acc[j][3]} * sr2) * f2::pf2{s4.z, s4.w};
        f2::f32x4 x;
        x[0] = x01[0]; x[1] = x01[1]; x[2] = x23[0]; x[3] = x23[1];
        if constexpr (i == 1) {   // + d sigma_raw x w_density (the density head reads h7)
            const float4 w4 = *reinterpret_cast<const float4*>(st.fx + f0);
            x[0] += st.gr0 * w4.x; x[1] += st.gr0 * w4.y; x[2] += st.gr0 * w4.z; x[3] += st.gr0 * w4.w;
        }
        if constexpr (i >= 1) {   // the input's ReLU bits: all-ones / zero masks by a signed bit extract
            const uint32_t bits = mw[j >> 1] >> ((j & 1) * 16 + g4);
#pragma unroll
            for (int c = 0; c < 4; ++c)
                x[c] = __int_as_float(__float_as_int(x[c]) & __builtin_amdgcn_sbfe((int)bits, c, 1));
        }
        st.xs[j] = x;
        if constexpr (false) {   // (v_max3 here spills this kernel: 23 scratch ops against 2)
            rmx = f2::max3abs(f2::max3abs(rmx, x[0], x[1]), x[2], x[3]);
        } else {
            rmx = fmaxf(rmx, fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3]))));
        }
        if constexpr (last) {
            f2::tile_store4<256>(p.dy[NL] + st.m0 * 256, st.vrow, 64 * j, x);
            if constexpr (CMQ == 1)
                f2::colmax4(x, reinterpret_cast<uint32_t*>(st.lds + O_CMX) + (NL & 1) * 256 + f0, st.n == 0);
            else
                f2::colmax4<CMQ>(x, reinterpret_cast<uint32_t*>(st.lds + O_CMX + 16 * st.g +
                                                                 4 * f2::CMS * (st.n >> (CMQ == 2 ? 3 : 2))) +
                                        (NL & 1) * 256 + 16 * j,
                                 (st.n & (16 / CMQ - 1)) == 0);
        }
    }
    // the row's max over its four 16-lane rows (lanes n, n + 16, n + 32, n + 48)
    const float m = f2::rows_max(rmx);
    if (st.g == 0) p.dy_rmax[i + 1][st.m0 + f2::fresh(st.rl)] = m;
    if constexpr (!last) {
        st.er = f2::chain_exp(m);
        st.ser = __builtin_amdgcn_ldexpf(1.f, st.er);
        f2::split_hi<0>(st);
        f2::split_lo<0>(st);
    }
}

__device__ __forceinline__ void layers(const nerf_chain_bwd& p, State& st) {
    layer<0>(p, st);
    layer<1>(p, st);
    layer<2>(p, st);
    layer<3>(p, st);
    layer<4>(p, st);
    layer<5>(p, st);
    layer<6>(p, st);
    layer<7>(p, st);
    layer<8>(p, st);
}

}  // namespace b2

__global__ __launch_bounds__(512, 2) void k_mlp_chain_bwd(ChainBwdArgs args) {
    using namespace b2;
    const nerf_chain_bwd& p = args.a;
    __shared__ __attribute__((aligned(16))) char smem[BYTES];
    State st;
    st.lds = smem;
    st.lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(clds_t*)smem);
    st.fx = reinterpret_cast<float*>(smem + O_FX);
    st.tid = threadIdx.x;
    st.wave = __builtin_amdgcn_readfirstlane(st.tid >> 6);
    st.lane = st.tid & 63; st.n = st.lane & 15; st.g = st.lane >> 4;
    st.m0 = (size_t)blockIdx.x * CROWS;
    st.rl = 16 * st.wave + st.n;
    st.voff16 = 16u * st.lane;
    st.vrow = (st.rl * 256 + 4 * st.g) * 4;
    st.fr = (st.g >> 1) * b2::SBYTES + (st.g & 1) * b2::SHALF + st.n * 16;
    if (st.wave >= 4) __builtin_amdgcn_s_setprio(1);
    // head weights into LDS, both column-max parities cleared
    if (st.tid < 256) st.fx[st.tid] = p.wd[st.tid];
    for (int e = st.tid; e < 384; e += NTH) st.fx[256 + e] = p.wc[e];
    for (int e = st.tid; e < f2::cm_words(CMQ); e += NTH) reinterpret_cast<uint32_t*>(smem + O_CMX)[e] = 0u;
    const size_t row = st.m0 + st.rl;
    const float4 gr = *reinterpret_cast<const float4*>(p.graw4 + row * 4);
    const uint4 mr = *reinterpret_cast<const uint4*>(p.hr_mask + row * p.ld_hr_mask);
    st.gr0 = gr.x;
    __syncthreads();
    // D_0 = dyr: (d rgb logits) . fc_rgb, gated by the colour layer's ReLU bits (render.hip
    // k_heads_dyr), in the tile layout of an epilogue output: xs[j][c] = feature 16 j + 4 g + c
    float m = 0.f;
    const uint32_t mwr[4] = {mr.x, mr.y, mr.z, mr.w};
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int f = 16 * j + 4 * st.g + c;
            float v = fmaf(gr.w, st.fx[256 + 256 + f], fmaf(gr.z, st.fx[256 + 128 + f], gr.y * st.fx[256 + f]));
            v = ((mwr[j >> 1] >> ((j & 1) * 16 + 4 * st.g + c)) & 1u) ? v : 0.f;
            st.xs[j][c] = v;
            m = fmaxf(m, fabsf(v));
        }
    m = f2::rows_max(m);
    if (st.g == 0) p.dy_rmax[0][row] = m;
    st.er = f2::chain_exp(m);
    st.ser = __builtin_amdgcn_ldexpf(1.f, st.er);
    f2::split_hi<0>(st);
    f2::split_lo<0>(st);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    dma_n<0, 2 * (NPAIR - 1)>(p, st);   // steps 0 .. NPAIR - 2
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(wait_prologue()) : "memory");
    __syncthreads();   // B_0
    layers(p, st);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // D_8's (parity 0, saved by layer 8's k-steps) and D_9's (parity 1, the last epilogue)
    // column maxima
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const size_t grp = (size_t)blockIdx.x;
    const int par = tid >> 8, f = tid & 255;
    p.dy_cmax[NL - 1 + par][grp * 256 + f] =
        __uint_as_float(f2::cm_read<CMQ>(reinterpret_cast<const uint32_t*>(smem + O_CMX), tid));
}
}  // namespace nerf

using namespace nerf;

static unsigned long long* g_chain_stamps = nullptr;

extern "C" int nerf_mlp_chain_fwd(const float* enc_p, const float* enc_d, const float* enc_p_rmax,
                                  const float* enc_d_rmax, int n_pad, const nerf_chain_layer* layers, void* stream) {
    NERF_CHECK_PTR(enc_p); NERF_CHECK_PTR(enc_d); NERF_CHECK_PTR(enc_p_rmax); NERF_CHECK_PTR(enc_d_rmax);
    NERF_CHECK_PTR(layers);
    NERF_CHECK(n_pad > 0 && n_pad % CROWS == 0, "%s: n_pad=%d must be a positive multiple of %d", __func__, n_pad,
               CROWS);
    NERF_CHECK(gemm_precision() == 2, "%s: the fused chain runs in GEMM precision mode 2 (fp16 pair images)", __func__);
    NERF_CHECK_ALIGN16(enc_p); NERF_CHECK_ALIGN16(enc_d);
    ChainFwdArgs a{};
    a.enc_p = enc_p; a.enc_d = enc_d; a.rp = enc_p_rmax; a.rd = enc_d_rmax; a.n_pad = n_pad;
    for (int l = 0; l < CNL; ++l) {
        const nerf_chain_layer& L = layers[l];
        NERF_CHECK(L.img && L.bias, "%s: layer %d needs its weight image and bias", __func__, l);
        NERF_CHECK((((uintptr_t)L.bias) & 15u) == 0, "%s: layer %d: bias not 16-byte aligned (16-byte LDS-DMA)",
                   __func__, l);
        NERF_CHECK(L.img_rows >= L_OUT[l] && (((uintptr_t)L.img) & 15u) == 0,
                   "%s: layer %d: image rows %d < %d or image not 16-byte aligned", __func__, l, L.img_rows, L_OUT[l]);
        NERF_CHECK(L.out == nullptr || (L.ldo >= L_OUT[l] && L.ldo % 4 == 0 && (((uintptr_t)L.out) & 15u) == 0),
                   "%s: layer %d: bad output (ldo %d)", __func__, l, L.ldo);
        NERF_CHECK(L.mask == nullptr || L.ldmask >= L_OUT[l] / 32, "%s: layer %d: ldmask %d", __func__, l, L.ldmask);
        NERF_CHECK(l != CNL - 1 || L.cmax == nullptr, "%s: the colour layer has no column maxima", __func__);
        a.L[l] = L;
    }
    a.stamps = g_chain_stamps;
    hipLaunchKernelGGL(k_mlp_chain_fwd<false>, dim3(n_pad / CROWS), dim3(256), 0, as_stream(stream), a);
    return check_launch(__func__);
}

extern "C" int nerf_mlp_chain_train(const float* enc_p, const float* enc_d, const float* enc_p_rmax,
                                    const float* enc_d_rmax, int n_pad, const nerf_chain_layer* layers, const float* wd,
                                    const float* bd, const float* wc, const float* bc, float* raw4, void* stream) {
    NERF_CHECK_PTR(enc_p); NERF_CHECK_PTR(enc_d); NERF_CHECK_PTR(enc_p_rmax); NERF_CHECK_PTR(enc_d_rmax);
    NERF_CHECK_PTR(layers); NERF_CHECK_PTR(wd); NERF_CHECK_PTR(bd); NERF_CHECK_PTR(wc); NERF_CHECK_PTR(bc);
    NERF_CHECK_PTR(raw4);
    NERF_CHECK(n_pad > 0 && n_pad % CROWS == 0, "%s: n_pad=%d must be a positive multiple of %d", __func__, n_pad,
               CROWS);
    NERF_CHECK(gemm_precision() == 2, "%s: the fused chain runs in GEMM precision mode 2 (fp16 pair images)", __func__);
    NERF_CHECK_ALIGN16(enc_p); NERF_CHECK_ALIGN16(enc_d); NERF_CHECK_ALIGN16(raw4);
    ChainFwdArgs a{};
    a.enc_p = enc_p; a.enc_d = enc_d; a.rp = enc_p_rmax; a.rd = enc_d_rmax; a.n_pad = n_pad;
    for (int l = 0; l < CNL; ++l) {
        const nerf_chain_layer& L = layers[l];
        NERF_CHECK(L.img && L.bias, "%s: layer %d needs its weight image and bias", __func__, l);
        NERF_CHECK((((uintptr_t)L.bias) & 15u) == 0 && (((uintptr_t)L.img) & 15u) == 0 && L.img_rows == L_OUT[l],
                   "%s: layer %d: image / bias not 16-byte aligned or chain image rows %d != %d", __func__, l,
                   L.img_rows, L_OUT[l]);
        // every output is mandatory: the k-steps' vmcnt waits count these stores at compile time
        NERF_CHECK(L.out && L.ldo == L_OUT[l] && (((uintptr_t)L.out) & 15u) == 0,
                   "%s: layer %d: the training chain saves every layer output (ldo %d: 256 for l0..lf, 128 for the "
                   "colour layer)", __func__, l, L.ldo);
        NERF_CHECK(l == 8 || (L.mask && L.ldmask >= L_OUT[l] / 32 && L.ldmask % 2 == 0 &&
                              (((uintptr_t)L.mask) & 7u) == 0),
                   "%s: layer %d: the ReLU words are mandatory (ldmask %d, even, 8-byte aligned)", __func__, l, L.ldmask);
        NERF_CHECK(l != 8 || L.mask == nullptr, "%s: the feature layer has no ReLU", __func__);
        NERF_CHECK(l == CNL - 1 ? L.cmax == nullptr : L.cmax != nullptr,
                   "%s: layer %d: column maxima are mandatory for l0..lf and absent for the colour layer", __func__, l);
        a.L[l] = L;
    }
    a.wd = wd; a.bd = bd; a.wc = wc; a.bc = bc; a.raw4 = raw4;
    a.stamps = g_chain_stamps;
    // algorithmic work per row: the ten linears over their unpadded inputs (63, 256 x 3, 319,
    // 256 x 4, colour 283) + both heads = 593 408 MACs; HBM: the two encodings
    // read, every output (f32), ReLU word and raw4 written
    const double rows = (double)n_pad;
    prof_next(NERF_PROF_CHAIN_FWD, rows * (2 * 64 * 4 + 9 * 256 * 4 + 128 * 4 + 9 * 32 + 4 * 4));
    prof_begin(as_stream(stream));
    hipLaunchKernelGGL(k_mlp_chain_train2, dim3(n_pad / CROWS), dim3(f2::NTH), 0, as_stream(stream), a);
    prof_end(as_stream(stream), 2.0 * rows * (256.0 * 63 + 7 * 256 * 256 + 256 * 319 + 128 * 283 + 256 + 3 * 128), 3);
    return check_launch(__func__);
}

extern "C" int nerf_render_eval_fused(const float* pts_o, const float* pts_d, const float* view, int n_rays,
                                      int n_samples, float near_z, float far_z, int flags,
                                      const nerf_chain_layer* layers, const float* wd, const float* bd,
                                      const float* wc, const float* bc, float* rgb, float* dist, float* alpha,
                                      float* z, void* stream) {
    NERF_CHECK_PTR(pts_o); NERF_CHECK_PTR(pts_d); NERF_CHECK_PTR(view); NERF_CHECK_PTR(layers);
    NERF_CHECK_PTR(wd); NERF_CHECK_PTR(bd); NERF_CHECK_PTR(wc); NERF_CHECK_PTR(bc);
    NERF_CHECK_PTR(rgb); NERF_CHECK_PTR(dist); NERF_CHECK_PTR(alpha); NERF_CHECK_PTR(z);
    NERF_CHECK(n_rays > 0 && n_samples >= 2 && CROWS % n_samples == 0,
               "%s: n_rays=%d, n_samples=%d: the samples of a ray must tile the %d-row block (S >= 2 divides %d)",
               __func__, n_rays, n_samples, CROWS, CROWS);
    NERF_CHECK((int64_t)n_rays * n_samples <= (int64_t)1 << 30, "%s: too many samples", __func__);
    NERF_CHECK(gemm_precision() == 2, "%s: the fused chain runs in GEMM precision mode 2 (fp16 pair images)", __func__);
    NERF_CHECK((flags & ~7) == 0, "%s: unknown flags %d", __func__, flags);
    ChainFwdArgs a{};
    const int64_t n = (int64_t)n_rays * n_samples;
    a.n_pad = (int)((n + CROWS - 1) / CROWS * CROWS);
    for (int l = 0; l < CNL; ++l) {
        const nerf_chain_layer& L = layers[l];
        NERF_CHECK(L.img && L.bias, "%s: layer %d needs its weight image and bias", __func__, l);
        NERF_CHECK((((uintptr_t)L.bias) & 15u) == 0 && (((uintptr_t)L.img) & 15u) == 0 && L.img_rows == L_OUT[l],
                   "%s: layer %d: image / bias not 16-byte aligned or chain image rows %d != %d", __func__, l,
                   L.img_rows, L_OUT[l]);
        NERF_CHECK(L.out == nullptr && L.mask == nullptr && L.cmax == nullptr,
                   "%s: layer %d: the eval render saves no activations, masks or column maxima", __func__, l);
        a.L[l] = L;
    }
    a.po = pts_o; a.pd = pts_d; a.view = view;
    a.R = n_rays; a.S = n_samples; a.flags = flags; a.near_z = near_z; a.far_z = far_z;
    a.wd = wd; a.bd = bd; a.wc = wc; a.bc = bc;
    a.rgb = rgb; a.dist = dist; a.alpha = alpha; a.z = z;
    a.stamps = g_chain_stamps;
    hipLaunchKernelGGL(k_render_fused2, dim3(a.n_pad / CROWS), dim3(f2::NTH), 0, as_stream(stream), a);
    return check_launch(__func__);
}

// diagnostics: per-block phase cycles of the chain kernels (wait, barrier, MFMA section,
// epilogue, total, end realtime) into a device buffer of (n_pad / 128) * 6 uint64; NULL off.
// The two-wave kernels stamp only in a NERF_CHAIN_STAMPS build (their production code has no
// stamp instructions); the one-wave k_mlp_chain_fwd always can
extern "C" int nerf_chain_debug_stamps(void* buf) {
    g_chain_stamps = reinterpret_cast<unsigned long long*>(buf);
    return NERF_OK;
}
extern "C" int nerf_chain_stamps_built(void) { return NERF_CHAIN_STAMPS; }

extern "C" int nerf_mlp_chain_bwd(const nerf_chain_bwd* a, void* stream) {
    NERF_CHECK_PTR(a);
    const nerf_chain_bwd& p = *a;
    NERF_CHECK(p.n_pad > 0 && p.n_pad % CROWS == 0, "%s: n_pad=%d must be a positive multiple of %d", __func__,
               p.n_pad, CROWS);
    NERF_CHECK(gemm_precision() == 2, "%s: the chain runs in GEMM precision mode 2 (fp16 pair images)", __func__);
    NERF_CHECK(p.graw4 && p.hr_mask && p.ld_hr_mask >= 4 && p.wd && p.wc && p.scratch,
               "%s: graw4, the colour layer's ReLU words (ld >= 4), wd, wc and a scratch row are required", __func__);
    NERF_CHECK_ALIGN16(p.graw4); NERF_CHECK_ALIGN16(p.wd);
    NERF_CHECK((((uintptr_t)p.hr_mask) & 15u) == 0 && p.ld_hr_mask % 4 == 0, "%s: hr_mask 16-byte rows", __func__);
    for (int i = 0; i < 9; ++i) {
        NERF_CHECK(p.wt_img[i] && (((uintptr_t)p.wt_img[i]) & 15u) == 0 && p.wt_img_rows[i] == b2::KPB[i],
                   "%s: layer %d: weight-transpose chain image missing, unaligned or not %d rows", __func__, i,
                   b2::KPB[i]);
        NERF_CHECK(i == 0 || (p.in_mask[i] && p.ld_in_mask[i] >= 8 && (((uintptr_t)p.in_mask[i]) & 15u) == 0 &&
                              p.ld_in_mask[i] % 4 == 0),
                   "%s: layer %d: the input's ReLU words (ld >= 8, 16-byte rows) are required", __func__, i);
    }
    for (int i = 0; i < 10; ++i) {
        const int w = i == 0 ? 128 : 256;
        NERF_CHECK(p.dy[i] && p.lddy[i] == w && (((uintptr_t)p.dy[i]) & 15u) == 0 && p.dy_cmax[i] && p.dy_rmax[i],
                   "%s: D_%d: output, column maxima and row maxima are mandatory (ld == %d, 16-byte aligned)", __func__,
                   i, w);
    }
    ChainBwdArgs args{p};
    // algorithmic work per row: dyr (3 x 128) and nine 256-output GEMMs (K = 128, then 256);
    // HBM: graw4 and the ReLU words read, D_0 .. D_9 (f32) and their row maxima written
    const double rows = (double)p.n_pad;
    prof_next(NERF_PROF_CHAIN_BWD, rows * (16 + 16 + 8 * 32 + 128 * 4 + 9 * 256 * 4 + 10 * 4));
    prof_begin(as_stream(stream));
    hipLaunchKernelGGL(k_mlp_chain_bwd, dim3(p.n_pad / CROWS), dim3(f2::NTH), 0, as_stream(stream), args);
    prof_end(as_stream(stream), 2.0 * rows * (3.0 * 128 + 128 * 256 + 8 * 256 * 256), 3);
    return check_launch(__func__);
}
