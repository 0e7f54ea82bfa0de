// Weight packing, the Adam step and the point-cloud nearest-neighbour kernel.
#include "common.hpp"

#include <cmath>

namespace nerf {

struct PackBatch {
    nerf_pack_desc d[NERF_MAX_PACK];
    int n;
    int f16;   // GEMM precision mode 2: images in the fp16 pair form (pack_h), not bf16x3
};

// x -> three bf16 words (RNE each) with x = hi + mid + lo (same split as gemm_x6.hip)
__device__ __forceinline__ void split3(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
    const __bf16 bh = (__bf16)x;
    const float r = x - (float)bh;
    const __bf16 bm = (__bf16)r;
    const __bf16 bl = (__bf16)(r - (float)bm);
    h = __builtin_bit_cast(uint16_t, bh);
    m = __builtin_bit_cast(uint16_t, bm);
    l = __builtin_bit_cast(uint16_t, bl);
}

// element (r, c) of a [N][K] operand into its bf16x3 image [3][K/8][N][8]
__device__ __forceinline__ void put_split(uint16_t* img, int N, int K, int r, int c, float x) {
    uint16_t h, m, l;
    split3(x, h, m, l);
    const size_t plane = (size_t)K * N;
    const size_t o = ((size_t)(c >> 3) * N + r) * 8 + (c & 7);
    img[o] = h;
    img[o + plane] = m;
    img[o + 2 * plane] = l;
}

// descriptor d; block bx of nb grid-strides over the padded destination
__device__ __forceinline__ void pack_f32(const PackBatch& pb, const nerf_pack_desc& d, int bx, int nb) {
#pragma clang fp contract(off)
    const int rows_s = d.rows_s > d.rows ? d.rows_s : d.rows;
    const int total = (d.dst_s != nullptr ? rows_s : d.rows) * d.ld_dst;
    const int gs = nb * blockDim.x;
    for (int e = bx * blockDim.x + threadIdx.x; e < total; e += gs) {
        const int r = e / d.ld_dst, c = e % d.ld_dst;
        const float x = (c < d.cols && r < d.rows) ? d.src[(size_t)r * d.cols + c] : 0.f;
        if (r < d.rows) d.dst[e] = x;
        if (d.dst_s != nullptr && !pb.f16) put_split(d.dst_s, rows_s, d.ld_dst, r, c, x);
    }
    if (d.dst_t != nullptr) {
        const int tt = d.rows_t * d.rows;  // dst_t[c][r], c < rows_t, r < rows
        for (int e = bx * blockDim.x + threadIdx.x; e < tt; e += gs) {
            const int c = e / d.rows, r = e % d.rows;
            d.dst_t[(size_t)c * d.ld_t + r] = c < d.cols ? d.src[(size_t)r * d.cols + c] : 0.f;
        }
    }
    if (d.dst_ts != nullptr && !pb.f16) {
        const int tt = d.rows_t * d.ld_t;  // whole image of dst_t, zero past the source
        for (int e = bx * blockDim.x + threadIdx.x; e < tt; e += gs) {
            const int c = e / d.ld_t, r = e % d.ld_t;   // dst_t row c, column r
            const float x = (c < d.cols && r < d.rows) ? d.src[(size_t)r * d.cols + c] : 0.f;
            put_split(d.dst_ts, d.rows_t, d.ld_t, c, r, x);
        }
    }
}

// Row r of the fp16 pair image of a [N][K] operand (x(c) = element (r, c)): one wave per
// row; the row max sets the scale 2^e, planes 0 / 1 get hi / lo of x 2^e (RNE fp16 each),
// e goes into the first word of the row's plane-2 chunk 0 (gemm_x6.hip, mode 2).  The row
// stays in registers between the max and the split (all its loads in flight at once: one
// memory latency per row, not one per 64 elements and pass).
constexpr int PACK_H_MAXK = 16 * kWave;
// chain images (cexp = true) also get the row exponents as one compact int array in plane 2's
// chunk 1 (unused otherwise): the chain kernels fetch a layer's 256 exponents with one 1 KB
// LDS-DMA instead of one 16-byte chunk per row
template <typename F>
__device__ __forceinline__ void put_row_h(uint16_t* img, int N, int K, int r, F&& x, bool cexp = false) {
    const int lane = lane_id();
    float v[PACK_H_MAXK / kWave];
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < PACK_H_MAXK / kWave; ++i) {
        const int c = lane + kWave * i;
        v[i] = c < K ? x(c) : 0.f;
        m = fmaxf(m, fabsf(v[i]));
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    const int e = row_exp(m);
    const size_t plane = (size_t)K * N;
#pragma unroll
    for (int i = 0; i < PACK_H_MAXK / kWave; ++i) {
        const int c = lane + kWave * i;
        if (c >= K) break;
        const float y = __builtin_amdgcn_ldexpf(v[i], e);
        const _Float16 h = (_Float16)y;
        const _Float16 l = (_Float16)(y - (float)h);
        const size_t o = ((size_t)(c >> 3) * N + r) * 8 + (c & 7);
        img[o] = __builtin_bit_cast(uint16_t, h);
        img[o + plane] = __builtin_bit_cast(uint16_t, l);
    }
    if (lane == 0) *reinterpret_cast<int*>(img + 2 * plane + (size_t)r * 8) = e;
    if (cexp && lane == 0) reinterpret_cast<int*>(img + 2 * plane + (size_t)N * 8)[r] = e;
}

// fp16 pair images of the packed weights (GEMM precision mode 2): one wave per image row,
// rows of dst_s, dst_ts, then of the chain images dst_cs (the first perm_k columns in
// chain_perm order) and dst_cts (every column in chain order) (block bx of nb)
__device__ __forceinline__ void pack_h(const nerf_pack_desc& d, int bx, int nb) {
    const int rows_s = d.rows_s > d.rows ? d.rows_s : d.rows;
    const int ns = d.dst_s ? rows_s : 0, nt = d.dst_ts ? d.rows_t : 0;
    const int ncs = d.dst_cs ? rows_s : 0, nct = d.dst_cts ? d.rows_t : 0;
    const int wave = (bx * blockDim.x + threadIdx.x) >> 6;
    const int nwaves = (nb * blockDim.x) >> 6;
    auto w_at = [&](int r, int c) { return (c < d.cols && r < d.rows) ? d.src[(size_t)r * d.cols + c] : 0.f; };
    for (int w = wave; w < ns + nt + ncs + nct; w += nwaves) {
        if (w < ns) {
            const int r = w;
            put_row_h(d.dst_s, rows_s, d.ld_dst, r, [&](int c) { return w_at(r, c); });
        } else if (w < ns + nt) {
            const int c = w - ns;   // dst_t row = source column c, its columns = source rows
            put_row_h(d.dst_ts, d.rows_t, d.ld_t, c, [&](int r) { return w_at(r, c); });
        } else if (w < ns + nt + ncs) {
            const int r = w - ns - nt;
            put_row_h(d.dst_cs, rows_s, d.ld_dst, r, [&](int c) { return w_at(r, c < d.perm_k ? chain_perm(c) : c); },
                      true);
        } else {
            const int c = w - ns - nt - ncs;
            put_row_h(d.dst_cts, d.rows_t, d.ld_t, c, [&](int r) { return w_at(chain_perm(r), c); }, true);
        }
    }
}

// one launch for both packs: blockIdx.y = descriptor; blocks [0, PACK_F32) the padded f32
// copies (and the bf16x3 images), blocks [PACK_F32, +PACK_H) the fp16 pair images (mode 2).
// Sized for latency, not bandwidth (a 256x256 layer is ~1.5 MB of traffic): ~2 elements per
// thread of the f32 copies, one image row per wave (512 rows of a 256-wide layer + its
// transpose); blocks of the small descriptors (biases, head weights) exit at once
constexpr int PACK_F32 = 128, PACK_H = 128;
__global__ __launch_bounds__(256) void k_pack(PackBatch pb) {
    const nerf_pack_desc& d = pb.d[blockIdx.y];
    if ((int)blockIdx.x < PACK_F32) pack_f32(pb, d, blockIdx.x, PACK_F32);
    else pack_h(d, blockIdx.x - PACK_F32, PACK_H);
}

// torch.optim.Adam (amsgrad=False, maximize=False), the foreach formulation torch runs on GPU
// tensors by default (torch/optim/adam.py _multi_tensor_adam), op for op:
//   m.lerp_(g, 1 - b1); v.mul_(b2); v.addcmul_(g, g, 1 - b2); d = sqrt(v) / sqrt(bc2) + eps;
//   p.addcdiv_(m, d, -lr / bc1)
// with every scalar the f32 rounding of the Python double torch forms (1 - b1, 1 - b2,
// sqrt(1 - b2^t), lr / (1 - b1^t)).  Hyper-parameters and the step count live in device
// memory (hyper, 16 floats = {step, lr, b1, b2, eps, wd, 1 - b2, ticket, lr, b1, b2 as doubles
// in slots 8-13, 1 - b1, doubles-valid flag}) so a captured hipGraph replays correct bias
// corrections; an lr change reaches a replay once the host pushes it into the device block
// (HipAdam.sync_hyper() between replays).  Every workgroup uses step + 1; the last one to
// finish (ticket) stores it.
__device__ __forceinline__ float adam_one(float& p, float g, float& m, float& v, float om1, float b2, float om2,
                                          float eps, float wd, float sbc2, float step_size) {
    if (wd != 0.f) g = __fmaf_rn(wd, p, g);                        // grad.add(param, alpha=wd)
    const float mi = __fmaf_rn(om1, g - m, m);                       // exp_avg.lerp_(grad, 1 - beta1)
    const float vi = __fmaf_rn(om2, __fmul_rn(g, g), __fmul_rn(v, b2));   // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
    m = mi;
    v = vi;
    const float denom = sqrtf(vi) / sbc2 + eps;                      // sqrt, div_(bc2 sqrt), add_(eps): three roundings
    p = __fmaf_rn(-step_size, mi / denom, p);                        // addcdiv_(m, denom, value=-step_size)
    return p;
}

// float4 over the flat buffer (n4 = n / 4 vectors, the n % 4 tail by thread 0 of block 0);
// at most ADAM_BLOCKS workgroups so the completion ticket costs few atomics
constexpr int ADAM_BLOCKS = 512;
__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, const float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v, int64_t n,
                                              float* __restrict__ hyper) {
    const float step = hyper[0] + 1.f, b2 = hyper[3], eps = hyper[4], wd = hyper[5];
    // the scalars as torch forms them: from the host's doubles (slots 8-14, flag slot 15 = 1);
    // the bias corrections in double like torch's Python scalars (1 - beta2^t cancels: in f32
    // it is ~1e-5 off at small t)
    const bool dbl = hyper[15] == 1.f;
    const double* hd = reinterpret_cast<const double*>(hyper + 8);
    const double lr_d = dbl ? hd[0] : (double)hyper[1], b1_d = dbl ? hd[1] : (double)hyper[2];
    const double b2_d = dbl ? hd[2] : (double)b2;
    const float om1 = dbl ? hyper[14] : (float)(1.0 - b1_d);
    const float om2 = hyper[6] != 0.f ? hyper[6] : (float)(1.0 - b2_d);
    const double bc1 = 1.0 - pow(b1_d, (double)step);
    const float sbc2 = (float)sqrt(1.0 - pow(b2_d, (double)step));
    const float step_size = (float)(lr_d / bc1);
    const int64_t n4 = n >> 2;
    float4* p4 = reinterpret_cast<float4*>(p);
    float4* m4 = reinterpret_cast<float4*>(m);
    float4* v4 = reinterpret_cast<float4*>(v);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        float4 pp = p4[i], mm = m4[i], vv = v4[i];
        const float4 gg = g4[i];
        adam_one(pp.x, gg.x, mm.x, vv.x, om1, b2, om2, eps, wd, sbc2, step_size);
        adam_one(pp.y, gg.y, mm.y, vv.y, om1, b2, om2, eps, wd, sbc2, step_size);
        adam_one(pp.z, gg.z, mm.z, vv.z, om1, b2, om2, eps, wd, sbc2, step_size);
        adam_one(pp.w, gg.w, mm.w, vv.w, om1, b2, om2, eps, wd, sbc2, step_size);
        p4[i] = pp; m4[i] = mm; v4[i] = vv;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (int64_t i = n4 * 4; i < n; ++i) adam_one(p[i], g[i], m[i], v[i], om1, b2, om2, eps, wd, sbc2, step_size);
    __syncthreads();                              // this workgroup has read hyper[0]
    if (threadIdx.x == 0) {
        unsigned* ticket = reinterpret_cast<unsigned*>(hyper + 7);   // (hyper is 8-byte aligned: slots 8-13 doubles)
        if (atomicAdd(ticket, 1u) == gridDim.x - 1) {
            hyper[0] = step;
            *ticket = 0u;
        }
    }
}

// nearest neighbour, one thread per query point, reference points staged through LDS
constexpr int NN_TILE = 256;
__global__ __launch_bounds__(256) void k_chamfer_nn(const float* __restrict__ x, int P,
                                                    const float* __restrict__ y, int Q,
                                                    int64_t* __restrict__ idx) {
    __shared__ float4 ys[NN_TILE];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float px = 0.f, py = 0.f, pz = 0.f;
    if (i < P) { px = x[3 * i]; py = x[3 * i + 1]; pz = x[3 * i + 2]; }
    float best = INFINITY;
    int bi = 0;
    for (int t0 = 0; t0 < Q; t0 += NN_TILE) {
        const int j = t0 + threadIdx.x;
        if (j < Q) ys[threadIdx.x] = make_float4(y[3 * j], y[3 * j + 1], y[3 * j + 2], 0.f);
        __syncthreads();
        const int nt = min(NN_TILE, Q - t0);
        for (int k = 0; k < nt; ++k) {
            const float4 q = ys[k];
            const float dx = px - q.x, dy = py - q.y, dz = pz - q.z;
            const float d = sqrtf(__fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz)));
            if (d < best) { best = d; bi = t0 + k; }  // strict: first index wins ties (torch.argmin)
        }
        __syncthreads();
    }
    if (i < P) idx[i] = bi;
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_pack_weights(const nerf_pack_desc* descs, int n, void* stream) {
    NERF_CHECK_PTR(descs);
    NERF_CHECK(n > 0 && n <= NERF_MAX_PACK, "%s: n=%d outside 1..%d", __func__, n, NERF_MAX_PACK);
    PackBatch pb{};
    pb.n = n;
    pb.f16 = gemm_precision() == 2;
    for (int i = 0; i < n; ++i) {
        const nerf_pack_desc& d = descs[i];
        NERF_CHECK(d.src && d.dst && d.rows > 0 && d.cols > 0 && d.ld_dst >= d.cols,
                   "%s: bad descriptor %d", __func__, i);
        NERF_CHECK(d.dst_t == nullptr || (d.rows_t >= d.cols && d.ld_t >= d.rows),
                   "%s: descriptor %d: rows_t < cols or ld_t < rows", __func__, i);
        NERF_CHECK(d.dst_s == nullptr || d.ld_dst % 8 == 0, "%s: descriptor %d: split image needs ld_dst %% 8 == 0",
                   __func__, i);
        NERF_CHECK(!pb.f16 || ((d.dst_s == nullptr || d.ld_dst <= PACK_H_MAXK) &&
                               (d.dst_ts == nullptr || d.ld_t <= PACK_H_MAXK)),
                   "%s: descriptor %d: fp16 pair image rows longer than %d", __func__, i, PACK_H_MAXK);
        NERF_CHECK(d.dst_ts == nullptr || (d.rows_t >= d.cols && d.ld_t >= d.rows && d.ld_t % 8 == 0),
                   "%s: descriptor %d: transposed split image needs rows_t >= cols, ld_t >= rows, ld_t %% 8 == 0",
                   __func__, i);
        NERF_CHECK((d.dst_cs == nullptr && d.dst_cts == nullptr) ||
                       (pb.f16 && d.perm_k >= 0 && d.perm_k % 32 == 0 && d.perm_k <= d.ld_dst && d.ld_dst % 8 == 0 &&
                        d.ld_dst <= PACK_H_MAXK),
                   "%s: descriptor %d: chain images need precision mode 2, perm_k %% 32 == 0 (<= ld_dst)", __func__, i);
        NERF_CHECK(d.dst_cts == nullptr || (d.rows_t >= d.cols && d.ld_t >= d.rows && d.ld_t % 32 == 0 &&
                                            d.ld_t <= PACK_H_MAXK),
                   "%s: descriptor %d: the transposed chain image needs rows_t >= cols, ld_t >= rows, ld_t %% 32 == 0",
                   __func__, i);
        pb.d[i] = d;
    }
    bool images = false;
    for (int i = 0; i < n; ++i)
        images = images || descs[i].dst_s != nullptr || descs[i].dst_ts != nullptr || descs[i].dst_cs != nullptr ||
                 descs[i].dst_cts != nullptr;
    const int bx = PACK_F32 + ((pb.f16 && images) ? PACK_H : 0);
    hipLaunchKernelGGL(k_pack, dim3(bx, n), dim3(256), 0, as_stream(stream), pb);
    return check_launch(__func__);
}

extern "C" int nerf_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                              int64_t n, float* hyper, void* stream) {
    NERF_CHECK_PTR(param); NERF_CHECK_PTR(grad); NERF_CHECK_PTR(exp_avg); NERF_CHECK_PTR(exp_avg_sq);
    NERF_CHECK_PTR(hyper);
    NERF_CHECK(n > 0, "%s: n=%lld", __func__, (long long)n);
    NERF_CHECK((((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) & 15) == 0,
               "%s: buffers must be 16-byte aligned", __func__);
    NERF_CHECK((((uintptr_t)hyper) & 7) == 0, "%s: hyper must be 8-byte aligned (doubles in slots 8-13)", __func__);
    int64_t blocks = (n / 4 + 255) / 256;
    if (blocks < 1) blocks = 1;
    if (blocks > ADAM_BLOCKS) blocks = ADAM_BLOCKS;
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(256), 0, s, param, grad, exp_avg, exp_avg_sq, n, hyper);
    return check_launch(__func__);
}

extern "C" int nerf_chamfer_nn(const float* x, int p, const float* y, int q, int64_t* idx, void* stream) {
    NERF_CHECK_PTR(x); NERF_CHECK_PTR(y); NERF_CHECK_PTR(idx);
    NERF_CHECK(p > 0 && q > 0, "%s: empty point cloud (p=%d q=%d)", __func__, p, q);
    hipLaunchKernelGGL(k_chamfer_nn, dim3((p + 255) / 256), dim3(256), 0, as_stream(stream), x, p, y, q, idx);
    return check_launch(__func__);
}
