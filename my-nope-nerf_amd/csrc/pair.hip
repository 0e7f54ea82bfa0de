// Image-pair terms of the full NoPe-NeRF step: point clouds of
// the two depth maps at the pc resolution, the relative pose, the dense chamfer distance and
// the reprojection (rgb_s) loss, forward and backward (training.py:359-405, losses.py:116-159,
// common.py:75-109, 112-160, 436-457).
//
// The reference runs this as ~200 small ATen launches per step (4x4 products through
// hipBLASLt, grid_sample, a (3,P,P) brute-force difference per chamfer direction, gathers
// whose backward sorts the indices).  Here:
//   forward : k_pair_points (P points: pc1, pc2, X, Y, reprojection + rgb_s partials),
//             k_nn_part (both chamfer directions, query x chunk grid), k_nn_final (argmin over
//             chunks + |X - Y[nn]| partials), k_pair_reduce (one workgroup, fixed order);
//   backward: k_pair_bwd_scatter (the gathered-point chamfer gradients, 64-bit fixed-point atomics),
//             k_pair_bwd_points (per-point gradients -> d1, d2 and R, t, scale partials),
//             k_pair_bwd_reduce.
// Sizes are tiny (47 x 155 = 7285 points at V_KITTI): the budget is launches, and the NN
// search (2 x 53 M pair distances) is spread over ~2000 workgroups instead of 29.
#include "common.hpp"
#include "mat4.hpp"

#include <cmath>

namespace nerf {

// kernel arguments: device pointers of the call's inputs
struct PairArgs {
    const float* d1; const float* d2;    // [P] depth at the pc resolution (after the nl clamp)
    int h, w, P;
    const float* Kg;                     // camera_mat [4][4]
    const float* Rtg;                    // Rt_rel_12 [4][4]
    const float* s1g;                    // scale1 (scale_pcs) [1] or NULL (= 1)
    float nl;                            // nearest_limit
    const float* img1; const float* img2;   // [3][h][w] (bilinear-resized images) or NULL: no rgb_s
    int rgbs_detach_scale;               // detach_rgbs_scale: pc1 of the reprojection carries no grad
};

// the per-thread copy of the small operands: K, inv(K) (transform_to_world's M =
// (inv(I) @ inv(I)) @ inv(K), common.py:139-141, same elimination as nerf_unproject_matrix),
// R, t, s1
struct PairConst {
    float K[16], Kinv[16], R[9], t[3], s1;
    __device__ __forceinline__ void load(const PairArgs& a) {
        load4(a.Kg, K);
        inverse4(K, Kinv);
#pragma unroll
        for (int r = 0; r < 3; ++r) {
#pragma unroll
            for (int c = 0; c < 3; ++c) R[3 * r + c] = a.Rtg[4 * r + c];
            t[r] = a.Rtg[4 * r + 3];
        }
        s1 = a.s1g ? *a.s1g : 1.f;
    }
};

// arange_pixels at (h, w) (common.py:36-39)
__device__ __forceinline__ void pc_pixel(int i, int h, int w, float& x, float& y) {
    const int row = i / w, col = i - row * w;
    x = 2.f * (float)col / (float)(w - 1) - 1.f;
    y = 2.f * (float)row / (float)(h - 1) - 1.f;
}

// transform_to_world(p, d, K) = (inv(K) [x d, y d, d, 1])[:3]
__device__ __forceinline__ void unproject_pt(const float* Mi, float x, float y, float d, float p[3]) {
#pragma clang fp contract(off)
    const float xd = x * d, yd = y * d;
#pragma unroll
    for (int r = 0; r < 3; ++r) p[r] = ((Mi[4 * r] * xd + Mi[4 * r + 1] * yd) + Mi[4 * r + 2] * d) + Mi[4 * r + 3];
}

// grid_sample(img, p, bilinear, align_corners=True, zeros padding) of one channel plane and
// the derivatives of the sample w.r.t. p (common.py:75-109)
__device__ __forceinline__ float bilinear(const float* __restrict__ plane, int h, int w, float px, float py,
                                          float* dpx = nullptr, float* dpy = nullptr) {
    const float ix = (px + 1.f) * 0.5f * (float)(w - 1);
    const float iy = (py + 1.f) * 0.5f * (float)(h - 1);
    const float fx = floorf(ix), fy = floorf(iy);
    const int x0 = (int)fx, y0 = (int)fy;
    const float ax = ix - fx, ay = iy - fy;
    auto at = [&](int yy, int xx) -> float {
        return (xx >= 0 && xx < w && yy >= 0 && yy < h) ? plane[yy * w + xx] : 0.f;
    };
    const float v00 = at(y0, x0), v01 = at(y0, x0 + 1), v10 = at(y0 + 1, x0), v11 = at(y0 + 1, x0 + 1);
    if (dpx) {
        const float gx = ((v01 - v00) * (1.f - ay) + (v11 - v10) * ay) * 0.5f * (float)(w - 1);
        const float gy = ((v10 - v00) * (1.f - ax) + (v11 - v01) * ax) * 0.5f * (float)(h - 1);
        *dpx = gx;
        *dpy = gy;
    }
    return v00 * (1.f - ax) * (1.f - ay) + v01 * ax * (1.f - ay) + v10 * (1.f - ax) * ay + v11 * ax * ay;
}

// rgb_s geometry of point i: rotated pc1 (nl-clamped), projected p_re, validity
struct Reproj {
    float q[3];      // pc1_rot after the clamp
    bool bad;        // -z < nl: all three coordinates replaced by nl (no gradient)
    float h3[3];     // K[:3] [q, 1]
    float px, py;
    bool valid;
};

__device__ __forceinline__ Reproj reproject(const PairArgs& a, const PairConst& m, const float pc1[3]) {
#pragma clang fp contract(off)
    Reproj r;
#pragma unroll
    for (int k = 0; k < 3; ++k) r.q[k] = ((pc1[0] * m.R[3 * k] + pc1[1] * m.R[3 * k + 1]) + pc1[2] * m.R[3 * k + 2]) + m.t[k];
    r.bad = -r.q[2] < a.nl;
    if (r.bad) r.q[0] = r.q[1] = r.q[2] = a.nl;
#pragma unroll
    for (int k = 0; k < 3; ++k)
        r.h3[k] = ((m.K[4 * k] * r.q[0] + m.K[4 * k + 1] * r.q[1]) + m.K[4 * k + 2] * r.q[2]) + m.K[4 * k + 3];
    r.px = r.h3[0] / r.h3[2];
    r.py = r.h3[1] / r.h3[2];
    r.valid = fmaxf(fabsf(r.px), fabsf(r.py)) <= 1.f;
    return r;
}

constexpr int PT = 256;   // threads per point-kernel workgroup

// forward per point: X, Y and the rgb_s partial sums (sum of clamped |diff| over valid
// points and channels, number of valid elements) per workgroup
__global__ __launch_bounds__(PT) void k_pair_points(PairArgs a, float* __restrict__ X, float* __restrict__ Y,
                                                    float* __restrict__ rgbs_part) {
#pragma clang fp contract(off)
    __shared__ float red[PT / 64][2];
    const int i = blockIdx.x * PT + threadIdx.x;
    float s = 0.f, n = 0.f;
    if (i < a.P) {
        PairConst m;
        m.load(a);
        float x, y, pc1[3], pc2[3];
        pc_pixel(i, a.h, a.w, x, y);
        unproject_pt(m.Kinv, x, y, a.d1[i], pc1);
        unproject_pt(m.Kinv, x, y, a.d2[i], pc2);
        if (a.img1 != nullptr) {
            const Reproj r = reproject(a, m, pc1);
            if (r.valid) {
                const int hw = a.h * a.w;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float v1 = bilinear(a.img1 + c * hw, a.h, a.w, x, y);
                    const float v2 = bilinear(a.img2 + c * hw, a.h, a.w, r.px, r.py);
                    s += fminf(fmaxf(fabsf(v1 - v2), 0.f), 1.f);
                }
                n = 3.f;
            }
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            pc1[k] = pc1[k] / m.s1;
            pc2[k] = pc2[k] / m.s1;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            X[3 * i + k] = ((pc1[0] * m.R[3 * k] + pc1[1] * m.R[3 * k + 1]) + pc1[2] * m.R[3 * k + 2]) + m.t[k];
            Y[3 * i + k] = pc2[k];
        }
    }
    s = wave_sum(s);
    n = wave_sum(n);
    if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6][0] = s; red[threadIdx.x >> 6][1] = n; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float ss = 0.f, nn = 0.f;
        for (int wv = 0; wv < PT / 64; ++wv) { ss += red[wv][0]; nn += red[wv][1]; }
        rgbs_part[2 * blockIdx.x] = ss;
        rgbs_part[2 * blockIdx.x + 1] = nn;
    }
}

// chamfer nearest neighbours, both directions (blockIdx.z: 0 = X -> Y, 1 = Y -> X), the
// reference set split into gridDim.y chunks staged through LDS: part[z][chunk][i] =
// (first minimal |q - r| within the chunk, its index)
constexpr int NN_T = 256;
__global__ __launch_bounds__(NN_T) void k_nn_part(const float* __restrict__ X, const float* __restrict__ Y, int P,
                                                  int chunk, float2* __restrict__ part) {
    __shared__ float4 rs[NN_T];
    const float* Q = blockIdx.z == 0 ? X : Y;
    const float* Rf = blockIdx.z == 0 ? Y : X;
    const int i = blockIdx.x * NN_T + threadIdx.x;
    float px = 0.f, py = 0.f, pz = 0.f;
    if (i < P) { px = Q[3 * i]; py = Q[3 * i + 1]; pz = Q[3 * i + 2]; }
    const int j0 = blockIdx.y * chunk, j1 = min(P, j0 + chunk);
    float best = INFINITY;
    int bi = j0;
    for (int t0 = j0; t0 < j1; t0 += NN_T) {
        const int j = t0 + threadIdx.x;
        if (j < j1) rs[threadIdx.x] = make_float4(Rf[3 * j], Rf[3 * j + 1], Rf[3 * j + 2], 0.f);
        __syncthreads();
        const int nt = min(NN_T, j1 - t0);
        for (int k = 0; k < nt; ++k) {
            const float4 q = rs[k];
            const float dx = px - q.x, dy = py - q.y, dz = pz - q.z;
            const float d = sqrtf(__fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz)));
            if (d < best) { best = d; bi = t0 + k; }   // strict: first index on ties (torch.argmin)
        }
        __syncthreads();
    }
    if (i < P) part[((size_t)blockIdx.z * gridDim.y + blockIdx.y) * P + i] = make_float2(best, __int_as_float(bi));
}

// argmin over the chunks (in chunk order: ties keep the first index), the distance terms
// |X_i - Y_a(i)| and |Y_j - X_b(j)| as recomputed by the reference (linalg.norm of the
// gathered difference) and their per-workgroup sums
__global__ __launch_bounds__(PT) void k_nn_final(const float* __restrict__ X, const float* __restrict__ Y, int P,
                                                 int nchunk, const float2* __restrict__ part,
                                                 int* __restrict__ nn, float* __restrict__ dist_part) {
#pragma clang fp contract(off)
    __shared__ float red[PT / 64][2];
    const int i = blockIdx.x * PT + threadIdx.x;
    float dsum[2] = {0.f, 0.f};
    if (i < P) {
#pragma unroll
        for (int z = 0; z < 2; ++z) {
            float best = INFINITY;
            int bi = 0;
            for (int c = 0; c < nchunk; ++c) {
                const float2 v = part[((size_t)z * nchunk + c) * P + i];
                if (v.x < best) { best = v.x; bi = __float_as_int(v.y); }
            }
            if (!(best < INFINITY)) bi = __float_as_int(part[(size_t)z * nchunk * P + i].y);   // all NaN: chunk 0
            nn[z * P + i] = bi;
            const float* Q = z == 0 ? X : Y;
            const float* Rf = z == 0 ? Y : X;
            const float dx = Q[3 * i] - Rf[3 * bi], dy = Q[3 * i + 1] - Rf[3 * bi + 1], dz = Q[3 * i + 2] - Rf[3 * bi + 2];
            dsum[z] = sqrtf(dx * dx + dy * dy + dz * dz);
        }
    }
#pragma unroll
    for (int z = 0; z < 2; ++z) {
        const float s = wave_sum(dsum[z]);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][z] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float a = 0.f, b = 0.f;
        for (int wv = 0; wv < PT / 64; ++wv) { a += red[wv][0]; b += red[wv][1]; }
        dist_part[2 * blockIdx.x] = a;
        dist_part[2 * blockIdx.x + 1] = b;
    }
}

// one workgroup: loss_pc = mean |X - Y[a]| + mean |Y - X[b]| (losses.py:116-150),
// loss_rgb_s = sum / count over the valid elements, 0 without any (losses.py:79-87, 152-159);
// out = {pc, rgb_s, count}
__global__ __launch_bounds__(256) void k_pair_reduce(const float* __restrict__ dist_part,
                                                     const float* __restrict__ rgbs_part, int nblk, int P,
                                                     float* __restrict__ out) {
    __shared__ float red[4][4];
    float a = 0.f, b = 0.f, s = 0.f, n = 0.f;
    for (int k = threadIdx.x; k < nblk; k += blockDim.x) {
        a += dist_part[2 * k]; b += dist_part[2 * k + 1];
        if (rgbs_part) { s += rgbs_part[2 * k]; n += rgbs_part[2 * k + 1]; }
    }
    a = wave_sum(a); b = wave_sum(b); s = wave_sum(s); n = wave_sum(n);
    if ((threadIdx.x & 63) == 0) {
        const int wv = threadIdx.x >> 6;
        red[wv][0] = a; red[wv][1] = b; red[wv][2] = s; red[wv][3] = n;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float A = 0.f, B = 0.f, S = 0.f, N = 0.f;
        for (int wv = 0; wv < (int)(blockDim.x >> 6); ++wv) { A += red[wv][0]; B += red[wv][1]; S += red[wv][2]; N += red[wv][3]; }
        out[0] = A / (float)P + B / (float)P;
        out[1] = N > 0.f ? S / N : 0.f;
        out[2] = N;
    }
}

// ---------------------------------------------------------------------------- backward
// chamfer terms whose gradient lands on a gathered point: d|X_i - Y_a(i)| / dY_a(i) and
// d|Y_j - X_b(j)| / dX_b(j), scatter-added as 64-bit fixed point: each term is g * u with
// u = -(Q_i - R_j) / |Q_i - R_j| in [-1, 1], and u * 2^48 (rounded) is added by an integer
// atomic.  Integer sums do not depend on the order the atomics land in, so the gradient is the
// same bits on every run (float atomics are not: a resumed run would drift from the uninterrupted
// one in the last bit); the scale g = go_pc / P is applied once per point when the sums are read
// (pair_scattered).  The scale: a point of one cloud gathers at most the other cloud's P terms,
// each |u| 2^e <= 2^e, so P 2^e < 2^63 needs e <= 62 - ceil(log2 P): 2^48 up to P = 2^14
// (every V_KITTI depth grid; cfg3's P = 7 285), smaller beyond (pair_fix_scale)
__host__ __device__ inline double pair_fix_scale(int P) {
    int b = 0;
    while (b < 31 && (1LL << b) < (long long)P) ++b;
    const int e = 62 - b < 48 ? 62 - b : 48;
    return (double)(1LL << e);
}
__global__ __launch_bounds__(PT) void k_pair_bwd_scatter(const float* __restrict__ X, const float* __restrict__ Y,
                                                         int P, const int* __restrict__ nn,
                                                         unsigned long long* __restrict__ gX,
                                                         unsigned long long* __restrict__ gY) {
    const int i = blockIdx.x * PT + threadIdx.x;
    if (i >= P) return;
    const double fix = pair_fix_scale(P);
#pragma unroll
    for (int z = 0; z < 2; ++z) {
        const float* Q = z == 0 ? X : Y;
        const float* Rf = z == 0 ? Y : X;
        unsigned long long* gR = z == 0 ? gY : gX;
        const int j = nn[z * P + i];
        const float dx = Q[3 * i] - Rf[3 * j], dy = Q[3 * i + 1] - Rf[3 * j + 1], dz = Q[3 * i + 2] - Rf[3 * j + 2];
        const float d = sqrtf(dx * dx + dy * dy + dz * dz);
        if (d > 0.f) {
            atomicAdd(&gR[3 * j], (unsigned long long)llrint((double)(-dx / d) * fix));
            atomicAdd(&gR[3 * j + 1], (unsigned long long)llrint((double)(-dy / d) * fix));
            atomicAdd(&gR[3 * j + 2], (unsigned long long)llrint((double)(-dz / d) * fix));
        }
    }
}

// a point's scattered chamfer gradient: its fixed-point sum times g (one rounding to float)
__device__ __forceinline__ float pair_scattered(const unsigned long long* s, int k, double g, double fix) {
    return (float)((double)(long long)s[k] * (g / fix));
}

// per point: the direct chamfer terms plus the scattered ones -> dX_i, dY_i; the rgb_s term
// -> d pc1_rot; then d1 / d2 gradients and the R, t, scale partials of the workgroup
// (part[block][13] = {R (9), t (3), s1})
__global__ __launch_bounds__(PT) void k_pair_bwd_points(PairArgs a, const float* __restrict__ X,
                                                        const float* __restrict__ Y, const int* __restrict__ nn,
                                                        const float* __restrict__ go_pc,
                                                        const float* __restrict__ go_rgbs,
                                                        const float* __restrict__ red_out,
                                                        const unsigned long long* __restrict__ gX,
                                                        const unsigned long long* __restrict__ gY,
                                                        float* __restrict__ g_d1, float* __restrict__ g_d2,
                                                        float* __restrict__ part) {
    __shared__ float red[PT / 64][13];
    const int i = blockIdx.x * PT + threadIdx.x;
    const int P = a.P;
    float acc[13];
#pragma unroll
    for (int k = 0; k < 13; ++k) acc[k] = 0.f;
    if (i < P) {
        PairConst m;
        m.load(a);
        const float gpc = go_pc ? *go_pc / (float)P : 0.f;
        float x, y, pc1[3], pc2[3];
        pc_pixel(i, a.h, a.w, x, y);
        unproject_pt(m.Kinv, x, y, a.d1[i], pc1);
        unproject_pt(m.Kinv, x, y, a.d2[i], pc2);
        // dX_i, dY_i: own terms + scattered terms
        float gx[3], gy[3];
        const double gsc = (double)gpc;   // the scatter's g
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            gx[k] = gX ? pair_scattered(gX + 3 * i, k, gsc, pair_fix_scale(P)) : 0.f;
            gy[k] = gY ? pair_scattered(gY + 3 * i, k, gsc, pair_fix_scale(P)) : 0.f;
        }
        if (go_pc) {
#pragma unroll
            for (int z = 0; z < 2; ++z) {
                const float* Q = z == 0 ? X : Y;
                const float* Rf = z == 0 ? Y : X;
                const int j = nn[z * P + i];
                const float dx = Q[3 * i] - Rf[3 * j], dy = Q[3 * i + 1] - Rf[3 * j + 1], dz = Q[3 * i + 2] - Rf[3 * j + 2];
                const float d = sqrtf(dx * dx + dy * dy + dz * dz);
                if (d > 0.f) {
                    const float f = gpc / d;
                    float* gq = z == 0 ? gx : gy;
                    gq[0] += f * dx; gq[1] += f * dy; gq[2] += f * dz;
                }
            }
        }
        // X = R (pc1 / s1) + t, Y = pc2 / s1
        float gpc1[3] = {0.f, 0.f, 0.f}, gpc2[3];
        float ps1[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) ps1[k] = pc1[k] / m.s1;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                acc[3 * r + c] += gx[r] * ps1[c];
                gpc1[c] += m.R[3 * r + c] * gx[r] / m.s1;
            }
            acc[9 + r] += gx[r];
        }
        float gs = 0.f;   // d/ds1 of pc / s1 = -pc / s1^2
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float rg = 0.f;
#pragma unroll
            for (int r = 0; r < 3; ++r) rg += m.R[3 * r + c] * gx[r];
            gs -= rg * pc1[c] / (m.s1 * m.s1);
            gs -= gy[c] * pc2[c] / (m.s1 * m.s1);
            gpc2[c] = gy[c] / m.s1;
        }
        acc[12] += gs;
        // rgb_s: d/d(v2_c) of clamp(|v1_c - v2_c|, 0, 1) / N  (N valid elements)
        if (a.img1 != nullptr && go_rgbs != nullptr && red_out[2] > 0.f) {
            const Reproj r = reproject(a, m, pc1);
            if (r.valid && !r.bad) {
                const int hw = a.h * a.w;
                const float g = *go_rgbs / red_out[2];
                float gpx = 0.f, gpy = 0.f;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float v1 = bilinear(a.img1 + c * hw, a.h, a.w, x, y);
                    float dpx, dpy;
                    const float v2 = bilinear(a.img2 + c * hw, a.h, a.w, r.px, r.py, &dpx, &dpy);
                    const float e = v1 - v2;
                    const float ae = fabsf(e);
                    // abs' = sign (0 at 0); clamp(., 0, 1) passes the gradient on [0, 1]
                    const float gv2 = (ae <= 1.f) ? -g * (e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f)) : 0.f;
                    gpx += gv2 * dpx;
                    gpy += gv2 * dpy;
                }
                // p = h3[:2] / h3[2]
                const float iz = 1.f / r.h3[2];
                float gh[3] = {gpx * iz, gpy * iz, -(gpx * r.px + gpy * r.py) * iz};
                float gq[3];
#pragma unroll
                for (int c = 0; c < 3; ++c) gq[c] = gh[0] * m.K[c] + gh[1] * m.K[4 + c] + gh[2] * m.K[8 + c];
                // q = R pc1 + t
#pragma unroll
                for (int rr = 0; rr < 3; ++rr) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) acc[3 * rr + c] += gq[rr] * pc1[c];
                    acc[9 + rr] += gq[rr];
                }
                if (!a.rgbs_detach_scale) {
#pragma unroll
                    for (int c = 0; c < 3; ++c)
#pragma unroll
                        for (int rr = 0; rr < 3; ++rr) gpc1[c] += m.R[3 * rr + c] * gq[rr];
                }
            }
        }
        // pc = inv(K)[:3] [x d, y d, d, 1]  ->  d pc / d d = inv(K)[:3,:3] (x, y, 1)
        float u[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) u[r] = m.Kinv[4 * r] * x + m.Kinv[4 * r + 1] * y + m.Kinv[4 * r + 2];
        if (g_d1) g_d1[i] = gpc1[0] * u[0] + gpc1[1] * u[1] + gpc1[2] * u[2];
        if (g_d2) g_d2[i] = gpc2[0] * u[0] + gpc2[1] * u[1] + gpc2[2] * u[2];
    }
#pragma unroll
    for (int k = 0; k < 13; ++k) {
        const float s = wave_sum(acc[k]);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][k] = s;
    }
    __syncthreads();
    if (threadIdx.x < 13) {
        float s = 0.f;
        for (int wv = 0; wv < PT / 64; ++wv) s += red[wv][threadIdx.x];
        part[13 * blockIdx.x + threadIdx.x] = s;
    }
}

__global__ __launch_bounds__(64) void k_pair_bwd_reduce(const float* __restrict__ part, int nblk,
                                                        float* __restrict__ out13) {
    const int k = threadIdx.x;
    if (k >= 13) return;
    float s = 0.f;
    for (int b = 0; b < nblk; ++b) s += part[13 * b + k];
    out13[k] = s;
}

}  // namespace nerf

using namespace nerf;

static int fill_args(PairArgs& a, const float* d1, const float* d2, int h, int w, const float* K16,
                     const float* Rt16, const float* s1, float nl, const float* img1, const float* img2,
                     int rgbs_detach_scale) {
    NERF_CHECK_PTR(d1); NERF_CHECK_PTR(d2); NERF_CHECK_PTR(K16); NERF_CHECK_PTR(Rt16);
    NERF_CHECK(h > 1 && w > 1, "nerf_pair: resolution %dx%d", h, w);
    NERF_CHECK((img1 == nullptr) == (img2 == nullptr), "nerf_pair: img1 and img2 go together");
    NERF_CHECK((long long)h * w < (1LL << 28), "nerf_pair: %dx%d points", h, w);
    a.d1 = d1; a.d2 = d2; a.h = h; a.w = w; a.P = h * w;
    a.Kg = K16; a.Rtg = Rt16; a.s1g = s1; a.nl = nl;
    a.img1 = img1; a.img2 = img2; a.rgbs_detach_scale = rgbs_detach_scale;
    return NERF_OK;
}

extern "C" int nerf_pair_workspace(int n_points, int* n_chunks, int64_t* floats) {
    NERF_CHECK(n_points > 0, "%s: n_points=%d", __func__, n_points);
    const int qb = (n_points + NN_T - 1) / NN_T;
    int nc = 2048 / (2 * qb);
    if (nc < 1) nc = 1;
    const int maxc = (n_points + NN_T - 1) / NN_T;
    if (nc > maxc) nc = maxc;
    if (n_chunks) *n_chunks = nc;
    const int64_t nb = (n_points + PT - 1) / PT;
    // X, Y (3P each), NN partials (2 * nc * P float2), rgb_s and distance partials (2 nb each),
    // out (3 + 1 pad)
    if (floats) *floats = 6LL * n_points + 4LL * nc * n_points + 4 * nb + 4;
    return NERF_OK;
}

extern "C" int nerf_pair_forward(const float* d1, const float* d2, int h, int w, const float* K16,
                                 const float* Rt16, const float* s1, float nl, const float* img1,
                                 const float* img2, float* work, int* nn, float* out3, void* stream) {
    PairArgs a;
    const int rc = fill_args(a, d1, d2, h, w, K16, Rt16, s1, nl, img1, img2, 0);
    if (rc != NERF_OK) return rc;
    NERF_CHECK_PTR(work); NERF_CHECK_PTR(nn); NERF_CHECK_PTR(out3);
    const int P = a.P;
    int nc = 1;
    nerf_pair_workspace(P, &nc, nullptr);
    const int nb = (P + PT - 1) / PT;
    float* X = work;
    float* Y = X + 3 * (size_t)P;
    float2* part = reinterpret_cast<float2*>(Y + 3 * (size_t)P);
    float* rgbs_part = reinterpret_cast<float*>(part + 2 * (size_t)nc * P);
    float* dist_part = rgbs_part + 2 * nb;
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(k_pair_points, dim3(nb), dim3(PT), 0, s, a, X, Y, rgbs_part);
    const int chunk = ((P + nc - 1) / nc + NN_T - 1) / NN_T * NN_T;
    hipLaunchKernelGGL(k_nn_part, dim3((P + NN_T - 1) / NN_T, nc, 2), dim3(NN_T), 0, s, X, Y, P, chunk, part);
    hipLaunchKernelGGL(k_nn_final, dim3(nb), dim3(PT), 0, s, X, Y, P, nc, part, nn, dist_part);
    hipLaunchKernelGGL(k_pair_reduce, dim3(1), dim3(256), 0, s, dist_part, img1 ? rgbs_part : nullptr, nb, P, out3);
    return check_launch(__func__);
}

extern "C" int nerf_pair_backward(const float* d1, const float* d2, int h, int w, const float* K16,
                                  const float* Rt16, const float* s1, float nl, const float* img1,
                                  const float* img2, int rgbs_detach_scale, const float* work, const int* nn,
                                  const float* out3, const float* go_pc, const float* go_rgbs, float* gXY,
                                  float* g_d1, float* g_d2, float* g13, float* part13, void* stream) {
    PairArgs a;
    const int rc = fill_args(a, d1, d2, h, w, K16, Rt16, s1, nl, img1, img2, rgbs_detach_scale);
    if (rc != NERF_OK) return rc;
    NERF_CHECK_PTR(work); NERF_CHECK_PTR(nn); NERF_CHECK_PTR(out3); NERF_CHECK_PTR(gXY); NERF_CHECK_PTR(g13);
    NERF_CHECK_PTR(part13);
    const int P = a.P;
    const int nb = (P + PT - 1) / PT;
    const float* X = work;
    const float* Y = X + 3 * (size_t)P;
    NERF_CHECK(((uintptr_t)gXY & 7u) == 0, "%s: gXY must be 8-byte aligned (64-bit fixed-point sums)", __func__);
    unsigned long long* gX = reinterpret_cast<unsigned long long*>(gXY);
    unsigned long long* gY = gX + 3 * (size_t)P;
    hipStream_t s = as_stream(stream);
    (void)hipMemsetAsync(gXY, 0, 6 * (size_t)P * sizeof(unsigned long long), s);
    if (go_pc != nullptr) hipLaunchKernelGGL(k_pair_bwd_scatter, dim3(nb), dim3(PT), 0, s, X, Y, P, nn, gX, gY);
    hipLaunchKernelGGL(k_pair_bwd_points, dim3(nb), dim3(PT), 0, s, a, X, Y, nn, go_pc, go_rgbs, out3,
                       (const unsigned long long*)gX, (const unsigned long long*)gY, g_d1, g_d2, part13);
    hipLaunchKernelGGL(k_pair_bwd_reduce, dim3(1), dim3(64), 0, s, (const float*)part13, nb, g13);
    return check_launch(__func__);
}
