// Ray prologue and loss epilogue of the training step.
//
// Everything the reference runs around the per-sample work of one step, as a handful of
// launches instead of ~150 ATen ones:
//   * k_sample_rays   : randperm(H*W)[:R] + the pixel / colour gathers (training.py:277-283,
//                       common.py:13-40) -- one workgroup, a deterministic LDS hash set;
//   * k_mat4          : batched 4x4 inverse, SO(3) x R^3 pose composition (common.py:277-310,
//                       poses.py:23-31) and the unprojection matrix
//                       inv(scale) @ inv(world) @ inv(K) (common.py:139-141, 205-208);
//   * k_camera_rays   : origin, unit direction, |P1 - o|, d_src and the depth mask per ray
//                       (rendering.py:52-80) and its backward (pose / distortion learning);
//   * k_ray_loss(_bwd): rgb l1/l2 + masked depth l1 + l2_mean and their gradients
//                       (losses.py:28-33, 60-66, 164-228).
// All are launch-latency bound (a few KB per step); the point is the launch count.
#include "common.hpp"
#include "mat4.hpp"

#include <cmath>

namespace nerf {

// ------------------------------------------------------------------------------------
// Philox-4x32-10 (Salmon et al., SC'11), the counter-based generator torch's CUDA/HIP RNG
// also uses; keyed by the host seed, counter = (ray slot, round, stream, 0).
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
    constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
        const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += W0;
        k.y += W1;
    }
    return c;
}

// uniform integer in [0, n) from 64 random bits: floor(u * n / 2^64) (bias < n / 2^64)
__device__ __forceinline__ uint32_t uniform_below(uint4 r, uint32_t n) {
    const uint64_t u = ((uint64_t)r.x << 32) | r.y;
    return (uint32_t)__umul64hi(u, (uint64_t)n);
}

constexpr int SR_THREADS = 1024;
constexpr int SR_LOG_TABLE = 14;
constexpr int SR_TABLE = 1 << SR_LOG_TABLE;     // hash slots; load factor <= 1/4 at SR_MAX
constexpr int SR_PER_THREAD = NERF_SAMPLE_MAX_RAYS / SR_THREADS;
constexpr uint32_t SR_EMPTY = 0xFFFFFFFFu;
constexpr int SR_MAX_ROUNDS = NERF_SAMPLE_MAX_ROUNDS;

// R distinct pixel indices drawn uniformly from [0, n_pix) -- the set randperm(n)[:R]
// returns, with its own (deterministic) generator.  Each pending ray slot draws a
// candidate, inserts it into an LDS hash set (linear probing), and the slot whose
// (round, slot) key is smallest owns the value; the others draw again next round.  The
// outcome depends only on (seed, n, R), never on wave timing.
__global__ __launch_bounds__(SR_THREADS) void k_sample_rays(int n_pix, int R, uint2 key, int width, int height,
                                                            const float* __restrict__ img,
                                                            int64_t* __restrict__ idx, float* __restrict__ pix,
                                                            float* __restrict__ rgb, int* __restrict__ status,
                                                            unsigned long long* __restrict__ ctr) {
    __shared__ uint32_t table[SR_TABLE];
    __shared__ uint32_t owner[SR_TABLE];
    const int tid = threadIdx.x;
    // device step counter (graph replays): the key mixes in the counter, thread 0 advances it
    // once every thread has read it (the kernel is a single workgroup)
    const unsigned long long c = ctr ? *ctr : 0ull;
    if (ctr) {
        const unsigned long long m = (c + 1) * 0x9E3779B97F4A7C15ull;
        key.x ^= (uint32_t)m;
        key.y ^= (uint32_t)(m >> 32);
    }
    for (int i = tid; i < SR_TABLE; i += SR_THREADS) {
        table[i] = SR_EMPTY;
        owner[i] = 0xFFFFFFFFu;
    }
    __syncthreads();
    uint32_t val[SR_PER_THREAD], pos[SR_PER_THREAD];
    bool pend[SR_PER_THREAD];
#pragma unroll
    for (int q = 0; q < SR_PER_THREAD; ++q) pend[q] = (tid + q * SR_THREADS) < R;
    int round = 0, done = 0;
    for (; round < SR_MAX_ROUNDS; ++round) {
#pragma unroll
        for (int q = 0; q < SR_PER_THREAD; ++q) {
            if (!pend[q]) continue;
            const uint32_t slot = tid + q * SR_THREADS;
            const uint32_t v = uniform_below(philox4x32_10(make_uint4(slot, round, 0x5a4d, 0), key), n_pix);
            val[q] = v;
            uint32_t h = (v * 2654435761u) >> (32 - SR_LOG_TABLE);
            while (true) {
                const uint32_t old = atomicCAS(&table[h], SR_EMPTY, v);
                if (old == SR_EMPTY || old == v) break;
                h = (h + 1) & (SR_TABLE - 1);
            }
            pos[q] = h;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < SR_PER_THREAD; ++q)
            if (pend[q]) atomicMin(&owner[pos[q]], (uint32_t)(round * NERF_SAMPLE_MAX_RAYS + tid + q * SR_THREADS));
        __syncthreads();
        int any = 0;
#pragma unroll
        for (int q = 0; q < SR_PER_THREAD; ++q) {
            if (!pend[q]) continue;
            if (owner[pos[q]] == (uint32_t)(round * NERF_SAMPLE_MAX_RAYS + tid + q * SR_THREADS)) pend[q] = false;
            else any = 1;
        }
        if (!__syncthreads_or(any)) { done = 1; break; }
    }
    if (tid == 0 && status != nullptr) *status = done ? round + 1 : 0;   // rounds used, 0 = gave up
    const int hw = width * height;
#pragma unroll
    for (int q = 0; q < SR_PER_THREAD; ++q) {
        const int j = tid + q * SR_THREADS;
        if (j >= R) continue;
        const uint32_t v = pend[q] ? 0u : val[q];
        idx[j] = v;
        if (pix != nullptr) {   // arange_pixels: 2*col/(W-1) - 1, 2*row/(H-1) - 1 (common.py:36-39)
            const int row = v / width, col = v - row * width;
            pix[2 * j] = 2.f * (float)col / (float)(width - 1) - 1.f;
            pix[2 * j + 1] = 2.f * (float)row / (float)(height - 1) - 1.f;
        }
        if (rgb != nullptr) {   // img.view(1,3,H*W).permute(0,2,1)[:, idx]
            rgb[3 * j] = img[v];
            rgb[3 * j + 1] = img[hw + v];
            rgb[3 * j + 2] = img[2 * hw + v];
        }
    }
    if (ctr != nullptr) {
        __syncthreads();
        if (tid == 0) *ctr = c + 1;
    }
}

__global__ void k_mat4_inv(const float* __restrict__ a, int n, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float m[16], r[16];
    load4(a + 16 * (size_t)i, m);
    inverse4(m, r);
    store4(out + 16 * (size_t)i, r);
}

// c2w = [Exp(r) | t; 0 0 0 1] @ init (common.py:290-310, poses.py:27-30);
// Exp(r) = I + sin(th)/th [r]x + (1 - cos th)/th^2 [r]x^2,  th = |r| + 1e-15
__global__ void k_pose_c2w(const float* __restrict__ r, const float* __restrict__ t,
                           const float* __restrict__ init, float* __restrict__ out) {
#pragma clang fp contract(off)
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const float x = r[0], y = r[1], z = r[2];
    const float th = sqrtf(x * x + y * y + z * z) + 1e-15f;
    const float K[9] = {0.f, -z, y, z, 0.f, -x, -y, x, 0.f};
    float KK[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) KK[3 * i + j] = K[3 * i] * K[j] + K[3 * i + 1] * K[3 + j] + K[3 * i + 2] * K[6 + j];
    const float s = sinf(th) / th, c = (1.f - cosf(th)) / (th * th);
    float m[16];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) m[4 * i + j] = ((i == j ? 1.f : 0.f) + s * K[3 * i + j]) + c * KK[3 * i + j];
        m[4 * i + 3] = t[i];
    }
    m[12] = 0.f; m[13] = 0.f; m[14] = 0.f; m[15] = 1.f;
    if (init != nullptr) {
        float b[16], o[16];
        load4(init, b);
        matmul4(m, b, o);
        store4(out, o);
    } else {
        store4(out, m);
    }
}

// Backward of k_pose_c2w (the closed form of torch autograd through common.py:277-310):
// G = g @ init^T is the gradient of [R | t]; g_t = G[:3, 3];
//   dL/dK = s G_R + c (G_R K^T + K^T G_R),  dL/dth = s'(th) <G_R, K> + c'(th) <G_R, K^2>,
//   s = sin th / th, c = (1 - cos th) / th^2, dth/dr = r / |r| (0 at r = 0, torch's norm
//   subgradient), K = [r]x so dL/dx = dK[2][1] - dK[1][2] etc.  Evaluated in f64.
__global__ void k_pose_c2w_bwd(const float* __restrict__ r, const float* __restrict__ init,
                               const float* __restrict__ g, float* __restrict__ gr, float* __restrict__ gt) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double G[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0.0;
            if (init != nullptr) {
                for (int k = 0; k < 4; ++k) s += (double)g[4 * i + k] * (double)init[4 * j + k];
            } else {
                s = g[4 * i + j];
            }
            G[4 * i + j] = s;
        }
    if (gt != nullptr)
        for (int i = 0; i < 3; ++i) gt[i] = (float)G[4 * i + 3];
    if (gr == nullptr) return;
    const double x = r[0], y = r[1], z = r[2];
    const double nr = sqrt(x * x + y * y + z * z);
    const double th = (double)(float)((float)nr + 1e-15f);
    const double K[9] = {0.0, -z, y, z, 0.0, -x, -y, x, 0.0};
    double KK[9], GR[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            KK[3 * i + j] = K[3 * i] * K[j] + K[3 * i + 1] * K[3 + j] + K[3 * i + 2] * K[6 + j];
            GR[3 * i + j] = G[4 * i + j];
        }
    const double sn = sin(th), cs = cos(th);
    const double s = sn / th, c = (1.0 - cs) / (th * th);
    const double ds = cs / th - sn / (th * th);
    const double dc = sn / (th * th) - 2.0 * (1.0 - cs) / (th * th * th);
    double dK[9], gk = 0.0, gkk = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double a = 0.0, b = 0.0;   // (G_R K^T)_ij, (K^T G_R)_ij
            for (int k = 0; k < 3; ++k) {
                a += GR[3 * i + k] * K[3 * j + k];
                b += K[3 * k + i] * GR[3 * k + j];
            }
            dK[3 * i + j] = s * GR[3 * i + j] + c * (a + b);
            gk += GR[3 * i + j] * K[3 * i + j];
            gkk += GR[3 * i + j] * KK[3 * i + j];
        }
    const double dth = ds * gk + dc * gkk;
    const double w = nr > 0.0 ? dth / nr : 0.0;
    gr[0] = (float)(dK[7] - dK[5] + w * x);
    gr[1] = (float)(dK[2] - dK[6] + w * y);
    gr[2] = (float)(dK[3] - dK[1] + w * z);
}

// d inv(A) = -Y dA Y  ->  gA = -Y^T g Y^T, batched ([n][4][4])
__global__ void k_mat4_inv_bwd(const float* __restrict__ y, const float* __restrict__ g, int n,
                               float* __restrict__ ga) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float Y[16], Yt[16], G[16], t[16], o[16];
    load4(y + 16 * (size_t)i, Y);
    load4(g + 16 * (size_t)i, G);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) Yt[4 * a + b] = Y[4 * b + a];
    matmul4(Yt, G, t);
    matmul4(t, Yt, o);
#pragma unroll
    for (int k = 0; k < 16; ++k) o[k] = -o[k];
    store4(ga + 16 * (size_t)i, o);
}

// C = A @ B (batched [n][4][4]) and its backward gA = g B^T, gB = A^T g (either optional)
__global__ void k_mat4_mul(const float* __restrict__ a, const float* __restrict__ b, int n, float* __restrict__ c) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float A[16], B[16], C[16];
    load4(a + 16 * (size_t)i, A);
    load4(b + 16 * (size_t)i, B);
    matmul4(A, B, C);
    store4(c + 16 * (size_t)i, C);
}
__global__ void k_mat4_mul_bwd(const float* __restrict__ a, const float* __restrict__ b, const float* __restrict__ g,
                               int n, float* __restrict__ ga, float* __restrict__ gb) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float A[16], B[16], G[16], T[16], O[16];
    load4(g + 16 * (size_t)i, G);
    if (ga != nullptr) {
        load4(b + 16 * (size_t)i, B);
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int q = 0; q < 4; ++q) T[4 * p + q] = B[4 * q + p];
        matmul4(G, T, O);
        store4(ga + 16 * (size_t)i, O);
    }
    if (gb != nullptr) {
        load4(a + 16 * (size_t)i, A);
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int q = 0; q < 4; ++q) T[4 * p + q] = A[4 * q + p];
        matmul4(T, G, O);
        store4(gb + 16 * (size_t)i, O);
    }
}

// Backward of k_unproject: M = Si Wi Ki with Xi = inv(X) and d inv(A) = -Ai dA Ai:
//   gK = -Ki^T ((Si Wi)^T g) Ki^T,  gW = -Wi^T (Si^T g Ki^T) Wi^T,  gS = -Si^T (g (Wi Ki)^T) Si^T
// (each output optional; inverses = {Ki, Wi, Si} from the forward)
__global__ void k_unproject_bwd(const float* __restrict__ inverses, const float* __restrict__ g,
                                float* __restrict__ gK, float* __restrict__ gW, float* __restrict__ gS) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    float Ki[16], Wi[16], Si[16], G[16], A[16], B[16], T[16], O[16];
    load4(inverses, Ki);
    load4(inverses + 16, Wi);
    load4(inverses + 32, Si);
    load4(g, G);
    auto tr = [](const float (&x)[16], float (&y)[16]) {
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int q = 0; q < 4; ++q) y[4 * p + q] = x[4 * q + p];
    };
    auto neg_sandwich = [&](const float (&Xi)[16], const float (&inner)[16], float* out) {
        float Xt[16], t1[16], t2[16];
        tr(Xi, Xt);
        matmul4(Xt, inner, t1);
        matmul4(t1, Xt, t2);
#pragma unroll
        for (int k = 0; k < 16; ++k) t2[k] = -t2[k];
        store4(out, t2);
    };
    if (gK != nullptr) {
        matmul4(Si, Wi, A);
        tr(A, T);
        matmul4(T, G, O);
        neg_sandwich(Ki, O, gK);
    }
    if (gW != nullptr) {
        tr(Si, T);
        matmul4(T, G, A);
        tr(Ki, T);
        matmul4(A, T, O);
        neg_sandwich(Wi, O, gW);
    }
    if (gS != nullptr) {
        matmul4(Wi, Ki, B);
        tr(B, T);
        matmul4(G, T, O);
        neg_sandwich(Si, O, gS);
    }
}

// Depth-prior distortion on gathered prior values (training.py:259-264, 325-329, 346-347):
// y = d s + t (or (d + t) s with shift_first), then y < lo -> lo (the pc resize's
// d[d < nearest_limit] = nearest_limit; lo = -inf for none).  Backward: the clamped entries
// pass no gradient; g_s = sum g (d [+ t]), g_t = sum g (x s with shift_first) -- one
// workgroup, a fixed-order tree (deterministic).
constexpr int AF_THREADS = 1024;
__global__ __launch_bounds__(AF_THREADS) void k_depth_affine(const float* __restrict__ d, int n,
                                                             const float* __restrict__ s, const float* __restrict__ t,
                                                             int shift_first, float lo, float* __restrict__ y) {
#pragma clang fp contract(off)
    const float sc = s[0], sh = t[0];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float v = shift_first ? (d[i] + sh) * sc : d[i] * sc + sh;
        y[i] = v < lo ? lo : v;
    }
}
__global__ __launch_bounds__(AF_THREADS) void k_depth_affine_bwd(const float* __restrict__ d, int n,
                                                                 const float* __restrict__ s,
                                                                 const float* __restrict__ t, int shift_first,
                                                                 float lo, const float* __restrict__ g,
                                                                 float* __restrict__ gs, float* __restrict__ gt) {
#pragma clang fp contract(off)
    __shared__ float red[2][AF_THREADS / 64];
    const float sc = s[0], sh = t[0];
    float as = 0.f, at = 0.f;
    for (int i = threadIdx.x; i < n; i += AF_THREADS) {
        const float v = shift_first ? (d[i] + sh) * sc : d[i] * sc + sh;
        if (v < lo) continue;
        const float gi = g[i];
        as += shift_first ? gi * (d[i] + sh) : gi * d[i];
        at += shift_first ? gi * sc : gi;
    }
    as = wave_sum(as);
    at = wave_sum(at);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][w] = as; red[1][w] = at; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float a = 0.f, b = 0.f;
        for (int k = 0; k < AF_THREADS / 64; ++k) { a += red[0][k]; b += red[1][k]; }
        if (gs) gs[0] = a;
        if (gt) gt[0] = b;
    }
}

// M = (inv(scale) @ inv(world)) @ inv(K)  (common.py:139-141); inverses kept for backward
__global__ void k_unproject(const float* __restrict__ K, const float* __restrict__ world,
                            const float* __restrict__ scale, float* __restrict__ M, float* __restrict__ inverses) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    float a[16], ki[16], wi[16], si[16], t[16], m[16];
    load4(K, a);
    inverse4(a, ki);
    load4(world, a);
    inverse4(a, wi);
    load4(scale, a);
    inverse4(a, si);
    matmul4(si, wi, t);
    matmul4(t, ki, m);
    store4(M, m);
    if (inverses != nullptr) {
        store4(inverses, ki);
        store4(inverses + 16, wi);
        store4(inverses + 32, si);
    }
}

// ------------------------------------------------------------------------------------
// camera rays (rendering.py:52-80 with transform_to_world / origin_to_world, common.py:112-215):
//   o = M[:3,3];  v = M[:3,:3] (x, y, 1) = P1 - o;  |v|;  P_d - o = M[:3,:3] (x d, y d, d)
//   normalise: dir = v/|v|, d_src = |P_d - o|;  else dir = v, d_src = |P_d - o| / |v|
//   mask = isfinite(d_src) & d_src != 0;  view = -dir (use_ray_dir) or 1
constexpr int CR_THREADS = 256;

__global__ __launch_bounds__(CR_THREADS) void k_camera_rays(const float* __restrict__ Mg, const float* __restrict__ pix,
                                                            const float* __restrict__ depth, int R, int flags,
                                                            float* __restrict__ cam, float* __restrict__ ray,
                                                            float* __restrict__ view, float* __restrict__ ray_norm,
                                                            float* __restrict__ d_src, uint8_t* __restrict__ mask) {
#pragma clang fp contract(off)
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    float M[16];
    load4(Mg, M);
    const float x = pix[2 * r], y = pix[2 * r + 1];
    float v[3], n2 = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        v[i] = (M[4 * i] * x + M[4 * i + 1] * y) + M[4 * i + 2];
        n2 = n2 + v[i] * v[i];
    }
    const float n = sqrtf(n2);
    float ds = 1.f;
    if (depth != nullptr) {
        const float d = depth[r];
        const float xd = x * d, yd = y * d;
        float q2 = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const float pi = (M[4 * i] * xd + M[4 * i + 1] * yd) + M[4 * i + 2] * d;
            q2 = q2 + pi * pi;
        }
        ds = sqrtf(q2);
    }
    const bool normalise = flags & NERF_RAYS_NORMALISE;
    if (!normalise) ds = ds / n;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float di = normalise ? v[i] / n : v[i];
        cam[3 * r + i] = M[4 * i + 3];
        ray[3 * r + i] = di;
        if (view != nullptr) view[3 * r + i] = (flags & NERF_RAYS_VIEW_ONES) ? 1.f : -di;
    }
    ray_norm[r] = n;
    d_src[r] = ds;
    if (mask != nullptr) mask[r] = (isfinite(ds) && ds != 0.f) ? 1 : 0;
}

// Backward: gradient of (cam, ray, view, ray_norm, d_src) w.r.t. M (16, rows 3 stay 0) and
// depth.  One workgroup; per-thread partial sums over a fixed ray stride, then a fixed-order
// tree (deterministic).  Rays with d = 0 contribute nothing through d_src, as torch's norm
// backward at 0.
__global__ __launch_bounds__(1024) void k_camera_rays_bwd(const float* __restrict__ Mg, const float* __restrict__ pix,
                                                          const float* __restrict__ depth, int R, int flags,
                                                          const float* __restrict__ g_cam,
                                                          const float* __restrict__ g_ray,
                                                          const float* __restrict__ g_view,
                                                          const float* __restrict__ g_norm,
                                                          const float* __restrict__ g_dsrc,
                                                          float* __restrict__ gM, float* __restrict__ g_depth) {
    __shared__ float red[16][12];
    float M[16];
    load4(Mg, M);
    const bool normalise = flags & NERF_RAYS_NORMALISE;
    float acc[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) acc[i] = 0.f;
    for (int r = threadIdx.x; r < R; r += blockDim.x) {
        const float x = pix[2 * r], y = pix[2 * r + 1];
        float v[3], n2 = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            v[i] = M[4 * i] * x + M[4 * i + 1] * y + M[4 * i + 2];
            n2 += v[i] * v[i];
        }
        const float n = sqrtf(n2), inv_n = 1.f / n;
        float gv[3] = {0.f, 0.f, 0.f};
        // direction (and view = -direction)
        float gd[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            gd[i] = g_ray ? g_ray[3 * r + i] : 0.f;
            if (g_view && !(flags & NERF_RAYS_VIEW_ONES)) gd[i] -= g_view[3 * r + i];
        }
        if (normalise) {
            const float dot = (gd[0] * v[0] + gd[1] * v[1] + gd[2] * v[2]) * inv_n;
#pragma unroll
            for (int i = 0; i < 3; ++i) gv[i] += (gd[i] - v[i] * inv_n * dot) * inv_n;
        } else {
#pragma unroll
            for (int i = 0; i < 3; ++i) gv[i] += gd[i];
        }
        if (g_norm) {
            const float g = g_norm[r] * inv_n;
#pragma unroll
            for (int i = 0; i < 3; ++i) gv[i] += g * v[i];
        }
        float gdep = 0.f;
        if (depth != nullptr && g_dsrc != nullptr) {
            const float d = depth[r], g = g_dsrc[r];
            if (d != 0.f) {
                const float ad = fabsf(d), sd = d > 0.f ? 1.f : -1.f;
                if (normalise) {            // d_src = |d| |v|
                    gdep = g * sd * n;
                    const float gg = g * ad * inv_n;
#pragma unroll
                    for (int i = 0; i < 3; ++i) gv[i] += gg * v[i];
                } else {                    // d_src = |d| |v| / |v|
                    gdep = g * sd;
                }
            }
        }
        if (g_depth != nullptr) g_depth[r] = gdep;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            acc[3 * i] += gv[i] * x;
            acc[3 * i + 1] += gv[i] * y;
            acc[3 * i + 2] += gv[i];
            if (g_cam) acc[9 + i] += g_cam[3 * r + i];
        }
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        const float s = wave_sum(acc[i]);
        if (lane == 0) red[wv][i] = s;
    }
    __syncthreads();
    if (threadIdx.x < 16) {
        const int e = threadIdx.x, row = e >> 2, col = e & 3;
        float s = 0.f;
        if (row < 3) {
            const int slot = col < 3 ? 3 * row + col : 9 + row;
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w][slot];
        }
        gM[e] = s;
    }
}

// ------------------------------------------------------------------------------------
// losses.py:28-33 (rgb l1/l2 over R rays), :60-66 (depth l1 over the masked rays), l2_mean
// = mse(rgb, gt), total = w_rgb l_rgb + w_depth l_depth.  out = {total, l_rgb, l_depth,
// l2_mean} (four scalars), cnt = number of depth rays used (for the backward).
__global__ __launch_bounds__(1024) void k_ray_loss(const float* __restrict__ rgb, const float* __restrict__ gt,
                                                   int R, const float* __restrict__ dp,
                                                   const float* __restrict__ dg, const uint8_t* __restrict__ mask,
                                                   int M, int l1, float w_rgb, float w_depth,
                                                   float* __restrict__ total, float* __restrict__ l_rgb,
                                                   float* __restrict__ l_depth, float* __restrict__ l2_mean,
                                                   float* __restrict__ cnt_out) {
    __shared__ float red[16][4];
    float s2 = 0.f, s1 = 0.f, sd = 0.f, cnt = 0.f;
    for (int i = threadIdx.x; i < 3 * R; i += blockDim.x) {
        const float e = rgb[i] - gt[i];
        s2 += e * e;
        s1 += fabsf(e);
    }
    if (dp != nullptr)
        for (int i = threadIdx.x; i < M; i += blockDim.x) {
            if (mask == nullptr || mask[i]) {
                sd += fabsf(dp[i] - dg[i]);
                cnt += 1.f;
            }
        }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    s2 = wave_sum(s2); s1 = wave_sum(s1); sd = wave_sum(sd); cnt = wave_sum(cnt);
    if (lane == 0) { red[wv][0] = s2; red[wv][1] = s1; red[wv][2] = sd; red[wv][3] = cnt; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float a = 0.f, b = 0.f, c = 0.f, n = 0.f;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { a += red[w][0]; b += red[w][1]; c += red[w][2]; n += red[w][3]; }
        const float lr = (l1 ? b : a) / (float)R;
        const float ld = dp != nullptr ? c / fmaxf(n, 1.f) : 0.f;   // 0 (not 0/0) with no valid ray
        *l_rgb = lr;
        *l_depth = ld;
        *l2_mean = a / (float)(3 * R);
        *total = w_rgb * lr + w_depth * ld;
        *cnt_out = n;
    }
}

// d(total, l_rgb, l_depth, l2_mean)/d(rgb, depth_pred, depth_gt) contracted with the
// upstream scalars go[0..3] (NULL = 0)
__global__ void k_ray_loss_bwd(const float* __restrict__ rgb, const float* __restrict__ gt, int R,
                               const float* __restrict__ dp, const float* __restrict__ dg,
                               const uint8_t* __restrict__ mask, int M, int l1, float w_rgb, float w_depth,
                               const float* __restrict__ go_total, const float* __restrict__ go_rgb,
                               const float* __restrict__ go_depth, const float* __restrict__ go_l2,
                               const float* __restrict__ cnt, float* __restrict__ g_rgb,
                               float* __restrict__ g_dp, float* __restrict__ g_dg) {
    const float gt_ = go_total ? *go_total : 0.f;
    const float a_rgb = gt_ * w_rgb + (go_rgb ? *go_rgb : 0.f);
    const float a_dep = gt_ * w_depth + (go_depth ? *go_depth : 0.f);
    const float a_l2 = go_l2 ? *go_l2 : 0.f;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (g_rgb != nullptr && i < 3 * R) {
        const float e = rgb[i] - gt[i];
        const float dl = l1 ? (e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f)) : 2.f * e;
        g_rgb[i] = a_rgb * dl / (float)R + a_l2 * (2.f * e) / (float)(3 * R);
    }
    if (dp != nullptr && i < M) {
        float g = 0.f;
        if (mask == nullptr || mask[i]) {
            const float e = dp[i] - dg[i];
            g = a_dep * (e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f)) / fmaxf(*cnt, 1.f);
        }
        if (g_dp) g_dp[i] = g;
        if (g_dg) g_dg[i] = -g;
    }
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_sample_rays(int n_pix, int n_rays, uint64_t seed, int width, int height, const float* img,
                                int64_t* idx, float* pixels, float* rgb, int* status, uint64_t* seed_counter,
                                void* stream) {
    NERF_CHECK_PTR(idx);
    NERF_CHECK(n_rays > 0 && n_rays <= NERF_SAMPLE_MAX_RAYS, "%s: n_rays=%d outside 1..%d", __func__, n_rays,
               NERF_SAMPLE_MAX_RAYS);
    NERF_CHECK(n_pix >= 2 * n_rays, "%s: n_pix=%d < 2*n_rays=%d (draw a permutation instead)", __func__, n_pix,
               2 * n_rays);
    NERF_CHECK(pixels == nullptr || (width > 1 && height > 1 && width * height == n_pix),
               "%s: pixels need width, height > 1 with width*height == n_pix", __func__);
    NERF_CHECK(rgb == nullptr || (img != nullptr && width * height == n_pix), "%s: rgb needs img [3][n_pix]",
               __func__);
    const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
    hipLaunchKernelGGL(k_sample_rays, dim3(1), dim3(SR_THREADS), 0, as_stream(stream), n_pix, n_rays, key,
                       width, height, img, idx, pixels, rgb, status,
                       reinterpret_cast<unsigned long long*>(seed_counter));
    return check_launch(__func__);
}

extern "C" int nerf_mat4_inv(const float* a, int n, float* out, void* stream) {
    NERF_CHECK_PTR(a); NERF_CHECK_PTR(out);
    NERF_CHECK(n > 0, "%s: n=%d", __func__, n);
    hipLaunchKernelGGL(k_mat4_inv, dim3((n + 63) / 64), dim3(64), 0, as_stream(stream), a, n, out);
    return check_launch(__func__);
}

extern "C" int nerf_pose_c2w(const float* r, const float* t, const float* init_c2w, float* c2w, void* stream) {
    NERF_CHECK_PTR(r); NERF_CHECK_PTR(t); NERF_CHECK_PTR(c2w);
    hipLaunchKernelGGL(k_pose_c2w, dim3(1), dim3(64), 0, as_stream(stream), r, t, init_c2w, c2w);
    return check_launch(__func__);
}

extern "C" int nerf_unproject_matrix(const float* K, const float* world, const float* scale, float* M,
                                     float* inverses, void* stream) {
    NERF_CHECK_PTR(K); NERF_CHECK_PTR(world); NERF_CHECK_PTR(scale); NERF_CHECK_PTR(M);
    hipLaunchKernelGGL(k_unproject, dim3(1), dim3(64), 0, as_stream(stream), K, world, scale, M, inverses);
    return check_launch(__func__);
}

extern "C" int nerf_pose_c2w_bwd(const float* r, const float* init_c2w, const float* g_c2w, float* g_r, float* g_t,
                                 void* stream) {
    NERF_CHECK_PTR(r); NERF_CHECK_PTR(g_c2w);
    hipLaunchKernelGGL(k_pose_c2w_bwd, dim3(1), dim3(64), 0, as_stream(stream), r, init_c2w, g_c2w, g_r, g_t);
    return check_launch(__func__);
}

extern "C" int nerf_mat4_inv_bwd(const float* inv_a, const float* g, int n, float* g_a, void* stream) {
    NERF_CHECK_PTR(inv_a); NERF_CHECK_PTR(g); NERF_CHECK_PTR(g_a);
    NERF_CHECK(n > 0, "%s: n=%d", __func__, n);
    hipLaunchKernelGGL(k_mat4_inv_bwd, dim3((n + 63) / 64), dim3(64), 0, as_stream(stream), inv_a, g, n, g_a);
    return check_launch(__func__);
}

extern "C" int nerf_mat4_mul(const float* a, const float* b, int n, float* c, void* stream) {
    NERF_CHECK_PTR(a); NERF_CHECK_PTR(b); NERF_CHECK_PTR(c);
    NERF_CHECK(n > 0, "%s: n=%d", __func__, n);
    hipLaunchKernelGGL(k_mat4_mul, dim3((n + 63) / 64), dim3(64), 0, as_stream(stream), a, b, n, c);
    return check_launch(__func__);
}

extern "C" int nerf_mat4_mul_bwd(const float* a, const float* b, const float* g, int n, float* g_a, float* g_b,
                                 void* stream) {
    NERF_CHECK_PTR(g);
    NERF_CHECK(n > 0, "%s: n=%d", __func__, n);
    NERF_CHECK(g_a == nullptr || b != nullptr, "%s: g_a needs b", __func__);
    NERF_CHECK(g_b == nullptr || a != nullptr, "%s: g_b needs a", __func__);
    hipLaunchKernelGGL(k_mat4_mul_bwd, dim3((n + 63) / 64), dim3(64), 0, as_stream(stream), a, b, g, n, g_a, g_b);
    return check_launch(__func__);
}

extern "C" int nerf_unproject_matrix_bwd(const float* inverses, const float* g_M, float* g_K, float* g_world,
                                         float* g_scale, void* stream) {
    NERF_CHECK_PTR(inverses); NERF_CHECK_PTR(g_M);
    hipLaunchKernelGGL(k_unproject_bwd, dim3(1), dim3(64), 0, as_stream(stream), inverses, g_M, g_K, g_world,
                       g_scale);
    return check_launch(__func__);
}

extern "C" int nerf_depth_affine(const float* d, int n, const float* scale, const float* shift, int shift_first,
                                 float lo, float* y, void* stream) {
    NERF_CHECK_PTR(d); NERF_CHECK_PTR(scale); NERF_CHECK_PTR(shift); NERF_CHECK_PTR(y);
    NERF_CHECK(n > 0, "%s: n=%d", __func__, n);
    const int blocks = (n + AF_THREADS - 1) / AF_THREADS;
    hipLaunchKernelGGL(k_depth_affine, dim3(blocks < 64 ? blocks : 64), dim3(AF_THREADS), 0, as_stream(stream), d,
                       n, scale, shift, shift_first, lo, y);
    return check_launch(__func__);
}

extern "C" int nerf_depth_affine_bwd(const float* d, int n, const float* scale, const float* shift, int shift_first,
                                     float lo, const float* g, float* g_scale, float* g_shift, void* stream) {
    NERF_CHECK_PTR(d); NERF_CHECK_PTR(scale); NERF_CHECK_PTR(shift); NERF_CHECK_PTR(g);
    NERF_CHECK(n > 0, "%s: n=%d", __func__, n);
    hipLaunchKernelGGL(k_depth_affine_bwd, dim3(1), dim3(AF_THREADS), 0, as_stream(stream), d, n, scale, shift,
                       shift_first, lo, g, g_scale, g_shift);
    return check_launch(__func__);
}

extern "C" int nerf_camera_rays(const float* M, const float* pixels, const float* depth, int n_rays, int flags,
                                float* cam, float* ray, float* view, float* ray_norm, float* d_src, uint8_t* mask,
                                void* stream) {
    NERF_CHECK_PTR(M); NERF_CHECK_PTR(pixels); NERF_CHECK_PTR(cam); NERF_CHECK_PTR(ray);
    NERF_CHECK_PTR(ray_norm); NERF_CHECK_PTR(d_src);
    NERF_CHECK(n_rays > 0, "%s: n_rays=%d", __func__, n_rays);
    hipLaunchKernelGGL(k_camera_rays, dim3((n_rays + CR_THREADS - 1) / CR_THREADS), dim3(CR_THREADS), 0,
                       as_stream(stream), M, pixels, depth, n_rays, flags, cam, ray, view, ray_norm, d_src, mask);
    return check_launch(__func__);
}

extern "C" int nerf_camera_rays_bwd(const float* M, const float* pixels, const float* depth, int n_rays, int flags,
                                    const float* g_cam, const float* g_ray, const float* g_view,
                                    const float* g_norm, const float* g_dsrc, float* gM, float* g_depth,
                                    void* stream) {
    NERF_CHECK_PTR(M); NERF_CHECK_PTR(pixels); NERF_CHECK_PTR(gM);
    NERF_CHECK(n_rays > 0, "%s: n_rays=%d", __func__, n_rays);
    NERF_CHECK(g_depth == nullptr || depth != nullptr, "%s: g_depth without depth", __func__);
    hipLaunchKernelGGL(k_camera_rays_bwd, dim3(1), dim3(1024), 0, as_stream(stream), M, pixels, depth, n_rays,
                       flags, g_cam, g_ray, g_view, g_norm, g_dsrc, gM, g_depth);
    return check_launch(__func__);
}

extern "C" int nerf_ray_loss(const float* rgb, const float* rgb_gt, int n_rays, const float* depth_pred,
                             const float* depth_gt, const uint8_t* mask, int n_depth, int rgb_l1, float w_rgb,
                             float w_depth, float* total, float* l_rgb, float* l_depth, float* l2_mean,
                             float* cnt, void* stream) {
    NERF_CHECK_PTR(rgb); NERF_CHECK_PTR(rgb_gt); NERF_CHECK_PTR(total); NERF_CHECK_PTR(l_rgb);
    NERF_CHECK_PTR(l_depth); NERF_CHECK_PTR(l2_mean); NERF_CHECK_PTR(cnt);
    NERF_CHECK(n_rays > 0, "%s: n_rays=%d", __func__, n_rays);
    NERF_CHECK(depth_pred == nullptr || (depth_gt != nullptr && n_depth >= 0), "%s: depth_pred without depth_gt",
               __func__);
    hipLaunchKernelGGL(k_ray_loss, dim3(1), dim3(1024), 0, as_stream(stream), rgb, rgb_gt, n_rays, depth_pred,
                       depth_gt, mask, n_depth, rgb_l1, w_rgb, w_depth, total, l_rgb, l_depth, l2_mean, cnt);
    return check_launch(__func__);
}

extern "C" int nerf_ray_loss_bwd(const float* rgb, const float* rgb_gt, int n_rays, const float* depth_pred,
                                 const float* depth_gt, const uint8_t* mask, int n_depth, int rgb_l1, float w_rgb,
                                 float w_depth, const float* go_total, const float* go_rgb, const float* go_depth,
                                 const float* go_l2, const float* cnt, float* g_rgb, float* g_depth_pred,
                                 float* g_depth_gt, void* stream) {
    NERF_CHECK_PTR(rgb); NERF_CHECK_PTR(rgb_gt); NERF_CHECK_PTR(cnt);
    NERF_CHECK(n_rays > 0, "%s: n_rays=%d", __func__, n_rays);
    NERF_CHECK((g_depth_pred == nullptr && g_depth_gt == nullptr) || depth_pred != nullptr,
               "%s: depth gradients without depth inputs", __func__);
    const int n = 3 * n_rays > n_depth ? 3 * n_rays : n_depth;
    hipLaunchKernelGGL(k_ray_loss_bwd, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), rgb, rgb_gt, n_rays,
                       depth_pred, depth_gt, mask, n_depth, rgb_l1, w_rgb, w_depth, go_total, go_rgb, go_depth,
                       go_l2, cnt, g_rgb, g_depth_pred, g_depth_gt);
    return check_launch(__func__);
}
