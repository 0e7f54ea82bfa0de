/*
 * nerf_hip.h -- C-ABI of the MI355X-native NoPe-NeRF render + training hot path.
 *
 * The reference (js0n-lai/my-nope-nerf) is pure Python/PyTorch and has no FFI; its
 * "plugin boundary" for this path is the Python call chain
 *   Trainer.train_step -> nope_nerf.forward -> Renderer.nope_nerf -> OfficialStaticNerf.forward
 *   -> Loss.forward -> loss.backward -> Adam.step
 * (model/training.py:70-100, model/network.py:19-33, model/rendering.py:36-168,
 *  model/official_nerf.py:60-119, model/losses.py:164-228).  Each entry point below
 * replaces the ATen work one of those functions launches;
 * the replaced reference lines are cited per function.  The host side that binds
 * these symbols is my-nope-nerf_amd/model/_hip.py (ctypes); INTEGRATION.md shows it.
 *
 * Conventions (all entry points):
 *  - plain device pointers (fp32 unless stated, row-major, 16-byte aligned),
 *    element counts / leading dimensions in elements, a hipStream_t passed as void*;
 *  - nothing allocates, nothing synchronises the host: work is enqueued on `stream`;
 *  - return 0 on success, a negative NERF_E* code on a bad argument or launch
 *    failure; nerf_hip_last_error() returns the message (thread-local).
 */
#ifndef NERF_HIP_H
#define NERF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NERF_OK 0
#define NERF_EINVAL (-1)   /* bad argument (null pointer, shape, alignment) */
#define NERF_ELAUNCH (-2)  /* hipGetLastError after a launch */

/* Row tile of every per-sample GEMM: sample buffers are padded to a multiple of it. */
#define NERF_ROW_TILE 128

/* ABI version: 5 added nerf_prof_read_kinds and nerf_render_eval_fused, 6 the 4x4-chain
 * backwards (nerf_pose_c2w_bwd, nerf_mat4_inv_bwd, nerf_mat4_mul(_bwd), nerf_unproject_matrix_bwd)
 * and the depth-prior distortion (nerf_depth_affine(_bwd)), 7 nerf_linear_fwd_heads, 8 nerf_heads_bwd_mode,
 * 9 precision mode 2 as the default, 10 nerf_mlp_chain_train, 11 nerf_linear_bwd_weight_seg and
 * nerf_field_backward, 12 nerf_mlp_chain_bwd, nerf_field_bwd.bwd_chain, TN policy 8 and the
 * Adam hyper slot 6 (1 - beta2), 13 the chain images (nerf_pack_desc dst_cs / dst_cts, nerf_field_bwd
 * wt_cimg) and torch-exact Adam, 14 nerf_linear_bwd_weight_jobs and nerf_pair_backward's 12P gXY,
 * 15 the chain images' compact exponent arrays (nerf_pack_desc dst_cs / dst_cts) and
 * nerf_linear_bwd_weight_job_groups. */
#define NERF_HIP_ABI_VERSION 15
int nerf_hip_abi_version(void);
const char* nerf_hip_last_error(void);

/* ---------------------------------------------------------------------------
 * Samples + positional encodings.
 * Replaces Renderer.sample_uniform / sample_ndc z + pts (rendering.py:169-198,
 * linspace :89-90) and encode_position (official_nerf.py:99-119, L=10 / L=4).
 * pts = pts_o[r] + pts_d[r] * z[r,s];  z = lerp(near,far,s/(S-1)) jittered by
 * noise[r,s] in its stratified bin when noise != NULL (rendering.py:187-191).
 * view[r] is the (already negated) direction fed to the colour branch.
 * enc_p : [n_pad][64]  = [x(3), sin(2^i x)(3), cos(2^i x)(3) ... i<10, 0]   (63 + 1 pad)
 * enc_d : [n_pad][64]  = same with L=4 on view (27 + 37 pad)
 * z     : [n_pad]; rows >= R*S of all outputs are written as 0.
 * enc_p_rmax, enc_d_rmax (optional, [n_pad]): max |.| of each encoding row (the row scales
 * of GEMM precision mode 2).  enc_p_cmax, enc_d_cmax (optional, [n_pad/128][64], n_pad %
 * 128 == 0): per 128-row group an upper bound of max |.| per column -- exact for the three
 * coordinate columns, 1 for the sin / cos columns, 0 for the pad (column scales of mode 2).
 */
int nerf_encode_samples(const float* pts_o, const float* pts_d, const float* view,
                        const float* noise, int n_rays, int n_samples, int n_pad,
                        float near_z, float far_z, float* z, float* enc_p, float* enc_d,
                        float* enc_p_rmax, float* enc_d_rmax, float* enc_p_cmax, float* enc_d_cmax,
                        void* stream);

/* ---------------------------------------------------------------------------
 * Linear layer forward on FP32 MFMA (v_mfma_f32_32x32x2_f32).
 * Replaces nn.Linear (+ReLU) and the skip / colour torch.cat of
 * OfficialStaticNerf.infer_occ / forward (official_nerf.py:62-64, 88-91).
 *   y[m, n] = act( sum_k x1[m,k] w[n,k] + sum_k x2[m,k] w[n,k1+k] + bias[n] )
 * x1: [m][ldx1] (k1 cols used), x2: [m][ldx2] (k2 cols, may be NULL with k2 = 0),
 * w : [n][k1+k2] (padded packed weight), y: [m][ldy]. m % 128 == 0, n % 64 == 0,
 * k1 % 32 == 0, k2 % 32 == 0. relu: 0/1.  mask_out (optional): ReLU mask bits of y,
 * word [m][n/32] (row stride ldmo words), bit b of word w = y[m][32w+b] > 0.
 * w_split (optional, used by GEMM precision mode 1): the same weight as a bf16x3 split
 * image (nerf_pack_weights dst_s): element (plane p, row r, col c) at
 * w_split[((p*(K/8) + c/8)*w_split_rows + r)*8 + c%8], K = k1+k2; w_split may point at
 * a row offset inside a larger image whose row count is w_split_rows.  NULL: this call
 * runs on the exact-f32 kernel even in modes 1 and 2.  In mode 2 the image is the fp16
 * pair form written by nerf_pack_weights in that mode.
 * x1_rmax / x2_rmax ([m], precision mode 2, required there): max |x| over each row of the
 * segment (as written by the producer of x: nerf_encode_samples, this function, ...).
 * y_rmax (optional, mode 2 only): receives max |y| per row; with n > 256 (several column
 * blocks) it is max-accumulated and must be zeroed by the caller.
 * y_cmax (optional, mode 2 only): receives max |y| per column and 128-row group,
 * [m/128][n] (the column scales of nerf_linear_bwd_weight in mode 2).
 */
int nerf_linear_fwd(const float* x1, int ldx1, int k1, const float* x2, int ldx2, int k2,
                    const float* w, const uint16_t* w_split, int w_split_rows, const float* bias, float* y,
                    int ldy, int m, int n, int relu, uint32_t* mask_out, int ldmo,
                    const float* x1_rmax, const float* x2_rmax, float* y_rmax, float* y_cmax, void* stream);
/* nerf_linear_fwd with the output heads fused into its epilogue (precision mode 2, n = 128 or
 * 256 -- one column block holds whole output rows): raw4[r][raw_col + c] = sum_f y[r][f]
 * head_w[c][f] + head_b[c] for c < n_heads, head_w [n_heads][n] (16-byte aligned) -- the
 * density head on the trunk output (official_nerf.py:66, n_heads 1, raw_col 0) and the colour
 * head on the colour layer (official_nerf.py:91, n_heads 3, raw_col 1).  Per-row partial
 * dots are summed in a fixed order (deterministic). */
int nerf_linear_fwd_heads(const float* x1, int ldx1, int k1, const float* x2, int ldx2, int k2,
                          const float* w, const uint16_t* w_split, int w_split_rows, const float* bias,
                          float* y, int ldy, int m, int n, int relu, uint32_t* mask_out, int ldmo,
                          const float* x1_rmax, const float* x2_rmax, float* y_rmax, float* y_cmax,
                          const float* head_w, int n_heads, const float* head_b, float* raw4, int raw_col,
                          void* stream);

/* Backward w.r.t. the layer input (autograd of official_nerf.py:62-91).
 *   dx[m, j] = ( sum_o dy[m,o] wt[j,o]  + (u ? u[m*ldu] * v[j] : 0) ) * (mask ? bit(m,j) : 1)
 * wt: [n][k] = transpose of the packed weight restricted to the wanted input columns
 * (n = number of input columns produced, k = layer outputs), mask: ReLU mask bits of
 * the previous layer's output as written by nerf_linear_fwd (ldmask words per row) or
 * NULL.  m%128==0, n%64==0, k%32==0.  wt_split / wt_split_rows: optional bf16x3 image of
 * wt as for nerf_linear_fwd (K = k).  dy_rmax / dx_rmax / dx_cmax: row and column maxima as
 * x1_rmax / y_rmax / y_cmax of nerf_linear_fwd (mode 2). */
int nerf_linear_bwd_data(const float* dy, int lddy, int k, const float* wt, const uint16_t* wt_split,
                         int wt_split_rows, const float* u, int ldu, const float* v, const uint32_t* mask,
                         int ldmask, float* dx, int lddx, int m, int n, const float* dy_rmax, float* dx_rmax,
                         float* dx_cmax, void* stream);

/* Backward w.r.t. weight and bias, split over sample rows:
 *   slab[split][o][col0 + j] = sum_{rows of split} dy[row, o] * x[row, j]   (j < kin)
 *   bslab[split][o]          = sum_{rows of split} dy[row, o]   (if bslab != NULL)
 * dy: [m][lddy] (nout columns), x: [m][ldx] (kin columns), slab row stride ldslab.
 * Rows are split into `splits` equal chunks; nout % 64 == 0, kin % 64 == 0,
 * m % (32*splits) == 0.  dy_cmax [m/128][nout], x_cmax [m/128][kin] (optional, mode 2): upper
 * bounds of max |.| per column and 128-row group (as y_cmax of nerf_linear_fwd); given both and
 * splits of whole 128-row groups, mode 2 runs the fp16 pair kernel (column-scaled operands,
 * three products), else the bf16x3 one. */
int nerf_linear_bwd_weight(const float* dy, int lddy, int nout, const float* x, int ldx,
                           int kin, int m, int splits, float* slab, int ldslab, int col0,
                           float* bslab, const float* dy_cmax, const float* x_cmax, void* stream);

/* The weight gradient of a layer whose input is two segments [x1 | x2] (l4's [h3 | enc_p],
 * official_nerf.py:62-64; the colour layer's [f | enc_d], :88-90): the same slab as
 *   nerf_linear_bwd_weight(dy, .., x1, k1, .., col0 = 0, bslab, dy_cmax, x1_cmax) followed by
 *   nerf_linear_bwd_weight(dy, .., x2, k2, .., col0 = k1, NULL, dy_cmax, x2_cmax)
 * bit for bit.  In precision mode 2 under TN policy 7 with nout 256 or 128, k1 = 256, k2 = 64
 * and splits % 8 == 0 it is ONE launch whose column tiles of a split share an XCD, so dy is
 * read from HBM once (two launches read it twice); any other case runs the two calls. */
int nerf_linear_bwd_weight_seg(const float* dy, int lddy, int nout, const float* x1, int ldx1, int k1,
                               const float* x2, int ldx2, int k2, int m, int splits, float* slab, int ldslab,
                               float* bslab, const float* dy_cmax, const float* x1_cmax, const float* x2_cmax,
                               void* stream);

/* The weight gradients of n (1..8) layers of 256 outputs over 256 inputs with one split count
 * (the field's consecutive hidden layers, official_nerf.py:65-86 under training.py:92): the same
 * slabs as n nerf_linear_bwd_weight(dy_i, lddy_i, 256, x_i, ldx_i, 256, m, splits, slab_i,
 * ldslab_i, 0, bslab_i, dy_cmax_i, x_cmax_i) calls, bit for bit.  In precision mode 2 under TN
 * policy 8 with every job's column maxima it is ONE launch whose blocks walk the layers in
 * order (a layer's first loads overlap the previous layer's slab stores); otherwise the n calls. */
typedef struct nerf_wgrad_job {   /* (slab columns from 0, ldslab >= 256) */
    const float* dy; int lddy;
    const float* x; int ldx;
    float* slab; int ldslab;
    float* bslab;
    const float* dy_cmax; const float* x_cmax;
} nerf_wgrad_job;
int nerf_linear_bwd_weight_multi(const nerf_wgrad_job* jobs, int n, int m, int splits, void* stream);

/* Weight gradients of several shapes in one launch (ABI 14; the chain backward's weight-gradient
 * schedule 3, field_bwd.cpp): job i is nerf_linear_bwd_weight(dy_i, lddy_i, nout_i, x_i, ldx_i,
 * kin_i, m, splits_i, slab_i, ldslab_i, col0_i, bslab_i, dy_cmax_i, x_cmax_i), and the slabs are
 * those calls' bit for bit.  With S = `splits` (a multiple of 8) the shapes are 256 x 256 at S
 * splits, 256 x 64 at S or 2 S, 128 x 256 and 128 x 64 at 2 S; in precision mode 2 under TN
 * policy 8, with every job's column maxima and 128-row multiples per split, ONE launch of 2 S
 * blocks walks the jobs in order (k_wgrad_jobs); otherwise the n calls. */
typedef struct nerf_wgrad_tile_job {
    const float* dy; int lddy; int nout;
    const float* x; int ldx; int kin;
    int splits;
    float* slab; int ldslab; int col0;
    float* bslab;
    const float* dy_cmax; const float* x_cmax;
} nerf_wgrad_tile_job;
int nerf_linear_bwd_weight_jobs(const nerf_wgrad_tile_job* jobs, int n, int m, int splits, void* stream);
/* The same with the jobs in n_groups block groups (ABI 15): job i runs on group[i]'s own range of
 * 2 S blocks (one launch of n_groups x 2 S blocks), so two job lists share the chip side by side
 * at half the split count each -- half the split-K slab bytes for the same work.  The slabs are
 * those of the per-job calls at each job's split count, bit for bit; group == NULL with
 * n_groups == 1 is nerf_linear_bwd_weight_jobs. */
int nerf_linear_bwd_weight_job_groups(const nerf_wgrad_tile_job* jobs, const int* group, int n, int m, int splits,
                                      int n_groups, void* stream);

/* ---------------------------------------------------------------------------
 * The training backward of the field in one host call (ABI 11): FieldRunner.backward's
 * launch schedule -- composite backward (or a given graw4), heads, then per layer from the
 * colour layer down the input-gradient GEMM on `stream` and the weight gradient + slab
 * reduce on `side_stream` behind an event, the last `tail_main` layers' weight gradients on
 * `stream` after the chain, the encoding backward for ray gradients -- for hidden 256 /
 * colour 128 in GEMM precision mode 2 (the autograd of official_nerf.py:60-96 and
 * rendering.py:113-141 that training.py:92 runs).  The same launches in the same order as
 * the Python schedule, so the gradients are bit-identical to it; the host cost is a few
 * microseconds per launch instead of a ctypes call + temporaries each.  Layer index l:
 * 0..7 the trunk l0..l7, 8 the feature layer, 9 the colour layer.  On return `stream` has
 * waited for `side_stream`.  No allocation: temporaries live in `workspace`
 * (nerf_field_bwd_workspace_bytes). */
#define NERF_BWD_LAYERS 10
typedef struct nerf_field_bwd {
    int n_pad, n_rays, n_samples, flags, ray_grad, tail_main;   /* tail_main: the per-layer schedule only
                                                                   (bwd_chain = 0); ignored by the chain's */
    int bwd_chain;   /* 1: the input gradients by nerf_mlp_chain_bwd (ABI 12), 0: the per-layer schedule */
    /* forward state (nerf_mlp_chain_train / nerf_encode_samples outputs) */
    const float* z;
    const float* raw4;
    const float* enc_p;
    const float* enc_d;
    const float* enc_p_cmax;
    const float* enc_d_cmax;
    const float* act[NERF_BWD_LAYERS];      /* layer outputs [n_pad][256] (colour layer [n_pad][128]) */
    const uint32_t* mask[NERF_BWD_LAYERS];  /* ReLU words [n_pad][out/32] (feature layer: NULL) */
    const float* cmax[NERF_BWD_LAYERS];     /* column maxima [n_pad/128][out] (colour layer: NULL) */
    const float* pts_o;                     /* ray inputs of nerf_encode_samples (ray_grad only) */
    const float* pts_d;
    const float* view;
    /* packed parameters (nerf_pack_weights, mode 2) */
    const float* wt[NERF_BWD_LAYERS];       /* f32 W^T [kp][out_p] */
    const uint16_t* wt_img[NERF_BWD_LAYERS];/* fp16 pair image of W^T */
    const uint16_t* wt_cimg[NERF_BWD_LAYERS];/* its chain image (nerf_pack_desc dst_cts; ABI 13): the
                                               input-gradient chain's operand (bwd_chain = 1) */
    const float* wd;                        /* fc_density weight [256], 16-byte aligned */
    const float* wc;                        /* fc_rgb weight [3][128] */
    /* upstream gradient: graw4 [n_pad][4], or g_rgb [R][3] + g_dist [R] through the composite */
    const float* g_rgb;
    const float* g_dist;
    const float* graw4;
    /* outputs, reference layout */
    float* gw[NERF_BWD_LAYERS];
    float* gb[NERF_BWD_LAYERS];
    float* g_wd;
    float* g_bd;
    float* g_wc;
    float* g_bc;
    float* g_pts_o;
    float* g_pts_d;
    float* g_view;
    void* workspace;
} nerf_field_bwd;
size_t nerf_field_bwd_workspace_bytes(int n_pad, int ray_grad);
int nerf_field_backward(const nerf_field_bwd* args, void* stream, void* side_stream);

/* Recommended `splits` for nerf_linear_bwd_weight at this shape and tile policy. */
int nerf_linear_bwd_weight_splits(int nout, int kin, int m);

/* Sum the split-K slabs (slab[split][nout][ldslab], bslab[split][nout]) into a
 * parameter gradient in the reference layout (unpadded gw[nout_ref][kin_ref],
 * gb[nout_ref]); accumulate != 0 adds into gw/gb. */
int nerf_slab_reduce(const float* slab, int splits, int nout, int ldslab, int nout_ref,
                     int kin_ref, const float* bslab, float* gw, float* gb, int accumulate,
                     void* stream);

/* GEMM tile policy (tuning knob; 0 = built-in default).  nt: 1 = 128x128 / 4 waves,
 * 2 = 128x256 / 8 waves, 3 = 256x256 / 8 waves (exact-f32 kernels; the fp16 pair kernels
 * run 128x256 tiles at 3, and the fused-heads launches always one column block);
 * tn (weight gradient): 3 = 256x256 tiles, 7 = in the split modes a 256 x 256 layer as
 * XCD-paired 256x128 column tiles of 8 waves, the 64-wide inputs' 256x64 tile and the
 * colour layer's 128x256 tile at 8 waves; 8 (default) = the splits and tiles of 7 with the
 * 4-wave kernels of wgrad.hip in precision mode 2 (bit-identical slabs; shapes they do not
 * cover run as 7).  The policy changes nerf_linear_bwd_weight_splits (7 and 8 alike). */
int nerf_gemm_set_policy(int nt_policy, int tn_policy);

/* f32 arithmetic of the GEMM family (process-wide; default 2 since ABI 9):
 *   0  exact-f32 v_mfma_f32_32x32x2_f32 (a k-ordered f32 fma chain);
 *   1  f32 emulated on v_mfma_f32_32x32x16_bf16: operands split into three bf16
 *      words (exact), the six cross products >= 2^-16 |a||b| accumulated in f32.
 *      nerf_linear_fwd / nerf_linear_bwd_data use it when given the weight's split
 *      image (w_split / wt_split), nerf_linear_bwd_weight always.
 *   2  f32 emulated on v_mfma_f32_32x32x16_f16: every operand row (nerf_linear_fwd,
 *      nerf_linear_bwd_data; nerf_linear_bwd_weight: every column of a split, from the
 *      producers' per-128-row-group column maxima, else it runs as 1) is scaled by a power of two
 *      (row max -> [2^14, 2^15)) and split into two fp16 words (exact to 2^-22), the
 *      three products hi.lo + lo.hi + hi.hi accumulated in f32, the scales undone in the
 *      epilogue.  Needs the row maxima of the A operand (x1_rmax, ...) and the fp16 pair
 *      weight image (nerf_pack_weights in mode 2).
 * Returns NERF_EINVAL for other modes. */
int nerf_gemm_set_precision(int mode);
int nerf_gemm_get_precision(void);
/* Diagnostics only (results are wrong while non-zero): bits 0-3 NT GEMM (1 = skip the
 * epilogue stores, 2 = skip the K-loop loads), bits 4-7 TN GEMM (16 = skip the slab stores,
 * 32 = skip the K-loop loads, 64 = skip the bias column sums). */
int nerf_gemm_debug_stamps(void* buf);
int nerf_gemm_debug_ablate(int mask);

/* ---------------------------------------------------------------------------
 * Fused forward chain of the whole field MLP (GEMM precision mode 2, hidden width 256,
 * colour width 128).  Replaces OfficialStaticNerf.infer_occ / forward's ten linears with
 * their ReLUs, the skip concat and the colour concat (official_nerf.py:60-91) -- the ten
 * nerf_linear_fwd calls -- by ONE launch that keeps each 128-row tile's activations in
 * registers from layer to layer (row-scaled fp16 pairs, three MFMA products, as mode 2).
 * layers[10] = l0..l7, fc_feature, rgb_layers[0]; per layer the fp16 pair weight image
 * written by nerf_pack_weights in mode 2 ([out_p][K]: K = 64, 256, 256, 256, 320, 256,
 * 256, 256, 256, 320; out_p = 256 except 128 for the colour layer; for THIS entry the plain
 * image dst_s, for nerf_mlp_chain_train and nerf_render_eval_fused the chain image dst_cs
 * with perm_k = 256 for l1..lr, 0 for l0 -- ABI 13) and the bias; optional
 * outputs: the f32 activation (the backward's saved tensor; NULL in eval renders), the ReLU
 * bits and the column maxima per 128-row group (mode 2's weight-gradient scales; not for
 * the colour layer).  enc_p / enc_d and their row maxima as written by nerf_encode_samples.
 * n_pad % 128 == 0. */
typedef struct {
    const uint16_t* img;   /* fp16 pair image of the packed weight */
    int img_rows;          /* its rows (>= the layer's outputs) */
    const float* bias;     /* [outputs] (the colour layer: padded to 128) */
    float* out; int ldo;   /* f32 output [n_pad][ldo] or NULL */
    uint32_t* mask; int ldmask;   /* ReLU bits [n_pad][ldmask words] or NULL */
    float* cmax;           /* [n_pad/128][outputs] or NULL */
} nerf_chain_layer;
int nerf_mlp_chain_fwd(const float* enc_p, const float* enc_d, const float* enc_p_rmax,
                       const float* enc_d_rmax, int n_pad, const nerf_chain_layer* layers, void* stream);
/* The training forward chain (official_nerf.py:60-96 under training.py:70-92): the ten
 * linears of nerf_mlp_chain_fwd in ONE launch at two waves per SIMD, saving what the per-layer
 * kernels (nerf_linear_fwd) save for the backward -- every layer output (out, mandatory; the
 * f32 epilogue values -- ABI 12 saved the trunk layers' rebuilt from the fp16 pair the next
 * layer consumed), the weight images being the chain images (dst_cs, ABI 13),
 * the ReLU words (mask, mandatory except for lf, ldmask even) and the per-128-row-group column
 * maxima (cmax, mandatory except for the colour layer) -- plus raw4 [n_pad][4] = (sigma_raw,
 * rgb logits) from the density / colour heads in the l7 / colour-layer epilogues (wd [256],
 * bd [1], wc [3][128] padded, bc [3], as nerf_render_eval_fused).  Encodings and their row
 * maxima as nerf_encode_samples writes them.  GEMM precision mode 2, hidden width 256. */
int nerf_mlp_chain_train(const float* enc_p, const float* enc_d, const float* enc_p_rmax, const float* enc_d_rmax,
                         int n_pad, const nerf_chain_layer* layers, const float* wd, const float* bd, const float* wc,
                         const float* bc, float* raw4, void* stream);
/* The fused per-ray eval render (BASELINE.json north_star; rendering.py:36-168 with eval_ /
 * no noise, official_nerf.py:60-119): ONE launch per ray chunk computes, per 128-row block
 * of S-sample rays (S divides 128), the stratified sample positions and both positional
 * encodings in-kernel, runs the ten linears of nerf_mlp_chain_fwd with the activations in
 * registers, the density / colour heads in the layer epilogues and the sigma -> alpha ->
 * exclusive-product composite of the block's rays -- no per-sample tensor touches HBM
 * except alpha [R][S] and z [R*S] (outputs of the reference's out-dict).
 * pts_o / pts_d / view: [R][3] ray origins, sample directions, view directions; layers: the
 * ten chain descriptors with out / mask / cmax NULL; wd [256], bd [1]: fc_density; wc [3][128]
 * (padded), bc [3]: fc_rgb.  flags as nerf_composite_fwd.  Outputs rgb [R][3], dist [R]
 * (ray distance; the caller applies the eval z-depth division), alpha [R][S], z [R*S].
 * GEMM precision mode 2, hidden width 256.  Replaces rendering.py:89-141 +
 * official_nerf.py:60-96 for the render callers (extracting_images.py:65-76,
 * training.py:103-165). */
int nerf_render_eval_fused(const float* pts_o, const float* pts_d, const float* view, int n_rays, int n_samples,
                           float near_z, float far_z, int flags, const nerf_chain_layer* layers, const float* wd,
                           const float* bd, const float* wc, const float* bc, float* rgb, float* dist, float* alpha,
                           float* z, void* stream);

/* The input-gradient chain (ABI 12; official_nerf.py:60-96 backward as training.py:92 runs
 * it, for hidden 256 / colour 128 in GEMM precision mode 2): ONE launch computes, per
 * 128-row block, dyr (the colour layer's output gradient: graw4's rgb-logit gradients . fc_rgb,
 * gated by the colour layer's ReLU words -- replaces nerf_heads_bwd_mode 1) and the nine input
 * gradients dx = dy W [+ d sigma_raw x w_density at the feature layer], masked by the ReLU
 * words of each layer's input, with dy resident in registers as row-scaled fp16 pairs and
 * W^T streamed by LDS-DMA -- the nine nerf_linear_bwd_data launches of the per-layer path.
 * Layer order i = 0..8: colour layer, feature layer, l7 .. l1.  D_0 = dyr [n_pad][128],
 * D_i (i >= 1) the gradient at the output of forward layer 9 - i ([n_pad][256]; D_9 is the
 * gradient at l0's output).  Every D_i is saved (the f32 value; ABI 12 saved it rebuilt from
 * the fp16 pair consumed), with its per-128-row-group column maxima
 * ([n_pad/128][128 or 256]) and row maxima ([n_pad]) -- the weight-gradient and ray-gradient
 * GEMMs' operands. */
typedef struct nerf_chain_bwd {
    const float* graw4;             /* [n_pad][4]: d(sigma_raw, rgb logits), 16-byte aligned */
    const uint32_t* hr_mask;        /* the colour layer's ReLU words [n_pad][ld_hr_mask >= 4] */
    int ld_hr_mask;
    const float* wd;                /* fc_density weight [256], 16-byte aligned */
    const float* wc;                /* fc_rgb weight [3][128] (padded) */
    const uint16_t* wt_img[9];      /* chain images of W^T (nerf_pack_desc dst_cts: rows = input
                                       features, K in chain order; ABI 13), layer order */
    int wt_img_rows[9];
    const uint32_t* in_mask[9];     /* ReLU words of layer i's input [n_pad][ld >= 8] (i = 0 unused) */
    int ld_in_mask[9];
    float* dy[10];                  /* D_0 .. D_9 (lddy 128 for D_0, 256 for the others) */
    int lddy[10];
    float* dy_cmax[10];
    float* dy_rmax[10];
    float* scratch;                 /* >= 512 floats of device scratch */
    int n_pad;
} nerf_chain_bwd;
int nerf_mlp_chain_bwd(const nerf_chain_bwd* a, void* stream);

/* Diagnostics only: per-block phase cycles of nerf_mlp_chain_fwd into buf[(n_pad/128)*6]
 * uint64 (DMA wait, barrier, MFMA section, epilogue, total, end time); NULL switches off. */
int nerf_chain_debug_stamps(void* buf);
/* 1 when the library was built with NERF_CHAIN_STAMPS (the two-wave chains then stamp too;
 * production builds carry no stamp instructions in them), else 0. */
int nerf_chain_stamps_built(void);

/* ---------------------------------------------------------------------------
 * Output heads (density + colour logits), forward and backward.
 * Replaces fc_density and fc_rgb (official_nerf.py:66, 91).
 *   raw4[s] = ( h8[s].wd + bd,  hr[s].Wc[c] + bc[c] for c<3 )
 * h8: [n_pad][256] trunk output, hr: [n_pad][128] colour hidden (D/2), hidden = D. */
int nerf_heads_fwd(const float* h8, int ld8, const float* hr, int ldr, int hidden,
                   const float* wd, const float* bd, const float* wc, const float* bc,
                   float* raw4, int n_pad, void* stream);

/* graw4[s] = dL/draw4[s].  Writes dyr = (graw4[s,1:4] @ Wc) * (hr > 0)  [n_pad][hidden/2]
 * and per-block partial sums of dWc (3 x hidden/2), dbc (3), dwd (hidden), dbd (1) into
 * part[blocks][4*hidden/2... ] -- see nerf_heads_part_size(). */
int nerf_heads_part_size(int hidden, int n_pad);
int nerf_heads_bwd(const float* graw4, const float* h8, int ld8, const float* hr, int ldr,
                   int hidden, const float* wc, float* dyr, int lddyr, float* part, int n_pad,
                   float* dyr_rmax, float* dyr_cmax, void* stream);
/* dyr_rmax (optional): max |dyr| per row; dyr_cmax (optional, [n_pad/128][hidden/2 padded to
 * 64], n_pad % 128 == 0): max |dyr| per column and 128-row group (mode 2 scales). */
/* The same backward in parts (ABI 8): mode 1 writes dyr and its maxima only (h8, part unused,
 * may be NULL), mode 2 the head-weight partials only (dyr and its maxima unused), mode 3 both
 * (= nerf_heads_bwd).  Modes 1 and 2 together give the same results as mode 3; the training
 * backward runs mode 2 on a side stream, off the input-gradient chain.  hr_mask (mode 1,
 * optional): the colour layer's ReLU bits [n_pad][ldm] (bit = hr > 0, its forward's mask_out)
 * gate dyr instead of hr, which may then be NULL (2 MB read instead of 67 MB at cfg2). */
int nerf_heads_bwd_mode(int mode, const float* graw4, const float* h8, int ld8, const float* hr, int ldr,
                        const uint32_t* hr_mask, int ldm, int hidden, const float* wc, float* dyr, int lddyr,
                        float* part, int n_pad, float* dyr_rmax, float* dyr_cmax, void* stream);
/* Reduce the heads partials into gwd[hidden], gbd[1], gwc[3][hidden/2], gbc[3]. */
int nerf_heads_reduce(const float* part, int hidden, int n_pad, float* gwd, float* gbd,
                      float* gwc, float* gbc, int accumulate, void* stream);

/* ---------------------------------------------------------------------------
 * Fused per-ray compositing: sigma->alpha, exclusive transmittance product with
 * eps = 1e-6, weighted sums (rendering.py:113-141, official_nerf.py:77-83, 92).
 *   flags bit0: dist_alpha (alpha = 1-exp(-sigma*delta), delta_last = 1e10, alpha_last = 1)
 *         bit1: white_background       bit2: occ_activation relu (else softplus)
 * Outputs rgb[R][3], dist[R], alpha[R*S]. One wavefront per ray (S <= 1024). */
int nerf_composite_fwd(const float* raw4, const float* z, int n_rays, int n_samples, int flags,
                       float* rgb, float* dist, float* alpha, void* stream);

/* Backward of nerf_composite_fwd: grad_rgb[R][3], grad_dist[R] -> graw4[R*S][4]
 * (rows >= R*S up to n_pad are zeroed). */
int nerf_composite_bwd(const float* raw4, const float* z, int n_rays, int n_samples, int flags,
                       const float* grad_rgb, const float* grad_dist, float* graw4, int n_pad,
                       void* stream);

/* Gradient w.r.t. the ray inputs of nerf_encode_samples (pose learning):
 * genc_p[s][64] (+ genc_p2[s][64] when not NULL: the skip layer's gradient of the same
 * encoding), genc_d[s][64] -> per ray g_pts_o[R][3] = sum_s dL/dpts,
 * g_pts_d[R][3] = sum_s z dL/dpts, g_view[R][3] = sum_s dL/dview. */
int nerf_encode_bwd(const float* pts_o, const float* pts_d, const float* view, const float* z,
                    const float* genc_p, const float* genc_p2, const float* genc_d, int n_rays, int n_samples,
                    float* g_pts_o, float* g_pts_d, float* g_view, void* stream);

/* ---------------------------------------------------------------------------
 * Weight packing: src [rows][cols] (reference nn.Linear layout) -> dst [rows][ld_dst]
 * zero padded, and (if dst_t != NULL) its transpose dst_t[c][r] (row stride ld_t,
 * rows c >= cols zero).  Padding rows/cols outside the written ranges keep their
 * previous contents (callers zero the buffers once).  Up to NERF_MAX_PACK descriptors.
 * dst_s / dst_ts (optional): the whole padded dst / dst_t as bf16x3 split images, the B
 * operand format of GEMM precision mode 1 (hi, mid, lo planes; ld_dst, ld_t % 8 == 0).
 * In GEMM precision mode 2 the same buffers receive the fp16 pair form instead: each image
 * row r scaled by 2^e_r (row max -> [2^14, 2^15)), planes 0 / 1 = fp16 hi / lo, and e_r as
 * an int32 in the first word of plane 2's chunk 0 of that row (u16 index
 * ((2*K/8)*rows + r)*8).
 * dst_cs / dst_cts (optional, mode 2 only; ABI 13): the CHAIN images of dst / dst_t -- the
 * same fp16 pair form, with the first perm_k columns of dst_cs (every column of dst_cts) in
 * chain order: within each 32 columns, image column 8 g + i holds column 4 g + i (i < 4) or
 * 16 + 4 g + i - 4 (i >= 4) of the 32 (common.hpp chain_perm), the order in which the
 * 16x16x32 MFMA accumulators of the two-wave chains hold a layer's outputs.  perm_k % 32 == 0,
 * ld_t % 32 == 0 when dst_cts is given.  Since ABI 15 the chain images also hold every row's
 * exponent in a compact int32 array at plane 2's chunk 1 (u16 index ((2*K/8 + 1)*rows + 2 r)),
 * which the chain kernels load with one 1 KB LDS-DMA per layer. */
#define NERF_MAX_PACK 24
typedef struct {
    const float* src;
    float* dst;    /* [rows][ld_dst] */
    float* dst_t;  /* [rows_t][ld_t] or NULL */
    int rows, cols, ld_dst, rows_t, ld_t;
    uint16_t* dst_s;   /* optional bf16x3 split image of dst:   [3][ld_dst/8][rows_s][8] */
    uint16_t* dst_ts;  /* optional bf16x3 split image of dst_t: [3][ld_t/8][rows_t][8]  */
    int rows_s;        /* image rows of dst_s (>= rows, rows past `rows` zero; 0 = rows) */
    uint16_t* dst_cs;  /* optional chain image of dst (mode 2): dst_s's form, K in chain order */
    uint16_t* dst_cts; /* optional chain image of dst_t (mode 2) */
    int perm_k;        /* leading columns of dst_cs in chain order (multiple of 32) */
} nerf_pack_desc;
int nerf_pack_weights(const nerf_pack_desc* descs, int n, void* stream);

/* ---------------------------------------------------------------------------
 * Adam (torch.optim.Adam semantics, amsgrad False) over one flat fp32 buffer.
 * Replaces optimizer.step() (training.py:93-99): torch's foreach Adam op for op (lerp_, mul_,
 * addcmul_, sqrt, div_, add_, addcdiv_).  hyper (device, 16 floats, 8-byte aligned; ABI 13) =
 * {step, lr, beta1, beta2, eps, weight_decay, 1 - beta2, ticket, lr, beta1, beta2 as doubles in
 * slots 8-13, 1 - beta1, 1.0}: 1 - beta1 / 1 - beta2 rounded once from the caller's doubles and
 * the bias corrections lr / (1 - beta1^t), sqrt(1 - beta2^t) taken in double, as torch forms
 * them (slot 15 != 1: the doubles are ignored and derived from the f32 slots; slot 6 == 0:
 * 1 - beta2 from the f32 beta2).  The update uses step + 1 and the last workgroup to finish
 * stores it back (one launch; a captured graph replays the correct bias corrections).
 * hyper[7] is a completion counter: zero it once. */
int nerf_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                   int64_t n, float* hyper, void* stream);

/* ---------------------------------------------------------------------------
 * Brute-force nearest neighbour for the dense point-cloud loss
 * (losses.py:129-150): idx[i] = argmin_j |x[i] - y[j]| (first index on ties).
 * x: [p][3], y: [q][3] fp32, idx: int64 [p]. */
int nerf_chamfer_nn(const float* x, int p, const float* y, int q, int64_t* idx, void* stream);

/* ---------------------------------------------------------------------------
 * Ray prologue / loss epilogue of the training step (rays.hip).
 *
 * nerf_sample_rays: R distinct pixel indices drawn uniformly from [0, n_pix), the set
 *   torch.randperm(n_pix)[:R] draws (training.py:277-283), from a Philox-4x32-10 stream
 *   keyed by `seed` (deterministic in (seed, n_pix, R)); optionally the pixel coordinates
 *   of arange_pixels (common.py:13-40; pixels [R][2], needs width*height == n_pix) and the
 *   colours img.view(3, H*W)[:, idx]^T (rgb [R][3], img = [3][H][W]).  One workgroup.
 *   Requires R <= NERF_SAMPLE_MAX_RAYS and n_pix >= 2R.  status (optional, int) receives
 *   the number of draw rounds used, 0 if NERF_SAMPLE_MAX_ROUNDS did not suffice. */
#define NERF_SAMPLE_MAX_RAYS 4096
#define NERF_SAMPLE_MAX_ROUNDS 64
int nerf_sample_rays(int n_pix, int n_rays, uint64_t seed, int width, int height, const float* img,
                     int64_t* idx, float* pixels, float* rgb, int* status, uint64_t* seed_counter,
                     void* stream);
/* seed_counter (optional, device uint64): mixed into the Philox key and advanced by one per
 * launch on the device -- successive replays of a captured hipGraph draw new rays. */

/* Batched 4x4 inverse (torch.inverse / linalg.inv_ex, common.py:139-141, training.py:255-257):
 * Gauss-Jordan with partial pivoting, a [n][4][4] -> out [n][4][4]. */
int nerf_mat4_inv(const float* a, int n, float* out, void* stream);

/* LearnPose.forward (poses.py:23-31, common.py:277-310): c2w = [Exp(r) | t; 0 0 0 1] @ init_c2w
 * with Exp(r) = I + sin(th)/th [r]x + (1-cos th)/th^2 [r]x^2, th = |r| + 1e-15.
 * r, t: [3]; init_c2w: [4][4] or NULL (identity). */
int nerf_pose_c2w(const float* r, const float* t, const float* init_c2w, float* c2w, void* stream);

/* Unprojection matrix M = (inv(scale) @ inv(world)) @ inv(K) (common.py:139-141, 205-208).
 * inverses (optional, [3][4][4]) = {inv(K), inv(world), inv(scale)} for the backward. */
int nerf_unproject_matrix(const float* K, const float* world, const float* scale, float* M,
                          float* inverses, void* stream);

/* Backwards of the 4x4 chain (the autograd of training.py:255-265, 334-343 when poses are
 * learned), one launch each instead of torch's per-op graph:
 *  nerf_pose_c2w_bwd: g_c2w [4][4] of nerf_pose_c2w -> g_r [3], g_t [3] (each optional);
 *    the closed form of the Exp map's derivative (common.py:277-310) in f64, the r = 0
 *    subgradient of |r| taken as 0 (torch's norm backward).
 *  nerf_mat4_inv_bwd: g_a = -inv_a^T g inv_a^T for [n][4][4] (inv_a: the forward's output).
 *  nerf_mat4_mul / _bwd: c = a @ b ([n][4][4]); g_a = g b^T, g_b = a^T g (each optional).
 *  nerf_unproject_matrix_bwd: g_M of nerf_unproject_matrix -> g_K, g_world, g_scale (each
 *    optional), from the forward's inverses. */
int nerf_pose_c2w_bwd(const float* r, const float* init_c2w, const float* g_c2w, float* g_r, float* g_t,
                      void* stream);
int nerf_mat4_inv_bwd(const float* inv_a, const float* g, int n, float* g_a, void* stream);
int nerf_mat4_mul(const float* a, const float* b, int n, float* c, void* stream);
int nerf_mat4_mul_bwd(const float* a, const float* b, const float* g, int n, float* g_a, float* g_b,
                      void* stream);
int nerf_unproject_matrix_bwd(const float* inverses, const float* g_M, float* g_K, float* g_world,
                              float* g_scale, void* stream);

/* Depth-prior distortion of the gathered prior values d [n] (training.py:259-264, 325-329,
 * with the nearest_limit clamp of :346-347): y = d*scale + shift (shift_first: (d + shift)*scale),
 * then y < lo -> lo (lo = -INFINITY: no clamp).  scale, shift: device scalars.  Backward:
 * g_scale / g_shift (device scalars, each optional) = the sums over the unclamped entries;
 * one workgroup, deterministic. */
int nerf_depth_affine(const float* d, int n, const float* scale, const float* shift, int shift_first, float lo,
                      float* y, void* stream);
int nerf_depth_affine_bwd(const float* d, int n, const float* scale, const float* shift, int shift_first, float lo,
                          const float* g, float* g_scale, float* g_shift, void* stream);

/* Camera rays of Renderer.nope_nerf (rendering.py:52-80): for pixels [R][2], depth [R]
 * (NULL = no depth prior, d_src = 1): cam [R][3] = M[:3,3]; v = M[:3,:3](x,y,1);
 * ray_norm = |v|; ray = v/|v| (NERF_RAYS_NORMALISE) else v; d_src = |M[:3,:3](xd,yd,d)|
 * (divided by |v| without NORMALISE); mask [R] (u8, optional) = isfinite(d_src) & d_src != 0;
 * view [R][3] (optional) = -ray, or 1 with NERF_RAYS_VIEW_ONES (use_ray_dir False). */
#define NERF_RAYS_NORMALISE 1
#define NERF_RAYS_VIEW_ONES 2
int nerf_camera_rays(const float* M, const float* pixels, const float* depth, int n_rays, int flags,
                     float* cam, float* ray, float* view, float* ray_norm, float* d_src, uint8_t* mask,
                     void* stream);
/* Its backward: upstream gradients (each optional) -> gM [4][4] (row 3 zero) and
 * g_depth [R] (optional).  One workgroup, deterministic. */
int nerf_camera_rays_bwd(const float* M, const float* pixels, const float* depth, int n_rays, int flags,
                         const float* g_cam, const float* g_ray, const float* g_view, const float* g_norm,
                         const float* g_dsrc, float* gM, float* g_depth, void* stream);

/* Loss.forward's render terms (losses.py:28-33, 60-66, 195-228), four device scalars:
 * total = w_rgb l_rgb + w_depth l_depth, l_rgb = sum|e| or sum e^2 over rgb [R][3] / R,
 * l_depth = sum over mask of |depth_pred - depth_gt| / max(count, 1), l2_mean = mean e^2;
 * cnt receives count.
 * depth_pred NULL = no depth term; mask NULL = all n_depth rays.  One workgroup. */
int nerf_ray_loss(const float* rgb, const float* rgb_gt, int n_rays, const float* depth_pred,
                  const float* depth_gt, const uint8_t* mask, int n_depth, int rgb_l1, float w_rgb,
                  float w_depth, float* total, float* l_rgb, float* l_depth, float* l2_mean, float* cnt,
                  void* stream);
/* Its backward: the four upstream scalars (device, each optional) -> g_rgb [R][3],
 * g_depth_pred [n_depth], g_depth_gt [n_depth] (each optional). */
int nerf_ray_loss_bwd(const float* rgb, const float* rgb_gt, int n_rays, const float* depth_pred,
                      const float* depth_gt, const uint8_t* mask, int n_depth, int rgb_l1, float w_rgb,
                      float w_depth, const float* go_total, const float* go_rgb, const float* go_depth,
                      const float* go_l2, const float* cnt, float* g_rgb, float* g_depth_pred,
                      float* g_depth_gt, void* stream);

/* ---------------------------------------------------------------------------
 * Image-pair terms of the full step (pair.hip; training.py:359-405, losses.py:116-159):
 * at the point-cloud resolution h x w (P = h w points, pixel grid of arange_pixels),
 *   pc1 = (inv(K) [x d1, y d1, d1, 1])[:3], pc2 likewise (transform_to_world),
 *   X = R (pc1 / s1) + t, Y = pc2 / s1 (s1 = NULL: 1; Rt = Rt_rel_12 [4][4]),
 *   loss_pc = mean |X - Y[nn(X)]| + mean |Y - X[nn(Y)]| (dense chamfer, first index on ties),
 *   loss_rgb_s = mean over valid elements of clamp(|img1(p) - img2(proj(R pc1 + t))|, 0, 1)
 *   (bilinear, align_corners, zero padding; the rotated point is replaced by (nl, nl, nl)
 *   when -z < nl; valid = |proj| <= 1), only when img1/img2 ([3][h][w]) are given.
 * All operands are device pointers (K, Rt, s1 included).  work: nerf_pair_workspace floats;
 * nn: int [2][P]; out3 = {loss_pc, loss_rgb_s, valid element count}. */
int nerf_pair_workspace(int n_points, int* n_chunks, int64_t* floats);
int nerf_pair_forward(const float* d1, const float* d2, int h, int w, const float* K, const float* Rt,
                      const float* s1, float nl, const float* img1, const float* img2, float* work, int* nn,
                      float* out3, void* stream);
/* Backward: upstream scalars go_pc / go_rgbs (device, optional) -> g_d1, g_d2 [P] (optional),
 * g13 = {dR (9, row-major), dt (3), ds1}; gXY: scratch [12P] floats, 8-byte aligned (ABI 14: the
 * gathered-point chamfer gradients as 6P int64 fixed-point sums, order-independent); part13: scratch
 * [13 * ceil(P / 256)] floats.  rgbs_detach_scale: detach_rgbs_scale (training.py:372-375). */
int nerf_pair_backward(const float* d1, const float* d2, int h, int w, const float* K, const float* Rt,
                       const float* s1, float nl, const float* img1, const float* img2, int rgbs_detach_scale,
                       const float* work, const int* nn, const float* out3, const float* go_pc,
                       const float* go_rgbs, float* gXY, float* g_d1, float* g_d2, float* g13, float* part13,
                       void* stream);

/* ---------------------------------------------------------------------------
 * Timing hooks for bench.py: when enabled, every GEMM launch is bracketed by
 * hipEvents on its stream; nerf_prof_read returns, for the GEMM family since the last
 * reset, the summed launch durations, the launch count, the padded FLOPs issued and the
 * union of the launch intervals (launches overlapping on two streams count once);
 * synchronises the events. */
int nerf_prof_enable(int on);
int nerf_prof_read(double* gemm_ms, int64_t* gemm_launches, double* gemm_flops, double* union_ms);

/* Per-kind breakdown of the same records (call before nerf_prof_read, which resets them):
 * kind 0 = forward NT (nerf_linear_fwd), 1 = input gradient NT (nerf_linear_bwd_data),
 * 2 = weight gradient TN (nerf_linear_bwd_weight) on 256 x 256 output tiles, 3 = the narrow
 * weight gradients (an output or K side below 256: the encoding segments, the colour layer).  flops: algorithmic f32 FLOPs of the
 * launches (2*m*n*k, padded shapes); bytes: their algorithmic HBM bytes (operands read
 * once, outputs written once: A, B, C and the ReLU bit masks; for the weight gradient the
 * dY and X panels plus ONE nout x kin gradient, not the split-K slabs); mfma_flops: flops
 * times the MFMA products each f32 product costs in the arithmetic that ran (1 exact f32,
 * 6 bf16x6, 3 fp16 pair) -- divided by the dense bf16/f16 MFMA rate it gives the
 * launches' MFMA-bound time; exact_f32: 1 if any launch ran on the f32 MFMA (then
 * mfma_flops / f32 peak). */
#define NERF_PROF_FWD 0
#define NERF_PROF_DX 1
#define NERF_PROF_DW 2
#define NERF_PROF_DW_NARROW 3
#define NERF_PROF_CHAIN_FWD 4   /* nerf_mlp_chain_train: the ten forward linears + heads in one launch */
#define NERF_PROF_CHAIN_BWD 5   /* nerf_mlp_chain_bwd: dyr + the nine input gradients in one launch */
#define NERF_PROF_KINDS 6
typedef struct nerf_prof_kind {
    double ms;
    int64_t launches;
    double flops;
    double bytes;
    double mfma_flops;
    int exact_f32;
} nerf_prof_kind;
int nerf_prof_read_kinds(nerf_prof_kind* out, int n_kinds);

#ifdef __cplusplus
}
#endif
#endif /* NERF_HIP_H */
