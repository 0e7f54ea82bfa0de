// Native executor of the field backward (nerf_field_backward): the launch schedule of
// FieldRunner.backward for the D = 256 / colour 128 field in precision mode 2 in one host
// call -- the autograd of official_nerf.py:60-96 and rendering.py:113-141 as launched by
// training.py:92.  The Python schedule issues ~60 ctypes launches, ~20 temporaries and ~10
// cross-stream events per step (0.8 ms of host time at cfg2, profiles/r03/host_split_cfg2.json);
// here the same launches, in the same order on the same two streams, take a few microseconds
// each, so the eager step stays GPU-bound on a slow host core.
//
// Schedule (per layer, from the colour layer down): the input-gradient GEMM on the caller's
// stream, the weight gradient + its split-K slab reduce on the side stream once that layer's
// dy exists (an event), the last `tail_main` layers' weight gradients on the caller's stream
// after the input-gradient chain.  The head-weight partials run first on the side stream,
// dyr (the colour layer's dy, gated by its ReLU words) on the caller's.
#include "common.hpp"

#include <cstdlib>
#include <vector>

namespace {

constexpr int L = NERF_BWD_LAYERS;
constexpr int D = 256, HR = 128;
// layer table (FieldRunner.layers): output rows, first-segment K, padded K, second segment
// (0 none, 1 enc_p, 2 enc_d)
constexpr int OUT_P[L] = {D, D, D, D, D, D, D, D, D, HR};
constexpr int K1[L] = {64, D, D, D, D, D, D, D, D, D};
constexpr int KP[L] = {64, D, D, D, D + 64, D, D, D, D, D + 64};
constexpr int SEG[L] = {0, 0, 0, 0, 1, 0, 0, 0, 0, 2};
constexpr int NREF[L] = {D, D, D, D, D, D, D, D, D, HR};
constexpr int KREF[L] = {63, D, D, D, D + 63, D, D, D, D, D + 27};
constexpr int LF = 8, LR = 9;

struct Carve {
    char* base;
    size_t off = 0;
    float* take(size_t n) {
        off = (off + 255) & ~size_t(255);
        float* p = base ? reinterpret_cast<float*>(base + off) : nullptr;
        off += n * sizeof(float);
        return p;
    }
};

struct Work {
    float *graw4, *dyr, *dyr_rm, *dyr_cm, *part, *hpart, *scratch;
    float *dx[L], *dx_rm[L], *dx_cm[L];   // dx[l]: gradient w.r.t. layer l's first input (l = 1..9)
    float *genc_p0, *genc_p4, *genc_d;
    float *slab[L], *bslab[L];
    int splits[L];
};

size_t carve(char* base, int np, int ray_grad, Work& w) {
    Carve c{base};
    w.graw4 = c.take((size_t)np * 4);
    w.dyr = c.take((size_t)np * HR);
    w.dyr_rm = c.take(np);
    w.dyr_cm = c.take((size_t)(np / 128) * HR);
    w.part = c.take((size_t)nerf_heads_part_size(D, np));
    w.hpart = c.take((size_t)nerf::heads_part_blocks(np) * (256 + 384 + 4));
    w.scratch = c.take(512);
    for (int l = 1; l < L; ++l) {
        w.dx[l] = c.take((size_t)np * K1[l]);
        w.dx_rm[l] = c.take(np);
        w.dx_cm[l] = c.take((size_t)(np / 128) * K1[l]);
    }
    w.dx[0] = w.dx_rm[0] = w.dx_cm[0] = nullptr;
    w.genc_p0 = ray_grad ? c.take((size_t)np * 64) : nullptr;
    w.genc_p4 = ray_grad ? c.take((size_t)np * 64) : nullptr;
    w.genc_d = ray_grad ? c.take((size_t)np * 64) : nullptr;
    for (int l = 0; l < L; ++l) w.splits[l] = nerf_linear_bwd_weight_splits(OUT_P[l], K1[l], np);
    for (int l = 0; l < L; ++l) {
        w.slab[l] = c.take((size_t)w.splits[l] * OUT_P[l] * KP[l]);
        w.bslab[l] = c.take((size_t)w.splits[l] * OUT_P[l]);
    }
    return c.off + 256;
}

// events: a per-thread pool (the autograd engine runs backwards on one thread per device)
struct EventPool {
    std::vector<hipEvent_t> ev;
    size_t next = 0;
    hipEvent_t get() {
        if (next == ev.size()) {
            hipEvent_t e;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
            ev.push_back(e);
        }
        return ev[next++];
    }
};
thread_local EventPool g_events;

#define RC(x)                \
    do {                     \
        const int rc_ = (x); \
        if (rc_) return rc_; \
    } while (0)

// side waits for everything issued on main so far
int fork(hipStream_t main, hipStream_t side) {
    hipEvent_t e = g_events.get();
    NERF_CHECK(e != nullptr, "nerf_field_backward: hipEventCreate failed");
    NERF_CHECK(hipEventRecord(e, main) == hipSuccess && hipStreamWaitEvent(side, e, 0) == hipSuccess,
               "nerf_field_backward: cross-stream event failed");
    return NERF_OK;
}

// weight + bias gradient of layer l (dy: its output gradient) on stream s
int weight_grad(const nerf_field_bwd& a, const Work& w, int l, const float* dy, const float* dy_cm, void* s) {
    const int np = a.n_pad;
    const float* x = l == 0 ? a.enc_p : a.act[l - 1];
    const float* x_cm = l == 0 ? a.enc_p_cmax : a.cmax[l - 1];
    if (SEG[l]) {
        RC(nerf_linear_bwd_weight_seg(dy, OUT_P[l], OUT_P[l], x, K1[l], K1[l], SEG[l] == 1 ? a.enc_p : a.enc_d, 64, 64,
                                      np, w.splits[l], w.slab[l], KP[l], w.bslab[l], dy_cm, x_cm,
                                      SEG[l] == 1 ? a.enc_p_cmax : a.enc_d_cmax, s));
    } else {
        RC(nerf_linear_bwd_weight(dy, OUT_P[l], OUT_P[l], x, K1[l], K1[l], np, w.splits[l], w.slab[l], KP[l], 0,
                                  w.bslab[l], dy_cm, x_cm, s));
    }
    return nerf_slab_reduce(w.slab[l], w.splits[l], OUT_P[l], KP[l], NREF[l], KREF[l], w.bslab[l], a.gw[l], a.gb[l], 0,
                            s);
}

// The schedule with the input-gradient chain (bwd_chain): dyr and the nine input gradients in
// one launch (nerf_mlp_chain_bwd) on the caller's stream; then every layer's weight gradient on
// the caller's stream (each 4-wave TN launch fills the chip on its own) with its split-K
// reduce on the side stream behind an event, so a reduce runs beside the next layer's TN; the
// ray gradients (pose learning) as three input-gradient GEMMs over the saved dy of the colour
// layer, l4 and l0.  The head-weight partials were forked to the side stream before the chain.
int chain_schedule(const nerf_field_bwd& a, Work& w, const float* graw4, void* stream, void* side_stream,
                   bool heads_after, const nerf::SlabJobDesc* extra, int n_extra) {
    const int np = a.n_pad;
    hipStream_t main = nerf::as_stream(stream), side = nerf::as_stream(side_stream);
    // D_0 = dyr, D_i = dx[10 - i]: the gradient at the output of layer 9 - i
    nerf_chain_bwd c{};
    c.graw4 = graw4;
    c.hr_mask = a.mask[LR];
    c.ld_hr_mask = HR / 32;
    c.wd = a.wd;
    c.wc = a.wc;
    for (int i = 0; i < 9; ++i) {
        const int l = LR - i;
        c.wt_img[i] = a.wt_cimg[l];   // the chain image: K in chain order (ABI 13)
        c.wt_img_rows[i] = KP[l];
        c.in_mask[i] = l == LR ? nullptr : a.mask[l - 1];
        c.ld_in_mask[i] = OUT_P[l - 1 < 0 ? 0 : l - 1] / 32;
    }
    c.dy[0] = w.dyr; c.lddy[0] = HR; c.dy_cmax[0] = w.dyr_cm; c.dy_rmax[0] = w.dyr_rm;
    for (int i = 1; i < 10; ++i) {
        const int l = 10 - i;
        c.dy[i] = w.dx[l]; c.lddy[i] = K1[l]; c.dy_cmax[i] = w.dx_cm[l]; c.dy_rmax[i] = w.dx_rm[l];
    }
    c.scratch = w.scratch;
    c.n_pad = np;
    RC(nerf_mlp_chain_bwd(&c, stream));
    if (heads_after) {   // (NERF_HEADS_PLACE=2, A/B only) the head-weight partials behind the chain
        RC(nerf_heads_bwd_mode(2, graw4, a.act[7], D, a.act[LR], HR, nullptr, 0, D, a.wc, nullptr, 0, w.part, np,
                               nullptr, nullptr, stream));
        RC(nerf_heads_reduce(w.part, D, np, a.g_wd, a.g_bd, a.g_wc, a.g_bc, 0, stream));
    }
    auto dy_of = [&](int l, const float*& dy, const float*& cm, const float*& rm) {
        if (l == LR) { dy = w.dyr; cm = w.dyr_cm; rm = w.dyr_rm; }
        else { dy = w.dx[l + 1]; cm = w.dx_cm[l + 1]; rm = w.dx_rm[l + 1]; }
    };
    // the weight-gradient schedule (NERF_WGRAD_SCHED): 3 (the default) two k_wgrad_jobs launches,
    // 2.062 vs 2.093 ms/step for 1 (profiles/r05/wgrad_sched_ab.json); 1 the round-4 schedule (r04n);
    // 2 one eight-layer launch with the encoding segments of l4 and l0 together (= 1 in-step)
    const char* ws = std::getenv("NERF_WGRAD_SCHED");
    const int sched = ws ? std::atoi(ws) : 3;
    if (sched == 3) {
        // every weight gradient as a job of one of two k_wgrad_jobs launches (2 S blocks, S the
        // 256 x 256 layers' split count; the narrow tiles fill the same grid instead of a launch
        // of their own): the colour layer's two segments + l_f .. l5, then l4's two segments +
        // l3 .. l1 + l0.  Same splits and slab columns as schedule 1, so the same slabs.  Each
        // launch's slab reduces follow it on the caller's stream.
        nerf::SlabJobDesc jobs[nerf::kSlabJobsMax];
        int nj = 0;
        for (int e = 0; e < n_extra; ++e) jobs[nj++] = extra[e];   // the head-weight reduces ride in the first batch
        auto flush = [&](hipStream_t s) -> int {
            if (s != main) RC(fork(main, s));
            RC(nerf::slab_reduce_jobs(jobs, nj, s));
            nj = 0;
            return NERF_OK;
        };
        auto job = [&](int l) {
            jobs[nj++] = nerf::SlabJobDesc{w.slab[l], w.splits[l], OUT_P[l], KP[l], NREF[l], KREF[l], w.bslab[l], a.gw[l],
                                           a.gb[l]};
        };
        auto enc_rows = [&](int l) -> int {
            if (!a.ray_grad) return NERF_OK;
            const float *dy, *cm, *rm;
            dy_of(l, dy, cm, rm);
            const int op = OUT_P[l];
            const int k0 = l == 0 ? 0 : K1[l];
            float* out = l == LR ? w.genc_d : l == 4 ? w.genc_p4 : w.genc_p0;
            return nerf_linear_bwd_data(dy, op, op, a.wt[l] + (size_t)k0 * op, a.wt_img[l] + (size_t)k0 * 8, KP[l], nullptr,
                                        0, nullptr, nullptr, 0, out, 64, np, 64, rm, nullptr, nullptr, stream);
        };
        nerf_wgrad_tile_job tj[nerf::kWgradJobsMax];
        int tgrp[nerf::kWgradJobsMax];
        int nt = 0, cur_grp = 0;
        // layer l's main segment (x = its input; l0: enc_p) and, for l4 / the colour layer, the
        // 64-wide encoding segment at slab column K1[l]
        auto tiles = [&](int l) {
            const float *dy, *cm, *rm;
            dy_of(l, dy, cm, rm);
            const int op = OUT_P[l];
            const float* x = l == 0 ? a.enc_p : a.act[l - 1];
            const float* xcm = l == 0 ? a.enc_p_cmax : a.cmax[l - 1];
            tgrp[nt] = cur_grp;
            tj[nt++] = nerf_wgrad_tile_job{dy, op, op, x, K1[l], K1[l], w.splits[l], w.slab[l], KP[l], 0, w.bslab[l], cm, xcm};
            if (SEG[l]) {
                tgrp[nt] = cur_grp;
                tj[nt++] = nerf_wgrad_tile_job{dy, op, op, SEG[l] == 1 ? a.enc_p : a.enc_d, 64, 64, w.splits[l], w.slab[l],
                                               KP[l], K1[l], nullptr, cm, SEG[l] == 1 ? a.enc_p_cmax : a.enc_d_cmax};
            }
            job(l);
        };
        auto launch = [&]() -> int {
            RC(nerf_linear_bwd_weight_jobs(tj, nt, np, w.splits[LF], stream));
            nt = 0;
            return NERF_OK;
        };
        // NERF_WGRAD_GROUPS: 2 (the default) both launches as two block groups of 2 S' blocks
        // (S' = S / 2: each job twice the rows per split, half the jobs per block and half the
        // split-K slab bytes written and read back); 1 the second launch only; 0 one job list per
        // launch on 2 S blocks.  1.9125 / 1.9525 / 1.9721 ms per cfg2 step (2 / 1 / 0, fresh
        // processes interleaved, profiles/r06/wgrad_groups_lib_ab.txt)
        const char* wgg = std::getenv("NERF_WGRAD_GROUPS");
        const int groups = w.splits[LF] % 16 == 0 ? (wgg ? std::atoi(wgg) : 2) : 0;
        const int s2 = w.splits[LF] / 2;
        if (groups >= 2) {
            // group 0 the colour layer's f segment + l_f + l7, group 1 its enc_d segment + l6 + l5
            // (5 vs 4.5 1024-row tile-times per block against 4.75 in one list, three jobs each
            // instead of six); the slab buffers are sized for S: room to spare
            for (int l : {LF, 7, 6, 5}) w.splits[l] = s2;
            w.splits[LR] = 2 * s2;
            tiles(LR);
            tgrp[nt - 1] = 1;
            for (int l : {LF, 7}) tiles(l);
            cur_grp = 1;
            for (int l : {6, 5}) tiles(l);
            cur_grp = 0;
            RC(nerf_linear_bwd_weight_job_groups(tj, tgrp, nt, np, s2, 2, stream));
            nt = 0;
        } else {
            for (int l : {LR, LF, 7, 6, 5}) tiles(l);
            RC(launch());
        }
        // NERF_WGRAD_BATCH1: the first launch's slab reduces 2 (the default) in ONE reduce launch with
        // the second's, after it; 1 on the caller's stream between the two launches; 0 on the side
        // stream (it can only start once the second launch frees CUs; replayed as a hipGraph the
        // side-stream branch cost ~55 us per step, profiles/r05/batch1_ab.json)
        const char* b1 = std::getenv("NERF_WGRAD_BATCH1");
        const int batch1 = b1 ? std::atoi(b1) : 2;
        if (batch1 != 2) RC(flush(batch1 == 0 ? side : main));
        RC(enc_rows(LR));
        // grouped (NERF_WGRAD_GROUPS >= 1)
        if (groups >= 1) {
            for (int l : {1, 2, 3, 4}) w.splits[l] = s2;   // the slab buffers are sized for S: room to spare
            w.splits[0] = 2 * s2;
            // group 0 l4's h3 segment + l3 + l0, group 1 l4's enc_p segment + l2 + l1 (4.83 / 5
            // tile-times): with groups k_wgrad_jobs runs a group's narrow jobs before its pairs, so the
            // two reads of l4's dy start together (group 0's first job and group 1's): 1.8580 vs 1.8677
            // ms per cfg2 step (profiles/r06/wgrad_l4_groups_ab.txt)
            tiles(4);
            tgrp[nt - 1] = 1;
            for (int l : {3, 0}) tiles(l);
            cur_grp = 1;
            for (int l : {2, 1}) tiles(l);
            cur_grp = 0;
            RC(nerf_linear_bwd_weight_job_groups(tj, tgrp, nt, np, s2, 2, stream));
            nt = 0;
        } else {
            for (int l : {3, 2, 1, 4, 0}) tiles(l);   // l4's h3 job the last 256 x 256 one: its enc_p job follows
            RC(launch());
        }
        RC(flush(main));
        RC(enc_rows(4));
        RC(enc_rows(0));
    } else if (sched == 2) {
        // the weight gradients back to back on the caller's stream (each needs only the chain's
        // saved dy): the colour layer's two segments (f, enc_d) as two launches; l_f .. l1 -- with
        // l4's h3 segment -- as ONE launch (k_wgrad_pairs: a block walks the eight 256 x 256
        // layers); l4's enc_p segment and l0 as one launch (both 256 x 64 over enc_p). The slab
        // reduces: every layer but l4 and l0 on the side stream after the eight-layer launch (beside
        // the last one), l4's and l0's on the caller's stream at the end (a cross-stream event costs
        // ~7 us of idle on the stream that records it; one fork per layer was ~80 us per step)
        nerf::SlabJobDesc jobs[nerf::kSlabJobsMax];
        int nj = 0;
        for (int e = 0; e < n_extra; ++e) jobs[nj++] = extra[e];   // the head-weight reduces ride in the first batch
        auto flush = [&](hipStream_t s) -> int {
            if (s != main) RC(fork(main, s));
            RC(nerf::slab_reduce_jobs(jobs, nj, s));
            nj = 0;
            return NERF_OK;
        };
        auto job = [&](int l) {
            jobs[nj++] = nerf::SlabJobDesc{w.slab[l], w.splits[l], OUT_P[l], KP[l], NREF[l], KREF[l], w.bslab[l], a.gw[l],
                                           a.gb[l]};
        };
        // the encoding rows of W^T against a layer's dy (ray gradients: lr, l4, l0)
        auto enc_rows = [&](int l) -> int {
            if (!a.ray_grad) return NERF_OK;
            const float *dy, *cm, *rm;
            dy_of(l, dy, cm, rm);
            const int op = OUT_P[l];
            const int k0 = l == 0 ? 0 : K1[l];
            float* out = l == LR ? w.genc_d : l == 4 ? w.genc_p4 : w.genc_p0;
            return nerf_linear_bwd_data(dy, op, op, a.wt[l] + (size_t)k0 * op, a.wt_img[l] + (size_t)k0 * 8, KP[l], nullptr,
                                        0, nullptr, nullptr, 0, out, 64, np, 64, rm, nullptr, nullptr, stream);
        };
        {   // the colour layer: [f | enc_d]
            const float *dy, *cm, *rm;
            dy_of(LR, dy, cm, rm);
            RC(nerf_linear_bwd_weight(dy, HR, HR, a.act[LF], K1[LR], K1[LR], np, w.splits[LR], w.slab[LR], KP[LR], 0,
                                      w.bslab[LR], cm, a.cmax[LF], stream));
            RC(nerf_linear_bwd_weight(dy, HR, HR, a.enc_d, 64, 64, np, w.splits[LR], w.slab[LR], KP[LR], K1[LR], nullptr,
                                      cm, a.enc_d_cmax, stream));
            job(LR);
            RC(enc_rows(LR));
        }
        {   // l_f .. l1 (l4: its h3 segment) in one launch
            nerf_wgrad_job wj[nerf::kWgradPairsMax];
            int n = 0;
            for (int l = LF; l >= 1; --l) {
                const float *dy, *cm, *rm;
                dy_of(l, dy, cm, rm);
                NERF_CHECK(OUT_P[l] == D && K1[l] == D && w.splits[l] == w.splits[LF], "layer %d", l);
                wj[n++] = nerf_wgrad_job{dy, D, a.act[l - 1], D, w.slab[l], KP[l], w.bslab[l], cm, a.cmax[l - 1]};
                if (l != 4) job(l);
            }
            RC(nerf_linear_bwd_weight_multi(wj, n, np, w.splits[LF], stream));
        }
        RC(flush(side));
        {   // l4's enc_p segment and l0 in one launch
            const float *dy4, *cm4, *rm4, *dy0, *cm0, *rm0;
            dy_of(4, dy4, cm4, rm4);
            dy_of(0, dy0, cm0, rm0);
            RC(nerf::wgrad_narrow_pair(dy4, D, a.enc_p, 64, w.splits[4], w.slab[4], KP[4], K1[4], nullptr, cm4, a.enc_p_cmax,
                                       dy0, D, a.enc_p, 64, w.splits[0], w.slab[0], KP[0], 0, w.bslab[0], cm0, a.enc_p_cmax,
                                       np, main));
            job(4);
            job(0);
            RC(enc_rows(4));
            RC(enc_rows(0));
        }
        RC(flush(main));
    } else {
        // the weight gradients back to back on the caller's stream (each needs only the chain's
        // saved dy): the colour layer (two segments), l_f .. l5 in one launch, l4 (two segments),
        // l3 .. l1 in one launch, l0. Their slab reduces are batched: lr .. l5 on the side stream
        // after l5's (beside l4 .. l1's), l4 .. l1 on the side stream after l1's (beside l0's),
        // l0's on the caller's stream at the end (a cross-stream event costs ~7 us of idle on the
        // stream that records it, and the join another; one fork per layer was ~80 us per step)
        nerf::SlabJobDesc jobs[nerf::kSlabJobsMax];
        int nj = 0;
        for (int e = 0; e < n_extra; ++e) jobs[nj++] = extra[e];   // the head-weight reduces ride in the first batch
        auto flush = [&](hipStream_t s) -> int {
            if (s != main) RC(fork(main, s));
            RC(nerf::slab_reduce_jobs(jobs, nj, s));
            nj = 0;
            return NERF_OK;
        };
        auto job = [&](int l) {
            jobs[nj++] = nerf::SlabJobDesc{w.slab[l], w.splits[l], OUT_P[l], KP[l], NREF[l], KREF[l], w.bslab[l], a.gw[l],
                                           a.gb[l]};
        };
        auto x_of = [&](int l, const float*& x, const float*& x_cm) {
            x = l == 0 ? a.enc_p : a.act[l - 1];
            x_cm = l == 0 ? a.enc_p_cmax : a.cmax[l - 1];
        };
        // one layer's weight gradient (+ its encoding-row input gradient for ray gradients)
        auto single = [&](int l) -> int {
            const float *dy, *cm, *rm, *x, *x_cm;
            dy_of(l, dy, cm, rm);
            x_of(l, x, x_cm);
            const int op = OUT_P[l];
            if (SEG[l])
                RC(nerf_linear_bwd_weight_seg(dy, op, op, x, K1[l], K1[l], SEG[l] == 1 ? a.enc_p : a.enc_d, 64, 64, np,
                                              w.splits[l], w.slab[l], KP[l], w.bslab[l], cm, x_cm,
                                              SEG[l] == 1 ? a.enc_p_cmax : a.enc_d_cmax, stream));
            else
                RC(nerf_linear_bwd_weight(dy, op, op, x, K1[l], K1[l], np, w.splits[l], w.slab[l], KP[l], 0, w.bslab[l], cm,
                                          x_cm, stream));
            job(l);
            if (a.ray_grad && (l == LR || l == 4 || l == 0)) {
                // d enc: the encoding segment's rows of W^T (l0: all of them) against this dy
                const int k0 = l == 0 ? 0 : K1[l];
                float* out = l == LR ? w.genc_d : l == 4 ? w.genc_p4 : w.genc_p0;
                RC(nerf_linear_bwd_data(dy, op, op, a.wt[l] + (size_t)k0 * op, a.wt_img[l] + (size_t)k0 * 8, KP[l], nullptr, 0,
                                        nullptr, nullptr, 0, out, 64, np, 64, rm, nullptr, nullptr, stream));
            }
            return NERF_OK;
        };
        // the 256 x 256 layers hi .. lo (descending) in one launch
        auto pairs = [&](int hi, int lo) -> int {
            nerf_wgrad_job wj[nerf::kWgradPairsMax];
            int n = 0;
            for (int l = hi; l >= lo; --l) {
                const float *dy, *cm, *rm, *x, *x_cm;
                dy_of(l, dy, cm, rm);
                x_of(l, x, x_cm);
                NERF_CHECK(!SEG[l] && OUT_P[l] == D && K1[l] == D && w.splits[l] == w.splits[hi], "layer %d", l);
                wj[n++] = nerf_wgrad_job{dy, OUT_P[l], x, K1[l], w.slab[l], KP[l], w.bslab[l], cm, x_cm};
                job(l);
            }
            return nerf_linear_bwd_weight_multi(wj, n, np, w.splits[hi], stream);
        };
        RC(single(LR));
        RC(pairs(LF, 5));
        RC(flush(side));
        RC(single(4));
        RC(pairs(3, 1));
        RC(flush(side));
        RC(single(0));
        RC(flush(main));
    }
    if (a.ray_grad)
        RC(nerf_encode_bwd(a.pts_o, a.pts_d, a.view, a.z, w.genc_p0, w.genc_p4, w.genc_d, a.n_rays, a.n_samples,
                           a.g_pts_o, a.g_pts_d, a.g_view, stream));
    RC(fork(side, main));
    return NERF_OK;
}

}  // namespace

extern "C" size_t nerf_field_bwd_workspace_bytes(int n_pad, int ray_grad) {
    if (n_pad <= 0 || n_pad % 128) return 0;
    Work w;
    return carve(nullptr, n_pad, ray_grad, w);
}

namespace {
int schedule(const nerf_field_bwd& a, void* stream, void* side_stream);
}  // namespace

extern "C" int nerf_field_backward(const nerf_field_bwd* ap, void* stream, void* side_stream) {
    NERF_CHECK_PTR(ap);
    const int rc = schedule(*ap, stream, side_stream);
    if (rc == NERF_OK || !side_stream || stream == side_stream) return rc;
    // a launch failed part-way: the side stream may still run weight-gradient kernels on the
    // workspace; join it into the caller's stream on this exit too, so the caller's allocator
    // cannot hand the workspace out again while they write it (the error code is kept)
    hipEvent_t e = g_events.get();
    if (e && hipEventRecord(e, nerf::as_stream(side_stream)) == hipSuccess)
        (void)hipStreamWaitEvent(nerf::as_stream(stream), e, 0);
    return rc;
}

namespace {

int schedule(const nerf_field_bwd& a, void* stream, void* side_stream) {
    const int np = a.n_pad;
    NERF_CHECK(np > 0 && np % 128 == 0 && a.workspace && side_stream && stream != side_stream,
               "%s: n_pad=%d (a positive multiple of 128), a workspace and a second stream are required", __func__, np);
    NERF_CHECK(nerf::gemm_precision() == 2, "%s: the native backward runs GEMM precision mode 2", __func__);
    NERF_CHECK(a.tail_main >= 0 && a.tail_main <= L, "%s: tail_main=%d", __func__, a.tail_main);
    NERF_CHECK(a.graw4 || (a.g_rgb && a.g_dist && a.z && a.raw4), "%s: need graw4 or (g_rgb, g_dist, raw4, z)",
               __func__);
    for (int l = 0; l < L; ++l) {
        NERF_CHECK(a.act[l] && a.wt[l] && a.wt_img[l] && a.gw[l] && a.gb[l], "%s: layer %d: missing tensor", __func__,
                   l);
        NERF_CHECK(!a.bwd_chain || l == 0 || a.wt_cimg[l], "%s: layer %d: the input-gradient chain needs the chain "
                   "image of W^T (wt_cimg)", __func__, l);
        NERF_CHECK((l == LF) == (a.mask[l] == nullptr), "%s: layer %d: ReLU words (none for the feature layer)",
                   __func__, l);
        NERF_CHECK((l == LR) == (a.cmax[l] == nullptr), "%s: layer %d: column maxima (none for the colour layer)",
                   __func__, l);
    }
    NERF_CHECK(a.enc_p && a.enc_d && a.enc_p_cmax && a.enc_d_cmax && a.wd && a.wc && a.g_wd && a.g_bd && a.g_wc &&
                   a.g_bc,
               "%s: missing encoding / head tensor", __func__);
    NERF_CHECK(!a.ray_grad || (a.pts_o && a.pts_d && a.view && a.z && a.g_pts_o && a.g_pts_d && a.g_view),
               "%s: ray gradients need pts_o / pts_d / view / z and their gradient outputs", __func__);
    Work w;
    carve(reinterpret_cast<char*>(a.workspace), np, a.ray_grad, w);
    hipStream_t main = nerf::as_stream(stream), side = nerf::as_stream(side_stream);
    g_events.next = 0;

    const float* graw4 = a.graw4;
    if (!graw4) {
        RC(nerf_composite_bwd(a.raw4, a.z, a.n_rays, a.n_samples, a.flags, a.g_rgb, a.g_dist, w.graw4, np, stream));
        graw4 = w.graw4;
    }
    // heads: the head-weight partials (re-reading h8 and hr).  With the input-gradient chain on
    // the caller's stream BEFORE the chain: NERF_HEADS_PLACE 1 (the default since round 6) k_heads_bwd
    // mode 2 and k_heads_reduce both there (1.8609 vs 1.8665 ms/step against 5 on the round-6 weight-
    // gradient schedule, profiles/r06/heads_place_r06_ab.txt); 5 the reduce (11 blocks, ~13 us)
    // forked to the side stream beside the chain (the round-5 default: 2.009 vs 2.030 ms/step then,
    // profiles/r05/heads_reduce_side_ab.json); 3 by k_heads_part (16-byte buffer loads, 4x the
    // waves: ~62 us in-step) with the reduces in the first slab batch (2.066 vs 2.058 ms/step,
    // profiles/r05/heads_part_ab.json); beside the chain (0, the round-4 placement) the partials and their reduce stretch
    // to ~240 us sharing the CUs with the chain, and the step is 13 us slower than 1
    // (profiles/r05/heads_place_ab.json; 2 = after the chain: 7 us slower).  The per-layer
    // schedule keeps them on the side stream
    const char* hp = std::getenv("NERF_HEADS_PLACE");
    const int heads_place = a.bwd_chain ? (hp ? std::atoi(hp) : 1) : 0;
    auto heads = [&](hipStream_t s) -> int {
        RC(nerf_heads_bwd_mode(2, graw4, a.act[7], D, a.act[LR], HR, nullptr, 0, D, a.wc, nullptr, 0, w.part, np,
                               nullptr, nullptr, s));
        return nerf_heads_reduce(w.part, D, np, a.g_wd, a.g_bd, a.g_wc, a.g_bc, 0, s);
    };
    // NERF_HEADS_PLACE 3 (an A/B option; 1 is the default): the partials by k_heads_part (16-byte
    // loads, 4x the waves) before the chain, their reduces in the weight gradients' first slab batch
    nerf::SlabJobDesc hjobs[2];
    int n_hjobs = 0;
    if (heads_place == 0) {
        RC(fork(main, side));
        RC(heads(side));
    } else if (heads_place == 1) {
        RC(heads(main));
    } else if (heads_place == 5) {
        // the partials before the chain, their reduce (11 blocks) forked to the side stream
        RC(nerf_heads_bwd_mode(2, graw4, a.act[7], D, a.act[LR], HR, nullptr, 0, D, a.wc, nullptr, 0, w.part, np,
                               nullptr, nullptr, main));
        RC(fork(main, side));
        RC(nerf_heads_reduce(w.part, D, np, a.g_wd, a.g_bd, a.g_wc, a.g_bc, 0, side));
    } else if (heads_place == 3) {
        RC(nerf::heads_partials(graw4, a.act[7], D, a.act[LR], HR, np, w.hpart, a.g_wd, a.g_bd, a.g_wc, a.g_bc, hjobs,
                                main));
        n_hjobs = 2;
    }
    if (!a.bwd_chain)
        RC(nerf_heads_bwd_mode(1, graw4, nullptr, 0, nullptr, 0, a.mask[LR], HR / 32, D, a.wc, w.dyr, HR, nullptr, np,
                               w.dyr_rm, w.dyr_cm, stream));

    if (a.bwd_chain) {
        return chain_schedule(a, w, graw4, stream, side_stream, heads_place == 2, hjobs, n_hjobs);
    }

    const float *dy = w.dyr, *dy_rm = w.dyr_rm, *dy_cm = w.dyr_cm;
    int deferred[L], nd = 0;
    const float *def_dy[L], *def_cm[L];
    for (int step = 0; step < L; ++step) {
        const int l = L - 1 - step;   // lr, lf, l7, ..., l0
        if (step >= L - a.tail_main) {
            deferred[nd] = l; def_dy[nd] = dy; def_cm[nd] = dy_cm; ++nd;
        } else {
            RC(fork(main, side));
            RC(weight_grad(a, w, l, dy, dy_cm, side_stream));
        }
        // input gradient: dx = (dy W) masked by the ReLU words of the layer's input
        const int op = OUT_P[l];
        const uint16_t* img = a.wt_img[l];
        const int img_rows = KP[l];
        if (l == 0) {
            if (a.ray_grad)
                RC(nerf_linear_bwd_data(dy, op, op, a.wt[l], img, img_rows, nullptr, 0, nullptr, nullptr, 0, w.genc_p0,
                                        64, np, 64, dy_rm, nullptr, nullptr, stream));
            break;
        }
        if (SEG[l] && a.ray_grad)
            RC(nerf_linear_bwd_data(dy, op, op, a.wt[l] + (size_t)K1[l] * op, img + (size_t)K1[l] * 8, img_rows,
                                    nullptr, 0, nullptr, nullptr, 0, SEG[l] == 1 ? w.genc_p4 : w.genc_d, 64, np, 64,
                                    dy_rm, nullptr, nullptr, stream));
        const uint32_t* mask = l == LR ? nullptr : a.mask[l - 1];
        const int ldmask = OUT_P[l - 1 < 0 ? 0 : l - 1] / 32;
        if (l == LF)   // + the density path: d sigma_raw (graw4[:, 0]) x w_density, rank one
            RC(nerf_linear_bwd_data(dy, op, op, a.wt[l], img, img_rows, graw4, 4, a.wd, mask, ldmask, w.dx[l], K1[l],
                                    np, K1[l], dy_rm, w.dx_rm[l], w.dx_cm[l], stream));
        else
            RC(nerf_linear_bwd_data(dy, op, op, a.wt[l], img, img_rows, nullptr, 0, nullptr, mask, ldmask, w.dx[l],
                                    K1[l], np, K1[l], dy_rm, w.dx_rm[l], w.dx_cm[l], stream));
        dy = w.dx[l]; dy_rm = w.dx_rm[l]; dy_cm = w.dx_cm[l];
    }
    for (int i = 0; i < nd; ++i) RC(weight_grad(a, w, deferred[i], def_dy[i], def_cm[i], stream));
    // join: the side stream's gradients are complete before the caller's stream goes on
    RC(fork(side, main));
    if (a.ray_grad)
        RC(nerf_encode_bwd(a.pts_o, a.pts_d, a.view, a.z, w.genc_p0, w.genc_p4, w.genc_d, a.n_rays, a.n_samples,
                           a.g_pts_o, a.g_pts_d, a.g_view, stream));
    return NERF_OK;
}
}  // namespace
