// Error reporting and GEMM timing hooks of the nerf_hip C-ABI.
#include "common.hpp"

#include <algorithm>
#include <mutex>
#include <vector>

namespace nerf {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// ---- GEMM timing: hipEvent pairs around each GEMM launch (bench.py roofline) ----
struct ProfRec {
    hipEvent_t a, b;
    double flops, bytes;
    int kind, products;
};
static std::mutex g_prof_mu;
static bool g_prof_on = false;
static std::vector<ProfRec> g_pool;
static size_t g_used = 0;

static thread_local int g_next_kind = 0;
static thread_local double g_next_bytes = 0;

void prof_next(int kind, double bytes) {
    g_next_kind = kind;
    g_next_bytes = bytes;
}

void prof_begin(hipStream_t s) {
    if (!g_prof_on) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (g_used == g_pool.size()) {
        ProfRec r;
        (void)hipEventCreate(&r.a);
        (void)hipEventCreate(&r.b);
        r.flops = r.bytes = 0;
        r.kind = 0;
        r.products = 1;
        g_pool.push_back(r);
    }
    (void)hipEventRecord(g_pool[g_used].a, s);
}

void prof_end(hipStream_t s, double flops, int products) {
    if (!g_prof_on) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    (void)hipEventRecord(g_pool[g_used].b, s);
    g_pool[g_used].flops = flops;
    g_pool[g_used].bytes = g_next_bytes;
    g_pool[g_used].kind = g_next_kind;
    g_pool[g_used].products = products;
    ++g_used;
}

}  // namespace nerf

extern "C" {

int nerf_hip_abi_version(void) { return NERF_HIP_ABI_VERSION; }

const char* nerf_hip_last_error(void) { return nerf::g_err; }

int nerf_prof_enable(int on) {
    std::lock_guard<std::mutex> lk(nerf::g_prof_mu);
    nerf::g_prof_on = on != 0;
    nerf::g_used = 0;
    return NERF_OK;
}

int nerf_prof_read_kinds(nerf_prof_kind* out, int n_kinds) {
    NERF_CHECK_PTR(out);
    NERF_CHECK(n_kinds >= NERF_PROF_KINDS, "%s: need %d slots", __func__, NERF_PROF_KINDS);
    std::lock_guard<std::mutex> lk(nerf::g_prof_mu);
    for (int k = 0; k < n_kinds; ++k) out[k] = nerf_prof_kind{};
    for (size_t i = 0; i < nerf::g_used; ++i) {
        const auto& r = nerf::g_pool[i];
        (void)hipEventSynchronize(r.b);
        float t = 0;
        (void)hipEventElapsedTime(&t, r.a, r.b);
        nerf_prof_kind& o = out[r.kind];
        o.ms += t;
        o.launches += 1;
        o.flops += r.flops;
        o.bytes += r.bytes;
        o.mfma_flops += r.flops * r.products;
        o.exact_f32 |= r.products == 1;
    }
    return NERF_OK;
}

int nerf_prof_read(double* gemm_ms, int64_t* gemm_launches, double* gemm_flops, double* union_ms) {
    NERF_CHECK_PTR(gemm_ms);
    NERF_CHECK_PTR(gemm_launches);
    NERF_CHECK_PTR(gemm_flops);
    std::lock_guard<std::mutex> lk(nerf::g_prof_mu);
    double ms = 0, fl = 0;
    // launch intervals relative to the first start event: summed durations (per-launch
    // average) and the union of the intervals (GEMM family running concurrently on two
    // streams counts once)
    std::vector<std::pair<double, double>> iv;
    for (size_t i = 0; i < nerf::g_used; ++i) {
        (void)hipEventSynchronize(nerf::g_pool[i].b);
        float t = 0, a = 0, b = 0;
        (void)hipEventElapsedTime(&t, nerf::g_pool[i].a, nerf::g_pool[i].b);
        (void)hipEventElapsedTime(&a, nerf::g_pool[0].a, nerf::g_pool[i].a);
        (void)hipEventElapsedTime(&b, nerf::g_pool[0].a, nerf::g_pool[i].b);
        iv.emplace_back(a, b);
        ms += t;
        fl += nerf::g_pool[i].flops;
    }
    std::sort(iv.begin(), iv.end());
    double un = 0, cs = -1e30, ce = -1e30;
    for (auto& x : iv) {
        if (x.first > ce) {
            if (ce > cs) un += ce - cs;
            cs = x.first;
            ce = x.second;
        } else if (x.second > ce) {
            ce = x.second;
        }
    }
    if (ce > cs) un += ce - cs;
    *gemm_ms = ms;
    *gemm_launches = (int64_t)nerf::g_used;
    *gemm_flops = fl;
    if (union_ms) *union_ms = un;
    nerf::g_used = 0;
    return NERF_OK;
}

}  // extern "C"
