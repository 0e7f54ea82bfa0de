// Error reporting and GEMM timing hooks of the nerf_hip C-ABI.
#include "common.hpp"

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
    double flops;
};
static std::mutex g_prof_mu;
static bool g_prof_on = false;
static std::vector<ProfRec> g_pool;
static size_t g_used = 0;

void prof_begin(hipStream_t s) {
    if (!g_prof_on) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (g_used == g_pool.size()) {
        ProfRec r;
        (void)hipEventCreate(&r.a);
        (void)hipEventCreate(&r.b);
        r.flops = 0;
        g_pool.push_back(r);
    }
    (void)hipEventRecord(g_pool[g_used].a, s);
}

void prof_end(hipStream_t s, double flops) {
    if (!g_prof_on) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    (void)hipEventRecord(g_pool[g_used].b, s);
    g_pool[g_used].flops = flops;
    ++g_used;
}

}  // namespace nerf

extern "C" {

int nerf_hip_abi_version(void) { return 1; }

const char* nerf_hip_last_error(void) { return nerf::g_err; }

int nerf_prof_enable(int on) {
    std::lock_guard<std::mutex> lk(nerf::g_prof_mu);
    nerf::g_prof_on = on != 0;
    nerf::g_used = 0;
    return NERF_OK;
}

int nerf_prof_read(double* gemm_ms, int64_t* gemm_launches, double* gemm_flops) {
    NERF_CHECK_PTR(gemm_ms);
    NERF_CHECK_PTR(gemm_launches);
    NERF_CHECK_PTR(gemm_flops);
    std::lock_guard<std::mutex> lk(nerf::g_prof_mu);
    double ms = 0, fl = 0;
    for (size_t i = 0; i < nerf::g_used; ++i) {
        (void)hipEventSynchronize(nerf::g_pool[i].b);
        float t = 0;
        (void)hipEventElapsedTime(&t, nerf::g_pool[i].a, nerf::g_pool[i].b);
        ms += t;
        fl += nerf::g_pool[i].flops;
    }
    *gemm_ms = ms;
    *gemm_launches = (int64_t)nerf::g_used;
    *gemm_flops = fl;
    nerf::g_used = 0;
    return NERF_OK;
}

}  // extern "C"
