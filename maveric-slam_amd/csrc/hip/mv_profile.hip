// mv_profile.hip -- per-kernel device-time accounting with hipEvents (bench.py's
// live roofline measurement).  Disabled by default: one branch per launch.
#include <mutex>
#include <string.h>
#include <vector>

#include "mv_internal.hpp"

namespace {
struct Rec {
    const char *name;
    hipEvent_t a, b;
    bool closed;
};
std::mutex g_mu;
bool g_on = false;
std::vector<Rec> g_recs;
std::vector<hipEvent_t> g_pool;

hipEvent_t take_event() {
    if (!g_pool.empty()) {
        hipEvent_t e = g_pool.back();
        g_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

void recycle_all() {
    for (auto &r : g_recs) {
        g_pool.push_back(r.a);
        g_pool.push_back(r.b);
    }
    g_recs.clear();
}
}  // namespace

namespace mv {
bool prof_on() { return g_on; }

void prof_begin(hipStream_t s, const char *kernel) {
    std::lock_guard<std::mutex> lk(g_mu);
    Rec r{kernel, take_event(), take_event(), false};
    (void)hipEventRecord(r.a, s);
    g_recs.push_back(r);
}

void prof_end(hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto it = g_recs.rbegin(); it != g_recs.rend(); ++it)
        if (!it->closed) {
            (void)hipEventRecord(it->b, s);
            it->closed = true;
            return;
        }
}
}  // namespace mv

extern "C" int mv_profile_enable(int on) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (on) {
        for (auto &r : g_recs) (void)hipEventSynchronize(r.b);
        recycle_all();
    }
    g_on = on != 0;
    return MV_OK;
}

extern "C" int mv_profile_query(const char *kernel, double *total_ms, int *launches) {
    MV_REQUIRE(kernel && total_ms && launches);
    std::lock_guard<std::mutex> lk(g_mu);
    double tot = 0;
    int n = 0;
    for (auto &r : g_recs) {
        if (!r.closed || strcmp(r.name, kernel) != 0) continue;
        MV_HIP_TRY(hipEventSynchronize(r.b));
        float ms = 0;
        MV_HIP_TRY(hipEventElapsedTime(&ms, r.a, r.b));
        tot += ms;
        n++;
    }
    *total_ms = tot;
    *launches = n;
    return MV_OK;
}
