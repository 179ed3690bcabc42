// cg_ktime.hip -- live device time of the hot kernels, for the bench's
// roofline: a pair of HIP events around each timed launch, recorded on the
// stream the kernel is launched on (the certificate kernels of a batched call
// run on the context's auxiliary stream, the rasteriser's overlapped frames on
// its lane streams: events on the caller's stream would time the wrong span).
// Off by default: a disabled scope records nothing.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <utility>
#include <vector>

#include "cg_internal.h"

namespace cg {

static const char *const kKtNames[KT_COUNT] = {
    "rt_prepare_kernel",        "rt_tile_cert_kernel",   "rt_lattice_units_kernel", "rt_lattice_kernel",
    "rt_lattice_lights_kernel", "rt_pixel_kernel",       "rt_big_primary_kernel",   "rt_shadow_hints_kernel",
    "rt_big_frame",             "rast_fill_kernel",      "rast_post_kernel",
};

namespace {
constexpr size_t kKtPoolEvents = 512;   // pre-created when timing is switched on (256 timed launches)
struct Pending {
    int id;
    hipEvent_t a, b;
    bool a_is_ref = false;   // a is `ref` itself (the session's first timed launch): never pooled
};
struct KtState {
    std::mutex mu;
    bool on = false;
    bool all = false;                   // also time the certificate launches (CG_KTIME_ALL=1)
    std::atomic<bool> on_fast{false};   // read without the lock: a disabled scope costs one load
    std::vector<hipEvent_t> pool;
    std::vector<Pending> pending;
    double ms[KT_COUNT] = {};
    long long n[KT_COUNT] = {};
    // each launch's [start, end] in ms after `ref` (the first timed launch since
    // timing was switched on): launches of one kernel that overlap (two frames in
    // flight on two streams) count once in its busy time
    hipEvent_t ref = nullptr;
    bool ref_set = false;
    std::vector<std::pair<double, double>> spans[KT_COUNT];
    void settle(const Pending &p)
    {
        float ms1 = 0.f, t0 = 0.f;
        if (hipEventElapsedTime(&ms1, p.a, p.b) == hipSuccess) {
            ms[p.id] += ms1;
            ++n[p.id];
            if (ref_set && hipEventElapsedTime(&t0, ref, p.a) == hipSuccess)
                spans[p.id].emplace_back((double)t0, (double)t0 + ms1);
        }
        if (!p.a_is_ref) pool.push_back(p.a);
        pool.push_back(p.b);
    }
    // Settle the recorded pairs into the totals (blocks until they completed).
    void flush()
    {
        for (const Pending &p : pending) {
            (void)hipEventSynchronize(p.b);
            settle(p);
        }
        pending.clear();
    }
    // Settle the pairs that already completed, without blocking (keeps
    // `pending` bounded in long timed runs).
    void settle_completed()
    {
        size_t k = 0;
        for (const Pending &p : pending) {
            if (hipEventQuery(p.b) == hipSuccess) settle(p);
            else pending[k++] = p;
        }
        pending.resize(k);
    }
    // union length of a kernel's launch spans
    double busy(int id)
    {
        std::vector<std::pair<double, double>> v = spans[id];
        std::sort(v.begin(), v.end());
        double tot = 0.0, s = 0.0, e = -1e300;
        for (const auto &x : v) {
            if (x.first > e) {
                if (e > s) tot += e - s;
                s = x.first;
                e = x.second;
            } else {
                e = std::max(e, x.second);
            }
        }
        if (!v.empty() && e > s) tot += e - s;
        return tot;
    }
    hipEvent_t get()
    {
        if (pool.empty()) settle_completed();   // recycle the pairs that completed
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        return hipEventCreate(&e) == hipSuccess ? e : nullptr;
    }
};
KtState &kt()
{
    static KtState s;
    return s;
}
}  // namespace

KtScope::KtScope(int id, hipStream_t st) : id_(id), st_(st)
{
    KtState &s = kt();
    if (!s.on_fast.load(std::memory_order_relaxed)) return;
    std::lock_guard<std::mutex> g(s.mu);
    if (!s.on || id < 0 || id >= KT_COUNT) return;
    if (!s.ref_set) {
        if (!s.ref && hipEventCreate(&s.ref) != hipSuccess) s.ref = nullptr;
        s.ref_set = s.ref && hipEventRecord(s.ref, st) == hipSuccess;
    }
    a_ = s.get();
    if (a_ && hipEventRecord(a_, st) != hipSuccess) {
        s.pool.push_back(a_);
        a_ = nullptr;
    }
}

KtScope::~KtScope()
{
    if (!a_) return;
    KtState &s = kt();
    std::lock_guard<std::mutex> g(s.mu);
    hipEvent_t b = s.get();
    if (!s.on || !b || hipEventRecord(b, st_) != hipSuccess) {
        s.pool.push_back(a_);
        if (b) s.pool.push_back(b);
        return;
    }
    s.pending.push_back({id_, a_, b});
    if (s.pending.size() >= 2048) s.settle_completed();
}

KtLaunch::KtLaunch(int id, hipStream_t st) : id_(id)
{
    KtState &s = kt();
    if (!s.on_fast.load(std::memory_order_relaxed)) return;
    std::lock_guard<std::mutex> g(s.mu);
    if (!s.on || id < 0 || id >= KT_COUNT) return;
    // the certificate launches ride untimed unless CG_KTIME_ALL=1: no roofline reads them, and a
    // timed (profiled) dispatch costs host time in front of the lattice launch that follows
    if (!s.all && (id == KT_RT_PREPARE || id == KT_RT_TILE_CERT || id == KT_RT_LATTICE_UNITS)) return;
    // the session's first timed launch records the anchor of the busy-time spans as its own
    // start event: no marker packet of its own in front of the launch (one cost ~1 % of the
    // metric's 20-frame call)
    const bool first = !s.ref_set && s.ref;
    a = first ? s.ref : s.get();
    b = s.get();
    if (!a || !b) {
        if (a && !first) s.pool.push_back(a);
        if (b) s.pool.push_back(b);
        a = b = nullptr;
        return;
    }
    if (first) {
        s.ref_set = true;
        ref_ = true;
    }
}

KtLaunch::~KtLaunch()
{
    if (!a) return;
    KtState &s = kt();
    std::lock_guard<std::mutex> g(s.mu);
    if (!s.on) {
        if (!ref_) s.pool.push_back(a);
        s.pool.push_back(b);
        return;
    }
    s.pending.push_back({id_, a, b, ref_});
    if (s.pending.size() >= 2048) s.settle_completed();
}

}  // namespace cg

using namespace cg;

extern "C" int cg_kernel_timing(int enable)
{
    KtState &s = kt();
    std::lock_guard<std::mutex> g(s.mu);
    s.flush();
    std::memset(s.ms, 0, sizeof(s.ms));
    std::memset(s.n, 0, sizeof(s.n));
    for (auto &v : s.spans) v.clear();
    s.ref_set = false;
    s.on = enable != 0;
    {
        const char *e = std::getenv("CG_KTIME_ALL");
        s.all = e && e[0] == '1';
    }
    if (s.on) {
        // every event a timed region will record, created here rather than in front of
        // the timed launches: a hipEventCreate per event in the launch path cost ~15 us of
        // host time per call (two launches), which a band call's second launch waited for
        if (!s.ref && hipEventCreate(&s.ref) != hipSuccess) s.ref = nullptr;
        while (s.pool.size() < kKtPoolEvents) {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) break;
            s.pool.push_back(e);
        }
    }
    s.on_fast.store(s.on);
    return CG_OK;
}

extern "C" int cg_kernel_time(const char *kernel, double *total_ms, double *busy_ms, long long *launches)
{
    if (!kernel || !total_ms || !busy_ms || !launches) return CG_E_INVALID;
    KtState &s = kt();
    std::lock_guard<std::mutex> g(s.mu);
    s.flush();
    for (int k = 0; k < KT_COUNT; ++k)
        if (std::strcmp(kernel, kKtNames[k]) == 0) {
            *total_ms = s.ms[k];
            *busy_ms = s.ref_set ? s.busy(k) : s.ms[k];
            *launches = s.n[k];
            return CG_OK;
        }
    return CG_E_INVALID;
}
