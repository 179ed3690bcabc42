// cg_dist.hip -- multi-GPU raytracer frames, one process per GPU.
//
// The reference's Draw (raytracer/Source/skeleton.cpp:104-169) renders every
// pixel independently on one CPU thread, so the frame shards by rows with no
// exchange while rendering.  Rank r renders the contiguous band of frame
// rows [row0_r, row0_r + rows_r); ranks > 0 render it in the RGB24 wire
// format (PutPixelSDL's alpha is constant) and only in the columns the camera
// can see anything in (cg_rt_frame_columns: the rest is certainly black), and
// send it to rank 0 with one RCCL point-to-point send per chunk of frames --
// on MI355X every peer has its own xGMI link to rank 0, so the sends run in
// parallel; rank 0 renders its own band straight into the caller's frames and
// expands the received bands in place (rt_assemble_kernel).  The transfer of
// a chunk of frames (on the transfer stream) overlaps the render of the later
// frames (on the caller's stream): by default (CG_DIST_SIGNALLED) a call's
// frames render in full-size lattice launches that count each frame's stored
// tiles in uncached device memory, and the transfer stream waits on those
// counts (hipStreamWaitValue32) before sending a chunk -- small per-chunk
// launches would lose ~15-25 % to launch tails, more so on a 1/8 band;
// CG_DIST_CHUNKED instead launches chunk by chunk through two buffer slots
// ordered by events.  Band boundaries come from measured per-rank times
// (cg_dist_rebalance): the row cost of the Cornell box is far from uniform
// (tiles that certainly miss everything exit at once, the floor and boxes
// cost most).
//
// Transports: RCCL (cg_dist_create) or, for tests, an in-process group of
// contexts whose bands move by device-to-device copies (cg_dist_create_local).
//
// Bounded failure: the communicator is non-blocking (ncclConfig_t.blocking =
// 0), so no RCCL call blocks the host; every host wait of this file (init,
// the rebalance's collectives, cg_dist_wait, destroy) polls completion and
// ncclCommGetAsyncError against a deadline (cg_dist_set_timeout, default
// CG_DIST_TIMEOUT_MS or 60 s).  On an RCCL error or a passed deadline the
// communicator is aborted (ncclCommAbort: RCCL kernels still waiting on a
// peer exit), the call returns CG_E_HIP / CG_E_TIMEOUT, and every later call
// on the handle fails -- a missing peer ends the job with an error code
// instead of hanging it.
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "cg_internal.h"

namespace cg {
int rt_render_frames(cg_ctx *c, const cg_light *lights, int n_lights, const cg_rt_camera *cams, int n_frames,
                     const cg_rt_shard *shard, void *d_out, size_t frame_stride, int pix_format, void *stream,
                     uint32_t *d_done, uint32_t *target, const int *group_starts, int ngroups);
int ctx_device(const cg_ctx *c);
hipStream_t ctx_stream(const cg_ctx *c);
void ctx_set_error(cg_ctx *c, const std::string &e);
void ctx_rt_columns(const cg_ctx *c, const cg_rt_camera *cam, int *c0, int *c1);
}  // namespace cg

using namespace cg;

namespace {

constexpr int kBandAlign = kLatTileH;   // default band boundaries: whole lattice tile rows

struct Mem {
    void *p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t n)
    {
        if (n <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    ~Mem()
    {
        if (p) (void)hipFree(p);
    }
};

struct TimedPair {
    hipEvent_t a = nullptr, b = nullptr;
    int frames = 0;
};

struct LocalGroup;

}  // namespace

struct cg_dist {
    cg_ctx *ctx = nullptr;
    int nranks = 1, rank = 0;
    ncclComm_t comm = nullptr;        // RCCL transport
    LocalGroup *group = nullptr;      // in-process transport (tests)
    hipStream_t xs = nullptr;         // transfer stream
    int height = 0;                   // frame height the bands are for
    std::vector<int> row0, rows;      // band of every rank
    int chunk = 4;                    // frames per chunk
    Mem sbuf[2], rbuf[2];             // send (ranks > 0) / receive (rank 0) slots
    Mem sall;                         // local transport: a peer's whole call
    hipEvent_t ev_rend[2] = {}, ev_sent[2] = {}, ev_recv[2] = {}, ev_asm[2] = {}, ev_done = nullptr;
    std::vector<hipEvent_t> ev_chunk; // local transport: a peer's chunk j rendered
    std::vector<TimedPair> t_rend, t_asm;   // timing of the last call (reused event pool)
    size_t n_rend = 0, n_asm = 0;
    Mem stats;                        // rebalance: gathered per-rank times (device)
    int last_pitch = 0;               // local transport: the peer's window pitch of its last call
    size_t last_frames = 0;
    // Signalled pipeline (when the device supports stream waits on memory):
    // a call renders all its frames in one launch and the transfer stream
    // waits on per-frame completion counts (rt_render_frames' d_done).
    bool signals = false;
    unsigned calls = 0;               // call parity selects the slot below
    uint32_t *done[2] = {nullptr, nullptr};
    size_t done_cap[2] = {0, 0};
    std::vector<uint32_t> target[2];
    hipEvent_t ev_call[2] = {};       // ranks > 0: slot free again (its sends / copies done)
    hipEvent_t ev_zero[2] = {};       // ranks > 0: the slot's counts zeroed for this call (on st)
    hipEvent_t ev_start = nullptr;    // rank 0: the caller's stream at the start of the call
    int cur = 0;                      // slot of the last call
    // bounded waits
    int timeout_ms = 60000;           // deadline of every host wait
    bool aborted = false;             // communicator aborted after an error / timeout
    bool leaked = false;              // the abort did not finish in time: device memory kept (see abort_comm)
    hipStream_t last_st = nullptr;    // render stream of the last call
    hipEvent_t ev_wait[2] = {};       // cg_dist_wait: render stream, transfer stream
};

namespace {

struct LocalGroup {
    std::vector<cg_dist *> members;
};

int fail(cg_dist *d, int code, const std::string &what)
{
    if (d && d->ctx) ctx_set_error(d->ctx, what);
    return code;
}
#define DT(d, call, what)                                                                          \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess) return fail((d), CG_E_HIP, std::string(what) + ": " + hipGetErrorString(e_)); \
    } while (0)

using Clock = std::chrono::steady_clock;

int default_timeout_ms()
{
    const char *e = std::getenv("CG_DIST_TIMEOUT_MS");
    const long v = e ? std::strtol(e, nullptr, 10) : 0;
    return v > 0 && v < (1L << 30) ? (int)v : 60000;
}

// Pause between two polls of a bounded wait that began at `since`: the first 5 ms only yield
// (a wait at the end of a call is timed by its caller -- bench.py's N > 1 loop ends on
// cg_dist_wait -- and a 20 us sleep rounds up to the kernel's timer slack, ~50-60 us), then
// sleep 20 us per poll.
void poll_pause(Clock::time_point since = Clock::time_point::min())
{
    if (since != Clock::time_point::min() && Clock::now() - since < std::chrono::milliseconds(5))
        std::this_thread::yield();
    else
        std::this_thread::sleep_for(std::chrono::microseconds(20));
}

// ncclCommAbort on a helper thread, joined for at most 10 s: an abort that
// itself stalls (a peer's socket never answering) must not turn the error
// return into the hang it reports.
void abort_comm(cg_dist *d)
{
    d->aborted = true;
    ncclComm_t c = d->comm;
    d->comm = nullptr;
    if (!c) return;
    auto done = std::make_shared<std::atomic<bool>>(false);
    std::thread t([c, done] {
        (void)ncclCommAbort(c);
        done->store(true);
    });
    const auto end = Clock::now() + std::chrono::seconds(10);
    while (!done->load() && Clock::now() < end) poll_pause();
    if (done->load()) {
        t.join();
    } else {
        // the abort is still running, and RCCL kernels it has not yet ended may
        // still read or write this handle's buffers: cg_dist_destroy leaks them
        // (and the streams) rather than free memory a running kernel may touch
        t.detach();
        d->leaked = true;
    }
}

// The communicator's state after an RCCL call: ncclInProgress (non-blocking
// mode) is polled through ncclCommGetAsyncError until it settles or the
// deadline passes.  Errors and timeouts abort the communicator.
int nccl_settle(cg_dist *d, ncclResult_t r, const char *what)
{
    if (r == ncclInProgress && d->comm) {
        const auto t0 = Clock::now(), end = t0 + std::chrono::milliseconds(d->timeout_ms);
        for (;;) {
            ncclResult_t st = ncclSuccess;
            const ncclResult_t q = ncclCommGetAsyncError(d->comm, &st);
            r = q == ncclSuccess ? st : q;
            if (r != ncclInProgress) break;
            if (Clock::now() >= end) {
                abort_comm(d);
                return fail(d, CG_E_TIMEOUT, std::string(what) + ": no progress within " + std::to_string(d->timeout_ms) +
                                                 " ms (a peer missing?); communicator aborted");
            }
            poll_pause(t0);
        }
    }
    if (r == ncclSuccess) return CG_OK;
    abort_comm(d);
    return fail(d, CG_E_HIP, std::string(what) + ": " + ncclGetErrorString(r) + "; communicator aborted");
}
#define DN(d, call, what)                                      \
    do {                                                       \
        if ((d)->aborted) return fail((d), CG_E_HIP, "communicator was aborted by an earlier error"); \
        int rc_ = nccl_settle((d), (call), (what));            \
        if (rc_) return rc_;                                   \
    } while (0)

// Rank 0's receives of one chunk from ranks 1 .. n-1 (bytes[p] each, packed
// from buf in rank order) as one RCCL group.  The group is always closed --
// ncclGroupEnd runs even when a receive inside it failed -- before the error
// is settled (and the communicator aborted), so the calling thread's RCCL group
// depth never stays open after an error return.
int recv_group(cg_dist *d, uint8_t *buf, const size_t *bytes, int n)
{
    if (d->aborted) return fail(d, CG_E_HIP, "communicator was aborted by an earlier error");
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return nccl_settle(d, r, "ncclGroupStart");
    ncclResult_t first = ncclSuccess;
    size_t off = 0;
    for (int p = 1; p < n; ++p) {
        if (bytes[p] && first == ncclSuccess) {
            r = ncclRecv(buf + off, bytes[p], ncclUint8, p, d->comm, d->xs);
            if (r != ncclSuccess && r != ncclInProgress) first = r;
        }
        off += bytes[p];
    }
    const ncclResult_t e = ncclGroupEnd();
    return first != ncclSuccess ? nccl_settle(d, first, "ncclRecv") : nccl_settle(d, e, "ncclGroupEnd");
}

// Host wait for events (nullptr entries skipped) against the deadline, polling
// the communicator's asynchronous error meanwhile.  The deadline runs from the
// last progress -- the start of the wait, or the latest event seen complete --
// so a healthy rank that queued more than timeout_ms of work in several steps
// is not aborted; a wait on ONE event still covers everything queued before it.
int wait_events(cg_dist *d, const hipEvent_t *ev, int n, const char *what)
{
    const auto t0 = Clock::now();
    auto end = t0 + std::chrono::milliseconds(d->timeout_ms);
    for (int i = 0; i < n;) {
        if (!ev[i]) {
            ++i;
            continue;
        }
        const hipError_t q = hipEventQuery(ev[i]);
        if (q == hipSuccess) {
            ++i;
            end = Clock::now() + std::chrono::milliseconds(d->timeout_ms);
            continue;
        }
        if (q != hipErrorNotReady) return fail(d, CG_E_HIP, std::string(what) + ": " + hipGetErrorString(q));
        if (d->comm) {
            ncclResult_t st = ncclSuccess;
            const ncclResult_t r = ncclCommGetAsyncError(d->comm, &st);
            const ncclResult_t e = r == ncclSuccess ? st : r;
            if (e != ncclSuccess && e != ncclInProgress) {
                abort_comm(d);
                return fail(d, CG_E_HIP, std::string(what) + ": " + ncclGetErrorString(e) + "; communicator aborted");
            }
        }
        if (Clock::now() >= end) {
            abort_comm(d);
            return fail(d, CG_E_TIMEOUT, std::string(what) + ": not done within " + std::to_string(d->timeout_ms) +
                                             " ms; communicator aborted");
        }
        poll_pause(t0);
    }
    return CG_OK;
}

// Bounded host wait for everything this rank enqueued: the last call's render
// stream and the transfer stream.
int drain(cg_dist *d, hipStream_t st, const char *what)
{
    if (!d->ev_done) return CG_OK;   // nothing enqueued yet
    DT(d, hipSetDevice(ctx_device(d->ctx)), "hipSetDevice");
    for (int k = 0; k < 2; ++k)
        if (!d->ev_wait[k]) DT(d, hipEventCreateWithFlags(&d->ev_wait[k], hipEventDisableTiming), "event");
    if (!st) st = d->last_st ? d->last_st : ctx_stream(d->ctx);
    DT(d, hipEventRecord(d->ev_wait[0], st), "event");
    DT(d, hipEventRecord(d->ev_wait[1], d->xs), "event");
    return wait_events(d, d->ev_wait, 2, what);
}

void equal_bands(int H, int n, std::vector<int> &row0, std::vector<int> &rows)
{
    const int units = (H + kBandAlign - 1) / kBandAlign;
    row0.assign(n, 0);
    rows.assign(n, 0);
    for (int r = 0; r < n; ++r) {
        const int a = std::min(H, (int)((long long)units * r / n) * kBandAlign);
        const int b = r + 1 == n ? H : std::min(H, (int)((long long)units * (r + 1) / n) * kBandAlign);
        row0[r] = a;
        rows[r] = b - a;
    }
}

// Bisection on the makespan T with a greedy sweep (cgdist.band_partition).
void band_partition(const double *cost, int H, int n, const double *ovh, int *row0, int *rows)
{
    std::vector<double> C(H + 1, 0.0), o(n, 0.0);
    for (int i = 0; i < H; ++i) C[i + 1] = C[i] + cost[i];
    if (ovh)
        for (int r = 0; r < n; ++r) o[r] = ovh[r];
    auto sweep = [&](double T, std::vector<int> &b) {
        b.assign(1, 0);
        for (int r = 0; r < n - 1; ++r) {
            const int lo = b.back(), left = n - 1 - r;
            const int hi_max = H >= n ? std::max(lo + 1, H - left) : lo + (lo < H ? 1 : 0);
            // largest end with cost <= T (at least one row, leaving one per later rank)
            const double target = C[lo] + T - o[r];
            int end = (int)(std::upper_bound(C.begin(), C.end(), target) - C.begin()) - 1;
            end = std::min(std::max(end, lo < H ? lo + 1 : lo), hi_max);
            b.push_back(end);
        }
        b.push_back(H);
    };
    double lo_T = 0.0, hi_T = C[H] + *std::max_element(o.begin(), o.end()) + 1.0;
    std::vector<int> b;
    for (int it = 0; it < 60; ++it) {
        const double T = 0.5 * (lo_T + hi_T);
        sweep(T, b);
        const double last = C[b[n]] - C[b[n - 1]] + o[n - 1];
        if (last <= T) hi_T = T;
        else lo_T = T;
    }
    sweep(hi_T, b);
    for (int r = 0; r < n; ++r) {
        row0[r] = b[r];
        rows[r] = b[r + 1] - b[r];
    }
}

int ensure_events(cg_dist *d)
{
    if (d->ev_done) return CG_OK;
    DT(d, hipSetDevice(ctx_device(d->ctx)), "hipSetDevice");
    DT(d, hipStreamCreateWithFlags(&d->xs, hipStreamNonBlocking), "transfer stream");
    for (int k = 0; k < 2; ++k) {
        DT(d, hipEventCreateWithFlags(&d->ev_rend[k], hipEventDisableTiming), "event");
        DT(d, hipEventCreateWithFlags(&d->ev_sent[k], hipEventDisableTiming), "event");
        DT(d, hipEventCreateWithFlags(&d->ev_recv[k], hipEventDisableTiming), "event");
        DT(d, hipEventCreateWithFlags(&d->ev_asm[k], hipEventDisableTiming), "event");
        // recorded once so the first waits on them are satisfied
        DT(d, hipEventRecord(d->ev_sent[k], d->xs), "event");
        DT(d, hipEventRecord(d->ev_asm[k], d->xs), "event");
    }
    DT(d, hipEventCreateWithFlags(&d->ev_done, hipEventDisableTiming), "event");
    for (int k = 0; k < 2; ++k) {
        DT(d, hipEventCreateWithFlags(&d->ev_call[k], hipEventDisableTiming), "event");
        DT(d, hipEventRecord(d->ev_call[k], d->xs), "event");
        DT(d, hipEventCreateWithFlags(&d->ev_zero[k], hipEventDisableTiming), "event");
        DT(d, hipEventRecord(d->ev_zero[k], d->xs), "event");
    }
    DT(d, hipEventCreateWithFlags(&d->ev_start, hipEventDisableTiming), "event");
    int wait_value = 0;
    d->signals = hipDeviceGetAttribute(&wait_value, hipDeviceAttributeCanUseStreamWaitValue, ctx_device(d->ctx)) ==
                     hipSuccess && wait_value != 0;
    return CG_OK;
}

// the next timing pair of a pool (events created on first use)
int timed(cg_dist *d, std::vector<TimedPair> &pool, size_t &n, TimedPair *&out)
{
    if (n == pool.size()) {
        TimedPair t;
        DT(d, hipEventCreate(&t.a), "event");
        DT(d, hipEventCreate(&t.b), "event");
        pool.push_back(t);
    }
    out = &pool[n++];
    return CG_OK;
}

double pool_ms_per_frame(const std::vector<TimedPair> &pool, size_t n)
{
    double ms = 0.0;
    int f = 0;
    for (size_t i = 0; i < n; ++i) {
        float m = 0.f;
        if (hipEventSynchronize(pool[i].b) == hipSuccess && hipEventElapsedTime(&m, pool[i].a, pool[i].b) == hipSuccess)
            ms += m;
        f += pool[i].frames;
    }
    return f ? ms / f : 0.0;
}

// The columns whose pixels ranks > 0 send: the union of every camera's window.
void call_window(const cg_dist *d, const cg_rt_camera *cams, int n, int &c0, int &cols)
{
    const int W = cams[0].width;
    int a = W, b = 0;
    for (int f = 0; f < n; ++f) {
        int x0, x1;
        ctx_rt_columns(d->ctx, &cams[f], &x0, &x1);
        a = std::min(a, x0);
        b = std::max(b, x1);
    }
    if (b <= a) {   // nothing visible anywhere: keep a minimal window
        a = 0;
        b = std::min(W, 16);
    }
    if ((a == 0 && b == W) || (b - a) % 4) {
        c0 = 0;
        cols = 0;   // whole rows (the assembly needs a 4-aligned window)
    } else {
        c0 = a;
        cols = b - a;
    }
}

int render_band(cg_dist *d, const cg_light *lights, int n_lights, const cg_rt_camera *cams, int nf, int r0, int nr,
                int c0, int cols, void *dst, size_t stride, int fmt, hipStream_t st, uint32_t *d_done = nullptr,
                uint32_t *target = nullptr, const std::vector<int> *groups = nullptr)
{
    cg_rt_shard sh{0, 1, kLatTileH, r0, nr, fmt == CG_PIX_RGB24 ? c0 : 0, fmt == CG_PIX_RGB24 ? cols : 0};
    TimedPair *t;
    int rc = timed(d, d->t_rend, d->n_rend, t);
    if (rc) return rc;
    t->frames = nf;
    DT(d, hipEventRecord(t->a, st), "event");
    rc = rt_render_frames(d->ctx, lights, n_lights, cams, nf, &sh, dst, stride, fmt, st, d_done, target,
                          groups ? groups->data() : nullptr, groups ? (int)groups->size() - 1 : 0);
    if (rc) return rc;
    DT(d, hipEventRecord(t->b, st), "event");
    return CG_OK;
}

}  // namespace

extern "C" int cg_dist_unique_id(cg_dist_id *id)
{
    if (!id) return CG_E_INVALID;
    static_assert(sizeof(cg_dist_id) == sizeof(ncclUniqueId), "cg_dist_id must hold an ncclUniqueId");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return CG_E_HIP;
    std::memcpy(id->bytes, u.internal, sizeof(u.internal));
    return CG_OK;
}

extern "C" int cg_dist_create_timed(cg_ctx *ctx, int nranks, int rank, const cg_dist_id *id, int timeout_ms,
                                    cg_dist **out)
{
    if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks || timeout_ms < 0) return CG_E_INVALID;
    *out = nullptr;
    cg_dist *d = new cg_dist;
    d->ctx = ctx;
    d->nranks = nranks;
    d->rank = rank;
    d->timeout_ms = timeout_ms ? timeout_ms : default_timeout_ms();
    ncclUniqueId u;
    std::memcpy(u.internal, id->bytes, sizeof(u.internal));
    if (hipSetDevice(ctx_device(ctx)) != hipSuccess) {
        delete d;
        return fail(nullptr, CG_E_HIP, "hipSetDevice");
    }
    // non-blocking: the init (every rank meeting at the id's bootstrap root)
    // runs in the background and is polled against the deadline
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    const ncclResult_t r = ncclCommInitRankConfig(&d->comm, nranks, u, rank, &cfg);
    const int rc = nccl_settle(d, r, "ncclCommInitRankConfig");
    if (rc) {
        delete d;   // nccl_settle aborted the communicator
        return rc;
    }
    *out = d;
    return CG_OK;
}

extern "C" int cg_dist_create(cg_ctx *ctx, int nranks, int rank, const cg_dist_id *id, cg_dist **out)
{
    return cg_dist_create_timed(ctx, nranks, rank, id, 0, out);
}

extern "C" int cg_dist_set_timeout(cg_dist *d, int timeout_ms)
{
    if (!d || timeout_ms <= 0) return CG_E_INVALID;
    d->timeout_ms = timeout_ms;
    return CG_OK;
}

extern "C" int cg_dist_wait(cg_dist *d, void *stream)
{
    if (!d) return CG_E_INVALID;
    if (d->aborted) return fail(d, CG_E_HIP, "communicator was aborted by an earlier error");
    return drain(d, (hipStream_t)stream, "cg_dist_wait");
}

extern "C" int cg_dist_create_local(cg_ctx *const *ctxs, int nranks, cg_dist **outs)
{
    if (!ctxs || !outs || nranks < 1) return CG_E_INVALID;
    for (int r = 0; r < nranks; ++r)
        if (!ctxs[r]) return CG_E_INVALID;
    LocalGroup *g = new LocalGroup;
    for (int r = 0; r < nranks; ++r) {
        cg_dist *d = new cg_dist;
        d->ctx = ctxs[r];
        d->nranks = nranks;
        d->rank = r;
        d->group = g;
        g->members.push_back(d);
        outs[r] = d;
    }
    return CG_OK;
}

extern "C" void cg_dist_destroy(cg_dist *d)
{
    if (!d) return;
    (void)hipSetDevice(ctx_device(d->ctx));
    // bounded: a peer that never answers ends in ncclCommAbort, not a hang
    if (!d->aborted && drain(d, nullptr, "cg_dist_destroy") == CG_OK && d->comm) {
        if (nccl_settle(d, ncclCommFinalize(d->comm), "ncclCommFinalize") == CG_OK) {
            (void)ncclCommDestroy(d->comm);
            d->comm = nullptr;
        }
    }
    if (d->comm) abort_comm(d);
    for (hipEvent_t e : d->ev_wait)
        if (e) (void)hipEventDestroy(e);
    for (int k = 0; k < 2; ++k)
        for (hipEvent_t e : {d->ev_rend[k], d->ev_sent[k], d->ev_recv[k], d->ev_asm[k]})
            if (e) (void)hipEventDestroy(e);
    if (d->ev_done) (void)hipEventDestroy(d->ev_done);
    if (d->ev_start) (void)hipEventDestroy(d->ev_start);
    for (int k = 0; k < 2; ++k) {
        if (d->ev_call[k]) (void)hipEventDestroy(d->ev_call[k]);
        if (d->ev_zero[k]) (void)hipEventDestroy(d->ev_zero[k]);
        if (d->done[k] && !d->leaked) (void)hipFree(d->done[k]);
    }
    for (hipEvent_t e : d->ev_chunk) (void)hipEventDestroy(e);
    for (auto *pool : {&d->t_rend, &d->t_asm})
        for (TimedPair &t : *pool) {
            (void)hipEventDestroy(t.a);
            (void)hipEventDestroy(t.b);
        }
    if (d->leaked) {
        // an abort that did not finish (abort_comm): keep every device buffer and
        // the transfer stream alive for the process's lifetime
        for (Mem *m : {&d->sbuf[0], &d->sbuf[1], &d->rbuf[0], &d->rbuf[1], &d->sall, &d->stats}) m->p = nullptr;
        d->xs = nullptr;
    }
    if (d->xs) (void)hipStreamDestroy(d->xs);
    if (d->group) {   // the last member frees the group
        auto &m = d->group->members;
        m.erase(std::remove(m.begin(), m.end(), d), m.end());
        if (m.empty()) delete d->group;
    }
    delete d;
}

extern "C" int cg_dist_set_bands(cg_dist *d, int height, const int *row0, const int *rows)
{
    if (!d || height <= 0 || !row0 || !rows) return CG_E_INVALID;
    int next = 0;
    for (int r = 0; r < d->nranks; ++r) {
        if (row0[r] != next || rows[r] < 0) return CG_E_INVALID;
        next += rows[r];
    }
    if (next != height) return CG_E_INVALID;
    d->height = height;
    d->row0.assign(row0, row0 + d->nranks);
    d->rows.assign(rows, rows + d->nranks);
    return CG_OK;
}

extern "C" int cg_dist_get_bands(const cg_dist *d, int *row0, int *rows)
{
    if (!d || !row0 || !rows) return CG_E_INVALID;
    if (d->row0.empty()) return CG_E_INVALID;
    std::copy(d->row0.begin(), d->row0.end(), row0);
    std::copy(d->rows.begin(), d->rows.end(), rows);
    return d->height;
}

extern "C" int cg_dist_set_pipeline(cg_dist *d, int mode)
{
    if (!d || (mode != CG_DIST_SIGNALLED && mode != CG_DIST_CHUNKED)) return CG_E_INVALID;
    int rc = ensure_events(d);
    if (rc) return rc;
    if (mode == CG_DIST_CHUNKED) d->signals = false;
    else if (!d->signals) return fail(d, CG_E_INVALID, "stream waits on memory are not supported on this device");
    return CG_OK;
}

extern "C" int cg_dist_set_chunk(cg_dist *d, int frames)
{
    if (!d || frames < 1) return CG_E_INVALID;
    d->chunk = frames;
    return CG_OK;
}

extern "C" int cg_dist_last_times(cg_dist *d, double *render_ms_per_frame, double *assemble_ms_per_frame)
{
    if (!d) return CG_E_INVALID;
    if (!d->group) {   // the timing events sit behind the transfers: bounded wait first
        const int rc = drain(d, nullptr, "cg_dist_last_times");
        if (rc) return rc;
    }
    if (render_ms_per_frame) *render_ms_per_frame = pool_ms_per_frame(d->t_rend, d->n_rend);
    if (assemble_ms_per_frame) *assemble_ms_per_frame = pool_ms_per_frame(d->t_asm, d->n_asm);
    return CG_OK;
}

extern "C" int cg_dist_band_partition(const double *row_cost, int height, int nranks, const double *overhead,
                                      int *row0, int *rows)
{
    if (!row_cost || height < 0 || nranks < 1 || !row0 || !rows) return CG_E_INVALID;
    band_partition(row_cost, height, nranks, overhead, row0, rows);
    return CG_OK;
}

// New bands from per-rank (render ms/frame, fixed ms/frame) pairs t[2 r], t[2 r + 1].
// The fixed term (rank 0's assembly) adds to rank 0's time only in the chunked
// pipeline, where the assembly runs on the render stream; the signalled
// pipeline assembles on the transfer stream beside rank 0's own render.
static void rebalance_bands(cg_dist *d, const double *t)
{
    const int n = d->nranks, H = d->height;
    std::vector<double> cost(H, 0.0), ovh(n);
    for (int r = 0; r < n; ++r) {
        for (int y = d->row0[r]; y < d->row0[r] + d->rows[r]; ++y) cost[y] = std::max(t[2 * r], 1e-12) / d->rows[r];
        ovh[r] = d->signals ? 0.0 : t[2 * r + 1];
    }
    std::vector<int> a(n), b(n);
    band_partition(cost.data(), H, n, ovh.data(), a.data(), b.data());
    d->row0 = a;
    d->rows = b;
}

extern "C" int cg_dist_rebalance(cg_dist *d)
{
    if (!d) return CG_E_INVALID;
    if (d->height <= 0 || d->nranks == 1) return CG_OK;
    const int n = d->nranks;
    if (d->group) {   // every member's last call is enqueued: gather directly
        if (d->rank != 0) return CG_OK;   // rank 0 rebalances the whole group
        std::vector<double> t(2 * n);
        for (cg_dist *m : d->group->members) {
            t[2 * m->rank] = pool_ms_per_frame(m->t_rend, m->n_rend);
            t[2 * m->rank + 1] = pool_ms_per_frame(m->t_asm, m->n_asm);
        }
        rebalance_bands(d, t.data());
        for (cg_dist *m : d->group->members) {
            m->height = d->height;
            m->row0 = d->row0;
            m->rows = d->rows;
        }
        return CG_OK;
    }
    int rc = ensure_events(d);
    if (rc) return rc;
    rc = drain(d, nullptr, "cg_dist_rebalance");   // the last call's timing events, bounded
    if (rc) return rc;
    const double mine[2] = {pool_ms_per_frame(d->t_rend, d->n_rend), pool_ms_per_frame(d->t_asm, d->n_asm)};
    DT(d, d->stats.ensure((size_t)(2 * n + 2) * sizeof(double) + (size_t)2 * n * sizeof(int)), "alloc stats");
    double *dt = (double *)d->stats.p;
    int *dband = (int *)(dt + 2 * n + 2);
    DT(d, hipMemcpyAsync(dt + 2 * n, mine, sizeof(mine), hipMemcpyHostToDevice, d->xs), "stats upload");
    DN(d, ncclAllGather(dt + 2 * n, dt, 2, ncclFloat64, d->comm, d->xs), "ncclAllGather");
    std::vector<double> t(2 * n);
    DT(d, hipMemcpyAsync(t.data(), dt, 2 * n * sizeof(double), hipMemcpyDeviceToHost, d->xs), "stats download");
    DT(d, hipEventRecord(d->ev_wait[1], d->xs), "event");
    rc = wait_events(d, &d->ev_wait[1], 1, "cg_dist_rebalance: ncclAllGather");
    if (rc) return rc;
    // rank 0 decides; every rank adopts its boundaries
    std::vector<int> band(2 * n);
    if (d->rank == 0) {
        rebalance_bands(d, t.data());
        for (int r = 0; r < n; ++r) {
            band[2 * r] = d->row0[r];
            band[2 * r + 1] = d->rows[r];
        }
        DT(d, hipMemcpyAsync(dband, band.data(), band.size() * sizeof(int), hipMemcpyHostToDevice, d->xs), "bands");
    }
    DN(d, ncclBroadcast(dband, dband, 2 * n, ncclInt32, 0, d->comm, d->xs), "ncclBroadcast");
    DT(d, hipMemcpyAsync(band.data(), dband, band.size() * sizeof(int), hipMemcpyDeviceToHost, d->xs), "bands");
    DT(d, hipEventRecord(d->ev_wait[1], d->xs), "event");
    rc = wait_events(d, &d->ev_wait[1], 1, "cg_dist_rebalance: ncclBroadcast");
    if (rc) return rc;
    for (int r = 0; r < n; ++r) {
        d->row0[r] = band[2 * r];
        d->rows[r] = band[2 * r + 1];
    }
    return CG_OK;
}

// The signalled pipeline's chunks of a call: up to C frames each, tapering
// at the end (half the frames left, at least one), so the transfer and the
// assembly left after the last frame renders cover one frame, not C (20
// frames, C = 4: 4 4 4 4 2 1 1).  Senders and rank 0 derive the same plan.
static std::vector<std::pair<int, int>> chunk_plan(int n_frames, int C)
{
    std::vector<std::pair<int, int>> plan;
    for (int f0 = 0; f0 < n_frames;) {
        const int left = n_frames - f0;
        const int nf = left > 2 * C ? C : std::max(1, std::min(C, left / 2));
        plan.emplace_back(f0, nf);
        f0 += nf;
    }
    return plan;
}

// One call, signalled: every rank renders its band for all the call's frames
// in one render call (one lattice launch per 32 frames: full-size launches
// even for a 1/8 band); ranks > 0 render into the call's send slot and their
// transfer stream sends each chunk as soon as its frames' tiles are all
// stored (hipStreamWaitValue32 on the per-frame counts), while later frames
// are still rendering; rank 0 receives and assembles chunk by chunk on its
// transfer stream, beside its own band's render.
static int render_signalled(cg_dist *d, const cg_light *lights, int n_lights, const cg_rt_camera *cams, int n_frames,
                            uint32_t *d_frames, size_t frame_stride, hipStream_t st, int c0, int cols)
{
    const int n = d->nranks, me = d->rank, W = cams[0].width, H = cams[0].height;
    const int pitch = cols ? cols : W;
    const size_t row_bytes = (size_t)pitch * 3;
    const int C = std::max(1, std::min(d->chunk, n_frames));
    const int r0 = d->row0[me], nr = d->rows[me];
    const int s = (int)(d->calls++ & 1u);
    d->cur = s;
    int rc;
    if (me > 0) {
        // the slot's previous reader: this rank's sends (RCCL) or rank 0's
        // copies (local transport) of the call two calls ago
        hipEvent_t prev = d->group ? d->group->members[0]->ev_call[s] : d->ev_call[s];
        if (prev) DT(d, hipStreamWaitEvent(st, prev, 0), "wait");
        const size_t bytes = (size_t)n_frames * nr * row_bytes;
        Mem &out = d->sbuf[s];   // the whole call's band (rank 0 pulls from it in the local transport)
        DT(d, out.ensure(std::max<size_t>(bytes, 1)), "alloc send buffer");
        if (d->done_cap[s] < (size_t)n_frames) {
            // bounded: st may wait on the slot's previous sends
            rc = drain(d, st, "grow signals");
            if (rc) return rc;
            if (d->done[s]) DT(d, hipFree(d->done[s]), "free signals");
            d->done[s] = nullptr;
            // uncached fine-grained device memory: the kernels' atomics land in
            // memory, where the command processor's waits poll them
            DT(d, hipExtMallocWithFlags((void **)&d->done[s], (size_t)n_frames * sizeof(uint32_t),
                                        hipDeviceMallocUncached), "alloc signals");
            d->done_cap[s] = n_frames;
        }
        d->target[s].assign(n_frames, 0u);
        DT(d, hipMemsetAsync(d->done[s], 0, (size_t)n_frames * sizeof(uint32_t), st), "zero signals");
        // The slot's counts still hold the totals of the call two calls ago,
        // and the targets repeat for the same frame size: every wait on them
        // (this rank's transfer stream, or rank 0's in the local transport)
        // is ordered after this memset, else it could pass on stale counts
        // and send a half-written band.
        DT(d, hipEventRecord(d->ev_zero[s], st), "event");
        if (!d->group) DT(d, hipStreamWaitEvent(d->xs, d->ev_zero[s], 0), "wait");
        if (nr > 0) {
            // the lattice dispatches the chunks' frames in turn (heavy tiles first
            // inside each), so chunk j's frames complete before chunk j + 1's
            std::vector<int> gs;
            for (const auto &ch : chunk_plan(n_frames, C)) gs.push_back(ch.first);
            gs.push_back(n_frames);
            rc = render_band(d, lights, n_lights, cams, n_frames, r0, nr, c0, cols, out.p, (size_t)nr * pitch,
                             CG_PIX_RGB24, st, d->done[s], d->target[s].data(), &gs);
            if (rc) return rc;
        } else {
            for (int f = 0; f < n_frames; ++f) d->target[s][f] = 0u;   // nothing to wait for
        }
        d->last_pitch = pitch;
        d->last_frames = n_frames;
        if (d->group) return CG_OK;   // rank 0 pulls the chunks
        for (const auto &ch : chunk_plan(n_frames, C)) {
            const int f0 = ch.first, nf = ch.second;
            for (int f = f0; f < f0 + nf; ++f)
                if (d->target[s][f])
                    DT(d, hipStreamWaitValue32(d->xs, d->done[s] + f, d->target[s][f], hipStreamWaitValueGte,
                                               0xffffffffu), "wait frame");
            const size_t cb = (size_t)nf * nr * row_bytes;
            if (cb) DN(d, ncclSend((uint8_t *)out.p + (size_t)f0 * nr * row_bytes, cb, ncclUint8, 0, d->comm, d->xs),
                       "ncclSend");
        }
        DT(d, hipEventRecord(d->ev_call[s], d->xs), "event");
        return CG_OK;
    }
    // rank 0: the assembly below writes the caller's frames on the transfer
    // stream, so it is ordered after whatever the caller queued on `st`
    // before this call (e.g. a copy-out of the previous call's frames).
    DT(d, hipEventRecord(d->ev_start, st), "event");
    // own band straight into the frames (ARGB), on the caller's stream
    if (nr > 0) {
        rc = render_band(d, lights, n_lights, cams, n_frames, r0, nr, 0, 0, d_frames + (size_t)r0 * W, frame_stride,
                         CG_PIX_ARGB8888, st);
        if (rc) return rc;
    }
    if (n > 1) {
        bool ordered = false;   // xs waited on ev_start
        size_t per_frame = 0;
        for (int p = 1; p < n; ++p) per_frame += (size_t)d->rows[p] * row_bytes;
        DT(d, d->rbuf[0].ensure(std::max<size_t>((size_t)n_frames * per_frame, 1)), "alloc receive buffer");
        uint8_t *rb = (uint8_t *)d->rbuf[0].p;
        std::vector<int> br0(n - 1), brows(n - 1);
        for (int p = 1; p < n; ++p) {
            br0[p - 1] = d->row0[p];
            brows[p - 1] = d->rows[p];
        }
        for (const auto &ch : chunk_plan(n_frames, C)) {
            const int f0 = ch.first, nf = ch.second;
            uint8_t *cb = rb + (size_t)f0 * per_frame;   // blocks of this chunk, peers in order
            size_t off = 0;
            if (d->group) {
                for (int p = 1; p < n; ++p) {
                    const cg_dist *m = d->group->members[p];
                    const size_t bytes = (size_t)nf * d->rows[p] * row_bytes;
                    if (m->last_frames != (size_t)n_frames || m->last_pitch != pitch || m->cur != s ||
                        m->calls != d->calls)
                        return fail(d, CG_E_INVALID, "local transport: ranks > 0 must render this call first");
                    // the peer's counts for this call are zeroed before we poll them
                    if (f0 == 0) DT(d, hipStreamWaitEvent(d->xs, m->ev_zero[s], 0), "wait");
                    for (int f = f0; f < f0 + nf; ++f)
                        if (m->target[s][f])
                            DT(d, hipStreamWaitValue32(d->xs, m->done[s] + f, m->target[s][f],
                                                       hipStreamWaitValueGte, 0xffffffffu), "wait frame");
                    if (bytes)
                        DT(d, hipMemcpyAsync(cb + off, (const uint8_t *)m->sbuf[s].p + (size_t)f0 * d->rows[p] * row_bytes,
                                             bytes, hipMemcpyDeviceToDevice, d->xs), "band copy");
                    off += bytes;
                }
            } else {
                std::vector<size_t> bytes(n, 0);
                for (int p = 1; p < n; ++p) {
                    bytes[p] = (size_t)nf * d->rows[p] * row_bytes;
                    off += bytes[p];
                }
                rc = recv_group(d, cb, bytes.data(), n);
                if (rc) return rc;
            }
            // assembly of the chunk on the transfer stream (rows disjoint from
            // the render's own band)
            TimedPair *t;
            rc = timed(d, d->t_asm, d->n_asm, t);
            if (rc) return rc;
            t->frames = nf;
            if (!ordered) {   // the receives may start earlier; the writes into d_frames may not
                DT(d, hipStreamWaitEvent(d->xs, d->ev_start, 0), "wait");
                ordered = true;
            }
            DT(d, hipEventRecord(t->a, d->xs), "event");
            rc = cg_rt_assemble_device(d->ctx, cb, CG_PIX_RGB24, br0.data(), brows.data(), n - 1, W, H, nf,
                                       d_frames + (size_t)f0 * frame_stride, frame_stride, cols ? c0 : 0, cols, d->xs);
            if (rc) return rc;
            DT(d, hipEventRecord(t->b, d->xs), "event");
        }
        // local transport: the peers' slot s is free once these copies ran
        DT(d, hipEventRecord(d->ev_call[s], d->xs), "event");
    }
    DT(d, hipEventRecord(d->ev_done, d->xs), "event");
    DT(d, hipStreamWaitEvent(st, d->ev_done, 0), "wait");
    return CG_OK;
}

extern "C" int cg_rt_render_frames_dist(cg_dist *d, const cg_light *lights, int n_lights, const cg_rt_camera *cams,
                                        int n_frames, uint32_t *d_frames, size_t frame_stride, void *stream)
{
    if (!d || n_frames < 0 || (n_frames && !cams)) return CG_E_INVALID;
    if (d->aborted) return fail(d, CG_E_HIP, "communicator was aborted by an earlier error");
    if (n_frames == 0) return CG_OK;
    const int W = cams[0].width, H = cams[0].height;
    if (W <= 0 || H <= 0) return CG_E_INVALID;
    for (int f = 1; f < n_frames; ++f)
        if (cams[f].width != W || cams[f].height != H) return CG_E_INVALID;
    if (d->rank == 0 && !d_frames) return CG_E_INVALID;
    if (frame_stride == 0) frame_stride = (size_t)W * H;
    if (frame_stride < (size_t)W * H) return CG_E_INVALID;
    int rc = ensure_events(d);
    if (rc) return rc;
    DT(d, hipSetDevice(ctx_device(d->ctx)), "hipSetDevice");
    if (d->height != H || (int)d->row0.size() != d->nranks) {
        d->height = H;
        equal_bands(H, d->nranks, d->row0, d->rows);
    }
    hipStream_t st = stream ? (hipStream_t)stream : ctx_stream(d->ctx);
    d->last_st = st;
    const int n = d->nranks, me = d->rank;
    int c0, cols;
    call_window(d, cams, n_frames, c0, cols);
    const int pitch = cols ? cols : W;
    const size_t row_bytes = (size_t)pitch * 3;
    const int C = std::max(1, std::min(d->chunk, n_frames));
    d->n_rend = d->n_asm = 0;
    const int r0 = d->row0[me], nr = d->rows[me];
    if (d->signals)
        return render_signalled(d, lights, n_lights, cams, n_frames, d_frames, frame_stride, st, c0, cols);
    if (d->group && me > 0) {
        // local transport: the whole call's band in one buffer, chunk events
        // for rank 0's copies (no slot reuse: rank 0's call comes later)
        const int chunks = (n_frames + C - 1) / C;
        DT(d, d->sall.ensure(std::max<size_t>(1, (size_t)n_frames * nr * row_bytes)), "alloc band");
        while ((int)d->ev_chunk.size() < chunks) {
            hipEvent_t e;
            DT(d, hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
            d->ev_chunk.push_back(e);
        }
        for (int j = 0; j < chunks; ++j) {
            const int f0 = j * C, nf = std::min(C, n_frames - f0);
            if (nr > 0) {
                rc = render_band(d, lights, n_lights, cams + f0, nf, r0, nr, c0, cols,
                                 (uint8_t *)d->sall.p + (size_t)f0 * nr * row_bytes, (size_t)nr * pitch, CG_PIX_RGB24,
                                 st);
                if (rc) return rc;
            }
            DT(d, hipEventRecord(d->ev_chunk[j], st), "event");
        }
        d->last_pitch = pitch;
        d->last_frames = n_frames;
        return CG_OK;
    }
    for (int f0 = 0, j = 0; f0 < n_frames; f0 += C, ++j) {
        const int nf = std::min(C, n_frames - f0), s = j & 1;
        if (me == 0) {
            // own band straight into the frames (ARGB)
            if (nr > 0) {
                rc = render_band(d, lights, n_lights, cams + f0, nf, r0, nr, 0, 0,
                                 d_frames + (size_t)f0 * frame_stride + (size_t)r0 * W, frame_stride, CG_PIX_ARGB8888,
                                 st);
                if (rc) return rc;
            }
            if (n == 1) continue;
            size_t total = 0;
            for (int p = 1; p < n; ++p) total += (size_t)nf * d->rows[p] * row_bytes;
            DT(d, d->rbuf[s].ensure(std::max<size_t>(total, 1)), "alloc receive buffer");
            // the slot was last read by the assembly of chunk j - 2
            DT(d, hipStreamWaitEvent(d->xs, d->ev_asm[s], 0), "wait");
            uint8_t *rb = (uint8_t *)d->rbuf[s].p;
            if (d->group) {
                size_t off = 0;
                for (int p = 1; p < n; ++p) {
                    const cg_dist *m = d->group->members[p];
                    const size_t bytes = (size_t)nf * d->rows[p] * row_bytes;
                    if (m->last_frames != (size_t)n_frames || m->last_pitch != pitch || (int)m->ev_chunk.size() <= j)
                        return fail(d, CG_E_INVALID, "local transport: ranks > 0 must render this call first");
                    DT(d, hipStreamWaitEvent(d->xs, m->ev_chunk[j], 0), "wait");
                    if (bytes)
                        DT(d, hipMemcpyAsync(rb + off, (const uint8_t *)m->sall.p + (size_t)f0 * d->rows[p] * row_bytes,
                                             bytes, hipMemcpyDeviceToDevice, d->xs), "band copy");
                    off += bytes;
                }
            } else {
                std::vector<size_t> bytes(n, 0);
                for (int p = 1; p < n; ++p) bytes[p] = (size_t)nf * d->rows[p] * row_bytes;
                rc = recv_group(d, rb, bytes.data(), n);
                if (rc) return rc;
            }
            DT(d, hipEventRecord(d->ev_recv[s], d->xs), "event");
            // assembly of the received bands on the render stream
            DT(d, hipStreamWaitEvent(st, d->ev_recv[s], 0), "wait");
            std::vector<int> br0(n - 1), brows(n - 1);
            for (int p = 1; p < n; ++p) {
                br0[p - 1] = d->row0[p];
                brows[p - 1] = d->rows[p];
            }
            TimedPair *t;
            rc = timed(d, d->t_asm, d->n_asm, t);
            if (rc) return rc;
            t->frames = nf;
            DT(d, hipEventRecord(t->a, st), "event");
            rc = cg_rt_assemble_device(d->ctx, rb, CG_PIX_RGB24, br0.data(), brows.data(), n - 1, W, H, nf,
                                       d_frames + (size_t)f0 * frame_stride, frame_stride, cols ? c0 : 0, cols, st);
            if (rc) return rc;
            DT(d, hipEventRecord(t->b, st), "event");
            DT(d, hipEventRecord(d->ev_asm[s], st), "event");
        } else {
            const size_t bytes = (size_t)nf * nr * row_bytes;
            DT(d, d->sbuf[s].ensure(std::max<size_t>(bytes, 1)), "alloc send buffer");
            // the slot was last read by the send of chunk j - 2
            DT(d, hipStreamWaitEvent(st, d->ev_sent[s], 0), "wait");
            if (nr > 0) {
                rc = render_band(d, lights, n_lights, cams + f0, nf, r0, nr, c0, cols, d->sbuf[s].p, (size_t)nr * pitch,
                                 CG_PIX_RGB24, st);
                if (rc) return rc;
            }
            DT(d, hipEventRecord(d->ev_rend[s], st), "event");
            DT(d, hipStreamWaitEvent(d->xs, d->ev_rend[s], 0), "wait");
            if (bytes) DN(d, ncclSend(d->sbuf[s].p, bytes, ncclUint8, 0, d->comm, d->xs), "ncclSend");
            DT(d, hipEventRecord(d->ev_sent[s], d->xs), "event");
        }
    }
    // the caller's stream covers the transfers too
    DT(d, hipEventRecord(d->ev_done, d->xs), "event");
    DT(d, hipStreamWaitEvent(st, d->ev_done, 0), "wait");
    return CG_OK;
}
