// cg_shim.hip -- the extern "C" boundary (include/cg_render.h): context,
// device-resident scene, launches, error mapping.  Nothing here throws
// across the ABI; HIP failures become CG_E_HIP with the HIP message kept in
// the context for cg_last_error().
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "cg_internal.h"
#include "cg_rast_dev.h"

namespace cg {
hipError_t launch_rt_prepare(const cg_tri *, const RtGeo *, int, const RtFrameCams &, int, RtTri *, hipStream_t,
                             const RtFrame *, const RtSphere *, unsigned long long *, unsigned long long *,
                             LatFlatten * = nullptr, LatPublish * = nullptr);
hipError_t launch_rt_scene(const cg_tri *, int, RtGeo *, RtShade *, hipStream_t);
hipError_t rt_render_brute(const RtFrame &, const cg_tri *, int, const RtSphere *, int, int, uint32_t *, hipStream_t);
size_t rt_sup_units(const RtFrame &);
hipError_t launch_rt_lattice_frames(const RtFrame &, const RtTri *, const RtShade *, const RtSphere *,
                                    const unsigned long long *, const unsigned long long *, const RtFrameCams &,
                                    int, size_t, uint32_t *, hipStream_t, uint32_t *, const LatOrder *,
                                    const LatReady * = nullptr);
hipError_t launch_rt_lattice_units(const RtFrame &, const RtTri *, const RtShade *, const RtSphere *,
                                   const unsigned long long *, const RtFrameCams &, int, unsigned long long *,
                                   hipStream_t);
size_t rt_lattice_unit_bytes(const RtFrame &, int);
hipError_t launch_rt_pixels(const RtFrame &, const RtTri *, const RtShade *, const RtSphere *,
                            const unsigned long long *, unsigned long long *, uint32_t *, hipStream_t);
bool rt_use_lattice(const RtFrame &);
int rt_lattice_kind(const RtFrame &);
void rt_scene_box(const cg_tri *tris, int n_tris, const cg_sphere *spheres, int n_spheres, double lo[3],
                  double hi[3]);
void rt_box_columns(const double lo[3], const double hi[3], const cg_rt_camera *cam, int *col0, int *col1);
size_t rt_lattice_tiles(const RtFrame &);
hipError_t launch_rt_big(const RtFrame &, RtTri *, const RtShade *, const RtSphere *, const RtGrid &, void *,
                         uint32_t *, hipStream_t, const RtGeo *, const cg_tri *, int, const BigCaps &,
                         unsigned long long *, int);
bool rt_big_shadow_lists(const RtFrame &);
int rt_big_mode(const RtFrame &);
bool rt_grid_build(const cg_tri *, int, RtGrid &, std::vector<int> &, std::vector<int> &, size_t);
size_t rt_big_scratch_bytes(const RtFrame &, const BigCaps &);
hipError_t launch_rt_unstripe(const uint32_t *, int, int, int, int, int, int, uint32_t *, hipStream_t);
hipError_t launch_rt_pack_rgb24(const uint32_t *, int, int, int, int, uint8_t *, hipStream_t);
hipError_t launch_rt_assemble(const uint8_t *, const RtBlocks &, int, uint32_t *, size_t, hipStream_t);
hipError_t launch_rt_probe_closest(const RtFrame &, const cg_tri *, const RtSphere *,
                                   const cg_vec4 *, const cg_vec4 *, int, cg_isect *, int *,
                                   hipStream_t);
hipError_t launch_rt_probe_direct_light(const RtFrame &, const RtTri *, const RtShade *,
                                        const RtSphere *, const cg_isect *, int, cg_vec3 *,
                                        hipStream_t);
int rast_render_device(cg_ctx *ctx, const cg_rtri *d_tris, int n, const cg_rast_params *p,
                       cg_vec4 light, uint32_t *d_argb, float *d_depth, int32_t *d_shadow,
                       hipStream_t st, cg_stats *stats, int tex_mask);
int rast_draw_device(cg_ctx *c, const cg_rtri *d_room, int n_room, const cg_rtri *d_boxes, int n_boxes,
                     const cg_rast_params *p, uint32_t *d_argb, float *d_depth, int32_t *d_shadow,
                     hipStream_t st, cg_stats *stats, int **n_out, int tex_mask);
void rast_release(cg_ctx *ctx);
}  // namespace cg

using namespace cg;

// Grow-only device buffer.
struct DevBuf {
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
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

// Host threads that store the certified-black columns of frames delivered
// into host memory (cg_rt_render / cg_rt_render_frames): a frame's 3.2 MB of
// black columns (C2) take one thread longer than the PCIe copy of its
// window, so the rows are shared by the workers and the caller.  run() hands
// out a job; wait() helps and returns when every row is stored.
class HostFill {
  public:
    struct Frame {
        uint32_t *dst;   // W x rows pixels, row pitch W
    };
    explicit HostFill(int n)
    {
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    ~HostFill()
    {
        {
            std::lock_guard<std::mutex> g(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    void run(std::vector<Frame> frames, int W, int rows, int c0, int c1)
    {
        wait();
        {
            std::lock_guard<std::mutex> g(mu_);
            fr_ = std::move(frames);
            W_ = W;
            rows_ = rows;
            c0_ = c0;
            c1_ = c1;
            total_ = (int)fr_.size() * rows;
            next_.store(0);
            busy_ = (int)th_.size();
            ++gen_;
        }
        cv_.notify_all();
    }
    void wait()
    {
        work();
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [this] { return busy_ == 0; });
    }

  private:
    static constexpr int kRowsPerGrab = 32;
    void work()
    {
        for (;;) {
            const int r0 = next_.fetch_add(kRowsPerGrab);
            if (r0 >= total_) return;
            const int r1 = std::min(total_, r0 + kRowsPerGrab);
            for (int r = r0; r < r1; ++r) {
                uint32_t *row = fr_[r / rows_].dst + (size_t)(r % rows_) * W_;
                std::fill(row, row + c0_, 0x80000000u);   // PutPixelSDL(0, 0, 0)
                std::fill(row + c1_, row + W_, 0x80000000u);
            }
        }
    }
    void loop()
    {
        unsigned seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
            }
            work();
            std::lock_guard<std::mutex> g(mu_);
            if (--busy_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    bool quit_ = false;
    unsigned gen_ = 0;
    int busy_ = 0;
    std::vector<Frame> fr_;
    int W_ = 0, rows_ = 1, c0_ = 0, c1_ = 0, total_ = 0;
    std::atomic<int> next_{0};
};

struct cg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string err;
    // RT scene
    int n_tris = -1, n_sph = 0;
    float nbound = 0.f;   // largest |normal component| of the scene (shadow certificate)
    DevBuf tris, geo, tc, shade, sph, frame, probe_a, probe_b, probe_c, probe_d, lights, big, gstart, gtris;
    DevBuf latmask;                     // lattice tiles' certificates (two masks per tile)
    DevBuf supmask;                     // their super-tiles' certificates (two-level path)
    DevBuf umask;                       // light sets: the tiles' per-unit shadow masks
    // Batched lattice launches pipeline their certificate kernels on `aux`:
    // call j+1's certificates run beside call j's lattice kernel, each call
    // with its own slot of buffers (rt_enqueue_lattice_batch).
    hipStream_t aux = nullptr;
    hipEvent_t ev_cert[2] = {nullptr, nullptr}, ev_lat[2] = {nullptr, nullptr};
    int slot = 0;
    DevBuf ptc[2], plat[2], psup[2], pumask[2];
    // measured lattice order (LatOrder, cg_internal.h): per slot, the recording
    // of its last lattice launch (class per tile) and the order sorted for it
    DevBuf lcost[2], lflat[2];
    int umask_frames = 0;                            // light sets: frames the unit-mask slots are sized for
    DevBuf pflag[2];                  // published-certificate words per slot (LatPublish / LatReady)
    uint32_t cert_gen = 0u;           // generation of the latest published call
    unsigned long long lrec_key[2] = {0ull, 0ull};   // geometry key of the slot's recording (0: none)
    unsigned rt_scene_gen = 0;                       // cg_rt_set_scene count (part of the key)
    // cg_rt_render_frames (host output): chunks render into two device slots
    // and download on `xfer` while the next chunk renders
    hipStream_t xfer = nullptr;
    hipEvent_t ev_rdone[2] = {nullptr, nullptr}, ev_cdone[2] = {nullptr, nullptr};
    DevBuf hslot[2];
    std::unique_ptr<HostFill> hfill;    // their black columns (created on first use)
    RtGrid grid{};                      // large scenes only (n_tris > 64)
    int pend_cap = 0;                   // cg_rt_set_pending_cap (0 = default)
    // large-scene pools (cg_rt_big.hip): capacities in entries, sized on the
    // scene's first frame, then grown from the demand later frames report
    BigCaps big_caps{};
    bool big_sized = false;
    long long big_key = -1;                     // frame shape / path the pools were sized for
    bool big_fixed = false;                     // cg_rt_set_pool_caps: capacities pinned (test hook)
    unsigned long long *big_demand = nullptr;   // pinned [4]: the latest frame's demand
    hipEvent_t big_ev = nullptr;
    bool big_ev_live = false;
    unsigned long long big_last[4] = {};
    long long big_overflows = 0;
    // Large scenes, several frames in flight (rt_render_frames): slots 1 ..
    // kBigSlots - 1 with their own buffers, stream and demand read-back; slot 0
    // is tc / shade / big / frame / big_demand / big_ev above.  A frame's list
    // building and walks are latency-bound phases; independent frames fill
    // each other's gaps.
    static constexpr int kBigSlots = 4;
    struct ExtraSlot {
        DevBuf tc, big, frame;
        unsigned long long *demand = nullptr;
        hipEvent_t ev = nullptr, done = nullptr;
        bool ev_live = false;
        hipStream_t st = nullptr;
    } xs[kBigSlots - 1];
    hipEvent_t bev_start = nullptr;
    // the scene's box (rt_scene_box, once per cg_rt_set_scene): cg_dist's column
    // window of any camera from it in O(1) per frame -- no per-camera pass over
    // the scene (1M triangles: ~6 ms on the host) and no per-camera cache
    double box_lo[3] = {1e300, 1e300, 1e300}, box_hi[3] = {-1e300, -1e300, -1e300};
    std::vector<RtLight> lights_host;   // what `lights` holds (re-uploaded only on change)
    // RAST scratch (owned by cg_rast.hip)
    DevBuf rtris, rhdr, rspan, rpix, rargb, rdepth, rshadow, rcount, rrecs, rgeo, rroom, rboxes;
    DevBuf rpc, rtl, rrnd, rjt;          // colour modes 1-2 (cg_rast_colour.hip)
    DevBuf sstars, sframe;               // starfield (cg_starfield.hip)
    DevBuf iscratch;                     // JPEG decode (cg_image.hip)
    int n_room = -1, n_boxes = 0;
    int scene_tex = 0;                   // bit k: the uploaded room/boxes carry texture k
    // texture modes 1-3 (cg_rast_set_textures): device copies of the maps
    DevBuf tmarble, tnoise, twoven, twoven_ao, twoven_op, twoven_nrm, tgrill, tgrill_op, tgrill_nrm, rtexel;
    int tex_loaded = 0;                  // bit k: texture k renderable
    cg_ctx *tex_owner = nullptr;         // a lane reads its parent's maps
    // cg_rast_draw_frames_device: frames overlap on `lanes` (child contexts,
    // each with its own stream and scratch; scene copied device to device)
    static constexpr int kRastLanes = 8;
    cg_ctx *lanes[kRastLanes] = {};
    hipEvent_t lane_ev[kRastLanes] = {};
    hipEvent_t start_ev = nullptr;
    unsigned scene_gen = 0, lane_gen[kRastLanes] = {};
};

namespace cg {
// exposed to cg_dist.hip
int ctx_device(const cg_ctx *c) { return c->device; }
hipStream_t ctx_stream(const cg_ctx *c) { return c->stream; }
void ctx_set_error(cg_ctx *c, const std::string &e) { c->err = e; }
// cg_rt_frame_columns over the context's scene (the full width without one)
void ctx_rt_columns(const cg_ctx *c, const cg_rt_camera *cam, int *c0, int *c1)
{
    *c0 = 0;
    *c1 = cam->width;
    if (c->n_tris >= 0 && cam->width > 0) rt_box_columns(c->box_lo, c->box_hi, cam, c0, c1);
}
// exposed to cg_rast.hip
void *ctx_buf(cg_ctx *c, int which, size_t bytes, hipError_t *e)
{
    DevBuf *b = nullptr;
    switch (which) {
    case 0: b = &c->rtris; break;
    case 1: b = &c->rhdr; break;
    case 2: b = &c->rspan; break;
    case 3: b = &c->rpix; break;
    case 4: b = &c->rargb; break;
    case 5: b = &c->rdepth; break;
    case 6: b = &c->rshadow; break;
    case 7: b = &c->rcount; break;
    case 8: b = &c->rrecs; break;
    case 9: b = &c->rgeo; break;
    case 10: b = &c->rpc; break;
    case 11: b = &c->rtl; break;
    case 12: b = &c->rrnd; break;
    case 13: b = &c->rjt; break;
    case 14: b = &c->sstars; break;
    case 15: b = &c->sframe; break;
    case 16: b = &c->rtexel; break;
    case 17: b = &c->iscratch; break;
    default: *e = hipErrorInvalidValue; return nullptr;
    }
    *e = b->ensure(bytes);
    return *e == hipSuccess ? b->p : nullptr;
}
hipStream_t ctx_stream(cg_ctx *c) { return c->stream; }
int ctx_device(cg_ctx *c) { return c->device; }
int ctx_invalid(cg_ctx *c, const char *what)
{
    c->err = what;
    return CG_E_INVALID;
}
int ctx_fail(cg_ctx *c, hipError_t e, const char *what)
{
    c->err = std::string(what) + ": " + hipGetErrorString(e);
    return CG_E_HIP;
}
void ctx_events(cg_ctx *c, hipEvent_t *a, hipEvent_t *b)
{
    *a = c->ev0;
    *b = c->ev1;
}
void rast_release(cg_ctx *c)
{
    c->rtris.release(); c->rhdr.release(); c->rspan.release(); c->rpix.release();
    c->rargb.release(); c->rdepth.release(); c->rshadow.release(); c->rcount.release();
    c->rrecs.release(); c->rgeo.release(); c->rroom.release(); c->rboxes.release();
    c->rpc.release(); c->rtl.release(); c->rrnd.release(); c->rjt.release();
    c->sstars.release(); c->sframe.release();
    c->tmarble.release(); c->tnoise.release(); c->twoven.release(); c->twoven_ao.release();
    c->twoven_op.release(); c->twoven_nrm.release(); c->tgrill.release(); c->tgrill_op.release();
    c->tgrill_nrm.release(); c->rtexel.release();
}
// the device texture maps and which textures are renderable (bit k: texture k)
int rast_tex_maps(cg_ctx *c, RastTexMaps *m)
{
    if (c->tex_owner) c = c->tex_owner;
    m->marble = (const uint8_t *)c->tmarble.p;
    m->marble_noise = (const float *)c->tnoise.p;
    m->woven = (const uint8_t *)c->twoven.p;
    m->woven_ao = (const uint8_t *)c->twoven_ao.p;
    m->woven_op = (const uint8_t *)c->twoven_op.p;
    m->woven_nrm = (const uint8_t *)c->twoven_nrm.p;
    m->grill = (const uint8_t *)c->tgrill.p;
    m->grill_op = (const uint8_t *)c->tgrill_op.p;
    m->grill_nrm = (const uint8_t *)c->tgrill_nrm.p;
    return c->tex_loaded;
}
}  // namespace cg

#define CG_TRY(ctx, call, what)                       \
    do {                                              \
        hipError_t e_ = (call);                       \
        if (e_ != hipSuccess) return ctx_fail((ctx), e_, (what)); \
    } while (0)

extern "C" int cg_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" int cg_create(int device, cg_ctx **out)
{
    if (!out) return CG_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return CG_E_NODEVICE;
    if (device < 0 || device >= n) return CG_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return CG_E_NODEVICE;
    cg_ctx *c = new (std::nothrow) cg_ctx;
    if (!c) return CG_E_INVALID;
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        delete c;
        return CG_E_HIP;
    }
    *out = c;
    return CG_OK;
}

extern "C" void cg_destroy(cg_ctx *c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    DevBuf *bufs[] = {&c->tris, &c->geo, &c->tc, &c->shade, &c->sph, &c->frame,
                      &c->probe_a, &c->probe_b, &c->probe_c, &c->probe_d, &c->lights, &c->big,
                      &c->gstart, &c->gtris};
    if (c->big_ev) {
        (void)hipEventSynchronize(c->big_ev);
        (void)hipEventDestroy(c->big_ev);
    }
    for (DevBuf *b : bufs) b->release();
    if (c->big_demand) (void)hipHostFree(c->big_demand);
    for (auto &x : c->xs) {
        if (x.st) (void)hipStreamSynchronize(x.st);
        if (x.ev) {
            (void)hipEventSynchronize(x.ev);
            (void)hipEventDestroy(x.ev);
        }
        if (x.done) (void)hipEventDestroy(x.done);
        if (x.demand) (void)hipHostFree(x.demand);
        x.tc.release(); x.big.release(); x.frame.release();
        if (x.st) (void)hipStreamDestroy(x.st);
    }
    if (c->bev_start) (void)hipEventDestroy(c->bev_start);
    if (c->aux) (void)hipStreamSynchronize(c->aux);
    for (int k = 0; k < cg_ctx::kRastLanes; ++k) {
        if (c->lanes[k]) cg_destroy(c->lanes[k]);
        if (c->lane_ev[k]) (void)hipEventDestroy(c->lane_ev[k]);
    }
    if (c->start_ev) (void)hipEventDestroy(c->start_ev);
    for (int k = 0; k < 2; ++k) {
        c->ptc[k].release(); c->plat[k].release(); c->pflag[k].release(); c->psup[k].release();
        c->pumask[k].release();
        if (c->ev_cert[k]) (void)hipEventDestroy(c->ev_cert[k]);
        if (c->ev_lat[k]) (void)hipEventDestroy(c->ev_lat[k]);
    }
    if (c->aux) (void)hipStreamDestroy(c->aux);
    if (c->xfer) (void)hipStreamSynchronize(c->xfer);
    for (int k = 0; k < 2; ++k) {
        c->hslot[k].release();
        if (c->ev_rdone[k]) (void)hipEventDestroy(c->ev_rdone[k]);
        if (c->ev_cdone[k]) (void)hipEventDestroy(c->ev_cdone[k]);
    }
    if (c->xfer) (void)hipStreamDestroy(c->xfer);
    rast_release(c);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

extern "C" const char *cg_last_error(const cg_ctx *c) { return c ? c->err.c_str() : "no context"; }

// ---------------------------------------------------------------------------
// RT

extern "C" int cg_rt_set_scene(cg_ctx *c, const cg_tri *tris, int n_tris, const cg_sphere *spheres,
                               int n_spheres)
{
    if (!c || n_tris < 0 || n_spheres < 0 || (n_tris && !tris) || (n_spheres && !spheres))
        return CG_E_INVALID;
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    // frames still in flight on the caller's, auxiliary or slot streams read the
    // scene buffers rewritten below (triangles, RtGeo, RtShade): let them finish
    CG_TRY(c, hipDeviceSynchronize(), "scene change");
    ++c->rt_scene_gen;
    size_t nt = n_tris > 0 ? (size_t)n_tris : 1;
    CG_TRY(c, c->tris.ensure(nt * sizeof(cg_tri)), "alloc tris");
    CG_TRY(c, c->tc.ensure(nt * sizeof(RtTri)), "alloc tri constants");
    CG_TRY(c, c->shade.ensure(nt * sizeof(RtShade)), "alloc tri shading");
    CG_TRY(c, c->geo.ensure(nt * sizeof(RtGeo)), "alloc tri geometry");
    CG_TRY(c, c->sph.ensure((size_t)(n_spheres > 0 ? n_spheres : 1) * sizeof(RtSphere)), "alloc spheres");
    if (n_tris) {
        CG_TRY(c, hipMemcpyAsync(c->tris.p, tris, (size_t)n_tris * sizeof(cg_tri),
                                 hipMemcpyHostToDevice, c->stream), "upload tris");
        // the camera-independent constants (RtGeo) and shading attributes
        // (RtShade), once per scene: every frame, slot and path reads them
        CG_TRY(c, launch_rt_scene((const cg_tri *)c->tris.p, n_tris, (RtGeo *)c->geo.p, (RtShade *)c->shade.p,
                                  c->stream), "rt_scene launch");
    }
    std::vector<RtSphere> S((size_t)n_spheres);
    for (int i = 0; i < n_spheres; ++i) {
        S[i] = RtSphere{spheres[i].centre.x, spheres[i].centre.y, spheres[i].centre.z,
                        spheres[i].radiusSquared, spheres[i].color.x, spheres[i].color.y,
                        spheres[i].color.z, 0.f};
    }
    if (n_spheres)
        CG_TRY(c, hipMemcpyAsync(c->sph.p, S.data(), S.size() * sizeof(RtSphere),
                                 hipMemcpyHostToDevice, c->stream), "upload spheres");
    rt_scene_box(tris, n_tris, spheres, n_spheres, c->box_lo, c->box_hi);
    c->grid = RtGrid{};
    c->big_sized = false;   // the next large-scene frame sizes the pools
    if (n_tris > 64) {   // large scene: grid for the shadow-ray blocker search
        std::vector<int> gs, gt;
        RtGrid g{};
        if (rt_grid_build(tris, n_tris, g, gs, gt, (size_t)64 << 20)) {
            CG_TRY(c, c->gstart.ensure(gs.size() * 4), "alloc grid");
            CG_TRY(c, c->gtris.ensure(std::max<size_t>(gt.size(), 1) * 4), "alloc grid");
            CG_TRY(c, hipMemcpy(c->gstart.p, gs.data(), gs.size() * 4, hipMemcpyHostToDevice), "upload grid");
            if (!gt.empty())
                CG_TRY(c, hipMemcpy(c->gtris.p, gt.data(), gt.size() * 4, hipMemcpyHostToDevice), "upload grid");
            g.start = (const int *)c->gstart.p;
            g.tris = (const int *)c->gtris.p;
        }
        // hit positions lie on a triangle or a sphere: the box of both
        for (int k = 0; k < 3; ++k) {
            g.blo[k] = FLT_MAX;
            g.bhi[k] = -FLT_MAX;
        }
        auto grow = [&](int k, float lo, float hi) {
            g.blo[k] = std::min(g.blo[k], lo);
            g.bhi[k] = std::max(g.bhi[k], hi);
        };
        for (int i = 0; i < n_tris; ++i) {
            const cg_vec4 *v[3] = {&tris[i].v0, &tris[i].v1, &tris[i].v2};
            for (const cg_vec4 *p : v) {
                grow(0, p->x, p->x);
                grow(1, p->y, p->y);
                grow(2, p->z, p->z);
            }
        }
        for (int i = 0; i < n_spheres; ++i) {   // radius from radiusSquared, rounded up
            const float r = (float)(std::sqrt((double)spheres[i].radiusSquared) * (1.0 + 1e-6));
            grow(0, spheres[i].centre.x - r, spheres[i].centre.x + r);
            grow(1, spheres[i].centre.y - r, spheres[i].centre.y + r);
            grow(2, spheres[i].centre.z - r, spheres[i].centre.z + r);
        }
        for (int k = 0; k < 3; ++k) {   // float hit positions stray by rounding: widen
            g.blo[k] -= 1e-4f + 1e-5f * std::fabs(g.blo[k]);
            g.bhi[k] += 1e-4f + 1e-5f * std::fabs(g.bhi[k]);
        }
        c->grid = g;
    }
    CG_TRY(c, hipStreamSynchronize(c->stream), "scene upload");
    // Hit normals: the triangles' own (skeleton.cpp:378) and normalize(pos -
    // centre) for spheres (:385), whose components are <= 1 up to rounding.
    float nb = n_spheres > 0 ? 1.00000095367431640625f : 0.f;   // 1 + 2^-20
    for (int i = 0; i < n_tris; ++i) {
        const float q[3] = {tris[i].normal.x, tris[i].normal.y, tris[i].normal.z};
        for (float x : q) nb = std::isfinite(x) ? std::max(nb, std::fabs(x)) : INFINITY;
    }
    c->nbound = nb;
    c->n_tris = n_tris;
    c->n_sph = n_spheres;
    return CG_OK;
}

// Lights to the device buffer (ordered on `st`; skipped when unchanged) and
// the light-set summary the shadow certificate uses.
static int set_lights(cg_ctx *c, const cg_light *lights, int n, hipStream_t st, RtFrame &F)
{
    std::vector<RtLight> L((size_t)n);
    for (int l = 0; l < n; ++l)
        L[l] = RtLight{lights[l].position.x, lights[l].position.y, lights[l].position.z, lights[l].position.w,
                       lights[l].colour.x,   lights[l].colour.y,   lights[l].colour.z,   0.f};
    F.n_lights = n;
    for (int k = 0; k < 3; ++k) F.lmin[k] = F.lmax[k] = F.lc[k] = 0.f;
    F.lrho = 0.0;
    if (n > 0) {
        for (int k = 0; k < 3; ++k) F.lmin[k] = F.lmax[k] = (&L[0].x)[k];
        for (const RtLight &q : L)
            for (int k = 0; k < 3; ++k) {
                F.lmin[k] = std::min(F.lmin[k], (&q.x)[k]);
                F.lmax[k] = std::max(F.lmax[k], (&q.x)[k]);
            }
        for (int k = 0; k < 3; ++k) F.lc[k] = 0.5f * F.lmin[k] + 0.5f * F.lmax[k];
        double rho = 0.0;
        for (const RtLight &q : L) {
            double dx = (double)q.x - F.lc[0], dy = (double)q.y - F.lc[1], dz = (double)q.z - F.lc[2];
            rho = std::max(rho, std::sqrt(dx * dx + dy * dy + dz * dz));
        }
        F.lrho = rho > 0.0 ? rho * (1.0 + 1e-9) + 1e-12 : 0.0;
    }
    const bool same = L.size() == c->lights_host.size() &&
                      (L.empty() || std::memcmp(L.data(), c->lights_host.data(), L.size() * sizeof(RtLight)) == 0);
    CG_TRY(c, c->lights.ensure(std::max<size_t>(L.size(), 1) * sizeof(RtLight)), "alloc lights");
    if (!same && n > 0) {
        c->lights_host = L;
        CG_TRY(c, hipMemcpyAsync(c->lights.p, c->lights_host.data(), L.size() * sizeof(RtLight),
                                 hipMemcpyHostToDevice, st), "upload lights");
    }
    F.lights = (const RtLight *)c->lights.p;
    return CG_OK;
}

// The frame's shape and sharding (no scene, lights or device state).
static int frame_shape(const cg_rt_camera *cam, const cg_rt_shard *shard, RtFrame &F)
{
    std::memset(&F, 0, sizeof(F));
    F.W = cam->width;
    F.H = cam->height;
    F.focal = cam->focal;
    F.indirect = cam->indirect;
    F.cam[0] = cam->camera.x; F.cam[1] = cam->camera.y; F.cam[2] = cam->camera.z; F.cam[3] = cam->camera.w;
    std::memcpy(F.R, cam->R, sizeof(F.R));
    cg_rt_shard one{0, 1, kRtTileH, 0, 0, 0, 0};
    const cg_rt_shard *s = shard ? shard : &one;
    if (s->rows > 0) {   // band: rows row0 .. row0 + rows - 1
        if (s->row0 < 0) return CG_E_INVALID;
        F.rank = 0;
        F.nranks = 1;
        F.stripe_h = s->rows;
        F.row0 = s->row0;
        F.rows_out = s->rows;
    } else {
        if (s->rows < 0 || s->nranks < 1 || s->rank < 0 || s->rank >= s->nranks || s->stripe_h <= 0)
            return CG_E_INVALID;
        F.rank = s->rank;
        F.nranks = s->nranks;
        F.stripe_h = s->stripe_h;
        F.rows_out = cg_rt_shard_rows(F.H, s);
    }
    F.out_fmt = CG_PIX_ARGB8888;
    if (s->cols < 0 || s->col0 < 0) return CG_E_INVALID;
    if (s->cols > 0) {   // RGB24 window (checked against the format by the caller)
        if (s->col0 % 16 || s->col0 + s->cols > F.W || (s->cols % 16 && s->col0 + s->cols != F.W))
            return CG_E_INVALID;
        F.wcol0 = s->col0;
        F.wcols = s->cols;
    }
    F.cull_primary = 1;   // exact certificates (cg_rt_dev.h); the probes run without them
    F.cull_shadow = 1;
    return CG_OK;
}

static int fill_frame(cg_ctx *c, const cg_light *lights, int n_lights, const cg_rt_camera *cam,
                      const cg_rt_shard *shard, hipStream_t st, RtFrame &F)
{
    if (!cam || cam->width <= 0 || cam->height <= 0 || n_lights < 0 || n_lights > kMaxLights ||
        (n_lights && !lights))
        return CG_E_INVALID;
    if (c->n_tris < 0) {
        c->err = "render before cg_rt_set_scene";
        return CG_E_NOSCENE;
    }
    const int rc = frame_shape(cam, shard, F);
    if (rc) return rc;
    F.n_tris = c->n_tris;
    F.n_sph = c->n_sph;
    F.nbound = c->nbound;
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    return set_lights(c, lights, n_lights, st, F);
}

// Test hook: rows row0 .. row0 + rows - 1 of the frame by
// the reference's loop with no acceleration (cg_rt_brute.hip), synchronous.
extern "C" int cg_rt_render_brute_device(cg_ctx *c, const cg_light *lights, int n_lights, const cg_rt_camera *cam,
                                         int row0, int rows, uint32_t *d_out, void *stream)
{
    if (!c || !d_out || !cam || row0 < 0 || rows <= 0 || row0 + rows > cam->height || n_lights > 64)
        return CG_E_INVALID;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    RtFrame F;
    int rc = fill_frame(c, lights, n_lights, cam, nullptr, st, F);
    if (rc) return rc;
    CG_TRY(c, rt_render_brute(F, (const cg_tri *)c->tris.p, c->n_tris, (const RtSphere *)c->sph.p, row0, rows, d_out,
                              st),
           "brute-force render");
    return CG_OK;
}

extern "C" int cg_rt_route(const cg_rt_camera *cam, int n_tris, int n_spheres, int n_lights, const cg_rt_shard *shard)
{
    if (!cam || cam->width <= 0 || cam->height <= 0 || n_tris < 0 || n_spheres < 0 || n_lights < 0 ||
        n_lights > kMaxLights)
        return CG_E_INVALID;
    RtFrame F;
    const int rc = frame_shape(cam, shard, F);
    if (rc) return rc;
    F.n_tris = n_tris;
    F.n_sph = n_spheres;
    F.n_lights = n_lights;
    if (F.n_tris > 64) {   // rt_enqueue_kernels: the large-scene path
        const int m = rt_big_mode(F);
        return m == 0 ? CG_RT_ROUTE_BIG_PIXEL : m == 1 ? CG_RT_ROUTE_BIG_LATTICE : CG_RT_ROUTE_BIG_LATTICE_YAW;
    }
    const int k = rt_lattice_kind(F);
    if (k == 0) return CG_RT_ROUTE_PIXEL;
    if (n_lights == 1) return k == 1 ? CG_RT_ROUTE_LATTICE : CG_RT_ROUTE_LATTICE_YAW;
    return k == 1 ? CG_RT_ROUTE_LIGHTS : CG_RT_ROUTE_LIGHTS_YAW;
}

// A large-scene frame slot's buffers (slot 0: the context's own; slot 1: the
// second frame in flight of rt_render_frames).
struct BigSlot {
    DevBuf *tc, *big, *frame;
    unsigned long long **demand;
    hipEvent_t *ev;
    bool *ev_live;
};
static BigSlot big_slot(cg_ctx *c, int q)
{
    if (q) {
        cg_ctx::ExtraSlot &x = c->xs[q - 1];
        return BigSlot{&x.tc, &x.big, &x.frame, &x.demand, &x.ev, &x.ev_live};
    }
    return BigSlot{&c->tc, &c->big, &c->frame, &c->big_demand, &c->big_ev, &c->big_ev_live};
}

static bool big_observe(cg_ctx *c, bool sizing, int q);

// Settle both slots' outstanding pool demand (blocks on their last frames).
static int big_observe_all(cg_ctx *c)
{
    for (int q = 0; q < cg_ctx::kBigSlots; ++q) {
        const BigSlot b = big_slot(c, q);
        if (*b.ev_live) {
            CG_TRY(c, hipEventSynchronize(*b.ev), "pool demand");
            big_observe(c, false, q);
        }
    }
    return CG_OK;
}

extern "C" int cg_rt_scratch_info(cg_ctx *c, uint64_t *out)
{
    if (!c || !out) return CG_E_INVALID;
    if (int rc = big_observe_all(c)) return rc;
    const unsigned long long *d = c->big_last;
    out[0] = c->big.bytes;
    for (const auto &x : c->xs) out[0] += x.big.bytes;
    out[1] = d[0] + d[1] + d[2] + d[3];
    out[2] = (uint64_t)(c->big_caps.sup + c->big_caps.bin + c->big_caps.sbin + c->big_caps.sorted);
    out[3] = (uint64_t)c->big_overflows;
    return CG_OK;
}

extern "C" int cg_rt_pool_demand(cg_ctx *c, uint64_t *out)
{
    if (!c || !out) return CG_E_INVALID;
    if (int rc = big_observe_all(c)) return rc;
    for (int k = 0; k < 4; ++k) out[k] = c->big_last[k];
    return CG_OK;
}

extern "C" int cg_rt_set_pool_caps(cg_ctx *c, long long sup, long long bin, long long sbin, long long sorted)
{
    if (!c || sup < 0 || bin < 0 || sbin < 0 || sorted < 0) return CG_E_INVALID;
    if (c->stream) CG_TRY(c, hipDeviceSynchronize(), "drain before resizing pools");
    c->big_fixed = sup > 0 || bin > 0 || sbin > 0 || sorted > 0;
    c->big_caps = c->big_fixed ? BigCaps{sup, bin, sbin, sorted} : BigCaps{};
    c->big_sized = false;
    c->big_key = -1;
    c->big_overflows = 0;
    return CG_OK;
}

extern "C" int cg_rt_set_pending_cap(cg_ctx *c, int cap)
{
    if (!c || cap < 0) return CG_E_INVALID;
    c->pend_cap = cap;
    return CG_OK;
}

extern "C" int cg_rt_shard_rows(int height, const cg_rt_shard *shard)
{
    cg_rt_shard one{0, 1, kRtTileH, 0, 0, 0, 0};
    const cg_rt_shard *s = shard ? shard : &one;
    if (height <= 0) return CG_E_INVALID;
    if (s->rows > 0) return s->rows;
    if (s->rows < 0 || s->nranks < 1 || s->stripe_h <= 0) return CG_E_INVALID;
    int stripes = (height + s->stripe_h - 1) / s->stripe_h;
    int per = (stripes + s->nranks - 1) / s->nranks;
    return per * s->stripe_h;
}

static int rt_enqueue_kernels(cg_ctx *c, const RtFrame &F, uint32_t *d_out, hipStream_t st, int slot);

// slot: a large scene's frame slot (rt_render_frames' second frame in flight: 1)
static int rt_enqueue(cg_ctx *c, const RtFrame &Fin, void *d_out_v, hipStream_t st, int slot = 0)
{
    // RGB24 output: the lattice kernel stores it directly; the other kernels
    // render ARGB into the context's scratch frame, then one pack pass
    RtFrame F = Fin;
    uint32_t *d_out = (uint32_t *)d_out_v;
    const bool pack = F.out_fmt == CG_PIX_RGB24 && !rt_use_lattice(F);
    if (pack) {
        DevBuf &fr = *big_slot(c, slot).frame;
        CG_TRY(c, fr.ensure((size_t)F.rows_out * F.W * sizeof(uint32_t)), "alloc frame");
        d_out = (uint32_t *)fr.p;
        F.out_fmt = CG_PIX_ARGB8888;
    }
    int rc = rt_enqueue_kernels(c, F, d_out, st, slot);
    if (rc || !pack) return rc;
    CG_TRY(c, launch_rt_pack_rgb24(d_out, F.W, F.rows_out, Fin.wcols ? Fin.wcol0 : 0, Fin.wcols ? Fin.wcols : F.W,
                                   (uint8_t *)d_out_v, st), "pack launch");
    return CG_OK;
}

// The large-scene pools' demand of the latest finished frame: capacities grow
// to 1.25x a demand that came within 80 % of them (so steady frames neither
// overflow nor hold more than ~1.6x what they list); a sizing frame sets them
// to 1.25x its demand either way.  True when the frame overflowed a pool (it
// was still right: the consumers fell back to every triangle).
static bool big_observe(cg_ctx *c, bool sizing, int q)
{
    const BigSlot b = big_slot(c, q);
    std::memcpy(c->big_last, *b.demand, sizeof(c->big_last));
    const unsigned long long *d = c->big_last;
    long long *cap[4] = {&c->big_caps.sup, &c->big_caps.bin, &c->big_caps.sbin, &c->big_caps.sorted};
    bool over = false;
    for (int k = 0; k < 4; ++k) {
        const long long need = (long long)d[k];
        over |= need > *cap[k];
        if (!c->big_fixed && (sizing || need * 5 > *cap[k] * 4))
            *cap[k] = std::min<long long>(need + need / 4 + 4096, (1ll << 31) - 1);
    }
    if (!sizing) c->big_overflows += over;
    *b.ev_live = false;
    return over;
}

// Large scene: binned certificates (cg_rt_big.hip).  The first frame of a
// scene (or of a new frame shape / path) is sized first: dry passes of the
// list kernels alone report the pools' demand until it fits (a pass in which
// a list overflowed under-counts what depends on it), then -- when the frame
// shades through per-bin shadow lists -- dry passes up to those lists.  Later
// frames stay asynchronous and grow the pools for the next ones from their
// reported demand; a frame that still overflows renders through the fallback.
static int rt_big_enqueue(cg_ctx *c, const RtFrame &F, uint32_t *d_out, hipStream_t st, int slot)
{
    const BigSlot S = big_slot(c, slot);
    if (!*S.demand) {
        CG_TRY(c, hipHostMalloc((void **)S.demand, 4 * sizeof(unsigned long long), hipHostMallocDefault),
               "alloc pool demand");
        std::memset(*S.demand, 0, 4 * sizeof(unsigned long long));
        CG_TRY(c, hipEventCreateWithFlags(S.ev, hipEventDisableTiming), "pool event");
    }
    if (c->big_caps.sup == 0) {   // first guess; the first frame corrects it
        const long long g = 2ll * F.n_tris + 65536;
        c->big_caps = BigCaps{g, g, 4096, 2 * g};
    }
    // a new frame shape or path (lattice / per-pixel, many lights) is sized again
    const int mode = rt_big_mode(F);   // per-pixel / lattice / lattice with per-pixel columns
    const int lclass = F.n_lights == 0 ? 0 : F.n_lights <= 7 ? 1 : F.n_lights <= 64 ? 2 : 3;
    const long long key = ((((long long)F.W * 65536 + F.rows_out) * 4 + lclass) * 4 + mode) * 2 + (F.nranks == 1);
    if (key != c->big_key) {
        c->big_key = key;
        c->big_sized = false;
    }
    if (c->big_fixed) c->big_sized = true;
    for (int q = 0; q < cg_ctx::kBigSlots; ++q) {   // any slot's finished frame reports its demand
        const BigSlot b = big_slot(c, q);
        if (*b.ev_live && hipEventQuery(*b.ev) == hipSuccess) big_observe(c, false, q);
    }
    int stage = c->big_sized ? 0 : 1;   // dry stage of the next pass (0: render)
    DevBuf &big = *S.big;
    for (int pass = 0; pass < 8; ++pass) {
        const int dry = pass == 7 ? 0 : stage;
        const size_t need = rt_big_scratch_bytes(F, c->big_caps);
        if ((need > big.bytes || need < big.bytes / 2) && big.p) {   // grow, or give back a sized-down half
            CG_TRY(c, hipDeviceSynchronize(), "drain before resizing scratch");
            big.release();
        }
        CG_TRY(c, big.ensure(need), "alloc large-scene scratch");
        CG_TRY(c, launch_rt_big(F, (RtTri *)S.tc->p, (const RtShade *)c->shade.p, (const RtSphere *)c->sph.p,
                                c->grid, big.p, d_out, st, (const RtGeo *)c->geo.p, (const cg_tri *)c->tris.p,
                                c->pend_cap, c->big_caps,
                                *S.demand, dry),
               "rt_big launch");
        CG_TRY(c, hipEventRecord(*S.ev, st), "pool event");
        *S.ev_live = true;
        if (!dry) break;
        CG_TRY(c, hipEventSynchronize(*S.ev), "pool demand");
        if (big_observe(c, true, slot)) continue;          // grown: the same stage again
        if (stage == 1 && rt_big_shadow_lists(F)) {
            stage = 2;
        } else {
            c->big_sized = true;                     // fits: the next pass renders
            stage = 0;
        }
    }
    return CG_OK;
}

static int rt_enqueue_kernels(cg_ctx *c, const RtFrame &F, uint32_t *d_out, hipStream_t st, int slot)
{
    // a large scene's whole frame (prepare .. shading), for the bench's frame figures
    KtScope kt(F.n_tris > 64 && F.cull_primary && F.cull_shadow ? KT_RT_BIG_FRAME : -1, st);
    unsigned long long *lat = nullptr;
    if (rt_use_lattice(F)) {
        CG_TRY(c, c->latmask.ensure(rt_lattice_tiles(F) * 2 * sizeof(unsigned long long)), "alloc lattice masks");
        lat = (unsigned long long *)c->latmask.p;
    }
    RtFrameCams cams{};
    for (int k = 0; k < 4; ++k) cams.c[0][k] = F.cam[k];
    unsigned long long *supm = nullptr, *um = nullptr;
    if (lat && rt_lattice_unit_bytes(F, 1)) {
        CG_TRY(c, c->umask.ensure(rt_lattice_unit_bytes(F, 1)), "alloc lattice unit masks");
        um = (unsigned long long *)c->umask.p;
    }
    if (lat) {   // two-level tile certificates: super-tiles, then tiles
        CG_TRY(c, c->supmask.ensure(rt_sup_units(F) * 2 * sizeof(unsigned long long)), "alloc super-tile masks");
        supm = (unsigned long long *)c->supmask.p;
    }
    const BigSlot S = big_slot(c, slot);   // slot 1 only for large scenes (rt_render_frames)
    if (slot) {
        const size_t nt = (size_t)std::max(c->n_tris, 1);
        CG_TRY(c, S.tc->ensure(nt * sizeof(RtTri)), "alloc tri constants");
    }
    // large scenes: the super-bin pass forms the frame's RtTri itself (no prepare launch)
    if (F.n_tris > 64 && F.cull_primary && F.cull_shadow) return rt_big_enqueue(c, F, d_out, st, slot);
    CG_TRY(c, launch_rt_prepare((const cg_tri *)c->tris.p, (const RtGeo *)c->geo.p, c->n_tris, cams, 1,
                                (RtTri *)S.tc->p, st, &F, (const RtSphere *)c->sph.p, lat, supm), "rt_prepare launch");
    CG_TRY(c, launch_rt_pixels(F, (const RtTri *)c->tc.p, (const RtShade *)c->shade.p,
                               (const RtSphere *)c->sph.p, lat, um, d_out, st), "rt_pixel launch");
    return CG_OK;
}

extern "C" int cg_rt_render_device(cg_ctx *c, const cg_light *lights, int n_lights,
                                   const cg_rt_camera *cam, const cg_rt_shard *shard,
                                   uint32_t *d_out, void *stream)
{
    if (!c || !d_out) return CG_E_INVALID;
    RtFrame F;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    int rc = fill_frame(c, lights, n_lights, cam, shard, st, F);
    if (rc) return rc;
    if (F.wcols) return CG_E_INVALID;   // windows are for the RGB24 wire format
    return rt_enqueue(c, F, d_out, st);
}

// Frames f0 .. f0 + nf - 1 of a batch, one prepare + one lattice launch
// (rt_use_lattice(F) holds for every frame; they differ only in cameraPos).
static int lat_tiles_x_host(const RtFrame &F) { return (F.W + kLatTileW - 1) / kLatTileW; }

// The launch geometry a lattice order is recorded for (0 never occurs): the
// same key means the same tiles in the same window, so the recording predicts
// the next launch's per-tile cost.  (A different key would still give a valid
// permutation -- the key only avoids a useless order.)
static unsigned long long lat_order_key(const cg_ctx *c, const RtFrame &F)
{
    unsigned long long h = 1469598103934665603ull;
    auto mix = [&h](long long v) { h = (h ^ (unsigned long long)v) * 1099511628211ull; };
    mix(F.W); mix(F.H); mix(F.rows_out); mix(F.row0); mix(F.rank); mix(F.nranks); mix(F.stripe_h);
    mix(F.tx0); mix(F.txn); mix(F.n_lights); mix(F.n_tris); mix(F.n_sph); mix(c->rt_scene_gen);
    uint32_t b;
    std::memcpy(&b, &F.focal, 4); mix(b);
    for (int k : {0, 8, 12}) { std::memcpy(&b, &F.R[k], 4); mix(b); }
    return h | 1ull;
}
// CG_LAT_ORDER (A/B runs): 0 the default dispatch order, 1 frame-major measured order, 2
// interleaved measured order (frame groups, tile-major inside a group; the default).  Measured on
// C2's 20-frame calls (profiles/r05_ab_order.json): interleaved takes the 1/8 bands of the N = 8
// split from 163-169 to 145-168 us (the floor bands gain most: their launch ended on a heavy
// tile's tail), frame-major gains nothing there; both cost whole frames 1-2 % (0.920 -> 0.935 ms
// per 20-frame lattice launch), so only launches of at most kLatOrderRounds rounds of resident
// workgroups take the order (a band's ~13k workgroups: yes; a whole frame's 105k: no).
// Published certificates beside the lattice launch: CG_CERT_CONC=1 (read per call; off by
// default).  Measured on one MI355X (profiles/r06_ab_conc.json, the driver's 20-frame C2 call):
// 14.2-14.5k frames/s against 18.7-18.9k with the certificates first -- once the lattice launch
// holds the CUs the certificate launch is dispatched only as its workgroups retire (its span
// 80 -> 420 us; a high-priority auxiliary stream changes nothing), so lattice workgroups wait for
// their words or, past the bound, render uncertified, which costs ~15x a certified tile (every
// tile uncertified: 1.45k frames/s).  The path stays as the uncertified-path exactness test
// (CG_LAT_FORCE_UNCERT=1, tests/test_rt_conc_gpu.py).
static bool cert_concurrent()
{
    const char *e = std::getenv("CG_CERT_CONC");
    return e && e[0] == '1';
}
// How long a lattice workgroup waits for its published certificates before it renders the tile
// uncertified: wall-clock ticks (100 MHz), default 1 ms; CG_LAT_SPIN for A/B runs (0: never wait).
static uint32_t lat_spin_ticks()
{
    const char *e = std::getenv("CG_LAT_SPIN");
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 100000u;
}

static int lat_order_mode()
{
    static const int m = [] {
        const char *e = std::getenv("CG_LAT_ORDER");
        return e && *e ? std::atoi(e) : 2;
    }();
    return m;
}
constexpr long long kLatOrderRounds = 12;
static long long lat_resident_wgs()
{
    static const long long r = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return (long long)cus * 6;   // rt_lattice_kernel: 6 workgroups per CU
    }();
    return r;
}

static int rt_enqueue_lattice_batch(cg_ctx *c, const RtFrame &F0, const cg_rt_camera *cams, int nf,
                                    void *d_out, size_t stride, hipStream_t st, uint32_t *d_done,
                                    uint32_t *tiles_per_frame, const uint8_t *groups, int ngroups)
{
    // Workgroups only for the tile columns the scene's box can be seen in by
    // some camera of the batch (O(1) per camera from the box, rt_box_columns);
    // the launch's edge workgroups store the rest black.  C2: 73 of 120 tile
    // columns -- the other 47 cost a workgroup each (~1.6 us) per tile row.
    RtFrame F = F0;
    static const bool window = [] {   // CG_LAT_WINDOW=0: every tile column (A/B runs)
        const char *e = std::getenv("CG_LAT_WINDOW");
        return !(e && e[0] == '0');
    }();
    if (window) {
        int a = F.W, b = 0;
        for (int f = 0; f < nf; ++f) {
            int c0, c1;
            ctx_rt_columns(c, &cams[f], &c0, &c1);
            if (c0 < c1) {
                a = std::min(a, c0);
                b = std::max(b, c1);
            }
        }
        const int tx = (F.W + kLatTileW - 1) / kLatTileW;
        int t0 = a / kLatTileW, t1 = (b + kLatTileW - 1) / kLatTileW;
        if (t0 >= t1) {   // nothing visible: one tile column (certified black) and the edges
            t0 = 0;
            t1 = 1;
        }
        if (t0 > 0 || t1 < tx) {
            F.tx0 = t0;
            F.txn = t1 - t0;
        }
    }
    *tiles_per_frame = (uint32_t)((F.txn ? F.txn : (F.W + kLatTileW - 1) / kLatTileW) *
                                  ((F.rows_out + kLatTileH - 1) / kLatTileH));
    if (!c->aux) {
        // default priority: a high-priority auxiliary stream (certificates
        // dispatched ahead of a running lattice launch) gained ~2 % on
        // back-to-back calls, but left the process's later streams sharing
        // hardware queues -- the rasteriser's overlapped frames then ran
        // serialised (C3 10.1-11.1k instead of 21.0-21.3k frames/s)
        {
            // A/B knob: CG_AUX_PRIO=1 creates the auxiliary stream at the highest priority
            const char *pe = std::getenv("CG_AUX_PRIO");
            int lo = 0, hi = 0;
            if (pe && pe[0] == '1' && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess)
                CG_TRY(c, hipStreamCreateWithPriority(&c->aux, hipStreamNonBlocking, hi), "aux stream");
            else
                CG_TRY(c, hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking), "aux stream");
        }
        for (int k = 0; k < 2; ++k) {
            CG_TRY(c, hipEventCreateWithFlags(&c->ev_cert[k], hipEventDisableTiming), "aux event");
            CG_TRY(c, hipEventCreateWithFlags(&c->ev_lat[k], hipEventDisableTiming), "aux event");
            CG_TRY(c, hipEventRecord(c->ev_lat[k], c->aux), "aux event");
        }
    }
    // this call's slot (its buffers were last read by the lattice launch two
    // calls ago, ev_lat[k])
    const int k = c->slot;
    c->slot ^= 1;
    DevBuf &btc = c->ptc[k], &blat = c->plat[k], &bsup = c->psup[k], &bum = c->pumask[k];
    const size_t tiles = rt_lattice_tiles(F);
    // Both slots' certificate buffers are sized together, for a full batch
    // (kMaxFrameBatch frames): a call never allocates -- hipMalloc / hipFree,
    // the latter a device-wide wait -- in front of its kernels merely because
    // it batches more frames than the previous one or is the first on its
    // slot.  The light sets' unit masks (40 MB per 4K frame) are the
    // exception: they are sized for the largest batch this context has asked
    // for so far (a one-frame or band call keeps ~40 MB per slot, not 1.3 GB),
    // growing both slots together when a call batches more.
    const size_t nfa = std::max(nf, kMaxFrameBatch);
    for (int q = 0; q < 2; ++q) {
        CG_TRY(c, c->plat[q].ensure(nfa * tiles * 2 * sizeof(unsigned long long)), "alloc lattice masks");
        CG_TRY(c, c->ptc[q].ensure(nfa * std::max(F.n_tris, 1) * sizeof(RtTri)), "alloc tri constants");
        CG_TRY(c, c->psup[q].ensure(nfa * rt_sup_units(F) * 2 * sizeof(unsigned long long)), "alloc super-tile masks");
    }
    if (rt_lattice_unit_bytes(F, nf)) {
        c->umask_frames = std::max(c->umask_frames, nf);
        for (int q = 0; q < 2; ++q)
            CG_TRY(c, c->pumask[q].ensure(rt_lattice_unit_bytes(F, c->umask_frames)), "alloc lattice unit masks");
    }
    RtFrameCams fc{};
    for (int f = 0; f < nf; ++f) {
        fc.c[f][0] = cams[f].camera.x; fc.c[f][1] = cams[f].camera.y;
        fc.c[f][2] = cams[f].camera.z; fc.c[f][3] = cams[f].camera.w;
    }
    unsigned long long *lat = (unsigned long long *)blat.p;
    unsigned long long *supm = (unsigned long long *)bsup.p;
    // certificates on aux, after the slot's previous reader, so that they run
    // beside the lattice launch still queued before them.  A cold call (every
    // earlier lattice launch of this context complete: nothing to run beside)
    // keeps them on the caller's stream -- the cross-stream wait would leave
    // the GPU idle for ~12 us between certificates and lattice.
    const bool cold = hipEventQuery(c->ev_lat[0]) == hipSuccess && hipEventQuery(c->ev_lat[1]) == hipSuccess;
    // Measured order (one-light lattice kernel): sort the latest complete
    // recording of this geometry -- the other slot's (the previous call) when
    // every lattice launch is done, else this slot's (two calls ago, complete:
    // cst waited on it) -- in the certificate launch; this launch records into
    // this slot.
    const int gx = F.txn ? F.txn : lat_tiles_x_host(F), gy = (F.rows_out + kLatTileH - 1) / kLatTileH;
    const unsigned long long key = lat_order_key(c, F);
    LatOrder order{};
    LatFlatten flat{};
    const bool ordered = lat_order_mode() > 0 && F.n_lights == 1 &&
                         (long long)gx * gy * nf <= kLatOrderRounds * lat_resident_wgs();
    // Published certificates (LatReady, cg_internal.h): the one-light lattice
    // launch starts beside its certificate launch instead of after it, each
    // workgroup waiting only for its own super-tile (calls in the default
    // order: whole frames; band calls keep the measured order, whose sort the
    // certificate launch does first)
    const bool conc = cert_concurrent() && !ordered && F.n_lights == 1 && F.n_tris <= 62 &&
                      !rt_lattice_unit_bytes(F, nf);
    // certificates on aux, after the slot's previous reader, so that they run
    // beside the lattice launch still queued before them (or, published, beside
    // this call's own).  A cold call with unpublished certificates (every
    // earlier lattice launch of this context complete: nothing to run beside)
    // keeps them on the caller's stream -- the cross-stream wait would leave
    // the GPU idle for ~12 us between certificates and lattice.
    hipStream_t cst = (cold && !conc) ? st : c->aux;
    if (!cold) CG_TRY(c, hipStreamWaitEvent(cst, c->ev_lat[k], 0), "aux wait");
    LatPublish pub{};
    LatReady ready{};
    if (conc) {
        const size_t units = rt_sup_units(F), words = nfa * units;
        for (int q = 0; q < 2; ++q) {
            const size_t had = c->pflag[q].bytes;
            CG_TRY(c, c->pflag[q].ensure(words * sizeof(uint32_t)), "alloc certificate words");
            if (c->pflag[q].bytes != had) {   // fresh words: zero (no generation), before any launch reads them
                CG_TRY(c, hipMemsetAsync(c->pflag[q].p, 0, c->pflag[q].bytes, st), "zero certificate words");
                CG_TRY(c, hipStreamSynchronize(st), "zero certificate words");
            }
        }
        uint32_t gen = ++c->cert_gen;
        if (gen == 0u) gen = ++c->cert_gen;
        pub = LatPublish{(uint32_t *)c->pflag[k].p, gen, (int)units};
        const char *fe = std::getenv("CG_LAT_FORCE_UNCERT");   // test hook, read per call
        ready = LatReady{(const uint32_t *)c->pflag[k].p, gen, (int)units, (lat_tiles_x_host(F) + kSup - 1) / kSup,
                         fe && fe[0] == '1', lat_spin_ticks(), (const RtGeo *)c->geo.p, (RtTri *)btc.p};
    }
    if (ordered) {
        for (int q = 0; q < 2; ++q) {
            // a reallocated cost map holds no recording: forget both slots' keys, or a later
            // call of the earlier geometry would sort uninitialised memory
            if ((size_t)gx * gy > c->lcost[q].bytes) c->lrec_key[0] = c->lrec_key[1] = 0ull;
            CG_TRY(c, c->lcost[q].ensure((size_t)gx * gy), "alloc lattice order");
            CG_TRY(c, c->lflat[q].ensure((size_t)gx * gy * sizeof(uint32_t)), "alloc lattice order");
        }
        const int src = (cold && c->lrec_key[k ^ 1] == key) ? (k ^ 1) : c->lrec_key[k] == key ? k : -1;
        if (src >= 0) flat = LatFlatten{(const uint8_t *)c->lcost[src].p, (uint32_t *)c->lflat[k].p, gx * gy};
    }
    CG_TRY(c, launch_rt_prepare((const cg_tri *)c->tris.p, (const RtGeo *)c->geo.p, c->n_tris, fc, nf,
                                (RtTri *)btc.p, cst, &F, (const RtSphere *)c->sph.p, lat, supm,
                                flat.n > 0 ? &flat : nullptr, conc ? &pub : nullptr),
           "rt_prepare launch");
    if (conc && !pub.done) ready = LatReady{};   // not published (the split certificate form): nothing to wait for
    if (ordered) {
        if (flat.n < 0) order.flat = (const uint32_t *)c->lflat[k].p;   // sorted by the certificate launch
        order.cost = (uint8_t *)c->lcost[k].p;
        c->lrec_key[k] = key;
        order.ngroups = -1;   // frame-major
        if (lat_order_mode() == 2) {
            order.ngroups = 0;
            if (groups && ngroups > 0 && ngroups <= kLatMaxGroups) {
                order.ngroups = ngroups;
                for (int g = 0; g <= ngroups; ++g) order.gs[g] = groups[g];
            }
        }
    }
    // light sets: the per-unit shadow certificates, with the other certificates
    unsigned long long *um = nullptr;
    if (rt_lattice_unit_bytes(F, nf)) {
        um = (unsigned long long *)bum.p;
        CG_TRY(c, launch_rt_lattice_units(F, (const RtTri *)btc.p, (const RtShade *)c->shade.p, (const RtSphere *)c->sph.p,
                                          lat, fc, nf, um, cst),
               "rt_lattice_units launch");
    }
    if (!cold || conc) CG_TRY(c, hipEventRecord(c->ev_cert[k], cst), "aux record");
    if (!cold && !conc) CG_TRY(c, hipStreamWaitEvent(st, c->ev_cert[k], 0), "aux wait");
    CG_TRY(c, launch_rt_lattice_frames(F, (const RtTri *)btc.p, (const RtShade *)c->shade.p,
                                       (const RtSphere *)c->sph.p, lat, um, fc, nf, stride, (uint32_t *)d_out, st,
                                       d_done, ordered ? &order : nullptr, ready.flags ? &ready : nullptr),
           "rt_lattice launch");
    // published: whatever the caller queues after this call follows the certificates too
    if (conc) CG_TRY(c, hipStreamWaitEvent(st, c->ev_cert[k], 0), "aux wait");
    CG_TRY(c, hipEventRecord(c->ev_lat[k], st), "aux record");
    return CG_OK;
}

// Large-scene frames in flight: 2 by default; CG_BIG_SLOTS = 1 .. kBigSlots for A/B runs.
static int big_slots()
{
    static const int n = [] {
        const char *e = std::getenv("CG_BIG_SLOTS");
        const int v = e ? std::atoi(e) : 2;
        return std::max(1, std::min(v, cg_ctx::kBigSlots));
    }();
    return n;
}

static size_t pix_bytes(int fmt) { return fmt == CG_PIX_RGB24 ? 3 : 4; }

namespace cg {
int rt_render_frames(cg_ctx *c, const cg_light *lights, int n_lights, const cg_rt_camera *cams, int n_frames,
                     const cg_rt_shard *shard, void *d_out, size_t frame_stride, int pix_format, void *stream,
                     uint32_t *d_done, uint32_t *target, const int *group_starts, int ngroups);
}

extern "C" int cg_rt_render_frames_device(cg_ctx *c, const cg_light *lights, int n_lights,
                                          const cg_rt_camera *cams, int n_frames, const cg_rt_shard *shard,
                                          void *d_out, size_t frame_stride, int pix_format, void *stream)
{
    return rt_render_frames(c, lights, n_lights, cams, n_frames, shard, d_out, frame_stride, pix_format, stream,
                            nullptr, nullptr, nullptr, 0);
}

namespace cg {
// cg_rt_render_frames_device, plus per-frame completion signals for cg_dist:
// with d_done (signal memory, zeroed by the caller), frame f is complete once
// d_done[f] >= target[f] (the lattice kernels count the frame's tiles as they
// are stored; other paths write 1 after the frame's kernels).
// group_starts (optional, ngroups + 1 entries, the last n_frames): frames
// dispatched group after group (cg_dist's chunks, sent as each completes).
int rt_render_frames(cg_ctx *c, const cg_light *lights, int n_lights, const cg_rt_camera *cams, int n_frames,
                     const cg_rt_shard *shard, void *d_out, size_t frame_stride, int pix_format, void *stream,
                     uint32_t *d_done, uint32_t *target, const int *group_starts, int ngroups)
{
    if (!c || !d_out || n_frames < 0 || (n_frames && !cams)) return CG_E_INVALID;
    if (pix_format != CG_PIX_ARGB8888 && pix_format != CG_PIX_RGB24) return CG_E_INVALID;
    if (n_frames == 0) return CG_OK;
    for (int f = 1; f < n_frames; ++f)
        if (cams[f].width != cams[0].width || cams[f].height != cams[0].height) return CG_E_INVALID;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    RtFrame F;
    int rc = fill_frame(c, lights, n_lights, &cams[0], shard, st, F);
    if (rc) return rc;
    F.out_fmt = pix_format;
    if (F.wcols && pix_format != CG_PIX_RGB24) return CG_E_INVALID;
    const size_t px = (size_t)F.rows_out * (F.wcols ? F.wcols : F.W);
    const size_t stride = frame_stride ? frame_stride : px;   // pixels
    if (stride < px) return CG_E_INVALID;
    uint8_t *out = (uint8_t *)d_out;
    const size_t fbytes = stride * pix_bytes(pix_format);
    // one batched launch needs the lattice path for every frame, frames that
    // differ only in cameraPos (same focal, R, indirect)
    bool batch = rt_use_lattice(F);
    for (int f = 1; batch && f < n_frames; ++f)
        batch = cams[f].focal == cams[0].focal && cams[f].indirect == cams[0].indirect &&
                std::memcmp(cams[f].R, cams[0].R, sizeof(cams[0].R)) == 0;
    if (!batch) {
        // Large scenes: consecutive frames are dealt round-robin to big_slots()
        // slots, each with its own buffers and stream: independent frames in flight
        const int ns = (n_frames > 1 && F.n_tris > 64 && F.cull_primary && F.cull_shadow)
                           ? std::min(big_slots(), n_frames) : 1;
        if (ns > 1) {
            if (!c->bev_start) CG_TRY(c, hipEventCreateWithFlags(&c->bev_start, hipEventDisableTiming), "slot event");
            // the other slots start after what the caller queued before this
            // call (the scene, the lights just uploaded on st)
            CG_TRY(c, hipEventRecord(c->bev_start, st), "slot event");
            for (int q = 1; q < ns; ++q) {
                cg_ctx::ExtraSlot &x = c->xs[q - 1];
                if (!x.st) {
                    CG_TRY(c, hipStreamCreateWithFlags(&x.st, hipStreamNonBlocking), "slot stream");
                    CG_TRY(c, hipEventCreateWithFlags(&x.done, hipEventDisableTiming), "slot event");
                }
                CG_TRY(c, hipStreamWaitEvent(x.st, c->bev_start, 0), "slot wait");
            }
        }
        for (int f = 0; f < n_frames; ++f) {
            if (f) {
                rc = fill_frame(c, lights, n_lights, &cams[f], shard, st, F);
                if (rc) return rc;
                F.out_fmt = pix_format;
            }
            const int q = f % ns;
            hipStream_t fs = q ? c->xs[q - 1].st : st;
            rc = rt_enqueue(c, F, out + (size_t)f * fbytes, fs, q);
            if (rc) return rc;
            if (d_done) {
                CG_TRY(c, hipStreamWriteValue32(fs, d_done + f, 1u, 0), "frame signal");
                target[f] = 1u;
            }
        }
        for (int q = 1; q < ns; ++q) {   // the call ends on the caller's stream
            cg_ctx::ExtraSlot &x = c->xs[q - 1];
            CG_TRY(c, hipEventRecord(x.done, x.st), "slot event");
            CG_TRY(c, hipStreamWaitEvent(st, x.done, 0), "slot wait");
        }
        return CG_OK;
    }
    // (A cold call split into a head batch, whose lattice launch runs beside
    // the rest's certificates on a high-priority auxiliary stream, measured
    // slower: 16.0k against 17.2k frames/s for the driver's 20-frame C2 call --
    // the certificates beside a lattice launch took 0.56 ms instead of 0.12.)
    for (int f0 = 0; f0 < n_frames;) {
        const int nf = std::min(kMaxFrameBatch, n_frames - f0);
        uint32_t wg = 0;
        uint8_t gs[kLatMaxGroups + 1];   // the groups within this launch's frames
        int ng = 0;
        if (group_starts && ngroups > 0) {
            gs[0] = 0;
            for (int g = 1; g <= ngroups && ng < kLatMaxGroups; ++g) {
                const int e = std::min(group_starts[g], f0 + nf) - f0;
                if (e > gs[ng]) gs[++ng] = (uint8_t)e;
            }
            if (ng == 0 || gs[ng] != nf) ng = 0;   // not covering the launch: one group
        }
        rc = rt_enqueue_lattice_batch(c, F, cams + f0, nf, out + (size_t)f0 * fbytes, stride, st,
                                      d_done ? d_done + f0 : nullptr, &wg, ng ? gs : nullptr, ng);
        if (rc) return rc;
        if (d_done)
            for (int f = f0; f < f0 + nf; ++f) target[f] = wg;   // the launch's workgroups per frame
        f0 += nf;
    }
    return CG_OK;
}
}  // namespace cg

extern "C" int cg_rt_assemble_device(cg_ctx *c, const void *d_src, int pix_format, const int *row0,
                                     const int *rows, int n_blocks, int width, int height, int n_frames,
                                     uint32_t *d_frames, size_t frame_stride, int col0, int cols, void *stream)
{
    if (cols < 0 || col0 < 0 || (cols > 0 && (col0 % 4 || cols % 4 || col0 + cols > width))) return CG_E_INVALID;
    if (!c || !d_src || !d_frames || !row0 || !rows || n_blocks < 1 || n_blocks > kMaxBlocks || width <= 0 ||
        height <= 0 || n_frames < 1 || n_frames > 65535)
        return CG_E_INVALID;
    if (pix_format != CG_PIX_ARGB8888 && pix_format != CG_PIX_RGB24) return CG_E_INVALID;
    if (frame_stride == 0) frame_stride = (size_t)width * height;
    if (frame_stride < (size_t)width * height) return CG_E_INVALID;
    RtBlocks B{};
    B.n = n_blocks;
    B.W = width;
    B.H = height;
    B.bpp = (int)pix_bytes(pix_format);
    B.wcol0 = col0;
    B.wcols = cols;
    B.cum[0] = 0;
    for (int b = 0; b < n_blocks; ++b) {
        if (rows[b] < 0 || row0[b] < 0) return CG_E_INVALID;
        B.row0[b] = row0[b];
        B.rows[b] = rows[b];
        B.cum[b + 1] = B.cum[b] + rows[b];
    }
    if (B.cum[n_blocks] > 65535) return CG_E_INVALID;
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    CG_TRY(c, launch_rt_assemble((const uint8_t *)d_src, B, n_frames, d_frames, frame_stride,
                                 stream ? (hipStream_t)stream : c->stream), "assemble launch");
    return CG_OK;
}

// Host-buffer delivery of frames (cg_rt_render, cg_rt_render_frames): only the
// columns the camera can see anything in (cg_rt_frame_columns, from the
// scene's box) cross PCIe; the columns outside are certainly
// PutPixelSDL(0, 0, 0) = 0x80000000 (no ray there can hit anything,
// skeleton.cpp:160-166) and the host stores them itself while the GPU renders
// and copies.  C2: columns 384-1551, 61 % of the bytes.  CG_DRAW_WINDOW=0:
// whole rows (A/B runs).
static bool draw_window_on()
{
    static const bool on = [] {
        const char *e = std::getenv("CG_DRAW_WINDOW");
        return !(e && e[0] == '0');
    }();
    return on;
}
// [c0, c1) of frame f's download; false: whole rows
static bool draw_window(const cg_ctx *c, const cg_rt_camera *cam, int &c0, int &c1)
{
    c0 = 0;
    c1 = cam->width;
    if (!draw_window_on()) return false;
    ctx_rt_columns(c, cam, &c0, &c1);
    if (c1 <= c0) c0 = c1 = 0;   // nothing visible: a black frame, nothing to copy
    return c0 > 0 || c1 < cam->width;
}
// frames of rows x W pixels (row pitch W): columns outside [c0, c1) black, on
// the context's fill threads (CG_DRAW_THREADS, default min(8, cores / 2));
// returns at once, HostFill::wait() before the frames are complete
static HostFill *host_black_outside(cg_ctx *c, std::vector<HostFill::Frame> frames, int W, int rows, int c0, int c1)
{
    if (!c->hfill) {
        const char *e = std::getenv("CG_DRAW_THREADS");
        const int hw = (int)std::thread::hardware_concurrency();
        const int n = e && *e ? std::atoi(e) : std::min(8, std::max(1, hw / 2));
        c->hfill.reset(new HostFill(std::max(0, std::min(n, 64))));
    }
    c->hfill->run(std::move(frames), W, rows, c0, c1);
    return c->hfill.get();
}
// D2H of frames [nf frames of W x H at src (pitch W, frame stride px)] into
// dst (frame stride `stride`): the window's columns only (one pitched copy
// when the frames are contiguous on both sides), or everything.
static hipError_t download_frames(uint32_t *dst, size_t stride, const uint32_t *src, int W, int H, int nf, int c0,
                                  int c1, bool window, hipStream_t st)
{
    const size_t px = (size_t)W * H;
    if (!window) {
        if (stride == px) return hipMemcpyAsync(dst, src, (size_t)nf * px * 4, hipMemcpyDeviceToHost, st);
        for (int f = 0; f < nf; ++f) {
            const hipError_t e = hipMemcpyAsync(dst + (size_t)f * stride, src + (size_t)f * px, px * 4,
                                                hipMemcpyDeviceToHost, st);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    if (c1 <= c0) return hipSuccess;
    if (stride == px)
        return hipMemcpy2DAsync(dst + c0, (size_t)W * 4, src + c0, (size_t)W * 4, (size_t)(c1 - c0) * 4,
                                (size_t)nf * H, hipMemcpyDeviceToHost, st);
    for (int f = 0; f < nf; ++f) {
        const hipError_t e = hipMemcpy2DAsync(dst + (size_t)f * stride + c0, (size_t)W * 4, src + (size_t)f * px + c0,
                                              (size_t)W * 4, (size_t)(c1 - c0) * 4, H, hipMemcpyDeviceToHost, st);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

extern "C" int cg_rt_render(cg_ctx *c, const cg_light *lights, int n_lights, const cg_rt_camera *cam,
                            uint32_t *argb, cg_stats *stats)
{
    if (!c || !argb) return CG_E_INVALID;
    auto t0 = std::chrono::steady_clock::now();
    RtFrame F;
    int rc = fill_frame(c, lights, n_lights, cam, nullptr, c->stream, F);
    if (rc) return rc;
    size_t bytes = (size_t)F.rows_out * F.W * sizeof(uint32_t);
    CG_TRY(c, c->frame.ensure(bytes), "alloc frame");
    CG_TRY(c, hipEventRecord(c->ev0, c->stream), "event");
    rc = rt_enqueue(c, F, (uint32_t *)c->frame.p, c->stream);
    if (rc) return rc;
    CG_TRY(c, hipEventRecord(c->ev1, c->stream), "event");
    int c0, c1;
    const bool window = draw_window(c, cam, c0, c1);
    // the black columns beside the render and the copy
    HostFill *hf = window ? host_black_outside(c, {{argb}}, F.W, F.H, c0, c1) : nullptr;
    const hipError_t e = download_frames(argb, (size_t)F.W * F.H, (const uint32_t *)c->frame.p, F.W, F.H, 1, c0, c1,
                                         window, c->stream);
    if (hf) hf->wait();
    CG_TRY(c, e, "download frame");
    CG_TRY(c, hipStreamSynchronize(c->stream), "rt frame");
    if (stats) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
        stats->kernel_ms = ms;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        stats->n_tris = c->n_tris;
        stats->n_spans = 0;
    }
    return CG_OK;
}

// n_frames frames into host memory: chunks of `chunk` frames render through
// rt_render_frames into two device slots on the context's stream; each
// chunk's download runs on `xfer` while the next chunk renders.  The download
// of chunk j is issued after chunk j + 1's render is enqueued: a pageable
// destination makes hipMemcpyAsync stage through the runtime's pinned buffers
// and return only when the copy is done, so issued in the other order the
// host would hold back the next render.
extern "C" int cg_rt_render_frames(cg_ctx *c, const cg_light *lights, int n_lights, const cg_rt_camera *cams,
                                   int n_frames, uint32_t *argb, size_t frame_stride, int chunk, cg_stats *stats)
{
    if (!c || !argb || n_frames < 0 || (n_frames && !cams) || chunk < 0) return CG_E_INVALID;
    if (n_frames == 0) return CG_OK;
    auto t0 = std::chrono::steady_clock::now();
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    const int W = cams[0].width, H = cams[0].height;
    if (W <= 0 || H <= 0) return CG_E_INVALID;
    for (int f = 1; f < n_frames; ++f)   // the slots hold chunks of W x H frames
        if (cams[f].width != W || cams[f].height != H) return CG_E_INVALID;
    const size_t px = (size_t)W * H;
    const size_t stride = frame_stride ? frame_stride : px;
    if (stride < px) return CG_E_INVALID;
    const int ch = chunk ? std::min(chunk, 64) : 8;
    if (!c->xfer) {
        CG_TRY(c, hipStreamCreateWithFlags(&c->xfer, hipStreamNonBlocking), "copy stream");
        for (int k = 0; k < 2; ++k) {
            CG_TRY(c, hipEventCreateWithFlags(&c->ev_rdone[k], hipEventDisableTiming), "copy event");
            CG_TRY(c, hipEventCreateWithFlags(&c->ev_cdone[k], hipEventDisableTiming), "copy event");
        }
    }
    // Every return below, error or not, leaves nothing of this call running:
    // earlier chunks' downloads may still be writing into argb (asynchronous
    // when it is pinned), and the stream may wait on their events.
    struct Drain {
        cg_ctx *c;
        ~Drain()
        {
            if (c->hfill) c->hfill->wait();   // the host's black columns
            (void)hipStreamSynchronize(c->xfer);
            (void)hipStreamSynchronize(c->stream);
        }
    } drain_on_exit{c};
    for (int k = 0; k < 2; ++k) CG_TRY(c, c->hslot[k].ensure((size_t)ch * px * sizeof(uint32_t)), "alloc frame slots");
    const int nchunks = (n_frames + ch - 1) / ch;
    auto download = [&](int j) -> int {
        const int s = j & 1, f0 = j * ch, nf = std::min(ch, n_frames - f0);
        CG_TRY(c, hipStreamWaitEvent(c->xfer, c->ev_rdone[s], 0), "copy wait");
        // the chunk's union window (cg_rt_render's delivery, above)
        int a = W, b = 0;
        bool window = true;
        for (int f = f0; f < f0 + nf && window; ++f) {
            int x0, x1;
            window = draw_window(c, &cams[f], x0, x1);
            if (x1 > x0) {
                a = std::min(a, x0);
                b = std::max(b, x1);
            }
        }
        if (a >= b) a = b = 0;
        if (window) {   // the fill threads beside the copy (a pageable copy returns only when done)
            std::vector<HostFill::Frame> fr;
            for (int f = f0; f < f0 + nf; ++f) fr.push_back({argb + (size_t)f * stride});
            host_black_outside(c, std::move(fr), W, H, a, b);
        }
        CG_TRY(c, download_frames(argb + (size_t)f0 * stride, stride, (const uint32_t *)c->hslot[s].p, W, H, nf, a, b,
                                  window, c->xfer), "download frames");
        CG_TRY(c, hipEventRecord(c->ev_cdone[s], c->xfer), "copy event");
        return CG_OK;
    };
    CG_TRY(c, hipEventRecord(c->ev0, c->stream), "event");
    for (int j = 0; j < nchunks; ++j) {
        const int s = j & 1, f0 = j * ch, nf = std::min(ch, n_frames - f0);
        if (j >= 2) CG_TRY(c, hipStreamWaitEvent(c->stream, c->ev_cdone[s], 0), "slot wait");   // chunk j - 2 downloaded
        int rc = rt_render_frames(c, lights, n_lights, cams + f0, nf, nullptr, c->hslot[s].p, px, CG_PIX_ARGB8888,
                                  c->stream, nullptr, nullptr, nullptr, 0);
        if (rc) return rc;
        CG_TRY(c, hipEventRecord(c->ev_rdone[s], c->stream), "render event");
        if (j >= 1 && (rc = download(j - 1))) return rc;
    }
    CG_TRY(c, hipEventRecord(c->ev1, c->stream), "event");
    if (int rc = download(nchunks - 1)) return rc;
    CG_TRY(c, hipStreamSynchronize(c->xfer), "download frames");
    CG_TRY(c, hipStreamSynchronize(c->stream), "rt frames");
    if (stats) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
        stats->kernel_ms = ms;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        stats->n_tris = c->n_tris;
        stats->n_spans = 0;
        stats->n_shaded = -1;
    }
    return CG_OK;
}

extern "C" int cg_rt_unstripe_batch_device(cg_ctx *c, const uint32_t *d_gathered, int width, int height,
                                           int nranks, int stripe_h, int nframes, uint32_t *d_frames, void *stream)
{
    if (!c || !d_gathered || !d_frames || width <= 0 || height <= 0 || nranks < 1 || stripe_h <= 0 ||
        nframes < 1 || nframes > 65535)
        return CG_E_INVALID;
    cg_rt_shard s{0, nranks, stripe_h, 0, 0, 0, 0};
    int rows = cg_rt_shard_rows(height, &s);
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    CG_TRY(c, launch_rt_unstripe(d_gathered, width, height, nranks, stripe_h, rows, nframes, d_frames,
                                 stream ? (hipStream_t)stream : c->stream), "unstripe launch");
    return CG_OK;
}

extern "C" int cg_rt_unstripe_device(cg_ctx *c, const uint32_t *d_gathered, int width, int height,
                                     int nranks, int stripe_h, uint32_t *d_frame, void *stream)
{
    return cg_rt_unstripe_batch_device(c, d_gathered, width, height, nranks, stripe_h, 1, d_frame, stream);
}

extern "C" int cg_rt_probe_closest(cg_ctx *c, const cg_vec4 *starts, const cg_vec4 *dirs, int n,
                                   cg_isect *out, int *hit)
{
    if (!c || n < 0 || (n && (!starts || !dirs || !out || !hit))) return CG_E_INVALID;
    if (c->n_tris < 0) return CG_E_NOSCENE;
    if (n == 0) return CG_OK;
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    CG_TRY(c, c->probe_a.ensure((size_t)n * sizeof(cg_vec4)), "alloc");
    CG_TRY(c, c->probe_b.ensure((size_t)n * sizeof(cg_vec4)), "alloc");
    CG_TRY(c, c->probe_c.ensure((size_t)n * sizeof(cg_isect)), "alloc");
    CG_TRY(c, c->probe_d.ensure((size_t)n * sizeof(int)), "alloc");
    CG_TRY(c, hipMemcpyAsync(c->probe_a.p, starts, (size_t)n * sizeof(cg_vec4), hipMemcpyHostToDevice, c->stream), "h2d");
    CG_TRY(c, hipMemcpyAsync(c->probe_b.p, dirs, (size_t)n * sizeof(cg_vec4), hipMemcpyHostToDevice, c->stream), "h2d");
    RtFrame F;
    std::memset(&F, 0, sizeof(F));
    F.n_tris = c->n_tris;
    F.n_sph = c->n_sph;
    F.nbound = c->nbound;
    CG_TRY(c, launch_rt_probe_closest(F, (const cg_tri *)c->tris.p, (const RtSphere *)c->sph.p,
                                      (const cg_vec4 *)c->probe_a.p, (const cg_vec4 *)c->probe_b.p, n,
                                      (cg_isect *)c->probe_c.p, (int *)c->probe_d.p, c->stream), "probe");
    CG_TRY(c, hipMemcpyAsync(out, c->probe_c.p, (size_t)n * sizeof(cg_isect), hipMemcpyDeviceToHost, c->stream), "d2h");
    CG_TRY(c, hipMemcpyAsync(hit, c->probe_d.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, c->stream), "d2h");
    CG_TRY(c, hipStreamSynchronize(c->stream), "probe sync");
    return CG_OK;
}

extern "C" int cg_rt_probe_direct_light(cg_ctx *c, const cg_isect *isects, const cg_light *light,
                                        int n, cg_vec3 *out)
{
    if (!c || !light || n < 0 || (n && (!isects || !out))) return CG_E_INVALID;
    if (c->n_tris < 0) return CG_E_NOSCENE;
    if (n == 0) return CG_OK;
    for (int i = 0; i < n; ++i) {
        int ti = isects[i].triangleIndex, si = isects[i].sphereIndex;
        if (ti != -1 ? (ti < 0 || ti >= c->n_tris) : (si < 0 || si >= c->n_sph)) return CG_E_INVALID;
    }
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    RtFrame F;
    std::memset(&F, 0, sizeof(F));
    F.n_tris = c->n_tris;
    F.n_sph = c->n_sph;
    F.nbound = c->nbound;
    int rc = set_lights(c, light, 1, c->stream, F);
    if (rc) return rc;
    // shadow rays use generic starts: RtTri constants are camera-independent
    // except s/detT/K2/K3, which the shadow path does not read.
    RtFrameCams zero{};
    zero.c[0][3] = 1.0f;
    CG_TRY(c, launch_rt_prepare((const cg_tri *)c->tris.p, (const RtGeo *)c->geo.p, c->n_tris, zero, 1,
                                (RtTri *)c->tc.p, c->stream, nullptr, nullptr, nullptr, nullptr), "prepare");
    CG_TRY(c, c->probe_c.ensure((size_t)n * sizeof(cg_isect)), "alloc");
    CG_TRY(c, c->probe_a.ensure((size_t)n * sizeof(cg_vec3) + 16), "alloc");
    CG_TRY(c, hipMemcpyAsync(c->probe_c.p, isects, (size_t)n * sizeof(cg_isect), hipMemcpyHostToDevice, c->stream), "h2d");
    CG_TRY(c, launch_rt_probe_direct_light(F, (const RtTri *)c->tc.p, (const RtShade *)c->shade.p,
                                           (const RtSphere *)c->sph.p, (const cg_isect *)c->probe_c.p,
                                           n, (cg_vec3 *)c->probe_a.p, c->stream), "probe");
    CG_TRY(c, hipMemcpyAsync(out, c->probe_a.p, (size_t)n * sizeof(cg_vec3), hipMemcpyDeviceToHost, c->stream), "d2h");
    CG_TRY(c, hipStreamSynchronize(c->stream), "probe sync");
    return CG_OK;
}

// ---------------------------------------------------------------------------
// RAST entry points (kernels in cg_rast.hip)

extern "C" int cg_glibc_rand(uint64_t offset, int n, int32_t *out);

// bit k set: some triangle of the list carries texture k (1-3)
static int rast_tex_mask(const cg_rtri *t, int n)
{
    int m = 0;
    for (int i = 0; i < n; ++i)
        if (t[i].color.x >= 0 && t[i].texture != 0)
            m |= (t[i].texture >= 1 && t[i].texture <= 3) ? 1 << t[i].texture : 1 << 4;   // 16: no such texture
    return m;
}

extern "C" int cg_rast_render_device(cg_ctx *c, const cg_rtri *d_tris, int n,
                                     const cg_rast_params *p, cg_vec4 light, uint32_t *d_argb,
                                     float *d_depth, int32_t *d_shadow, void *stream)
{
    if (!c || !p || !d_argb || n < 0 || (n && !d_tris)) return CG_E_INVALID;
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    // device lists are not inspected: textures run if any maps are loaded
    return rast_render_device(c, d_tris, n, p, light, d_argb, d_depth, d_shadow,
                              stream ? (hipStream_t)stream : c->stream, nullptr, c->tex_loaded);
}

extern "C" int cg_rast_render(cg_ctx *c, const cg_rtri *tris, int n, const cg_rast_params *p,
                              cg_vec4 light, uint32_t *argb, float *depth, int32_t *shadow,
                              cg_stats *stats)
{
    if (!c || !p || !argb || n < 0 || (n && !tris) || p->width <= 2 || p->height <= 2 ||
        p->height > kRastMaxH)
        return CG_E_INVALID;
    auto t0 = std::chrono::steady_clock::now();
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    size_t npx = (size_t)p->width * p->height;
    hipError_t e;
    cg_rtri *d_tris = (cg_rtri *)ctx_buf(c, 0, (size_t)(n > 0 ? n : 1) * sizeof(cg_rtri), &e);
    if (!d_tris) return ctx_fail(c, e, "alloc rast tris");
    uint32_t *d_argb = (uint32_t *)ctx_buf(c, 4, npx * 4, &e);
    if (!d_argb) return ctx_fail(c, e, "alloc argb");
    float *d_depth = (float *)ctx_buf(c, 5, npx * 4, &e);
    if (!d_depth) return ctx_fail(c, e, "alloc depth");
    int32_t *d_shadow = (int32_t *)ctx_buf(c, 6, npx * 4, &e);
    if (!d_shadow) return ctx_fail(c, e, "alloc shadow");
    if (n) CG_TRY(c, hipMemcpyAsync(d_tris, tris, (size_t)n * sizeof(cg_rtri), hipMemcpyHostToDevice, c->stream), "upload tris");
    int rc = rast_render_device(c, d_tris, n, p, light, d_argb, d_depth, d_shadow, c->stream, stats,
                                rast_tex_mask(tris, n));
    if (rc) return rc;
    CG_TRY(c, hipMemcpyAsync(argb, d_argb, npx * 4, hipMemcpyDeviceToHost, c->stream), "d2h argb");
    if (depth) CG_TRY(c, hipMemcpyAsync(depth, d_depth, npx * 4, hipMemcpyDeviceToHost, c->stream), "d2h depth");
    if (shadow) CG_TRY(c, hipMemcpyAsync(shadow, d_shadow, npx * 4, hipMemcpyDeviceToHost, c->stream), "d2h shadow");
    CG_TRY(c, hipStreamSynchronize(c->stream), "rast frame");
    if (stats) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
        stats->kernel_ms = ms;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        stats->n_tris = n;
    }
    return CG_OK;
}

extern "C" int cg_rast_set_scene(cg_ctx *c, const cg_rtri *room, int n_room, const cg_rtri *boxes, int n_boxes)
{
    if (!c || n_room < 0 || n_boxes < 0 || (n_room && !room) || (n_boxes && !boxes) || n_room + 7 * n_boxes > 4096)
        return CG_E_INVALID;
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    CG_TRY(c, c->rroom.ensure((size_t)(n_room > 0 ? n_room : 1) * sizeof(cg_rtri)), "alloc room");
    CG_TRY(c, c->rboxes.ensure((size_t)(n_boxes > 0 ? n_boxes : 1) * sizeof(cg_rtri)), "alloc boxes");
    if (n_room)
        CG_TRY(c, hipMemcpyAsync(c->rroom.p, room, (size_t)n_room * sizeof(cg_rtri), hipMemcpyHostToDevice, c->stream), "upload room");
    if (n_boxes)
        CG_TRY(c, hipMemcpyAsync(c->rboxes.p, boxes, (size_t)n_boxes * sizeof(cg_rtri), hipMemcpyHostToDevice, c->stream), "upload boxes");
    CG_TRY(c, hipStreamSynchronize(c->stream), "scene upload");
    c->n_room = n_room;
    c->n_boxes = n_boxes;
    c->scene_tex = rast_tex_mask(room, n_room) | rast_tex_mask(boxes, n_boxes);
    ++c->scene_gen;
    return CG_OK;
}

extern "C" int cg_rast_draw_frames_device(cg_ctx *c, const cg_rast_params *ps, int n_frames, uint32_t *d_argb,
                                          float *d_depth, int32_t *d_shadow, size_t frame_stride, void *stream)
{
    if (!c || n_frames < 0 || (n_frames && (!ps || !d_argb))) return CG_E_INVALID;
    if (c->n_room < 0) {
        c->err = "draw before cg_rast_set_scene";
        return CG_E_NOSCENE;
    }
    if (n_frames == 0) return CG_OK;
    const size_t px = (size_t)ps[0].width * ps[0].height;
    const size_t stride = frame_stride ? frame_stride : px;
    for (int f = 0; f < n_frames; ++f)
        if (ps[f].colour_mode != 0 || ps[f].width != ps[0].width || ps[f].height != ps[0].height || stride < px)
            return ctx_invalid(c, "draw_frames: colour mode 0 frames of one size (modes 1-2 chain rand offsets)");
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    // lanes in flight (CG_RAST_LANES for A/B runs): 6 -- C3 1080p, 64 frames per call, round 6:
    // 2 lanes 21.3-21.4k frames/s, 3 18.0k, 4 21.2k, 5 22.6-22.7k, 6 23.1-23.3k, 7 20.7-20.9k,
    // 8 21.3-22.4k (profiles/r06_ab_session2.json; round 1 had found 2 best).  The lanes' streams
    // share the process's 4 hardware queues, so the count sets how the frames' latency-bound
    // kernels interleave; 6 was best both alone and inside the default bench line
    static const int lanes = [] {
        const char *e = std::getenv("CG_RAST_LANES");
        const int v = e ? std::atoi(e) : 6;
        return std::max(1, std::min(v, (int)cg_ctx::kRastLanes));
    }();
    const int L = std::min(lanes, n_frames);
    if (!c->start_ev) CG_TRY(c, hipEventCreateWithFlags(&c->start_ev, hipEventDisableTiming), "event");
    for (int k = 0; k < L; ++k) {
        if (!c->lanes[k]) {
            int rc = cg_create(c->device, &c->lanes[k]);
            if (rc) return ctx_invalid(c, "lane context");
            c->lanes[k]->tex_owner = c;
            CG_TRY(c, hipEventCreateWithFlags(&c->lane_ev[k], hipEventDisableTiming), "event");
            c->lane_gen[k] = c->scene_gen - 1;
        }
        cg_ctx *l = c->lanes[k];
        if (c->lane_gen[k] != c->scene_gen) {   // the parent's scene, device to device
            CG_TRY(c, l->rroom.ensure(c->rroom.bytes), "alloc lane room");
            CG_TRY(c, l->rboxes.ensure(c->rboxes.bytes), "alloc lane boxes");
            CG_TRY(c, hipMemcpyAsync(l->rroom.p, c->rroom.p, c->rroom.bytes, hipMemcpyDeviceToDevice, c->stream),
                   "lane scene");
            CG_TRY(c, hipMemcpyAsync(l->rboxes.p, c->rboxes.p, c->rboxes.bytes, hipMemcpyDeviceToDevice, c->stream),
                   "lane scene");
            CG_TRY(c, hipStreamSynchronize(c->stream), "lane scene");
            l->n_room = c->n_room;
            l->n_boxes = c->n_boxes;
            l->scene_tex = c->scene_tex;
            c->lane_gen[k] = c->scene_gen;
        }
    }
    CG_TRY(c, hipEventRecord(c->start_ev, st), "event");
    for (int k = 0; k < L; ++k) CG_TRY(c, hipStreamWaitEvent(c->lanes[k]->stream, c->start_ev, 0), "lane wait");
    for (int f = 0; f < n_frames; ++f) {
        cg_ctx *l = c->lanes[f % L];
        const size_t o = (size_t)f * stride;
        int rc = rast_draw_device(l, (const cg_rtri *)l->rroom.p, l->n_room, (const cg_rtri *)l->rboxes.p, l->n_boxes,
                                  &ps[f], d_argb + o, d_depth ? d_depth + o : nullptr, d_shadow ? d_shadow + o : nullptr,
                                  l->stream, nullptr, nullptr, l->scene_tex);
        if (rc) {
            c->err = std::string("lane: ") + l->err;
            return rc;
        }
    }
    for (int k = 0; k < L; ++k) {
        CG_TRY(c, hipEventRecord(c->lane_ev[k], c->lanes[k]->stream), "event");
        CG_TRY(c, hipStreamWaitEvent(st, c->lane_ev[k], 0), "lane join");
    }
    return CG_OK;
}

extern "C" int cg_rast_opacity_map(const uint8_t *bgr, int n, uint8_t *out)
{
    if (n < 0 || (n && (!bgr || !out))) return CG_E_INVALID;
    for (int i = 0; i < n; ++i) {   // RGB2Gray<uchar> (blueIdx 0), then threshold(100, 255, BINARY)
        const int y = (bgr[3 * i] * 1868 + bgr[3 * i + 1] * 9617 + bgr[3 * i + 2] * 4899 + (1 << 13)) >> 14;
        out[i] = y > 100 ? 255 : 0;
    }
    return CG_OK;
}

extern "C" int cg_rast_set_textures(cg_ctx *c, const cg_rast_textures *t)
{
    if (!c) return CG_E_INVALID;
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    CG_TRY(c, hipStreamSynchronize(c->stream), "sync");
    DevBuf *all[] = {&c->tmarble, &c->tnoise, &c->twoven, &c->twoven_ao, &c->twoven_op, &c->twoven_nrm,
                     &c->tgrill, &c->tgrill_op, &c->tgrill_nrm};
    for (DevBuf *b : all) b->release();
    c->tex_loaded = 0;
    if (!t) return CG_OK;
    const size_t tn = (size_t)kTexN * kTexN, mn = (size_t)kMarbleN * kMarbleN;
    auto up = [&](DevBuf &b, const void *src, size_t bytes) -> int {
        CG_TRY(c, b.ensure(bytes), "alloc texture");
        CG_TRY(c, hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice), "upload texture");
        return CG_OK;
    };
    auto up_op = [&](DevBuf &b, const uint8_t *bgr) -> int {   // skeleton.cpp:149-155
        std::vector<uint8_t> op(tn);
        cg_rast_opacity_map(bgr, (int)tn, op.data());
        return up(b, op.data(), tn);
    };
    int rc = 0;
    if (t->grill && t->grill_opacity && t->grill_normal) {
        if ((rc = up(c->tgrill, t->grill, 3 * tn)) || (rc = up_op(c->tgrill_op, t->grill_opacity)) ||
            (rc = up(c->tgrill_nrm, t->grill_normal, 3 * tn)))
            return rc;
        c->tex_loaded |= 1 << 2;
    }
    if (t->woven && t->woven_ao && t->woven_opacity && t->woven_normal) {
        if ((rc = up(c->twoven, t->woven, 3 * tn)) || (rc = up(c->twoven_ao, t->woven_ao, 3 * tn)) ||
            (rc = up_op(c->twoven_op, t->woven_opacity)) || (rc = up(c->twoven_nrm, t->woven_normal, 3 * tn)))
            return rc;
        c->tex_loaded |= 1 << 3;
    }
    if (t->marble) {
        // normalMap_marble (:158-170): the process's first 3 * 2000 * 2000 rand() calls
        std::vector<int32_t> r(3 * mn);
        if ((rc = cg_glibc_rand(0, (int)r.size(), r.data()))) return rc;
        std::vector<float> noise(3 * mn);
        const float LO = -0.000002f, HI = 0.000002f;
        for (size_t i = 0; i < r.size(); ++i) noise[i] = LO + (float)r[i] / ((float)((float)RAND_MAX / HI - LO));
        if ((rc = up(c->tmarble, t->marble, 3 * mn)) || (rc = up(c->tnoise, noise.data(), noise.size() * 4))) return rc;
        c->tex_loaded |= 1 << 1;
    }
    return CG_OK;
}

extern "C" int cg_rast_draw_device(cg_ctx *c, const cg_rast_params *p, uint32_t *d_argb, float *d_depth,
                                   int32_t *d_shadow, void *stream)
{
    if (!c || !p || !d_argb) return CG_E_INVALID;
    if (c->n_room < 0) {
        c->err = "draw before cg_rast_set_scene";
        return CG_E_NOSCENE;
    }
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    return rast_draw_device(c, (const cg_rtri *)c->rroom.p, c->n_room, (const cg_rtri *)c->rboxes.p, c->n_boxes, p,
                            d_argb, d_depth, d_shadow, stream ? (hipStream_t)stream : c->stream, nullptr, nullptr,
                            c->scene_tex);
}

extern "C" int cg_rast_draw(cg_ctx *c, const cg_rast_params *p, uint32_t *argb, float *depth, int32_t *shadow,
                            cg_stats *stats)
{
    if (!c || !p || !argb || p->width <= 2 || p->height <= 2) return CG_E_INVALID;
    if (c->n_room < 0) {
        c->err = "draw before cg_rast_set_scene";
        return CG_E_NOSCENE;
    }
    auto t0 = std::chrono::steady_clock::now();
    CG_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    size_t npx = (size_t)p->width * p->height;
    hipError_t e;
    uint32_t *d_argb = (uint32_t *)ctx_buf(c, 4, npx * 4, &e);
    if (!d_argb) return ctx_fail(c, e, "alloc argb");
    float *d_depth = (float *)ctx_buf(c, 5, npx * 4, &e);
    if (!d_depth) return ctx_fail(c, e, "alloc depth");
    int32_t *d_shadow = (int32_t *)ctx_buf(c, 6, npx * 4, &e);
    if (!d_shadow) return ctx_fail(c, e, "alloc shadow");
    int *d_n = nullptr;
    int rc = rast_draw_device(c, (const cg_rtri *)c->rroom.p, c->n_room, (const cg_rtri *)c->rboxes.p, c->n_boxes, p,
                              d_argb, d_depth, d_shadow, c->stream, stats, &d_n, c->scene_tex);
    if (rc) return rc;
    int n = 0;
    CG_TRY(c, hipMemcpyAsync(&n, d_n, sizeof(int), hipMemcpyDeviceToHost, c->stream), "d2h count");
    CG_TRY(c, hipMemcpyAsync(argb, d_argb, npx * 4, hipMemcpyDeviceToHost, c->stream), "d2h argb");
    if (depth) CG_TRY(c, hipMemcpyAsync(depth, d_depth, npx * 4, hipMemcpyDeviceToHost, c->stream), "d2h depth");
    if (shadow) CG_TRY(c, hipMemcpyAsync(shadow, d_shadow, npx * 4, hipMemcpyDeviceToHost, c->stream), "d2h shadow");
    CG_TRY(c, hipStreamSynchronize(c->stream), "rast frame");
    if (stats) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
        stats->kernel_ms = ms;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        stats->n_tris = n;
    }
    return CG_OK;
}
