/*
 * cg_render.h -- C-ABI of the MI355X-native renderer (gfx950 HIP kernels).
 *
 * This is the drop-in boundary for the two pixel-loop hot paths of
 * fznsakib/Computer-Graphics.  The reference has no plugin/FFI API: its hot
 * paths sit behind `void Draw(screen*)`, which reads mutable globals and
 * writes ARGB pixels into the caller-owned `screen->buffer`.
 * The host surface in computer-graphics_amd/host/ keeps that exact shape
 * (same Draw(screen*), same globals, same Triangle/Sphere/Intersection/Light
 * structs, same PutPixelSDL pixel layout) and calls the entry points below.
 *
 * Conventions: plain pointers and sizes only; POD structs with the
 * reference's field order; every call returns 0 (CG_OK) or a negative
 * CG_E* code and never throws across the ABI.  A context is bound to one
 * GPU and is not thread-safe (one host thread per context, like the
 * reference's single main thread).  Host buffers are caller-owned; device
 * buffers are context-owned unless a *_device entry point is given a
 * caller-owned device pointer.  `stream` arguments are hipStream_t values
 * (NULL = the context's own stream).
 */
#ifndef CG_RENDER_H
#define CG_RENDER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CG_OK 0
#define CG_E_INVALID (-1)     /* bad argument / shape */
#define CG_E_NODEVICE (-2)    /* no HIP device / HIP init failed */
#define CG_E_HIP (-3)         /* HIP runtime error (see cg_last_error) */
#define CG_E_NOSCENE (-4)     /* render before cg_rt_set_scene */
#define CG_E_CAPACITY (-5)    /* output capacity too small */
#define CG_E_TIMEOUT (-6)     /* multi-GPU: a peer did not answer within the deadline (communicator aborted) */

typedef struct cg_ctx cg_ctx;

typedef struct { float x, y, z; } cg_vec3;
typedef struct { float x, y, z, w; } cg_vec4;

/* raytracer/Source/TestModelH.h:80-115 `Triangle` (76 B: v0@0 v1@16 v2@32 normal@48 color@64). */
typedef struct { cg_vec4 v0, v1, v2, normal; cg_vec3 color; } cg_tri;
/* raytracer/Source/TestModelH.h:14-22 `Sphere` (44 B). */
typedef struct { float radius, radiusSquared; cg_vec3 centre, color, normal; } cg_sphere;
/* raytracer/Source/skeleton.cpp:47-50 `Light` (28 B). */
typedef struct { cg_vec4 position; cg_vec3 colour; } cg_light;
/* raytracer/Source/skeleton.cpp:40-45 `Intersection` (28 B). */
typedef struct { cg_vec4 position; float distance; int triangleIndex; int sphereIndex; } cg_isect;

/* The RT globals Draw reads (raytracer/Source/skeleton.cpp:56-60, :110). */
typedef struct {
    int width, height;     /* SCREEN_WIDTH / SCREEN_HEIGHT (:19-20) */
    float focal;           /* focalLength (:56) */
    cg_vec4 camera;        /* cameraPos (:57) */
    float R[16];           /* R (:60), glm::mat4 column-major: R[c*4+r] */
    float indirect;        /* indirectLight scale (:110), 0.5 */
} cg_rt_camera;

/* Row sharding for the multi-GPU path.  Stripes (rows == 0): stripes of
 * `stripe_h` rows are dealt round-robin over `nranks`; this rank renders
 * stripes k with k % nranks == rank, packed in order into its output.  Any
 * stripe_h >= 1 is exact; for speed use a multiple of 15 for a one-light
 * camera that is unrotated or only yawed, or an unrotated light set (the
 * lattice kernels' tile height), and of 8 otherwise.
 * Band (rows > 0): this shard renders frame rows row0 .. row0 + rows - 1
 * (rows past the frame are padding); rank / nranks / stripe_h are ignored.
 * Window (cols > 0, CG_PIX_RGB24 output only): only columns col0 .. col0 +
 * cols - 1 are stored, rows `cols` pixels apart -- the caller asserts the other
 * columns are black (cg_rt_frame_columns); col0 and cols are multiples of 16
 * (cols may end at the frame's right edge). */
typedef struct { int rank, nranks, stripe_h; int row0, rows; int col0, cols; } cg_rt_shard;

/* Pixel formats of device outputs.  ARGB8888 is PutPixelSDL's uint32
 * (SDLauxiliary.h:149-161).  RGB24 is its wire form for transfers between
 * GPUs: the low three bytes (B, G, R) of each pixel, 3 bytes per pixel --
 * PutPixelSDL's alpha is always 128, so cg_rt_assemble_device restores the
 * exact uint32. */
#define CG_PIX_ARGB8888 0
#define CG_PIX_RGB24 1

/* rasteriser/Source/TestModelH.h:13-42 `Triangle` (84 B). */
typedef struct { cg_vec4 v0, v1, v2, normal; cg_vec3 color; int texture; int index; } cg_rtri;

/* The RAST globals Draw reads (rasteriser/Source/skeleton.cpp:30-86). */
typedef struct {
    int width, height;        /* SCREEN_WIDTH / SCREEN_HEIGHT (:21-22) */
    float focal;              /* focalLength (:30) */
    cg_vec4 camera;           /* cameraPos (:31) */
    float R[16];              /* R (:35) */
    cg_vec4 light_scene;      /* sceneCoordinatesLightPos (:52) */
    cg_vec3 light_power;      /* lightPower (:53) */
    float indirect_first;     /* indirectLightPowerPerArea at frame start (:54, :581-585):
                                 0.15 on the very first frame, 0.2 after the first
                                 colour-mode-0 fragment was shaded */
    int colour_mode;          /* randColourSelect (:81, SPACE key :408): 0 lit triangle colour,
                                 1 random colour, 2 night vision (:647-662) */
    float yaw;                /* yaw (:34): findU/findV (:1756-1825) map through inverse(R)
                                 when it is non-zero (texture modes 1-3 only) */
    uint64_t rand_offset;     /* modes 1-2: glibc rand() calls made before this frame (the
                                 reference never seeds: srand(1)); each shaded fragment
                                 consumes 3 (cg_stats.n_shaded) */
} cg_rast_params;

typedef struct {
    double kernel_ms;        /* device time of the frame's kernels (HIP events) */
    double total_ms;         /* host wall time of the call */
    int n_tris;              /* triangles rendered (RAST: after clipping) */
    int n_spans;             /* RAST: row spans produced by span setup */
    long long n_shaded;      /* RAST colour modes 1-2: fragments shaded (rand() calls / 3); -1 otherwise */
} cg_stats;

/* ---- context ---------------------------------------------------------- */
int  cg_create(int device, cg_ctx **out);
void cg_destroy(cg_ctx *ctx);
const char *cg_last_error(const cg_ctx *ctx);
/* Number of visible HIP devices (0 without a GPU); never fails loudly. */
int  cg_device_count(void);

/* ---- raytracer -------------------------------------------------------- */
/* LoadTestModel (raytracer/Source/TestModelH.h:121-279): 28 triangles +
 * one sphere, scaled to [-1,1]^3.  Returns the triangle count. */
int cg_rt_load_test_model(cg_tri *tris, int cap, cg_sphere *sphere);
/* Build-defined workloads of SURVEY.md 8d (not in the reference; host-only,
 * no device work).  C4: n x n point lights at the cell centres of a square of
 * side `side` in the xz-plane centred on *centre, each with colour/(n*n);
 * light (i, j) -> out[j*n + i], x = c.x + side*(((float)i + 0.5f)/n - 0.5f),
 * z likewise with j.  Returns n*n.  C5: n random triangles from PCG32
 * (seed, stream 54): centroid ~ U[-1,1]^3, each vertex = centroid +
 * U[-0.02,0.02]^3, colour ~ U[0.15,0.75]^3, w = 1, normal by ComputeNormal
 * (TestModelH.h:96-105).  Returns n. */
int cg_rt_area_lights(const cg_light *centre, float side, int n, cg_light *out, int cap);
int cg_rt_random_scene(uint64_t seed, int n, cg_tri *out);
/* Upload the scene LoadTestModel built (TestModelH.h:121-279); kept device
 * resident until the next call.  Replaces the per-frame `vector<Triangle>`
 * the reference rebuilds in Draw (skeleton.cpp:113-116). */
int cg_rt_set_scene(cg_ctx *ctx, const cg_tri *tris, int n_tris,
                    const cg_sphere *spheres, int n_spheres);
/* One frame of raytracer Draw (skeleton.cpp:104-169): per pixel 3x3
 * sub-rays, ClosestIntersection (:263-363) and DirectLight (:366-415),
 * PutPixelSDL packing (SDLauxiliary.h:149-161).  Writes W*H ARGB into the
 * caller-owned host buffer `argb` (row-major, top row first), exactly what
 * the reference leaves in screen->buffer. */
int cg_rt_render(cg_ctx *ctx, const cg_light *lights, int n_lights, const cg_rt_camera *cam,
                 uint32_t *argb, cg_stats *stats);   /* 0 <= n_lights <= 4096 */
/* n_frames successive Draw()s into caller-owned HOST memory (pageable, as
 * screen->buffer, or pinned): frame f with camera cams[f] at argb + f *
 * frame_stride pixels (0 = W*H), each what cg_rt_render leaves.  The frames
 * render `chunk` at a time (0 = 8) through cg_rt_render_frames_device into
 * device slots while the previous chunk downloads on a second stream (the
 * main loop of skeleton.cpp:91-94 with the D2H of frame N overlapped with
 * the render of later frames).  Returns once every frame is in host memory;
 * stats->kernel_ms spans the renders, total_ms the call. */
int cg_rt_render_frames(cg_ctx *ctx, const cg_light *lights, int n_lights, const cg_rt_camera *cams,
                        int n_frames, uint32_t *argb, size_t frame_stride, int chunk, cg_stats *stats);
/* Device-resident form: renders this shard's rows into the caller-owned
 * device buffer d_out (cg_rt_shard_rows() rows of W pixels), enqueued on
 * `stream`, no synchronisation.  shard may be NULL (= whole frame). */
int cg_rt_render_device(cg_ctx *ctx, const cg_light *lights, int n_lights, const cg_rt_camera *cam,
                        const cg_rt_shard *shard, uint32_t *d_out, void *stream);
/* n_frames successive frames (the reference's main loop: Update() moves the
 * camera, Draw() renders, raytracer/Source/skeleton.cpp:91-94 + :104-169),
 * frame f with camera cams[f] into d_out + f * frame_stride pixels
 * (frame_stride 0 = cg_rt_shard_rows() * W) in pix_format (CG_PIX_*; for
 * RGB24, d_out is a byte buffer and pixel offsets count 3 bytes).  All
 * cameras share width and height; lights and the shard are common.  Frames of
 * the unrotated one-light camera that differ only in cameraPos are rendered up
 * to 32 per kernel launch (a whole GPU's worth of tiles even for a small
 * shard); others are enqueued one by one.  Each frame equals
 * cg_rt_render_device's. */
int cg_rt_render_frames_device(cg_ctx *ctx, const cg_light *lights, int n_lights, const cg_rt_camera *cams,
                               int n_frames, const cg_rt_shard *shard, void *d_out, size_t frame_stride,
                               int pix_format, void *stream);
/* Frame assembly after a transfer of band shards: d_src holds n_blocks row
 * blocks in order, block b = n_frames x rows[b] rows of `width` pixels in
 * pix_format, landing at frame rows row0[b] .. row0[b] + rows[b] - 1 (rows
 * outside the frame are skipped) of frame f = d_frames + f * frame_stride
 * pixels (ARGB8888).  With cols > 0 the source rows hold only the window
 * columns col0 .. col0 + cols - 1 (4-aligned) and the rest of each row is set
 * to 0x80000000.  row0 / rows are host arrays, n_blocks <= 64. */
int cg_rt_assemble_device(cg_ctx *ctx, const void *d_src, int pix_format, const int *row0, const int *rows,
                          int n_blocks, int width, int height, int n_frames, uint32_t *d_frames,
                          size_t frame_stride, int col0, int cols, void *stream);
/* The columns an unrotated camera can see anything in: every sub-ray of the
 * pixels outside [*col0, *col1) certainly misses all triangles and spheres,
 * so those pixels are PutPixelSDL(0, 0, 0) = 0x80000000 (skeleton.cpp:160-166).
 * From the scene's bounding box widened by 0.02 (every accepted float hit
 * lies within ~1e-6 relative of its triangle and within 4e-3 |cameraPos -
 * centre| of its sphere), projected through the pinhole (the projection of a
 * box in front of the camera lies in the hull of its corners' projections),
 * plus 2 pixels, rounded out to 16-pixel boundaries.  Returns the full width
 * for rotated cameras or when the box reaches behind the camera.  Host-only
 * (no device work), usable to crop CG_PIX_RGB24 transfers (cg_rt_shard). */
int cg_rt_frame_columns(const cg_tri *tris, int n_tris, const cg_sphere *spheres, int n_spheres,
                        const cg_rt_camera *cam, int *col0, int *col1);
/* Rows a shard renders (including padding rows of its last stripe). */
int cg_rt_shard_rows(int height, const cg_rt_shard *shard);
/* Which kernels a frame of this shape takes (host-only, no device work):
 * CG_RT_ROUTE_* below, or CG_E_INVALID.  The lattice kernels share sub-rays
 * between pixels (half-pixel columns for an unrotated camera, per-pixel
 * columns with shared rows under a yaw); the large-scene path (n_tris > 64)
 * has the same two lattice modes and a per-pixel mode.  Every route gives
 * the reference's image; this only says how. */
enum {
    CG_RT_ROUTE_PIXEL = 0,            /* rt_pixel_kernel: 9 sub-rays per pixel */
    CG_RT_ROUTE_LATTICE = 1,          /* rt_lattice_kernel, one light */
    CG_RT_ROUTE_LATTICE_YAW = 2,      /* the same, per-pixel columns */
    CG_RT_ROUTE_LIGHTS = 3,           /* rt_lattice_lights_kernel, 2..64 lights */
    CG_RT_ROUTE_LIGHTS_YAW = 4,
    CG_RT_ROUTE_BIG_PIXEL = 5,        /* large scene, per-pixel mode */
    CG_RT_ROUTE_BIG_LATTICE = 6,      /* large scene, lattice mode */
    CG_RT_ROUTE_BIG_LATTICE_YAW = 7
};
int cg_rt_route(const cg_rt_camera *cam, int n_tris, int n_spheres, int n_lights, const cg_rt_shard *shard);
/* Reassemble a frame from gathered shards: d_gathered holds nranks blocks of
 * cg_rt_shard_rows() rows each, in rank order. */
int cg_rt_unstripe_device(cg_ctx *ctx, const uint32_t *d_gathered, int width, int height,
                          int nranks, int stripe_h, uint32_t *d_frame, void *stream);
/* Batched form: d_gathered holds, per rank in rank order, `nframes` shards of
 * cg_rt_shard_rows() rows each (frame-major); d_frames receives nframes
 * frames of W*H.  Lets a caller gather several frames per collective. */
int cg_rt_unstripe_batch_device(cg_ctx *ctx, const uint32_t *d_gathered, int width, int height,
                                int nranks, int stripe_h, int nframes, uint32_t *d_frames, void *stream);
/* Single-ray probes for known-answer tests: device evaluation of
 * ClosestIntersection (:263-363) and DirectLight (:366-415) on n rays. */
int cg_rt_probe_closest(cg_ctx *ctx, const cg_vec4 *starts, const cg_vec4 *dirs, int n,
                        cg_isect *out, int *hit);
int cg_rt_probe_direct_light(cg_ctx *ctx, const cg_isect *isects, const cg_light *light, int n,
                             cg_vec3 *out);
/* DirectLight's three divides by one area (:412) as the light-set sweep performs
 * them (a shared reciprocal inside a range guard, IEEE x / d outside it), on
 * device arrays: d_q[3i + k] = d_x[3i + k] / d_den[i]; a test that they are
 * IEEE-exact. */
int cg_rt_probe_div3_device(const float *d_x, const float *d_den, int n, float *d_q, void *stream);
/* Test hook for large scenes (n_tris > 64): capacity of the device queue of
 * shadow rays the blocker hints leave to the certified lit search (0 = the
 * default, 65536).  Rays past the queue are searched per pixel by the shading
 * kernel instead; the image is the same either way. */
int cg_rt_set_pending_cap(cg_ctx *ctx, int cap);
/* Large-scene scratch after the latest frame (waits for it): out[0] device
 * bytes held, out[1] entries the frame listed in the pools (super-bin, bin,
 * bucketed and shadow lists), out[2] the pools' capacity in entries, out[3]
 * frames that overflowed a pool (rendered correctly through the fallback). */
int cg_rt_scratch_info(cg_ctx *ctx, uint64_t *out);
/* Large-scene list demand of the latest frame, per pool (waits for it): out[0]
 * super-bin lists, out[1] bin lists, out[2] many-light shadow lists, out[3]
 * bucketed (per half-bin) lists, in entries. */
int cg_rt_pool_demand(cg_ctx *ctx, uint64_t *out);
/* Test hook: pin the large-scene pool capacities (entries: super-bin, bin,
 * many-light shadow and bucketed lists; all 0 = automatic sizing).  Lists past a capacity take the fallback over every triangle; the
 * image is the same. */
int cg_rt_set_pool_caps(cg_ctx *ctx, long long sup, long long bin, long long sbin, long long sorted);
/* Test hook, a defect detector for the certificate machinery (never a product
 * path): rows row0 .. row0 + rows - 1 of the camera's frame (rows x width
 * pixels into d_out, device memory) by the reference's own loop with no
 * acceleration at all -- every sub-ray against every triangle and sphere, every
 * shadow ray against every triangle and sphere until its first blocker
 * (raytracer/Source/skeleton.cpp:120-166, 263-415).  Synchronous; at most 64
 * lights.  C5 at 1080p: tens of seconds on one MI355X. */
int cg_rt_render_brute_device(cg_ctx *ctx, const cg_light *lights, int n_lights, const cg_rt_camera *cam,
                              int row0, int rows, uint32_t *d_out, void *stream);

/* ---- multi-GPU raytracer ------------------------------- */
/* One process per GPU.  The reference renders every pixel of Draw
 * (raytracer/Source/skeleton.cpp:104-169) on one CPU thread; pixels are
 * independent, so N GPUs each render one contiguous band of frame rows and
 * rank 0 assembles the frames: ranks > 0 render their band in CG_PIX_RGB24
 * (only the columns the camera can see anything in, cg_rt_frame_columns) and
 * send it to rank 0 with RCCL point-to-point over xGMI (every peer has its own
 * link to rank 0); rank 0 renders its own band straight into the frames and
 * expands the received bands in place (cg_rt_assemble_device).  Frames are
 * processed in chunks: the transfer of chunk j overlaps the render of chunk
 * j + 1.  A cg_dist is bound to one context and is not thread-safe. */
typedef struct cg_dist cg_dist;
typedef struct { char bytes[128]; } cg_dist_id;    /* an RCCL unique id (ncclUniqueId) */
/* Rank 0 creates the id and hands it to every rank (MPI, sockets, ...). */
int cg_dist_unique_id(cg_dist_id *id);
/* Collective over the nranks processes: RCCL communicator on ctx's device.
 * Every host wait of the multi-GPU path is bounded: the communicator is
 * non-blocking, and init, cg_dist_rebalance, cg_dist_last_times, cg_dist_wait
 * and cg_dist_destroy poll completion and the communicator's asynchronous
 * error against a deadline (default: CG_DIST_TIMEOUT_MS from the environment,
 * else 60000 ms).  An RCCL error returns CG_E_HIP and a passed deadline
 * CG_E_TIMEOUT; either aborts the communicator (ncclCommAbort: kernels still
 * waiting on a peer exit) and every later call on the handle fails CG_E_HIP.
 * A missing peer therefore ends the job with an error instead of a hang.
 * The deadline runs from the last progress of a wait (its start, or the
 * latest of its events seen complete), but one event covers everything queued
 * before it: cg_dist_wait's deadline must exceed the rank's queued backlog.
 * If the abort itself does not return within 10 s it is left running and
 * cg_dist_destroy deliberately leaks the handle's device buffers and transfer
 * stream (RCCL kernels may still be using them). */
int cg_dist_create(cg_ctx *ctx, int nranks, int rank, const cg_dist_id *id, cg_dist **out);
/* cg_dist_create with an explicit deadline in ms (0: the default above). */
int cg_dist_create_timed(cg_ctx *ctx, int nranks, int rank, const cg_dist_id *id, int timeout_ms, cg_dist **out);
/* Deadline (ms, > 0) of every later host wait on this handle. */
int cg_dist_set_timeout(cg_dist *d, int timeout_ms);
/* Bounded host wait until this rank's work of its calls so far has drained:
 * `stream` (NULL: the last call's stream) and the transfer stream.  0, or
 * CG_E_TIMEOUT / CG_E_HIP after aborting the communicator.  Use it instead of
 * an unbounded device synchronise after cg_rt_render_frames_dist. */
int cg_dist_wait(cg_dist *d, void *stream);
/* In-process transport for tests: nranks contexts (any devices, possibly one)
 * in one process and thread, one cg_dist per rank in outs[]; bands move by
 * device-to-device copies.  Each render call must be made on ranks
 * nranks-1 .. 1 before rank 0 (their work is only enqueued). */
int cg_dist_create_local(cg_ctx *const *ctxs, int nranks, cg_dist **outs);
void cg_dist_destroy(cg_dist *d);
/* Band partition: rank r renders rows row0[r] .. row0[r] + rows[r] - 1; the
 * bands must tile [0, height) in rank order.  Default (and after a height
 * change): equal bands on multiples of 15 rows (the lattice tile height). */
int cg_dist_set_bands(cg_dist *d, int height, const int *row0, const int *rows);
int cg_dist_get_bands(const cg_dist *d, int *row0, int *rows);
/* Frames per chunk of the render/transfer pipeline (default 4). */
int cg_dist_set_chunk(cg_dist *d, int frames);
/* Pipeline: CG_DIST_SIGNALLED (the default where the device supports stream
 * waits on memory) renders a call's frames in full-size launches and sends
 * each chunk when its frames' tiles are all stored (per-frame completion
 * counts); CG_DIST_CHUNKED launches each chunk separately and orders the
 * transfers with events. */
#define CG_DIST_SIGNALLED 0
#define CG_DIST_CHUNKED 1
int cg_dist_set_pipeline(cg_dist *d, int mode);
/* Collective: new bands from every rank's measured render time per frame in
 * its last cg_rt_render_frames_dist call (cost density uniform within each
 * old band; rank 0 also pays the assembly), so the bands take equal time. */
int cg_dist_rebalance(cg_dist *d);
/* This rank's device time per frame in its last cg_rt_render_frames_dist
 * call (waits for it): its band's render and, on rank 0, the assembly. */
int cg_dist_last_times(cg_dist *d, double *render_ms_per_frame, double *assemble_ms_per_frame);
/* Collective: n_frames frames (cams as cg_rt_render_frames_device; one size),
 * assembled on rank 0 into d_frames + f * frame_stride pixels (ARGB8888;
 * frame_stride 0 = W*H).  d_frames is ignored on ranks > 0.  Enqueued on
 * `stream` (NULL: the context's); when `stream` has drained, rank 0's frames
 * are complete. */
int cg_rt_render_frames_dist(cg_dist *d, const cg_light *lights, int n_lights, const cg_rt_camera *cams,
                             int n_frames, uint32_t *d_frames, size_t frame_stride, void *stream);
/* Host-only: contiguous bands minimising max_r (sum of row_cost over band r
 * + overhead[r]) (overhead may be NULL); every rank gets >= 1 row when
 * height >= nranks. */
int cg_dist_band_partition(const double *row_cost, int height, int nranks, const double *overhead, int *row0,
                           int *rows);

/* ---- rasteriser ------------------------------------------------------- */
/* glibc rand() as colour modes 1-2 consume it (seed 1, never reseeded by the
 * reference): n values starting at call index `offset`.  Host-only probe of
 * the generator the device path uses (jump-ahead restatement of glibc's
 * TYPE_3 random_r). */
int cg_glibc_rand(uint64_t offset, int n, int32_t *out);
/* LoadTestModel (rasteriser/Source/TestModelH.h:48-312) with texture
 * selectors 0: room (10) and boxes (20). Returns n_room + n_boxes. */
int cg_rast_load_test_model(cg_rtri *room, int room_cap, int *n_room, cg_rtri *boxes,
                            int boxes_cap, int *n_boxes);
/* Host geometry of rasteriser Draw (skeleton.cpp:205-241): camera space
 * (:701-716), createShadowVolume (:1676-1722), rotation by R (:223-228),
 * clip space w = z/f (:691-699), clip planes 1..6 (:720-1673).  Writes the
 * ordered clipped triangle list (up to `cap`) and the rotated camera-space
 * light; returns the triangle count (may exceed cap: CG_E_CAPACITY is not
 * raised, the caller re-sizes) or a negative error. */
int cg_rast_prepare(const cg_rast_params *p, const cg_rtri *room, int n_room,
                    const cg_rtri *boxes, int n_boxes, cg_rtri *out, int cap,
                    cg_vec4 *light_out);
/* One frame of the rasteriser fill + post-pass (skeleton.cpp:243-307):
 * DrawPolygon / VertexShader / ComputePolygonRows / DrawPolygonRows /
 * Interpolate / PixelShader / calculateIllumination over the ordered list,
 * then surroundingShadowSum + antiAliasing + PutPixelSDL.  Outputs are
 * caller-owned host buffers of W*H (any may be NULL except argb):
 * argb = screen->buffer, depth = depthBuffer, shadow = shadowBuffer. */
int cg_rast_render(cg_ctx *ctx, const cg_rtri *tris, int n, const cg_rast_params *p,
                   cg_vec4 light, uint32_t *argb, float *depth, int32_t *shadow,
                   cg_stats *stats);
/* Device-resident form: triangles already on the device (d_tris), outputs
 * into caller-owned device buffers (d_depth / d_shadow may be NULL). */
int cg_rast_render_device(cg_ctx *ctx, const cg_rtri *d_tris, int n, const cg_rast_params *p,
                          cg_vec4 light, uint32_t *d_argb, float *d_depth, int32_t *d_shadow,
                          void *stream);

/* Whole rasteriser Draw on the device (skeleton.cpp:203-308): upload the
 * LoadTestModel room/boxes once, then each frame runs the geometry
 * (shadow volumes, rotation, clip) AND the fill + post-pass on the GPU --
 * the same lists cg_rast_prepare builds on the host. */
int cg_rast_set_scene(cg_ctx *ctx, const cg_rtri *room, int n_room, const cg_rtri *boxes, int n_boxes);
int cg_rast_draw(cg_ctx *ctx, const cg_rast_params *p, uint32_t *argb, float *depth, int32_t *shadow,
                 cg_stats *stats);
int cg_rast_draw_device(cg_ctx *ctx, const cg_rast_params *p, uint32_t *d_argb, float *d_depth,
                        int32_t *d_shadow, void *stream);
/* n_frames whole Draws (colour mode 0, one size; each frame its own params --
 * camera, light, R, first-frame indirect) into frame f at d_argb + f *
 * frame_stride pixels (0: W*H), likewise d_depth / d_shadow (may be NULL).
 * The frames overlap on internal streams (the reference's main loop draws
 * them one after another; frames are independent given their params);
 * `stream` waits for all of them.  Colour modes 1-2 chain the rand() offset
 * from frame to frame: use cg_rast_draw_device per frame for those. */
int cg_rast_draw_frames_device(cg_ctx *ctx, const cg_rast_params *ps, int n_frames, uint32_t *d_argb,
                               float *d_depth, int32_t *d_shadow, size_t frame_stride, void *stream);

/* Texture modes 1-3 (skeleton.cpp:588-645; a triangle's `texture` field,
 * TestModelH.h:21: 1 marble, 2 metal grill, 3 woven wood -- set it on the
 * room/boxes lists, as `setting` / `settingBoxes` do, TestModelH.h:9-10).
 * The maps as cv::imread(..., CV_LOAD_IMAGE_UNCHANGED) returns them
 * (:135-146): row-major BGR, 3 bytes per texel; marble 2000 x 2000, the rest
 * 1024 x 1024.  NULL = not loaded; a texture is renderable when all its maps
 * are (marble: marble; grill: grill, grill_opacity, grill_normal; woven: all
 * four woven maps), and rendering a triangle with a texture that is not
 * fails with CG_E_INVALID (the reference reads an empty cv::Mat). */
typedef struct {
    const uint8_t *marble;                                   /* Marble2000x2000.jpg */
    const uint8_t *woven;                                    /* woven1024x1024.jpg */
    const uint8_t *woven_ao;                                 /* Wood_wicker_003_ambientOcclusion.jpg */
    const uint8_t *woven_opacity;                            /* Wood_wicker_003_opacity.jpg */
    const uint8_t *woven_normal;                             /* Wood_wicker_003_normal.jpg */
    const uint8_t *grill;                                    /* Metal_Grill_002_basecolor.jpg */
    const uint8_t *grill_opacity;                            /* Metal_Grill_002_opacity.jpg */
    const uint8_t *grill_normal;                             /* Metal_Grill_002_normal.jpg */
} cg_rast_textures;
/* Upload the maps and build what main() derives from them at start-up
 * (:148-170): the opacity maps (cg_rast_opacity_map) and, with marble, the
 * normal-noise map from the process's first 3 * 2000 * 2000 rand() calls --
 * colour modes 1-2 then start at rand_offset 12,000,000.  NULL unloads. */
int cg_rast_set_textures(cg_ctx *ctx, const cg_rast_textures *tex);
/* Host-only: OpenCV 3.4 cvtColor(CV_BGR2GRAY) on 8-bit BGR (fixed point,
 * 14-bit coefficients) then threshold(100, 255, THRESH_BINARY) (:149-155):
 * n texels in, n bytes (0 or 255) out. */
int cg_rast_opacity_map(const uint8_t *bgr, int n, uint8_t *out);

/* ---- texture loading (rasteriser/Source/skeleton.cpp:135-146) ----------- */
/* The reference loads its maps with cv::imread(path, CV_LOAD_IMAGE_UNCHANGED)
 * (OpenCV 3.4 over IJG libjpeg 9).  These decode a JPEG file's bytes to what
 * that call returns: row-major BGR (3 bytes per pixel; gray for 1-component
 * files), bit-identical to libjpeg 9's islow IDCT with 16x16 scaled chroma.
 * Baseline and progressive Huffman JPEG, 8-bit, 1 or 3 components, 4:4:4 or
 * 4:2:0; anything else is CG_E_INVALID.  Entropy decoding runs on the host,
 * the IDCT and colour conversion on the context's GPU. */
int cg_image_jpeg_info(const uint8_t *data, size_t n, int *width, int *height, int *channels);
/* Host-only: entropy-decode the whole file without a device (0, or CG_E_INVALID
 * for a corrupt or unsupported stream). */
int cg_image_jpeg_check(const uint8_t *data, size_t n);
/* out: caller-owned host buffer of >= width * height * channels bytes (cap). */
int cg_image_decode_jpeg(cg_ctx *ctx, const uint8_t *data, size_t n, uint8_t *out, size_t cap);
/* Same into device memory, enqueued on `stream` (NULL: the context's). */
int cg_image_decode_jpeg_device(cg_ctx *ctx, const uint8_t *data, size_t n, uint8_t *d_out, size_t cap,
                                void *stream);

/* ---- measurement ----------------------------------------------------- */
/* Live device time of the hot kernels: while on, a start / stop HIP event
 * pair rides on each launch's own dispatch (hipExtLaunchKernel) of
 * rt_prepare_kernel, rt_tile_cert_kernel,
 * rt_lattice_units_kernel, rt_lattice_kernel, rt_lattice_lights_kernel,
 * rt_pixel_kernel, rt_big_primary_kernel, rt_shadow_hints_kernel,
 * rast_fill_kernel and rast_post_kernel, on the stream it runs on, plus
 * "rt_big_frame" (a large scene's whole frame: events recorded around it).  cg_kernel_timing(on)
 * resets the totals (process-wide); cg_kernel_time waits for the recorded
 * launches and returns one kernel's summed launch milliseconds, its busy
 * milliseconds (the union of its launches' spans: launches that overlap on
 * two streams count once) and its launch count. */
int cg_kernel_timing(int enable);
int cg_kernel_time(const char *kernel, double *total_ms, double *busy_ms, long long *launches);

/* ---- starfield (starfield/Source/skeleton.cpp) -------------------------- */
/* n stars as (x, y, z) float triples from glibc rand() (:41-46, seed 1). */
int cg_starfield_init(float *stars, int n);
/* Update() (:82-104) for a frame time dt in ms (the reference's float(t2 - t)). */
int cg_starfield_update(float *stars, int n, float dt);
/* Draw() (:66-79): clear, project each star, PutPixelSDL white; W*H ARGB
 * into the caller-owned host buffer. */
int cg_starfield_draw(cg_ctx *ctx, const float *stars, int n, int width, int height, uint32_t *argb);

#ifdef __cplusplus
}
#endif
#endif /* CG_RENDER_H */
