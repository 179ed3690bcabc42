// cg_internal.h -- device-side data layouts shared by the shim and kernels.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cg_render.h"
#include "cg_math.h"

namespace cg {

constexpr int kMaxLights = 4096;   // lights live in a device buffer (scalar loads)
constexpr int kRtTileW = 32;   // RT workgroup: 4 waves, each an 8x8 pixel tile
constexpr int kRtTileH = 8;
constexpr int kRtThreads = 256;
constexpr int kLatTileW = 16, kLatTileH = 15;   // RT lattice kernel tile (cg_rt.hip): 33 x 31 lattice rays
constexpr int kSup = 4;              // lattice super-tile: kSup x kSup tiles (two-level certificates)
constexpr int kMaxFrameBatch = 32;   // frames per batched RT launch (cg_rt_render_frames_device); 16: ~1 % slower on C2

constexpr int kMaxBlocks = 64;       // row blocks of one assembly launch (cg_rt_assemble_device)

// Measured-cost dispatch order of the lattice launch (cg_rt.hip rt_lattice_kernel).
// A launch's frame-0 workgroups record each tile's duration as a cost class
// (heavy first); the next call's certificate launch counting-sorts that
// recording into `flat` (LatFlatten, its first block) and the lattice
// workgroups take tiles in that order -- every frame's heaviest tile first,
// the cheap tiles last, so the launch ends on short workgroups instead of a
// heavy tile's tail.  Only the schedule changes: each workgroup still renders
// one whole (frame, tile), and `flat` is always a permutation of the launch's
// tiles (a counting sort of any recording is), so the image cannot depend on it.
constexpr int kLatClasses = 64;
constexpr int kLatMaxGroups = 32;
struct LatOrder {
    const uint32_t *flat;    // the launch's tiles heavy first (window-relative: by * gx + bx); null: default order
    uint8_t *cost;           // this launch's recording (class per tile of frame 0); null: none
    int ngroups;             // < 0: frame-major (each frame heavy first, frames in turn); >= 0: frames dispatched
                             // in groups (cg_dist chunks), every frame of a group at each tile, heavy first; 0: one group
    uint8_t gs[kLatMaxGroups + 1];   // group starts (frames of the launch), gs[ngroups] = frames
};
struct RtGeo;
struct RtTri;
// Certificates beside the lattice launch instead of before it (one-light
// lattice, whole-frame calls).  The certificate launch (rt_tile_cert_kernel,
// on the auxiliary stream, frame-major) publishes each (frame, super-tile)
// once its 16 tiles' masks and the frame's RtTri are stored: flags[frame *
// units + super-tile] = gen, an agent-scope release.  A lattice workgroup waits
// for its super-tile's word (acquire, bounded by `spin` wall-clock ticks) and
// otherwise -- or with `force`, the test hook -- takes the uncertified path:
// every triangle and sphere is a candidate for its primary and shadow rays (a
// certificate only ever removes candidates that cannot change a pixel, so the
// image is the same) and the workgroup stores the frame's RtTri itself (the
// same values the certificate launch stores).  flags null: the certificates
// completed before the launch (stream order), nothing to wait for.
struct LatReady {
    const uint32_t *flags;   // [frames][units] publication words of the launch's slot
    uint32_t gen;            // this call's generation (words are only ever raised)
    int units, sx;           // super-tiles per frame / per super-tile row
    int force;               // test hook: every workgroup uncertified
    uint32_t spin;           // wall-clock ticks (100 MHz) to wait before taking the uncertified path
    const RtGeo *geo;        // the scene's per-triangle constants (uncertified path)
    RtTri *tc;               // the launch's RtTri (uncertified path: written by the workgroup)
};
struct LatPublish {
    uint32_t *flags;         // null: no publication (certificates complete before the lattice starts)
    uint32_t gen;
    int units;
    int done;                // out (launch_rt_prepare): 1 when the launch publishes (the fused form)
};
struct LatFlatten {
    const uint8_t *cost;     // a recording of the launch's tile geometry
    uint32_t *flat;          // out: its counting sort
    int n;                   // tiles (gx * gy); 0: nothing to do
};

// Row blocks of frames for rt_assemble_kernel: block b is rows[b] rows that
// land at frame rows row0[b] ..; cum = prefix sums of rows.
struct RtBlocks {
    int n, W, H, bpp;
    int wcol0, wcols;   // source rows hold columns wcol0 .. + wcols - 1 (wcols 0: all); the rest is black
    int row0[kMaxBlocks], rows[kMaxBlocks], cum[kMaxBlocks + 1];
};

// cameraPos of each frame of a batched launch (kernarg; blockIdx.z / .y = frame).
struct RtFrameCams {
    float c[kMaxFrameBatch][4];
};

// Per-frame, per-triangle constants of ClosestIntersection for rays that
// start at the camera (skeleton.cpp:279-306).  Every field is computed with
// exactly the reference's float ops, so reusing it across rays is exact:
//   e1 = v1 - v0, e2 = v2 - v0 (:283-284), s = cameraPos - v0 (:296-297),
//   K1 = e1.y*e2.z - e2.y*e1.z   (first cofactor of det(-d, e1, e2))
//   K2 = s.y*e2.z - e2.y*s.z     (first cofactor of det(-d, s, e2))
//   K3 = e1.y*s.z - s.y*e1.z     (first cofactor of det(-d, e1, s))
//   detT = det(s, e1, e2) = (s.x*K1 - e1.x*K2) + e2.x*(s.y*e1.z - e1.y*s.z)
// 64 B per triangle: one s_load_dwordx16 per loop iteration.
struct alignas(16) RtTri {
    float e1x, e1y, e1z, e2x, e2y, e2z;
    float sx, sy, sz, detT;
    float K1, K2, K3;
    float v0x, v0y, v0z;
};
static_assert(sizeof(RtTri) == 64, "RtTri must be 64 B");

// The camera-independent part of RtTri, formed once per scene (rt_scene_kernel
// at cg_rt_set_scene): e1, e2, v0 and K1, the same float ops as RtTri's.  48 B,
// three 16-byte loads, so the per-frame prepare pass streams 48 B in and 64 B
// out per triangle instead of gathering the 76-byte Triangle records.
struct alignas(16) RtGeo {
    float e1x, e1y, e1z, e2x;
    float e2y, e2z, v0x, v0y;
    float v0z, K1, pad0, pad1;
};
static_assert(sizeof(RtGeo) == 48, "RtGeo must be 48 B");

// Shading attributes, read only on a hit.  Camera-independent: written once
// per scene (rt_scene_kernel), shared by every slot and frame.
struct alignas(16) RtShade {
    float nx, ny, nz, nw;   // Triangle::normal (w = 1)
    float cr, cg, cb, pad;  // Triangle::color
};

// Light (skeleton.cpp:47-50), 32 B.
struct alignas(16) RtLight {
    float x, y, z, w;
    float r, g, b, pad;
};

struct RtSphere {
    float cx, cy, cz, r2;   // centre, radiusSquared
    float cr, cg, cb, pad;  // color
};

// Uniform grid over a large scene's triangles: each triangle is listed in
// every cell its bounding box touches (float floor of (x - lo) * inv_h per
// axis, clamped).  Used by the shadow blocker hints and by the certified lit
// search (cg_rt_big.hip).
struct RtGrid {
    float lo[3], inv_h, h;      // cell (i, j, k) spans lo + h * [i, i + 1) x ...
    int res[3];
    const int *start;           // [cells + 1] prefix offsets into tris; null = no grid
    const int *tris;
    float blo[3], bhi[3];       // box of every possible hit position (triangles and spheres)
};

// Pool capacities (entries) of the large-scene path (cg_rt_big.hip): the
// super-bin lists, the bin lists, the many-light shadow lists, the bin
// lists' bucketed half-bin copies.
struct BigCaps {
    long long sup, bin, sbin, sorted;
};

// Frame arguments, passed by value (kernarg -> SGPRs).
struct RtFrame {
    int W, H;
    float focal, indirect;
    float cam[4];
    float R[16];
    int n_tris, n_sph, n_lights;
    int rank, nranks, stripe_h, rows_out;
    int row0;      // first global row (band shards; 0 for stripes): v = row0 + stripe map of L
    int out_fmt;   // CG_PIX_ARGB8888 (uint32 per pixel) or CG_PIX_RGB24 (3 bytes: B, G, R)
    int wcol0, wcols;   // RGB24 output window: columns wcol0 .. wcol0 + wcols - 1 (wcols 0: all)
    int cull_primary, cull_shadow;   // certificates on (always, except inside the probes)
    const RtLight *lights;           // n_lights entries, device memory
    // The light set as the shadow certificate sees it: componentwise min/max
    // of the positions, a centre lc and rho >= max_k |L_k - lc| (FP64, rounded up).
    float lmin[3], lmax[3], lc[3];
    double lrho;
    float nbound;   // >= |component| of every hit normal (triangle normals; spheres <= 1 + 2^-20)
    // Batched lattice launches (cg_rt.hip): workgroups only for tile columns tx0 .. tx0 + txn - 1,
    // the columns the scene's box can be seen in over the batch's cameras; the edge workgroups
    // store the other columns black.  txn 0: every tile column.
    int tx0 = 0, txn = 0;
};

// ---- RAST --------------------------------------------------------------
constexpr int kRastMaxH = 8192;
constexpr int kGeomMaxLeaves = 32;   // clip survivors per input triangle (planes 1-4 and 6 split; 5 never)

// Row span of one triangle (output of ComputePolygonRows, skeleton.cpp:433-498),
// already reduced to what Interpolate (:524-551) needs for DrawPolygonRows:
//   x_i = lx + i, zinv_i = lz + sz*i, X_i = (lX + sX*i)/zinv_i, Y_i likewise,
//   shaded for i in [0, rx - lx).
struct alignas(16) RastSpan {
    int lx, rx;
    float lz, sz;      // left zinv, step_z
    float lX, sX;      // left pos3d.x * zinv, step
    float lY, sY;
};

struct RastTriHdr {
    int ymin, rows;      // rows of this triangle (VertexShader y's), span base offset below
    int span0;           // first span index in the span array
    int pad;
};

// ---- live kernel timing (cg_ktime.hip, cg_kernel_timing) ---------------
enum KtId {
    KT_RT_PREPARE, KT_RT_TILE_CERT, KT_RT_LATTICE_UNITS, KT_RT_LATTICE, KT_RT_LATTICE_LIGHTS, KT_RT_PIXEL,
    KT_RT_BIG_PRIMARY, KT_RT_SHADOW_HINTS, KT_RT_BIG_FRAME, KT_RAST_FILL, KT_RAST_POST, KT_COUNT
};
// HIP events on `st` around the scope's launches while timing is on (id
// outside [0, KT_COUNT): nothing).
class KtScope {
  public:
    KtScope(int id, hipStream_t st);
    ~KtScope();
    KtScope(const KtScope &) = delete;
    KtScope &operator=(const KtScope &) = delete;

  private:
    int id_;
    hipStream_t st_;
    hipEvent_t a_ = nullptr;
};

// One timed launch while timing is on: the start / stop events ride on the
// kernel's own dispatch (hipExtLaunchKernel), so no marker packets sit between
// the launches; a and b are null (a plain launch) while timing is off.
class KtLaunch {
  public:
    KtLaunch(int id, hipStream_t st);
    ~KtLaunch();
    KtLaunch(const KtLaunch &) = delete;
    KtLaunch &operator=(const KtLaunch &) = delete;
    hipEvent_t a = nullptr, b = nullptr;

  private:
    int id_;
    bool ref_ = false;   // a is the session's anchor event
};
template <class K, class... A>
inline void kt_launch(int id, K kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t st, A... args)
{
    KtLaunch t(id, st);
    hipExtLaunchKernelGGL(kernel, grid, block, lds, st, t.a, t.b, 0u, args...);
}

}  // namespace cg
