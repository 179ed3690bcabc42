// cg_rt.hip -- raytracer hot path for gfx950 (MI355X).
//
// One thread per output pixel; a 256-thread workgroup is four waves, each an
// 8x8 pixel tile (coherent rays per wave).  Triangle constants are
// wave-uniform and fetched with scalar loads (one s_load_dwordx16 per
// triangle), so the VALU only sees per-ray work.  Parity with the reference
// CPU render is bit-exact: every float op follows raytracer/Source/
// skeleton.cpp + GLM 0.9.7.2 association, compiled with -ffp-contract=off,
// IEEE div/sqrt and denormals on, FP64 where the reference promotes.
#include <float.h>
#include <stdlib.h>

#include <vector>

#include "cg_rt_dev.h"

namespace cg {

// ---------------------------------------------------------------------------
// Per-frame setup: RtTri constants for camera-origin rays (skeleton.cpp:279-306).
__device__ __forceinline__ RtTri rt_tri_const(const cg_tri &T, float cx, float cy, float cz, float cw)
{
    vec3 e1 = v3(T.v1.x - T.v0.x, T.v1.y - T.v0.y, T.v1.z - T.v0.z);   // :283
    vec3 e2 = v3(T.v2.x - T.v0.x, T.v2.y - T.v0.y, T.v2.z - T.v0.z);   // :284
    vec4 sol = v4(cx, cy, cz, cw) - v4(T.v0.x, T.v0.y, T.v0.z, T.v0.w); // :296
    vec3 s = xyz(sol);
    RtTri r;
    r.e1x = e1.x; r.e1y = e1.y; r.e1z = e1.z;
    r.e2x = e2.x; r.e2y = e2.y; r.e2z = e2.z;
    r.sx = s.x; r.sy = s.y; r.sz = s.z;
    r.detT = det3(s, e1, e2);                                          // :305-306
    r.K1 = e1.y * e2.z - e2.y * e1.z;
    r.K2 = s.y * e2.z - e2.y * s.z;
    r.K3 = e1.y * s.z - s.y * e1.z;
    r.v0x = T.v0.x; r.v0y = T.v0.y; r.v0z = T.v0.z;
    return r;
}

// Lattice geometry (rt_lattice_ok).  R leaves y alone (dir.y = v - H/2 bit
// for bit: mat4_mul adds only +-0 terms) and turns x into a function of x
// alone, so sub-ray (i, j) of pixel (u, v) is (fl(dir.x(u) + 0.5 i), y + 0.5 j,
// focal) (skeleton.cpp:126-137) and the rays of a column of pixels share rows.
//  shared columns (dir.x = x exactly, R the identity): the x values are the
//    half-pixel lattice too, pixel tx's sub-ray i is column 2 tx + 1 + i of
//    2 nu + 1, shared with the neighbours;
//  per-pixel columns (a yaw, :236-238): pixel tx keeps its three columns
//    3 tx + 1 + i of 3 nu, x = fl(dir.x(u) + 0.5 i) formed as the reference
//    forms it -- only the rows are shared (1488 rays for 240 pixels, not 2160).
// dir.x is computed with y = 0: R's y weight is +-0, so y only adds a +-0 term,
// which can change at most the sign of a zero dir.x, and fl(+-0 + 0.5 i) is the
// same for both signs (for i = 0, -0 + +0 = +0).
__host__ __device__ __forceinline__ bool lat_yaw(const RtFrame &F)
{
    return !(F.R[0] == 1.0f && F.R[8] == 0.0f && F.R[12] == 0.0f);
}
__host__ __device__ __forceinline__ float lat_dir_x(const RtFrame &F, int u)
{
    return mat4_mul(F.R, v4((float)(u - F.W / 2), 0.0f, F.focal, 1.0f)).x;   // :126-128
}

// A lattice tile (see rt_lattice_kernel): pixels u0 .. u0 + nu - 1 of rows
// v0 .. v0 + nv - 1 (local rows L0 ..), lattice point (cx, cy) <-> ray
// (lat_x(cx), 0.5 (ay0 + cy), focal), needed points cols x rows.
struct LatTile {
    int u0, L0, v0, nu, nv, ax0, ay0, cols, rows;
    bool yaw;   // per-pixel columns
};
__device__ __forceinline__ LatTile lat_tile(const RtFrame &F, int bx, int by)
{
    LatTile G;
    G.u0 = bx * kLatTileW;
    G.L0 = by * kLatTileH;
    G.v0 = shard_row(F, G.L0);   // the tile's rows v0 .. v0 + 14 lie in one stripe
    G.nu = min(kLatTileW, F.W - G.u0);
    G.nv = max(0, min(min(kLatTileH, F.rows_out - G.L0), F.H - G.v0));
    G.yaw = lat_yaw(F);
    G.ax0 = 2 * (G.u0 - F.W / 2) - 1;
    G.ay0 = 2 * (G.v0 - F.H / 2) - 1;
    G.cols = G.yaw ? 3 * G.nu : 2 * G.nu + 1;
    G.rows = G.nv > 0 ? 2 * G.nv + 1 : 0;
    return G;
}
// x of lattice column cx (the sub-ray's newDir.x, :137)
__device__ __forceinline__ float lat_x(const RtFrame &F, const LatTile &G, int cx)
{
    if (!G.yaw) return 0.5f * (float)(G.ax0 + cx);
    const int p = cx / 3, i = cx - 3 * p - 1;
    return lat_dir_x(F, G.u0 + p) + (0.5f * (float)i);
}
// The x extent [x0, x1] of the sub-rays of tiles A .. B of one tile row.  Per-
// pixel columns: every float op of dir.x(u) is monotone in u, and so is
// fl(d + 0.5 i) in d, so the end pixels' outer sub-rays bound it exactly.
__device__ __forceinline__ void lat_xrange(const RtFrame &F, const LatTile &A, const LatTile &B, float &x0,
                                           float &x1)
{
    if (!A.yaw) {
        x0 = 0.5f * (float)A.ax0;
        x1 = 0.5f * (float)(B.ax0 + B.cols - 1);
        return;
    }
    const float a = lat_dir_x(F, A.u0), b = lat_dir_x(F, B.u0 + B.nu - 1);
    x0 = fminf(a, b) + (0.5f * -1.0f);
    x1 = fmaxf(a, b) + (0.5f * 1.0f);
}

// Tile row of a lattice workgroup: bottom rows first.  Workgroups are
// dispatched x, then y, then frame; the floor and box tiles at the bottom of
// the Cornell frame are the costliest, so starting them first leaves the
// cheap ceiling tiles for the launch's tail.
__device__ __forceinline__ int lat_tile_row() { return (int)(gridDim.y - 1 - blockIdx.y); }
// Tile column of a lattice workgroup (launches over the window RtFrame::tx0 / txn), and the
// frame's full tile-grid width (mask and unit-mask indices).
__device__ __forceinline__ int lat_tile_col(const RtFrame &F) { return F.tx0 + (int)blockIdx.x; }
__host__ __device__ __forceinline__ int lat_tiles_x(const RtFrame &F) { return (F.W + kLatTileW - 1) / kLatTileW; }

#ifdef CG_WG_TIMING
// Diagnostic build only (make OUT=_build_wgt EXTRA=-DCG_WG_TIMING): per-workgroup
// wall-clock stamps (100 MHz) of the certificate and lattice kernels, read by
// scripts/wg_timing.py.  Record: {kind << 56 | z << 40 | y << 20 | x, t0, t1, t2, t3, hardware
// slot << 24 | blockIdx.x}; kind 1
// (certificates) in the first half of the buffer, kind 2 (lattice) in the second, unused
// slots zero.
__device__ unsigned long long *g_wgt;
__device__ unsigned int g_wgt_n, g_wgt_cap;
__device__ __forceinline__ void wgt_record(unsigned long long kind, unsigned long long t0, unsigned long long t1,
                                           unsigned long long t2, unsigned long long t3)
{
    if (threadIdx.x != 0 || !g_wgt) return;
    // a slot per workgroup (no shared counter: its atomics serialised the launch)
    const unsigned s = (kind == 1 ? 0u : g_wgt_cap / 2) +
                       (unsigned)(((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x);
    if (s >= (kind == 1 ? g_wgt_cap / 2 : g_wgt_cap)) return;
    unsigned long long *r = g_wgt + 6ull * s;
    r[0] = kind << 56 | (unsigned long long)blockIdx.z << 40 | (unsigned long long)blockIdx.y << 20 | blockIdx.x;
    r[1] = t0;
    r[2] = t1;
    r[3] = t2;
    r[4] = t3;
    // the hardware slot: XCC_ID (hwreg 20, bits 3:0) and HW_ID (hwreg 4: wave, SIMD, CU, SH, SE)
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20), hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    r[5] = (unsigned long long)xcc << 56 | (unsigned long long)hw << 24 | blockIdx.x;
}
#define WGT_STAMP(v)          \
    __syncthreads();          \
    const unsigned long long v = wall_clock64()
#else
#define WGT_STAMP(v)
#endif

// Certificate units of a frame: tiles, or super-tiles of kSup x kSup tiles.
__host__ __device__ __forceinline__ int rt_cert_units(const RtFrame &F, int sup)
{
    const int tx = (F.W + kLatTileW - 1) / kLatTileW, ty = (F.rows_out + kLatTileH - 1) / kLatTileH;
    return sup ? ((tx + kSup - 1) / kSup) * ((ty + kSup - 1) / kSup) : tx * ty;
}

// Blocks [0, n_prep_blocks): RtTri / RtShade per triangle.  With lat_masks,
// the blocks after them certify the lattice tiles' camera rays (one wave per
// tile, lane k = triangle k, the same certificate as rt_pixel_kernel's over
// the tile's exact lattice box), so the lattice kernel starts from its mask.
// blockIdx.y = frame of a batched launch (camera cams.c[frame]; its RtTri at
// out + frame * n, its masks at lat_masks + frame * tiles).
// Per tile it stores two masks: [0] the primary certificate (bit 63: a
// sphere may be hit), [1] the shadow certificate for every hit the tile's
// rays can produce (primary_hit_box / sphere_hit_box), so the lattice kernel
// needs no certificate pass of its own.
// With sup = 1 the certified units are super-tiles of kSup x kSup tiles (the
// bundle: the box of all their lattice rays) and the masks go to the
// super-tile buffer; rt_tile_cert_kernel then refines them per tile.
__device__ __forceinline__ bool unit_bundle(const RtFrame &F, int unit, int sup, float &x0, float &x1, float &y0,
                                            float &y1)
{
    const int tiles_x = (F.W + kLatTileW - 1) / kLatTileW, tiles_y = (F.rows_out + kLatTileH - 1) / kLatTileH;
    int bx0 = unit, bx1 = unit, by0 = 0, by1 = 0;
    if (sup) {
        const int sx = (tiles_x + kSup - 1) / kSup;
        bx0 = (unit % sx) * kSup;
        bx1 = min(bx0 + kSup, tiles_x) - 1;
        by0 = (unit / sx) * kSup;
        by1 = min(by0 + kSup, tiles_y) - 1;
    } else {
        bx0 = bx1 = unit % tiles_x;
        by0 = by1 = unit / tiles_x;
    }
    const LatTile A = lat_tile(F, bx0, by0), B = lat_tile(F, bx1, by0);
    lat_xrange(F, A, B, x0, x1);
    bool any = false;
    y0 = FLT_MAX;
    y1 = -FLT_MAX;
    for (int by = by0; by <= by1; ++by) {   // rows of a shard need not be contiguous
        const LatTile G = lat_tile(F, bx0, by);
        if (G.rows <= 0) continue;
        any = true;
        y0 = fminf(y0, 0.5f * (float)G.ay0);
        y1 = fmaxf(y1, 0.5f * (float)(G.ay0 + G.rows - 1));
    }
    return any;
}

// The certificates of one unit (a tile, or a super-tile with sup = 1) over
// lpt = 64 / tpw lanes of the calling wave (lane sl = triangle sl, the last
// lane takes the spheres; sub = which of the wave's tpw units): on return the
// unit's primary mask (bit 63: a sphere may be hit) and shadow mask (bit 63:
// a sphere may block a shadow ray), valid in every lane of the unit.  Every
// lane of the wave calls it (ballots, butterflies).
__device__ __forceinline__ void unit_cert(const cg_tri *__restrict__ tris, int n, const float camf[4], const RtFrame &F,
                                          const RtSphere *__restrict__ sph, int unit, int sup, bool tv, int tpw,
                                          unsigned long long &m_out, unsigned long long &sm_out)
{
    const int lane = threadIdx.x & 63, lpt = 64 / tpw;
    const int sub = lane / lpt, sl = lane - sub * lpt;
    float x0, x1, y0, y1;
    const bool act = unit_bundle(F, tv ? unit : 0, sup, x0, x1, y0, y1) && tv;
    bool keep = false, sphere = false;
    RtTri c{};
    LanePosBox pb;   // this lane's share of the unit's possible hit positions
    pb.init();
    PrimDet pd;
    double tlo = 0.0, thi = INFINITY;
    if (act && sl < n) {
        c = rt_tri_const(tris[sl], camf[0], camf[1], camf[2], camf[3]);
        keep = !cull_primary(c, x0, x1, y0, y1, F.focal, &pd);
        if (keep && !primary_t_range(c, pd, tlo, thi)) {
            tlo = 0.0;
            thi = INFINITY;
        }
    }
    // Occlusion: a triangle A that every ray of the tile certainly hits
    // (primary_covers) hides every triangle B whose t certainly exceeds A's:
    // t_B >= tlo_B > thi_A (1 + 2^-18) gives distance_B > distance_A for every
    // ray, so B is never the closest hit (:313 keeps the strictly closer one)
    // and is dropped from the mask and from the box of hit positions.  (The
    // sphere is never dropped: its test compares a parametric t, :348.)
    double occ = (keep && primary_covers(c, pd)) ? thi : INFINITY;
    for (int o = lpt >> 1; o > 0; o >>= 1) occ = fmin(occ, __shfl_xor(occ, o, 64));
    if (keep && tlo > occ * (1.0 + 0x1p-18)) keep = false;
    const cg_tri *Tp = (act && sl < n) ? &tris[sl] : nullptr;
    if (keep && !primary_hit_box(c, pd, camf, x0, x1, y0, y1, F.focal, pb.lo, pb.hi, Tp))
        for (int k = 0; k < 3; ++k) {
            pb.lo[k] = -INFINITY;
            pb.hi[k] = INFINITY;
        }
    if (act && sl == lpt - 1)   // spheres (lattice scenes have n <= 63 triangles)
        for (int q = 0; q < F.n_sph; ++q)
            if (!sphere_surely_missed(sph[q], camf, x0, x1, y0, y1, F.focal)) {
                sphere = true;
                sphere_hit_box(sph[q], camf, x0, x1, y0, y1, F.focal, pb.lo, pb.hi);
            }
    const unsigned long long half = tpw == 2 ? 0xffffffffull : ~0ull;
    const unsigned long long m = ((__ballot(keep) >> (sub * lpt)) & half) |
                                 (((__ballot(sphere) >> (sub * lpt)) & half) ? (1ull << 63) : 0ull);
    // the unit's box of possible hit positions (reduction within its lanes)
    float blo[3], bhi[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float lo = pb.lo[k], hi = pb.hi[k];
        for (int o = lpt >> 1; o > 0; o >>= 1) {
            lo = fminf(lo, __shfl_xor(lo, o, 64));
            hi = fmaxf(hi, __shfl_xor(hi, o, 64));
        }
        blo[k] = lo;
        bhi[k] = hi;
    }
    const bool cert = F.cull_shadow && F.n_lights > 0;
    bool keep_s = true;
    if (cert && act && m != 0ull && sl < n && blo[0] <= bhi[0])
        keep_s = !cull_shadow(c, v3(F.lc[0], F.lc[1], F.lc[2]), F.lrho, shadow_box_of_range(F, blo, bhi));
    // a unit whose every hit lies on one triangle k: k never shadows its own hits
    if (cert && keep && keep_s && m == (1ull << sl)) {
        const double Lp[3] = {(double)F.lc[0], (double)F.lc[1], (double)F.lc[2]};   // the light set's centre
        if (own_shadow_rejects(tris[sl], c, pd, thi, camf, x0, x1, y0, y1, F.focal, Lp, F.lrho, blo, bhi))
            keep_s = false;
    }
    unsigned long long sm = (__ballot(keep_s && sl < n) >> (sub * lpt)) & half;
    bool sph_shadow = F.n_sph > 0;   // bit 63 of the shadow mask: a sphere may block a shadow ray
    if (m == 0ull) {
        sm = 0ull;                   // no ray of the unit can hit anything: no shadow rays
        sph_shadow = false;
    } else if (cert && blo[0] <= bhi[0]) {
        bool any = false;
        for (int q = 0; q < F.n_sph; ++q) any |= !sphere_shadow_surely_missed_set(sph[q], F, blo, bhi);
        sph_shadow = any;
    }
    sm = (sm & ~(1ull << 63)) | (sph_shadow ? (1ull << 63) : 0ull);
    m_out = act ? m : 0ull;
    sm_out = act ? sm : 0ull;
}

// Per-scene constants of triangle i (rt_scene_kernel): the camera-independent
// part of rt_tri_const (e1, e2, v0, K1: the same float ops) and the shading
// attributes.
__global__ void rt_scene_kernel(const cg_tri *__restrict__ tris, int n, RtGeo *__restrict__ geo,
                                RtShade *__restrict__ shade)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const cg_tri T = tris[i];
    const RtTri c = rt_tri_const(T, 0.f, 0.f, 0.f, 0.f);
    RtGeo g;
    g.e1x = c.e1x; g.e1y = c.e1y; g.e1z = c.e1z; g.e2x = c.e2x;
    g.e2y = c.e2y; g.e2z = c.e2z; g.v0x = c.v0x; g.v0y = c.v0y;
    g.v0z = c.v0z; g.K1 = c.K1; g.pad0 = 0.f; g.pad1 = 0.f;
    geo[i] = g;
    RtShade sh;
    sh.nx = T.normal.x; sh.ny = T.normal.y; sh.nz = T.normal.z; sh.nw = T.normal.w;
    sh.cr = T.color.x; sh.cg = T.color.y; sh.cb = T.color.z; sh.pad = 0.f;
    shade[i] = sh;
}

// Per-frame RtTri of triangle i (one thread; the small scenes' certificate launch).
__device__ __forceinline__ void prep_tri(const RtGeo *__restrict__ geo, int n, int i, int frame, const float camf[4],
                                         RtTri *__restrict__ out)
{
    if (i >= n) return;
    out[(size_t)frame * n + i] = rt_tri_frame(geo[i], camf);
}

// Per-frame RtTri of the 256 triangles of block blk, staged through LDS so
// that both streams are coalesced 16-byte accesses: the block's 256 x 48 B of
// RtGeo are read as 768 consecutive float4s (3 per thread), each thread forms
// its triangle's RtTri into LDS, and the block's 256 x 64 B go out as 1024
// consecutive float4s (4 per thread).  A pure streaming pass (C5: 1M
// triangles, 48 MB in, 64 MB out per frame).
__device__ __forceinline__ void prep_block(const RtGeo *__restrict__ geo, int n, int blk, int frame,
                                           const float camf[4], RtTri *__restrict__ out)
{
    __shared__ float4 s_buf[kRtThreads * 4];     // 16 KB: RtGeo in (12 KB), then RtTri out
    const int t = threadIdx.x, i0 = blk * kRtThreads, cnt = min(kRtThreads, n - i0);
    const float4 *src = reinterpret_cast<const float4 *>(geo + i0);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int q = t + k * kRtThreads;
        if (q < 3 * cnt) s_buf[q] = src[q];
    }
    __syncthreads();
    RtTri r{};
    if (t < cnt) {
        const float4 a = s_buf[3 * t], b = s_buf[3 * t + 1], c = s_buf[3 * t + 2];
        RtGeo g;
        g.e1x = a.x; g.e1y = a.y; g.e1z = a.z; g.e2x = a.w;
        g.e2y = b.x; g.e2z = b.y; g.v0x = b.z; g.v0y = b.w;
        g.v0z = c.x; g.K1 = c.y; g.pad0 = c.z; g.pad1 = c.w;
        r = rt_tri_frame(g, camf);
    }
    __syncthreads();
    if (t < cnt) {
        s_buf[4 * t] = make_float4(r.e1x, r.e1y, r.e1z, r.e2x);
        s_buf[4 * t + 1] = make_float4(r.e2y, r.e2z, r.sx, r.sy);
        s_buf[4 * t + 2] = make_float4(r.sz, r.detT, r.K1, r.K2);
        s_buf[4 * t + 3] = make_float4(r.K3, r.v0x, r.v0y, r.v0z);
    }
    __syncthreads();
    float4 *dst = reinterpret_cast<float4 *>(out + (size_t)frame * n + i0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int q = t + k * kRtThreads;
        if (q < 4 * cnt) dst[q] = s_buf[q];
    }
}

__global__ __launch_bounds__(kRtThreads) void rt_prepare_kernel(const cg_tri *__restrict__ tris,
                                                                const RtGeo *__restrict__ geo, int n, RtFrameCams cams,
                                                                RtTri *__restrict__ out, int n_prep_blocks,
                                                                RtFrame F, const RtSphere *__restrict__ sph,
                                                                unsigned long long *__restrict__ lat_masks, int sup)
{
    const int frame = blockIdx.y;
    const float camf[4] = {cams.c[frame][0], cams.c[frame][1], cams.c[frame][2], cams.c[frame][3]};
    if ((int)blockIdx.x < n_prep_blocks) {
        prep_block(geo, n, blockIdx.x, frame, camf, out);
        return;
    }
    // Unit certificates: lpt lanes per unit (lane k = triangle k; the last lane
    // takes the spheres), two units per wave when the scene has <= 31 triangles.
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tiles = rt_cert_units(F, sup);
    lat_masks += (size_t)frame * tiles * 2;
    const int tpw = n <= 31 ? 2 : 1, lpt = 64 / tpw;
    const int sub = lane / lpt, sl = lane - sub * lpt;
    int tile = (((int)blockIdx.x - n_prep_blocks) * (kRtThreads / 64) + wave) * tpw + sub;
    // single-level over a tile-column window (RtFrame::txn): the window's tiles only
    const int units = (!sup && F.txn) ? F.txn * (tiles / lat_tiles_x(F)) : tiles;
    if (__ballot(tile < units) == 0ull) return;   // whole wave
    const bool tv = tile < units;
    if (!sup && F.txn) tile = (tile / F.txn) * lat_tiles_x(F) + F.tx0 + tile % F.txn;
    unsigned long long m, sm;
    unit_cert(tris, n, camf, F, sph, tile, sup, tv, tpw, m, sm);
    if (tv && sl == 0) {
        lat_masks[2 * tile] = m;
        lat_masks[2 * tile + 1] = sm;
    }
}


// ---------------------------------------------------------------------------
// Second level of the tile certificates: one wave per super-tile refines its
// masks for each of its kSup x kSup tiles.  Only the super-tile's candidates
// are certified again -- a certificate over the super-tile's bundle (or box of
// hit positions) is a proof for every tile inside it -- and the (tile,
// candidate) pairs are packed densely into the wave's lanes: cp lanes per tile
// (cp = the candidate count rounded up to a power of two), segments aligned, so
// the per-tile reductions are xor butterflies within a segment.  Phase 1:
// primary certificate, occlusion, hit-position box, sphere; phase 2: shadow
// certificate of the tile's box.  Same functions and exactness arguments as
// rt_prepare_kernel's single-level path.

__device__ __forceinline__ int pow2_at_least(int c)
{
    int p = 1;
    while (p < c) p <<= 1;
    return p;
}
// index of the i-th set bit of m (m has more than i bits)
__device__ __forceinline__ int nth_bit(unsigned long long m, int i)
{
    for (int k = 0; k < i; ++k) m &= m - 1ull;
    return __builtin_ctzll(m);
}
__device__ __forceinline__ unsigned long long seg_or(unsigned long long v, int cp)
{
    for (int o = cp >> 1; o > 0; o >>= 1) {
        const unsigned lo = __shfl_xor((unsigned)v, o, 64), hi = __shfl_xor((unsigned)(v >> 32), o, 64);
        v |= ((unsigned long long)hi << 32) | lo;
    }
    return v;
}

// The workgroup is 1 or 4 waves (blockDim.x 64 or 256): wave w takes
// iterations w, w + waves, ... of each phase, so a call with few super-tiles
// (one rank's band) is not bound by one wave's serial chain of certificates.
// Fused (sup_masks == null): one launch does the whole two-level chain -- the
// first n_prep_blocks blocks write the frame's RtTri / RtShade (as
// rt_prepare_kernel's), every other block first certifies its super-tile
// (wave 0, unit_cert) into LDS and then refines it per tile; no super-tile
// masks round-trip through memory and no second dependent launch.
__device__ __forceinline__ void lat_flatten(const LatFlatten &Z);   // below, with the lattice kernel

#ifndef CG_CERT_WAVES
// waves per SIMD of the certificate launch (A/B: -DCG_CERT_WAVES=n): 3 -- 154 VGPRs and no scratch
// (4: 128 VGPRs and 80 B of scratch): the driver-shaped call's certificates 81.8 -> 73.6 us live
// (CG_KTIME_ALL, four runs each; profiles/r06_ab_session2.json); 5 waves (236 B of scratch) slower
#define CG_CERT_WAVES 3
#endif
__global__ __launch_bounds__(256, CG_CERT_WAVES) void rt_tile_cert_kernel(const cg_tri *__restrict__ tris,
                                                           const RtGeo *__restrict__ geo, int n, RtFrameCams cams,
                                                           RtFrame F, const RtSphere *__restrict__ sph,
                                                           const unsigned long long *__restrict__ sup_masks,
                                                           unsigned long long *__restrict__ lat_masks,
                                                           RtTri *__restrict__ tc_out,
                                                           int n_prep_blocks, int frame_fast, LatFlatten Z,
                                                           LatPublish P)
{
    constexpr int kT = kSup * kSup;
    // frame_fast: blockIdx.x = frame (dispatched fastest), blockIdx.y = prep block, then
    // super-tile; else the other way round (grids beyond 65,535 blocks in y)
    const int frame = frame_fast ? blockIdx.x : blockIdx.y, blk = frame_fast ? blockIdx.y : blockIdx.x;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
    const float camf[4] = {cams.c[frame][0], cams.c[frame][1], cams.c[frame][2], cams.c[frame][3]};
    if (blk < n_prep_blocks) {
        prep_tri(geo, n, blk * blockDim.x + threadIdx.x, frame, camf, tc_out);
        // the first block (dispatched first) also sorts the lattice launch's order
        if (Z.n > 0 && blk == 0 && frame == 0) lat_flatten(Z);
        return;
    }
#ifdef CG_WG_TIMING
    const unsigned long long wt0 = wall_clock64();
#endif
    const int tiles_x = (F.W + kLatTileW - 1) / kLatTileW, tiles_y = (F.rows_out + kLatTileH - 1) / kLatTileH;
    const int sx = (tiles_x + kSup - 1) / kSup;
    // the launch's super-tile columns: those over the window's tiles (all when F.txn = 0)
    const int s0 = F.txn ? F.tx0 / kSup : 0, sxw = F.txn ? (F.tx0 + F.txn + kSup - 1) / kSup - s0 : sx;
    // super-tile rows bottom first, each row's super-tiles for every frame of the launch in turn:
    // the floor and box rows carry the longest certificate chains (up to 3x the median), and
    // dispatched last they set the launch's tail (C2, 20 frames: 107 -> 84 us simulated)
    const int sy = (tiles_y + kSup - 1) / kSup, ud = blk - n_prep_blocks;
    const int uw = (sy - 1 - ud / sxw) * sxw + ud % sxw, unit = (uw / sxw) * sx + s0 + uw % sxw;
    lat_masks += (size_t)frame * tiles_x * tiles_y * 2;
    // published certificates (LatPublish): the frame's RtTri stored by this workgroup too, so
    // that a published super-tile implies a complete RtTri (every workgroup of the frame
    // stores the same values)
    if (P.flags && wave == 0 && lane < n) tc_out[(size_t)frame * n + lane] = rt_tri_frame(geo[lane], camf);
    __shared__ unsigned long long s_sup[2];
    if (!sup_masks) {
        if (wave == 0) {
            unsigned long long m, sm;
            unit_cert(tris, n, camf, F, sph, unit, 1, true, 1, m, sm);
            if (lane == 0) {
                s_sup[0] = m;
                s_sup[1] = sm;
            }
        }
        __syncthreads();
    } else if (threadIdx.x == 0) {
        const unsigned long long *sm = sup_masks + ((size_t)frame * rt_cert_units(F, 1) + unit) * 2;
        s_sup[0] = sm[0];
        s_sup[1] = sm[1];
    }
    __syncthreads();
    WGT_STAMP(wt1);
    const unsigned long long SP = s_sup[0], SS = s_sup[1];
    const unsigned long long SPt = SP & ~(1ull << 63), SSt = SS & ~(1ull << 63);
    const bool cert = F.cull_shadow && F.n_lights > 0;
    const double Lp[3] = {(double)F.lc[0], (double)F.lc[1], (double)F.lc[2]};   // the light set's centre
    __shared__ unsigned long long s_pm[kT], s_own[kT];
    __shared__ float s_box[kT][6];
    __shared__ int s_sphsh[kT];
    auto tile_of = [&](int tl, int &t, LatTile &G) {
        const int bx = (unit % sx) * kSup + tl % kSup, by = (unit / sx) * kSup + tl / kSup;
        const bool in = tl < kT && bx < tiles_x && by < tiles_y;
        G = lat_tile(F, in ? bx : 0, in ? by : 0);
        t = in ? by * tiles_x + bx : -1;
        return in && G.rows > 0;
    };
    // Phase 1: primary candidates (triangles of SP, then the sphere if flagged)
    const int ntp = __popcll(SPt), cand = ntp + (int)(SP >> 63);
    const int cp = pow2_at_least(max(cand, 1)), tpi = 64 / cp;
    for (int it = wave; it * tpi < kT; it += nwaves) {
        const int seg = lane / cp, ci = lane - seg * cp, tl = it * tpi + seg;
        int t;
        LatTile G;
        const bool act = tile_of(tl, t, G) && ci < cand;
        float x0, x1;
        lat_xrange(F, G, G, x0, x1);
        const float y0 = 0.5f * (float)G.ay0, y1 = 0.5f * (float)(G.ay0 + G.rows - 1);
        const bool is_tri = act && ci < ntp;
        const int k = is_tri ? nth_bit(SPt, ci) : 0;
        bool keep = false, sphere = false;
        RtTri c{};
        PrimDet pd;
        double tlo = 0.0, thi = INFINITY;
        LanePosBox pb;
        pb.init();
        if (is_tri) {
            c = rt_tri_const(tris[k], camf[0], camf[1], camf[2], camf[3]);
            keep = !cull_primary(c, x0, x1, y0, y1, F.focal, &pd);
            if (keep && !primary_t_range(c, pd, tlo, thi)) {
                tlo = 0.0;
                thi = INFINITY;
            }
        }
        double occ = (keep && primary_covers(c, pd)) ? thi : INFINITY;
        for (int o = cp >> 1; o > 0; o >>= 1) occ = fmin(occ, __shfl_xor(occ, o, 64));
        if (keep && tlo > occ * (1.0 + 0x1p-18)) keep = false;
        if (keep && !primary_hit_box(c, pd, camf, x0, x1, y0, y1, F.focal, pb.lo, pb.hi,
                                     &tris[k]))
            for (int q = 0; q < 3; ++q) {
                pb.lo[q] = -INFINITY;
                pb.hi[q] = INFINITY;
            }
        if (act && !is_tri)   // the sphere candidate
            for (int q = 0; q < F.n_sph; ++q)
                if (!sphere_surely_missed(sph[q], camf, x0, x1, y0, y1, F.focal)) {
                    sphere = true;
                    sphere_hit_box(sph[q], camf, x0, x1, y0, y1, F.focal, pb.lo, pb.hi);
                }
        unsigned long long m = seg_or((keep ? (1ull << k) : 0ull) | (sphere ? (1ull << 63) : 0ull), cp);
        // bit 62: the tile's only candidate is one triangle that every ray
        // certainly hits -- the lattice kernel then skips the u, v tests
        const unsigned long long cov = seg_or((keep && primary_covers(c, pd)) ? (1ull << k) : 0ull, cp);
        float blo[3], bhi[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            float lo = pb.lo[q], hi = pb.hi[q];
            for (int o = cp >> 1; o > 0; o >>= 1) {
                lo = fminf(lo, __shfl_xor(lo, o, 64));
                hi = fmaxf(hi, __shfl_xor(hi, o, 64));
            }
            blo[q] = lo;
            bhi[q] = hi;
        }
        bool own = false;
        if (cert && keep && m == (1ull << k))
            own = own_shadow_rejects(tris[k], c, pd, thi, camf, x0, x1, y0, y1, F.focal, Lp, F.lrho, blo, bhi);
        const unsigned long long ownm = seg_or(own ? (1ull << k) : 0ull, cp);
        if (tl < kT && ci == 0) {
            const bool live = tile_of(tl, t, G);
            const bool single = m != 0ull && (m & (m - 1ull)) == 0ull && !(m >> 63);
            s_pm[tl] = live ? (m | ((single && (cov & m)) ? (1ull << 62) : 0ull)) : 0ull;
            s_own[tl] = ownm;
            for (int q = 0; q < 3; ++q) {
                s_box[tl][q] = blo[q];
                s_box[tl][3 + q] = bhi[q];
            }
            bool sphsh = F.n_sph > 0 && (SS >> 63);
            if (live && m != 0ull && cert && blo[0] <= bhi[0] && sphsh) {
                bool any = false;
                for (int q = 0; q < F.n_sph; ++q) any |= !sphere_shadow_surely_missed_set(sph[q], F, blo, bhi);
                sphsh = any;
            }
            s_sphsh[tl] = sphsh ? 1 : 0;
        }
    }
    __syncthreads();
    WGT_STAMP(wt2);
    // Phase 2: shadow candidates (triangles of SS)
    const int nts = __popcll(SSt);
    const int sp = pow2_at_least(max(nts, 1)), tpi2 = 64 / sp;
    for (int it = wave; it * tpi2 < kT; it += nwaves) {
        const int seg = lane / sp, ci = lane - seg * sp, tl = it * tpi2 + seg;
        int t;
        LatTile G;
        const bool live = tile_of(tl, t, G);
        const unsigned long long pm = tl < kT ? s_pm[tl] : 0ull;
        const bool act = live && ci < nts && pm != 0ull;
        const int k = act ? nth_bit(SSt, ci) : 0;
        bool keep_s = false;
        if (act) {
            keep_s = true;
            const float blo[3] = {s_box[tl][0], s_box[tl][1], s_box[tl][2]};
            const float bhi[3] = {s_box[tl][3], s_box[tl][4], s_box[tl][5]};
            if (cert && blo[0] <= bhi[0]) {
                const RtTri c = rt_tri_const(tris[k], camf[0], camf[1], camf[2], camf[3]);
                keep_s = !cull_shadow(c, v3(F.lc[0], F.lc[1], F.lc[2]), F.lrho, shadow_box_of_range(F, blo, bhi));
            }
            if ((s_own[tl] >> k) & 1ull) keep_s = false;
        }
        const unsigned long long sm = seg_or(keep_s ? (1ull << k) : 0ull, sp);
        if (tl < kT && ci == 0 && t >= 0) {
            lat_masks[2 * t] = live ? pm : 0ull;
            lat_masks[2 * t + 1] = (live && pm != 0ull) ? (sm | (s_sphsh[tl] ? (1ull << 63) : 0ull)) : 0ull;
        }
    }
    if (P.flags) {   // publish: every wave's stores written back, then the word (agent-scope release)
        __threadfence();
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(P.flags + (size_t)frame * P.units + unit, P.gen, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
#ifdef CG_WG_TIMING
    WGT_STAMP(wt3);
    wgt_record(1, wt0, wt1, wt2, wt3);
#endif
}


// Draw (skeleton.cpp:104-169), one thread per pixel.  CULL: n_tris <= 64,
// one certificate mask per wave (lane k certifies triangle k).
#ifndef CG_LAT_WAVES
#define CG_LAT_WAVES 6    // A/B: -DCG_LAT_WAVES=n
#endif
constexpr int kRtMinWaves = CG_LAT_WAVES;   // waves per SIMD of rt_lattice_kernel (68 VGPRs: 7 fit)
// The pixel kernel (rotations other than a yaw; no bench configuration) at 5
// waves per SIMD: 96 VGPRs and no scratch -- 6 spilled 52 B per lane for ~1 %.
constexpr int kRtPixelWaves = 5;
template <bool CULL>
__global__ __launch_bounds__(kRtThreads, kRtPixelWaves) void rt_pixel_kernel(RtFrame F, const RtTri *__restrict__ tc,
                                                              const RtShade *__restrict__ shade,
                                                              const RtSphere *__restrict__ sph,
                                                              uint32_t *__restrict__ out)
{
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int u = blockIdx.x * kRtTileW + wave * 8 + (lane & 7);
    const int L = blockIdx.y * kRtTileH + (lane >> 3);
    const bool inside = u < F.W && L < F.rows_out;
    const int v = inside ? shard_row(F, L) : 0;
    const bool active = inside && v < F.H;
    vec4 dir = v4((float)(u - F.W / 2), (float)(v - F.H / 2), F.focal, 1.0f);        // :126
    dir = mat4_mul(F.R, dir);                                                         // :128
    unsigned long long mask = ~0ull;
    if (CULL) {
        // exact float extremes of the wave's sub-ray directions (:137): newDir.x =
        // fl(dir.x + 0.5 i) is monotone in dir.x, so the bundle lies in this box
        float ax = active ? dir.x : __int_as_float(0x7fc00000), ay = active ? dir.y : __int_as_float(0x7fc00000);
        float x0 = wave_min(active ? ax : FLT_MAX), x1 = wave_max(active ? ax : -FLT_MAX);
        float y0 = wave_min(active ? ay : FLT_MAX), y1 = wave_max(active ? ay : -FLT_MAX);
        x0 = x0 - 0.5f; x1 = x1 + 0.5f; y0 = y0 - 0.5f; y1 = y1 + 0.5f;
        bool keep = true;
        if (lane < F.n_tris && x0 <= x1 && y0 <= y1) keep = !cull_primary(tc[lane], x0, x1, y0, y1, F.focal);
        mask = __ballot(keep && lane < F.n_tris);
    }
    // every lane stays to the end: the certificates' wave reductions read all 64
    uint32_t px = 0u;
    // Pass 1: the 9 primary rays (:134-140); hits staged in LDS (bi, t) so one
    // shadow certificate covers the whole wave's hits and all lights at once.
    __shared__ int s_bi[9][kRtThreads];
    __shared__ float s_t[9][kRtThreads];
    const float m = 0.5f;
    if (active) {
        // sub-ray k = 3 (i + 1) + (j + 1): d = (dir.x + m i, dir.y + m j, focal)  (:137),
        // walked in three groups sharing d.y (closest_primary_group)
        float dx[3], dy[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            dx[q] = dir.x + (m * (float)(q - 1));
            dy[q] = dir.y + (m * (float)(q - 1));
        }
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) {
            int bi[3];
            float t[3];
            const float dyj[1] = {dy[jj]};
            closest_primary_group<CULL, 3, 1>(F, tc, sph, dx, dyj, mask, bi, t);         // :140
#pragma unroll
            for (int ii = 0; ii < 3; ++ii) {
                s_bi[3 * ii + jj][threadIdx.x] = bi[ii];
                s_t[3 * ii + jj][threadIdx.x] = t[ii];
            }
        }
    }
    // one mask for every light of the set (the mask walk must stop at n_tris)
    unsigned long long smask = F.n_tris >= 64 ? ~0ull : ((1ull << F.n_tris) - 1ull);
    if (CULL && F.cull_shadow && F.n_lights > 0) {
        LanePosBox pb;
        pb.init();
        if (active)
            for (int k = 0; k < 9; ++k) {
                const int bi = s_bi[k][threadIdx.x];
                if (bi == INT_MIN) continue;
                const float t = s_t[k][threadIdx.x];
                const int i = k / 3 - 1, j = k % 3 - 1;
                vec3 nd = v3(dir.x + (m * (float)i), dir.y + (m * (float)j), F.focal);
                pb.add(v3(F.cam[0] + t * nd.x, F.cam[1] + t * nd.y, F.cam[2] + t * nd.z));   // :326/:345
            }
        smask = shadow_mask_box(F, tc, shadow_box_of_positions(F, pb), lane);
    }
    if (active) {
        // Pass 2: shading in the reference's order (:143-157)
        vec3 pc = v3(0.0f, 0.0f, 0.0f);
        bool valid = false;
        const vec3 ind = v3(F.indirect, F.indirect, F.indirect);
        for (int k = 0; k < 9; ++k) {
            const int i = k / 3 - 1, j = k % 3 - 1;
            const int bi = s_bi[k][threadIdx.x];
            if (bi == INT_MIN) continue;
            const float t = s_t[k][threadIdx.x];
            vec3 nd = v3(dir.x + (m * (float)i), dir.y + (m * (float)j), F.focal);
            vec3 pos = v3(F.cam[0] + t * nd.x, F.cam[1] + t * nd.y, F.cam[2] + t * nd.z);  // :326/:345
            valid = true;
            vec3 oc = object_colour(shade, sph, bi);
            for (int l = 0; l < F.n_lights; ++l)                                          // :151-153
                pc = pc + direct_light<CULL>(F, tc, shade, sph, bi, pos, oc, l, smask);
            pc = pc + (oc * ind);                                                         // :156
        }
        px = valid ? put_pixel(div_const(pc, 9.0f, 1.0f / 9.0f)) : put_pixel(v3(0.0f, 0.0f, 0.0f));             // :160-166
    }
    if (inside) out[(size_t)L * F.W + u] = px;
}

// ---------------------------------------------------------------------------
// Lattice form of Draw (skeleton.cpp:104-169) for one light -- the C2
// configuration; described here for the unrotated camera (shared columns; a
// yawed camera keeps per-pixel columns, see lat_yaw).  With R the identity, a pixel's direction is
// (u - W/2, v - H/2) exactly (mat4_mul adds only +-0 terms), and sub-ray
// (i, j) is (x + 0.5 i, y + 0.5 j), exactly representable: the 9 sub-rays of
// all pixels lie on a half-pixel lattice, and pixel (u, v)'s sub-ray (i, j) IS
// the lattice ray (2u + i, 2v + j) of its neighbours, bit for bit.  A sub-ray's
// whole contribution -- closest hit (:140), DirectLight (:151-153) and the
// ambient term (:156) -- depends only on the ray, so each lattice ray is traced
// once per tile (65 x 17 rays for 32 x 8 pixels instead of 2304) and every
// pixel then adds its nine contributions in the reference's order
// (pc += DirectLight; pc += objColor * indirect, k = 0..8), so the float sums
// are formed exactly as the reference forms them.
// kLatTileW x kLatTileH = 16 x 15 pixels: 33 x 31 = 1023 lattice rays = 4 passes of 256 lanes
constexpr int kLatW = 2 * kLatTileW + 1, kLatH = 2 * kLatTileH + 1;
#ifndef CG_LAT_INTERLEAVE
#define CG_LAT_INTERLEAVE 1   // rt_lattice_kernel's points dealt to waves in 64-point chunks (A/B: 0)
#endif
constexpr int kLatWY = 3 * kLatTileW;   // per-pixel columns (a yawed camera): 48 x 31 = 1488 rays
#ifndef CG_LAT_SOA
#define CG_LAT_SOA 1   // per-pixel-column lattice: point values and hit indices in separate LDS arrays (A/B: 0)
#endif
constexpr int kLatSoaNoHit = -128;   // int8 hit index of a miss (hits: -kLatMaxSph .. 62)

// Shared pieces of the two lattice kernels.
//
// Shading attributes of every object a lattice ray can hit, in LDS: slot k
// for triangle k (normal, colour), slot kLatSphSlot + q for sphere q
// (centre, colour).  One table for both kinds keeps these reads LDS reads
// (separate shade / sphere arrays make the compiler fetch through a flat
// pointer, which waits for the vector memory counter as well).
constexpr int kLatMaxSph = 8, kLatSphSlot = 64;
struct LatObj {
    float x, y, z, pad0;   // triangle normal, or sphere centre
    float r, g, b, pad1;   // colour
};
__device__ __forceinline__ void lat_load_objs(LatObj *s_obj, const RtShade *__restrict__ shade,
                                              const RtSphere *__restrict__ sph, int n_tris, int n_sph)
{
    const int t = threadIdx.x;
    if (t < n_tris) {
        const RtShade h = shade[t];
        s_obj[t] = LatObj{h.nx, h.ny, h.nz, 0.0f, h.cr, h.cg, h.cb, 0.0f};
    } else if (t >= kLatSphSlot && t < kLatSphSlot + n_sph) {
        const RtSphere S = sph[t - kLatSphSlot];
        s_obj[t] = LatObj{S.cx, S.cy, S.cz, 0.0f, S.cr, S.cg, S.cb, 0.0f};
    }
}
__device__ __forceinline__ int lat_slot(int bi) { return bi >= 0 ? bi : kLatSphSlot - 1 - bi; }
// object colour (skeleton.cpp:147-148, :378 / :382)
__device__ __forceinline__ vec3 lat_colour(const LatObj *s_obj, int bi)
{
    const LatObj o = s_obj[lat_slot(bi)];
    return v3(o.r, o.g, o.b);
}
// normal at the hit (:377-387): the triangle's, or Sphere::getNormal
__device__ __forceinline__ vec3 lat_normal(const LatObj *s_obj, int bi, vec3 pos)
{
    const LatObj o = s_obj[lat_slot(bi)];
    if (bi >= 0) return v3(o.x, o.y, o.z);
    return normalize(pos - v3(o.x, o.y, o.z));
}
// DirectLight (skeleton.cpp:366-415) of light Lt for a hit on bi at pos, the
// shadow ray walking the candidates of smask (as direct_light<true>)
template <bool SHARED = false>
__device__ __forceinline__ vec3 lat_direct_light(const RtFrame &Fs, const RtTri *__restrict__ tc,
                                                 const RtSphere *__restrict__ sph, const LatObj *s_obj,
                                                 const RtLight &Lt, int bi, vec3 pos, unsigned long long smask)
{
    cg_work(W_DL);
    const vec3 r = v3(Lt.x, Lt.y, Lt.z) - pos;                          // :370
    const float rmag = light_rmag(r);                                   // :371
    const vec3 normal = lat_normal(s_obj, bi, pos);                     // :377-387
    const vec3 origin = pos + normal * 0.00001f;                        // :394
    if (shadowed<true>(Fs, tc, sph, origin, r, rmag, smask)) return v3(0.0f, 0.0f, 0.0f);   // :394-398
    return direct_light_lit<SHARED>(Lt, r, rmag, normal, lat_colour(s_obj, bi));
}

//
// Output of one tile: the pixel value px of (tx, ty) (have = inside the tile),
// stored as ARGB at row L0 + ty, or in the RGB24 wire format (the pixel's low
// three bytes, B, G, R; alpha is always 128) inside the output window, full
// tiles writing each row's 48 bytes as 12 dwords through s_px.  Called by
// every thread of the workgroup (RGB24 has a barrier).
struct LatOut {
    uint32_t *out;
    uint8_t *out8;
    int pitch, wc0;
};
__device__ __forceinline__ LatOut lat_out(const RtFrame &F, int frame, size_t out_stride, uint32_t *out)
{
    LatOut o;
    o.out8 = (uint8_t *)out + (size_t)frame * out_stride * 3;   // CG_PIX_RGB24
    o.out = out + (size_t)frame * out_stride;
    // RGB24 window (a caller's contract: the columns outside are black);
    // windows are 16-pixel aligned
    o.pitch = (F.out_fmt == CG_PIX_RGB24 && F.wcols) ? F.wcols : F.W;
    o.wc0 = (F.out_fmt == CG_PIX_RGB24 && F.wcols) ? F.wcol0 : 0;
    return o;
}
__device__ __forceinline__ void lat_store(const RtFrame &F, const LatTile &G, const LatOut &o, uint32_t px, int tx,
                                          int ty, uint32_t *s_px)
{
    const bool have = tx < G.nu && ty < G.nv;
    if (F.out_fmt == CG_PIX_ARGB8888) {
        if (have) o.out[(size_t)(G.L0 + ty) * F.W + G.u0 + tx] = px;
        return;
    }
    if (have) s_px[ty * kLatTileW + tx] = px;
    __syncthreads();
    if (G.nu == kLatTileW && (o.pitch & 3) == 0 && ((uintptr_t)o.out8 & 3) == 0) {
        const int t = threadIdx.x, row = t / 12, j = t - 12 * row;
        if (row < G.nv) {
            uint32_t w = 0u;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int byte = 4 * j + b, p = byte / 3, ch = byte - 3 * p;
                w |= ((s_px[row * kLatTileW + p] >> (8 * ch)) & 0xffu) << (8 * b);
            }
            *(uint32_t *)(o.out8 + ((size_t)(G.L0 + row) * o.pitch + (G.u0 - o.wc0)) * 3 + 4 * j) = w;
        }
    } else if (have) {
        uint8_t *q = o.out8 + ((size_t)(G.L0 + ty) * o.pitch + (G.u0 - o.wc0) + tx) * 3;
        q[0] = (uint8_t)px;
        q[1] = (uint8_t)(px >> 8);
        q[2] = (uint8_t)(px >> 16);
    }
}

// Pass 1 of the lattice kernels: the closest hit (:140) of lattice points
// p_lo .. p_hi - 1 (row-major at pitch kLatW; columns >= cols exist only in
// tiles cut by the right edge), two points per lane per step (p, p + 64) with
// one triangle load for both; store(p, t, hit index) for each needed point.
// covered: the tile's one candidate triangle k is certainly accepted by every
// ray (rt_tile_cert_kernel: t > 0, u, v inside, nothing else can be hit), so
// the reference's closest hit is k with t = detT / det (:306), formed with
// closest_primary_n's float ops; the u, v tests and the distance are not needed.
template <int PITCH, class Store, int NP = 2>
__device__ __forceinline__ void lat_closest(const RtFrame &Fp, const RtTri *__restrict__ tc,
                                            const RtSphere *__restrict__ sph, unsigned long long mask, bool covered,
                                            const LatTile &G, int p_lo, int p_hi, int lane, Store store,
                                            int step = 128, int ray_stride = 64, bool wc = true)
{
    for (int p0 = p_lo; p0 < p_hi; p0 += step) {
        float X[NP], Y[NP];
        bool live[NP];
        int pp[NP];
#pragma unroll
        for (int n = 0; n < NP; ++n) {
            const int p = p0 + ray_stride * n + lane;
            const int cy = p / PITCH, cx = p - cy * PITCH;
            pp[n] = p;
            live[n] = p < p_hi && cx < G.cols;
            X[n] = lat_x(Fp, G, cx);
            Y[n] = 0.5f * (float)(G.ay0 + cy);
        }
        int bi[NP];
        float t[NP];
        if (covered) {
            const int k = __builtin_ctzll(mask);
            const RtTri c = tc[k];
#pragma unroll
            for (int n = 0; n < NP; ++n) {
                if (wc && live[n]) {   // the t stage of the ray's one candidate
                    cg_work(W_RAY_PRI);
                    cg_work(W_T_PRI);
                }
                const vec3 nd = -v3(X[n], Y[n], Fp.focal);
                const float Q2 = nd.y * c.e2z - c.e2y * nd.z;
                const float Q1 = nd.y * c.e1z - c.e1y * nd.z;
                const float det = (nd.x * c.K1 - c.e1x * Q2) + c.e2x * Q1;   // :289
                t[n] = c.detT / det;                                         // :306
                bi[n] = k;
            }
        } else {
            closest_primary_n<NP>(Fp, tc, sph, X, Y, live, mask, bi, t, wc);   // :140
        }
#pragma unroll
        for (int n = 0; n < NP; ++n)
            if (live[n]) store(pp[n], t[n], bi[n]);
    }
}

// A tile no ray of which can hit anything (certified): every pixel is
// PutPixelSDL(0, 0, 0) = 0x80000000 (:160-166).
__device__ __forceinline__ void lat_store_black(const RtFrame &F, const LatTile &G, const LatOut &o)
{
    const int tx = threadIdx.x % kLatTileW, ty = threadIdx.x / kLatTileW;
    if (tx < G.nu && ty < G.nv) {
        const uint32_t px = put_pixel(v3(0.0f, 0.0f, 0.0f));
        if (F.out_fmt == CG_PIX_ARGB8888) {
            o.out[(size_t)(G.L0 + ty) * F.W + G.u0 + tx] = px;
        } else {
            const size_t q = (size_t)(G.L0 + ty) * o.pitch + (G.u0 - o.wc0) + tx;
            o.out8[3 * q] = (uint8_t)px;
            o.out8[3 * q + 1] = (uint8_t)(px >> 8);
            o.out8[3 * q + 2] = (uint8_t)(px >> 16);
        }
    }
}

// A windowed launch (RtFrame::txn > 0): the first and last workgroup of each
// tile row also store the output's columns left / right of the window black
// -- no ray there can hit the scene's box (rt_box_columns), so those pixels
// are PutPixelSDL(0, 0, 0) -- instead of a workgroup per black tile.
__device__ __forceinline__ void lat_store_outside(const RtFrame &F, const LatTile &G, const LatOut &o,
                                                  int bxw = -1)
{
    if (F.txn <= 0 || G.nv <= 0) return;
    if (bxw < 0) bxw = (int)blockIdx.x;   // the workgroup's column within the launch's window
    const bool left = bxw == 0, right = bxw == (int)gridDim.x - 1;
    if (!left && !right) return;
    const uint32_t px = put_pixel(v3(0.0f, 0.0f, 0.0f));
    for (int side = 0; side < 2; ++side) {
        if (!(side ? right : left)) continue;
        const int c0 = side ? max(o.wc0, (F.tx0 + F.txn) * kLatTileW) : o.wc0;
        const int c1 = side ? o.wc0 + o.pitch : min(o.wc0 + o.pitch, F.tx0 * kLatTileW);
        const int w = c1 - c0;
        if (w <= 0) continue;
        for (int i = threadIdx.x; i < w * G.nv; i += blockDim.x) {
            const int r = i / w, col = c0 + (i - r * w);
            if (F.out_fmt == CG_PIX_ARGB8888) {
                o.out[(size_t)(G.L0 + r) * F.W + col] = px;
            } else {
                uint8_t *q = o.out8 + ((size_t)(G.L0 + r) * o.pitch + (col - o.wc0)) * 3;
                q[0] = (uint8_t)px;
                q[1] = (uint8_t)(px >> 8);
                q[2] = (uint8_t)(px >> 16);
            }
        }
    }
}

// The (frame, tile) of a lattice workgroup.  Default: blockIdx.z = frame, tile
// rows bottom first (lat_tile_row), bx = blockIdx.x.  With a measured order
// (LatOrder::flat, cg_internal.h), by the workgroup's dispatch rank (blockIdx
// linear: workgroups are dispatched in that order): frame-major (ngroups < 0)
// takes each frame's tiles heavy first, frame after frame -- a CU's
// consecutive workgroups keep one frame's triangle constants in its scalar
// cache; interleaved (ngroups >= 0) walks frame groups in turn and, inside a
// group, the tiles heavy first with every frame of the group at each tile:
// rank r of a group of nfg frames is tile flat[r / nfg] of frame r % nfg.
// flat is a permutation of the window's gx * gy tiles, so every (frame, tile)
// is still rendered exactly once.
struct LatSlot {
    int frame, bx, by;   // bx: column within the launch's window (tile column F.tx0 + bx)
};
__device__ __forceinline__ LatSlot lat_slot_of(const LatOrder &O)
{
    LatSlot S;
    const int gx = (int)gridDim.x, gy = (int)gridDim.y, n = gx * gy;
    if (!O.flat) {
        S.frame = (int)blockIdx.z;
        S.by = lat_tile_row();
        S.bx = (int)blockIdx.x;
        return S;
    }
    const int id = (int)blockIdx.x + gx * ((int)blockIdx.y + gy * (int)blockIdx.z);
    if (O.ngroups < 0) {   // frame-major: each frame's tiles heavy first, frames in turn
        S.frame = (int)blockIdx.z;
        const int t = (int)O.flat[id - S.frame * n];
        S.by = t / gx;
        S.bx = t - S.by * gx;
        return S;
    }
    int g0 = 0, g1 = (int)gridDim.z;
    if (O.ngroups > 0) {
        int g = 0;
        while (g + 1 < O.ngroups && id >= (int)O.gs[g + 1] * n) ++g;
        g0 = O.gs[g];
        g1 = O.gs[g + 1];
    }
    const int local = id - g0 * n, nfg = g1 - g0, r = local / nfg;
    S.frame = g0 + (local - r * nfg);
    const int t = (int)O.flat[r];   // uniform: a scalar load
    S.by = t / gx;
    S.bx = t - S.by * gx;
    return S;
}
// Heavy-first cost class of a workgroup's duration (wall_clock64 ticks, 100 MHz):
// four classes per octave, class 0 the longest.
__device__ __forceinline__ int lat_cost_class(unsigned long long d)
{
    const unsigned v = (unsigned)(d < 0xffffffffull ? d : 0xffffffffull) | 1u;
    const int lg = 31 - __clz(v);
    const int q = lg >= 2 ? (int)((v >> (lg - 2)) & 3u) : 0;
    return kLatClasses - 1 - min(kLatClasses - 1, max(0, 4 * lg + q - 16));
}
// rt_tile_cert_kernel's first block: counting sort of the recording Z.cost
// (class per tile) into Z.flat, heavy first.  Any recording gives a
// permutation of the n tiles.
__device__ __forceinline__ void lat_flatten(const LatFlatten &Z)
{
    __shared__ uint32_t s_cnt[kLatClasses], s_off[kLatClasses];
    const int t = threadIdx.x, nt = blockDim.x;
    if (t < kLatClasses) s_cnt[t] = 0u;
    __syncthreads();
    for (int j0 = 0; j0 < Z.n; j0 += 8 * nt) {
        int c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = j0 + u * nt + t;
            c[u] = j < Z.n ? min((int)Z.cost[j], kLatClasses - 1) : -1;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (c[u] >= 0) atomicAdd(&s_cnt[c[u]], 1u);
    }
    __syncthreads();
    if (t == 0) {
        uint32_t a = 0u;
        for (int k = 0; k < kLatClasses; ++k) {
            s_off[k] = a;
            a += s_cnt[k];
        }
    }
    __syncthreads();
    for (int j0 = 0; j0 < Z.n; j0 += 8 * nt) {
        int c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = j0 + u * nt + t;
            c[u] = j < Z.n ? min((int)Z.cost[j], kLatClasses - 1) : -1;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (c[u] >= 0) Z.flat[atomicAdd(&s_off[c[u]], 1u)] = (uint32_t)(j0 + u * nt + t);
    }
}

// Frame S.frame of a batched launch: camera cams.c[frame], RtTri at
// tc + frame * n_tris, masks at lat_masks + frame * tiles, output at
// out + frame * out_stride.
// PITCH: the LDS row pitch of the lattice, kLatW (shared columns) or kLatWY
// (per-pixel columns; rt_lattice_ok).
template <int PITCH>
__device__ __forceinline__ void lattice_body(const RtFrame &F0, const RtTri *__restrict__ tc,
                                             const RtShade *__restrict__ shade, const RtSphere *__restrict__ sph,
                                             const unsigned long long *__restrict__ lat_masks, const RtFrameCams &cams,
                                             size_t out_stride, uint32_t *__restrict__ out, const LatSlot &S,
                                             const LatReady &R)
{
    const int frame = S.frame;
    RtFrame F = F0;
#pragma unroll
    for (int c = 0; c < 4; ++c) F.cam[c] = cams.c[frame][c];
    tc += (size_t)frame * F.n_tris;
    lat_masks += (size_t)frame * lat_tiles_x(F) * gridDim.y * 2;
    const LatOut o = lat_out(F, frame, out_stride, out);
    // (wave as a uniform SGPR value -- readfirstlane -- measured 5 % slower here: 0.913 -> 0.960 ms
    // per 20-frame launch, more VGPRs and SGPRs; the yawed form 0.7 % faster; profiles/r05_ab_walk.json)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int by = S.by, bx = F.tx0 + S.bx;
    LatTile G = lat_tile(F, bx, by);
    G.yaw = PITCH != kLatW;   // the launch's choice (lat_yaw), a constant here
    lat_store_outside(F, G, o, S.bx);
    const int ay0 = G.ay0, cols = G.cols, rows = G.rows;
    // per lattice point: .w = hit index bits (INT_MIN: no hit); .x = t after
    // pass 1, .xyz = DirectLight after pass 2 (one ds_read_b128 per sample).
    // Per-pixel columns (PITCH 48, CG_LAT_SOA): the three values and the hit
    // index (int8, kLatSoaNoHit: none) in separate arrays, 13 bytes a point
    // instead of 16, so that seven workgroups fit a CU's LDS instead of five.
    constexpr bool kSoA = CG_LAT_SOA && PITCH == kLatWY;
    __shared__ float4 s_pt[kSoA ? 1 : PITCH * kLatH];
    __shared__ float s_v[kSoA ? 3 : 1][kSoA ? PITCH * kLatH : 1];
    __shared__ int8_t s_h[kSoA ? PITCH * kLatH : 1];
    __shared__ LatObj s_obj[kLatSphSlot + kLatMaxSph];
    __shared__ uint32_t s_px[kLatTileH * kLatTileW];
    lat_load_objs(s_obj, shade, sph, F.n_tris, F.n_sph);
    // the needed points, walked row-major at the full pitch; wave w takes the
    // w-th quarter
    const int npts = PITCH * rows;
#if CG_LAT_INTERLEAVE
    // 64-point chunks dealt round-robin to the four waves (pass 1: pairs of
    // chunks): hits and shadow tests are spatially clustered, so contiguous
    // quarters leave some waves idle at the barrier.  Pass 2 walks the same
    // points as the wave's pass 1 (no barrier between them).
    // shared columns: four points per lane per step, 256 apart -- the wave's 64-point chunks w,
    // w + 4, w + 8, .. -- each walked triangle's constants loaded once for four rays (lattice
    // kernel 0.930 -> 0.913 ms per 20-frame launch, 66 VGPRs, 90 SGPRs); the per-pixel-column
    // form keeps two per lane in pairs of chunks (four measured 2.48 -> 2.54 ms there)
    constexpr bool kNP4 = PITCH == kLatW;
    const int p_lo = kNP4 ? wave * 64 : wave * 128, p_hi = npts, step1 = kNP4 ? 1024 : 512;
#else
    constexpr bool kNP4 = false;
    const int q = (npts + 3) / 4, p_lo = min(npts, wave * q), p_hi = min(npts, p_lo + q);
    const int step1 = 128;
#endif
    if (G.u0 + G.nu <= o.wc0 || G.u0 >= o.wc0 + o.pitch) return;   // outside the RGB24 window: whole workgroup
    // Certificates published beside this launch (LatReady): wait for the tile's
    // super-tile, or take the uncertified path.
    bool certified = true;
    if (R.flags) {
        __shared__ int s_cert;
        if (threadIdx.x == 0) {
            int ok = 0;
            if (!R.force) {
                const uint32_t *w = R.flags + (size_t)frame * R.units + (by / kSup) * R.sx + bx / kSup;
                const unsigned long long t0 = wall_clock64();
                for (;;) {
                    const uint32_t v = __hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                    if (v == R.gen) {
                        ok = 1;
                        break;
                    }
                    if (wall_clock64() - t0 > R.spin) break;
                    __builtin_amdgcn_s_sleep(2);
                }
            }
            s_cert = ok;
        }
        __syncthreads();
        certified = s_cert != 0;
        if (!certified) {   // the frame's RtTri from the scene's constants, as the certificates store it
            if ((int)threadIdx.x < F.n_tris)
                R.tc[(size_t)frame * F.n_tris + threadIdx.x] = rt_tri_frame(R.geo[threadIdx.x], F.cam);
            __threadfence();
            __syncthreads();
        }
        // the loads of the constants and masks below stay after the acquire and the
        // barrier (fences order them for the compiler as well).  An opaque pointer
        // here would cost the scalar loads of RtTri (68 -> 80 VGPRs).  Scalar-cache
        // lines of this frame's RtTri are only ever fetched after a publication (or
        // this workgroup's own stores), and every RtTri of a frame is stored before
        // any of its super-tiles is published, so no stale line can be read.
    }
    // the tile's certificates (rt_prepare_kernel): primary mask (bit 63: the
    // sphere may be hit; bit 62: covered) and shadow mask for every hit the
    // tile can produce; uncertified: every triangle and sphere, not covered
    const size_t tix = (size_t)by * lat_tiles_x(F) + bx;
    const unsigned long long all = ((1ull << F.n_tris) - 1ull) | (F.n_sph > 0 ? (1ull << 63) : 0ull);
    const unsigned long long m0 = certified ? uniform_u64(lat_masks[2 * tix]) : all;
    const unsigned long long s0 = certified ? uniform_u64(lat_masks[2 * tix + 1]) : all;
    const unsigned long long mask = m0 & ~(3ull << 62), smask = s0 & ~(1ull << 63);
    const bool covered = (m0 >> 62) & 1ull;
    RtFrame Fp = F;                        // pass 1: spheres only where one may be hit
    if (!(m0 >> 63)) Fp.n_sph = 0;
    RtFrame Fs = F;                        // pass 2: spheres only where one may block a shadow ray
    if (!(s0 >> 63)) Fs.n_sph = 0;
    if (m0 == 0ull) {
        lat_store_black(F, G, o);
        return;                            // the whole workgroup (m0 is uniform)
    }
    __syncthreads();                       // s_obj
    auto stt = [&](int p, float t, int bi) {
        if constexpr (kSoA) {
            s_v[0][p] = t;
            s_h[p] = (int8_t)(bi == INT_MIN ? kLatSoaNoHit : bi);
        } else {
            s_pt[p] = make_float4(t, 0.0f, 0.0f, __int_as_float(bi));
        }
    };
    if constexpr (kNP4)
        lat_closest<PITCH, decltype(stt), 4>(Fp, tc, sph, mask, covered, G, p_lo, p_hi, lane, stt, step1, 256);
    else
        lat_closest<PITCH>(Fp, tc, sph, mask, covered, G, p_lo, p_hi, lane, stt, step1);
    // Pass 2: DirectLight of each lattice ray that hit (:151-153); shading
    // attributes from the LDS table
    for (int pc = 0; p_lo + pc < p_hi; pc += 64) {
        // the chunks of this wave's pass 1
        const int p0 = kNP4 ? p_lo + 4 * pc : p_lo + (pc / 128) * step1 + (pc % 128);
        if (p0 >= p_hi) break;
        const int p = p0 + lane;
        const int cy = p / PITCH, cx = p - cy * PITCH, idx = p;
        if (p < p_hi && cx < cols) {
            float t;
            int bi;
            if constexpr (kSoA) {
                const int h = s_h[idx];
                bi = h == kLatSoaNoHit ? INT_MIN : h;
                t = s_v[0][idx];
            } else {
                const float4 q = s_pt[idx];
                bi = __float_as_int(q.w);
                t = q.x;
            }
            if (bi != INT_MIN) {
                const float X = lat_x(F, G, cx), Y = 0.5f * (float)(ay0 + cy);
                const vec3 pos = v3(F.cam[0] + t * X, F.cam[1] + t * Y, F.cam[2] + t * F.focal);
                const vec3 dl = lat_direct_light(Fs, tc, sph, s_obj, F.lights[0], bi, pos, smask);
                if constexpr (kSoA) {
                    s_v[0][idx] = dl.x;
                    s_v[1][idx] = dl.y;
                    s_v[2][idx] = dl.z;
                } else {
                    s_pt[idx] = make_float4(dl.x, dl.y, dl.z, __int_as_float(bi));
                }
            }
        }
    }
    __syncthreads();
    // Pixels: the nine contributions in the reference's order (:134-166)
    const int tx = threadIdx.x % kLatTileW, ty = threadIdx.x / kLatTileW;
    uint32_t px = 0u;
    if (tx < G.nu && ty < G.nv) {
        vec3 pc = v3(0.0f, 0.0f, 0.0f);
        bool valid = false;
        const vec3 ind = v3(F.indirect, F.indirect, F.indirect);
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int i = k / 3 - 1, j = k % 3 - 1;
            const int idx = (2 * ty + 1 + j) * PITCH + ((G.yaw ? 3 : 2) * tx + 1 + i);
            int bi;
            vec3 dl;
            if constexpr (kSoA) {
                const int h = s_h[idx];
                bi = h == kLatSoaNoHit ? INT_MIN : h;
                dl = v3(s_v[0][idx], s_v[1][idx], s_v[2][idx]);
            } else {
                const float4 q = s_pt[idx];
                bi = __float_as_int(q.w);
                dl = v3(q.x, q.y, q.z);
            }
            if (bi == INT_MIN) continue;
            valid = true;
            pc = pc + dl;                                                                 // :151-153
            pc = pc + (lat_colour(s_obj, bi) * ind);                                      // :156
        }
        px = valid ? put_pixel(div_const(pc, 9.0f, 1.0f / 9.0f)) : put_pixel(v3(0.0f, 0.0f, 0.0f));   // :160-166
    }
    lat_store(F, G, o, px, tx, ty, s_px);
}

// ---------------------------------------------------------------------------
// Lattice form of Draw for a light set (C4's 8 x 8 area light: 2..64 lights),
// described for the unrotated camera (per-pixel columns under a yaw: column c
// folds into pixel c/3 alone).  A pixel forms
//   pc = (((0 + DL(s0, l0)) + DL(s0, l1)) + ... + DL(s0, l_last)) + amb(s0) + DL(s1, l0) ...
// (:134-157): each lattice ray's per-light values are pixel-independent, but
// their sum is not -- float addition is ordered -- so a pixel needs every
// (sub-ray, light) value individually, in order.  Pixel (tx, ty)'s sub-rays
// are lattice points (2tx + 1 + i, 2ty + 1 + j), i outer: in column-major
// order they INCREASE (column first, then row).  So the tile sweeps its lattice
// columns left to right: step c computes DirectLight of every point of column
// c for every light into an LDS column buffer (all 256 threads, one (point,
// light) pair each), and the next step -- while column c + 1 is being
// computed into the other buffer -- 48 lanes fold column c into the pixels
// that use it (an even column is the first column of pixel c/2 and the last
// of pixel c/2 - 1, an odd one the middle column of pixel (c - 1)/2), one lane
// per (pixel, component), adding the column's three points in row order, each
// point's lights in order and then its ambient term.  Every sum is the
// reference's sum; each (point, light) pair is computed once instead of for
// up to four pixels (1023 points for 240 pixels instead of 2160 sub-rays).
// The tile's 15 pixel rows are swept in thirds (pixel rows 0-4, 5-9, 10-14;
// the lattice rows between two thirds are computed by both) so the column
// buffers stay small (2 x 11 rows x 3 x 64 floats): 28.2 KB of LDS per
// workgroup, 5 workgroups (waves per SIMD) per CU -- halves (17 rows, 40 KB)
// allowed 4 and ran 4 % slower; quarters (9 rows, 25.4 KB) allow 6 and ran
// 6 % slower (the shared rows cost more than the sixth wave gains), fifths
// 10 % slower.  The per-unit shadow certificates run in a kernel of their own
// (rt_lattice_units_kernel): inside this one their FP64 work needed ~120
// VGPRs and spilled 112 B per lane at 5 waves.
// Whether triangle c stays a shadow candidate for hits in [lo, hi] of camera
// rays (X, [y0, y1], focal) towards the frame's light set: cull_shadow, and
// when every hit lies on c (own) the own-triangle certificate.
__device__ __forceinline__ bool lat_unit_keeps(const RtFrame &F, const RtTri &c, const LatObj &sh, bool own, float X,
                                            float y0, float y1, const float (&lo)[3], const float (&hi)[3])
{
    if (cull_shadow(c, v3(F.lc[0], F.lc[1], F.lc[2]), F.lrho, shadow_box_of_range(F, lo, hi))) return false;
    if (!own) return true;
    PrimDet pd;
    double tlo, thi;
    if (cull_primary(c, X, X, y0, y1, F.focal, &pd) || !primary_t_range(c, pd, tlo, thi)) return true;
    cg_tri T{};
    T.v0.x = c.v0x; T.v0.y = c.v0y; T.v0.z = c.v0z;
    T.normal.x = sh.x; T.normal.y = sh.y; T.normal.z = sh.z;
    const double Lp[3] = {(double)F.lc[0], (double)F.lc[1], (double)F.lc[2]};
    return !own_shadow_rejects(T, c, pd, thi, F.cam, X, X, y0, y1, F.focal, Lp, F.lrho, lo, hi);
}

constexpr int kLatHalfH = 5;                        // pixel rows per part (sweep)
constexpr int kLatHalfRows = 2 * kLatHalfH + 1;     // lattice rows per part
constexpr int kLatParts = (kLatTileH + kLatHalfH - 1) / kLatHalfH;
constexpr int kLatMaxLights = 64;
// Column-buffer swizzle: light l of (row r, component c) sits at slot
// l ^ lat_swz(r, c).  The folding lanes read the same light group of 24
// different (r, c) rows at once; rows 64 floats apart would all hit one LDS
// bank, the xor spreads them over 16 float4 slots.  It keeps groups of four
// lights contiguous and in order, so one ds_read_b128 still yields l .. l + 3.
__device__ __forceinline__ int lat_swz(int r, int c) { return 4 * ((r * 3 + c) & 15); }

// The tile state both light-set kernels start from: the frame's camera, the
// tile, its certificates (rt_prepare_kernel) and pass 1 (the closest hit of
// every needed lattice point) in s_t / s_bi (kLatNoHit: no hit).  False: the tile is done (outside the
// RGB24 window, or certified black -- then stored black when store_black).
constexpr int kLatNoHit = -128;   // s_bi: hit indices are -kLatMaxSph .. 62
// A unit's sole hit object (rt_lattice_units_kernel): outside the hit-index
// range too, since sphere q's hits are stored as -1 - q (-1 .. -kLatMaxSph).
constexpr int kUnitNone = -128, kUnitSeveral = -127;
static_assert(-kLatMaxSph > kUnitSeveral, "unit markers clash with sphere hit indices");
struct LatLightsTile {
    RtFrame F, Fs;
    LatTile G;
    LatOut o;
    unsigned long long smask;
    size_t tix;
    int nhalf;
};
template <int PITCH>
__device__ __forceinline__ bool lat_lights_tile(const RtFrame &F0, const RtTri *__restrict__ &tc,
                                                const RtShade *__restrict__ shade, const RtSphere *__restrict__ sph,
                                                const unsigned long long *__restrict__ lat_masks,
                                                const RtFrameCams &cams, size_t out_stride, uint32_t *out,
                                                bool store_black, float *s_t, int8_t *s_bi, LatObj *s_obj,
                                                LatLightsTile &T)
{
    const int frame = blockIdx.z;
    RtFrame &F = T.F;
    F = F0;
#pragma unroll
    for (int c = 0; c < 4; ++c) F.cam[c] = cams.c[frame][c];
    tc += (size_t)frame * F.n_tris;
    lat_masks += (size_t)frame * lat_tiles_x(F) * gridDim.y * 2;
    T.o = lat_out(F, frame, out_stride, out);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int by = lat_tile_row(), bx = lat_tile_col(F);
    LatTile &G = T.G;
    G = lat_tile(F, bx, by);
    G.yaw = PITCH != kLatW;   // the launch's choice (lat_yaw), a constant here
    if (store_black) lat_store_outside(F, G, T.o);
    lat_load_objs(s_obj, shade, sph, F.n_tris, F.n_sph);
    const int npts = PITCH * G.rows;
    const int q = (npts + 3) / 4, p_lo = min(npts, wave * q), p_hi = min(npts, p_lo + q);
    if (G.u0 + G.nu <= T.o.wc0 || G.u0 >= T.o.wc0 + T.o.pitch) return false;   // outside the RGB24 window
    T.tix = (size_t)by * lat_tiles_x(F) + bx;
    const unsigned long long m0 = uniform_u64(lat_masks[2 * T.tix]);
    const unsigned long long s0 = uniform_u64(lat_masks[2 * T.tix + 1]);
    const unsigned long long mask = m0 & ~(3ull << 62);
    T.smask = s0 & ~(1ull << 63);
    const bool covered = (m0 >> 62) & 1ull;
    RtFrame Fp = F;
    if (!(m0 >> 63)) Fp.n_sph = 0;
    T.Fs = F;
    if (!(s0 >> 63)) T.Fs.n_sph = 0;
    T.nhalf = (G.nv + kLatHalfH - 1) / kLatHalfH;
    if (m0 == 0ull) {
        if (store_black) lat_store_black(F, G, T.o);
        return false;
    }
    __syncthreads();                       // s_obj
    // (work counts: the sweep's pass 1, not the units kernel's repeat of it)
    lat_closest<PITCH>(Fp, tc, sph, mask, covered, G, p_lo, p_hi, lane, [&](int p, float t, int bi) {
        s_t[p] = t;
        s_bi[p] = (int8_t)(bi == INT_MIN ? kLatNoHit : bi);
    }, 128, 64, store_black);
    return true;
}

// Shadow candidates per (part, column) unit of a light-set tile, from
// rt_lattice_units_kernel to rt_lattice_lights_kernel: [frame][tile][part][PITCH].
template <int PITCH>
__host__ __device__ constexpr int lat_unit_slots() { return kLatParts * PITCH; }

// The unit masks in HBM.  Each is a subset of its tile's shadow mask (plus
// bit 63, a sphere may block), so a tile with few candidates stores its units
// as codes in a byte array [frame][tile][slot]: with at most kUnitNibble
// candidates a unit is a nibble (bit i: the tile's i-th candidate is kept, bit
// 3: the sphere flag; units 2j and 2j + 1 share byte j), with at most
// kUnitNarrow a byte (sphere flag bit 7); a wider tile stores the units'
// 64-bit masks in the array that follows (8-byte aligned).  A tile with no
// candidate triangle and no sphere that may block (every unit mask 0) stores
// and reads nothing.  C4's tiles have 0-5 candidates.
constexpr int kUnitNibble = 3, kUnitNarrow = 7;
__device__ __forceinline__ bool lat_units_empty(unsigned long long smask, const RtFrame &Fs)
{
    return smask == 0ull && Fs.n_sph == 0;
}
template <int PITCH>
__device__ __forceinline__ size_t lat_unit_index(const RtFrame &F, size_t tix)
{
    return ((size_t)blockIdx.z * lat_tiles_x(F) * gridDim.y + tix) * lat_unit_slots<PITCH>() + threadIdx.x;
}
template <int PITCH>
__device__ __forceinline__ size_t lat_unit_wide_bytes(const RtFrame &F)   // byte offset of the 64-bit array
{
    const size_t n = (size_t)gridDim.z * lat_tiles_x(F) * gridDim.y * lat_unit_slots<PITCH>();
    return (n + 7) & ~(size_t)7;
}
__device__ __forceinline__ uint32_t lat_unit_code(unsigned long long um, unsigned long long smask, int sb)
{
    uint32_t c = (uint32_t)(um >> 63) << sb;
    int i = 0;
    for (unsigned long long m = smask; m; m &= m - 1ull, ++i)
        if (um & (m & (0ull - m))) c |= 1u << i;
    return c;
}
__device__ __forceinline__ unsigned long long lat_unit_mask(uint32_t code, unsigned long long smask, int sb)
{
    unsigned long long um = (unsigned long long)((code >> sb) & 1u) << 63;
    int i = 0;
    for (unsigned long long m = smask; m; m &= m - 1ull, ++i)
        if ((code >> i) & 1u) um |= m & (0ull - m);
    return um;
}

// The unit certificates of a light-set tile: the tile's shadow mask
// re-certified over each (part, column) unit's exact hit positions (pos as
// DirectLight forms it), plus the own-triangle certificate when every hit of
// the unit lies on one triangle -- the same exact functions as
// rt_tile_cert_kernel, over a box of up to 11 points instead of the tile's.
// A kernel of its own: the FP64 certificates need ~120 VGPRs, which would
// cost the sweep (82) its fifth wave per SIMD or spill.
template <int PITCH>
__device__ __forceinline__ void lattice_units_body(const RtFrame &F0, const RtTri *__restrict__ tc,
                                                   const RtShade *__restrict__ shade,
                                                   const RtSphere *__restrict__ sph,
                                                   const unsigned long long *__restrict__ lat_masks,
                                                   const RtFrameCams &cams, unsigned long long *__restrict__ umask)
{
    __shared__ float s_t[PITCH * kLatH];                               // pass 1: t and hit index
    __shared__ int8_t s_bi[PITCH * kLatH];
    __shared__ LatObj s_obj[kLatSphSlot + kLatMaxSph];
    __shared__ float s_ubox[kLatParts][PITCH][6];                     // the units' hit boxes
    __shared__ int s_uone[kLatParts][PITCH];                          // sole hit object (kUnitSeveral / kUnitNone)
    __shared__ unsigned long long s_umask[kLatParts][PITCH];
    static_assert(kLatParts * PITCH <= kRtThreads, "a thread per unit");
    LatLightsTile T;
    // black tiles are stored by the sweep kernel; no output here
    if (!lat_lights_tile<PITCH>(F0, tc, shade, sph, lat_masks, cams, 0, nullptr, false, s_t, s_bi, s_obj, T)) return;
    const RtFrame &F = T.F;
    const LatTile &G = T.G;
    const int ay0 = G.ay0, cols = G.cols, nhalf = T.nhalf;
    const unsigned long long smask = T.smask;
    __syncthreads();
    if (threadIdx.x < kLatParts * PITCH) {
        const int h = threadIdx.x / PITCH, cx = threadIdx.x - h * PITCH;
        if (h < nhalf && cx < cols) {
            const int lr0 = 2 * h * kLatHalfH, nlr = 2 * min(kLatHalfH, G.nv - h * kLatHalfH) + 1;
            LanePosBox pb;
            pb.init();
            int one = kUnitNone;
            const float X = lat_x(F, G, cx);
            for (int r = 0; r < nlr; ++r) {
                const int bi = s_bi[(lr0 + r) * PITCH + cx];
                if (bi == kLatNoHit) continue;
                const float Y = 0.5f * (float)(ay0 + lr0 + r), t = s_t[(lr0 + r) * PITCH + cx];
                pb.add(v3(F.cam[0] + t * X, F.cam[1] + t * Y, F.cam[2] + t * F.focal));
                one = (one == kUnitNone || one == bi) ? bi : kUnitSeveral;
            }
            for (int k = 0; k < 3; ++k) {
                s_ubox[h][cx][k] = pb.lo[k];
                s_ubox[h][cx][3 + k] = pb.hi[k];
            }
            s_uone[h][cx] = one;
            s_umask[h][cx] = 0ull;
        }
    }
    __syncthreads();
    const int nc = __popcll(smask), pairs = nhalf * PITCH * nc;
    for (int it = threadIdx.x; it < pairs; it += kRtThreads) {
        const int unit = it / nc, ci = it - unit * nc;
        const int h = unit / PITCH, cx = unit - h * PITCH;
        if (cx >= cols) continue;
        const int one = s_uone[h][cx];
        if (one == kUnitNone) continue;   // no hit, no shadow ray
        const int k = nth_bit(smask, ci);
        const float lo[3] = {s_ubox[h][cx][0], s_ubox[h][cx][1], s_ubox[h][cx][2]};
        const float hi[3] = {s_ubox[h][cx][3], s_ubox[h][cx][4], s_ubox[h][cx][5]};
        const int lr0 = 2 * h * kLatHalfH, nlr = 2 * min(kLatHalfH, G.nv - h * kLatHalfH) + 1;
        const float X = lat_x(F, G, cx);
        const float y0 = 0.5f * (float)(ay0 + lr0), y1 = 0.5f * (float)(ay0 + lr0 + nlr - 1);
        if (lat_unit_keeps(F, tc[k], s_obj[k], one == k, X, y0, y1, lo, hi))
            atomicOr(&s_umask[h][cx], 1ull << k);
    }
    // bit 63: a sphere may block a shadow ray of the unit -- the sphere-shadow
    // certificate of every light over the unit's hit box (the tile's flag,
    // rt_tile_cert_kernel, covers the whole tile)
    const int spairs = T.Fs.n_sph > 0 ? nhalf * PITCH * F.n_lights : 0;
    for (int it = threadIdx.x; it < spairs; it += kRtThreads) {
        const int unit = it / F.n_lights, l = it - unit * F.n_lights;
        const int h = unit / PITCH, cx = unit - h * PITCH;
        if (cx >= cols || s_uone[h][cx] == kUnitNone) continue;
        const float lo[3] = {s_ubox[h][cx][0], s_ubox[h][cx][1], s_ubox[h][cx][2]};
        const float hi[3] = {s_ubox[h][cx][3], s_ubox[h][cx][4], s_ubox[h][cx][5]};
        const RtLight Lt = F.lights[l];
        const double Lp[3] = {(double)Lt.x, (double)Lt.y, (double)Lt.z};
        bool may = false;
        for (int q = 0; q < T.Fs.n_sph && !may; ++q) may = !sphere_shadow_surely_missed(sph[q], Lp, lo, hi);
        if (may) atomicOr(&s_umask[h][cx], 1ull << 63);
    }
    __syncthreads();
    constexpr int kSlots = kLatParts * PITCH;
    if (lat_units_empty(smask, T.Fs)) return;
    const size_t ui = lat_unit_index<PITCH>(F, T.tix);
    if (nc <= kUnitNibble) {   // units 2j, 2j + 1 -> byte j (units outside the tile: 0)
        const int j = threadIdx.x;
        if (2 * j < kSlots) {
            uint32_t b = 0u;
            for (int e = 0; e < 2; ++e) {
                const int u = 2 * j + e, h = u / PITCH, cx = u - h * PITCH;
                if (u < kSlots && h < nhalf && cx < cols) b |= lat_unit_code(s_umask[h][cx], smask, 3) << (4 * e);
            }
            ((uint8_t *)umask)[ui - threadIdx.x + j] = (uint8_t)b;
        }
    } else if (threadIdx.x < kSlots) {
        const int h = threadIdx.x / PITCH, cx = threadIdx.x - h * PITCH;
        if (h < nhalf && cx < cols) {
            if (nc <= kUnitNarrow)
                ((uint8_t *)umask)[ui] = (uint8_t)lat_unit_code(s_umask[h][cx], smask, 7);
            else
                ((unsigned long long *)((uint8_t *)umask + lat_unit_wide_bytes<PITCH>(F)))[ui] = s_umask[h][cx];
        }
    }
}

template <int PITCH>
__device__ __forceinline__ void lattice_lights_body(const RtFrame &F0, const RtTri *__restrict__ tc,
                                                    const RtShade *__restrict__ shade,
                                                    const RtSphere *__restrict__ sph,
                                                    const unsigned long long *__restrict__ lat_masks,
                                                    const unsigned long long *__restrict__ umask,
                                                    const RtFrameCams &cams, size_t out_stride,
                                                    uint32_t *__restrict__ out)
{
    __shared__ float s_t[PITCH * kLatH];                              // pass 1: t and hit index
    __shared__ int8_t s_bi[PITCH * kLatH];
    __shared__ LatObj s_obj[kLatSphSlot + kLatMaxSph];
    __shared__ float s_dl[2][kLatHalfRows][3][kLatMaxLights];         // column buffers
    // pixel sums of the current part only: a part's pixels are resolved when
    // its sweep ends, into s_px = the start of s_t, whose lattice rows of
    // finished parts are dead (part h's pixels land in floats 80 h .. 80 h + 79,
    // rows < 10 h + 10 for both pitches).  2.2 KB less LDS than whole-tile
    // sums: six workgroups per CU instead of five.
    __shared__ float s_pc[kLatHalfH][kLatTileW][3];
    __shared__ uint8_t s_valid[kLatHalfH][kLatTileW];
    static_assert(kLatHalfH * kLatTileW * kLatParts <= 2 * kLatHalfH * 33, "s_px overlaps a live lattice row");
    uint32_t *s_px = (uint32_t *)s_t;
    __shared__ unsigned long long s_umask[kLatParts][PITCH];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    LatLightsTile T;
    if (!lat_lights_tile<PITCH>(F0, tc, shade, sph, lat_masks, cams, out_stride, out, true, s_t, s_bi, s_obj, T)) return;
    const RtFrame &F = T.F, &Fs = T.Fs;
    const LatTile &G = T.G;
    const int ay0 = G.ay0, cols = G.cols;
    {
        const int tx = threadIdx.x % kLatTileW, ty = threadIdx.x / kLatTileW;
        if (ty < kLatHalfH) {
            s_pc[ty][tx][0] = s_pc[ty][tx][1] = s_pc[ty][tx][2] = 0.0f;
            s_valid[ty][tx] = 0;
        }
        // the units' shadow candidates (rt_lattice_units_kernel)
        if (threadIdx.x < kLatParts * PITCH) {
            const int h = threadIdx.x / PITCH, cx = threadIdx.x - h * PITCH;
            if (h < T.nhalf && cx < cols) {
                const size_t ui = lat_unit_index<PITCH>(F, T.tix);
                const int nc = __popcll(T.smask);
                const uint8_t *code = (const uint8_t *)umask;
                s_umask[h][cx] =
                    lat_units_empty(T.smask, Fs) ? 0ull
                    : nc <= kUnitNibble
                        ? lat_unit_mask(code[ui - threadIdx.x + threadIdx.x / 2] >> (4 * (threadIdx.x & 1)), T.smask, 3)
                    : nc <= kUnitNarrow
                        ? lat_unit_mask(code[ui], T.smask, 7)
                        : ((const unsigned long long *)(code + lat_unit_wide_bytes<PITCH>(F)))[ui];
            }
        }
    }
    __syncthreads();
    const int nL = F.n_lights;
    const float ind = F.indirect;
    const bool fixed_l = 64 % nL == 0;
    const int my_l = lane % nL, r_stride = kRtThreads / nL;
    const RtLight my_light = F.lights[my_l];
    // folding lanes: lane = 24 k + 3 pr + comp (k = 0: the pixel whose first
    // or middle column this is, k = 1: the pixel whose last column it is)
    const int fk = lane / 24, fpr = (lane % 24) / 3, fcomp = lane % 3;
#ifdef CG_WALK_STATS
    int st_units = 0, st_cand = 0, st_sph = 0;
#endif
    for (int h = 0; h * kLatHalfH < G.nv; ++h) {
        const int pr0 = h * kLatHalfH, npr = min(kLatHalfH, G.nv - pr0);
        const int lr0 = 2 * pr0, nlr = 2 * npr + 1, items = nlr * nL;
        for (int step = 0; step <= cols; ++step) {
            // roles rotate over the waves step by step (logical wave lw): the
            // wave with lw = 0 takes the odd 17th row, lw = 3 also folds, so
            // every SIMD of the CU carries the same load over a sweep
            const int lw = (wave + step) & 3, lt = lw * 64 + lane;
            const bool folder = lw == 3 && lane < 48;
            if (step < cols) {   // DirectLight of column `step`, every light (:151-153, :366-415)
                const int cx = step;
                const unsigned long long um0 = uniform_u64(s_umask[h][cx]);
                const unsigned long long um = um0 & ~(1ull << 63);
#ifdef CG_WALK_STATS
                st_units += 1;
                st_cand += __popcll(um);
                st_sph += (int)(um0 >> 63);
#endif
                RtFrame Fu = Fs;                      // spheres only where one may block
                if (!(um0 >> 63)) Fu.n_sph = 0;
                const float X = lat_x(F, G, cx);
                auto item = [&](int r, int l, const RtLight &Lt) {
                    const int cy = lr0 + r;
                    const int bi = s_bi[cy * PITCH + cx];
                    if (bi == kLatNoHit) return;
                    const float Y = 0.5f * (float)(ay0 + cy), t = s_t[cy * PITCH + cx];
                    const vec3 pos = v3(F.cam[0] + t * X, F.cam[1] + t * Y, F.cam[2] + t * F.focal);
                    const vec3 dl = lat_direct_light<true>(Fu, tc, sph, s_obj, Lt, bi, pos, um);
                    float *b = &s_dl[step & 1][r][0][0];
                    b[l ^ lat_swz(r, 0)] = dl.x;
                    b[kLatMaxLights + (l ^ lat_swz(r, 1))] = dl.y;
                    b[2 * kLatMaxLights + (l ^ lat_swz(r, 2))] = dl.z;
                };
                if (fixed_l) {   // nL divides 64: each thread keeps one light (in registers)
                    for (int r = lt / nL; r < nlr; r += r_stride) item(r, my_l, my_light);
                } else {
                    for (int it = lt; it < items; it += kRtThreads) {
                        const int r = it / nL, l = it - r * nL;
                        item(r, l, F.lights[l]);
                    }
                }
            }
            if (step > 0 && folder) {   // fold column step - 1 into its pixels
                const int cx = step - 1;
                // shared columns: an even column is the first of pixel cx/2 and
                // the last of cx/2 - 1; per-pixel columns: column cx is pixel cx/3's
                const int tx = G.yaw ? cx / 3 : (fk == 0 ? cx / 2 : cx / 2 - 1);
                const bool use = fpr < npr && tx >= 0 && tx < G.nu && (fk == 0 || (!G.yaw && (cx & 1) == 0));
                if (use) {
                    const int ty = fpr;   // row of the part
                    float pc = s_pc[ty][tx][fcomp];
                    bool valid = false;
                    const float *buf = &s_dl[cx & 1][0][0][0];
                    for (int j = 0; j < 3; ++j) {
                        const int r = 2 * fpr + j;
                        const int bi = s_bi[(lr0 + r) * PITCH + cx];
                        if (bi == kLatNoHit) continue;
                        valid = true;
                        const float *b = buf + (r * 3 + fcomp) * kLatMaxLights;
                        const int sw = lat_swz(r, fcomp);
                        int l = 0;
                        for (; l + 4 <= nL; l += 4) {   // lights l .. l + 3, in order
                            const float4 v = *(const float4 *)(b + (l ^ sw));
                            pc = pc + v.x;
                            pc = pc + v.y;
                            pc = pc + v.z;
                            pc = pc + v.w;
                        }
                        for (; l < nL; ++l) pc = pc + b[l ^ sw];
                        const vec3 oc = lat_colour(s_obj, bi);                    // :147-148
                        const float a = fcomp == 0 ? oc.x : (fcomp == 1 ? oc.y : oc.z);
                        pc = pc + (a * ind);                                      // :156
                    }
                    s_pc[ty][tx][fcomp] = pc;
                    if (valid && fcomp == 0) s_valid[ty][tx] = 1;
                }
            }
            __syncthreads();
        }
        // the part's pixels (:160-166); their sums are then cleared for the
        // next part, whose first fold comes after its step 0's barrier
        const int tx = threadIdx.x % kLatTileW, ty = threadIdx.x / kLatTileW;
        if (ty < kLatHalfH) {
            if (ty < npr) {
                const vec3 pc = v3(s_pc[ty][tx][0], s_pc[ty][tx][1], s_pc[ty][tx][2]);
                s_px[(pr0 + ty) * kLatTileW + tx] =
                    s_valid[ty][tx] ? put_pixel(div_const(pc, 9.0f, 1.0f / 9.0f)) : put_pixel(v3(0.0f, 0.0f, 0.0f));
            }
            s_pc[ty][tx][0] = s_pc[ty][tx][1] = s_pc[ty][tx][2] = 0.0f;
            s_valid[ty][tx] = 0;
        }
    }
#ifdef CG_WALK_STATS
    if (threadIdx.x == 0 && blockIdx.z == 0 && blockIdx.x % 24 == 0 && blockIdx.y % 24 == 0)
        printf("LIGHTS bx %d by %d units %d cand %d sph %d\n", blockIdx.x, blockIdx.y, st_units, st_cand, st_sph);
#endif
    __syncthreads();
    const int tx = threadIdx.x % kLatTileW, ty = threadIdx.x / kLatTileW;
    const uint32_t px = (tx < G.nu && ty < G.nv) ? s_px[ty * kLatTileW + tx] : 0u;
    lat_store(F, G, T.o, px, tx, ty, (uint32_t *)&s_dl[0][0][0][0]);
}

// The kernels.  frame_done (optional, cg_dist's transfer pipeline): when a
// workgroup's tile is stored, frame_done[frame] counts it -- every wave first
// writes its stores back (__threadfence: agent-scope release, L2 write-back
// across the XCDs), then one lane adds -- so a stream that waits for a
// frame's count to reach its tile count (hipStreamWaitValue32) may read the
// frame while the launch is still rendering later frames.
__device__ __forceinline__ void lat_signal(uint32_t *frame_done, int frame)
{
    if (!frame_done) return;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(&frame_done[frame], 1u);
}

template <int PITCH>
__global__ __launch_bounds__(kRtThreads, kRtMinWaves) void rt_lattice_kernel(RtFrame F0, const RtTri *__restrict__ tc,
                                                                  const RtShade *__restrict__ shade,
                                                                  const RtSphere *__restrict__ sph,
                                                                  const unsigned long long *__restrict__ lat_masks,
                                                                  RtFrameCams cams, size_t out_stride,
                                                                  uint32_t *__restrict__ out, uint32_t *frame_done,
                                                                  LatOrder O, LatReady R)
{
#ifdef CG_WG_TIMING
    const unsigned long long wt0 = wall_clock64();
#endif
    const unsigned long long t_start = wall_clock64();
    const LatSlot S = lat_slot_of(O);
    lattice_body<PITCH>(F0, tc, shade, sph, lat_masks, cams, out_stride, out, S, R);
    // the recording for the next call's order: frame 0's tiles, one class each
    if (O.cost && S.frame == 0 && threadIdx.x == 0)
        O.cost[S.by * (int)gridDim.x + S.bx] = (uint8_t)lat_cost_class(wall_clock64() - t_start);
    lat_signal(frame_done, S.frame);
#ifdef CG_WG_TIMING
    WGT_STAMP(wt3);
    wgt_record(2, wt0, wt3, wt3, wt3);
#endif
}

template <int PITCH>
// 4 waves/SIMD: 128 VGPRs, 36 B of scratch (unbounded it took 137 VGPRs, 3 waves): C4 97.95 ->
// 98.5 fps; 5 waves (136 B) the same (profiles/r06_ab_session2.json)
#ifndef CG_UNITS_WAVES
#define CG_UNITS_WAVES 4
#endif
__global__ __launch_bounds__(kRtThreads, CG_UNITS_WAVES) void rt_lattice_units_kernel(RtFrame F0, const RtTri *__restrict__ tc,
                                                                      const RtShade *__restrict__ shade,
                                                                      const RtSphere *__restrict__ sph,
                                                                      const unsigned long long *__restrict__ lat_masks,
                                                                      RtFrameCams cams,
                                                                      unsigned long long *__restrict__ umask)
{
    lattice_units_body<PITCH>(F0, tc, shade, sph, lat_masks, cams, umask);
}

template <int PITCH>
__global__ __launch_bounds__(kRtThreads, 6) void rt_lattice_lights_kernel(RtFrame F0, const RtTri *__restrict__ tc,
                                                                          const RtShade *__restrict__ shade,
                                                                          const RtSphere *__restrict__ sph,
                                                                          const unsigned long long *__restrict__ lat_masks,
                                                                          const unsigned long long *__restrict__ umask,
                                                                          RtFrameCams cams, size_t out_stride,
                                                                          uint32_t *__restrict__ out,
                                                                          uint32_t *frame_done)
{
    lattice_lights_body<PITCH>(F0, tc, shade, sph, lat_masks, umask, cams, out_stride, out);
    lat_signal(frame_done, blockIdx.z);
}

// ARGB8888 -> RGB24 wire format (kernels without a fused RGB24 store): rows
// of W pixels -> rows of the window's wcols pixels (columns wcol0 ..), four
// pixels per lane, three dwords out when aligned.
__global__ void rt_pack_rgb24_kernel(const uint32_t *__restrict__ src, int W, int rows, int wcol0, int wcols,
                                     uint8_t *__restrict__ dst)
{
    const int x = 4 * (blockIdx.x * blockDim.x + threadIdx.x), y = blockIdx.y;
    if (x >= wcols || y >= rows) return;
    const uint32_t *s = src + (size_t)y * W + wcol0 + x;
    uint8_t *d = dst + ((size_t)y * wcols + x) * 3;
    if (x + 4 <= wcols && ((uintptr_t)d & 3) == 0 && ((uintptr_t)s & 15) == 0) {
        const uint4 p = *(const uint4 *)s;
        uint32_t *dw = (uint32_t *)d;
        dw[0] = (p.x & 0xffffffu) | (p.y << 24);
        dw[1] = ((p.y >> 8) & 0xffffu) | (p.z << 16);
        dw[2] = ((p.z >> 16) & 0xffu) | ((p.w & 0xffffffu) << 8);
        return;
    }
    for (int k = 0; k < 4 && x + k < wcols; ++k) {
        const uint32_t p = s[k];
        d[3 * k] = (uint8_t)p;
        d[3 * k + 1] = (uint8_t)(p >> 8);
        d[3 * k + 2] = (uint8_t)(p >> 16);
    }
}

// Frame assembly on the gathering rank: src holds row blocks in order, block
// b = nframes x rows[b] rows of W pixels (bpp 4: ARGB8888, 3: RGB24 + alpha
// 128 restored), landing at frame rows row0[b] ...  Four pixels per lane.
__global__ void rt_assemble_kernel(const uint8_t *__restrict__ src, RtBlocks B, int nframes,
                                   uint32_t *__restrict__ frames, size_t frame_stride)
{
    const int x = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
    const int y = blockIdx.y, f = blockIdx.z;   // y: row over all blocks
    int b = 0;
    while (b + 1 < B.n && B.cum[b + 1] <= y) ++b;   // uniform
    const int l = y - B.cum[b], g = B.row0[b] + l;
    if (x >= B.W || g < 0 || g >= B.H) return;
    const size_t srow = (size_t)nframes * B.cum[b] + (size_t)f * B.rows[b] + l;   // row index in src
    uint32_t *d = frames + (size_t)f * frame_stride + (size_t)g * B.W + x;
    const int n = min(4, B.W - x);
    const int wc0 = B.wcols ? B.wcol0 : 0, pitch = B.wcols ? B.wcols : B.W;
    if (x < wc0 || x >= wc0 + pitch) {   // outside the window: PutPixelSDL(0, 0, 0)
        for (int k = 0; k < n; ++k) d[k] = 0x80000000u;
        return;
    }
    const int xs = x - wc0;              // column in the source row (windows are 4-aligned)
    if (B.bpp == 4) {
        const uint32_t *s4 = (const uint32_t *)src + srow * pitch + xs;
        if (n == 4 && ((uintptr_t)s4 & 15) == 0 && ((uintptr_t)d & 15) == 0) *(uint4 *)d = *(const uint4 *)s4;
        else for (int k = 0; k < n; ++k) d[k] = s4[k];
        return;
    }
    const uint8_t *s3 = src + (srow * pitch + xs) * 3;
    if (n == 4 && ((uintptr_t)s3 & 3) == 0 && ((uintptr_t)d & 15) == 0) {
        const uint32_t a = ((const uint32_t *)s3)[0], bb = ((const uint32_t *)s3)[1], c = ((const uint32_t *)s3)[2];
        *(uint4 *)d = make_uint4(0x80000000u | (a & 0xffffffu), 0x80000000u | (a >> 24) | ((bb & 0xffffu) << 8),
                                 0x80000000u | (bb >> 16) | ((c & 0xffu) << 16), 0x80000000u | (c >> 8));
        return;
    }
    for (int k = 0; k < n; ++k)
        d[k] = 0x80000000u | (uint32_t)s3[3 * k] | ((uint32_t)s3[3 * k + 1] << 8) | ((uint32_t)s3[3 * k + 2] << 16);
}

// Reassemble striped frames after the gather (multi-GPU path): g holds, per
// rank, `nframes` shards of rows_per_rank rows; frame f of the output is
// [f][H][W].  A pure copy (HBM-bound): 16 B per lane when rows are 16-B
// aligned (W % 4 == 0), one pixel per lane otherwise.
__global__ void rt_unstripe4_kernel(const uint4 *__restrict__ g, int W4, int H, int nranks, int stripe_h,
                                    int rows_per_rank, int nframes, uint4 *__restrict__ frames)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y, f = blockIdx.z;
    if (x >= W4) return;
    const int k = y / stripe_h, r = k % nranks;
    const int L = (k / nranks) * stripe_h + (y - k * stripe_h);
    frames[((size_t)f * H + y) * W4 + x] = g[(((size_t)r * nframes + f) * rows_per_rank + L) * W4 + x];
}

__global__ void rt_unstripe_kernel(const uint32_t *__restrict__ g, int W, int H, int nranks,
                                   int stripe_h, int rows_per_rank, int nframes, uint32_t *__restrict__ frames)
{
    int x = blockIdx.x * blockDim.x + threadIdx.x;
    int y = blockIdx.y, f = blockIdx.z;
    if (x >= W || y >= H) return;
    int k = y / stripe_h;
    int r = k % nranks;
    int L = (k / nranks) * stripe_h + (y - k * stripe_h);
    frames[((size_t)f * H + y) * W + x] = g[(((size_t)r * nframes + f) * rows_per_rank + L) * W + x];
}

// Probe kernels (known-answer tests of ClosestIntersection / DirectLight on
// arbitrary rays): generic-start form of closest_primary.
__global__ void rt_probe_closest_kernel(RtFrame F, const cg_tri *__restrict__ tris,
                                        const RtSphere *__restrict__ sph, const cg_vec4 *starts,
                                        const cg_vec4 *dirs, int n, cg_isect *out, int *hit)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    vec4 s = v4(starts[i].x, starts[i].y, starts[i].z, starts[i].w);
    vec3 d = v3(dirs[i].x, dirs[i].y, dirs[i].z);
    const float bound = FLT_MAX;
    cg_isect ci;
    ci.distance = bound;
    ci.position = cg_vec4{0, 0, 0, 0};
    ci.triangleIndex = 0;
    ci.sphereIndex = 0;
    vec3 s3 = xyz(s);
    vec3 nd = -d;
    for (int k = 0; k < F.n_tris; ++k) {
        cg_tri T = tris[k];
        vec3 e1 = v3(T.v1.x - T.v0.x, T.v1.y - T.v0.y, T.v1.z - T.v0.z);
        vec3 e2 = v3(T.v2.x - T.v0.x, T.v2.y - T.v0.y, T.v2.z - T.v0.z);
        vec3 sol = v3(s.x - T.v0.x, s.y - T.v0.y, s.z - T.v0.z);
        float det = det3(nd, e1, e2);
        float t = det3(sol, e1, e2) / det;
        float distance = t * length(d);
        if (distance < 0.0f) continue;
        if (distance >= ci.distance || distance > bound) continue;
        float uu = det3(nd, sol, e2) / det;
        float vv = det3(nd, e1, sol) / det;
        vec3 td = d * t;
        if ((uu >= 0) && (vv >= 0) && ((uu + vv) <= 1)) {
            ci.position = cg_vec4{s.x + td.x, s.y + td.y, s.z + td.z, s.w + 0};
            ci.distance = distance;
            ci.triangleIndex = k;
            ci.sphereIndex = -1;
        }
    }
    for (int k = 0; k < F.n_sph; ++k) {
        float t;
        if (sphere_intersect(sph[k], s3, d, t)) {
            vec3 td = d * t;
            if (t < ci.distance) {
                ci.position = cg_vec4{s.x + td.x, s.y + td.y, s.z + td.z, s.w + 0};
                ci.distance = t;
                ci.triangleIndex = -1;
                ci.sphereIndex = k;
            }
        }
    }
    out[i] = ci;
    hit[i] = ci.distance < bound;
}

__global__ void rt_probe_direct_light_kernel(RtFrame F, const RtTri *__restrict__ tc,
                                             const RtShade *__restrict__ shade,
                                             const RtSphere *__restrict__ sph,
                                             const cg_isect *isects, int n, cg_vec3 *out)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    cg_isect is = isects[i];
    vec3 pos = v3(is.position.x, is.position.y, is.position.z);
    int bi = is.triangleIndex != -1 ? is.triangleIndex : -1 - is.sphereIndex;
    vec3 oc;
    if (bi >= 0) oc = v3(shade[bi].cr, shade[bi].cg, shade[bi].cb);
    else oc = v3(sph[-1 - bi].cr, sph[-1 - bi].cg, sph[-1 - bi].cb);
    vec3 r = direct_light<false>(F, tc, shade, sph, bi, pos, oc, 0);
    out[i] = cg_vec3{r.x, r.y, r.z};
}

// ---------------------------------------------------------------------------
// Launch helpers (called by the shim).
// d_sup_masks (optional): two-level certificates -- super-tiles, then their
// tiles.  By default one fused rt_tile_cert_kernel launch does both levels and
// the RtTri constants (the super-tile masks stay in LDS; d_sup_masks unused);
// CG_CERT_FUSED=0 restores the two launches (rt_prepare_kernel certifies the
// super-tiles into d_sup_masks, rt_tile_cert_kernel refines them), for A/B runs.
static bool cert_fused()
{
    static const bool on = [] {
        const char *e = std::getenv("CG_CERT_FUSED");
        return !(e && e[0] == '0');
    }();
    return on;
}

static int env_int(const char *name, int dflt)
{
    const char *e = std::getenv(name);
    return e && *e ? std::atoi(e) : dflt;
}

// Once per scene (cg_rt_set_scene): RtGeo + RtShade of every triangle.
hipError_t launch_rt_scene(const cg_tri *d_tris, int n, RtGeo *d_geo, RtShade *d_shade, hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(rt_scene_kernel, dim3((n + kRtThreads - 1) / kRtThreads), dim3(kRtThreads), 0, st, d_tris, n,
                       d_geo, d_shade);
    return hipGetLastError();
}

// Z (optional): a measured lattice order to sort in the fused certificate
// launch; on return Z->n < 0 iff it was (the other certificate paths skip it).
hipError_t launch_rt_prepare(const cg_tri *d_tris, const RtGeo *d_geo, int n, const RtFrameCams &cams, int nframes,
                             RtTri *d_tc, hipStream_t st, const RtFrame *F, const RtSphere *d_sph,
                             unsigned long long *d_lat_masks, unsigned long long *d_sup_masks, LatFlatten *Z,
                             LatPublish *pub)
{
    const LatPublish P = pub ? *pub : LatPublish{};
    if (pub) pub->done = 0;
    if (n <= 0) return hipSuccess;
    const int threads = kRtThreads, prep = (n + threads - 1) / threads;
    int cert = 0;
    RtFrame Fl{};
    // A/B knobs: CG_CERT_SINGLE_MAX = window tiles x frames below which the tiles are certified
    // in one level (measured slower for bands too: 182-217 vs 174-191 us); CG_CERT_THREADS
    // forces the fused kernel's threads per super-tile.
    static const int single_max = env_int("CG_CERT_SINGLE_MAX", 0);
    static const int force_threads = env_int("CG_CERT_THREADS", 0);
    // resident 4-wave workgroups of rt_tile_cert_kernel (CG_CERT_WAVES per SIMD)
    static const int resident4 = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return cus * CG_CERT_WAVES;
    }();
    const size_t wtiles = F ? (size_t)(F->txn ? F->txn : lat_tiles_x(*F)) * (rt_cert_units(*F, 0) / lat_tiles_x(*F)) : 0;
    const int sup = (d_sup_masks && !(F && wtiles * nframes < (size_t)single_max)) ? 1 : 0;
    if (sup && F && d_lat_masks) {
        Fl = *F;
        // few super-tiles (a band of one rank): four waves per super-tile, so
        // the call's certificate latency is a quarter of one wave's chain
        // (C2, 1/8 band, 20 frames, cold: 53.9 -> 28.7 us; 8 waves 49 us; a
        // whole frame's 10800 units stay at one wave: 85 us vs 106 with four)
        const int units = rt_cert_units(*F, 1);
        if (cert_fused()) {
            // only the super-tiles over the launch's tile-column window (RtFrame::txn)
            const int sx = (lat_tiles_x(*F) + kSup - 1) / kSup, sy = units / sx;
            const int sxw = F->txn ? (F->tx0 + F->txn + kSup - 1) / kSup - F->tx0 / kSup : sx;
            const int units_w = sy * sxw;
            // waves per super-tile: four while the call's super-tiles fit one round of resident
            // workgroups (a band: the latency of each super-tile's chain is the call's), else one
            // (throughput: the bottom-first order keeps the long chains off the tail).  C2, 20
            // frames: bands of 90-188 rows have 760-1,520 super-tiles (four waves 176-185 us per
            // band call, two 169-190), the whole frame 6,840 (one wave 77-78 us, two 88, four
            // 128; in the raster order one wave took 105-111, two 100-105).
            // Round 5: two waves while they fit one round (2 x resident4 128-thread workgroups) -- the
            // 1/8 bands of 9-13 tile rows (1,140-1,520 super-tile-frames) took one wave per chain
            // before, 24-44 us of certificates for their band call.
            const size_t cnt = (size_t)units_w * nframes;
            const int tthreads = force_threads ? force_threads
                                 : cnt <= (size_t)resident4 ? 256 : cnt <= 2 * (size_t)resident4 ? 128 : 64;
            const int tprep = (n + tthreads - 1) / tthreads;
            const int kt_id = KT_RT_TILE_CERT;
            // published certificates run beside the lattice launch: frame-major, as the lattice
            // takes its tiles, so its first frames' super-tiles come first
            const int ff = !P.flags && tprep + units_w <= 65535;
            const dim3 cg = ff ? dim3(nframes, tprep + units_w) : dim3(tprep + units_w, nframes);
            kt_launch(kt_id, rt_tile_cert_kernel, cg, dim3(tthreads), 0, st, d_tris, d_geo, n, cams, Fl, d_sph,
                               (const unsigned long long *)nullptr, d_lat_masks, d_tc, tprep, ff,
                               Z ? *Z : LatFlatten{}, P);
            if (pub) pub->done = P.flags != nullptr;
            if (Z) Z->n = -Z->n;   // done (the caller's flag: the lattice launch may use the order)
            return hipGetLastError();
        }
        Fl.txn = 0;   // the split form certifies every super-tile
        const int tthreads = (size_t)units * nframes <= (size_t)resident4 ? 256 : 64;
        const int tpw = n <= 31 ? 2 : 1;   // units per wave (rt_prepare_kernel)
        cert = (units + tpw * (threads / 64) - 1) / (tpw * (threads / 64));
        {
            const int kt_id = KT_RT_PREPARE;
            kt_launch(kt_id, rt_prepare_kernel, dim3(prep + cert, nframes), dim3(threads), 0, st, d_tris, d_geo, n,
                               cams, d_tc, prep, Fl, d_sph, d_sup_masks, 1);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        const int kt_id = KT_RT_TILE_CERT;
        const int ff = units <= 65535;
        kt_launch(kt_id, rt_tile_cert_kernel, ff ? dim3(nframes, units) : dim3(units, nframes), dim3(tthreads), 0, st,
                           d_tris, d_geo, n, cams, Fl, d_sph, (const unsigned long long *)d_sup_masks, d_lat_masks,
                           (RtTri *)nullptr, 0, ff, LatFlatten{}, LatPublish{});
        return hipGetLastError();
    }
    if (F && d_lat_masks) {   // single-level: every tile (of the window) certified by rt_prepare_kernel
        Fl = *F;
        const int units = (int)wtiles;
        const int tpw = n <= 31 ? 2 : 1;
        cert = (units + tpw * (threads / 64) - 1) / (tpw * (threads / 64));
    }
    const int kt_id = KT_RT_PREPARE;
    kt_launch(kt_id, rt_prepare_kernel, dim3(prep + cert, nframes), dim3(threads), 0, st, d_tris, d_geo, n, cams,
                       d_tc, prep, Fl, d_sph, d_lat_masks, 0);
    return hipGetLastError();
}

size_t rt_sup_units(const RtFrame &F) { return (size_t)rt_cert_units(F, 1); }

// The lattice kernels' precondition (lat_yaw): dir.y = y (R's y row (0, 1, 0,
// 0) up to the sign of its zeros) and dir.x a function of x alone (R's y
// weight +-0) -- shared columns when dir.x = x exactly (x row (1, 0, 0, 0)),
// else per-pixel columns (entries bounded, so dir.x stays finite and
// monotone); pixel offsets stay far inside float's
// exact integer range, and tiles do not straddle stripes.
static bool rt_lattice_ok(const RtFrame &F)
{
    const float *R = F.R;
    if (!(R[1] == 0.0f && R[5] == 1.0f && R[9] == 0.0f && R[13] == 0.0f && R[4] == 0.0f)) return false;
    if (lat_yaw(F)) {
        for (int k : {0, 8, 12})
            if (!(fabsf(R[k]) <= 1e6f)) return false;
        if (!(fabsf(F.focal) <= 1e6f)) return false;
    }
    return F.W < (1 << 20) && F.H < (1 << 20) && (F.nranks == 1 || F.stripe_h % kLatTileH == 0);
}

// Whether launch_rt_pixels runs the lattice kernel for this frame (then the
// caller has rt_prepare_kernel certify its tiles first).
bool rt_use_lattice(const RtFrame &F)
{
    return F.n_tris > 0 && F.n_tris <= 62 && F.n_sph <= kLatMaxSph && F.cull_primary && F.n_lights >= 1 &&
           F.n_lights <= kLatMaxLights && rt_lattice_ok(F);
}

// 0: no lattice kernel, 1: shared columns, 2: per-pixel columns (cg_rt_route)
int rt_lattice_kind(const RtFrame &F) { return rt_use_lattice(F) ? (lat_yaw(F) ? 2 : 1) : 0; }

size_t rt_lattice_tiles(const RtFrame &F)
{
    return (size_t)((F.W + kLatTileW - 1) / kLatTileW) * ((F.rows_out + kLatTileH - 1) / kLatTileH);
}

// Batched lattice launch: nframes frames of F's geometry, frame f with camera
// cams.c[f] into d_out + f * out_stride (rt_use_lattice(F) must hold).
// Light sets (n_lights > 1) need the per-unit shadow masks of
// rt_lattice_units_kernel: rt_lattice_unit_bytes(F, nframes) of scratch,
// filled by launch_rt_lattice_units before the lattice launch reads them.
size_t rt_lattice_unit_bytes(const RtFrame &F, int nframes)
{
    if (!rt_use_lattice(F) || F.n_lights <= 1) return 0;
    const int slots = lat_yaw(F) ? lat_unit_slots<kLatWY>() : lat_unit_slots<kLatW>();
    const size_t n = (size_t)nframes * rt_lattice_tiles(F) * slots;   // byte codes, then the 64-bit masks
    return ((n + 7) & ~(size_t)7) + n * sizeof(unsigned long long);
}

hipError_t launch_rt_lattice_units(const RtFrame &F, const RtTri *d_tc, const RtShade *d_shade,
                                   const RtSphere *d_sph, const unsigned long long *d_lat_masks,
                                   const RtFrameCams &cams, int nframes, unsigned long long *d_umask, hipStream_t st)
{
    if (F.n_lights <= 1) return hipSuccess;
    const dim3 grid(F.txn ? F.txn : lat_tiles_x(F), (F.rows_out + kLatTileH - 1) / kLatTileH, nframes);
    const int kt_id = KT_RT_LATTICE_UNITS;
    if (lat_yaw(F))
        kt_launch(kt_id, rt_lattice_units_kernel<kLatWY>, grid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph,
                           d_lat_masks, cams, d_umask);
    else
        kt_launch(kt_id, rt_lattice_units_kernel<kLatW>, grid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph,
                           d_lat_masks, cams, d_umask);
    return hipGetLastError();
}

hipError_t launch_rt_lattice_frames(const RtFrame &F, const RtTri *d_tc, const RtShade *d_shade,
                                    const RtSphere *d_sph, const unsigned long long *d_lat_masks,
                                    const unsigned long long *d_umask, const RtFrameCams &cams, int nframes,
                                    size_t out_stride, uint32_t *d_out, hipStream_t st, uint32_t *d_done,
                                    const LatOrder *order, const LatReady *ready)
{
    const LatOrder O = order ? *order : LatOrder{};
    const LatReady R = ready ? *ready : LatReady{};
    if (R.flags && (F.n_lights != 1 || F.n_tris > 62)) return hipErrorInvalidValue;
    const dim3 grid(F.txn ? F.txn : lat_tiles_x(F), (F.rows_out + kLatTileH - 1) / kLatTileH, nframes);
    if (F.n_lights > 1 && !d_umask) return hipErrorInvalidValue;
    if (F.txn && (F.tx0 < 0 || F.tx0 + F.txn > lat_tiles_x(F))) return hipErrorInvalidValue;
    const int kt_id = F.n_lights == 1 ? KT_RT_LATTICE : KT_RT_LATTICE_LIGHTS;
    if (F.n_lights == 1 && lat_yaw(F))
        kt_launch(kt_id, rt_lattice_kernel<kLatWY>, grid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph,
                           d_lat_masks, cams, out_stride, d_out, d_done, O, R);
    else if (F.n_lights == 1)
        kt_launch(kt_id, rt_lattice_kernel<kLatW>, grid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph, d_lat_masks,
                           cams, out_stride, d_out, d_done, O, R);
    else if (lat_yaw(F))
        kt_launch(kt_id, rt_lattice_lights_kernel<kLatWY>, grid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph,
                           d_lat_masks, d_umask, cams, out_stride, d_out, d_done);
    else
        kt_launch(kt_id, rt_lattice_lights_kernel<kLatW>, grid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph,
                           d_lat_masks, d_umask, cams, out_stride, d_out, d_done);
    return hipGetLastError();
}

hipError_t launch_rt_pixels(const RtFrame &F, const RtTri *d_tc, const RtShade *d_shade,
                            const RtSphere *d_sph, const unsigned long long *d_lat_masks,
                            unsigned long long *d_umask, uint32_t *d_out, hipStream_t st)
{
    dim3 grid((F.W + kRtTileW - 1) / kRtTileW, (F.rows_out + kRtTileH - 1) / kRtTileH);
    if (d_lat_masks && rt_use_lattice(F)) {
        RtFrameCams cams{};
        for (int c = 0; c < 4; ++c) cams.c[0][c] = F.cam[c];
        hipError_t e = launch_rt_lattice_units(F, d_tc, d_shade, d_sph, d_lat_masks, cams, 1, d_umask, st);
        if (e != hipSuccess) return e;
        return launch_rt_lattice_frames(F, d_tc, d_shade, d_sph, d_lat_masks, d_umask, cams, 1, 0, d_out, st,
                                        nullptr, nullptr, nullptr);
    }
    const int kt_id = KT_RT_PIXEL;
    if (F.n_tris <= 64 && F.cull_primary)
        kt_launch(kt_id, rt_pixel_kernel<true>, grid, dim3(kRtThreads), 0, st, F, d_tc, d_shade,
                           d_sph, d_out);
    else
        kt_launch(kt_id, rt_pixel_kernel<false>, grid, dim3(kRtThreads), 0, st, F, d_tc, d_shade,
                           d_sph, d_out);
    return hipGetLastError();
}

hipError_t launch_rt_pack_rgb24(const uint32_t *d_src, int W, int rows, int wcol0, int wcols, uint8_t *d_dst,
                                hipStream_t st)
{
    if (rows <= 0 || wcols <= 0) return hipSuccess;
    hipLaunchKernelGGL(rt_pack_rgb24_kernel, dim3(((wcols + 3) / 4 + 255) / 256, rows), dim3(256), 0, st, d_src, W,
                       rows, wcol0, wcols, d_dst);
    return hipGetLastError();
}

hipError_t launch_rt_assemble(const uint8_t *d_src, const RtBlocks &B, int nframes, uint32_t *d_frames,
                              size_t frame_stride, hipStream_t st)
{
    const int rows = B.cum[B.n];
    if (rows <= 0 || nframes <= 0) return hipSuccess;
    hipLaunchKernelGGL(rt_assemble_kernel, dim3(((B.W + 3) / 4 + 255) / 256, rows, nframes), dim3(256), 0, st, d_src, B,
                       nframes, d_frames, frame_stride);
    return hipGetLastError();
}

hipError_t launch_rt_unstripe(const uint32_t *d_g, int W, int H, int nranks, int stripe_h,
                              int rows_per_rank, int nframes, uint32_t *d_frames, hipStream_t st)
{
    if (W % 4 == 0 && ((uintptr_t)d_g & 15) == 0 && ((uintptr_t)d_frames & 15) == 0) {
        const int W4 = W / 4;
        hipLaunchKernelGGL(rt_unstripe4_kernel, dim3((W4 + 255) / 256, H, nframes), dim3(256), 0, st,
                           (const uint4 *)d_g, W4, H, nranks, stripe_h, rows_per_rank, nframes, (uint4 *)d_frames);
        return hipGetLastError();
    }
    dim3 grid((W + 255) / 256, H, nframes);
    hipLaunchKernelGGL(rt_unstripe_kernel, grid, dim3(256), 0, st, d_g, W, H, nranks, stripe_h,
                       rows_per_rank, nframes, d_frames);
    return hipGetLastError();
}

hipError_t launch_rt_probe_closest(const RtFrame &F, const cg_tri *d_tris, const RtSphere *d_sph,
                                   const cg_vec4 *d_s, const cg_vec4 *d_d, int n, cg_isect *d_out,
                                   int *d_hit, hipStream_t st)
{
    hipLaunchKernelGGL(rt_probe_closest_kernel, dim3((n + 63) / 64), dim3(64), 0, st, F, d_tris,
                       d_sph, d_s, d_d, n, d_out, d_hit);
    return hipGetLastError();
}

hipError_t launch_rt_probe_direct_light(const RtFrame &F, const RtTri *d_tc,
                                        const RtShade *d_shade, const RtSphere *d_sph,
                                        const cg_isect *d_is, int n, cg_vec3 *d_out,
                                        hipStream_t st)
{
    hipLaunchKernelGGL(rt_probe_direct_light_kernel, dim3((n + 63) / 64), dim3(64), 0, st, F, d_tc,
                       d_shade, d_sph, d_is, n, d_out);
    return hipGetLastError();
}

}  // namespace cg

#ifdef CG_WG_TIMING
extern "C" int cg_diag_wg_timing(void *buf, unsigned cap)
{
    unsigned long long *p = (unsigned long long *)buf;
    const unsigned zero = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(cg::g_wgt), &p, sizeof p) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(cg::g_wgt_cap), &cap, sizeof cap) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(cg::g_wgt_n), &zero, sizeof zero) != hipSuccess) return -1;
    return 0;
}
extern "C" int cg_diag_wg_count(unsigned *n)
{
    return hipMemcpyFromSymbol(n, HIP_SYMBOL(cg::g_wgt_n), sizeof *n) == hipSuccess ? 0 : -1;
}
#endif

namespace cg {
// div3_by<true> on n (numerator triple, denominator) pairs: the test of the shared-reciprocal
// division against IEEE x / d (tests/test_rt_gpu.py)
__global__ void rt_probe_div3_kernel(const float *__restrict__ x, const float *__restrict__ d, int n,
                                     float *__restrict__ q)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const vec3 r = div3_by<true>(v3(x[3 * i], x[3 * i + 1], x[3 * i + 2]), d[i]);
    q[3 * i] = r.x;
    q[3 * i + 1] = r.y;
    q[3 * i + 2] = r.z;
}
}  // namespace cg

extern "C" int cg_rt_probe_div3_device(const float *d_x, const float *d_den, int n, float *d_q, void *stream)
{
    if (n < 0 || (n && (!d_x || !d_den || !d_q))) return CG_E_INVALID;
    if (n == 0) return CG_OK;
    hipLaunchKernelGGL(cg::rt_probe_div3_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_x, d_den,
                       n, d_q);
    return hipGetLastError() == hipSuccess ? CG_OK : CG_E_HIP;
}

#ifdef CG_WORK_COUNT
// Counting build: this translation unit's work counters (cg_rt_dev.h WorkKind order); reset after reading.
extern "C" int cg_diag_work_counts_rt(unsigned long long *out, int reset)
{
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cg::g_work), sizeof(unsigned long long) * cg::W_KINDS) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[cg::W_KINDS] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(cg::g_work), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif
