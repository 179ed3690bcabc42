// cg_rast.hip -- rasteriser fill + post-pass for gfx950 (MI355X).
//
// Reference: rasteriser/Source/skeleton.cpp, texture mode 0 / colour mode 0.
// Launches per frame (after rast_geometry_kernel, cg_geometry.hip, when the
// geometry runs on the device), all order-exact (no atomics touch colour/depth):
//   1. rast_setup_kernel   (one workgroup per clipped triangle)
//        VertexShader (:510-522) x3, then ComputePolygonRows (:433-498):
//        every edge sample of Interpolate (:524-551) is reduced into its row
//        with a 64-bit LDS min/max whose key is (x, sample sequence), which
//        reproduces the reference's `<=` / `>=` "later sample wins ties"
//        updates exactly; each visible row becomes a RastSpan holding what
//        DrawPolygonRows' Interpolate needs.
//   2. rast_rows_kernel    (one wave per screen row)
//        64-byte RowRec per triangle covering the row, in triangle order
//        (ballot + popcount compaction).
//   3. rast_fill_kernel    (one wave per 64-pixel row segment)
//        walks its row's records in triangle order -- the reference's ordered
//        z-buffer (`>=` for colour, `>` for shadow marks, :574/:668) with
//        depth/shadow/shade state held in registers; PixelShader +
//        calculateIllumination (:559-586, :664-688), deferred to the winner.
//   4. rast_post_kernel    (one thread per pixel)
//        the in-place raster-order post-pass (:283-307): a pixel's up/left
//        neighbours are seen darkened and down/right ones not, which is
//        recomputed per pixel from the shadow buffer, then antiAliasing
//        (:1736-1753) and PutPixelSDL.  Border pixels stay 0x00000000.
#include <float.h>
#include <limits.h>

#include "cg_rast_dev.h"

namespace cg {

void *ctx_buf(cg_ctx *c, int which, size_t bytes, hipError_t *e);
int ctx_fail(cg_ctx *c, hipError_t e, const char *what);
int ctx_invalid(cg_ctx *c, const char *what);
void ctx_events(cg_ctx *c, hipEvent_t *a, hipEvent_t *b);

constexpr int kSetupThreads = 256;
constexpr int kSetupPreChunks = 16;  // input triangles counted in one round trip: < 64 * 16
constexpr int kRastMaxRows = 4096;   // LDS rows per triangle in span setup (H <= 4096)

// Workgroups are dispatched round-robin over the 8 XCDs, each with its own L2.
// The row-ordered kernels renumber them so that each group of kXcdRows rows
// is handled by one XCD (a row's records are then fetched into one L2, not
// all eight), with the groups dealt round-robin to keep the XCDs balanced
// (row cost varies a lot over the frame).  A kernel whose row group is
// `per_group` workgroups wide launches xcd_grid(H, per_group) of them.
constexpr int kXcds = 8, kXcdRows = 8;
__host__ __device__ constexpr int xcd_grid(int H, int per_group)
{
    return kXcds * ((((H + kXcdRows - 1) / kXcdRows) + kXcds - 1) / kXcds) * per_group;
}
// -> row group of this workgroup (-1: idle padding) and its index m within the group
__device__ __forceinline__ int xcd_group(int H, int per_group, int &m)
{
    const int k = (int)(blockIdx.x % kXcds), l = (int)(blockIdx.x / kXcds);
    m = l % per_group;
    const int g = k + kXcds * (l / per_group);
    return g < (H + kXcdRows - 1) / kXcdRows ? g : -1;
}

struct Pix {                // rasteriser Pixel (:88-94) minus w
    int x, y;
    float zinv, X, Y;
};

__device__ __forceinline__ Pix vertex_shader(const RastArgs &A, cg_vec4 v)
{
    // :512-521
    float x = (A.focal * (v.x / v.z)) + (float)(A.W / 2);
    float y = (A.focal * (v.y / v.z)) + (float)(A.H / 2);
    Pix p;
    p.x = f2i_x86(x);
    p.y = f2i_x86(y);
    p.zinv = 1 / v.z;
    p.X = v.x;
    p.Y = v.y;
    return p;
}

// Interpolate (:524-551) prepared for one edge a -> b with N samples.
struct Edge {
    float ax, ay, az, aX, aY;     // a.x, a.y as float; a.zinv; a.pos3d.xy * a.zinv
    float stx, sty, stz, sX, sY;
    int n;
};

__device__ __forceinline__ Edge make_edge(Pix a, Pix b)
{
    Edge e;
    float aX = a.X * a.zinv, aY = a.Y * a.zinv;   // :526-527
    float bX = b.X * b.zinv, bY = b.Y * b.zinv;   // :529-530
    int dx = a.x - b.x, dy = a.y - b.y;
    dx = dx < 0 ? -dx : dx;
    dy = dy < 0 ? -dy : dy;
    e.n = (dx > dy ? dx : dy) + 1;                // :473-475
    float den = (float)(e.n - 1 > 1 ? e.n - 1 : 1);
    e.ax = (float)a.x;
    e.ay = (float)a.y;
    e.az = a.zinv;
    e.aX = aX;
    e.aY = aY;
    e.stx = (float)(b.x - a.x) / den;             // :533-538
    e.sty = (float)(b.y - a.y) / den;
    e.stz = (b.zinv - a.zinv) / den;
    e.sX = (bX - aX) / den;
    e.sY = (bY - aY) / den;
    return e;
}

__device__ __forceinline__ int edge_x(const Edge &e, int j) { return f2i_x86(floorf(e.ax + (e.stx * (float)j))); }
__device__ __forceinline__ int edge_y(const Edge &e, int j) { return f2i_x86(floorf(e.ay + (e.sty * (float)j))); }

// sample j's zinv and pos3d.xy (:543-548)
__device__ __forceinline__ void edge_attr(const Edge &e, int j, float &zinv, float &X, float &Y)
{
    float fj = (float)j;
    zinv = e.az + (e.stz * fj);
    X = (e.aX + (e.sX * fj)) / zinv;
    Y = (e.aY + (e.sY * fj)) / zinv;
}

__device__ __forceinline__ unsigned long long key_left(int x, unsigned seq)
{
    return ((unsigned long long)((unsigned)x ^ 0x80000000u) << 32) | (unsigned long long)(~seq);
}
__device__ __forceinline__ unsigned long long key_right(int x, unsigned seq)
{
    return ((unsigned long long)((unsigned)x ^ 0x80000000u) << 32) | (unsigned long long)seq;
}

__device__ void rast_setup_one(const cg_rtri &T, const RastArgs &A, RastSpan *__restrict__ spans,
                               RastHdr *__restrict__ hdr, int *__restrict__ first_tri, int t,
                               unsigned long long *lkey, unsigned long long *rkey, unsigned long long &fkey);

// One workgroup per clipped triangle (grid-stride).  With the device
// geometry (stage != null) the clipped list is compacted here: the count
// prefix of the n_in input triangles (LDS) locates clipped triangle t among
// the staged survivors, the workgroup copies it to tris[t] for the later
// kernels, and workgroup 0 stores the total at n_dev.
__global__ __launch_bounds__(kSetupThreads) void rast_setup_kernel(
    cg_rtri *__restrict__ tris, RastArgs A, int *__restrict__ n_dev, RastSpan *__restrict__ spans,
    RastHdr *__restrict__ hdr, int *__restrict__ first_tri, const cg_rtri *__restrict__ stage,
    const int *__restrict__ counts, int n_in)
{
    extern __shared__ unsigned long long s_keys[];          // [2 * H]: left | right keys per row; then [n_in + 1] ints
    __shared__ unsigned long long fkey;
    __shared__ int s_carry;
    unsigned long long *lkey = s_keys, *rkey = s_keys + A.H;
    int *s_pre = (int *)(s_keys + 2 * A.H);
    int n = A.n;
    if (stage) {
        if (n_in < 64 * kSetupPreChunks) {
            // exclusive prefix of the counts: every count loaded at once (one round trip, all
            // threads), each wave scans its 64-count chunks, then thread 0 offsets the chunks
            __shared__ int s_tot[kSetupPreChunks];
            constexpr int kQ = kSetupPreChunks / (kSetupThreads / 64);
            const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
            int cnt[kQ];
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                const int i = (q * (kSetupThreads / 64) + w) * 64 + lane;
                cnt[q] = i < n_in ? counts[i] : 0;
            }
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                const int ch = q * (kSetupThreads / 64) + w, i = ch * 64 + lane;
                int x = cnt[q];
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int y = __shfl_up(x, o);
                    if (lane >= o) x += y;
                }
                if (i <= n_in) s_pre[i] = x - cnt[q];   // exclusive within the chunk (s_pre[n_in]: its total)
                if (lane == 63) s_tot[ch] = x;
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                int a = 0;
                for (int ch = 0; ch * 64 <= n_in; ++ch) {
                    const int t = s_tot[ch];
                    s_tot[ch] = a;
                    a += t;
                }
                s_carry = a;
            }
            __syncthreads();
            for (int i = threadIdx.x; i <= n_in; i += kSetupThreads) s_pre[i] += s_tot[i / 64];
        } else if (threadIdx.x < 64) {                     // wave 0: exclusive prefix of the counts
            const int lane = threadIdx.x;
            int carry = 0;
            for (int i0 = 0; i0 < n_in; i0 += 64) {
                const int c = i0 + lane < n_in ? counts[i0 + lane] : 0;
                int x = c;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int y = __shfl_up(x, o);
                    if (lane >= o) x += y;
                }
                if (i0 + lane < n_in) s_pre[i0 + lane] = carry + x - c;
                carry += __shfl(x, 63);
            }
            if (lane == 0) {
                s_pre[n_in] = carry;
                s_carry = carry;
            }
        }
        __syncthreads();
        n = min(s_carry, A.n);
        if (blockIdx.x == 0 && threadIdx.x == 0) *n_dev = n;
    } else if (n_dev) {
        n = min(*n_dev, A.n);
    }
    for (int t = blockIdx.x; t < n; t += gridDim.x) {
        cg_rtri T;
        if (stage) {
            int lo = 0, hi = n_in - 1;                     // the input triangle whose survivors hold t
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_pre[mid] <= t) lo = mid;
                else hi = mid - 1;
            }
            T = stage[(size_t)lo * kGeomMaxLeaves + (t - s_pre[lo])];
            if (threadIdx.x == 0) tris[t] = T;
        } else {
            T = tris[t];
        }
        rast_setup_one(T, A, spans, hdr, first_tri, t, lkey, rkey, fkey);
        __syncthreads();
    }
}

__device__ void rast_setup_one(const cg_rtri &T, const RastArgs &A, RastSpan *__restrict__ spans,
                               RastHdr *__restrict__ hdr, int *__restrict__ first_tri, int t,
                               unsigned long long *lkey, unsigned long long *rkey, unsigned long long &fkey)
{
    Pix vp[3] = {vertex_shader(A, T.v0), vertex_shader(A, T.v1), vertex_shader(A, T.v2)};
    int mx = -INT_MAX, mn = INT_MAX;                        // :434-447
    for (int i = 0; i < 3; ++i) {
        if (vp[i].y > mx) mx = vp[i].y;
        if (vp[i].y < mn) mn = vp[i].y;
    }
    long long rows = (long long)mx - (long long)mn + 1;     // :448
    int ylo = mn > 0 ? mn : 0;
    int yhi = mx < A.H - 1 ? mx : A.H - 1;
    RastHdr h;
    h.ylo = ylo;
    h.yhi = yhi;
    h.fy = INT_MAX;
    h.fx = INT_MAX;
    h.t_sh = (unsigned)t | (T.color.x >= 0 ? 0u : 0x80000000u);
    h.tex = T.texture;
    h.index = T.index;
    h.pad = 0;
    if (rows <= 0 || ylo > yhi) {
        if (threadIdx.x == 0) {
            h.ylo = 1;
            h.yhi = 0;
            hdr[t] = h;
        }
        return;
    }
    const int nv = yhi - ylo + 1;
    for (int k = threadIdx.x; k < nv; k += kSetupThreads) {
        lkey[k] = ~0ull;
        rkey[k] = 0ull;
    }
    if (threadIdx.x == 0) fkey = ~0ull;
    __syncthreads();
    // the three edges' Interpolate set-up (:524-538), shared by both passes
    const Edge E0 = make_edge(vp[0], vp[1]), E1 = make_edge(vp[1], vp[2]), E2 = make_edge(vp[2], vp[0]);
    // Edge samples -> rows (:466-497).  Rows outside the screen never shade.
    for (int ei = 0; ei < 3; ++ei) {
        const Edge &e = ei == 0 ? E0 : ei == 1 ? E1 : E2;
        // Only a sample that can still win its row issues an LDS atomic: the
        // left winner is the minimum x with the latest sequence among equals,
        // so a sample whose previous same-row neighbour has a smaller x, or
        // whose next same-row neighbour has a smaller-or-equal x, cannot win
        // (mirror for the right).  Exact for any order; a near-horizontal
        // edge then issues a few atomics per wave instead of 64 on one row.
        const int lane = threadIdx.x & 63;
        for (int jb = 0; jb < e.n; jb += kSetupThreads) {
            const int j = jb + (int)threadIdx.x;
            const bool in = j < e.n;
            int y = in ? edge_y(e, j) : INT_MIN;
            const bool vis = in && y >= ylo && y <= yhi;   // also covers :485's y - min >= 0
            if (!vis) y = INT_MIN + 1 + lane;              // never equals a real row
            const int x = vis ? edge_x(e, j) : 0;
            const int yp = __shfl_up(y, 1, 64), xp = __shfl_up(x, 1, 64);
            const int yn = __shfl_down(y, 1, 64), xn = __shfl_down(x, 1, 64);
            const bool hp = lane > 0 && yp == y, hn = lane < 63 && yn == y;
            if (vis) {
                const unsigned seq = ((unsigned)ei << 30) | (unsigned)j;
                if (!(hp && xp < x) && !(hn && xn <= x)) atomicMin(&lkey[y - ylo], key_left(x, seq));
                if (!(hp && xp > x) && !(hn && xn >= x)) atomicMax(&rkey[y - ylo], key_right(x, seq));
            }
        }
    }
    __syncthreads();
    const bool shade_tri = A.want_first && T.color.x >= 0;
    for (int k = threadIdx.x; k < nv; k += kSetupThreads) {
        RastSpan s;
        unsigned long long lk = lkey[k], rk = rkey[k];
        if (lk == ~0ull) {                                  // untouched row: shades nothing
            s.lx = 1; s.rx = 0;
            s.lz = s.sz = s.lX = s.sX = s.lY = s.sY = 0.f;
        } else {
            unsigned ls = ~(unsigned)(lk & 0xffffffffu), rs = (unsigned)(rk & 0xffffffffu);
            int le = (int)(ls >> 30), lj = (int)(ls & 0x3fffffffu);
            int re = (int)(rs >> 30), rj = (int)(rs & 0x3fffffffu);
            const Edge el = le == 0 ? E0 : le == 1 ? E1 : E2;
            const Edge er = re == 0 ? E0 : re == 1 ? E1 : E2;
            int lx = edge_x(el, lj), rx = edge_x(er, rj);
            float lz, lX, lY, rz, rX, rY;
            edge_attr(el, lj, lz, lX, lY);
            edge_attr(er, rj, rz, rX, rY);
            // DrawPolygonRows' Interpolate(left, right, N = rx - lx + 1) (:502-503, :524-538)
            long long span = (long long)rx - (long long)lx;
            if (span < 0 || span > (1 << 24)) {              // reference would not survive this row
                s.lx = 1; s.rx = 0;
                s.lz = s.sz = s.lX = s.sX = s.lY = s.sY = 0.f;
            } else {
                int N = (int)span + 1;
                float den = (float)(N - 1 > 1 ? N - 1 : 1);
                float aX = lX * lz, aY = lY * lz, bX = rX * rz, bY = rY * rz;
                s.lx = lx;
                s.rx = rx;
                s.lz = lz;
                s.sz = (rz - lz) / den;
                s.lX = aX;
                s.sX = (bX - aX) / den;
                s.lY = aY;
                s.sY = (bY - aY) / den;
                if (shade_tri) {
                    // first fragment of this row that PixelShader would shade on an empty z-buffer
                    int y = ylo + k;
                    for (int i = 0; i < N - 1; ++i) {
                        int x = lx + i;
                        if (x >= A.W) break;
                        if (x < 0) continue;
                        float zi = s.lz + (s.sz * (float)i);
                        // on an empty z-buffer a fragment shades unless it is a
                        // transparent texel of texture 2/3 (:602, :624)
                        if (zi >= 0.0f && (!A.textured || rast_opaque(A, T.texture, T.index, zi,
                                                                     s.lX + (s.sX * (float)i),
                                                                     s.lY + (s.sY * (float)i)))) {
                            atomicMin(&fkey, ((unsigned long long)(unsigned)y << 32) | (unsigned)x);
                            break;
                        }
                    }
                }
            }
        }
        spans[(size_t)(ylo + k) * A.n + t] = s;              // row-major: a row's spans are contiguous
    }
    if (shade_tri) {
        __syncthreads();
        if (threadIdx.x == 0 && fkey != ~0ull) {
            h.fy = (int)(fkey >> 32);
            h.fx = (int)(fkey & 0xffffffffu);
            atomicMin(first_tri, t);
        }
    }
    if (threadIdx.x == 0) hdr[t] = h;
}


// A wave per row: the records of the row's covering triangles in triangle
// order.  The headers of a group of 64 * kRowBatches triangles are loaded in
// one round trip (beside the triangle count), then the spans of those that
// cover the row, then the ballot compaction -- two dependent round trips per
// group instead of three per 64 triangles.
constexpr int kRowBatches = 8;
__global__ __launch_bounds__(256) void rast_rows_kernel(const cg_rtri *__restrict__ tris, RastArgs A,
                                                       const int *__restrict__ n_dev,
                                                       const RastSpan *__restrict__ spans,
                                                       const RastHdr *__restrict__ hdr,
                                                       const int *__restrict__ first_tri,
                                                       RowRec *__restrict__ recs, int *__restrict__ count)
{
    int m;
    const int g = xcd_group(A.H, kXcdRows / 4, m);
    if (g < 0) return;
    const int y = g * kXcdRows + m * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (y >= A.H) return;
    const int ft = A.want_first ? *first_tri : INT_MAX;
    const int n = n_dev ? min(*n_dev, A.n) : A.n;
    int c = 0;
    for (int g0 = 0; g0 == 0 || g0 < n; g0 += 64 * kRowBatches) {
        RastHdr h[kRowBatches];
#pragma unroll
        for (int j = 0; j < kRowBatches; ++j) {   // in flight together (t < A.n: a valid header slot)
            const int t = g0 + 64 * j + lane;
            if (t < A.n) h[j] = hdr[t];
        }
        RastSpan sp[kRowBatches];
        bool keep[kRowBatches];
#pragma unroll
        for (int j = 0; j < kRowBatches; ++j) {
            const int t = g0 + 64 * j + lane;
            keep[j] = t < n && h[j].ylo <= y && y <= h[j].yhi;
            if (keep[j]) sp[j] = spans[(size_t)y * A.n + t];
        }
#pragma unroll
        for (int j = 0; j < kRowBatches; ++j) {
            const int t = g0 + 64 * j + lane;
            // fragments x in [lx, rx - 1] (:504) intersecting [0, W)
            const bool k = keep[j] && sp[j].rx > sp[j].lx && sp[j].rx - 1 >= 0 && sp[j].lx <= A.W - 1;
            const unsigned long long mk = __ballot(k);
            if (k) {
                RowRec r;
                r.lx = sp[j].lx; r.rx = sp[j].rx;
                r.lz = sp[j].lz; r.sz = sp[j].sz; r.lX = sp[j].lX; r.sX = sp[j].sX; r.lY = sp[j].lY; r.sY = sp[j].sY;
                r.t_sh = h[j].t_sh;
                r.first_x = (t == ft && h[j].fy == y) ? h[j].fx : -1;
                r.tex = h[j].tex; r.index = h[j].index;
                recs[(size_t)y * A.n + c + __popcll(mk & ((1ull << lane) - 1ull))] = r;
            }
            c += __popcll(mk);
        }
    }
    if (lane == 0) count[y] = c;
}

// Colour mode 0: fill -> post state, 4 bytes per pixel: 1 + the row record of
// the last shading fragment (0 none) | the shadow mark << 31; 2 bytes (the
// mark in bit 15) when a row holds fewer than 32768 records (A.state16).  The post-pass
// rebuilds that fragment from the record -- zinv = lz + sz * i (:543) and the
// pos3d numerators with the same float ops, the normal, the texels -- and
// evaluates calculateIllumination there, so the fill keeps only what its
// ordered walk decides.
constexpr uint32_t kStShadow = 0x80000000u;

// One wave per kFillPx-pixel row segment, one pixel per lane, state in
// registers; records walked in triangle order (the reference's ordered
// z-buffer), one uniform overlap test per record.
constexpr int kFillPx = 64;   // pixels per wave; 128 / 256 measured 3 % / 10 % slower (C3, round 1)

// TEX: texture modes 1-3 possible (A.textured): a fragment of texture 2/3
// that passes the depth test but hits a transparent texel sets the depth to 0
// and shades nothing (:619, :643, :665) -- decided in the ordered walk.
template <bool TEX>
__global__ __launch_bounds__(256) void rast_fill_kernel(RastArgs A, const RowRec *__restrict__ recs,
                                                       const int *__restrict__ count, uint32_t *__restrict__ state,
                                                       float *__restrict__ depth_out, int32_t *__restrict__ shadow_out)
{
    const int segs = (A.W + kFillPx - 1) / kFillPx;
    // wave-uniform by construction; readfirstlane lets the compiler keep the
    // record walk on the scalar unit (uniform branches)
    int m;
    const int g = xcd_group(A.H, (segs * kXcdRows + 3) / 4, m);
    if (g < 0) return;
    const int unit = m * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // (row, segment) in the group
    const int lane = threadIdx.x & 63;
    const int y = g * kXcdRows + unit / segs;
    if (unit >= segs * kXcdRows || y >= A.H) return;
    const int x0 = (unit % segs) * kFillPx;
    const int x = x0 + lane;
    float depth = 0.0f;                                   // :247
    int shadow = 0, win = -1;                             // :259; record of the last shading fragment
    const int cnt = count[y];
    const RowRec *rr = recs + (size_t)y * A.n;
    // 64 records per round trip: lane q loads record base+q (coalesced), a
    // ballot keeps those with a fragment in this segment, and the set bits are
    // walked in ascending order (= triangle order) with readlane broadcasts.
    for (int base = 0; base < cnt; base += 64) {
        const int q = base + lane;
        int mlx = 0, mrx = 0, msh = 0, mtex = 0, midx = 0;
        float mlz = 0.f, msz = 0.f, mlX = 0.f, msX = 0.f, mlY = 0.f, msY = 0.f;
        if (q < cnt) {
            const RowRec &mr = rr[q];
            mlx = mr.lx; mrx = mr.rx; mlz = mr.lz; msz = mr.sz; msh = rec_shadow(mr);
            if (TEX) {
                mtex = mr.tex; midx = mr.index;
                mlX = mr.lX; msX = mr.sX; mlY = mr.lY; msY = mr.sY;
            }
        }
        const bool ov = q < cnt && !(mrx - 1 < x0 || mlx > x0 + kFillPx - 1);
        unsigned long long m = __ballot(ov);
        while (m) {
            const int b = __builtin_ctzll(m);
            m &= m - 1ull;
            const int lx = __builtin_amdgcn_readlane(mlx, b);
            const int rx = __builtin_amdgcn_readlane(mrx, b);
            const float lz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mlz), b));
            const float sz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(msz), b));
            const int shd = __builtin_amdgcn_readlane(msh, b);
            // every readlane sits here, where the whole wave is active: lane b
            // holds the record, and a readlane under a per-lane condition below
            // would read a register the compiler may have split under EXEC
            int tex = 0, idx = 0;
            float lX = 0.f, sX = 0.f, lY = 0.f, sY = 0.f;
            if (TEX) {
                tex = __builtin_amdgcn_readlane(mtex, b);
                idx = __builtin_amdgcn_readlane(midx, b);
                lX = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mlX), b));
                sX = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(msX), b));
                lY = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mlY), b));
                sY = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(msY), b));
            }
            const int i = x - lx;
            if (!(x < A.W && i >= 0 && x < rx)) continue;          // :504, :573
            const float zinv = lz + (sz * (float)i);               // :543
            if (!shd) {
                if (zinv >= depth) {                               // :574
                    bool opaque = true;
                    if (TEX && tex >= 2)                           // opacity-tested textures
                        opaque = rast_opaque(A, tex, idx, zinv, lX + (sX * (float)i), lY + (sY * (float)i));
                    if (opaque) {
                        depth = zinv;                              // :665
                        win = base + b;
                    } else {
                        depth = 0.0f;                              // p.zinv = 0 (:619, :643), :665
                    }
                }
            } else if (zinv > depth) {                             // :668-669
                shadow = 1;
            }
        }
    }
    if (x < A.W) {
        const size_t o = (size_t)y * A.W + x;
        if (A.state16) ((uint16_t *)state)[o] = (uint16_t)((win + 1) | (shadow ? 0x8000 : 0));
        else state[o] = (uint32_t)(win + 1) | (shadow ? kStShadow : 0u);
        if (depth_out) depth_out[o] = depth;
        if (shadow_out) shadow_out[o] = shadow;
    }
}

// shade buffers of one pixel as they stand after the fill (:580-585), from its
// state and its triangle's colour
__device__ __forceinline__ void shade3c(const RastArgs &A, float4 st, cg_vec3 col, vec3 &sc, vec3 &lo, vec3 &hi,
                                        int tex = 0, uint32_t texel = 0u)
{
    const int tb = __float_as_int(st.x);
    if (tb < 0) {
        sc = lo = hi = v3(0.f, 0.f, 0.f);
        return;
    }
    if (tb & kStateDirect) {                               // colour modes 1-2 (:652, :660)
        sc = v3(st.y, st.z, st.w);
        lo = hi = v3(0.f, 0.f, 0.f);                       // cleared buffers (:250-257)
        return;
    }
    const float ind = (tb & (1 << 30)) ? A.ind_first : 0.2f * 1;
    const vec3 D = v3(st.y, st.z, st.w);
    if (tex != 0) {
        // textureColour (:590, :611, :636) and, texture 3, the occlusion (:626-627)
        const vec3 c = v3((float)((texel >> 16) & 255u) / 255.0f, (float)((texel >> 8) & 255u) / 255.0f,
                          (float)(texel & 255u) / 255.0f);
        if (tex == 3) {
            float occ = (float)(texel >> 24);
            occ /= 255.0f;
            sc = c * ((D + v3(ind, ind, ind)) * occ);                                // :638
            lo = c * ((D + v3(0.0f * 1, 0.0f * 1, 0.0f * 1)) * occ);                 // :640
            hi = c * ((D + v3(0.4f * 1, 0.4f * 1, 0.4f * 1)) * occ);                 // :642
        } else {
            sc = c * (D + v3(ind, ind, ind));
            lo = c * (D + v3(0.0f * 1, 0.0f * 1, 0.0f * 1));
            hi = c * (D + v3(0.4f * 1, 0.4f * 1, 0.4f * 1));
        }
        return;
    }
    const vec3 c = v3(col.x, col.y, col.z);
    sc = c * (D + v3(ind, ind, ind));                      // :580
    lo = c * (D + v3(0.0f * 1, 0.0f * 1, 0.0f * 1));       // :582
    hi = c * (D + v3(0.4f * 1, 0.4f * 1, 0.4f * 1));       // :584
}

// soft-shadow darkening amount of a pixel whose 3x3 shadow neighbourhood is
// sh[cy-1..cy+1][cx-1..cx+1] (row stride ld), 0 if not shadowed
// (:286-303, :1725-1733; [y+1][x-1] counted twice, [y+1][x+1] omitted)
// (sh: the marks as ints, or the post state words with the mark in bit 31)
template <class T>
__device__ __forceinline__ float darken_at(const T *sh, int ld, int cy, int cx)
{
    const T *p = sh + cy * ld + cx;
    auto c = [&](int o) { return sizeof(T) == 4 && (T)-1 > (T)0 ? (int)((uint32_t)p[o] >> 31) : (int)p[o]; };
    if (c(0) != 1) return 0.0f;
    int k = c(0) + c(-ld) + c(-ld - 1) + c(-ld + 1) + c(ld - 1) + c(ld) + c(ld - 1) + c(-1) + c(1);
    float val = div_const((float)k, 9.0f, 1.0f / 9.0f);                 // val /= 9.0f
    if ((double)val < 0.6) return 0.05f;
    if ((double)val < 0.7) return 0.08f;
    if ((double)val < 0.8) return 0.1f;
    if ((double)val < 0.9) return 0.12f;
    return 0.3f;
}

// Post-pass (:283-307) on a 64x8 tile: the shadow marks (halo 2) go to LDS,
// then every pixel of the tile and its 1-pixel halo gets its three shade
// buffers and its darkening computed once, then each interior pixel runs
// antiAliasing (:1736-1753) on its 5 taps from LDS.  Raster order: the pixel
// itself and its up/left neighbours are seen darkened, down/right not (a
// darkening of 0 subtracts exactly nothing).  DIRECT (colour modes 1-2): the
// state is the colour fill's float4 (cg_rast_colour.hip) instead of the fill's
// record word, and the shadow marks come from the shadow plane.
constexpr int kPostTW = 64, kPostTH = 8;
constexpr int kPostHW = kPostTW + 2, kPostHH = kPostTH + 2;      // shade halo 1
constexpr int kPostSW = kPostTW + 4, kPostSH = kPostTH + 4;      // shadow halo 2

template <bool DIRECT, bool TEX>
__global__ __launch_bounds__(256) void rast_post_kernel(const cg_rtri *__restrict__ tris, RastArgs A0,
                                                       const void *__restrict__ state_v,
                                                       const RowRec *__restrict__ recs,
                                                       const int32_t *__restrict__ sh,
                                                       uint32_t *__restrict__ argb)
{
    RastArgs A = A0;
    if (!DIRECT && A.d_light) {                           // light from the device geometry (:223)
        const cg_vec4 L = *A.d_light;
        A.light[0] = L.x; A.light[1] = L.y; A.light[2] = L.z;
    }
    __shared__ float s_c[9][kPostHH][kPostHW];      // sc.xyz, lo.xyz, hi.xyz
    __shared__ float s_d[kPostHH][kPostHW];
    // The halo-2 words (colour modes 1-2: the shadow marks; mode 0: the state
    // words) live in s_c's space: every thread takes what it needs from them
    // (its pixels' records and darkenings) into registers before the barrier
    // after which s_c is written.  26.4 KB instead of 29.7: six workgroups
    // per CU instead of five.
    static_assert(sizeof(uint32_t) * kPostSH * kPostSW <= sizeof(float) * 9 * kPostHH * kPostHW, "halo words fit");
    int (*s_sh)[kPostSW] = reinterpret_cast<int (*)[kPostSW]>(&s_c[0][0][0]);
    const int W = A.W, H = A.H;
    static_assert(kPostTH == kXcdRows, "a post tile row is one XCD row group");
    int m;
    const int g = xcd_group(H, (W + kPostTW - 1) / kPostTW, m);
    if (g < 0) return;
    const int gx0 = m * kPostTW, gy0 = g * kPostTH;
    const uint32_t *st4 = static_cast<const uint32_t *>(state_v);
    const uint16_t *st2 = static_cast<const uint16_t *>(state_v);
    auto state_at = [&](size_t o) -> uint32_t {   // the 4-byte form
        if (!A.state16) return st4[o];
        const uint32_t v = st2[o];
        return (v & 0x7fffu) | ((v >> 15) << 31);
    };
    const float4 *st16 = static_cast<const float4 *>(state_v);
    // all global loads first (shadow marks, shade state), so each thread has them in flight together
    constexpr int kShR = (kPostSH * kPostSW + 255) / 256, kStR = (kPostHH * kPostHW + 255) / 256;
    // mode 0: the state words (record + 1, mark in bit 31) of the tile + halo 2
    uint32_t (*s_st)[kPostSW] = reinterpret_cast<uint32_t (*)[kPostSW]>(&s_c[0][0][0]);
    uint32_t shv[kShR];
#pragma unroll
    for (int r = 0; r < kShR; ++r) {
        const int i = threadIdx.x + 256 * r;
        const int cy = i / kPostSW, cx = i - cy * kPostSW;
        const int gx = gx0 - 2 + cx, gy = gy0 - 2 + cy;
        const bool in = i < kPostSH * kPostSW && gx >= 0 && gy >= 0 && gx < W && gy < H;
        if (DIRECT) shv[r] = in ? (uint32_t)sh[(size_t)gy * W + gx] : 0u;
        else shv[r] = in ? state_at((size_t)gy * W + gx) : 0u;
    }
#pragma unroll
    for (int r = 0; r < kShR; ++r) {
        const int i = threadIdx.x + 256 * r;
        if (i < kPostSH * kPostSW) {
            if (DIRECT) (&s_sh[0][0])[i] = (int)shv[r];
            else (&s_st[0][0])[i] = shv[r];
        }
    }
    __syncthreads();
    float dv[kStR];   // each pixel's darkening, from the marks before s_c is written
#pragma unroll
    for (int r = 0; r < kStR; ++r) {
        const int i = threadIdx.x + 256 * r;
        const int cy = i / kPostHW, cx = i - cy * kPostHW;
        const int gx = gx0 - 1 + cx, gy = gy0 - 1 + cy;
        dv[r] = 0.0f;
        if (i < kPostHH * kPostHW && gx >= 1 && gy >= 1 && gx < W - 1 && gy < H - 1)
            dv[r] = DIRECT ? darken_at(&s_sh[0][0], kPostSW, cy + 1, cx + 1)
                           : darken_at(&s_st[0][0], kPostSW, cy + 1, cx + 1);
    }
    if constexpr (DIRECT) {
        __syncthreads();   // the marks are dead: s_c's space is free
#pragma unroll
        for (int r = 0; r < kStR; ++r) {
            const int i = threadIdx.x + 256 * r;
            if (i >= kPostHH * kPostHW) break;
            const int cy = i / kPostHW, cx = i - cy * kPostHW;
            const int gx = gx0 - 1 + cx, gy = gy0 - 1 + cy;
            vec3 sc = v3(0.f, 0.f, 0.f), lo = sc, hi = sc;
            const float d = dv[r];
            if (gx >= 0 && gy >= 0 && gx < W && gy < H) {
                const float4 s4 = st16[(size_t)gy * W + gx];
                const int tb = __float_as_int(s4.x);
                const bool tri = tb >= 0 && !(tb & kStateDirect);
                shade3c(A, s4, tri ? tris[tb & ~(1 << 30)].color : cg_vec3{0.f, 0.f, 0.f}, sc, lo, hi);
            }
            s_c[0][cy][cx] = sc.x; s_c[1][cy][cx] = sc.y; s_c[2][cy][cx] = sc.z;
            s_c[3][cy][cx] = lo.x; s_c[4][cy][cx] = lo.y; s_c[5][cy][cx] = lo.z;
            s_c[6][cy][cx] = hi.x; s_c[7][cy][cx] = hi.y; s_c[8][cy][cx] = hi.z;
            s_d[cy][cx] = d;
        }
    } else {
        // The shading fragments of the tile + halo 1: each thread's record
        // loads go out together, then their triangles', then the arithmetic --
        // two dependent round trips instead of two per pixel.
        RowRec rv[kStR];
        int recv[kStR];
#pragma unroll
        for (int r = 0; r < kStR; ++r) {
            const int i = threadIdx.x + 256 * r;
            const int cy = i / kPostHW, cx = i - cy * kPostHW;
            const int gx = gx0 - 1 + cx, gy = gy0 - 1 + cy;
            const bool in = i < kPostHH * kPostHW && gx >= 0 && gy >= 0 && gx < W && gy < H;
            recv[r] = in ? (int)(s_st[cy + 1][cx + 1] & ~kStShadow) - 1 : -1;
            if (recv[r] >= 0) rv[r] = recs[(size_t)gy * A.n + recv[r]];
        }
        __syncthreads();   // the state words are dead: s_c's space is free
        cg_vec4 tnv[kStR];
        cg_vec3 colv[kStR];
#pragma unroll
        for (int r = 0; r < kStR; ++r)
            if (recv[r] >= 0) {
                const int t = rec_t(rv[r]);
                tnv[r] = tris[t].normal;
                colv[r] = tris[t].color;
            }
#pragma unroll
        for (int r = 0; r < kStR; ++r) {
            const int i = threadIdx.x + 256 * r;
            if (i >= kPostHH * kPostHW) break;
            const int cy = i / kPostHW, cx = i - cy * kPostHW;
            const int gx = gx0 - 1 + cx, gy = gy0 - 1 + cy;
            vec3 sc = v3(0.f, 0.f, 0.f), lo = sc, hi = sc;
            const float d = dv[r];
            if (recv[r] >= 0) {   // a shading fragment (:580-585, rebuilt as shade_from_record does)
                const RowRec &R = rv[r];
                const float fi = (float)(gx - R.lx);
                const float z = R.lz + (R.sz * fi);                               // :543, as the fill evaluated it
                const float X = R.lX + (R.sX * fi), Y = R.lY + (R.sY * fi);       // :547-548 numerators
                const int t = rec_t(R);
                vec3 N = v3(tnv[r].x, tnv[r].y, tnv[r].z);
                int tex = 0;
                uint32_t texel = 0u;
                if (TEX && R.tex != 0 && rast_tex_present(A, R.tex)) {
                    tex = R.tex;
                    N = rast_tex_normal(A, tex, R.index, z, X, Y, gx, gy, N, texel);
                }
                const vec3 D = illum_D(A, z, X, Y, N);                            // :580-585 (:590-645)
                const float4 s4 = make_float4(__int_as_float(t | (gx == R.first_x ? (1 << 30) : 0)), D.x, D.y, D.z);
                shade3c(A, s4, colv[r], sc, lo, hi, tex, texel);
            }
            s_c[0][cy][cx] = sc.x; s_c[1][cy][cx] = sc.y; s_c[2][cy][cx] = sc.z;
            s_c[3][cy][cx] = lo.x; s_c[4][cy][cx] = lo.y; s_c[5][cy][cx] = lo.z;
            s_c[6][cy][cx] = hi.x; s_c[7][cy][cx] = hi.y; s_c[8][cy][cx] = hi.z;
            s_d[cy][cx] = d;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kPostTH * kPostTW; i += 256) {
        const int ty = i / kPostTW, tx = i - ty * kPostTW;
        const int x = gx0 + tx, y = gy0 + ty;
        if (x >= W || y >= H) continue;
        const size_t o = (size_t)y * W + x;
        if (x < 1 || y < 1 || x >= W - 1 || y >= H - 1) {   // :283-284 border never written
            argb[o] = 0u;
            continue;
        }
        const int cy = ty + 1, cx = tx + 1;
        auto tap = [&](int b, int yy, int xx) { return v3(s_c[b][yy][xx], s_c[b + 1][yy][xx], s_c[b + 2][yy][xx]); };
        auto dk = [&](int yy, int xx) { const float d = s_d[yy][xx]; return v3(d, d, d); };
        const int ty5[5] = {cy, cy - 1, cy + 1, cy, cy}, tx5[5] = {cx, cx, cx, cx - 1, cx + 1};  // c, up, down, left, right
        vec3 sv[5], lv[5], hv[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            sv[k] = tap(0, ty5[k], tx5[k]);
            lv[k] = tap(3, ty5[k], tx5[k]);
            hv[k] = tap(6, ty5[k], tx5[k]);
        }
        sv[0] = sv[0] - dk(cy, cx);                        // darkened: itself, up, left
        sv[1] = sv[1] - dk(cy - 1, cx);
        sv[3] = sv[3] - dk(cy, cx - 1);
        // :1741-1750 (x / 5.0f and / 3.0f via div_const, bit-identical)
        vec3 val = div_const((((sv[0] + sv[1]) + sv[2]) + sv[3]) + sv[4], 5.0f, 1.0f / 5.0f);
        vec3 val1 = div_const((((lv[0] + lv[1]) + lv[2]) + lv[3]) + lv[4], 5.0f, 1.0f / 5.0f);
        vec3 val2 = div_const((((hv[0] + hv[1]) + hv[2]) + hv[3]) + hv[4], 5.0f, 1.0f / 5.0f);
        val = div_const((val + val1) + val2, 3.0f, 1.0f / 3.0f);
        argb[o] = put_pixel(val);
    }
}

int rast_colour_fill(cg_ctx *c, const RastArgs &A, const cg_rast_params *p, const RowRec *recs, const int *count,
                     const RastHdr *hdr, const int *n_dev, int max_recs, float4 *state, float *d_depth,
                     int32_t *shadow, hipStream_t st, long long *n_shaded);

hipError_t launch_rast_clip(const cg_rast_params &prm, const cg_rtri *d_room, int n_room, const cg_rtri *d_boxes,
                            int n_boxes, cg_rtri *d_stage, int *d_counts, cg_vec4 *d_light, int *d_first,
                            hipStream_t st);

// The fill + post pipeline.  Either the triangle count is known on the host
// (n_dev == nullptr, n = count) or it lives on the device (n_dev, n = capacity,
// light read from d_light).
// Staged survivors of the device clip (rast_draw_device): the setup compacts them.
struct RastStage {
    const cg_rtri *stage;   // null: d_tris is already the list
    const int *counts;
    int n_in;
};
static int rast_pipeline(cg_ctx *c, cg_rtri *d_tris, int n, int *n_dev, const cg_rast_params *p,
                         cg_vec4 light, const cg_vec4 *d_light, uint32_t *d_argb, float *d_depth,
                         int32_t *d_shadow, hipStream_t st, cg_stats *stats, bool events_open, int tex_mask,
                         RastStage sg);
int rast_tex_maps(cg_ctx *c, RastTexMaps *m);

// glm::inverse for mat4 (glm/detail/type_mat4x4.inl:37-90), column-major
// m[4c + r] = m[c][r]: findU / findV's inverse(R) (skeleton.cpp:1762).
static void mat4_inverse_glm(const float *m, float *out)
{
    auto M = [m](int c, int r) { return m[4 * c + r]; };
    const float c00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3), c02 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
    const float c03 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3);
    const float c04 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3), c06 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3);
    const float c07 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
    const float c08 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2), c10 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
    const float c11 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2);
    const float c12 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3), c14 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3);
    const float c15 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
    const float c16 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2), c18 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
    const float c19 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2);
    const float c20 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1), c22 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1);
    const float c23 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
    const float fac[6][4] = {{c00, c00, c02, c03}, {c04, c04, c06, c07}, {c08, c08, c10, c11},
                             {c12, c12, c14, c15}, {c16, c16, c18, c19}, {c20, c20, c22, c23}};
    const float vec[4][4] = {{M(1, 0), M(0, 0), M(0, 0), M(0, 0)}, {M(1, 1), M(0, 1), M(0, 1), M(0, 1)},
                             {M(1, 2), M(0, 2), M(0, 2), M(0, 2)}, {M(1, 3), M(0, 3), M(0, 3), M(0, 3)}};
    float inv[4][4];
    for (int k = 0; k < 4; ++k) {
        const float sa = (k & 1) ? -1.0f : 1.0f, sb = -sa;   // SignA (+,-,+,-), SignB (-,+,-,+)
        inv[0][k] = ((vec[1][k] * fac[0][k] - vec[2][k] * fac[1][k]) + vec[3][k] * fac[2][k]) * sa;
        inv[1][k] = ((vec[0][k] * fac[0][k] - vec[2][k] * fac[3][k]) + vec[3][k] * fac[4][k]) * sb;
        inv[2][k] = ((vec[0][k] * fac[1][k] - vec[1][k] * fac[3][k]) + vec[3][k] * fac[5][k]) * sa;
        inv[3][k] = ((vec[0][k] * fac[2][k] - vec[1][k] * fac[4][k]) + vec[2][k] * fac[5][k]) * sb;
    }
    const float d0 = M(0, 0) * inv[0][0], d1 = M(0, 1) * inv[1][0], d2 = M(0, 2) * inv[2][0],
                d3 = M(0, 3) * inv[3][0];
    const float one_over = 1.0f / ((d0 + d1) + (d2 + d3));
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out[4 * c + r] = inv[c][r] * one_over;
}

int rast_render_device(cg_ctx *c, const cg_rtri *d_tris, int n, const cg_rast_params *p, cg_vec4 light,
                       uint32_t *d_argb, float *d_depth, int32_t *d_shadow, hipStream_t st,
                       cg_stats *stats, int tex_mask)
{
    return rast_pipeline(c, const_cast<cg_rtri *>(d_tris), n, nullptr, p, light, nullptr, d_argb, d_depth, d_shadow,
                         st, stats, false, tex_mask, RastStage{nullptr, nullptr, 0});
}

// Whole rasteriser Draw on the device: geometry (shadow volumes + clip) then
// fill + post.  room/boxes are device pointers (cg_rast_set_scene).
int rast_draw_device(cg_ctx *c, const cg_rtri *d_room, int n_room, const cg_rtri *d_boxes, int n_boxes,
                     const cg_rast_params *p, uint32_t *d_argb, float *d_depth, int32_t *d_shadow,
                     hipStream_t st, cg_stats *stats, int **n_out, int tex_mask)
{
    if (p->width <= 2 || p->height <= 2 || p->height > kRastMaxRows || p->focal == 0.0f) return CG_E_INVALID;
    const int n_in = n_room + 7 * n_boxes;
    // planes 1-4 and 6 can each split a triangle in two; plane 5 never does
    const int cap = n_in > 0 ? 32 * n_in : 1;
    hipError_t e;
    // the clipped list, then each input triangle's staged survivors (32 each)
    cg_rtri *tris = (cg_rtri *)ctx_buf(c, 0, ((size_t)cap + 32 * (size_t)n_in) * sizeof(cg_rtri), &e);
    if (!tris) return ctx_fail(c, e, "alloc clipped triangles");
    int *geo = (int *)ctx_buf(c, 9, 64 + 4 * (size_t)n_in, &e);   // [0] count, [4..7] light, [16..] counts
    if (!geo) return ctx_fail(c, e, "alloc geometry header");
    int *misc = (int *)ctx_buf(c, 7, ((size_t)p->height + 16) * sizeof(int), &e);   // count[H] | first_tri
    if (!misc) return ctx_fail(c, e, "alloc counts");
    hipEvent_t e0, e1;
    ctx_events(c, &e0, &e1);
    if (stats && (e = hipEventRecord(e0, st)) != hipSuccess) return ctx_fail(c, e, "event");
    if ((e = launch_rast_clip(*p, d_room, n_room, d_boxes, n_boxes, tris + cap, geo + 16, (cg_vec4 *)(geo + 4),
                              misc + p->height, st)) != hipSuccess)
        return ctx_fail(c, e, "rast_clip launch");
    if (n_out) *n_out = geo;
    return rast_pipeline(c, tris, cap, geo, p, cg_vec4{0, 0, 0, 1}, (const cg_vec4 *)(geo + 4), d_argb, d_depth,
                         d_shadow, st, stats, true, tex_mask, RastStage{tris + cap, geo + 16, n_in});
}

static int rast_pipeline(cg_ctx *c, cg_rtri *d_tris, int n, int *n_dev, const cg_rast_params *p,
                         cg_vec4 light, const cg_vec4 *d_light, uint32_t *d_argb, float *d_depth,
                         int32_t *d_shadow, hipStream_t st, cg_stats *stats, bool events_open, int tex_mask,
                         RastStage sg)
{
    if (p->width <= 2 || p->height <= 2 || p->height > kRastMaxRows) return CG_E_INVALID;
    const int W = p->width, H = p->height;
    const size_t npx = (size_t)W * H;
    const int nn = n > 0 ? n : 1;
    hipError_t e;
    RastSpan *spans = (RastSpan *)ctx_buf(c, 2, (size_t)nn * H * sizeof(RastSpan), &e);
    if (!spans) return ctx_fail(c, e, "alloc spans");
    RastHdr *hdr = (RastHdr *)ctx_buf(c, 1, (size_t)nn * sizeof(RastHdr), &e);
    if (!hdr) return ctx_fail(c, e, "alloc hdr");
    // fill -> post state: 4 B/pixel in colour mode 0, the colour fill's 16 B in modes 1-2
    void *state = ctx_buf(c, 3, npx * (p->colour_mode == 0 ? sizeof(uint32_t) : sizeof(float4)), &e);
    if (!state) return ctx_fail(c, e, "alloc state");
    int *misc = (int *)ctx_buf(c, 7, ((size_t)H + 16) * sizeof(int), &e);   // count[H] | first_tri
    if (!misc) return ctx_fail(c, e, "alloc counts");
    int *count = misc, *first_tri = misc + H;
    RowRec *recs = (RowRec *)ctx_buf(c, 8, (size_t)H * nn * sizeof(RowRec), &e);
    if (!recs) return ctx_fail(c, e, "alloc row records");
    int32_t *shadow = d_shadow;   // mode 0 carries the marks in the state; modes 1-2 need the plane
    if (!shadow && p->colour_mode != 0) {
        shadow = (int32_t *)ctx_buf(c, 6, npx * sizeof(int32_t), &e);
        if (!shadow) return ctx_fail(c, e, "alloc shadow");
    }
    RastArgs A;
    A.W = W;
    A.H = H;
    A.n = n;
    A.focal = p->focal;
    A.light[0] = light.x; A.light[1] = light.y; A.light[2] = light.z;
    A.lp[0] = p->light_power.x; A.lp[1] = p->light_power.y; A.lp[2] = p->light_power.z;
    A.ind_first = p->indirect_first;
    A.want_first = p->colour_mode == 0 && p->indirect_first != 0.2f * 1;   // the :585 rewrite is mode 0 only
    A.d_light = d_light;
    // texture modes 1-3: the maps, cameraPos and, when yaw != 0, inverse(R)
    const int loaded = rast_tex_maps(c, &A.tx);
    if (tex_mask & 16) return ctx_invalid(c, "texture selector outside 0-3 (TestModelH.h:21)");
    if (tex_mask & ~loaded & 0xe)
        return ctx_invalid(c, "a triangle carries a texture whose maps are not loaded (cg_rast_set_textures)");
    if ((tex_mask & 2) && (size_t)(H - 1) * kMarbleN + (W - 1) >= (size_t)kMarbleN * kMarbleN)
        return ctx_invalid(c, "marble: normalMap_marble[y * 2000 + x] would index past the map");
    A.textured = (tex_mask & 0xe) != 0;
    A.use_inv = p->yaw != 0.0f;
    A.state16 = p->colour_mode == 0 && nn < 32768;
    A.tris = d_tris;
    A.cam[0] = p->camera.x; A.cam[1] = p->camera.y; A.cam[2] = p->camera.z; A.cam[3] = p->camera.w;
    mat4_inverse_glm(p->R, A.Rinv);
    hipEvent_t e0, e1;
    ctx_events(c, &e0, &e1);
    if (stats && !events_open && (e = hipEventRecord(e0, st)) != hipSuccess) return ctx_fail(c, e, "event");
    // the device clip initialises the first-fragment minimum (rast_clip_kernel)
    if (A.want_first && !(sg.stage && sg.n_in > 0) && (e = hipMemsetAsync(first_tri, 0x7f, sizeof(int), st)) != hipSuccess)
        return ctx_fail(c, e, "memset");
    if (n > 0) {
        const int grid = n < 1024 ? n : 1024;                // LDS 16 B per row: several workgroups per CU
        hipLaunchKernelGGL(rast_setup_kernel, dim3(grid), dim3(kSetupThreads),
                           2 * (size_t)H * 8 + ((size_t)sg.n_in + 1) * 4, st, d_tris, A, n_dev, spans, hdr, first_tri,
                           sg.stage, sg.counts, sg.n_in);
        if ((e = hipGetLastError()) != hipSuccess) return ctx_fail(c, e, "rast_setup launch");
    }
    hipLaunchKernelGGL(rast_rows_kernel, dim3(xcd_grid(H, kXcdRows / 4)), dim3(256), 0, st, d_tris, A, n_dev, spans, hdr,
                       first_tri, recs, count);
    if ((e = hipGetLastError()) != hipSuccess) return ctx_fail(c, e, "rast_rows launch");
    const int post_grid = xcd_grid(H, (W + kPostTW - 1) / kPostTW);
    if (p->colour_mode != 0) {
        long long ns = 0;
        const int rc = rast_colour_fill(c, A, p, recs, count, hdr, n_dev, nn, (float4 *)state, d_depth, shadow, st, &ns);
        if (rc) return rc;
        if (stats) stats->n_shaded = ns;
        hipLaunchKernelGGL((rast_post_kernel<true, false>), dim3(post_grid), dim3(256), 0, st, d_tris, A,
                           (const void *)state, (const RowRec *)recs, shadow, d_argb);
    } else {
        const int fgrid = xcd_grid(H, ((W + kFillPx - 1) / kFillPx * kXcdRows + 3) / 4);
        {
            const int kt_id = KT_RAST_FILL;
            if (A.textured)
                kt_launch(kt_id, rast_fill_kernel<true>, dim3(fgrid), dim3(256), 0, st, A, recs, count,
                                   (uint32_t *)state, d_depth, d_shadow);
            else
                kt_launch(kt_id, rast_fill_kernel<false>, dim3(fgrid), dim3(256), 0, st, A, recs, count,
                                   (uint32_t *)state, d_depth, d_shadow);
        }
        const int kt_id = KT_RAST_POST;
        if (A.textured)
            kt_launch(kt_id, (rast_post_kernel<false, true>), dim3(post_grid), dim3(256), 0, st, d_tris, A,
                               (const void *)state, (const RowRec *)recs, (const int32_t *)nullptr, d_argb);
        else
            kt_launch(kt_id, (rast_post_kernel<false, false>), dim3(post_grid), dim3(256), 0, st, d_tris, A,
                               (const void *)state, (const RowRec *)recs, (const int32_t *)nullptr, d_argb);
        if (stats) stats->n_shaded = -1;
    }
    if ((e = hipGetLastError()) != hipSuccess) return ctx_fail(c, e, "rast_post launch");
    if (stats && (e = hipEventRecord(e1, st)) != hipSuccess) return ctx_fail(c, e, "event");
    if (stats) {
        stats->n_tris = n_dev ? -1 : n;
        stats->n_spans = 0;
    }
    return CG_OK;
}

}  // namespace cg
