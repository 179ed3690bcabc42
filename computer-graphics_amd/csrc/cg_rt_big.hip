// cg_rt_big.hip -- raytracer hot path for large scenes (n_tris > 64, e.g. the
// build-defined C5 workload: 1M random triangles), same Draw semantics as
// cg_rt.hip (raytracer/Source/skeleton.cpp:104-169, ClosestIntersection
// :263-363, DirectLight :366-415), bit-identical to brute force.
//
// The per-wave culling certificates of cg_rt_dev.h are exact for any ray
// bundle, so they are applied hierarchically:
//   K0 rt_bin_primary    per (bin of 128x32 pixels, triangle): camera-ray
//                        certificate of the bin's bundle -> bin list, each
//                        entry with a certified lower bound ("key") on the
//                        float distance any ray of the bin can compute for it;
//      rt_bin_count / rt_bin_scan / rt_bin_scatter
//                        bucket each bin list by key (kDepthBuckets);
//   K1 rt_big_primary    per 8x8 wave: the bin's buckets nearest first; a
//                        candidate whose key exceeds every lane's current best
//                        distance cannot win and is skipped (exact: ties need
//                        distance == best <= key); certificate of the wave's
//                        bundle (64 candidates per pass, one per lane), then
//                        the closest-hit walk for the 9 sub-rays; hits
//                        (index, t) to HBM, the wave's shadow-ray box too;
//   K2 rt_bin_boxes      union of the wave boxes of each bin;
//   K3 rt_bin_shadow     per (bin, triangle): shadow-ray certificate of the
//                        light set against the bin's box -> shadow bin list;
//   K4 rt_big_shade      per wave: certificate against its own box, the
//                        survivors staged in LDS, DirectLight for every hit
//                        and light in the reference's order, PutPixelSDL.
// Bin lists are unordered (atomics): the closest hit is the minimum of
// (distance, index) over the valid hits, which is exactly what the
// reference's ascending loop with `distance >= best -> skip` returns, and a
// shadow test is an any-hit search, so visiting order does not matter.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <vector>

#include "cg_rt_dev.h"

namespace cg {

constexpr int kBinW = 128, kBinH = 32;        // pixels; multiples of the 8x8 wave tile
constexpr int kBinTilesX = kBinW / 8, kBinTilesY = kBinH / 8;
static_assert(kBinTilesX * kBinTilesY == 64, "one wave tile per lane in rt_bin_boxes");
constexpr int kBinTris = 1024;                // triangles per workgroup in the bin kernels
constexpr int kMaxPend = 65536;               // queue of shadow rays K4 leaves to K5 (the lit search)
constexpr int kSupBins = 4;                   // a super-bin is 4 x 4 bins (512 x 128 px)
constexpr int kDepthBuckets = 32;             // per bin: 0 = no key (det's sign uncertain), 1.. by key

// A shadow ray K4 could not resolve (skeleton.cpp:394 arguments, reference
// float values) and where its verdict goes.
struct PendRay {
    float ox, oy, oz, nx, ny, nz, len, rmag;
    int pix, bit;
};

// Pooled lists.  A list (the triangles a super-bin keeps, a bin's entries, a
// bin's shadow candidates) is a sequence of chunks in one pool per kind, a
// chunk being the survivors of one workgroup pass over <= 1024 candidates
// (one pool reservation); chunk c of list k is chunk[k * nch + c].  Pool
// capacities come from the host (cg_shim.hip: sized on a scene's first
// frame, grown from the demand each later frame reports); a reservation past
// the capacity marks the list overflowed and its consumers fall back to
// every triangle -- slower, the same image -- while the full demand is still
// counted for the host.
struct Chunk {
    int off, n;
};
enum { kPoolSup = 0, kPoolBin = 1, kPoolSbin = 2, kPoolSorted = 3 };

struct BigBufs {
    // primary bin lists with keys: key bits << 32 | triangle, unsorted (pool) and by bucket
    unsigned long long *bin_ent;                       // [cap_bin]
    unsigned long long *bin_pbox, *bin_pbox2;          // [cap_bin]: projected boxes (proj_box16) for the
                                                       // bin's left / right half, same order
    Chunk *bin_chunk;             // [n_bins][nch]
    int *bin_nch;                 // [n_bins]: chunks in use
    int *bin_pre, *bin_tot;       // [n_bins][nch]: entries before each chunk; [n_bins]: list sizes
    // the bin lists compacted (rt_bin_count_kernel): bin b at [bin_base[b], + bin_tot[b])
    unsigned long long *flat_ent, *flat_pbox, *flat_pbox2;   // [cap_bin]
    int *bin_base;                // [n_bins]
    // per half-bin (sub = 2 bin + half): the entries whose box meets the half, by bucket (global offsets)
    unsigned long long *bin_sorted, *bin_spbox;        // [cap_sorted]
    int *bkt_cnt;                 // [2 n_bins][kDepthBuckets]: counts, then scatter cursors
    int *bkt_off;                 // [2 n_bins][kDepthBuckets + 1]
    unsigned *bkt_min_inv;        // [2 n_bins][kDepthBuckets]: ~(smallest key bits) (0 = empty)
    unsigned *key_lo_inv, *key_hi;                     // [n_bins]: ~min / max bits of the positive keys
    int *sbin_pool;               // [cap_sbin] shadow candidates of the many-light path
    Chunk *sbin_chunk;            // [n_bins][nch]
    int *hit_bi;                  // ray slots (K1): closest hit index
    float *hit_t;
    ShadowBox *wave_box;          // [tiles_y][tiles_x]
    ShadowBox *bin_box;           // [n_bins]
    RtGrid grid;
    // shadow verdicts (9 * n_lights <= 64): per pixel, bit s * n_lights + l
    unsigned long long *sh_bits, *pend_bits;
    int *pend_n;                  // shadow rays left unresolved by K4 (counter)
    struct PendRay *pend_ray;     // [kMaxPend]
    int max_pend;                 // queue capacity used (<= kMaxPend; lowered only by cg_rt_set_pending_cap)
    // certified lit search (K5): triangles near the light, the walk margin and
    // the frame's bounds on |r| (componentwise) and on |p|
    int *near_list, *near_n;      // [n_tris], counter (pend_n[1])
    float lit_M;
    double litD[3], lit_pn;
    int bins_x, bins_y, tiles_x, tiles_y;
    int lat_w, lat_h;             // lattice mode: (2 W + 1) x (2 rows + 1) points; 0 = per-pixel mode
    int lat_yaw;                  // lattice columns per pixel (yawed camera): 3 W x (2 rows + 1) points
    int *sup_pool;                // [cap_sup] triangles the super-bins' certificates keep
    unsigned long long *sup_pbox_pool, *sup_flat_pbox;   // [cap_sup]: their projected boxes (super-bin bundle)
    Chunk *sup_chunk;             // [n_sups][nch]
    int *sup_pre, *sup_tot;       // [n_sups][nch], [n_sups] (as bin_pre / bin_tot)
    int *sup_flat, *sup_base;     // [cap_sup]: the super lists compacted, super-bin s at sup_base[s]
    int sups_x, sups_y;
    int nch;                      // chunks per list: ceil(n_tris / kBinTris)
    unsigned long long *pool_n;   // [4] demand per pool (kPool*; the sorted pool's is its total)
    long long cap_sup, cap_bin, cap_sbin, cap_sorted;  // pool capacities (entries)
    int *sup_over, *bin_over, *sbin_over;              // [n_sups], [n_bins], [n_bins]: list overflowed
    float *tile_bb;               // [2 n_bins][32][4]: each half-bin's wave-tile bundles (rt_half_mask_kernel)
    int *walk_order;              // [tiles]: the walk's workgroups, longest half-bin list first (null: grid order)
};

// ---------------------------------------------------------------------------
// One triangle, one camera sub-ray (camera-origin constants of RtTri):
// lexicographic (distance, index) minimum.
__device__ __forceinline__ void tri_closest(const RtTri &c, int k, vec3 nd, float len, float &best,
                                            float &bt, int &bi)
{
    cg_work(W_T_PRI);
    float Q2 = nd.y * c.e2z - c.e2y * nd.z;
    float Q1 = nd.y * c.e1z - c.e1y * nd.z;
    float det = (nd.x * c.K1 - c.e1x * Q2) + c.e2x * Q1;      // det(-d, e1, e2) :289
    if (surely_negative(c.detT, det, len)) return;
    if (best < FLT_MAX && surely_beyond(c.detT, det, len, best)) return;
    float t = c.detT / det;                                    // :306
    float distance = t * len;                                  // :307
    if (distance < 0.0f) return;                               // :311
    if (distance > best || distance > FLT_MAX) return;         // :313
    if (distance == best && k > bi) return;                    // ascending-index tie-break
    cg_work(W_UV_PRI);
    float Q3 = nd.y * c.sz - c.sy * nd.z;
    float detU = (nd.x * c.K2 - c.sx * Q2) + c.e2x * Q3;      // :317
    float detV = (nd.x * c.K3 - c.e1x * Q3) + c.sx * Q1;      // :320
    float u = detU / det;
    float v = detV / det;
    if ((u >= 0) && (v >= 0) && ((u + v) <= 1)) {             // :328-335
        best = distance;
        bt = t;
        bi = k;
    }
}

// One triangle, one shadow ray from `start` (generic start): accepted hit
// with distance < rmag (skeleton.cpp:394-395).
__device__ __forceinline__ bool tri_shadows(const RtTri &c, vec3 start, vec3 nd, float len, float rmag)
{
    cg_work(W_T_SH);
    float sx = start.x - c.v0x, sy = start.y - c.v0y, sz = start.z - c.v0z;   // :296
    float Q2 = nd.y * c.e2z - c.e2y * nd.z;
    float Q1 = nd.y * c.e1z - c.e1y * nd.z;
    float det = (nd.x * c.K1 - c.e1x * Q2) + c.e2x * Q1;
    float K2 = sy * c.e2z - c.e2y * sz;
    float K4 = sy * c.e1z - c.e1y * sz;
    float detT = (sx * c.K1 - c.e1x * K2) + c.e2x * K4;
    if (surely_negative(detT, det, len) || surely_beyond(detT, det, len, rmag)) return false;
    float Q3 = nd.y * sz - sy * nd.z;
    float K3 = c.e1y * sz - sy * c.e1z;
    float detU = (nd.x * K2 - sx * Q2) + c.e2x * Q3;
    float detV = (nd.x * K3 - c.e1x * Q3) + sx * Q1;
    // a certain u / v rejection (uv_decide: signs and the sum against det with
    // rounding margins) needs no divide; the conditions are a conjunction, so
    // testing them in another order gives the same verdict
    if (uv_decide(det, detU, detV) == 0) return false;
    float t = detT / det;
    float distance = t * len;
    if (distance < 0.0f) return false;
    if (distance >= rmag || distance > FLT_MAX) return false;
    cg_work(W_UV_SH);
    float u = detU / det;
    float v = detV / det;
    return (u >= 0) && (v >= 0) && ((u + v) <= 1);
}

// Exact float extremes of the camera sub-ray directions of a bin: dir =
// R (u - W/2, v - H/2, f, 1) is monotone in u and in v (each float op is),
// so the extremes are at the bin's corner pixels; +-0.5 as in the wave box.
__device__ bool bin_bundle(const RtFrame &F, int bx, int by, float &x0, float &x1, float &y0, float &y1)
{
    const int u0 = bx * kBinW, u1 = min(F.W, u0 + kBinW) - 1;
    const int L0 = by * kBinH, L1 = min(F.rows_out, L0 + kBinH) - 1;
    const int v0 = shard_row(F, L0);
    if (v0 >= F.H) return false;                      // padding rows only
    const int v1 = min(shard_row(F, L1), F.H - 1);   // shard_row is increasing in L
    x0 = y0 = FLT_MAX;
    x1 = y1 = -FLT_MAX;
    const int us[2] = {u0, u1}, vs[2] = {v0, v1};
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
            vec4 d = mat4_mul(F.R, v4((float)(us[a] - F.W / 2), (float)(vs[b] - F.H / 2), F.focal, 1.0f));
            x0 = fminf(x0, d.x); x1 = fmaxf(x1, d.x);
            y0 = fminf(y0, d.y); y1 = fmaxf(y1, d.y);
        }
    x0 = x0 - 0.5f; x1 = x1 + 0.5f; y0 = y0 - 0.5f; y1 = y1 + 0.5f;
    return true;
}

// The same for the super-bin (sx, sy): kSupBins x kSupBins bins.
__device__ bool sup_bundle(const RtFrame &F, int sx, int sy, float &x0, float &x1, float &y0, float &y1)
{
    const int u0 = sx * kSupBins * kBinW, u1 = min(F.W, u0 + kSupBins * kBinW) - 1;
    const int L0 = sy * kSupBins * kBinH, L1 = min(F.rows_out, L0 + kSupBins * kBinH) - 1;
    if (u0 > u1 || L0 > L1) return false;
    const int v0 = shard_row(F, L0);
    if (v0 >= F.H) return false;
    const int v1 = min(shard_row(F, L1), F.H - 1);
    x0 = y0 = FLT_MAX;
    x1 = y1 = -FLT_MAX;
    const int us[2] = {u0, u1}, vs[2] = {v0, v1};
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
            vec4 d = mat4_mul(F.R, v4((float)(us[a] - F.W / 2), (float)(vs[b] - F.H / 2), F.focal, 1.0f));
            x0 = fminf(x0, d.x); x1 = fmaxf(x1, d.x);
            y0 = fminf(y0, d.y); y1 = fmaxf(y1, d.y);
        }
    x0 = x0 - 0.5f; x1 = x1 + 0.5f; y0 = y0 - 0.5f; y1 = y1 + 0.5f;
    return true;
}

// The same for columns [part * kBinW / 2, (part + 1) * kBinW / 2) of the bin
// (its left / right half); false when that half has no pixel.
__device__ bool bin_half_bundle(const RtFrame &F, int bx, int by, int part, float &x0, float &x1, float &y0,
                                float &y1)
{
    const int u0 = bx * kBinW + part * (kBinW / 2), u1 = min(F.W, u0 + kBinW / 2) - 1;
    if (u0 > u1) return false;
    const int L0 = by * kBinH, L1 = min(F.rows_out, L0 + kBinH) - 1;
    const int v0 = shard_row(F, L0);
    if (v0 >= F.H) return false;
    const int v1 = min(shard_row(F, L1), F.H - 1);
    x0 = y0 = FLT_MAX;
    x1 = y1 = -FLT_MAX;
    const int us[2] = {u0, u1}, vs[2] = {v0, v1};
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
            vec4 d = mat4_mul(F.R, v4((float)(us[a] - F.W / 2), (float)(vs[b] - F.H / 2), F.focal, 1.0f));
            x0 = fminf(x0, d.x); x1 = fmaxf(x1, d.x);
            y0 = fminf(y0, d.y); y1 = fmaxf(y1, d.y);
        }
    x0 = x0 - 0.5f; x1 = x1 + 0.5f; y0 = y0 - 0.5f; y1 = y1 + 0.5f;
    return true;
}

// The same for the 8x8-pixel wave tile (tx, ty); false without pixels.
__device__ bool tile_bundle(const RtFrame &F, int tx, int ty, float &x0, float &x1, float &y0, float &y1)
{
    const int u0 = tx * 8, u1 = min(F.W, u0 + 8) - 1;
    const int L0 = ty * 8, L1 = min(F.rows_out, L0 + 8) - 1;
    if (u0 > u1 || L0 > L1) return false;
    const int v0 = shard_row(F, L0);
    if (v0 >= F.H) return false;
    const int v1 = min(shard_row(F, L1), F.H - 1);
    x0 = y0 = FLT_MAX;
    x1 = y1 = -FLT_MAX;
    const int us[2] = {u0, u1}, vs[2] = {v0, v1};
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
            vec4 d = mat4_mul(F.R, v4((float)(us[a] - F.W / 2), (float)(vs[b] - F.H / 2), F.focal, 1.0f));
            x0 = fminf(x0, d.x); x1 = fmaxf(x1, d.x);
            y0 = fminf(y0, d.y); y1 = fmaxf(y1, d.y);
        }
    x0 = x0 - 0.5f; x1 = x1 + 0.5f; y0 = y0 - 0.5f; y1 = y1 + 0.5f;
    return true;
}

// Reserve tot pool entries (thread 0): the offset, or -1 past the capacity
// (the list is then marked overflowed).  The demand is counted either way.
__device__ __forceinline__ int pool_reserve(unsigned long long *pool_n, long long cap, int tot, int *over)
{
    if (!tot) return 0;
    const unsigned long long g = atomicAdd(pool_n, (unsigned long long)tot);
    if ((long long)g + tot > cap) {
        *over = 1;
        return -1;
    }
    return (int)g;
}

// Append this workgroup's kept triangles (kept[r]: triangle base + r*256 +
// tid) to a pooled list as one chunk, recorded in *slot.
__device__ __forceinline__ void pooled_append(const bool kept[4], int base, int *pool, unsigned long long *pool_n,
                                              long long cap, Chunk *slot, int *over,
                                              const unsigned long long *val = nullptr, unsigned long long *vpool = nullptr)
{
    __shared__ int s_w[4][4];
    __shared__ int s_base;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    unsigned long long m[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        m[r] = __ballot(kept[r]);
        if (lane == 0) s_w[r][w] = __popcll(m[r]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int r = 0; r < 4; ++r)
            for (int q = 0; q < 4; ++q) tot += s_w[r][q];
        const int g = pool_reserve(pool_n, cap, tot, over);
        *slot = Chunk{g < 0 ? 0 : g, g < 0 ? 0 : tot};
        s_base = g;
    }
    __syncthreads();
    if (s_base < 0) return;
    int off = s_base;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        int before = 0;
        for (int q = 0; q < 4; ++q) before += q < w ? s_w[r][q] : 0;
        if (kept[r]) {
            const int at = off + before + __popcll(m[r] & lt);
            pool[at] = base + r * 256 + (int)threadIdx.x;
            if (vpool) vpool[at] = val[r];
        }
        for (int q = 0; q < 4; ++q) off += s_w[r][q];
    }
}

// Prefix sums of the chunk tables (one workgroup per list): pre[c] = entries
// of the list before chunk c, tot = the list's size.  Consumers then walk a
// list by flat index in full 1024-entry passes, whatever its chunks' sizes.
__global__ __launch_bounds__(1024) void rt_chunk_scan_kernel(const Chunk *__restrict__ tab, const int *__restrict__ ncs,
                                                             int nch, int *__restrict__ pre, int *__restrict__ tot)
{
    const int list = blockIdx.x, nc = ncs ? ncs[list] : nch;
    const Chunk *t = tab + (size_t)list * nch;
    int *p = pre + (size_t)list * nch;
    __shared__ int s_wave[16];
    __shared__ int s_carry;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (int c0 = 0; c0 < nc; c0 += 1024) {
        const int c = c0 + (int)threadIdx.x;
        const int n = c < nc ? t[c].n : 0;
        int x = n;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_wave[w] = x;
        __syncthreads();
        int before = s_carry;
        for (int q = 0; q < w; ++q) before += s_wave[q];
        if (c < nc) p[c] = before + x - n;
        __syncthreads();
        if (threadIdx.x == 1023) s_carry = before + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) tot[list] = s_carry;
}

// Exclusive prefix of n list sizes (one workgroup): where each list starts
// in its compacted array.
__global__ __launch_bounds__(1024) void rt_list_base_kernel(const int *__restrict__ tot, int n, int *__restrict__ base)
{
    __shared__ int s_wave[16];
    __shared__ int s_carry;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (int i0 = 0; i0 < n; i0 += 1024) {
        const int i = i0 + (int)threadIdx.x;
        const int v = i < n ? tot[i] : 0;
        int x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_wave[w] = x;
        __syncthreads();
        int before = s_carry;
        for (int q = 0; q < w; ++q) before += s_wave[q];
        if (i < n) base[i] = before + x - v;
        __syncthreads();
        if (threadIdx.x == 1023) s_carry = before + x;
        __syncthreads();
    }
}

// Append the kept triangles of this workgroup to a plain list (one atomic per
// workgroup); kept[r] is this thread's verdict on triangle base + r*256 + tid.
__device__ __forceinline__ void bin_append(const bool kept[4], int base, int *list, int *count)
{
    __shared__ int s_w[4][4];
    __shared__ int s_base;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    unsigned long long m[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        m[r] = __ballot(kept[r]);
        if (lane == 0) s_w[r][w] = __popcll(m[r]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int r = 0; r < 4; ++r)
            for (int q = 0; q < 4; ++q) tot += s_w[r][q];
        s_base = tot ? atomicAdd(count, tot) : 0;
    }
    __syncthreads();
    int off = s_base;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        int before = 0;
        for (int q = 0; q < 4; ++q) before += q < w ? s_w[r][q] : 0;
        if (kept[r]) list[off + before + __popcll(m[r] & lt)] = base + r * 256 + (int)threadIdx.x;
        for (int q = 0; q < 4; ++q) off += s_w[r][q];
    }
}

// Box (in the bundle's (x, y) units, 4 x int16: x0 | x1 << 16 | y0 << 32 |
// y1 << 48) holding the direction (x, y) of every camera ray of the bin that
// the reference's test can accept for this triangle.  With det's sign certain
// (pd: the bin's PrimDet), an accepted hit's exact plane point X lies in the
// triangle (v0, v0 + e1, v0 + e2) widened by sig (|e1| + |e2|), sig = 2 (Ed +
// Eu + Ev) / dmin + 2^-21 (the barycentric slack of primary_hit_box), and the
// ray through X has x = f (X - cam).x / (X - cam).z (nd.z = f, :137).  Without
// a certain sign, with the widened box reaching the camera plane, or past the
// int16 range, the box is everything.  (Projecting the three vertices' boxes
// instead of the triangle's box measured no shorter lists for C5 and a
// slower super-bin pass.)
constexpr unsigned long long kProjAll = 0x7fff8000ull | (0x7fff8000ull << 32);
constexpr unsigned long long kProjNone = 0x80007fffull | (0x80007fffull << 32);   // x0 > x1: meets nothing
__device__ unsigned long long proj_box16(const RtTri &c, const PrimDet &pd, const float cam[4],
                                         float f)
{
    double dmin;
    if (pd.dlo - pd.Ed > 0) dmin = pd.dlo - pd.Ed;
    else if (pd.dhi + pd.Ed < 0) dmin = -(pd.dhi + pd.Ed);
    else return kProjAll;
    // the slack is used doubled below; far from the camera it is ~|s| / |e|
    // times the rounding of the dets (1e-3 .. 1e-2 for C5's small triangles)
    const double sig = 2.0 * (pd.Ed + pd.Eu + pd.Ev) / dmin + 0x1p-21;
    if (!(isfinite(sig) && sig < 4.0)) return kProjAll;   // exact bound for any slack; a wide box still prunes
    const double v0[3] = {(double)c.v0x, (double)c.v0y, (double)c.v0z};   // the Triangle's v0, as RtTri keeps it
    const double a1[3] = {(double)c.e1x, (double)c.e1y, (double)c.e1z}, a2[3] = {(double)c.e2x, (double)c.e2y, (double)c.e2z};
    double lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        const double p1 = v0[k] + a1[k], p2 = v0[k] + a2[k];
        const double m = 2.0 * sig * (fabs(a1[k]) + fabs(a2[k])) + 1e-12 * (fabs(v0[k]) + fabs(a1[k]) + fabs(a2[k]) +
                                                                      fabs((double)cam[k]));
        lo[k] = fmin(v0[k], fmin(p1, p2)) - m - (double)cam[k];
        hi[k] = fmax(v0[k], fmax(p1, p2)) + m - (double)cam[k];
    }
    if (!(lo[2] > 0.0) || !isfinite(hi[2])) return kProjAll;
    const double fd = f;
    auto range = [&](double l, double h, double &rl, double &rh) {
        rl = fd * (l >= 0.0 ? l / hi[2] : l / lo[2]);
        rh = fd * (h >= 0.0 ? h / lo[2] : h / hi[2]);
        rl -= 1e-9 * fabs(rl) + 1e-3;
        rh += 1e-9 * fabs(rh) + 1e-3;
    };
    double xl, xh, yl, yh;
    range(lo[0], hi[0], xl, xh);
    range(lo[1], hi[1], yl, yh);
    auto q = [](double v, bool up) -> unsigned long long {
        const double r = up ? ceil(v) : floor(v);
        return (unsigned long long)(unsigned short)(short)(int)r;
    };
    // past the int16 range (frames over 64k pixels wide; NaN fails too) no box
    if (!(xl >= -32768.0 && xh <= 32766.0 && yl >= -32768.0 && yh <= 32766.0)) return kProjAll;
    return q(xl, false) | (q(xh, true) << 16) | (q(yl, false) << 32) | (q(yh, true) << 48);
}

// Does the box of proj_box16 meet the bundle [x0, x1] x [y0, y1]?
__device__ __forceinline__ bool proj_meets(unsigned long long b, float x0, float x1, float y0, float y1)
{
    const float bx0 = (float)(short)(b & 0xffff), bx1 = (float)(short)((b >> 16) & 0xffff);
    const float by0 = (float)(short)((b >> 32) & 0xffff), by1 = (float)(short)((b >> 48) & 0xffff);
    return !(x1 < bx0 || x0 > bx1 || y1 < by0 || y0 > by1);
}

// max |det| over the directions (x, y, f), x in [x0, x1], y in [y0, y1], of
// the exact linear form det = -d.(e1 x e2) (cull_primary's lin_range; its
// FP64 rounding is far inside the 2^-20 margins the keys carry).
__device__ __forceinline__ double det_abs_max(const RtTri &c, float x0, float x1, float y0, float y1, float f)
{
    const double Nx = (double)c.e1y * c.e2z - (double)c.e2y * c.e1z, Ny = (double)c.e1z * c.e2x - (double)c.e2z * c.e1x,
                 Nz = (double)c.e1x * c.e2y - (double)c.e2x * c.e1y;
    double lo, hi;
    lin_range(0.5 * ((double)x0 + x1), 0.5 * ((double)y0 + y1), 0.5 * ((double)x1 - x0), 0.5 * ((double)y1 - y0), f,
              Nx, Ny, Nz, lo, hi);
    return fmax(fabs(lo), fabs(hi)) * (1.0 + 1e-12);
}

// A super-list entry without a box (det's sign uncertain over the super-bin:
// a plane its rays graze, typically a triangle seen nearly edge-on somewhere
// along that line) carries instead the mask of the super-bin's 16 bins whose
// own certificate keeps it: low word kMaskTag (x0 = 32767 > x1 = 32766:
// neither a real box nor kProjNone), high word the mask (bit bx + 4 by).
constexpr unsigned kMaskTag = 0x7ffe7fffu;
constexpr unsigned kNeedTag = 0x7ffd7fffu;   // a bucketed entry waiting for its tile mask (high word: half-bin)
__device__ __forceinline__ bool is_bin_mask(unsigned long long b) { return (unsigned)b == kMaskTag; }

// cull_primary's certificate of one triangle over nb <= 64 bundles bb[k] =
// (x0, x1, y0, y1; x0 > x1 for none) lying in the bundle [ex0, ex1] x [ey0,
// ey1]: bit k set when bundle k keeps it.  The linear forms are formed once
// and the error bounds taken over the enclosing bundle (its |d| maxima bound
// every inner bundle's, and 2e-12 max |form| over it bounds the 1e-12 (|lo| +
// |hi|) rounding term of any inner one); every test of the certificate only
// gets harder as the error bounds grow, so each cleared bit is a bundle the
// exact certificate culls too.  Branch-free per bundle.
__device__ unsigned long long bundle_mask(const RtTri &c, const float (*bb)[4], int nb, float ex0, float ex1,
                                          float ey0, float ey1, float f)
{
    const double eps = 5.9604644775390625e-8;   // 2^-24
    const double g = 16.0 * eps;
    const vec3 e1 = v3(c.e1x, c.e1y, c.e1z), e2 = v3(c.e2x, c.e2y, c.e2z), s = v3(c.sx, c.sy, c.sz);
    const double Nx = (double)e1.y * e2.z - (double)e2.y * e1.z, Ny = (double)e1.z * e2.x - (double)e2.z * e1.x,
                 Nz = (double)e1.x * e2.y - (double)e2.x * e1.y;
    const double Ax = (double)s.y * e2.z - (double)e2.y * s.z, Ay = (double)s.z * e2.x - (double)e2.z * s.x,
                 Az = (double)s.x * e2.y - (double)e2.x * s.y;
    const double Bx = (double)e1.y * s.z - (double)s.y * e1.z, By = (double)e1.z * s.x - (double)s.z * e1.x,
                 Bz = (double)e1.x * s.y - (double)s.x * e1.y;
    const double Cx = Ax + Bx - Nx, Cy = Ay + By - Ny, Cz = Az + Bz - Nz;
    const double fz = f;
    const double hcx = 0.5 * ((double)ex0 + ex1), hcy = 0.5 * ((double)ey0 + ey1);
    const double hhx = 0.5 * ((double)ex1 - ex0), hhy = 0.5 * ((double)ey1 - ey0);
    const double Dx = fmax(fabs((double)ex0), fabs((double)ex1)), Dy = fmax(fabs((double)ey0), fabs((double)ey1)),
                 Dz = fabs(fz);
    auto amax = [&](double X, double Y, double Z) {
        double lo, hi;
        lin_range(hcx, hcy, hhx, hhy, fz, X, Y, Z, lo, hi);
        return fmax(fabs(lo), fabs(hi));
    };
    const double Ed = g * det3_bound(Dx, Dy, Dz, e1, e2) + 2e-12 * amax(Nx, Ny, Nz);
    const double Eu = g * det3_bound(Dx, Dy, Dz, s, e2) + 2e-12 * amax(Ax, Ay, Az);
    const double Ev = g * det3_bound(Dx, Dy, Dz, e1, s) + 2e-12 * amax(Bx, By, Bz);
    const double Eb = Ed + Eu + Ev + 2e-12 * amax(Cx, Cy, Cz);
    const double dT = c.detT;
    if (!isfinite(Ed + Eu + Ev + Eb)) return ~0ull;
    const double four_eps = 4.0 * eps;
    unsigned long long mask = 0ull;
    for (int k = 0; k < nb; ++k) {
        const float x0 = bb[k][0], x1 = bb[k][1], y0 = bb[k][2], y1 = bb[k][3];
        const double cx = 0.5 * ((double)x0 + x1), cy = 0.5 * ((double)y0 + y1);
        const double hx = 0.5 * ((double)x1 - x0), hy = 0.5 * ((double)y1 - y0);
        double dlo, dhi, ulo, uhi, vlo, vhi, blo, bhi;
        lin_range(cx, cy, hx, hy, fz, Nx, Ny, Nz, dlo, dhi);
        lin_range(cx, cy, hx, hy, fz, Ax, Ay, Az, ulo, uhi);
        lin_range(cx, cy, hx, hy, fz, Bx, By, Bz, vlo, vhi);
        lin_range(cx, cy, hx, hy, fz, Cx, Cy, Cz, blo, bhi);
        const bool pos = dlo - Ed > 0, neg = dhi + Ed < 0;
        // det's sign certain: cull_primary's tests
        const double dmin = pos ? dlo - Ed : -(dhi + Ed);
        const double dmax = pos ? dhi + Ed : -(dlo - Ed);
        const double tiny = 1e-20 * dmax;
        const double umx = fmax(fabs(ulo), fabs(uhi)) + Eu, vmx = fmax(fabs(vlo), fabs(vhi)) + Ev;
        const double num = pos ? blo - Eb : -(bhi + Eb);
        const bool c_sure = (dT != 0.0 && ((dT > 0) != pos) && fabs(dT) > tiny) |
                            (pos ? (uhi + Eu < -tiny) : (ulo - Eu > tiny)) |
                            (pos ? (vhi + Ev < -tiny) : (vlo - Ev > tiny)) |
                            (num > 0.0 && num * dmin > four_eps * (umx + vmx + dmin) * dmax * (1.0 + 0x1p-40));
        // sign uncertain: sign_free_reject
        const double dmx = fmax(fabs(dlo - Ed), fabs(dhi + Ed));
        const double ftiny = 1e-20 * dmx;
        const double Ew = Eb * (1.0 + four_eps) + four_eps * (umx + vmx + dmx) + ftiny;
        const bool p_ok = !(dhi + Ed > 0.0) || (uhi + Eu < -ftiny) || (vhi + Ev < -ftiny) || (blo > Ew);
        const bool n_ok = !(dlo - Ed < 0.0) || (ulo - Eu > ftiny) || (vlo - Ev > ftiny) || (bhi < -Ew);
        const bool fin = isfinite(dlo) && isfinite(dhi) && isfinite(ulo + uhi + vlo + vhi + blo + bhi);
        const bool cull = fin & ((pos | neg) ? c_sure : (p_ok & n_ok));
        mask |= (unsigned long long)(!(x0 > x1) & !cull) << k;
    }
    return mask;
}

// K00: camera-ray certificate per (super-bin, triangle) -> super list; the
// bins then certify only their super-bin's survivors (a bin's bundle lies in
// its super-bin's, so a triangle the super-bin culls is culled for the bin).
// The certificate's edge-function tests alone keep a small triangle whose
// edge lines all cross the bundle (4-5x the triangles the super-bin's pixels
// see); its projected box (proj_box16 over the super-bin's PrimDet) is the
// missing separating axis: a box that misses the bundle culls it too, and
// the box travels with the entry so that the bins test it before gathering
// the triangle (every direction a super-bin ray can accept lies in it, and a
// bin's rays are super-bin rays).
//
// One workgroup per (1,024-triangle chunk, group of super-bins: blockIdx.y of
// sup_groups(), at most 64 super-bins each): each triangle's constants are
// read once per group and its linear forms formed once for all the group's
// bundles (bundle_mask: a cleared bit is a super-bin the
// certificate culls over the group's enclosing bundle, hence over its own),
// and only the surviving (super-bin, triangle) pairs -- ~2.5 per triangle at
// C5 -- run cull_primary and the projected box.  Round 4 ran one workgroup per
// (chunk, super-bin), re-reading the 64 MB of triangle constants and
// re-forming them for each of C5's 36 super-bins (2.8 GB of the frame's HBM
// traffic).  The lists are the same: a pair is kept iff cull_primary keeps
// it and its box meets the bundle, appended in ascending triangle order, one
// chunk per (super-bin, workgroup) as before.
constexpr int kSupGroup = 64;
// Super-bin groups per chunk: at least 4 (C5's 36 super-bins: 4 groups of 9), so the
// pass has ~4 workgroups per chunk in flight rather than one long one.
__host__ __device__ __forceinline__ int sup_groups(int nsup) { return max(4, (nsup + kSupGroup - 1) / kSupGroup); }
#ifndef CG_SUP_WAVES
#define CG_SUP_WAVES 3   // 168 VGPRs; 2 waves (182) 562 us, 4 waves (136 B scratch) 468, 3: 452 (C5, one frame; r05)
#endif
__global__ __launch_bounds__(256, CG_SUP_WAVES) void rt_sup_primary_kernel(RtFrame F, const RtGeo *__restrict__ geo,
                                                             RtTri *__restrict__ tc_out, BigBufs B)
{
    __shared__ float s_sb[kSupGroup][4];         // the group's super-bin bundles (x0 > x1: no pixel)
    __shared__ int s_cnt[kSupGroup][4][4];       // kept per (super-bin, triangle slot r, wave)
    __shared__ int s_base[kSupGroup];            // the chunk's pool offset per super-bin (-1: overflow)
    const int nsup = B.sups_x * B.sups_y, base = blockIdx.x * kBinTris;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const int gsz = (nsup + (int)gridDim.y - 1) / (int)gridDim.y;   // <= kSupGroup
    {
        const int g0 = (int)blockIdx.y * gsz;
        const int ng = min(gsz, nsup - g0);
        if (ng <= 0) return;
        if ((int)threadIdx.x < ng) {
            const int sup = g0 + (int)threadIdx.x;
            float *q = s_sb[threadIdx.x];
            if (!sup_bundle(F, sup % B.sups_x, sup / B.sups_x, q[0], q[1], q[2], q[3])) {
                q[0] = 1.0f;
                q[1] = 0.0f;
                q[2] = q[3] = 0.0f;
            }
        }
        __syncthreads();
        float ex0 = FLT_MAX, ex1 = -FLT_MAX, ey0 = FLT_MAX, ey1 = -FLT_MAX;   // the enclosing bundle
        unsigned long long valid = 0ull;   // the group's super-bins with pixels
        for (int k = 0; k < ng; ++k)
            if (!(s_sb[k][0] > s_sb[k][1])) {
                valid |= 1ull << k;
                ex0 = fminf(ex0, s_sb[k][0]);
                ex1 = fmaxf(ex1, s_sb[k][1]);
                ey0 = fminf(ey0, s_sb[k][2]);
                ey1 = fmaxf(ey1, s_sb[k][3]);
            }
        // kept[r] bit k: triangle base + r * 256 + tid for super-bin g0 + k; the boxes of
        // each triangle's first two kept super-bins are kept for the write pass
        unsigned long long km[4], pbc[4][2];
        int kc[4][2];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            kc[r][0] = kc[r][1] = -1;
            pbc[r][0] = pbc[r][1] = kProjAll;
            const int i = base + r * 256 + (int)threadIdx.x;
            // (bundle_mask answers ~0 when its error terms are not finite: every valid bundle is tested)
            // the frame's RtTri of triangle i, formed here from the scene's RtGeo (rt_tri_frame,
            // bit for bit rt_tri_const) and published by the first group's workgroups for the
            // later passes -- no separate prepare launch for large scenes
            RtTri c{};
            if (i < F.n_tris) {
                c = rt_tri_frame(geo[i], F.cam);
                if (blockIdx.y == 0) tc_out[i] = c;
            }
            unsigned long long m = (i < F.n_tris && valid)
                                       ? bundle_mask(c, s_sb, ng, ex0, ex1, ey0, ey1, F.focal) & valid : 0ull;
            unsigned long long kept = 0ull;
            while (m) {
                const int k = __builtin_ctzll(m);
                m &= m - 1ull;
                const float x0 = s_sb[k][0], x1 = s_sb[k][1], y0 = s_sb[k][2], y1 = s_sb[k][3];
                PrimDet pd;
                if (!cull_primary(c, x0, x1, y0, y1, F.focal, &pd)) {
                    const unsigned long long pb = proj_box16(c, pd, F.cam, F.focal);
                    if (proj_meets(pb, x0, x1, y0, y1)) {
                        if (kc[r][0] < 0) {
                            kc[r][0] = k;
                            pbc[r][0] = pb;
                        } else if (kc[r][1] < 0) {
                            kc[r][1] = k;
                            pbc[r][1] = pb;
                        }
                        kept |= 1ull << k;
                    }
                }
            }
            km[r] = kept;
        }
        // counts per (super-bin, r, wave), then one pool reservation per super-bin
        for (int k = 0; k < ng; ++k)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const unsigned long long b = __ballot((km[r] >> k) & 1ull);
                if (lane == 0) s_cnt[k][r][w] = __popcll(b);
            }
        __syncthreads();
        if ((int)threadIdx.x < ng) {
            const int k = (int)threadIdx.x, sup = g0 + k;
            int tot = 0;
            for (int r = 0; r < 4; ++r)
                for (int q = 0; q < 4; ++q) tot += s_cnt[k][r][q];
            const int g = pool_reserve(B.pool_n + kPoolSup, B.cap_sup, tot, B.sup_over + sup);
            B.sup_chunk[(size_t)sup * B.nch + blockIdx.x] = Chunk{g < 0 ? 0 : g, g < 0 ? 0 : tot};
            s_base[k] = g;
        }
        __syncthreads();
        // the entries, in ascending triangle order within each chunk (pooled_append's)
        for (int k = 0; k < ng; ++k) {
            if (s_base[k] < 0) continue;   // overflowed: the list is redone at a larger capacity
            int off = s_base[k];
            const float x0 = s_sb[k][0], x1 = s_sb[k][1], y0 = s_sb[k][2], y1 = s_sb[k][3];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool kr = (km[r] >> k) & 1ull;
                const unsigned long long b = __ballot(kr);
                int before = 0;
                for (int q = 0; q < 4; ++q) before += q < w ? s_cnt[k][r][q] : 0;
                if (kr) {
                    const int i = base + r * 256 + (int)threadIdx.x;
                    unsigned long long pb;
                    if (kc[r][0] == k) {
                        pb = pbc[r][0];
                    } else if (kc[r][1] == k) {
                        pb = pbc[r][1];
                    } else {   // a third or later kept super-bin: the same box again
                        const RtTri c = rt_tri_frame(geo[i], F.cam);
                        PrimDet pd;
                        (void)cull_primary(c, x0, x1, y0, y1, F.focal, &pd);
                        pb = proj_box16(c, pd, F.cam, F.focal);
                    }
                    const int at = off + before + __popcll(b & lt);
                    B.sup_pool[at] = i;
                    B.sup_pbox_pool[at] = pb;
                }
                for (int q = 0; q < 4; ++q) off += s_cnt[k][r][q];
            }
        }
    }
}

// The super lists' chunks copied into one contiguous array per super-bin.
// (An entry without a box gets its bin mask here, in a dense pass.)
constexpr int kCompactPre = 4096;   // chunk prefixes staged in LDS (lists of up to 4M triangles)
__global__ __launch_bounds__(256, 6) void rt_sup_compact_kernel(RtFrame F, const RtTri *__restrict__ tc, BigBufs B)
{
    const int sup = blockIdx.y;
    if (B.sup_over[sup]) return;
    const int tot = B.sup_tot[sup];
    if ((int)blockIdx.x * 256 >= tot) return;
    __shared__ float s_bb[kSupBins * kSupBins][4];   // the super-bin's bins' bundles
    __shared__ int s_pre[kCompactPre];
    const int sx = sup % B.sups_x, sy = sup / B.sups_x;
    float ex0, ex1, ey0, ey1;
    const bool sv = sup_bundle(F, sx, sy, ex0, ex1, ey0, ey1);
    if (threadIdx.x < kSupBins * kSupBins) {
        const int bx = sx * kSupBins + (int)threadIdx.x % kSupBins, by = sy * kSupBins + (int)threadIdx.x / kSupBins;
        float *q = s_bb[threadIdx.x];
        if (!(bx < B.bins_x && by < B.bins_y && bin_bundle(F, bx, by, q[0], q[1], q[2], q[3]))) {
            q[0] = 1.0f;
            q[1] = 0.0f;
        }
    }
    const int nch = B.nch;
    const int *pre = B.sup_pre + (size_t)sup * nch;
    const bool lds = nch <= kCompactPre;
    if (lds)
        for (int c = (int)threadIdx.x; c < nch; c += 256) s_pre[c] = pre[c];
    __syncthreads();
    const Chunk *tab = B.sup_chunk + (size_t)sup * nch;
    const size_t at = (size_t)B.sup_base[sup];
    // the list's entries in flat order, strided over the super-bin's workgroups: entry j lies in
    // the last chunk c with pre[c] <= j (an empty chunk shares its successor's prefix)
    // (entries without a box -- a minority -- are queued in LDS and given their bin masks 256 at
    // a time, so bundle_mask runs on full waves)
    __shared__ int s_qi[512], s_qj[512];
    __shared__ int s_w[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    int qn = 0;   // queued (workgroup-uniform)
    auto masked = [&](int i, int j) {
        const unsigned long long m = bundle_mask(tc[i], s_bb, kSupBins * kSupBins, ex0, ex1, ey0, ey1, F.focal);
        B.sup_flat_pbox[at + j] = m ? (m << 32) | kMaskTag : kProjNone;
    };
    for (int j0 = (int)blockIdx.x * 256; j0 < tot; j0 += (int)gridDim.x * 256) {   // workgroup-uniform bounds
        const int j = j0 + (int)threadIdx.x;
        bool need = false;
        int i = 0;
        if (j < tot) {
            int lo = 0, hi = nch - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if ((lds ? s_pre[mid] : pre[mid]) <= j) lo = mid;
                else hi = mid - 1;
            }
            const Chunk ch = tab[lo];
            const int e = j - (lds ? s_pre[lo] : pre[lo]);
            i = B.sup_pool[ch.off + e];
            const unsigned long long pb = B.sup_pbox_pool[ch.off + e];
            B.sup_flat[at + j] = i;
            need = pb == kProjAll && sv;
            if (!need) B.sup_flat_pbox[at + j] = pb;
        }
        const unsigned long long m = __ballot(need);
        if (lane == 0) s_w[w] = __popcll(m);
        __syncthreads();
        int before = qn;
        for (int q = 0; q < w; ++q) before += s_w[q];
        if (need) {
            s_qi[before + __popcll(m & lt)] = i;
            s_qj[before + __popcll(m & lt)] = j;
        }
        qn += s_w[0] + s_w[1] + s_w[2] + s_w[3];
        __syncthreads();
        if (qn >= 256) {
            masked(s_qi[threadIdx.x], s_qj[threadIdx.x]);
            const bool mv = (int)threadIdx.x + 256 < qn;
            const int mi = mv ? s_qi[threadIdx.x + 256] : 0, mj = mv ? s_qj[threadIdx.x + 256] : 0;
            __syncthreads();
            if (mv) {
                s_qi[threadIdx.x] = mi;
                s_qj[threadIdx.x] = mj;
            }
            qn -= 256;
            __syncthreads();
        }
    }
    if ((int)threadIdx.x < qn) masked(s_qi[threadIdx.x], s_qj[threadIdx.x]);
}

// K0: camera-ray certificate per (bin, triangle of its super list), with the
// key: every float distance fl(t |nd|) a ray of the bin computes for the
// triangle is >= key (t >= tlo by primary_t_range; |nd| >= f (1 - 2^-23)
// since nd.z = f, :137).
// The super-bin's box is tested first (no gather for a bin it misses: ~1 in
// 10 entries meets a bin), and the entries that pass are compacted into an
// LDS queue certified 1024 at a time, so that every lane of the FP64
// certificate has work; each certified batch is one chunk of the bin list
// (a workgroup's batches never outnumber its 1024-entry passes, so a list
// keeps <= nch chunks).
__device__ void bin_certify_batch(const RtFrame &F, const RtTri *__restrict__ tc, const cg_tri *__restrict__ tris,
                                  const BigBufs &B, int bin, bool all, const int *slist,
                                  const unsigned long long *sbox, const int *q, int cnt, float x0, float x1,
                                  float y0, float y1)
{
    __shared__ int s_w[4][4];
    __shared__ int s_base;
    __shared__ unsigned s_lo, s_hi;
    if (threadIdx.x == 0) {
        s_lo = 0u;
        s_hi = 0u;
    }
    bool kept[4], ranged[4];
    int tri[4];
    unsigned kbits[4];
    unsigned long long pbox[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int k = r * 256 + (int)threadIdx.x;
        const int e = k < cnt ? q[k] : -1;
        const int i = e >= 0 ? (all ? e : slist[e]) : 0;
        tri[r] = i;
        kept[r] = ranged[r] = false;
        kbits[r] = 0u;
        pbox[r] = kProjAll;
        if (e >= 0) {
            // the bin's own certificate and box; a box that misses the bin
            // culls, and without one of its own the bin keeps the super-bin's
            const unsigned long long sb = all ? kProjAll : sbox[e];
            PrimDet pd;
            kept[r] = !cull_primary(tc[i], x0, x1, y0, y1, F.focal, &pd);
            if (kept[r]) {
                unsigned long long b = proj_box16(tc[i], pd, F.cam, F.focal);
                if (b == kProjAll && !is_bin_mask(sb)) b = sb;
                kept[r] = proj_meets(b, x0, x1, y0, y1);
                pbox[r] = b;
                // the key: t = fl(detT / det_f) and an accepting ray's
                // direction lies in the box, so |t| >= |detT| / dabs (1 -
                // 2^-20) with dabs = max |det| + Ed over the bin's part of the
                // box -- a bound for that triangle's own rays, not the whole
                // bin's (the walk then meets it at its depth), and one
                // whatever det's sign.  Keys of triangles whose plane the
                // bin's rays graze (sign uncertain) stay out of the bin's
                // bucketing range (ranged)
                double dabs = fmax(fabs(pd.dlo - pd.Ed), fabs(pd.dhi + pd.Ed));
                if (kept[r] && b != kProjAll) {
                    const float bx0 = fmaxf(x0, (float)(short)(b & 0xffff)), bx1 = fminf(x1, (float)(short)((b >> 16) & 0xffff));
                    const float by0 = fmaxf(y0, (float)(short)((b >> 32) & 0xffff)), by1 = fminf(y1, (float)(short)((b >> 48) & 0xffff));
                    dabs = fmin(dabs, det_abs_max(tc[i], bx0, bx1, by0, by1, F.focal) + pd.Ed);
                }
                const double tlo = fabs((double)tc[i].detT) / dabs * (1.0 - 0x1p-20);
                if (kept[r] && isfinite(tlo) && tlo > 0.0) {
                    const double kd = fmin(tlo * (double)F.focal * (1.0 - 0x1p-20), (double)FLT_MAX);
                    float kf = (float)kd;
                    if ((double)kf > kd) kf = nextafterf(kf, 0.0f);
                    kbits[r] = __float_as_uint(kf);
                    ranged[r] = pd.dlo - pd.Ed > 0 || pd.dhi + pd.Ed < 0;
                }
            }
        }
    }
    __syncthreads();
    // append (one reservation per batch), and the bin's positive key range
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    unsigned long long m[4];
    unsigned lo_inv = 0u, hi = 0u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        m[r] = __ballot(kept[r]);
        if (lane == 0) s_w[r][w] = __popcll(m[r]);
        if (kept[r] && kbits[r] && ranged[r]) {
            lo_inv = max(lo_inv, ~kbits[r]);
            hi = max(hi, kbits[r]);
        }
    }
    for (int o = 32; o; o >>= 1) {
        lo_inv = max(lo_inv, (unsigned)__shfl_xor((int)lo_inv, o));
        hi = max(hi, (unsigned)__shfl_xor((int)hi, o));
    }
    if (lane == 0) {
        atomicMax(&s_lo, lo_inv);
        atomicMax(&s_hi, hi);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int r = 0; r < 4; ++r)
            for (int qq = 0; qq < 4; ++qq) tot += s_w[r][qq];
        const int g = pool_reserve(B.pool_n + kPoolBin, B.cap_bin, tot, B.bin_over + bin);
        s_base = tot ? g : -1;
        if (tot && g >= 0) {
            B.bin_chunk[(size_t)bin * B.nch + atomicAdd(B.bin_nch + bin, 1)] = Chunk{g, tot};
            atomicMax(B.key_lo_inv + bin, s_lo);
            atomicMax(B.key_hi + bin, s_hi);
        }
    }
    __syncthreads();
    if (s_base >= 0) {
        int off = s_base;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            int before = 0;
            for (int qq = 0; qq < 4; ++qq) before += qq < w ? s_w[r][qq] : 0;
            if (kept[r]) {
                const size_t at = (size_t)off + before + __popcll(m[r] & lt);
                B.bin_ent[at] = ((unsigned long long)kbits[r] << 32) | (unsigned)tri[r];
                B.bin_pbox[at] = pbox[r];
                B.bin_pbox2[at] = pbox[r];
            }
            for (int qq = 0; qq < 4; ++qq) off += s_w[r][qq];
        }
    }
    __syncthreads();                                        // s_w / s_base / s_lo reused by the next batch
}

#ifndef CG_BINP_WAVES
#define CG_BINP_WAVES 4   // A/B: -DCG_BINP_WAVES=n
#endif
__global__ __launch_bounds__(256, CG_BINP_WAVES) void rt_bin_primary_kernel(RtFrame F, const RtTri *__restrict__ tc,
                                                             const cg_tri *__restrict__ tris, BigBufs B)
{
    const int bin = blockIdx.y;
    float x0, x1, y0, y1;
    if (!bin_bundle(F, bin % B.bins_x, bin / B.bins_x, x0, x1, y0, y1)) return;
    const int bx = bin % B.bins_x, by = bin / B.bins_x;
    const int sup = (bx / kSupBins) + (by / kSupBins) * B.sups_x;
    const bool all = B.sup_over[sup] != 0;               // overflowed super list: every triangle
    const int ns = all ? F.n_tris : B.sup_tot[sup];
    const int *slist = B.sup_flat + (all ? 0 : B.sup_base[sup]);
    const unsigned long long *sbox = B.sup_flat_pbox + (all ? 0 : B.sup_base[sup]);
    const int lbin = (bx % kSupBins) + kSupBins * (by % kSupBins);   // its bit in the super-bin's bin masks
    __shared__ int s_q[2 * kBinTris];                     // super-list entries waiting for the certificate
    __shared__ int s_w[4][4];
    int qn = 0;                                           // queued (workgroup-uniform)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int base = blockIdx.x * kBinTris; base < ns; base += gridDim.x * kBinTris) {   // over the super list
        bool pass[4];
        unsigned long long m[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = base + r * 256 + (int)threadIdx.x;
            const unsigned long long sb = e < ns && !all ? sbox[e] : kProjAll;
            pass[r] = e < ns && (is_bin_mask(sb) ? ((sb >> (32 + lbin)) & 1ull) != 0ull : proj_meets(sb, x0, x1, y0, y1));
            m[r] = __ballot(pass[r]);
            if (lane == 0) s_w[r][w] = __popcll(m[r]);
        }
        __syncthreads();
        int off = qn;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            int before = 0;
            for (int qq = 0; qq < 4; ++qq) before += qq < w ? s_w[r][qq] : 0;
            if (pass[r]) s_q[off + before + __popcll(m[r] & lt)] = base + r * 256 + (int)threadIdx.x;
            for (int qq = 0; qq < 4; ++qq) off += s_w[r][qq];
        }
        qn = off;
        __syncthreads();
        if (qn >= kBinTris) {
            bin_certify_batch(F, tc, tris, B, bin, all, slist, sbox, s_q, kBinTris, x0, x1, y0, y1);
            const int rest = qn - kBinTris;               // < kBinTris
            int mv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int k = r * 256 + (int)threadIdx.x;
                mv[r] = k < rest ? s_q[kBinTris + k] : 0;
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int k = r * 256 + (int)threadIdx.x;
                if (k < rest) s_q[k] = mv[r];
            }
            qn = rest;
            __syncthreads();
        }
    }
    if (qn > 0) bin_certify_batch(F, tc, tris, B, bin, all, slist, sbox, s_q, qn, x0, x1, y0, y1);
}

// Bucket of a key within its bin: 0 without a key, else 1 + its place in the
// bin's key range, keys past the range in the last bucket (the same float
// ops in count and scatter).  Which bucket an entry takes only orders the
// walk: K1 skips a bucket by its smallest key, so any assignment is exact.
__device__ __forceinline__ int depth_bucket(unsigned kbits, const BigBufs &B, int bin)
{
    if (kbits == 0u) return 0;
    const float lo = __uint_as_float(~B.key_lo_inv[bin]), hi = __uint_as_float(B.key_hi[bin]);
    const float k = __uint_as_float(kbits);
    if (!(hi > lo)) return 1;
    const float x = (k - lo) / (hi - lo) * (float)(kDepthBuckets - 1);
    return x < (float)(kDepthBuckets - 2) ? 1 + max((int)x, 0) : kDepthBuckets - 1;
}

// Per bin: bucket sizes and each bucket's smallest key (workgroups stride
// over the bin's chunks).
#ifndef CG_BINC_WAVES
#define CG_BINC_WAVES 4   // A/B: -DCG_BINC_WAVES=n
#endif
__global__ __launch_bounds__(256, CG_BINC_WAVES) void rt_bin_count_kernel(RtFrame F, const RtTri *__restrict__ tc,
                                                           const cg_tri *__restrict__ tris, BigBufs B)
{
    const int bin = blockIdx.y, nc = B.bin_nch[bin];
    if ((int)blockIdx.x >= nc) return;
    const Chunk *tab = B.bin_chunk + (size_t)bin * B.nch;
    const int *pre = B.bin_pre + (size_t)bin * B.nch;
    const size_t base = B.bin_base[bin];
    // an entry without a box for the whole bin (det's sign uncertain there)
    // gets one per half of the bin where the half's own certificate allows,
    // and none at all where it culls the triangle
    float hx0[2], hx1[2], hy0[2], hy1[2];
    bool hv[2];
    for (int h = 0; h < 2; ++h)
        hv[h] = bin_half_bundle(F, bin % B.bins_x, bin / B.bins_x, h, hx0[h], hx1[h], hy0[h], hy1[h]);
    __shared__ int s_cnt[2][kDepthBuckets];
    __shared__ unsigned s_min[2][kDepthBuckets];
    if (threadIdx.x < 2 * kDepthBuckets) {
        (&s_cnt[0][0])[threadIdx.x] = 0;
        (&s_min[0][0])[threadIdx.x] = 0u;
    }
    __syncthreads();
    // chunk by chunk, each entry also copied to its place in the compacted list; the box-less
    // entries (a minority, each two certificates) are queued in LDS and certified 256 at a time
    __shared__ unsigned long long s_qa[512], s_qd[512];   // (source, destination) of queued entries
    __shared__ int s_w[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    int qn = 0;   // queued (workgroup-uniform)
    auto finish = [&](size_t at, size_t d, bool boxless) {
        const unsigned long long ent = B.bin_ent[at];
        unsigned long long pb[2];
        pb[0] = B.bin_pbox[at];
        pb[1] = B.bin_pbox2[at];
        if (boxless) {
            const int i = (int)(unsigned)(ent & 0xffffffffull);
            for (int h = 0; h < 2; ++h) {
                PrimDet ph;
                pb[h] = kProjNone;
                if (hv[h] && !cull_primary(tc[i], hx0[h], hx1[h], hy0[h], hy1[h], F.focal, &ph))
                    pb[h] = proj_box16(tc[i], ph, F.cam, F.focal);
            }
        }
        B.flat_ent[d] = ent;
        B.flat_pbox[d] = pb[0];
        B.flat_pbox2[d] = pb[1];
        const unsigned kb = (unsigned)(ent >> 32);
        const int b = depth_bucket(kb, B, bin);
        for (int h = 0; h < 2; ++h)
            if (hv[h] && proj_meets(pb[h], hx0[h], hx1[h], hy0[h], hy1[h])) {
                atomicAdd(&s_cnt[h][b], 1);
                atomicMax(&s_min[h][b], ~kb);
            }
    };
    for (int c = blockIdx.x; c < nc; c += gridDim.x) {
        const Chunk ch = tab[c];
        const size_t dst = base + pre[c];
        for (int e0 = 0; e0 < ch.n; e0 += 256) {   // workgroup-uniform bounds
            const int e = e0 + (int)threadIdx.x;
            const size_t at = (size_t)ch.off + e;
            const bool in = e < ch.n;
            const bool boxless = in && B.bin_pbox[at] == kProjAll;
            if (in && !boxless) finish(at, dst + e, false);
            const unsigned long long m = __ballot(boxless);
            if (lane == 0) s_w[w] = __popcll(m);
            __syncthreads();
            int before = qn;
            for (int q = 0; q < w; ++q) before += s_w[q];
            if (boxless) {
                s_qa[before + __popcll(m & lt)] = at;
                s_qd[before + __popcll(m & lt)] = dst + e;
            }
            qn += s_w[0] + s_w[1] + s_w[2] + s_w[3];
            __syncthreads();
            if (qn >= 256) {
                finish(s_qa[threadIdx.x], s_qd[threadIdx.x], true);
                const bool mv = (int)threadIdx.x + 256 < qn;
                const unsigned long long ma = mv ? s_qa[threadIdx.x + 256] : 0ull, md = mv ? s_qd[threadIdx.x + 256] : 0ull;
                __syncthreads();
                if (mv) {
                    s_qa[threadIdx.x] = ma;
                    s_qd[threadIdx.x] = md;
                }
                qn -= 256;
                __syncthreads();
            }
        }
    }
    if ((int)threadIdx.x < qn) finish(s_qa[threadIdx.x], s_qd[threadIdx.x], true);
    __syncthreads();
    if (threadIdx.x < 2 * kDepthBuckets && (&s_cnt[0][0])[threadIdx.x]) {   // [h][b] -> sub 2 bin + h
        atomicAdd(&B.bkt_cnt[2 * bin * kDepthBuckets + threadIdx.x], (&s_cnt[0][0])[threadIdx.x]);
        atomicMax(&B.bkt_min_inv[2 * bin * kDepthBuckets + threadIdx.x], (&s_min[0][0])[threadIdx.x]);
    }
}

// Bucket offsets in the sorted pool, over every half-bin and bucket in order
// (one workgroup; a half-wave per half-bin, a lane per bucket); the counts
// become the scatter cursors, the total is the sorted pool's demand.  A
// half-bin reaching past the pool's capacity marks its bin overflowed (K1
// then walks every triangle; the scatter skips it).
constexpr int kMaxSubs = 16384;               // half-bins of one frame (8192 x 4096 pixels)
__global__ __launch_bounds__(1024) void rt_bin_scan_kernel(BigBufs B, int subs)
{
    static_assert(kDepthBuckets == 32, "one half-wave lane per bucket");
    __shared__ int s_tot[kMaxSubs];
    __shared__ int s_wave[16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane & 31, hw = threadIdx.x >> 5;
    // half-bin totals
    for (int sub = hw; sub < subs; sub += 32) {
        int x = B.bkt_cnt[sub * kDepthBuckets + hl];
#pragma unroll
        for (int o = 16; o; o >>= 1) x += __shfl_xor(x, o, 32);
        if (hl == 0) s_tot[sub] = x;
    }
    __syncthreads();
    // exclusive prefix of the totals: thread t owns a run of `per` half-bins
    const int per = (subs + 1023) / 1024;
    const int s0 = min(subs, (int)threadIdx.x * per), s1 = min(subs, s0 + per);
    int run = 0;
    for (int sub = s0; sub < s1; ++sub) run += s_tot[sub];
    int x = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_wave[w] = x;
    __syncthreads();
    int acc = x - run;
    for (int q = 0; q < w; ++q) acc += s_wave[q];
    if (threadIdx.x == 1023) B.pool_n[kPoolSorted] = (unsigned long long)(acc + run);
    __syncthreads();                                 // every thread has read s_tot: overwrite with the bases
    for (int sub = s0; sub < s1; ++sub) {
        const int t = s_tot[sub];
        s_tot[sub] = acc;
        acc += t;
    }
    __syncthreads();
    // per half-bin: bucket offsets = its base + exclusive prefix of its counts
    for (int sub = hw; sub < subs; sub += 32) {
        int *cnt = B.bkt_cnt + sub * kDepthBuckets, *off = B.bkt_off + sub * (kDepthBuckets + 1);
        const int c = cnt[hl];
        int y = c;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
            const int z = __shfl_up(y, o, 32);
            if (hl >= o) y += z;
        }
        const int o0 = s_tot[sub] + y - c;
        off[hl] = o0;
        cnt[hl] = o0;
        if (hl == 31) {
            off[kDepthBuckets] = o0 + c;
            if ((long long)(o0 + c) > B.cap_sorted) B.bin_over[sub >> 1] = 1;
        }
    }
}

// Per bin: each entry into the bucket lists of the half-bins its box meets
// (one global reservation per half, bucket and chunk).
__global__ __launch_bounds__(256) void rt_bin_scatter_kernel(RtFrame F, BigBufs B)
{
    const int bin = blockIdx.y, n = B.bin_over[bin] ? 0 : B.bin_tot[bin];
    const size_t base = B.bin_base[bin];
    float hx0[2], hx1[2], hy0[2], hy1[2];
    bool hv[2];
    for (int h = 0; h < 2; ++h)
        hv[h] = bin_half_bundle(F, bin % B.bins_x, bin / B.bins_x, h, hx0[h], hx1[h], hy0[h], hy1[h]);
    __shared__ int s_cnt[2][kDepthBuckets], s_base[2][kDepthBuckets];
    for (int e0 = (int)blockIdx.x * 1024; e0 < n; e0 += (int)gridDim.x * 1024) {
        if (threadIdx.x < 2 * kDepthBuckets) (&s_cnt[0][0])[threadIdx.x] = 0;
        __syncthreads();
        unsigned long long ent[4], pb[4][2];
        int bk[4], loc[4][2];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = e0 + r * 256 + (int)threadIdx.x;
            bk[r] = -1;
            loc[r][0] = loc[r][1] = -1;
            ent[r] = 0ull;
            pb[r][0] = pb[r][1] = kProjNone;
            if (e < n) {
                const size_t at = base + e;
                ent[r] = B.flat_ent[at];
                pb[r][0] = B.flat_pbox[at];
                pb[r][1] = B.flat_pbox2[at];
                bk[r] = depth_bucket((unsigned)(ent[r] >> 32), B, bin);
                for (int h = 0; h < 2; ++h)
                    if (hv[h] && proj_meets(pb[r][h], hx0[h], hx1[h], hy0[h], hy1[h]))
                        loc[r][h] = atomicAdd(&s_cnt[h][bk[r]], 1);
            }
        }
        __syncthreads();
        if (threadIdx.x < 2 * kDepthBuckets && (&s_cnt[0][0])[threadIdx.x])
            (&s_base[0][0])[threadIdx.x] = atomicAdd(&B.bkt_cnt[2 * bin * kDepthBuckets + threadIdx.x],
                                                      (&s_cnt[0][0])[threadIdx.x]);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 4; ++r)
            for (int h = 0; h < 2; ++h)
                if (loc[r][h] >= 0) {
                    const size_t at = (size_t)s_base[h][bk[r]] + loc[r][h];
                    B.bin_sorted[at] = ent[r];
                    // a box-less entry: its half-bin, for rt_half_mask_kernel
                    B.bin_spbox[at] = pb[r][h] == kProjAll ? ((unsigned long long)(2 * bin + h) << 32) | kNeedTag : pb[r][h];
                }
        __syncthreads();                                    // s_cnt / s_base reused by the next chunk
    }
}

// Tile masks for the bucketed half-bin entries without a box (det's sign
// uncertain over the half: mostly triangles seen nearly edge-on far along
// their plane's horizon, which every wave of the half would otherwise
// certify and cull): the mask of the half's 32 wave tiles (8 x 4, bit c +
// 8 r) whose certificate keeps the triangle (bundle_mask), in place of the
// box; the walk tests its tile's bit.  One flat pass over the bucketed pool
// (the scatter tagged those entries with their half-bin), the tile bundles
// from a table.
__global__ __launch_bounds__(64) void rt_half_tiles_kernel(RtFrame F, BigBufs B)
{
    const int sub = blockIdx.x, bin = sub >> 1, h = sub & 1, t = threadIdx.x;
    if (t >= 32) return;
    const int tx = (bin % B.bins_x) * kBinTilesX + h * (kBinTilesX / 2) + (t & 7);
    const int ty = (bin / B.bins_x) * kBinTilesY + (t >> 3);
    float *q = B.tile_bb + ((size_t)sub * 32 + t) * 4;
    float x0, x1, y0, y1;
    if (!tile_bundle(F, tx, ty, x0, x1, y0, y1)) {
        x0 = 1.0f;
        x1 = 0.0f;
        y0 = y1 = 0.0f;
    }
    *(float4 *)q = make_float4(x0, x1, y0, y1);
}

// The entries needing a mask are a minority scattered through the sorted pool: each
// workgroup queues them in LDS (ballot compaction) and certifies them 256 at a time, one per
// lane, instead of leaving most lanes of each grid-stride step idle beside bundle_mask.
__device__ __forceinline__ void half_mask_one(const RtFrame &F, const RtTri *__restrict__ tc, const BigBufs &B,
                                              long long p)
{
    const unsigned long long pb = B.bin_spbox[p];
    // (entries of an overflowed bin may be another frame's: never walked, skipped here)
    const int sub = (int)(pb >> 32), bin = sub >> 1;
    if (sub < 0 || sub >= 2 * B.bins_x * B.bins_y || B.bin_over[bin]) return;
    float hx0, hx1, hy0, hy1;
    if (!bin_half_bundle(F, bin % B.bins_x, bin / B.bins_x, sub & 1, hx0, hx1, hy0, hy1)) return;
    const int i = (int)(unsigned)(B.bin_sorted[p] & 0xffffffffull);
    if (i < 0 || i >= F.n_tris) return;
    const unsigned long long mk = bundle_mask(tc[i], (const float(*)[4])(B.tile_bb + (size_t)sub * 128), 32, hx0,
                                              hx1, hy0, hy1, F.focal);
    B.bin_spbox[p] = mk ? (mk << 32) | kMaskTag : kProjNone;
}
#ifdef CG_HALF_WAVES   // A/B builds
__global__ __launch_bounds__(256, CG_HALF_WAVES) void rt_half_mask_kernel(
#else
__global__ __launch_bounds__(256) void rt_half_mask_kernel(
#endif
    RtFrame F, const RtTri *__restrict__ tc, BigBufs B)
{
    const long long total = (long long)min((unsigned long long)B.pool_n[kPoolSorted], (unsigned long long)B.cap_sorted);
    __shared__ long long s_q[512];
    __shared__ int s_w[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    int qn = 0;   // queued (workgroup-uniform)
    for (long long b0 = (long long)blockIdx.x * 256; b0 < total; b0 += (long long)gridDim.x * 256) {
        const long long p = b0 + threadIdx.x;
        const bool need = p < total && (unsigned)B.bin_spbox[p] == kNeedTag;
        const unsigned long long m = __ballot(need);
        if (lane == 0) s_w[w] = __popcll(m);
        __syncthreads();
        int before = qn;
        for (int q = 0; q < w; ++q) before += s_w[q];
        if (need) s_q[before + __popcll(m & lt)] = p;
        qn += s_w[0] + s_w[1] + s_w[2] + s_w[3];
        __syncthreads();
        if (qn >= 256) {
            half_mask_one(F, tc, B, s_q[threadIdx.x]);
            const long long mv = (int)threadIdx.x + 256 < qn ? s_q[threadIdx.x + 256] : 0;
            __syncthreads();
            if ((int)threadIdx.x + 256 < qn) s_q[threadIdx.x] = mv;
            qn -= 256;
            __syncthreads();
        }
    }
    if ((int)threadIdx.x < qn) half_mask_one(F, tc, B, s_q[threadIdx.x]);
}

// Ray slots of one wave tile (K1, K4 and the shading kernel read them):
//  * per-pixel mode: the tile's 8x8 pixels, lane = pixel, slot s = its
//    sub-ray s (skeleton.cpp:134-140), stored at s * npix + pixel;
//  * lattice mode (rt_big_mode; rows contiguous, <= 64 lights): with R =
//    identity pixel (u, v)'s sub-ray (i, j) has the exact direction ((u - W/2)
//    + i/2, (v - H/2) + j/2, f) (cg_rt.hip), the half-pixel lattice point
//    (2u + i, 2v + j) its neighbours share.  Its closest hit and its shadow
//    verdicts depend only on the ray, so each point is traced once: the tile
//    owns lattice columns Xi = 2u + i + 1 in [16 tx, 16 tx + 16) and rows Yi
//    = 2 (v - row0) + j + 1 in [16 ty, 16 ty + 16) (the last tile of a row or
//    column also the one beyond), slot s of a lane is owned point s * 64 +
//    lane, stored at Yi * lat_w + Xi: 4 rays per lane instead of 9.
//    Under a yaw (rt_big_mode 2) the rows are still that lattice but each
//    pixel keeps its own three columns Xi = 3u + i + 1 (lat_x): the tile owns
//    [24 tx, 24 tx + 24), up to 7 slots per lane.
struct LatOwn {
    int xi0, nx, yi0, ny;
};
__device__ __forceinline__ LatOwn lat_own(const RtFrame &F, const BigBufs &B, int tx, int ty)
{
    LatOwn o;
    const int rows = min(F.rows_out, F.H - F.row0);    // rows with v < H
    const int cw = B.lat_yaw ? 24 : 16;                  // lattice columns of 8 pixels
    o.xi0 = cw * tx;
    o.yi0 = 16 * ty;
    const int xe = tx == (F.W - 1) / 8 ? B.lat_w : min(cw * tx + cw, B.lat_w);
    const int ye = ty == (rows - 1) / 8 ? B.lat_h : min(16 * ty + 16, B.lat_h);
    o.nx = max(0, xe - o.xi0);
    o.ny = ty > (rows - 1) / 8 ? 0 : max(0, ye - o.yi0);
    return o;
}
// x of lattice column Xi: the half-pixel lattice, or (yawed camera, see
// cg_rt.hip lat_yaw) pixel Xi / 3's sub-ray i = Xi % 3 - 1, fl(dir.x + 0.5 i)
// -- dir.x formed with y = 0, which only changes the sign of a zero dir.x.
// LM (the kernels' mode): 1 is the unrotated lattice, so the yaw form is not
// even compiled there (its uniform pieces otherwise held registers).
template <int LM = 0>
__device__ __forceinline__ float lat_x(const RtFrame &F, const BigBufs &B, int Xi)
{
    if (LM == 1 || !B.lat_yaw) return 0.5f * (float)(Xi - 1 - 2 * (F.W / 2));
    const int u = Xi / 3, i = Xi - 3 * u - 1;
    return mat4_mul(F.R, v4((float)(u - F.W / 2), 0.0f, F.focal, 1.0f)).x + (0.5f * (float)i);   // :126-137
}
__device__ __forceinline__ float lat_y(const RtFrame &F, int Yi)
{
    return 0.5f * (float)(Yi - 1 + 2 * F.row0 - 2 * (F.H / 2));
}

// K1: closest hits of every ray slot of the tile.
#ifdef CG_WG_TIMING
// Diagnostic build only: per-wave wall-clock stamps (100 MHz) of the walk (kind 3) and the
// shadow hints (kind 4), read by scripts/wg_timing_c5.py.  Record as cg_rt.hip's wgt_record,
// one per wave.
__device__ unsigned long long *g_wgtb;
__device__ unsigned int g_wgtb_cap;
__device__ __forceinline__ void wgtb_record(unsigned long long kind, unsigned long long t0)
{
    const unsigned long long t1 = wall_clock64();
    if ((threadIdx.x & 63) || !g_wgtb) return;
    const unsigned long long s = (kind == 3 ? 0ull : g_wgtb_cap / 2) +
                                 ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (s >= (kind == 3 ? g_wgtb_cap / 2 : g_wgtb_cap)) return;
    unsigned long long *r = g_wgtb + 6ull * s;
    r[0] = kind << 56 | (unsigned long long)blockIdx.y << 20 | ((unsigned long long)blockIdx.x * 4 + (threadIdx.x >> 6));
    r[1] = t0;
    r[2] = t1;
    r[3] = t1;
    r[4] = t1;
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20), hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    r[5] = (unsigned long long)xcc << 56 | (unsigned long long)hw << 24 | blockIdx.x;
}
#define WGTB_T0 const unsigned long long wgtb_t0 = wall_clock64()
#define WGTB_END(k) wgtb_record(k, wgtb_t0)
#else
#define WGTB_T0
#define WGTB_END(k)
#endif

// The walk's workgroup order: a workgroup (4 wave tiles of one half-bin) is
// keyed by its half-bin's sorted list length, the walk's work per ray slot;
// one workgroup counting-sorts the gx * gy keys, longest first (64 classes
// linear in the longest list; ties in any order -- the order only schedules
// the walk, every workgroup's pixels are its own).
__global__ __launch_bounds__(1024) void rt_walk_order_kernel(BigBufs B, int gx, int gy)
{
    __shared__ int s_cnt[64], s_max;
    const int n = gx * gy, t = threadIdx.x;
    auto key = [&](int w) {
        const int tx = (w % gx) * (kRtTileW / 8), ty = w / gx;
        const int bin = (tx / kBinTilesX) + (ty / kBinTilesY) * B.bins_x;
        const int sub = 2 * bin + ((tx % kBinTilesX) < kBinTilesX / 2 ? 0 : 1);
        const int *o = B.bkt_off + sub * (kDepthBuckets + 1);
        return o[kDepthBuckets] - o[0];
    };
    if (t < 64) s_cnt[t] = 0;
    if (t == 0) s_max = 0;
    __syncthreads();
    int mx = 0;
    for (int w = t; w < n; w += 1024) mx = max(mx, key(w));
    atomicMax(&s_max, mx);
    __syncthreads();
    const long long top = (long long)s_max + 1;
    auto cls = [&](int w) { return 63 - (int)((long long)key(w) * 64 / top); };   // 0 = longest
    for (int w = t; w < n; w += 1024) atomicAdd(&s_cnt[cls(w)], 1);
    __syncthreads();
    if (t == 0) {
        int a = 0;
        for (int c = 0; c < 64; ++c) {
            const int x = s_cnt[c];
            s_cnt[c] = a;
            a += x;
        }
    }
    __syncthreads();
    for (int w = t; w < n; w += 1024) B.walk_order[atomicAdd(&s_cnt[cls(w)], 1)] = w;
}

// An opaque copy of v: values derived from it are recomputed where they are
// used instead of being hoisted (and kept live) across a loop.
__device__ __forceinline__ int launder(int v)
{
    asm volatile("" : "+v"(v));
    return v;
}

#ifndef CG_WALK_PARK
#define CG_WALK_PARK 1   // the walk parks its ray slots in LDS around each certificate batch (A/B: 0)
#endif
// Waves per SIMD of the walk: the lattice mode (C5) fits 4 in 123 VGPRs with
// no scratch once its slots are parked and its wave index is uniform; the
// yawed (7 slots) and per-pixel (9 slots) modes need 3 for no scratch.  More
// waves with some scratch are faster now (below).  CG_WALK_WAVES overrides
// every mode (A/B builds).
#ifdef CG_WALK_WAVES
template <int LM> constexpr int walk_waves() { return CG_WALK_WAVES; }
#else
// Round 6, with the hints' grid walks queued: the lattice mode at 5 (96 VGPRs, 68 B of scratch;
// C5 210.9 -> 216.7 fps, 6 waves 216.3) and the yawed mode at 4 (C5-yaw 145.0 -> 151.2, 5 waves
// 149.6, 6 124.9); the per-pixel mode (no bench configuration) stays at 3
template <int LM> constexpr int walk_waves() { return LM == 1 ? 5 : LM == 2 ? 4 : 3; }
#endif

template <int LM>   // 0: per-pixel mode, 1: lattice, 2: lattice with per-pixel columns
__global__ __launch_bounds__(kRtThreads, walk_waves<LM>()) void rt_big_primary_kernel(RtFrame F, const RtTri *__restrict__ tc,
                                                                    const RtShade *__restrict__ shade,
                                                                    const RtSphere *__restrict__ sph, BigBufs B)
{
    WGTB_T0;
    constexpr bool kLat = LM > 0;
    constexpr int NS = LM == 0 ? 9 : (LM == 1 ? 5 : 7);   // ray slots per lane (lattice: owned points / 64)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;   // wave: uniform (SGPR)
    int bx = blockIdx.x, by = blockIdx.y;
    if (B.walk_order) {   // heavy-first (rt_walk_order_kernel): the long lists start early, not in the tail
        const int w = __builtin_amdgcn_readfirstlane(B.walk_order[blockIdx.y * gridDim.x + blockIdx.x]);
        bx = w % (int)gridDim.x;
        by = w / (int)gridDim.x;
    }
    const int tx = bx * (kRtTileW / 8) + wave, ty = by;
    if (tx >= B.tiles_x) return;
    const float m = 0.5f;
    // slot directions: per-pixel mode dir +- m (i, j); lattice mode rx / ry
    float rx[kLat ? NS : 1], ry[kLat ? NS : 1];
    bool on[NS];
    vec4 dir = v4(0.0f, 0.0f, 0.0f, 0.0f);
    int u = 0, L = 0, nsu = NS;
    float x0, x1, y0, y1;
    // The slots' geometry from the lane index (formed again after each parked
    // certificate batch, from a laundered lane, so it is not live across the
    // certificate's FP64 code)
    auto geom = [&](int ln) {
        if constexpr (kLat) {
            const LatOwn o = lat_own(F, B, tx, ty);
            const int n = o.nx * o.ny;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const int k = s * 64 + ln;
                on[s] = k < n;
                const int kk = on[s] ? k : 0;
                rx[s] = lat_x<LM>(F, B, o.xi0 + kk % max(o.nx, 1));
                ry[s] = lat_y(F, o.yi0 + kk / max(o.nx, 1));
            }
        } else {
            u = tx * 8 + (ln & 7);
            L = ty * 8 + (ln >> 3);
            const bool inside = u < F.W && L < F.rows_out;
            const int v = inside ? shard_row(F, L) : 0;
            const bool active = inside && v < F.H;
            dir = v4((float)(u - F.W / 2), (float)(v - F.H / 2), F.focal, 1.0f);        // :126
            dir = mat4_mul(F.R, dir);                                                    // :128
#pragma unroll
            for (int s = 0; s < NS; ++s) on[s] = active;
        }
    };
    geom(lane);
    if constexpr (kLat) {
        const LatOwn o = lat_own(F, B, tx, ty);
        nsu = __builtin_amdgcn_readfirstlane((o.nx * o.ny + 63) >> 6);
        float a0 = FLT_MAX, a1 = -FLT_MAX, b0 = FLT_MAX, b1 = -FLT_MAX;
#pragma unroll
        for (int s = 0; s < NS; ++s)
            if (on[s]) {
                a0 = fminf(a0, rx[s]); a1 = fmaxf(a1, rx[s]);
                b0 = fminf(b0, ry[s]); b1 = fmaxf(b1, ry[s]);
            }
        x0 = wave_min(a0); x1 = wave_max(a1); y0 = wave_min(b0); y1 = wave_max(b1);
    } else {
        const bool active = on[0];
        x0 = wave_min(active ? dir.x : FLT_MAX); x1 = wave_max(active ? dir.x : -FLT_MAX);
        y0 = wave_min(active ? dir.y : FLT_MAX); y1 = wave_max(active ? dir.y : -FLT_MAX);
        x0 = x0 - 0.5f; x1 = x1 + 0.5f; y0 = y0 - 0.5f; y1 = y1 + 0.5f;
    }
    // the wave's bundle is uniform: SGPRs, not four VGPRs live through the walk
    x0 = uniform_f32(x0); x1 = uniform_f32(x1); y0 = uniform_f32(y0); y1 = uniform_f32(y1);
    auto slot_nd = [&](int s) -> vec3 {                                              // :137
        if constexpr (kLat) return v3(rx[s], ry[s], F.focal);
        else return v3(dir.x + (m * (float)(s / 3 - 1)), dir.y + (m * (float)(s % 3 - 1)), F.focal);
    };
    const bool any = x0 <= x1;
    const int bin = (tx / kBinTilesX) + (ty / kBinTilesY) * B.bins_x;
    const int sub = 2 * bin + ((tx % kBinTilesX) < kBinTilesX / 2 ? 0 : 1);          // the wave's half-bin
    const int tbit = 32 + (tx % (kBinTilesX / 2)) + (kBinTilesX / 2) * (ty % kBinTilesY);   // its tile-mask bit
    const unsigned long long *list = B.bin_sorted;   // global offsets (rt_bin_scan_kernel)
    const unsigned long long *pboxes = B.bin_spbox;
    const int *boff = B.bkt_off + sub * (kDepthBuckets + 1);
    const unsigned *bmin_inv = B.bkt_min_inv + sub * kDepthBuckets;
    float best[NS], bt[NS], len[NS];
    int bi[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        len[s] = length(slot_nd(s));                                                 // :307
        best[s] = FLT_MAX;
        bt[s] = 0.0f;
        bi[s] = INT_MIN;
    }
    // buckets nearest first; tb = the largest best distance of any slot's ray
    // (FLT_MAX while one has no hit): a candidate whose key exceeds it cannot
    // win or tie for any of them
    float tb = FLT_MAX;
    // Entries passing the box and key tests are queued in LDS and certified
    // 64 at a time (full lanes for the FP64 certificate), the queue flushed
    // at every bucket end so that tb tightens before the next bucket.
    __shared__ int s_q[kRtThreads / 64][128];
    int *q_w = s_q[wave];
    int qn = 0;                                                    // wave-uniform
#ifdef CG_WALK_STATS
    int st_chunks = 0, st_pass = 0, st_batches = 0, st_walked = 0, st_buckets = 0, st_all = 0, st_wide = 0;
#endif
#if CG_WALK_PARK
    // the slots' running minima parked in LDS while the certificate's FP64
    // code runs (its registers would otherwise spill them to scratch)
    __shared__ float s_park[kRtThreads / 64][3 * NS][64];
#endif
    auto certify_walk = [&](int cnt) {                             // the first cnt (<= 64) queued entries
        const int cand = lane < cnt ? q_w[lane] : -1;
#if CG_WALK_PARK
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            s_park[wave][s][lane] = best[s];
            s_park[wave][NS + s][lane] = bt[s];
            s_park[wave][2 * NS + s][lane] = __int_as_float(bi[s]);
        }
#endif
        const bool keep = cand >= 0 && !cull_primary(tc[cand], x0, x1, y0, y1, F.focal);
        unsigned long long mask = __ballot(keep);
#if CG_WALK_PARK
        geom(launder(lane));
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            best[s] = s_park[wave][s][lane];
            bt[s] = s_park[wave][NS + s][lane];
            bi[s] = __float_as_int(s_park[wave][2 * NS + s][lane]);
            len[s] = length(slot_nd(s));                                             // :307
        }
#endif
#ifdef CG_WALK_STATS
        ++st_batches;
        st_walked += __popcll(mask);
#endif
        while (mask) {
            const int b = __builtin_ctzll(mask);
            mask &= mask - 1ull;
            const int k = __builtin_amdgcn_readlane(cand, b);
            // scalar loads; broadcasting the certificate's per-lane copy with
            // 16 readlanes instead measured slower (C5 primary 3.05 -> 3.11 ms)
            const RtTri T = tc[k];
#pragma unroll
            for (int s = 0; s < NS; ++s)
                if (s < nsu && on[s]) tri_closest(T, k, -slot_nd(s), len[s], best[s], bt[s], bi[s]);
        }
        float lm = -FLT_MAX;
#pragma unroll
        for (int s = 0; s < NS; ++s)
            if (on[s]) lm = fmaxf(lm, best[s]);
        tb = uniform_f32(wave_max(lm));
    };
    if (B.bin_over[bin]) {   // overflowed bin list: every triangle through the wave's certificate
        for (int c0 = 0; any && c0 < F.n_tris; c0 += 64) {
            q_w[lane] = c0 + lane;
            __builtin_amdgcn_wave_barrier();
            certify_walk(min(64, F.n_tris - c0));
            __builtin_amdgcn_wave_barrier();
        }
    }
    for (int q = 0; any && !B.bin_over[bin] && q < kDepthBuckets; ++q) {
        const int b0 = boff[q], b1 = boff[q + 1];
        if (b0 == b1 || __uint_as_float(~bmin_inv[q]) > tb) continue;
#ifdef CG_WALK_STATS
        ++st_buckets;
#endif
        // the next chunk's entries are loaded while this one is scanned (the
        // lane's addresses formed per bucket, not hoisted and spilled)
        const int ln = launder(lane);
        unsigned long long ent_n = b0 + ln < b1 ? list[b0 + ln] : 0ull;
        unsigned long long pb_n = b0 + ln < b1 ? pboxes[b0 + ln] : 0ull;
        for (int c0 = b0; c0 < b1; c0 += 64) {
            const bool in = c0 + ln < b1;
            const unsigned long long ent = ent_n, pb = pb_n;
            const int cn = c0 + 64 + ln;
            ent_n = cn < b1 ? list[cn] : 0ull;
            pb_n = cn < b1 ? pboxes[cn] : 0ull;
            // projected box first (no gather), then the key
            const bool pass = in && (is_bin_mask(pb) ? ((pb >> tbit) & 1ull) != 0ull : proj_meets(pb, x0, x1, y0, y1)) &&
                              !(__uint_as_float((unsigned)(ent >> 32)) > tb);
            const unsigned long long pm = __ballot(pass);
            if (pass) q_w[qn + __popcll(pm & ((1ull << lane) - 1ull))] = (int)(unsigned)(ent & 0xffffffffull);
            qn += __popcll(pm);
#ifdef CG_WALK_STATS
            ++st_chunks;
            st_pass += __popcll(pm);
            st_all += __popcll(__ballot(in && is_bin_mask(pb)));
            st_wide += __popcll(__ballot(in && pb != kProjAll &&
                                         (short)((pb >> 16) & 0xffff) - (short)(pb & 0xffff) > 40));
#endif
            __builtin_amdgcn_wave_barrier();
            if (qn >= 64) {
                certify_walk(64);
                const int rest = qn - 64;
                const int moved = lane < rest ? q_w[64 + lane] : 0;
                __builtin_amdgcn_wave_barrier();
                if (lane < rest) q_w[lane] = moved;
                qn = rest;
                __builtin_amdgcn_wave_barrier();
            }
        }
        if (qn > 0) {                                              // bucket end: flush
            certify_walk(qn);
            qn = 0;
            __builtin_amdgcn_wave_barrier();
        }
    }
#ifdef CG_WALK_STATS
    if (lane == 0 && tx % 30 == 0 && ty % 16 == 0)
        printf("WALK tx %d ty %d sub %d list %d buckets %d chunks %d pass %d batches %d walked %d tb %g all %d wide %d\n",
               tx, ty, sub, boff[kDepthBuckets] - boff[0], st_buckets, st_chunks, st_pass, st_batches, st_walked, tb,
               st_all, st_wide);
#endif
    LaneShadowBox sb;
    sb.init();
    const vec3 lmin = v3(F.lmin[0], F.lmin[1], F.lmin[2]), lmax = v3(F.lmax[0], F.lmax[1], F.lmax[2]);
    const vec3 s3 = v3(F.cam[0], F.cam[1], F.cam[2]);
    const size_t npix = (size_t)F.rows_out * F.W, pix = (size_t)L * F.W + u;
    LatOwn o{};
    if constexpr (kLat) o = lat_own(F, B, tx, ty);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        if (!(s < nsu && on[s])) continue;
        const vec3 nd = slot_nd(s);
        for (int q = 0; q < F.n_sph; ++q) {                                           // :341-355
            float t;
            if (sphere_intersect(sph[q], s3, nd, t) && t < best[s]) {
                best[s] = t;
                bt[s] = t;
                bi[s] = -1 - q;
            }
        }
        const int hit = best[s] < FLT_MAX ? bi[s] : INT_MIN;                         // :357
        size_t id;
        if constexpr (kLat) {
            const int k = s * 64 + launder(lane);   // not the start's k / nx, kept live (spilled) till here
            id = (size_t)(o.yi0 + k / o.nx) * B.lat_w + o.xi0 + k % o.nx;
        } else {
            id = s * npix + pix;
        }
        B.hit_bi[id] = hit;
        B.hit_t[id] = bt[s];
        if (!kLat && hit != INT_MIN && F.n_lights > 0) {
            const float t = bt[s];
            vec3 pos = v3(F.cam[0] + t * nd.x, F.cam[1] + t * nd.y, F.cam[2] + t * nd.z);
            shadow_box_add(sb, lmin, lmax, pos, hit_normal(shade, sph, hit, pos));
        }
    }
    if constexpr (!kLat) {   // the many-light path's boxes (per-pixel mode only)
        ShadowBox W;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            W.lo[q] = wave_min(sb.lo[q]);
            W.hi[q] = wave_max(sb.hi[q]);
        }
        W.pn = wave_max(sb.pn);
        if (lane == 0) B.wave_box[(size_t)ty * B.tiles_x + tx] = W;
    }
    WGTB_END(3);
}

// K2: union of the wave boxes of each bin (one wave tile per lane).
__global__ __launch_bounds__(64) void rt_bin_boxes_kernel(BigBufs B)
{
    const int bin = blockIdx.x, lane = threadIdx.x;
    const int tx = (bin % B.bins_x) * kBinTilesX + (lane % kBinTilesX);
    const int ty = (bin / B.bins_x) * kBinTilesY + (lane / kBinTilesX);
    ShadowBox w;
    w.lo[0] = w.lo[1] = w.lo[2] = FLT_MAX;
    w.hi[0] = w.hi[1] = w.hi[2] = -FLT_MAX;
    w.pn = 0.0f;
    if (tx < B.tiles_x && ty < B.tiles_y) w = B.wave_box[(size_t)ty * B.tiles_x + tx];
    ShadowBox r;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        r.lo[q] = wave_min(w.lo[q]);
        r.hi[q] = wave_max(w.hi[q]);
    }
    r.pn = wave_max(w.pn);
    if (lane == 0) B.bin_box[bin] = r;
}

// K3: shadow-ray certificate of the light set per (bin, triangle).
__global__ __launch_bounds__(256) void rt_bin_shadow_kernel(RtFrame F, const RtTri *__restrict__ tc, BigBufs B)
{
    const int bin = blockIdx.y;
    const ShadowBox box = B.bin_box[bin];
    const bool ok = box.lo[0] <= box.hi[0];                        // hits in this bin
    const vec3 lc = v3(F.lc[0], F.lc[1], F.lc[2]);
    const int base = blockIdx.x * kBinTris;
    bool kept[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = base + r * 256 + (int)threadIdx.x;
        kept[r] = ok && i < F.n_tris && !cull_shadow(tc[i], lc, F.lrho, box);
    }
    pooled_append(kept, base, B.sbin_pool, B.pool_n + kPoolSbin, B.cap_sbin,
                  B.sbin_chunk + (size_t)bin * B.nch + blockIdx.x, B.sbin_over + bin);
}

// Shadow ray of DirectLight (skeleton.cpp:370-394) for hit `pos` and light l.
struct ShadowRay {
    vec3 origin, nd, r;
    float len, rmag;
};
__device__ __forceinline__ ShadowRay shadow_ray(const RtLight &Lt, vec3 pos, vec3 normal)
{
    ShadowRay q;
    q.r = v3(Lt.x, Lt.y, Lt.z) - pos;                                    // :370
    double r0 = (double)q.r.x * (double)q.r.x, r1 = (double)q.r.y * (double)q.r.y,
           r2 = (double)q.r.z * (double)q.r.z;
    q.rmag = (float)sqrt((r0 + r1) + r2);                                // :371
    q.origin = pos + normal * 0.00001f;                                 // :394
    q.nd = -q.r;
    q.len = length(q.r);
    return q;
}

// DirectLight's value once the shadow verdict on the triangles is known
// (spheres are tested here, :341-355 then :395).
__device__ __forceinline__ vec3 big_direct_light(const RtFrame &F, const RtSphere *__restrict__ sph,
                                                 const RtLight &Lt, const ShadowRay &q, vec3 normal,
                                                 vec3 objColor, bool tri_shadow)
{
    cg_work(W_DL);
    bool shadow = tri_shadow;
    for (int k = 0; k < F.n_sph && !shadow; ++k) {
        float t;
        cg_work(W_SPH_SH);
        if (sphere_intersect(sph[k], q.origin, q.r, t) && t < q.rmag) shadow = true;
    }
    if (shadow) return v3(0.0f, 0.0f, 0.0f);                             // :394-398
    vec3 ndn = normalize(q.r);                                           // :400
    float a = dot(ndn, normal);                                          // :403
    const float b = (float)(4 * M_PI);                                   // :404
    float area = (float)((double)b * ((double)q.rmag * (double)q.rmag)); // :406
    if (a <= 0) a = 0.f;                                                 // :409
    vec3 lc = v3(Lt.r, Lt.g, Lt.b);
    return ((objColor * lc) * a) / area;                                 // :412
}

// any-hit of one shadow ray over a bin's certified shadow list (uniform per
// wave; every triangle when the list overflowed).
__device__ __forceinline__ bool any_hit_bin(const RtTri *__restrict__ tc, const BigBufs &B, int n_tris, int bin,
                                            const ShadowRay &q)
{
    if (B.sbin_over[bin]) {
        for (int k = 0; k < n_tris; ++k)
            if (tri_shadows(tc[k], q.origin, q.nd, q.len, q.rmag)) return true;
        return false;
    }
    for (int c = 0; c < B.nch; ++c) {
        const Chunk ch = B.sbin_chunk[(size_t)bin * B.nch + c];
        for (int e = 0; e < ch.n; ++e) {
            const int k = __builtin_amdgcn_readfirstlane(B.sbin_pool[ch.off + e]);
            if (tri_shadows(tc[k], q.origin, q.nd, q.len, q.rmag)) return true;
        }
    }
    return false;
}

// Blocker search along the shadow segment S + t (L - P), t in [0, 1], through
// the scene grid (3D DDA), testing each cell's triangles with the exact
// reference test.  Heuristic only: a triangle it returns really blocks the
// ray (the float test accepted it); when it finds none the caller runs the
// exhaustive certified search.
__device__ int grid_blocker(const RtGrid &G, const RtTri *__restrict__ tc, const ShadowRay &q, int *ntest = nullptr)
{
    if (!G.start) return -1;
    const float o[3] = {q.origin.x, q.origin.y, q.origin.z}, d[3] = {q.r.x, q.r.y, q.r.z};
    float t0 = 0.0f, t1 = 1.0f;
    for (int a = 0; a < 3; ++a) {
        const float lo = G.lo[a], hi = G.lo[a] + (float)G.res[a] * G.h;
        if (fabsf(d[a]) < 1e-30f) {
            if (o[a] < lo || o[a] > hi) return -1;
            continue;
        }
        float ta = (lo - o[a]) / d[a], tb = (hi - o[a]) / d[a];
        if (ta > tb) { float x = ta; ta = tb; tb = x; }
        t0 = fmaxf(t0, ta);
        t1 = fminf(t1, tb);
    }
    if (!(t0 <= t1)) return -1;
    int c[3], step[3];
    float tmax[3], tdel[3];
    for (int a = 0; a < 3; ++a) {
        const float p = o[a] + d[a] * t0;
        c[a] = min(max((int)floorf((p - G.lo[a]) * G.inv_h), 0), G.res[a] - 1);
        if (fabsf(d[a]) < 1e-30f) {
            step[a] = 0;
            tmax[a] = FLT_MAX;
            tdel[a] = FLT_MAX;
        } else {
            step[a] = d[a] > 0.0f ? 1 : -1;
            const float bound = G.lo[a] + (float)(c[a] + (step[a] > 0 ? 1 : 0)) * G.h;
            tmax[a] = (bound - o[a]) / d[a];
            tdel[a] = G.h / fabsf(d[a]);
        }
    }
    // the walk with one named variable per axis: indexing the arrays by the
    // runtime axis kept them in scratch memory (88 B per lane)
    int cx = c[0], cy = c[1], cz = c[2];
    float mx = tmax[0], my = tmax[1], mz = tmax[2];
    const float dx = tdel[0], dy = tdel[1], dz = tdel[2];
    const int sx = step[0], sy = step[1], sz = step[2];
    const int max_steps = G.res[0] + G.res[1] + G.res[2] + 3;
    for (int it = 0; it < max_steps; ++it) {
        const int cell = (cz * G.res[1] + cy) * G.res[0] + cx;
        for (int i = G.start[cell], e = G.start[cell + 1]; i < e; ++i) {
            const int k = G.tris[i];
            if (ntest) ++*ntest;
            if (tri_shadows(tc[k], q.origin, q.nd, q.len, q.rmag)) return k;
        }
        // axis a = tmax[0] < tmax[1] ? (tmax[0] < tmax[2] ? 0 : 2) : (tmax[1] < tmax[2] ? 1 : 2)
        const int a = mx < my ? (mx < mz ? 0 : 2) : (my < mz ? 1 : 2);
        const float ma = a == 0 ? mx : a == 1 ? my : mz;
        if (ma > t1) break;
        if (a == 0) {
            cx += sx;
            if (cx < 0 || cx >= G.res[0]) break;
            mx += dx;
        } else if (a == 1) {
            cy += sy;
            if (cy < 0 || cy >= G.res[1]) break;
            my += dy;
        } else {
            cz += sz;
            if (cz < 0 || cz >= G.res[2]) break;
            mz += dz;
        }
    }
    return -1;
}

// Shadow verdicts for 9 * n_lights <= 64 (one bit per (sub-ray s, light l)
// and pixel; lattice mode: n_lights <= 64, one bit per light and point), in
// two parallel steps:
//  K4 rt_shadow_hints   each shadow ray tries likely blockers: the triangle it
//                       starts on (the 1e-5 normal offset puts the origin
//                       behind it when the normal faces away from the light),
//                       the lane's previous blocker, then the scene grid.  Any
//                       triangle the exact test accepts blocks the ray -- an
//                       any-hit verdict does not depend on the order.  Rays
//                       still unresolved are queued;
//  K5 rt_pending_lit    the certified lit search for the queued rays (below).
__device__ __forceinline__ void hit_geometry(const RtFrame &F, const BigBufs &B, const RtShade *__restrict__ shade,
                                             const RtSphere *__restrict__ sph, vec3 nd, size_t id, int &bi,
                                             vec3 &pos, vec3 &normal)
{
    bi = B.hit_bi[id];
    if (bi == INT_MIN) return;
    const float t = B.hit_t[id];
    pos = v3(F.cam[0] + t * nd.x, F.cam[1] + t * nd.y, F.cam[2] + t * nd.z);         // :326/:345
    normal = hit_normal(shade, sph, bi, pos);
}

__device__ __forceinline__ vec4 pixel_dir(const RtFrame &F, int u, int v)
{
    return mat4_mul(F.R, v4((float)(u - F.W / 2), (float)(v - F.H / 2), F.focal, 1.0f));   // :126-128
}

// K4 over the tile's ray slots (see K1): per-pixel mode keeps pixel bits s *
// n_lights + l, lattice mode point bits l.  Every lane walks the same (slot,
// light) sequence, so the wave's lanes meet at each step of the neighbour
// exchange.
#ifndef CG_HINT_WAVES
// 6 waves/SIMD: 80 VGPRs, 72-80 B of scratch.  Round 5 measured 4 (no scratch), 5 and 6 the same
// speed; with the grid walks queued per wave (below) 6 is fastest: C5 204.5 / 208.7 / 211.7 fps and
// C5-yaw 140.8 / 143.4 / 146 at 4 / 5 / 6, 7 and 8 slower (profiles/r06_ab_session2.json)
#define CG_HINT_WAVES 6
#endif
// The grid walks of a wave's unresolved shadow rays are deferred to the end of
// the wave (a per-wave LDS queue, kHintQ rays) and then walked 64 at a time, one
// per lane: inline, only the ~quarter of the lanes the cheap tests left
// unresolved walk while the others wait (C5: 26 % of the rays, 18.5 triangle
// tests each).  A full queue walks inline, as before.  CG_HINT_QUEUE=0: inline.
#ifndef CG_HINT_QUEUE
#define CG_HINT_QUEUE 1
#endif
constexpr int kHintQ = 128;
#ifndef CG_HINT_REPS
#define CG_HINT_REPS 16   // blockers other lanes found, tried per unresolved ray before the grid
#endif
struct HintQ {
    float4 a[kHintQ], b[kHintQ];   // origin.xyz, len | r.xyz, rmag
    int2 e[kHintQ];                // the verdict's word (pixel or lattice point), bit
};
template <int LM>
__global__ __launch_bounds__(kRtThreads, CG_HINT_WAVES) void rt_shadow_hints_kernel(RtFrame F, const RtTri *__restrict__ tc,
                                                                     const RtShade *__restrict__ shade,
                                                                     const RtSphere *__restrict__ sph, BigBufs B)
{
    WGTB_T0;
    constexpr bool kLat = LM > 0;
    constexpr int NS = LM == 0 ? 9 : (LM == 1 ? 5 : 7);   // ray slots per lane (lattice: owned points / 64)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;   // wave: uniform (SGPR)
    const int tx = blockIdx.x * (kRtTileW / 8) + wave, ty = blockIdx.y;
    if (tx >= B.tiles_x) return;   // the whole wave (the queue is per wave: no barrier)
#if CG_HINT_QUEUE
    __shared__ HintQ s_hq[kRtThreads / 64];
    HintQ &hq = s_hq[wave];
    int qn = 0;                     // wave-uniform: entries queued
#endif
    const float m = 0.5f;
    int u = 0, L = 0, nsu = NS, n = 0;
    bool active = false;
    vec4 dir = v4(0.0f, 0.0f, 0.0f, 0.0f);
    LatOwn o{};
    if constexpr (kLat) {
        o = lat_own(F, B, tx, ty);
        n = o.nx * o.ny;
        nsu = __builtin_amdgcn_readfirstlane((n + 63) >> 6);
    } else {
        u = tx * 8 + (lane & 7);
        L = ty * 8 + (lane >> 3);
        const bool inside = u < F.W && L < F.rows_out;
        const int v = inside ? shard_row(F, L) : 0;
        active = inside && v < F.H;
        dir = pixel_dir(F, u, v);
    }
    const size_t npix = (size_t)F.rows_out * F.W, pix = (size_t)L * F.W + u;
    unsigned long long shadowed = 0ull, pending = 0ull;
    int last = -1, gtests = 0;
#ifdef CG_WALK_STATS
    int st_rays = 0, st_cheap = 0, st_grid_rays = 0, st_lit = 0;
#endif
    for (int s = 0; s < nsu; ++s) {
        bool on;
        vec3 nd;
        size_t id;
        if constexpr (kLat) {
            // per slot from a laundered lane: hoisted, these per-lane values
            // lived through the slot loop and spilled to scratch at 6 waves/SIMD
            const int k = s * 64 + launder(lane);
            on = k < n;
            const int kk = on ? k : 0, Xi = o.xi0 + kk % max(o.nx, 1), Yi = o.yi0 + kk / max(o.nx, 1);
            nd = v3(lat_x<LM>(F, B, Xi), lat_y(F, Yi), F.focal);
            id = (size_t)Yi * B.lat_w + Xi;
            shadowed = pending = 0ull;
        } else {
            on = active;
            nd = v3(dir.x + (m * (float)(s / 3 - 1)), dir.y + (m * (float)(s % 3 - 1)), F.focal);   // :137
            id = s * npix + pix;
        }
        int bi = INT_MIN;
        vec3 pos = v3(0.0f, 0.0f, 0.0f), normal = pos;
        if (on) hit_geometry(F, B, shade, sph, nd, id, bi, pos, normal);
        const bool ray = bi != INT_MIN;
        for (int l = 0; l < F.n_lights; ++l) {
            const RtLight Lt = F.lights[l];
            const ShadowRay q = shadow_ray(Lt, pos, normal);
            int k = -1;
            if (ray) {
                if (bi >= 0 && tri_shadows(tc[bi], q.origin, q.nd, q.len, q.rmag)) k = bi;
                else if (last >= 0 && tri_shadows(tc[last], q.origin, q.nd, q.len, q.rmag)) k = last;
            }
            // unresolved rays try up to sixteen distinct blockers other rays of the
            // wave found.  They are only hints: each is re-tested with the exact
            // tri_shadows, so the verdict does not depend on which lanes
            // contributed them
            unsigned long long have = __ballot(k >= 0);
            for (int rep = 0; rep < CG_HINT_REPS && have != 0ull && __ballot(ray && k < 0) != 0ull; ++rep) {
                const int kn = __shfl(k, __builtin_ctzll(have));
                have &= ~__ballot(k == kn);
                if (ray && k < 0 && tri_shadows(tc[kn], q.origin, q.nd, q.len, q.rmag)) k = kn;
            }
            const int bitno = kLat ? l : s * F.n_lights + l;
#if CG_HINT_QUEUE
            // every lane (qn stays wave-uniform): queue the unresolved rays while the
            // wave's queue has room for all of this step's
            bool queued = false;
            {
                const bool need = ray && k < 0;
                const unsigned long long want = __ballot(need);
                const int nw = __popcll(want);
                const bool fits = qn + nw <= kHintQ;
                if (need && fits) {
                    const int at = qn + __popcll(want & ((1ull << lane) - 1ull));
                    hq.a[at] = make_float4(q.origin.x, q.origin.y, q.origin.z, q.len);
                    hq.b[at] = make_float4(q.r.x, q.r.y, q.r.z, q.rmag);
                    hq.e[at] = make_int2((int)(kLat ? id : pix), bitno);
                }
                if (fits) qn += nw;
                queued = need && fits;
            }
#endif
            if (!ray) continue;
#ifdef CG_WALK_STATS
            ++st_rays;
            if (k >= 0) ++st_cheap;
            const int g0 = gtests;
#endif
#if CG_HINT_QUEUE
            if (queued) continue;   // its verdict comes from the deferred walk
#endif
            if (k < 0) k = grid_blocker(B.grid, tc, q, &gtests);
#ifdef CG_WALK_STATS
            if (gtests > g0) ++st_grid_rays;
            if (k < 0) ++st_lit;
#endif
            const unsigned long long bit = 1ull << bitno;
            if (k >= 0) {
                shadowed |= bit;
                last = k;
            } else {
                const int p = atomicAdd(B.pend_n, 1);
                if (p < B.max_pend)
                    B.pend_ray[p] = PendRay{q.origin.x, q.origin.y, q.origin.z, q.nd.x, q.nd.y, q.nd.z,
                                            q.len, q.rmag, (int)(kLat ? id : pix), bitno};
                else
                    pending |= bit;       // past the queue: rt_big_shade_kernel searches it
            }
        }
        if (kLat && on) {
            B.sh_bits[id] = shadowed;
            B.pend_bits[id] = pending;
        }
    }
#ifdef CG_WALK_STATS
    {
        int a = st_rays, b = st_cheap, c = st_grid_rays, d = st_lit, e = gtests;
        for (int o = 32; o; o >>= 1) {
            a += __shfl_xor(a, o); b += __shfl_xor(b, o); c += __shfl_xor(c, o); d += __shfl_xor(d, o);
            e += __shfl_xor(e, o);
        }
        if (lane == 0 && tx % 30 == 0 && ty % 16 == 0)
            printf("HINTS tx %d ty %d rays %d cheap %d grid_rays %d lit %d grid_tests %d\n", tx, ty, a, b, c, d, e);
    }
#endif
    if (!kLat && active) {
        B.sh_bits[pix] = shadowed;
        B.pend_bits[pix] = pending;
    }
#if CG_HINT_QUEUE
    // The deferred grid walks, one queued ray per lane.  A verdict ORs its bit into
    // the word this wave stored above: the wave's stores are acknowledged first
    // (vmcnt), so the OR reaches the word after them.
    if (qn > 0) {
        __asm__ volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0);   // vmcnt, expcnt, lgkmcnt all 0: the stores above are done, the queue written
        __asm__ volatile("" ::: "memory");
        for (int j = lane; j < qn; j += 64) {
            ShadowRay q;
            const float4 a = hq.a[j], b = hq.b[j];
            const int2 e = hq.e[j];
            q.origin = v3(a.x, a.y, a.z);
            q.len = a.w;
            q.r = v3(b.x, b.y, b.z);
            q.rmag = b.w;
            q.nd = -q.r;
            const int k = grid_blocker(B.grid, tc, q, &gtests);
            const unsigned long long bit = 1ull << e.y;
            if (k >= 0) {
                atomicOr(&B.sh_bits[e.x], bit);
            } else {
                const int p = atomicAdd(B.pend_n, 1);
                if (p < B.max_pend)
                    B.pend_ray[p] = PendRay{q.origin.x, q.origin.y, q.origin.z, q.nd.x, q.nd.y, q.nd.z, q.len, q.rmag,
                                            e.x, e.y};
                else
                    atomicOr(&B.pend_bits[e.x], bit);   // past the queue: rt_big_shade_kernel searches it
            }
        }
    }
#endif
    WGTB_END(4);
}

// ---------------------------------------------------------------------------
// K5: certified lit search for the shadow rays K4 left unresolved.
//
// A shadow ray (skeleton.cpp:394) starts at S = P + n 1e-5 with direction
// r = L - P (floats; tri_shadows receives nd = -r) and s = fl(S - v0).  Let D
// = det[-r, e1, e2] = -r.N, T = det[s, e1, e2] = s.N, U, V (N = e1 x e2) be
// the exact determinants of these float inputs; the float evaluations D_f,
// T_f, U_f, V_f differ from them by at most E_D, E_T, E_U, E_V (16 eps times
// the sum of their |triple products|, as in the certificates).  If the
// reference's float test accepts the triangle, the real quotients satisfy
// lambda = T_f / D_f in [-1e-6, 1 + 1e-6] (distance >= 0 and < rmag; rmag /
// len <= 1 + 4 eps), mu = U_f / D_f >= -tiny, nu = V_f / D_f >= -tiny and
// mu + nu <= 1 + 4 eps.  Then
//  (1) |D_f| >= |T_f - D_f| / (1 + 1e-6) and T - D = (s + r).N with s + r =
//      (L - v0) + p, |p| <= pn (the 1e-5 offset and the roundings): |D_f| >=
//      delta = (|(lc - v0).N| - (rho + pn) |N| - E_T - E_D) / (1 + 1e-6) for
//      every light within rho of lc -- delta > 0 unless the triangle's plane
//      passes near the light;
//  (2) Cramer's residual: Q = v0 + mu e1 + nu e2 and P = S + lambda r satisfy
//      |Q - P| <= (|r| E_T + |e1| E_U + |e2| E_V + |s| E_D) / |D_f| + |fl(S -
//      v0) - (S - v0)|, and Q lies within 1e-6 (|e1| + |e2|) of the closed
//      triangle.
// So an accepting triangle has a point within R = (2) / delta + 1e-6 (|e1| +
// |e2|) of the segment S + [-1e-6, 1 + 1e-6] r.  rt_lit_class_kernel bounds R
// per triangle over every shadow ray of the frame (hit positions in the
// scene's hit box, every light): a triangle with delta <= 0 or R > M (a
// quarter grid cell) is "near the light" and listed.  rt_pending_lit_kernel
// tests, with the reference's own test, every listed triangle and every
// triangle of the grid cells within M of the segment: when none accepts, no
// triangle of the scene can -- the ray is lit, the verdict of the reference's
// loop over all n triangles.  (Without a grid every triangle is listed.)
__device__ bool lit_near_light(const RtTri &c, const RtFrame &F, const BigBufs &B)
{
    const RtGrid &G = B.grid;
    if (!G.start) return true;
    const double eps = 5.9604644775390625e-8;   // 2^-24
    const double g = 16.0 * eps;
    const double e1[3] = {c.e1x, c.e1y, c.e1z}, e2[3] = {c.e2x, c.e2y, c.e2z}, v0[3] = {c.v0x, c.v0y, c.v0z};
    const double N[3] = {e1[1] * e2[2] - e2[1] * e1[2], e1[2] * e2[0] - e2[2] * e1[0], e1[0] * e2[1] - e2[0] * e1[1]};
    double S[3], a1[3], a2[3];
    for (int k = 0; k < 3; ++k) {   // |s| over every start in the hit box (+ the 1e-5 offset)
        S[k] = (fmax(fabs(v0[k] - (double)G.blo[k]), fabs((double)G.bhi[k] - v0[k])) + 1.01e-5 * (double)F.nbound) *
                   (1.0 + 1e-6) + 1e-12;
        a1[k] = fabs(e1[k]);
        a2[k] = fabs(e2[k]);
    }
    const double *D = B.litD;
    auto M3 = [](const double x[3], const double y[3], const double z[3]) {   // sum |triple products|
        return x[0] * (y[1] * z[2] + y[2] * z[1]) + y[0] * (x[1] * z[2] + x[2] * z[1]) +
               z[0] * (x[1] * y[2] + x[2] * y[1]);
    };
    const double Ed = g * M3(D, a1, a2), Et = g * M3(S, a1, a2), Eu = g * M3(D, S, a2), Ev = g * M3(D, a1, S);
    const double nN = sqrt_ub(N[0] * N[0] + N[1] * N[1] + N[2] * N[2]);
    const double n1 = sqrt_ub(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
    const double n2 = sqrt_ub(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
    const double sn = sqrt_ub(S[0] * S[0] + S[1] * S[1] + S[2] * S[2]);
    const double dn = sqrt_ub(D[0] * D[0] + D[1] * D[1] + D[2] * D[2]);
    const double ax = (double)F.lc[0] - v0[0], ay = (double)F.lc[1] - v0[1], az = (double)F.lc[2] - v0[2];
    const double aN = ax * N[0] + ay * N[1] + az * N[2];
    const double EaN = 1e-12 * (fabs(ax * N[0]) + fabs(ay * N[1]) + fabs(az * N[2]));
    const double delta = (fabs(aN) - EaN - (F.lrho + B.lit_pn) * nN - Et - Ed) * (1.0 - 2e-6);
    if (!(delta > 0.0)) return true;
    const double R = (dn * Et + n1 * Eu + n2 * Ev + sn * Ed) / delta * (1.0 + 1e-9) + 1e-6 * (n1 + n2) +
                     2.0 * eps * sn + 1e-9;
    return !(R <= (double)B.lit_M);
}

__global__ __launch_bounds__(256) void rt_lit_class_kernel(RtFrame F, const RtTri *__restrict__ tc, BigBufs B)
{
    const int base = blockIdx.x * kBinTris;
    bool near[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = base + r * 256 + (int)threadIdx.x;
        near[r] = i < F.n_tris && lit_near_light(tc[i], F, B);
    }
    bin_append(near, base, B.near_list, B.near_n);
}

// The cells of the walk: slabs of cells along r's major axis a; in slab i the
// part of the segment whose a-coordinate lies within Ms of the slab, and the
// rectangle of cells (axes b, c) within Ms of that part.  Ms = M plus a slack
// for the float evaluation of all of this and of the grid's own cell
// assignment (relative errors ~1e-7 of coordinates).
struct FatWalk {
    float o[3], d[3], Ms, tlo, thi;
    int a, b, c, ia0, ia1;
};

__device__ __forceinline__ int grid_cell(const RtGrid &G, int k, float x)
{
    const float q = fminf(fmaxf((x - G.lo[k]) * G.inv_h, -1.0f), (float)G.res[k]);
    return min(max((int)floorf(q), 0), G.res[k] - 1);
}

__device__ __forceinline__ FatWalk fat_walk_init(const RtGrid &G, vec3 S, vec3 r, float M)
{
    FatWalk w;
    w.o[0] = S.x; w.o[1] = S.y; w.o[2] = S.z;
    w.d[0] = r.x; w.d[1] = r.y; w.d[2] = r.z;
    const float ad[3] = {fabsf(r.x), fabsf(r.y), fabsf(r.z)};
    w.a = ad[0] >= ad[1] ? (ad[0] >= ad[2] ? 0 : 2) : (ad[1] >= ad[2] ? 1 : 2);
    w.b = (w.a + 1) % 3;
    w.c = (w.a + 2) % 3;
    const float big = fmaxf(fmaxf(fabsf(S.x), fabsf(S.y)), fabsf(S.z)) + fmaxf(fmaxf(ad[0], ad[1]), ad[2]);
    w.Ms = M * 1.00001f + 1e-5f * (1.0f + big);
    w.tlo = -1e-6f;
    w.thi = 1.000001f;
    const float p0 = w.o[w.a] + w.tlo * w.d[w.a], p1 = w.o[w.a] + w.thi * w.d[w.a];
    w.ia0 = grid_cell(G, w.a, fminf(p0, p1) - w.Ms);
    w.ia1 = grid_cell(G, w.a, fmaxf(p0, p1) + w.Ms);
    return w;
}

// Cell rectangle of slab i: false when the segment has no part there.
__device__ __forceinline__ bool fat_walk_slab(const RtGrid &G, const FatWalk &w, int i, int &jb0, int &jb1, int &jc0,
                                              int &jc1)
{
    const float xl = G.lo[w.a] + (float)i * G.h - w.Ms, xh = G.lo[w.a] + (float)(i + 1) * G.h + w.Ms;
    float t0 = (xl - w.o[w.a]) / w.d[w.a], t1 = (xh - w.o[w.a]) / w.d[w.a];
    if (!(w.d[w.a] != 0.0f)) {   // r = 0: a point
        t0 = w.tlo;
        t1 = w.thi;
    }
    if (t0 > t1) { const float x = t0; t0 = t1; t1 = x; }
    t0 = fmaxf(t0, w.tlo);
    t1 = fminf(t1, w.thi);
    if (!(t0 <= t1)) return false;
    const float b0 = w.o[w.b] + t0 * w.d[w.b], b1 = w.o[w.b] + t1 * w.d[w.b];
    const float c0 = w.o[w.c] + t0 * w.d[w.c], c1 = w.o[w.c] + t1 * w.d[w.c];
    jb0 = grid_cell(G, w.b, fminf(b0, b1) - w.Ms);
    jb1 = grid_cell(G, w.b, fmaxf(b0, b1) + w.Ms);
    jc0 = grid_cell(G, w.c, fminf(c0, c1) - w.Ms);
    jc1 = grid_cell(G, w.c, fmaxf(c0, c1) + w.Ms);
    return true;
}

__device__ __forceinline__ int fat_walk_cell(const RtGrid &G, const FatWalk &w, int i, int jb, int jc)
{
    int x[3];
    x[w.a] = i;
    x[w.b] = jb;
    x[w.c] = jc;
    return (x[2] * G.res[1] + x[1]) * G.res[0] + x[0];
}

// Whole wave, one (uniform) ray: true when a near-light triangle or a
// triangle of a cell within M of the segment accepts it.
__device__ bool lit_blocked_wave(const RtTri *__restrict__ tc, const BigBufs &B, const PendRay &R, int lane)
{
    const vec3 o = v3(R.ox, R.oy, R.oz), nd = v3(R.nx, R.ny, R.nz);
    const int nn = *B.near_n;
    for (int i0 = 0; i0 < nn; i0 += 64) {
        const int i = i0 + lane;
        const bool hit = i < nn && tri_shadows(tc[B.near_list[i]], o, nd, R.len, R.rmag);
        if (__ballot(hit)) return true;
    }
    const RtGrid &G = B.grid;
    if (!G.start) return false;
    const FatWalk w = fat_walk_init(G, o, -nd, B.lit_M);
    for (int i = w.ia0; i <= w.ia1; ++i) {
        int jb0, jb1, jc0, jc1;
        if (!fat_walk_slab(G, w, i, jb0, jb1, jc0, jc1)) continue;
        const int nb = jb1 - jb0 + 1, ncell = nb * (jc1 - jc0 + 1);
        for (int q0 = 0; q0 < ncell; q0 += 64) {
            // lane q: one cell of the rectangle; its triangles are flattened
            // across the wave by an exclusive scan of the cell sizes
            const int q = q0 + lane, m = min(64, ncell - q0);
            int st = 0, cnt = 0;
            if (q < ncell) {
                const int cell = fat_walk_cell(G, w, i, jb0 + q % nb, jc0 + q / nb);
                st = G.start[cell];
                cnt = G.start[cell + 1] - st;
            }
            int x = cnt;
#pragma unroll
            for (int s = 1; s < 64; s <<= 1) {
                const int y = __shfl_up(x, s);
                if (lane >= s) x += y;
            }
            const int excl = x - cnt, total = __shfl(x, 63);
            for (int j0 = 0; j0 < total; j0 += 64) {
                const int j = min(j0 + lane, total - 1);
                // the last cell whose prefix is <= j holds entry j (every lane
                // takes part in the shuffles)
                int lo = 0;
#pragma unroll
                for (int step = 32; step; step >>= 1) {
                    const int mid = lo + step;
                    const int pm = __shfl(excl, min(mid, 63));
                    if (mid < m && pm <= j) lo = mid;
                }
                const int e = __shfl(st, lo) + j - __shfl(excl, lo);
                const bool hit = j0 + lane < total && tri_shadows(tc[G.tris[e]], o, nd, R.len, R.rmag);
                if (__ballot(hit)) return true;
            }
        }
    }
    return false;
}

// The same for one lane's own ray (the shade kernel's overflow path).
__device__ bool lit_blocked_lane(const RtTri *__restrict__ tc, const BigBufs &B, vec3 o, vec3 nd, float len,
                                 float rmag)
{
    const int nn = *B.near_n;
    for (int i = 0; i < nn; ++i)
        if (tri_shadows(tc[B.near_list[i]], o, nd, len, rmag)) return true;
    const RtGrid &G = B.grid;
    if (!G.start) return false;
    const FatWalk w = fat_walk_init(G, o, -nd, B.lit_M);
    for (int i = w.ia0; i <= w.ia1; ++i) {
        int jb0, jb1, jc0, jc1;
        if (!fat_walk_slab(G, w, i, jb0, jb1, jc0, jc1)) continue;
        for (int jc = jc0; jc <= jc1; ++jc)
            for (int jb = jb0; jb <= jb1; ++jb) {
                const int cell = fat_walk_cell(G, w, i, jb, jc);
                for (int e = G.start[cell], ee = G.start[cell + 1]; e < ee; ++e)
                    if (tri_shadows(tc[G.tris[e]], o, nd, len, rmag)) return true;
            }
    }
    return false;
}

// One wave per unresolved shadow ray (grid-stride); a blocked ray sets its
// verdict bit.
#ifdef CG_PEND_WAVES   // A/B builds
__global__ __launch_bounds__(256, CG_PEND_WAVES) void rt_pending_lit_kernel(
#else
__global__ __launch_bounds__(256) void rt_pending_lit_kernel(
#endif
    RtFrame F, const RtTri *__restrict__ tc, BigBufs B)
{
    const int np = min(*B.pend_n, B.max_pend);
    const int lane = threadIdx.x & 63;
    for (int p = blockIdx.x * 4 + (int)(threadIdx.x >> 6); p < np; p += gridDim.x * 4) {
        const int pu = __builtin_amdgcn_readfirstlane(p);
        const PendRay R = B.pend_ray[pu];
        if (lit_blocked_wave(tc, B, R, lane) && lane == 0) atomicOr(&B.sh_bits[R.pix], 1ull << R.bit);
    }
}

// K7: shading in the reference's order (:143-166) from the shadow verdicts
// (per sub-ray in per-pixel mode, per lattice point in lattice mode); with
// more than 7 lights in per-pixel mode each (s, l) is resolved here (grid,
// then the bin's certified shadow list).
template <int LM>
#ifdef CG_SHADE_WAVES   // A/B builds
__global__ __launch_bounds__(kRtThreads, CG_SHADE_WAVES) void rt_big_shade_kernel(
#else
__global__ __launch_bounds__(kRtThreads) void rt_big_shade_kernel(
#endif
    RtFrame F, const RtTri *__restrict__ tc,
                                                                  const RtShade *__restrict__ shade,
                                                                  const RtSphere *__restrict__ sph, BigBufs B,
                                                                  uint32_t *__restrict__ out)
{
    constexpr bool kLat = LM > 0;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;   // wave: uniform (SGPR)
    const int tx = blockIdx.x * (kRtTileW / 8) + wave, ty = blockIdx.y;
    if (tx >= B.tiles_x) return;
    const int u = tx * 8 + (lane & 7), L = ty * 8 + (lane >> 3);
    const bool inside = u < F.W && L < F.rows_out;
    if (!inside) return;
    const int v = shard_row(F, L);
    const bool active = v < F.H;
    uint32_t px = 0u;
    if (active) {
        const size_t npix = (size_t)F.rows_out * F.W, pix = (size_t)L * F.W + u;
        const vec4 dir = pixel_dir(F, u, v);
        const bool flags_fit = kLat || 9 * F.n_lights <= 64;
        const unsigned long long pshadowed = !kLat && flags_fit && F.n_lights > 0 ? B.sh_bits[pix] : 0ull;
        // rays past the queue still carry pending bits: the lit search per lane
        const unsigned long long pleft = !kLat && flags_fit && F.n_lights > 0 ? B.pend_bits[pix] : 0ull;
        const int bin = (tx / kBinTilesX) + (ty / kBinTilesY) * B.bins_x;
        vec3 pc = v3(0.0f, 0.0f, 0.0f);
        bool valid = false;
        const vec3 ind = v3(F.indirect, F.indirect, F.indirect);
        const float m = 0.5f;
        for (int s = 0; s < 9; ++s) {
            const int i = s / 3 - 1, j = s % 3 - 1;
            const vec3 nd = v3(dir.x + (m * (float)i), dir.y + (m * (float)j), F.focal);   // :137
            const size_t id = kLat ? (size_t)(2 * L + j + 1) * B.lat_w + ((LM == 2 ? 3 : 2) * u + i + 1)
                                   : s * npix + pix;
            int bi;
            vec3 pos, normal;
            hit_geometry(F, B, shade, sph, nd, id, bi, pos, normal);
            if (bi == INT_MIN) continue;
            valid = true;
            unsigned long long shadowed = pshadowed, left = pleft;
            if (kLat && F.n_lights > 0) {
                shadowed = B.sh_bits[id];
                left = B.pend_bits[id];
            }
            vec3 oc = object_colour(shade, sph, bi);
            for (int l = 0; l < F.n_lights; ++l) {                                    // :151-153
                const RtLight Lt = F.lights[l];
                const ShadowRay q = shadow_ray(Lt, pos, normal);
                bool ts;
                const int bit = kLat ? l : s * F.n_lights + l;
                if (flags_fit) {
                    ts = ((shadowed >> bit) & 1ull) != 0;
                    if (!ts && ((left >> bit) & 1ull)) ts = lit_blocked_lane(tc, B, q.origin, q.nd, q.len, q.rmag);
                } else {
                    ts = grid_blocker(B.grid, tc, q) >= 0 || any_hit_bin(tc, B, F.n_tris, bin, q);
                }
                pc = pc + big_direct_light(F, sph, Lt, q, normal, oc, ts);
            }
            pc = pc + (oc * ind);                                                     // :156
        }
        px = valid ? put_pixel(div_const(pc, 9.0f, 1.0f / 9.0f)) : put_pixel(v3(0.0f, 0.0f, 0.0f));         // :160-166
    }
    out[(size_t)L * F.W + u] = px;
}

// ---------------------------------------------------------------------------
// Lattice mode (K1): contiguous rows (whole frame or band), verdict bits for
// every light in one word per point, and R leaving y alone with dir.x a
// function of x alone (cg_rt.hip rt_lattice_ok): 1 = shared half-pixel
// columns (dir.x = x exactly), 2 = per-pixel columns (a yaw; bounded entries).
int rt_big_mode(const RtFrame &F)
{
    const float *R = F.R;
    if (!(R[1] == 0.0f && R[5] == 1.0f && R[9] == 0.0f && R[13] == 0.0f && R[4] == 0.0f)) return 0;
    if (!(F.nranks == 1 && F.n_lights <= 64 && F.W < (1 << 20) && F.H < (1 << 20))) return 0;
    if (R[0] == 1.0f && R[8] == 0.0f && R[12] == 0.0f) return 1;
    for (int k : {0, 8, 12})
        if (!(std::fabs(R[k]) <= 1e6f)) return 0;
    return std::fabs(F.focal) <= 1e6f ? 2 : 0;
}
static bool rt_big_lattice(const RtFrame &F) { return rt_big_mode(F) != 0; }

BigBufs big_layout(const RtFrame &F, const BigCaps &caps)
{
    BigBufs B{};
    B.bins_x = (F.W + kBinW - 1) / kBinW;
    B.bins_y = (F.rows_out + kBinH - 1) / kBinH;
    B.tiles_x = (F.W + 7) / 8;
    B.tiles_y = (F.rows_out + 7) / 8;
    B.sups_x = (B.bins_x + kSupBins - 1) / kSupBins;
    B.sups_y = (B.bins_y + kSupBins - 1) / kSupBins;
    B.nch = std::max(1, (F.n_tris + kBinTris - 1) / kBinTris);
    B.cap_sup = caps.sup;
    B.cap_bin = caps.bin;
    B.cap_sbin = caps.sbin;
    B.cap_sorted = caps.sorted;
    const int rows = std::min(F.rows_out, F.H - F.row0);
    const int mode = rt_big_mode(F);
    if (mode && rows > 0) {
        B.lat_yaw = mode == 2;
        B.lat_w = mode == 2 ? 3 * F.W : 2 * F.W + 1;
        B.lat_h = 2 * rows + 1;
    }
    return B;
}

// The per-frame counters (cleared by one memset at the start of the scratch).
size_t big_counter_bytes(const BigBufs &B)
{
    const size_t bins = (size_t)B.bins_x * B.bins_y;
    const size_t sups = (size_t)B.sups_x * B.sups_y;
    return 4 * 8 + 16 + 4 * bins * kDepthBuckets * 4 + 2 * bins * 4 + bins * 4 + (sups + 2 * bins) * 4;
}

// Ray slots (hits) and verdict words of the mode.
static size_t big_slots(const BigBufs &B, const RtFrame &F)
{
    return B.lat_w ? (size_t)B.lat_w * B.lat_h : 9 * (size_t)F.rows_out * F.W;
}
static size_t big_words(const BigBufs &B, const RtFrame &F)
{
    return B.lat_w ? (size_t)B.lat_w * B.lat_h : (size_t)F.rows_out * F.W;
}

// Bytes of device scratch for big_layout(F, caps), and its carving: the
// frame-sized arrays, the chunk tables, then the pools.
size_t big_scratch_bytes(const BigBufs &B, const RtFrame &F)
{
    const size_t bins = (size_t)B.bins_x * B.bins_y, sups = (size_t)B.sups_x * B.sups_y;
    const size_t tiles = (size_t)B.tiles_x * B.tiles_y;
    return big_counter_bytes(B) + 2 * bins * (kDepthBuckets + 1) * 4 + 2 * bins * 32 * 16 + (tiles + bins) * sizeof(ShadowBox) +
           big_slots(B, F) * 8 + 2 * big_words(B, F) * 8 + (size_t)kMaxPend * sizeof(PendRay) +
           (size_t)F.n_tris * 4 + (sups + 2 * bins) * B.nch * sizeof(Chunk) + (sups + bins) * (B.nch + 2) * 4 +
           (size_t)B.cap_sup * 2 * (4 + 8) + (size_t)B.cap_sbin * 4 + (size_t)B.cap_bin * 6 * 8 + (size_t)B.cap_sorted * 2 * 8 +
           tiles * 4 + 9 * 64;
}
void big_carve(BigBufs &B, const RtFrame &F, void *base)
{
    const size_t bins = (size_t)B.bins_x * B.bins_y, sups = (size_t)B.sups_x * B.sups_y;
    const size_t slots = big_slots(B, F), words = big_words(B, F);
    const size_t tiles = (size_t)B.tiles_x * B.tiles_y;
    char *p = (char *)base;
    auto align = [&] { p = (char *)(((uintptr_t)p + 63) & ~(uintptr_t)63); };
    B.pool_n = (unsigned long long *)p; p += 4 * 8;   // counters first: one memset clears them
    B.pend_n = (int *)p;            p += 16;
    B.near_n = B.pend_n + 1;
    B.bkt_cnt = (int *)p;           p += 2 * bins * kDepthBuckets * 4;
    B.bkt_min_inv = (unsigned *)p;  p += 2 * bins * kDepthBuckets * 4;
    B.key_lo_inv = (unsigned *)p;   p += bins * 4;
    B.key_hi = (unsigned *)p;       p += bins * 4;
    B.bin_nch = (int *)p;           p += bins * 4;
    B.sup_over = (int *)p;          p += sups * 4;
    B.bin_over = (int *)p;          p += bins * 4;
    B.sbin_over = (int *)p;         p += bins * 4;
    B.bkt_off = (int *)p;           p += 2 * bins * (kDepthBuckets + 1) * 4;
    align();
    B.tile_bb = (float *)p;         p += 2 * bins * 32 * 16;
    align();
    B.wave_box = (ShadowBox *)p; p += tiles * sizeof(ShadowBox);
    B.bin_box = (ShadowBox *)p;  p += bins * sizeof(ShadowBox);
    align();
    B.walk_order = (int *)p;     p += tiles * 4;
    align();
    B.hit_bi = (int *)p;   p += slots * 4;
    B.hit_t = (float *)p;  p += slots * 4;
    align();
    B.sh_bits = (unsigned long long *)p;   p += words * 8;
    B.pend_bits = (unsigned long long *)p; p += words * 8;
    B.pend_ray = (PendRay *)p;             p += (size_t)kMaxPend * sizeof(PendRay);
    B.near_list = (int *)p;                p += (size_t)F.n_tris * 4;
    align();
    B.sup_chunk = (Chunk *)p;   p += sups * B.nch * sizeof(Chunk);
    B.bin_chunk = (Chunk *)p;   p += bins * B.nch * sizeof(Chunk);
    B.sbin_chunk = (Chunk *)p;  p += bins * B.nch * sizeof(Chunk);
    B.sup_pre = (int *)p;       p += sups * B.nch * 4;
    B.bin_pre = (int *)p;       p += bins * B.nch * 4;
    B.sup_tot = (int *)p;       p += sups * 4;
    B.bin_tot = (int *)p;       p += bins * 4;
    B.sup_base = (int *)p;      p += sups * 4;
    B.bin_base = (int *)p;      p += bins * 4;
    align();
    B.bin_ent = (unsigned long long *)p;    p += (size_t)B.cap_bin * 8;
    B.bin_pbox = (unsigned long long *)p;   p += (size_t)B.cap_bin * 8;
    B.bin_pbox2 = (unsigned long long *)p;  p += (size_t)B.cap_bin * 8;
    B.bin_sorted = (unsigned long long *)p; p += (size_t)B.cap_sorted * 8;
    B.bin_spbox = (unsigned long long *)p;  p += (size_t)B.cap_sorted * 8;
    B.flat_ent = (unsigned long long *)p;   p += (size_t)B.cap_bin * 8;
    B.flat_pbox = (unsigned long long *)p;  p += (size_t)B.cap_bin * 8;
    B.flat_pbox2 = (unsigned long long *)p; p += (size_t)B.cap_bin * 8;
    B.sup_pool = (int *)p;                  p += (size_t)B.cap_sup * 4;
    B.sup_flat = (int *)p;                  p += (size_t)B.cap_sup * 4;
    align();
    B.sup_pbox_pool = (unsigned long long *)p; p += (size_t)B.cap_sup * 8;
    B.sup_flat_pbox = (unsigned long long *)p; p += (size_t)B.cap_sup * 8;
    B.sbin_pool = (int *)p;
}

// Frame bounds of the lit search (K5): |r_k| = |fl(L - P)_k| over every
// light and hit position, |p| (see lit_near_light), the walk margin.
static void lit_bounds(BigBufs &B, const RtFrame &F, const RtGrid &G)
{
    const double eps = 5.9604644775390625e-8;
    double pmax = 0.0, dmax = 0.0, smax = 0.0;
    for (int k = 0; k < 3; ++k) {
        B.litD[k] = std::max(std::fabs((double)F.lmax[k] - G.blo[k]), std::fabs((double)G.bhi[k] - F.lmin[k])) *
                        (1.0 + 1e-6) + 1e-12;
        pmax = std::max(pmax, std::max(std::fabs((double)G.blo[k]), std::fabs((double)G.bhi[k])));
        dmax = std::max(dmax, B.litD[k]);
        smax = std::max(smax, (double)G.bhi[k] - G.blo[k]);
    }
    smax += 1.01e-5 * F.nbound + 1e-6 * pmax;
    // p = (S - P - n 1e-5) + n 1e-5 + (fl(L - P) - (L - P)) + (fl(S - v0) - (S - v0))
    B.lit_pn = std::sqrt(3.0) * (1.01e-5 * F.nbound + eps * (pmax + 1e-4) + eps * dmax + eps * smax) * (1.0 + 1e-6) +
               1e-12;
    B.lit_M = 0.25f * G.h;
}

hipError_t launch_rt_big(const RtFrame &F, RtTri *d_tc, const RtShade *d_shade, const RtSphere *d_sph,
                         const RtGrid &grid, void *scratch, uint32_t *d_out, hipStream_t st, const RtGeo *d_geo,
                         const cg_tri *d_tris,
                         int pend_cap, const BigCaps &caps, unsigned long long *h_demand, int dry)
{
    BigBufs B = big_layout(F, caps);
    if (2 * B.bins_x * B.bins_y > kMaxSubs) return hipErrorInvalidValue;   // rt_bin_scan_kernel's LDS table
    big_carve(B, F, scratch);
    B.grid = grid;
    B.max_pend = pend_cap > 0 ? std::min(pend_cap, kMaxPend) : kMaxPend;
    lit_bounds(B, F, grid);
    const int bins = B.bins_x * B.bins_y;
    hipError_t e = hipMemsetAsync(B.pool_n, 0, big_counter_bytes(B), st);
    if (e != hipSuccess) return e;
    const bool lat = B.lat_w != 0;
    const bool flags_fit = lat || 9 * F.n_lights <= 64;
    const dim3 bgrid((F.n_tris + kBinTris - 1) / kBinTris, bins);
    const dim3 pgrid((F.W + kRtTileW - 1) / kRtTileW, (F.rows_out + kRtTileH - 1) / kRtTileH);
    // the first pass also writes the frame's RtTri (rt_sup_primary_kernel)
    hipLaunchKernelGGL(rt_sup_primary_kernel, dim3(bgrid.x, sup_groups(B.sups_x * B.sups_y)), dim3(256), 0, st, F,
                       d_geo, d_tc, B);
    const int sups = B.sups_x * B.sups_y;
    hipLaunchKernelGGL(rt_chunk_scan_kernel, dim3(sups), dim3(1024), 0, st, B.sup_chunk, nullptr, B.nch, B.sup_pre,
                       B.sup_tot);
    hipLaunchKernelGGL(rt_list_base_kernel, dim3(1), dim3(1024), 0, st, B.sup_tot, sups, B.sup_base);
    // the compaction strides over each super list's flat entries with 128 workgroups per
    // super-bin (one per chunk left most lanes idle: ~70 entries per chunk at C5): C5 one frame
    // 320 -> 173 us (32: 386, 512: 203); CG_CMP_WGS: A/B runs
    static const int cmp_wgs = [] {
        const char *e = std::getenv("CG_CMP_WGS");
        const int v = e ? std::atoi(e) : 128;
        return v > 0 ? v : 128;
    }();
    hipLaunchKernelGGL(rt_sup_compact_kernel, dim3(std::min(cmp_wgs, (F.n_tris + 255) / 256), sups), dim3(256), 0, st,
                       F, d_tc, B);
    // workgroups per bin striding over its super list: fewer, longer workgroups fill the
    // certificate batches (1,024 entries per batch; C5's ~70k-entry super lists give each of 64
    // workgroups one ~110-entry batch) -- C5 bin pass 379 -> 272 us at 16, 266 at 8, 314 at 4;
    // C5 178 -> 181-182 fps (profiles/r05_ab_bins.json).  CG_BIN_WGS: A/B runs.
    static const int bin_wgs = [] {
        const char *e = std::getenv("CG_BIN_WGS");
        const int v = e ? std::atoi(e) : 16;
        return v > 0 ? v : 16;
    }();
    hipLaunchKernelGGL(rt_bin_primary_kernel, dim3(std::min(bin_wgs, (int)bgrid.x), bins), dim3(256), 0, st, F, d_tc,
                       d_tris, B);
    hipLaunchKernelGGL(rt_chunk_scan_kernel, dim3(bins), dim3(1024), 0, st, B.bin_chunk, B.bin_nch, B.nch, B.bin_pre,
                       B.bin_tot);
    hipLaunchKernelGGL(rt_list_base_kernel, dim3(1), dim3(1024), 0, st, B.bin_tot, bins, B.bin_base);
    // workgroups per bin for the bucket count and scatter passes over a bin's list: C5 count
    // 241 -> 165 us at 16, 166 at 8; scatter 106 -> 63 / 49 us; CG_CNT_WGS: A/B runs
    static const int cnt_wgs = [] {
        const char *e = std::getenv("CG_CNT_WGS");
        const int v = e ? std::atoi(e) : 8;
        return v > 0 ? v : 8;
    }();
    const dim3 egrid(std::min(cnt_wgs, (F.n_tris + 1023) / 1024), bins);   // workgroups stride over a bin's list
    hipLaunchKernelGGL(rt_bin_count_kernel, egrid, dim3(256), 0, st, F, d_tc, d_tris, B);
    hipLaunchKernelGGL(rt_bin_scan_kernel, dim3(1), dim3(1024), 0, st, B, 2 * bins);
    // sizing passes (cg_shim.hip) stop early and report the demand: dry 1
    // after the camera-ray lists, dry 2 after the many-light shadow lists
    auto demand = [&]() {
        const hipError_t c = h_demand ? hipMemcpyAsync(h_demand, B.pool_n, 4 * sizeof(unsigned long long),
                                                       hipMemcpyDeviceToHost, st)
                                      : hipSuccess;
        return c != hipSuccess ? c : hipGetLastError();
    };
    if (dry == 1) return demand();
    hipLaunchKernelGGL(rt_half_tiles_kernel, dim3(2 * bins), dim3(64), 0, st, F, B);
    hipLaunchKernelGGL(rt_bin_scatter_kernel, egrid, dim3(256), 0, st, F, B);
    static const int hm_wgs = [] {   // A/B: CG_HM_WGS
        const char *e = std::getenv("CG_HM_WGS");
        const int v = e ? std::atoi(e) : 2048;
        return v > 0 ? v : 2048;
    }();
    hipLaunchKernelGGL(rt_half_mask_kernel, dim3(hm_wgs), dim3(256), 0, st, F, d_tc, B);
    {
        const char *wo = std::getenv("CG_WALK_ORDER");
        if (wo && wo[0] == '0') B.walk_order = nullptr;
        else hipLaunchKernelGGL(rt_walk_order_kernel, dim3(1), dim3(1024), 0, st, B, (int)pgrid.x, (int)pgrid.y);
    }
    {
        const int kt_id = KT_RT_BIG_PRIMARY;
        if (lat && B.lat_yaw)
            kt_launch(kt_id, rt_big_primary_kernel<2>, pgrid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph, B);
        else if (lat)
            kt_launch(kt_id, rt_big_primary_kernel<1>, pgrid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph, B);
        else
            kt_launch(kt_id, rt_big_primary_kernel<0>, pgrid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph, B);
    }
    if (!flags_fit) {
        hipLaunchKernelGGL(rt_bin_boxes_kernel, dim3(bins), dim3(64), 0, st, B);
        hipLaunchKernelGGL(rt_bin_shadow_kernel, bgrid, dim3(256), 0, st, F, d_tc, B);
        if (dry == 2) return demand();
    } else if (F.n_lights > 0) {
        hipLaunchKernelGGL(rt_lit_class_kernel, dim3(bgrid.x), dim3(256), 0, st, F, d_tc, B);
        {
            const int kt_id = KT_RT_SHADOW_HINTS;
            if (lat && B.lat_yaw)
                kt_launch(kt_id, rt_shadow_hints_kernel<2>, pgrid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph, B);
            else if (lat)
                kt_launch(kt_id, rt_shadow_hints_kernel<1>, pgrid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph, B);
            else
                kt_launch(kt_id, rt_shadow_hints_kernel<0>, pgrid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph, B);
        }
        static const int pl_wgs = [] {   // A/B: CG_PL_WGS
            const char *e = std::getenv("CG_PL_WGS");
            const int v = e ? std::atoi(e) : 1024;
            return v > 0 ? v : 1024;
        }();
        hipLaunchKernelGGL(rt_pending_lit_kernel, dim3(pl_wgs), dim3(256), 0, st, F, d_tc, B);
    }
    if (lat && B.lat_yaw)
        hipLaunchKernelGGL(rt_big_shade_kernel<2>, pgrid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph, B, d_out);
    else if (lat)
        hipLaunchKernelGGL(rt_big_shade_kernel<1>, pgrid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph, B, d_out);
    else
        hipLaunchKernelGGL(rt_big_shade_kernel<0>, pgrid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph, B, d_out);
    return demand();   // the pools' demand, for the host's sizing of the next frames
}

// Whether a frame's shading uses the per-bin shadow lists (per-pixel mode
// with more than 7 lights): its sizing then needs a second dry stage.
bool rt_big_shadow_lists(const RtFrame &F)
{
    return !rt_big_lattice(F) && 9 * F.n_lights > 64;
}

// Does the closed triangle v meet the cell box centred at c with half-width
// hw, widened by eps?  Separating-axis test (the box's 3 axes, the
// triangle's normal, the 9 edge x axis products) in FP64 on the float
// vertices; the widening and the 1e-9 relative slack make it a superset of
// the exact overlap, which is all the certified lit search needs (a triangle
// is listed in every cell holding a point of it).
static bool tri_meets_cell(const double v[3][3], const double c[3], double hw, double eps)
{
    const double h = hw + eps;
    double p[3][3];
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) p[i][k] = v[i][k] - c[k];
    auto beyond = [](double a, double b, double d, double r) {   // [min, max] of a, b, d misses [-r, r]
        return std::min(a, std::min(b, d)) > r || std::max(a, std::max(b, d)) < -r;
    };
    for (int k = 0; k < 3; ++k)
        if (beyond(p[0][k], p[1][k], p[2][k], h)) return false;
    double e[3][3];
    for (int k = 0; k < 3; ++k) {
        e[0][k] = p[1][k] - p[0][k];
        e[1][k] = p[2][k] - p[1][k];
        e[2][k] = p[0][k] - p[2][k];
    }
    const double n[3] = {e[0][1] * e[1][2] - e[0][2] * e[1][1], e[0][2] * e[1][0] - e[0][0] * e[1][2],
                         e[0][0] * e[1][1] - e[0][1] * e[1][0]};
    const double nd = n[0] * p[0][0] + n[1] * p[0][1] + n[2] * p[0][2];
    if (std::fabs(nd) > h * (std::fabs(n[0]) + std::fabs(n[1]) + std::fabs(n[2])) * (1.0 + 1e-9)) return false;
    for (int a = 0; a < 3; ++a)
        for (int j = 0; j < 3; ++j) {
            double ax[3] = {0.0, 0.0, 0.0};   // unit axis a x edge j
            const int b = (a + 1) % 3, d = (a + 2) % 3;
            ax[b] = -e[j][d];
            ax[d] = e[j][b];
            const double q0 = ax[0] * p[0][0] + ax[1] * p[0][1] + ax[2] * p[0][2];
            const double q1 = ax[0] * p[1][0] + ax[1] * p[1][1] + ax[2] * p[1][2];
            const double q2 = ax[0] * p[2][0] + ax[1] * p[2][1] + ax[2] * p[2][2];
            if (beyond(q0, q1, q2, h * (std::fabs(ax[0]) + std::fabs(ax[1]) + std::fabs(ax[2])) * (1.0 + 1e-9)))
                return false;
        }
    return true;
}

// Host build of the scene grid: cubic cells sized for ~1/4 triangle centroid
// per cell, each triangle listed in every cell it meets (tri_meets_cell over
// the cells of its bounding box).  Against cells twice as wide listing whole
// bounding boxes, C5's shadow rays test ~2.8x fewer triangles per unit
// length.  Returns false (no grid) when the lists would exceed max_entries.
bool rt_grid_build(const cg_tri *t, int n, RtGrid &g, std::vector<int> &start, std::vector<int> &tris,
                   size_t max_entries)
{
    if (n <= 0) return false;
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    auto bb = [&](const cg_tri &q, float mn[3], float mx[3]) {
        const cg_vec4 *v[3] = {&q.v0, &q.v1, &q.v2};
        for (int a = 0; a < 3; ++a) { mn[a] = FLT_MAX; mx[a] = -FLT_MAX; }
        for (const cg_vec4 *p : v) {
            const float c[3] = {p->x, p->y, p->z};
            for (int a = 0; a < 3; ++a) { mn[a] = std::min(mn[a], c[a]); mx[a] = std::max(mx[a], c[a]); }
        }
    };
    for (int i = 0; i < n; ++i) {
        float mn[3], mx[3];
        bb(t[i], mn, mx);
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], mn[a]); hi[a] = std::max(hi[a], mx[a]); }
    }
    double ext[3], vol = 1.0;
    for (int a = 0; a < 3; ++a) {
        if (!std::isfinite(lo[a]) || !std::isfinite(hi[a])) return false;
        lo[a] -= 1e-4f;
        hi[a] += 1e-4f;
        ext[a] = (double)hi[a] - lo[a];
        vol *= ext[a];
    }
    double h = 0.5 * std::cbrt(vol / std::max(1.0, n / 2.0));
    for (int a = 0; a < 3; ++a) h = std::max(h, ext[a] / 512.0);
    for (int a = 0; a < 3; ++a) {
        g.lo[a] = lo[a];
        g.res[a] = std::max(1, std::min(512, (int)std::ceil(ext[a] / h)));
    }
    g.h = (float)h;
    g.inv_h = (float)(1.0 / h);
    const size_t cells = (size_t)g.res[0] * g.res[1] * g.res[2];
    const double gh = g.h, hw = 0.5 * gh, eps = 1e-4 * gh;
    // (cell, triangle) pairs in triangle order, then a counting sort by cell
    std::vector<std::pair<unsigned, int>> pairs;
    pairs.reserve((size_t)n * 8);
    for (int i = 0; i < n; ++i) {
        float mn[3], mx[3];
        bb(t[i], mn, mx);
        int c0[3], c1[3];
        for (int a = 0; a < 3; ++a) {   // the cells whose widened box meets the bounding box
            c0[a] = std::min(std::max((int)std::floor(((double)mn[a] - g.lo[a] - 2.0 * eps) / gh), 0), g.res[a] - 1);
            c1[a] = std::min(std::max((int)std::floor(((double)mx[a] - g.lo[a] + 2.0 * eps) / gh), 0), g.res[a] - 1);
        }
        const double v[3][3] = {{t[i].v0.x, t[i].v0.y, t[i].v0.z}, {t[i].v1.x, t[i].v1.y, t[i].v1.z},
                                {t[i].v2.x, t[i].v2.y, t[i].v2.z}};
        for (int z = c0[2]; z <= c1[2]; ++z)
            for (int y = c0[1]; y <= c1[1]; ++y)
                for (int x = c0[0]; x <= c1[0]; ++x) {
                    const double c[3] = {(double)g.lo[0] + (x + 0.5) * gh, (double)g.lo[1] + (y + 0.5) * gh,
                                         (double)g.lo[2] + (z + 0.5) * gh};
                    if (!tri_meets_cell(v, c, hw, eps)) continue;
                    if (pairs.size() >= max_entries) return false;
                    pairs.emplace_back((unsigned)(((size_t)z * g.res[1] + y) * g.res[0] + x), i);
                }
    }
    start.assign(cells + 1, 0);
    for (const auto &pr : pairs) ++start[pr.first + 1];
    for (size_t c = 0; c < cells; ++c) start[c + 1] += start[c];
    tris.assign(pairs.size(), 0);
    std::vector<int> fill(start.begin(), start.end() - 1);
    for (const auto &pr : pairs) tris[fill[pr.first]++] = pr.second;
    return true;
}

size_t rt_big_scratch_bytes(const RtFrame &F, const BigCaps &caps)
{
    BigBufs B = big_layout(F, caps);
    return big_scratch_bytes(B, F);
}

}  // namespace cg

#ifdef CG_WG_TIMING
extern "C" int cg_diag_wg_timing_big(void *buf, unsigned cap)
{
    unsigned long long *p = (unsigned long long *)buf;
    if (hipMemcpyToSymbol(HIP_SYMBOL(cg::g_wgtb), &p, sizeof p) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(cg::g_wgtb_cap), &cap, sizeof cap) != hipSuccess) return -1;
    return 0;
}
#endif

#ifdef CG_WORK_COUNT
// Counting build: this translation unit's work counters (cg_rt_dev.h WorkKind order); reset after reading.
extern "C" int cg_diag_work_counts_big(unsigned long long *out, int reset)
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
