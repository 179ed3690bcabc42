// cg_geometry.hip -- the rasteriser's per-frame geometry (skeleton.cpp:205-241)
// on the host (cg_rast_prepare, for callers that bring their own lists) and on
// the device (rast_geometry_kernel, used by cg_rast_draw*): camera space,
// shadow volumes, rotation, clip space and the six clip planes.  Both run the
// same __host__ __device__ code in cg_geom.h, so their lists are identical.
#include <cstring>
#include <vector>

#include "cg_geom.h"

namespace cg {

GeomParams geom_params(const cg_rast_params &p)
{
    GeomParams g;
    g.W = p.width;
    g.H = p.height;
    g.focal = p.focal;
    g.cam[0] = p.camera.x; g.cam[1] = p.camera.y; g.cam[2] = p.camera.z; g.cam[3] = p.camera.w;
    std::memcpy(g.R, p.R, sizeof(g.R));
    g.light_scene[0] = p.light_scene.x; g.light_scene[1] = p.light_scene.y;
    g.light_scene[2] = p.light_scene.z; g.light_scene[3] = p.light_scene.w;
    return g;
}

constexpr int kGeomThreads = 512;
constexpr int kGeomWaves = kGeomThreads / 64;
constexpr int kGeomLds = 512;      // list entries held in LDS per list (more spill to global)

// A list of triangles between clip planes: only the vertices change while
// clipping -- a split's extra triangle copies normal, colour, texture and index
// from its parent (skeleton.cpp:838-841) -- so an entry is three vertices plus
// the input triangle it descends from.  Entries [0, kGeomLds) live in LDS, the
// rest in a global spill buffer (vertices + `index` = parent).
struct GeomList {
    float4 v0[kGeomLds], v1[kGeomLds], v2[kGeomLds];
    int par[kGeomLds];
};

__device__ __forceinline__ void glist_put(GeomList &L, cg_rtri *spill, int i, const cg_rtri &t, int parent)
{
    if (i < kGeomLds) {
        L.v0[i] = make_float4(t.v0.x, t.v0.y, t.v0.z, t.v0.w);
        L.v1[i] = make_float4(t.v1.x, t.v1.y, t.v1.z, t.v1.w);
        L.v2[i] = make_float4(t.v2.x, t.v2.y, t.v2.z, t.v2.w);
        L.par[i] = parent;
    } else {
        cg_rtri &d = spill[i - kGeomLds];
        d.v0 = t.v0;
        d.v1 = t.v1;
        d.v2 = t.v2;
        d.index = parent;
    }
}

__device__ __forceinline__ cg_rtri glist_get(const GeomList &L, const cg_rtri *spill, int i, int &parent)
{
    cg_rtri t{};
    if (i < kGeomLds) {
        const float4 a = L.v0[i], b = L.v1[i], c = L.v2[i];
        t.v0 = cg_vec4{a.x, a.y, a.z, a.w};
        t.v1 = cg_vec4{b.x, b.y, b.z, b.w};
        t.v2 = cg_vec4{c.x, c.y, c.z, c.w};
        parent = L.par[i];
    } else {
        const cg_rtri &d = spill[i - kGeomLds];
        t.v0 = d.v0;
        t.v1 = d.v1;
        t.v2 = d.v2;
        parent = d.index;
    }
    return t;
}

// One workgroup, breadth-first -- the reference's own order (clip() walks the
// whole list plane by plane, a split inserting [modified, extra] in place):
// per plane, thread i clips list entry i into 0..2 children, a wave ballot
// scan plus an 8-entry LDS scan gives each child its slot, and the children
// land, in order, in the next list.  Plane 1 reads the input triangles built
// on the fly (room, then each box triangle and its 6 shadow triangles; kept in
// `inb` for their attributes); the lists ping-pong between the two LDS lists
// (spilling to scr0/scr1) and plane 6 writes whole triangles to `out`.
// out_n[0] = final count, out_light = rotated camera-space light (:223).
__global__ __launch_bounds__(kGeomThreads) void rast_geometry_kernel(
    GeomParams p, const cg_rtri *__restrict__ room, int n_room, const cg_rtri *__restrict__ boxes,
    int n_boxes, cg_rtri *__restrict__ out, cg_rtri *scr0, cg_rtri *scr1, cg_rtri *inb, int cap,
    int *__restrict__ out_n, cg_vec4 *__restrict__ out_light)
{
    __shared__ GeomList s_list[2];
    __shared__ int wsum[kGeomWaves];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    if (threadIdx.x == 0) *out_light = C4(mat4_mul(p.R, geom_light_camera(p)));
    int len = n_room + 7 * n_boxes;
    for (int pl = 1; pl <= 6; ++pl) {
        const int si = pl & 1, di = si ^ 1;                 // plane 1 writes list 0
        const cg_rtri *sspill = si ? scr1 : scr0;
        cg_rtri *dspill = di ? scr1 : scr0;
        int carry = 0;
        for (int base = 0; base < len; base += kGeomThreads) {
            const int i = base + (int)threadIdx.x;
            cg_rtri ch[2];
            int k = 0, parent = i;
            if (i < len) {
                cg_rtri t;
                if (pl == 1) {
                    t = geom_input(p, room, n_room, boxes, i);
                    inb[i] = t;
                } else {
                    t = glist_get(s_list[si], sspill, i, parent);
                }
                k = clip_plane(t, pl, p, ch);
            }
            const unsigned long long b0 = __ballot(k & 1), b1 = __ballot(k >> 1);
            const int pre = __popcll(b0 & lt) + 2 * __popcll(b1 & lt);
            if (lane == 63) wsum[wid] = pre + k;
            __syncthreads();
            int off = carry, tot = 0;
            for (int w = 0; w < kGeomWaves; ++w) {
                const int v = wsum[w];
                off += w < wid ? v : 0;
                tot += v;
            }
            off += pre;
            if (pl < 6) {
                if (k > 0 && off < cap) glist_put(s_list[di], dspill, off, ch[0], parent);
                if (k > 1 && off + 1 < cap) glist_put(s_list[di], dspill, off + 1, ch[1], parent);
            } else if (k > 0) {
                cg_rtri o = inb[parent];                      // normal, colour, texture, index
                if (off < cap) {
                    o.v0 = ch[0].v0; o.v1 = ch[0].v1; o.v2 = ch[0].v2;
                    out[off] = o;
                }
                if (k > 1 && off + 1 < cap) {
                    o.v0 = ch[1].v0; o.v1 = ch[1].v1; o.v2 = ch[1].v2;
                    out[off + 1] = o;
                }
            }
            carry += tot;
            __syncthreads();                 // wsum reuse
        }
        len = min(carry, cap);
        __threadfence_block();
        __syncthreads();                     // the new list (LDS and spill) visible to the workgroup
    }
    if (threadIdx.x == 0) *out_n = len;
}

hipError_t launch_rast_geometry(const cg_rast_params &prm, const cg_rtri *d_room, int n_room,
                                const cg_rtri *d_boxes, int n_boxes, cg_rtri *d_out, cg_rtri *d_scr0,
                                cg_rtri *d_scr1, cg_rtri *d_inb, int cap, int *d_n, cg_vec4 *d_light,
                                hipStream_t st)
{
    hipLaunchKernelGGL(rast_geometry_kernel, dim3(1), dim3(kGeomThreads), 0, st, geom_params(prm), d_room,
                       n_room, d_boxes, n_boxes, d_out, d_scr0, d_scr1, d_inb, cap, d_n, d_light);
    return hipGetLastError();
}

}  // namespace cg

using namespace cg;

extern "C" int cg_rast_prepare(const cg_rast_params *p, const cg_rtri *room, int n_room,
                               const cg_rtri *boxes, int n_boxes, cg_rtri *out, int cap,
                               cg_vec4 *light_out)
{
    if (!p || n_room < 0 || n_boxes < 0 || (n_room && !room) || (n_boxes && !boxes) || cap < 0 ||
        (cap && !out) || p->focal == 0.0f || p->width <= 0 || p->height <= 0)
        return CG_E_INVALID;
    const GeomParams g = geom_params(*p);
    const int n_in = n_room + 7 * n_boxes;
    int n = 0;
    for (int i = 0; i < n_in; ++i) {
        const cg_rtri t = geom_input(g, room, n_room, boxes, i);
        n += clip_dfs(t, g, [&](int k, const cg_rtri &c) {
            if (n + k < cap) out[n + k] = c;
        });
    }
    if (light_out) *light_out = C4(mat4_mul(g.R, geom_light_camera(g)));
    return n;
}
