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

// Device geometry in one launch spread over the chip.  Triangles
// never interact while clipping, and the reference's plane-by-plane list (a
// split inserting [modified, extra] in place, skeleton.cpp:720-1673) is, per
// input triangle in order, that triangle's own plane-by-plane list -- the
// depth-first pre-order clip_dfs emits on the host.
//  rast_clip_kernel     one wave per input triangle (the room, then each box
//                       triangle and its 6 shadow-volume triangles): the
//                       triangle's list through planes 1..6 in LDS, children
//                       placed by a ballot scan, the survivors staged at
//                       stage[i * kGeomMaxLeaves ..] with their count;
//  (the span setup, cg_rast.hip, compacts them: clipped triangle t is the
//  survivor t - pre[i] of the input triangle i whose prefix pre[i] of the
//  counts holds it, so the list is in the reference's order.)
// Every descendant carries its input triangle's normal, colour, texture and
// index (a split's extra triangle copies them, :838-841), so lists hold only
// vertices.  Planes 1-4 and 6 can split (plane 5 never does): at most 32
// survivors per input triangle.

__global__ __launch_bounds__(64) void rast_clip_kernel(GeomParams p, const cg_rtri *__restrict__ room, int n_room,
                                                       const cg_rtri *__restrict__ boxes, int n_boxes,
                                                       cg_rtri *__restrict__ stage, int *__restrict__ counts,
                                                       cg_vec4 *__restrict__ out_light, int *__restrict__ first_tri)
{
    __shared__ float4 s_v[2][kGeomMaxLeaves][3];
    const int i = blockIdx.x, lane = threadIdx.x;
    const unsigned long long lt = (1ull << lane) - 1ull;
    if (i == 0 && lane == 0) {
        *out_light = C4(mat4_mul(p.R, geom_light_camera(p)));
        if (first_tri) *first_tri = 0x7f7f7f7f;   // the span setup's first-fragment minimum: none yet
    }
    const cg_rtri root = geom_input(p, room, n_room, boxes, i);   // uniform over the wave
    int len = 1;
    for (int pl = 1; pl <= 6; ++pl) {
        const int si = pl & 1, di = si ^ 1;
        cg_rtri ch[2];
        int k = 0;
        if (lane < len) {
            cg_rtri t = root;
            if (pl > 1) {
                const float4 a = s_v[si][lane][0], b = s_v[si][lane][1], c = s_v[si][lane][2];
                t.v0 = cg_vec4{a.x, a.y, a.z, a.w};
                t.v1 = cg_vec4{b.x, b.y, b.z, b.w};
                t.v2 = cg_vec4{c.x, c.y, c.z, c.w};
            }
            k = clip_plane(t, pl, p, ch);
        }
        const unsigned long long b0 = __ballot(k & 1), b1 = __ballot(k >> 1);
        const int pre = __popcll(b0 & lt) + 2 * __popcll(b1 & lt);
        __syncthreads();   // the source list of the next plane is overwritten below
#pragma unroll
        for (int c = 0; c < 2; ++c)
            if (c < k) {
                s_v[di][pre + c][0] = make_float4(ch[c].v0.x, ch[c].v0.y, ch[c].v0.z, ch[c].v0.w);
                s_v[di][pre + c][1] = make_float4(ch[c].v1.x, ch[c].v1.y, ch[c].v1.z, ch[c].v1.w);
                s_v[di][pre + c][2] = make_float4(ch[c].v2.x, ch[c].v2.y, ch[c].v2.z, ch[c].v2.w);
            }
        len = __popcll(b0) + 2 * __popcll(b1);
        __syncthreads();
    }
    // plane 6 wrote list 1
    if (lane < len) {
        cg_rtri o = root;
        const float4 a = s_v[1][lane][0], b = s_v[1][lane][1], c = s_v[1][lane][2];
        o.v0 = cg_vec4{a.x, a.y, a.z, a.w};
        o.v1 = cg_vec4{b.x, b.y, b.z, b.w};
        o.v2 = cg_vec4{c.x, c.y, c.z, c.w};
        stage[(size_t)i * kGeomMaxLeaves + lane] = o;
    }
    if (lane == 0) counts[i] = len;
}

// The clip alone: each input triangle's survivors staged at d_stage + 32 i,
// their count at d_counts[i].  The span setup (cg_rast.hip) compacts them
// into d_out in order (offset = sum of the earlier counts) as it reads them.
hipError_t launch_rast_clip(const cg_rast_params &prm, const cg_rtri *d_room, int n_room, const cg_rtri *d_boxes,
                            int n_boxes, cg_rtri *d_stage, int *d_counts, cg_vec4 *d_light, int *d_first,
                            hipStream_t st)
{
    const int n_in = n_room + 7 * n_boxes;
    if (n_in <= 0) return hipSuccess;   // empty scene: the setup finds no triangle
    hipLaunchKernelGGL(rast_clip_kernel, dim3(n_in), dim3(64), 0, st, geom_params(prm), d_room, n_room, d_boxes,
                       n_boxes, d_stage, d_counts, d_light, d_first);
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
