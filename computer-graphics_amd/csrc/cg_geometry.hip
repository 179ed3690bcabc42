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

// One workgroup, breadth-first -- the reference's own order (clip() walks the
// whole list plane by plane, a split inserting [modified, extra] in place):
// per plane, thread i clips list entry i into 0..2 children, a wave ballot
// scan plus a 16-entry LDS scan gives each child its slot, and the children
// land, in order, in the next list.  Plane 1 reads the input triangles built
// on the fly (room, then each box triangle and its 6 shadow triangles); the
// lists ping-pong between scr0/scr1 (cap entries each) and plane 6 writes out.
// out_n[0] = final count, out_light = rotated camera-space light (:223).
__global__ __launch_bounds__(kGeomThreads) void rast_geometry_kernel(
    GeomParams p, const cg_rtri *__restrict__ room, int n_room, const cg_rtri *__restrict__ boxes,
    int n_boxes, cg_rtri *__restrict__ out, cg_rtri *scr0, cg_rtri *scr1, int cap, int *__restrict__ out_n,
    cg_vec4 *__restrict__ out_light)
{
    __shared__ int wsum[kGeomWaves];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    if (threadIdx.x == 0) *out_light = C4(mat4_mul(p.R, geom_light_camera(p)));
    int len = n_room + 7 * n_boxes;
    const cg_rtri *src = nullptr;
    for (int pl = 1; pl <= 6; ++pl) {
        cg_rtri *dst = pl == 6 ? out : (pl & 1) ? scr0 : scr1;
        int carry = 0;
        for (int base = 0; base < len; base += kGeomThreads) {
            const int i = base + (int)threadIdx.x;
            cg_rtri ch[2];
            int k = 0;
            if (i < len) {
                const cg_rtri t = pl == 1 ? geom_input(p, room, n_room, boxes, i) : src[i];
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
            if (k > 0 && off < cap) dst[off] = ch[0];
            if (k > 1 && off + 1 < cap) dst[off + 1] = ch[1];
            carry += tot;
            __syncthreads();                 // wsum reuse
        }
        len = min(carry, cap);
        src = dst;
        __syncthreads();                     // dst visible to the whole workgroup
    }
    if (threadIdx.x == 0) *out_n = len;
}

hipError_t launch_rast_geometry(const cg_rast_params &prm, const cg_rtri *d_room, int n_room,
                                const cg_rtri *d_boxes, int n_boxes, cg_rtri *d_out, cg_rtri *d_scr0,
                                cg_rtri *d_scr1, int cap, int *d_n, cg_vec4 *d_light, hipStream_t st)
{
    hipLaunchKernelGGL(rast_geometry_kernel, dim3(1), dim3(kGeomThreads), 0, st, geom_params(prm), d_room,
                       n_room, d_boxes, n_boxes, d_out, d_scr0, d_scr1, cap, d_n, d_light);
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
