// cg_rt_brute.hip -- the reference's raytracer loop with no acceleration at
// all, on the GPU: a defect detector for the certificate machinery of the
// product kernels, never a product path.
//
// Every sub-ray of every pixel tests every triangle and sphere of the scene
// (raytracer/Source/skeleton.cpp:263-363 ClosestIntersection), every lit hit
// traces its shadow ray against every triangle and sphere (:366-415
// DirectLight), and each pixel sums its nine sub-rays in the reference's order
// (:120-166) -- no tile masks, no bins, no grid, no lattice, no shared rays.
// The shadow ray stops at the first blocker: the reference's test is
// "closest distance < r_magnitude", i.e. "some accepted hit has distance <
// r_magnitude" (the closest is the minimum over the accepted hits, and a hit
// with det == 0 is never accepted: its u, v are infinite or NaN), so an early
// exit gives the same verdict.  Same numerics contract as the product
// (cg_math.h: GLM association, no FMA, IEEE div/sqrt, the FP64 islands).
//
// Work: for C5 (1920x1080, 1M triangles) ~1.9e13 primary triangle tests plus
// the shadow rays' -- tens of seconds on one MI355X, split into launches of
// kBruteRows rows so no launch runs long.
#include <float.h>
#include <limits.h>
#include <math.h>

#include <algorithm>

#include "cg_internal.h"

namespace cg {

namespace {

constexpr int kBruteRows = 32;     // pixel rows per launch (8,640 waves: enough to hide the scalar loads)

// A triangle's values that do not depend on the lane's ray, formed with the
// reference's own float ops (skeleton.cpp:283-306): e1 = v1 - v0, e2 = v2 - v0,
// s = cameraPos - v0, detT = det(s, e1, e2), and K1 = e1.y*e2.z - e2.y*e1.z --
// the first cofactor det3(-d, e1, e2) forms, the same operands and op for
// every ray.  64 B: one s_load_dwordx16 per triangle in the loops below.
struct alignas(16) BruteTri {
    float e1x, e1y, e1z, e2x;
    float e2y, e2z, v0x, v0y;
    float v0z, K1, sx, sy;
    float sz, detT, pad0, pad1;
};

// One sub-ray's closest hit: tri >= 0 a triangle, tri = -1 - k sphere k, tri =
// INT_MIN none.
struct BruteHit {
    float px, py, pz;
    int idx;
};

// TestModelH.h:24-40 (oracle cgo_sphere_solve_quadratic)
__device__ bool brute_solve_quadratic(float a, float b, float c, float &x0, float &x1)
{
    const float fa = 4 * a;
    const float disc = (b * b) - (fa * c);
    if (disc < 0) return false;
    if (disc == 0) {
        x1 = (float)((-0.5 * (double)b) / (double)a);
        x0 = x1;
    } else {
        const float q = b > 0 ? (float)(-0.5 * (double)(b + sqrtf(disc))) : (float)(-0.5 * (double)(b - sqrtf(disc)));
        x0 = q / a;
        x1 = c / q;
    }
    if (x0 > x1) {
        const float t = x0;
        x0 = x1;
        x1 = t;
    }
    return true;
}

// TestModelH.h:43-66
__device__ bool brute_sphere(const RtSphere &s, vec3 start, vec3 dir, float &t)
{
    float t0, t1;
    const vec3 L = start - v3(s.cx, s.cy, s.cz);
    const float a = dot(dir, dir), b = 2 * dot(dir, L), c = dot(L, L) - s.r2;
    if (!brute_solve_quadratic(a, b, c, t0, t1)) return false;
    if (t0 > t1) {
        const float q = t0;
        t0 = t1;
        t1 = q;
    }
    if (t0 < 0) {
        t0 = t1;
        if (t0 < 0) return false;
    }
    t = t0;
    return true;
}

// Sub-ray k (0..8, i = k / 3 - 1 outer, j = k % 3 - 1 inner) of pixel (u, v):
// skeleton.cpp:126-137.
__device__ vec3 brute_dir(const RtFrame &F, int u, int v, int k)
{
    const vec4 d = mat4_mul(F.R, v4((float)(u - F.W / 2), (float)(v - F.H / 2), F.focal, 1.0f));
    const int i = k / 3 - 1, j = k % 3 - 1;
    return v3(d.x + (0.5f * (float)i), d.y + (0.5f * (float)j), F.focal);
}

__global__ void rt_brute_tri_kernel(RtFrame F, const cg_tri *__restrict__ tris, int n, BruteTri *__restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const cg_tri T = tris[i];
    const vec3 e1 = v3(T.v1.x - T.v0.x, T.v1.y - T.v0.y, T.v1.z - T.v0.z);   // :283
    const vec3 e2 = v3(T.v2.x - T.v0.x, T.v2.y - T.v0.y, T.v2.z - T.v0.z);   // :284
    const vec3 s = v3(F.cam[0] - T.v0.x, F.cam[1] - T.v0.y, F.cam[2] - T.v0.z);   // :296-297
    BruteTri b;
    b.e1x = e1.x; b.e1y = e1.y; b.e1z = e1.z; b.e2x = e2.x;
    b.e2y = e2.y; b.e2z = e2.z; b.v0x = T.v0.x; b.v0y = T.v0.y;
    b.v0z = T.v0.z; b.K1 = e1.y * e2.z - e2.y * e1.z; b.sx = s.x; b.sy = s.y;
    b.sz = s.z; b.detT = det3(s, e1, e2); b.pad0 = 0.f; b.pad1 = 0.f;   // :305-306
    out[i] = b;
}

// det3(-d, e1, e2) (glm determinant, cg_math.h det3) with its first cofactor K1 precomputed:
// (c0.x*K1 - c1.x*(c0.y*c2.z - c2.y*c0.z)) + c2.x*(c0.y*c1.z - c1.y*c0.z), c0 = -d.
__device__ __forceinline__ float brute_det(const BruteTri &b, vec3 nd)
{
    const float a = nd.x * b.K1;
    const float q = b.e1x * (nd.y * b.e2z - b.e2y * nd.z);
    const float c = b.e2x * (nd.y * b.e1z - b.e1y * nd.z);
    return (a - q) + c;
}

// Primary rays: rows row0 .. row0 + rows - 1, one lane per sub-ray, every
// triangle (wave-uniform, scalar loads) then every sphere.
__global__ __launch_bounds__(256) void rt_brute_primary_kernel(RtFrame F, const BruteTri *__restrict__ bt, int n,
                                                             const RtSphere *__restrict__ sph, int row0, int rows,
                                                             BruteHit *__restrict__ hits)
{
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)rows * F.W * 9;
    const bool act = g < total;
    const int k = (int)(g % 9), p = (int)(g / 9);
    const int u = act ? p % F.W : 0, v = act ? row0 + p / F.W : 0;
    const vec3 dir = brute_dir(F, u, v, k);
    const vec3 ndir = -dir, start = v3(F.cam[0], F.cam[1], F.cam[2]);
    const float len = length(dir);
    float best = FLT_MAX;
    int idx = INT_MIN;
    float tb = 0.f;
    for (int i = 0; i < n; ++i) {
        const BruteTri b = bt[i];                                 // wave-uniform: scalar loads
        const float det = brute_det(b, ndir);                     // :289, :306
        const float t = b.detT / det;                             // :305-306
        const float d = t * len;                                  // :307
        if (d < 0.0f || d >= best || d > FLT_MAX) continue;       // :311-313
        const vec3 e1 = v3(b.e1x, b.e1y, b.e1z), e2 = v3(b.e2x, b.e2y, b.e2z), s = v3(b.sx, b.sy, b.sz);
        const float uu = det3(ndir, s, e2) / det, vv = det3(ndir, e1, s) / det;   // :317-321
        if (uu >= 0 && vv >= 0 && (uu + vv) <= 1) {               // :328
            best = d;
            idx = i;
            tb = t;
        }
    }
    vec3 pos = v3(0.f, 0.f, 0.f);
    if (idx >= 0) {                                               // :326 position = start + t * dir
        const vec3 td = dir * tb;
        pos = v3(start.x + td.x, start.y + td.y, start.z + td.z);
    }
    for (int q = 0; q < F.n_sph; ++q) {
        float t;
        if (brute_sphere(sph[q], start, dir, t) && t < best) {
            const vec3 td = dir * t;
            best = t;
            idx = -1 - q;
            pos = v3(start.x + td.x, start.y + td.y, start.z + td.z);
        }
    }
    if (act) hits[g] = BruteHit{pos.x, pos.y, pos.z, best < FLT_MAX ? idx : INT_MIN};
}

// The hit's normal and colour (skeleton.cpp:376-389; TestModelH.h:68-75 for spheres).
__device__ void brute_surface(const cg_tri *__restrict__ tris, const RtSphere *__restrict__ sph, const BruteHit &h,
                              vec4 &normal, vec3 &colour)
{
    if (h.idx >= 0) {
        const cg_tri &T = tris[h.idx];
        normal = v4(T.normal.x, T.normal.y, T.normal.z, T.normal.w);
        colour = v3(T.color.x, T.color.y, T.color.z);
    } else {
        const RtSphere &s = sph[-1 - h.idx];
        const vec3 n3 = normalize(v3(h.px - s.cx, h.py - s.cy, h.pz - s.cz));
        normal = v4(n3.x, n3.y, n3.z, 0.f);
        colour = v3(s.cr, s.cg, s.cb);
    }
}

// r_magnitude (:371): sqrt(pow(r0,2)+pow(r1,2)+pow(r2,2)) in double, narrowed.
__device__ float brute_rmag(vec3 r)
{
    const double a = (double)r.x * (double)r.x, b = (double)r.y * (double)r.y, c = (double)r.z * (double)r.z;
    return (float)sqrt((a + b) + c);
}

// Shadow rays of light l: one lane per sub-ray; blocked[g] = 1 when the
// reference's shadow test (:394-396) darkens it.  Every triangle in index
// order until the whole wave has found a blocker, then every sphere.
__global__ __launch_bounds__(256) void rt_brute_shadow_kernel(RtFrame F, const cg_tri *__restrict__ tris,
                                                            const BruteTri *__restrict__ bt, int n,
                                                            const RtSphere *__restrict__ sph, long long total,
                                                            const BruteHit *__restrict__ hits, int l,
                                                            uint8_t *__restrict__ blocked)
{
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = g < total;
    BruteHit h = act ? hits[g] : BruteHit{0.f, 0.f, 0.f, INT_MIN};
    bool live = h.idx != INT_MIN;
    vec3 o = v3(0.f, 0.f, 0.f), dir = v3(1.f, 0.f, 0.f);
    float rmag = 0.f, len = 1.f;
    if (live) {
        vec4 normal;
        vec3 colour;
        brute_surface(tris, sph, h, normal, colour);
        const RtLight L = F.lights[l];
        dir = v3(L.x - h.px, L.y - h.py, L.z - h.pz);                       // :369, :391
        rmag = brute_rmag(dir);
        const vec4 on = normal * 0.00001f;                                  // :394
        o = v3(h.px + on.x, h.py + on.y, h.pz + on.z);
        len = length(dir);
    }
    const vec3 ndir = -dir;
    bool hit = false;
    for (int i = 0; i < n; ++i) {
        if (__ballot(live && !hit) == 0ull) break;                          // the whole wave decided
        const BruteTri b = bt[i];                                           // uniform: scalar loads
        if (!live || hit) continue;
        const vec3 e1 = v3(b.e1x, b.e1y, b.e1z), e2 = v3(b.e2x, b.e2y, b.e2z);
        const vec3 s = v3(o.x - b.v0x, o.y - b.v0y, o.z - b.v0z);            // :296-297
        const float det = brute_det(b, ndir);
        const float t = det3(s, e1, e2) / det;
        const float d = t * len;
        if (!(d >= 0.0f && d < rmag)) continue;   // a closer accepted hit than the light
        const float uu = det3(ndir, s, e2) / det, vv = det3(ndir, e1, s) / det;
        hit = uu >= 0 && vv >= 0 && (uu + vv) <= 1;
    }
    for (int q = 0; q < F.n_sph && live && !hit; ++q) {
        float t;
        hit = brute_sphere(sph[q], o, dir, t) && t < rmag;
    }
    if (act) blocked[g] = (live && hit) ? 1 : 0;
}

// Each pixel's nine sub-rays in the reference's order (:134-165).
__global__ __launch_bounds__(256) void rt_brute_shade_kernel(RtFrame F, const cg_tri *__restrict__ tris,
                                                           const RtSphere *__restrict__ sph, int rows,
                                                           const BruteHit *__restrict__ hits,
                                                           const uint8_t *__restrict__ blocked, long long total,
                                                           uint32_t *__restrict__ out)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= rows * F.W) return;
    const vec3 ind = v3(F.indirect, F.indirect, F.indirect);
    vec3 pc = v3(0.f, 0.f, 0.f);
    bool valid = false;
    for (int k = 0; k < 9; ++k) {
        const long long g = (long long)p * 9 + k;
        const BruteHit h = hits[g];
        if (h.idx == INT_MIN) continue;
        valid = true;
        vec4 normal;
        vec3 oc;
        brute_surface(tris, sph, h, normal, oc);
        for (int l = 0; l < F.n_lights; ++l) {
            const RtLight L = F.lights[l];
            const vec3 r = v3(L.x - h.px, L.y - h.py, L.z - h.pz);
            vec3 dl = v3(0.f, 0.f, 0.f);
            if (!blocked[(long long)l * total + g]) {
                const float rmag = brute_rmag(r);
                const vec3 nd = normalize(r);                                           // :400
                float a = dot(nd, xyz(normal));                                         // :403
                const float b = (float)(4 * M_PI);                                      // :404
                const float area = (float)((double)b * ((double)rmag * (double)rmag)); // :406
                if (a <= 0) a = 0.f;                                                    // :409
                dl = ((oc * v3(L.r, L.g, L.b)) * a) / area;                              // :412
            }
            pc = pc + dl;
        }
        pc = pc + oc * ind;                                                             // :156
    }
    out[p] = valid ? put_pixel(pc / 9.0f) : put_pixel(v3(0.f, 0.f, 0.f));              // :160-165
}

}  // namespace

// Rows row0 .. row0 + rows - 1 of the frame F (rows x W pixels into d_out),
// brute force, synchronously on st (scratch allocated and freed here).
hipError_t rt_render_brute(const RtFrame &F, const cg_tri *d_tris, int n, const RtSphere *d_sph, int row0, int rows,
                           uint32_t *d_out, hipStream_t st)
{
    const long long per = (long long)kBruteRows * F.W * 9;
    BruteHit *hits = nullptr;
    uint8_t *blocked = nullptr;
    BruteTri *bt = nullptr;
    hipError_t e = hipMalloc(&hits, per * sizeof(BruteHit));
    if (e == hipSuccess) e = hipMalloc(&blocked, per * (size_t)std::max(F.n_lights, 1));
    if (e == hipSuccess) e = hipMalloc(&bt, (size_t)std::max(n, 1) * sizeof(BruteTri));
    if (e == hipSuccess && n > 0)
        hipLaunchKernelGGL(rt_brute_tri_kernel, dim3((n + 255) / 256), dim3(256), 0, st, F, d_tris, n, bt);
    for (int r = row0; e == hipSuccess && r < row0 + rows; r += kBruteRows) {
        const int nr = std::min(kBruteRows, row0 + rows - r);
        const long long total = (long long)nr * F.W * 9;
        const int blocks = (int)((total + 255) / 256);
        hipLaunchKernelGGL(rt_brute_primary_kernel, dim3(blocks), dim3(256), 0, st, F, (const BruteTri *)bt, n, d_sph, r,
                           nr, hits);
        for (int l = 0; l < F.n_lights; ++l)
            hipLaunchKernelGGL(rt_brute_shadow_kernel, dim3(blocks), dim3(256), 0, st, F, d_tris, (const BruteTri *)bt, n,
                               d_sph, total, (const BruteHit *)hits, l, blocked + (size_t)l * total);
        hipLaunchKernelGGL(rt_brute_shade_kernel, dim3((nr * F.W + 255) / 256), dim3(256), 0, st, F, d_tris, d_sph, nr,
                           (const BruteHit *)hits, (const uint8_t *)blocked, total,
                           d_out + (size_t)(r - row0) * F.W);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(st);   // one band at a time: no launch queue of minutes
    }
    if (hits) (void)hipFree(hits);
    if (blocked) (void)hipFree(blocked);
    if (bt) (void)hipFree(bt);
    return e;
}

}  // namespace cg
