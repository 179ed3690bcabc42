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

#include "cg_internal.h"

namespace cg {

// ---------------------------------------------------------------------------
// Per-frame setup: RtTri constants for camera-origin rays (skeleton.cpp:279-306).
__global__ void rt_prepare_kernel(const cg_tri *__restrict__ tris, int n, float cx, float cy,
                                  float cz, float cw, RtTri *__restrict__ out,
                                  RtShade *__restrict__ shade)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    cg_tri T = tris[i];
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
    out[i] = r;
    RtShade sh;
    sh.nx = T.normal.x; sh.ny = T.normal.y; sh.nz = T.normal.z; sh.nw = T.normal.w;
    sh.cr = T.color.x; sh.cg = T.color.y; sh.cb = T.color.z; sh.pad = 0.f;
    shade[i] = sh;
}

// ---------------------------------------------------------------------------
// Sphere::intersect + solveQuadratic (raytracer/Source/TestModelH.h:24-66).
__device__ __forceinline__ bool sphere_intersect(const RtSphere &S, vec3 start, vec3 dir, float &t)
{
    vec3 L = start - v3(S.cx, S.cy, S.cz);            // :48
    float a = dot(dir, dir);                           // :49
    float b = 2 * dot(dir, L);                         // :50
    float c = dot(L, L) - S.r2;                        // :51
    float x0, x1;
    float disc = (b * b) - ((4 * a) * c);              // :27
    if (disc < 0) return false;                        // :28
    if (disc == 0) {                                   // :29, FP64 divide
        x1 = (float)((-0.5 * (double)b) / (double)a);
        x0 = x1;
    } else {                                           // :31-35
        float q;
        if (b > 0) q = (float)(-0.5 * (double)(b + sqrtf(disc)));
        else q = (float)(-0.5 * (double)(b - sqrtf(disc)));
        x0 = q / a;
        x1 = c / q;
    }
    if (x0 > x1) { float tmp = x0; x0 = x1; x1 = tmp; }   // :37 (and :54)
    if (x0 < 0) {                                      // :57-61
        x0 = x1;
        if (x0 < 0) return false;
    }
    t = x0;
    return true;
}

// ClosestIntersection for camera-origin rays (skeleton.cpp:263-363).
// Returns best index: >= 0 triangle, -1 - k sphere k, INT_MIN no hit; t out.
__device__ __forceinline__ int closest_primary(const RtFrame &F, const RtTri *__restrict__ tc,
                                               const RtSphere *__restrict__ sph, vec3 d,
                                               float &best_t)
{
    const float bound = FLT_MAX;
    float best = bound;
    int bi = INT_MIN;
    float bt = 0.f;
    vec3 nd = -d;
    float len = length(d);                                   // :307
    for (int k = 0; k < F.n_tris; ++k) {
        const RtTri c = tc[k];
        float Q2 = nd.y * c.e2z - c.e2y * nd.z;
        float Q1 = nd.y * c.e1z - c.e1y * nd.z;
        float det = (nd.x * c.K1 - c.e1x * Q2) + c.e2x * Q1;  // det(-d, e1, e2) :289
        float t = c.detT / det;                               // :306
        float distance = t * len;                             // :307
        if (distance < 0.0f) continue;                        // :311
        if (distance >= best || distance > bound) continue;   // :313
        float Q3 = nd.y * c.sz - c.sy * nd.z;
        float detU = (nd.x * c.K2 - c.sx * Q2) + c.e2x * Q3;  // det(-d, s, e2) :317
        float detV = (nd.x * c.K3 - c.e1x * Q3) + c.sx * Q1;  // det(-d, e1, s) :320
        float u = detU / det;
        float v = detV / det;
        if ((u >= 0) && (v >= 0) && ((u + v) <= 1)) {        // :328-335
            best = distance;
            bt = t;
            bi = k;
        }
    }
    vec3 s3 = v3(F.cam[0], F.cam[1], F.cam[2]);
    for (int k = 0; k < F.n_sph; ++k) {                       // :341-355
        float t;
        if (sphere_intersect(sph[k], s3, d, t)) {
            if (t < best) {
                best = t;
                bt = t;
                bi = -1 - k;
            }
        }
    }
    best_t = bt;
    return best < bound ? bi : INT_MIN;                       // :357
}

// Shadow test of DirectLight (skeleton.cpp:394-398): ClosestIntersection
// from `start` towards the light, shadowed iff its distance < rmag.  The
// closest distance is < rmag iff SOME accepted hit is, so this is an
// any-hit search bounded by rmag with an early exit; triangles are tested
// with the reference's float ops (their acceptance does not depend on the
// running minimum, only on `distance < rmag` here).
__device__ __forceinline__ bool shadowed(const RtFrame &F, const RtTri *__restrict__ tc,
                                         const RtSphere *__restrict__ sph, vec3 start, vec3 d,
                                         float rmag)
{
    const float bound = FLT_MAX;
    vec3 nd = -d;
    float len = length(d);
    for (int k = 0; k < F.n_tris; ++k) {
        const RtTri c = tc[k];
        float sx = start.x - c.v0x, sy = start.y - c.v0y, sz = start.z - c.v0z;   // :296
        float Q2 = nd.y * c.e2z - c.e2y * nd.z;
        float Q1 = nd.y * c.e1z - c.e1y * nd.z;
        float det = (nd.x * c.K1 - c.e1x * Q2) + c.e2x * Q1;
        float K2 = sy * c.e2z - c.e2y * sz;
        float K4 = sy * c.e1z - c.e1y * sz;
        float detT = (sx * c.K1 - c.e1x * K2) + c.e2x * K4;                    // det(s, e1, e2)
        float t = detT / det;
        float distance = t * len;
        if (distance < 0.0f) continue;
        if (distance >= rmag || distance > bound) continue;
        float Q3 = nd.y * sz - sy * nd.z;
        float K3 = c.e1y * sz - sy * c.e1z;
        float detU = (nd.x * K2 - sx * Q2) + c.e2x * Q3;
        float detV = (nd.x * K3 - c.e1x * Q3) + sx * Q1;
        float u = detU / det;
        float v = detV / det;
        if ((u >= 0) && (v >= 0) && ((u + v) <= 1)) return true;
    }
    for (int k = 0; k < F.n_sph; ++k) {
        float t;
        if (sphere_intersect(sph[k], start, d, t) && t < rmag) return true;
    }
    return false;
}

// DirectLight (skeleton.cpp:366-415) for a hit at `pos` on object `bi`.
__device__ __forceinline__ vec3 direct_light(const RtFrame &F, const RtTri *__restrict__ tc,
                                             const RtShade *__restrict__ shade,
                                             const RtSphere *__restrict__ sph, int bi, vec3 pos,
                                             vec3 objColor, int l)
{
    vec3 lp = v3(F.lpos[l][0], F.lpos[l][1], F.lpos[l][2]);
    vec3 r = lp - pos;                                                   // :370
    double r0 = (double)r.x * (double)r.x, r1 = (double)r.y * (double)r.y,
           r2 = (double)r.z * (double)r.z;
    float rmag = (float)sqrt((r0 + r1) + r2);                            // :371
    vec3 normal;
    if (bi >= 0) {                                                       // :377-380
        RtShade s = shade[bi];
        normal = v3(s.nx, s.ny, s.nz);
    } else {                                                             // :381-387
        const RtSphere S = sph[-1 - bi];
        normal = normalize(pos - v3(S.cx, S.cy, S.cz));
    }
    vec3 origin = pos + normal * 0.00001f;                              // :394
    if (shadowed(F, tc, sph, origin, r, rmag)) return v3(0.0f, 0.0f, 0.0f);  // :394-398
    vec3 nd = normalize(r);                                              // :400
    float a = dot(nd, normal);                                           // :403
    const float b = (float)(4 * M_PI);                                   // :404
    float area = (float)((double)b * ((double)rmag * (double)rmag));     // :406
    if (a <= 0) a = 0.f;                                                 // :409
    vec3 lc = v3(F.lcol[l][0], F.lcol[l][1], F.lcol[l][2]);
    return ((objColor * lc) * a) / area;                                 // :412
}

__device__ __forceinline__ int shard_row(const RtFrame &F, int L)
{
    int k = L / F.stripe_h;
    return (k * F.nranks + F.rank) * F.stripe_h + (L - k * F.stripe_h);
}

// Draw (skeleton.cpp:104-169), one thread per pixel.
__global__ __launch_bounds__(kRtThreads) void rt_pixel_kernel(RtFrame F, const RtTri *__restrict__ tc,
                                                              const RtShade *__restrict__ shade,
                                                              const RtSphere *__restrict__ sph,
                                                              uint32_t *__restrict__ out)
{
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int u = blockIdx.x * kRtTileW + wave * 8 + (lane & 7);
    const int L = blockIdx.y * kRtTileH + (lane >> 3);
    if (u >= F.W || L >= F.rows_out) return;
    const int v = shard_row(F, L);
    uint32_t px = 0u;
    if (v < F.H) {
        vec4 dir = v4((float)(u - F.W / 2), (float)(v - F.H / 2), F.focal, 1.0f);   // :126
        dir = mat4_mul(F.R, dir);                                                    // :128
        vec3 pc = v3(0.0f, 0.0f, 0.0f);
        bool valid = false;
        const vec3 ind = v3(F.indirect, F.indirect, F.indirect);
        for (int i = -1; i <= 1; ++i) {
            for (int j = -1; j <= 1; ++j) {
                const float m = 0.5f;
                vec3 nd = v3(dir.x + (m * (float)i), dir.y + (m * (float)j), F.focal);  // :137
                float t;
                int bi = closest_primary(F, tc, sph, nd, t);                             // :140
                if (bi != INT_MIN) {
                    valid = true;
                    vec3 pos = v3(F.cam[0] + t * nd.x, F.cam[1] + t * nd.y, F.cam[2] + t * nd.z); // :326/:345
                    vec3 oc;
                    if (bi >= 0) {
                        RtShade s = shade[bi];
                        oc = v3(s.cr, s.cg, s.cb);
                    } else {
                        const RtSphere S = sph[-1 - bi];
                        oc = v3(S.cr, S.cg, S.cb);
                    }
                    for (int l = 0; l < F.n_lights; ++l)                                  // :151-153
                        pc = pc + direct_light(F, tc, shade, sph, bi, pos, oc, l);
                    pc = pc + (oc * ind);                                                 // :156
                }
            }
        }
        px = valid ? put_pixel(pc / 9.0f) : put_pixel(v3(0.0f, 0.0f, 0.0f));            // :160-166
    }
    out[(size_t)L * F.W + u] = px;
}

// Reassemble a striped frame after the gather (multi-GPU path).
__global__ void rt_unstripe_kernel(const uint32_t *__restrict__ g, int W, int H, int nranks,
                                   int stripe_h, int rows_per_rank, uint32_t *__restrict__ frame)
{
    int x = blockIdx.x * blockDim.x + threadIdx.x;
    int y = blockIdx.y;
    if (x >= W || y >= H) return;
    int k = y / stripe_h;
    int r = k % nranks;
    int L = (k / nranks) * stripe_h + (y - k * stripe_h);
    frame[(size_t)y * W + x] = g[((size_t)r * rows_per_rank + L) * W + x];
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
    vec3 r = direct_light(F, tc, shade, sph, bi, pos, oc, 0);
    out[i] = cg_vec3{r.x, r.y, r.z};
}

// ---------------------------------------------------------------------------
// Launch helpers (called by the shim).
hipError_t launch_rt_prepare(const cg_tri *d_tris, int n, const float cam[4], RtTri *d_tc,
                             RtShade *d_shade, hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    int threads = 256, blocks = (n + threads - 1) / threads;
    hipLaunchKernelGGL(rt_prepare_kernel, dim3(blocks), dim3(threads), 0, st, d_tris, n, cam[0],
                       cam[1], cam[2], cam[3], d_tc, d_shade);
    return hipGetLastError();
}

hipError_t launch_rt_pixels(const RtFrame &F, const RtTri *d_tc, const RtShade *d_shade,
                            const RtSphere *d_sph, uint32_t *d_out, hipStream_t st)
{
    dim3 grid((F.W + kRtTileW - 1) / kRtTileW, (F.rows_out + kRtTileH - 1) / kRtTileH);
    hipLaunchKernelGGL(rt_pixel_kernel, grid, dim3(kRtThreads), 0, st, F, d_tc, d_shade, d_sph,
                       d_out);
    return hipGetLastError();
}

hipError_t launch_rt_unstripe(const uint32_t *d_g, int W, int H, int nranks, int stripe_h,
                              int rows_per_rank, uint32_t *d_frame, hipStream_t st)
{
    dim3 grid((W + 255) / 256, H);
    hipLaunchKernelGGL(rt_unstripe_kernel, grid, dim3(256), 0, st, d_g, W, H, nranks, stripe_h,
                       rows_per_rank, d_frame);
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
