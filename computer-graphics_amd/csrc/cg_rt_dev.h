// cg_rt_dev.h -- raytracer device functions shared by the Cornell-box kernel
// (cg_rt.hip, <= 64 triangles, one certificate mask per wave) and the
// large-scene binned kernels (cg_rt_big.hip).  Every float op follows
// raytracer/Source/skeleton.cpp + GLM 0.9.7.2 association (see cg_math.h).
#pragma once

#include <float.h>

#include "cg_internal.h"

namespace cg {

// Work counters of a counting build (-DCG_WORK_COUNT; scripts/work_counts.py):
// the reference's own per-ray operations the kernels perform, in SURVEY 8d's
// units -- a triangle's t stage, its u, v stage (only when the distance tests
// pass, as in the reference), a sphere test, a ray, a DirectLight -- primary
// and shadow rays apart.  Wave-aggregated atomics into a per-translation-unit
// array (cg_diag_work_counts_*); the product build compiles none of it.
enum WorkKind { W_T_PRI, W_UV_PRI, W_SPH_PRI, W_RAY_PRI, W_T_SH, W_UV_SH, W_SPH_SH, W_RAY_SH, W_DL, W_KINDS };
#ifdef CG_WORK_COUNT
static __device__ unsigned long long g_work[W_KINDS];
__device__ __forceinline__ void cg_work(int k)
{
    const unsigned long long b = __ballot(1);
    if ((int)__lane_id() == __builtin_ctzll(b)) atomicAdd(&g_work[k], (unsigned long long)__popcll(b));
}
#else
__device__ __forceinline__ void cg_work(int) {}
#endif

// RtTri of a triangle for rays from camf, from its per-scene RtGeo: s =
// cameraPos - v0 (skeleton.cpp:296-297, the xyz of rt_tri_const's vec4
// difference), detT, K2, K3 -- bit for bit rt_tri_const's.
__device__ __forceinline__ RtTri rt_tri_frame(const RtGeo &g, const float camf[4])
{
    const vec3 e1 = v3(g.e1x, g.e1y, g.e1z), e2 = v3(g.e2x, g.e2y, g.e2z);
    const vec3 s = v3(camf[0] - g.v0x, camf[1] - g.v0y, camf[2] - g.v0z);
    RtTri r;
    r.e1x = e1.x; r.e1y = e1.y; r.e1z = e1.z;
    r.e2x = e2.x; r.e2y = e2.y; r.e2z = e2.z;
    r.sx = s.x; r.sy = s.y; r.sz = s.z;
    r.detT = det3(s, e1, e2);                                          // :305-306
    r.K1 = g.K1;
    r.K2 = s.y * e2.z - e2.y * s.z;
    r.K3 = e1.y * s.z - s.y * e1.z;
    r.v0x = g.v0x; r.v0y = g.v0y; r.v0z = g.v0z;
    return r;
}


// ---------------------------------------------------------------------------
// Sphere::intersect + solveQuadratic (raytracer/Source/TestModelH.h:24-66).
// The start-dependent terms come from the caller: L = start - centre (:48),
// c = dot(L, L) - r^2 (:51), so a primary ray's camera terms are hoisted.
__device__ __forceinline__ bool sphere_intersect_pre(vec3 L, float c, vec3 dir, float &t)
{
    float a = dot(dir, dir);                           // :49
    float b = 2 * dot(dir, L);                         // :50
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

__device__ __forceinline__ bool sphere_intersect(const RtSphere &S, vec3 start, vec3 dir, float &t)
{
    vec3 L = start - v3(S.cx, S.cy, S.cz);            // :48
    return sphere_intersect_pre(L, dot(L, L) - S.r2, dir, t);   // :51
}

__device__ __forceinline__ vec3 object_colour(const RtShade *__restrict__ shade,
                                              const RtSphere *__restrict__ sph, int bi)
{
    if (bi >= 0) {
        RtShade s = shade[bi];
        return v3(s.cr, s.cg, s.cb);
    }
    const RtSphere S = sph[-1 - bi];
    return v3(S.cr, S.cg, S.cb);
}

__device__ __forceinline__ vec3 hit_normal(const RtShade *__restrict__ shade, const RtSphere *__restrict__ sph,
                                           int bi, vec3 pos)
{
    if (bi >= 0) {                                                       // :377-380
        RtShade s = shade[bi];
        return v3(s.nx, s.ny, s.nz);
    }
    const RtSphere S = sph[-1 - bi];                                     // :381-387
    return normalize(pos - v3(S.cx, S.cy, S.cz));
}

// ---------------------------------------------------------------------------
// Per-wave culling certificate for camera-origin rays.
//
// For a ray d from the camera, the reference's triangle test (skeleton.cpp:
// 289-335) computes, in float, det = det3(-d, e1, e2), detU = det3(-d, s, e2),
// detV = det3(-d, e1, s) with s = cam - v0 -- in exact arithmetic the linear
// forms -d.(e1 x e2), -d.(s x e2), -d.(e1 x s).  A triangle is skipped for the
// whole wave only if, for EVERY d of the wave's bundle (the box spanned by the
// 9 sub-ray directions of its 64 pixels, exact float extremes), the float
// evaluation is certain to reject it: det has a certain sign and t < 0, or
// u < 0, or v < 0, or u + v > 1.  The linear forms are evaluated exactly
// enough in FP64 and each float det3 evaluation is bounded by 16*eps times the
// sum of its |triple products| (gamma_4 suffices), so a skipped triangle
// could never have been accepted: results are bit-identical to testing all.
// Upper bound of sqrt(x), x >= 0, without the FP64 square-root sequence:
// the argument is rounded up into float, v_sqrt_f32 (<= 1 ulp) is widened by
// 2^-20 relative plus 1e-18 absolute (covers float underflow).  Overflow
// gives +inf, which the certificates' isfinite checks turn into "keep".
__device__ __forceinline__ double sqrt_ub(double x)
{
    const float xf = (float)(x * 1.0000019073486328125);   // 1 + 2^-19
    return (double)__builtin_amdgcn_sqrtf(xf) * 1.00000095367431640625 + 1e-18;   // 1 + 2^-20
}

__device__ __forceinline__ void lin_range(double cx, double cy, double hx, double hy, double f,
                                          double X, double Y, double Z, double &lo, double &hi)
{
    // range of -d.(X,Y,Z) over d = (cx +- hx, cy +- hy, f)
    double c = -(cx * X + cy * Y + f * Z);
    double h = hx * fabs(X) + hy * fabs(Y);
    lo = c - h;
    hi = c + h;
}

__device__ __forceinline__ double det3_bound(double Dx, double Dy, double Dz, vec3 a, vec3 b)
{
    // sum of |triple products| of det3(-d, a, b) with |d| <= (Dx, Dy, Dz)
    return Dx * (fabs((double)a.y * b.z) + fabs((double)b.y * a.z)) +
           fabs((double)a.x) * (Dy * fabs((double)b.z) + fabs((double)b.y) * Dz) +
           fabs((double)b.x) * (Dy * fabs((double)a.z) + fabs((double)a.y) * Dz);
}

// The float det's sign is uncertain over the bundle.  A float hit still needs
// u, v >= 0 and u + v <= 1, i.e. detU, detV and W = det - detU - detV (exact
// linear forms over the bundle) all of the float det's sign, up to their
// error bounds.  Away from the triangle's plane detU, detV and W have mixed
// signs (they sum to det ~ 0), so the triangle is rejected when, for each
// sign the float det can take, one of them certainly has the other sign.
// b = detU + detV - det = -W (range [blo, bhi], evaluation error in Eb).
// Float u + v <= 1 with det_f > 0 implies U + V - D <= Ew (first-order
// rounding of the two quotients and their sum, 4 eps to spare).
__device__ __forceinline__ bool sign_free_reject(double dlo, double dhi, double Ed, double ulo, double uhi,
                                                 double Eu, double vlo, double vhi, double Ev, double blo,
                                                 double bhi, double Eb)
{
    const double eps = 5.9604644775390625e-8;   // 2^-24
    const double dmx = fmax(fabs(dlo - Ed), fabs(dhi + Ed));   // max |det_f|
    const double tiny = 1e-20 * dmx;                           // quotients stay clear of -0
    const double umx = fmax(fabs(ulo), fabs(uhi)) + Eu, vmx = fmax(fabs(vlo), fabs(vhi)) + Ev;
    const double Ew = Eb * (1.0 + 4.0 * eps) + 4.0 * eps * (umx + vmx + dmx) + tiny;
    if (dhi + Ed > 0.0 && !((uhi + Eu < -tiny) || (vhi + Ev < -tiny) || (blo > Ew))) return false;
    if (dlo - Ed < 0.0 && !((ulo - Eu > tiny) || (vlo - Ev > tiny) || (bhi < -Ew))) return false;
    return true;
}

// u + v > 1 certain (sg = sign of det, |det| in [dmin, dmax], b = detU +
// detV - det in [blo, bhi] +- Eb, X >= |detU| + |detV|): b/det > 4 eps
// (X/dmin + 1), multiplied out by dmin * dmax > 0 so no FP64 divide sits on
// the certificate's dependency chain; the 2^-40 factor covers the FP64
// rounding of both sides.
__device__ __forceinline__ bool uv_sum_reject(int sg, double blo, double bhi, double Eb, double X, double dmin,
                                              double dmax)
{
    const double eps = 5.9604644775390625e-8;   // 2^-24
    const double num = sg > 0 ? blo - Eb : -(bhi + Eb);
    return num > 0.0 && num * dmin > (4.0 * eps) * (X + dmin) * dmax * (1.0 + 0x1p-40);
}

// The float det's range over a bundle (cull_primary): [dlo - Ed, dhi + Ed].
struct PrimDet {
    double dlo, dhi, Ed;   // det
    double ulo, uhi, Eu;   // detU
    double vlo, vhi, Ev;   // detV
    double blo, bhi, Eb;   // detU + detV - det
};

__device__ static bool cull_primary(const RtTri &c, float x0, float x1, float y0, float y1, float f,
                                    PrimDet *pd = nullptr)
{
    const double eps = 5.9604644775390625e-8;   // 2^-24
    const double g = 16.0 * eps;
    vec3 e1 = v3(c.e1x, c.e1y, c.e1z), e2 = v3(c.e2x, c.e2y, c.e2z), s = v3(c.sx, c.sy, c.sz);
    // N = e1 x e2, A = s x e2, B = e1 x s (float inputs: products exact in FP64)
    double Nx = (double)e1.y * e2.z - (double)e2.y * e1.z, Ny = (double)e1.z * e2.x - (double)e2.z * e1.x,
           Nz = (double)e1.x * e2.y - (double)e2.x * e1.y;
    double Ax = (double)s.y * e2.z - (double)e2.y * s.z, Ay = (double)s.z * e2.x - (double)e2.z * s.x,
           Az = (double)s.x * e2.y - (double)e2.x * s.y;
    double Bx = (double)e1.y * s.z - (double)s.y * e1.z, By = (double)e1.z * s.x - (double)s.z * e1.x,
           Bz = (double)e1.x * s.y - (double)s.x * e1.y;
    double cx = 0.5 * ((double)x0 + x1), cy = 0.5 * ((double)y0 + y1);
    double hx = 0.5 * ((double)x1 - x0), hy = 0.5 * ((double)y1 - y0), fz = f;
    double Dx = fmax(fabs((double)x0), fabs((double)x1)), Dy = fmax(fabs((double)y0), fabs((double)y1)),
           Dz = fabs(fz);
    double dlo, dhi, ulo, uhi, vlo, vhi, blo, bhi;
    lin_range(cx, cy, hx, hy, fz, Nx, Ny, Nz, dlo, dhi);
    lin_range(cx, cy, hx, hy, fz, Ax, Ay, Az, ulo, uhi);
    lin_range(cx, cy, hx, hy, fz, Bx, By, Bz, vlo, vhi);
    lin_range(cx, cy, hx, hy, fz, Ax + Bx - Nx, Ay + By - Ny, Az + Bz - Nz, blo, bhi);
    double Ed = g * det3_bound(Dx, Dy, Dz, e1, e2) + 1e-12 * (fabs(dlo) + fabs(dhi));
    double Eu = g * det3_bound(Dx, Dy, Dz, s, e2) + 1e-12 * (fabs(ulo) + fabs(uhi));
    double Ev = g * det3_bound(Dx, Dy, Dz, e1, s) + 1e-12 * (fabs(vlo) + fabs(vhi));
    double Eb = Ed + Eu + Ev + 1e-12 * (fabs(blo) + fabs(bhi));
    if (pd) *pd = PrimDet{dlo, dhi, Ed, ulo, uhi, Eu, vlo, vhi, Ev, blo, bhi, Eb};
    if (!(isfinite(dlo) && isfinite(dhi) && isfinite(Ed + Eu + Ev + Eb) && isfinite(ulo + uhi + vlo + vhi + blo + bhi)))
        return false;
    int sg;
    if (dlo - Ed > 0) sg = 1;
    else if (dhi + Ed < 0) sg = -1;
    else return sign_free_reject(dlo, dhi, Ed, ulo, uhi, Eu, vlo, vhi, Ev, blo, bhi, Eb);   // det may vanish
    const double dmin = sg > 0 ? dlo - Ed : -(dhi + Ed);  // |det| >= dmin > 0
    const double dmax = sg > 0 ? dhi + Ed : -(dlo - Ed);
    // t = detT/det < 0 (and not underflowing to -0): distance < 0 rejects (:311)
    double dT = c.detT;
    if (dT != 0.0 && ((dT > 0) != (sg > 0)) && fabs(dT) > 1e-20 * dmax) return true;
    // u < 0 or v < 0 (:328)
    // (the quotient must not underflow to -0, which would pass u >= 0)
    const double tiny = 1e-20 * dmax;
    if (sg > 0 ? (uhi + Eu < -tiny) : (ulo - Eu > tiny)) return true;
    if (sg > 0 ? (vhi + Ev < -tiny) : (vlo - Ev > tiny)) return true;
    // u + v > 1 after float rounding of u, v and their sum: certain when
    // (U + V - 1) > 4 eps (|U| + |V| + 1), U = detU/det, V = detV/det
    if (uv_sum_reject(sg, blo, bhi, Eb, fmax(fabs(ulo), fabs(uhi)) + Eu + fmax(fabs(vlo), fabs(vhi)) + Ev,
                      dmin, dmax))
        return true;
    return false;
}

// Box of the positions (:326) of every hit a triangle can give to the camera
// rays d = (x, y, f), x in [x0, x1], y in [y0, y1] (cull_primary's bundle),
// from the float det's range pd: t = fl(detT / det) lies in
// [|detT| / dmax, |detT| / dmin] (widened by 2^-20; accepted hits have t >= 0
// and t of det's sign) when det's sign is certain, and position = fl(cam +
// fl(t d)) is widened by 2^-20 (|cam| + |t d|) per component for its two
// roundings.  Returns false (unbounded) when det's sign is uncertain.
// The box is then clipped to the triangle's own box: an accepted hit has float
// u, v >= 0 and u + v <= 1, so the exact plane point X has barycentrics >=
// -sig and sum <= 1 + sig with sig = 2 (Ed + Eu + Ev) / dmin + 2^-21 (PrimDet's
// error bounds), i.e. X lies in the box of (v0, v0 + e1, v0 + e2) widened by
// sig (|e1| + |e2|) per component; and the float position differs from X by
// the relative error of t (ET / |detT| + Ed / dmin + 2^-22, ET = the float
// detT's error bound) times |t d| plus its own two roundings.  This makes the
// box of a hit on an axis-aligned wall flat instead of the t-range's slab.
__device__ static bool primary_hit_box(const RtTri &c, const PrimDet &pd, const float cam[4], float x0, float x1,
                                       float y0, float y1, float f, float lo[3], float hi[3],
                                       const cg_tri *T = nullptr)
{
    double dmin, dmax;
    if (pd.dlo - pd.Ed > 0) {
        dmin = pd.dlo - pd.Ed;
        dmax = pd.dhi + pd.Ed;
    } else if (pd.dhi + pd.Ed < 0) {
        dmin = -(pd.dhi + pd.Ed);
        dmax = -(pd.dlo - pd.Ed);
    } else {
        return false;
    }
    const double aT = fabs((double)c.detT);
    double tlo = aT / dmax * (1.0 - 0x1p-20);
    const double thi = aT / dmin * (1.0 + 0x1p-20);
    if (tlo < 0x1p-100) tlo = 0.0;   // t may round to 0: the box then contains cam
    if (!(isfinite(thi) && thi < 1e30)) return false;
    const double dl[3] = {(double)x0, (double)y0, (double)f}, dh[3] = {(double)x1, (double)y1, (double)f};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double a = tlo * dl[k], b = tlo * dh[k], e = thi * dl[k], g = thi * dh[k];
        const double mn = fmin(fmin(a, b), fmin(e, g)), mx = fmax(fmax(a, b), fmax(e, g));
        const double w = 0x1p-20 * (fabs((double)cam[k]) + fmax(fabs(mn), fabs(mx))) + 1e-30;
        lo[k] = (float)((cam[k] + mn) - w);
        hi[k] = (float)((cam[k] + mx) + w);
    }
    if (T) {
        const double eps = 5.9604644775390625e-8;   // 2^-24
        const vec3 e1 = v3(c.e1x, c.e1y, c.e1z), e2 = v3(c.e2x, c.e2y, c.e2z);
        const double ET = 16.0 * eps * det3_bound(fabs((double)c.sx), fabs((double)c.sy), fabs((double)c.sz), e1, e2);
        const double aT = fabs((double)c.detT);
        const double sig = 2.0 * (pd.Ed + pd.Eu + pd.Ev) / dmin + 0x1p-21;
        const double trel = ET / aT + pd.Ed / dmin + 0x1p-22;
        if (!(aT > 0.0 && isfinite(sig) && isfinite(trel) && sig < 1e-3 && trel < 1e-3)) return true;
        const double v0[3] = {(double)T->v0.x, (double)T->v0.y, (double)T->v0.z};
        const double a1[3] = {(double)e1.x, (double)e1.y, (double)e1.z}, a2[3] = {(double)e2.x, (double)e2.y, (double)e2.z};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double p1 = v0[k] + a1[k], p2 = v0[k] + a2[k];
            const double td = thi * fmax(fabs(dl[k]), fabs(dh[k]));
            const double m = sig * (fabs(a1[k]) + fabs(a2[k])) + trel * td + 0x1p-21 * (fabs((double)cam[k]) + td) +
                             0x1p-40 * (fabs(v0[k]) + fabs(a1[k]) + fabs(a2[k])) + 1e-30;
            const float tl = (float)(fmin(v0[k], fmin(p1, p2)) - m), th = (float)(fmax(v0[k], fmax(p1, p2)) + m);
            lo[k] = fmaxf(lo[k], tl);
            hi[k] = fminf(hi[k], th);
        }
    }
    return true;
}

// Sphere::intersect (TestModelH.h:43-66) certainly misses every camera ray of
// the bundle: the float discriminant (:27) is negative.  With L = cam - centre,
// a = d.d, b = 2 d.L and c_f = fl(L.L - r^2) > 0 (camera outside), the float
// evaluation of b^2 - 4 a c_f is < 0 when (max|d.L| + 4 eps sum|d_i L_i|)^2 <
// min(d.d) c_f (1 - 2^-18): a_f >= d.d (1 - 3 eps), |b_f| <= 2 (|d.L| + 3 eps
// sum|d_i L_i|)(1 + eps), and the three rounded products / difference cost
// < 2^-18 relative.  max |d.L| over the box is at a corner; min d.d at the
// point of the box nearest the origin.
__device__ static bool sphere_surely_missed(const RtSphere &S, const float cam[4], float x0, float x1, float y0,
                                            float y1, float f)
{
    const vec3 L = v3(cam[0], cam[1], cam[2]) - v3(S.cx, S.cy, S.cz);   // :48 (float, as the kernels form it)
    const float cf = dot(L, L) - S.r2;                                   // :51
    if (!(cf > 0.0f)) return false;
    double mdl = 0.0, msum = 0.0;
    const double xs[2] = {(double)x0, (double)x1}, ys[2] = {(double)y0, (double)y1};
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const double dL = xs[i] * L.x + ys[j] * L.y + (double)f * L.z;
            mdl = fmax(mdl, fabs(dL));
            msum = fmax(msum, fabs(xs[i] * L.x) + fabs(ys[j] * L.y) + fabs((double)f * L.z));
        }
    const double nx = x0 > 0 ? (double)x0 : (x1 < 0 ? (double)x1 : 0.0);
    const double ny = y0 > 0 ? (double)y0 : (y1 < 0 ? (double)y1 : 0.0);
    const double dd = nx * nx + ny * ny + (double)f * f;
    const double U = mdl * (1.0 + 1e-12) + 4.0 * 5.9604644775390625e-8 * msum;
    return isfinite(U) && U * U < dd * (double)cf * (1.0 - 0x1p-18);
}

// The float t = fl(detT / det) of every ray of the bundle lies in [tlo, thi]
// (det's sign certain, both >= 0 as for primary_hit_box); false otherwise.
__device__ __forceinline__ bool primary_t_range(const RtTri &c, const PrimDet &pd, double &tlo, double &thi)
{
    double dmin, dmax;
    if (pd.dlo - pd.Ed > 0) {
        dmin = pd.dlo - pd.Ed;
        dmax = pd.dhi + pd.Ed;
    } else if (pd.dhi + pd.Ed < 0) {
        dmin = -(pd.dhi + pd.Ed);
        dmax = -(pd.dlo - pd.Ed);
    } else {
        return false;
    }
    const double aT = fabs((double)c.detT);
    tlo = aT / dmax * (1.0 - 0x1p-20);
    thi = aT / dmin * (1.0 + 0x1p-20);
    return isfinite(thi);
}

// Every ray of the bundle certainly passes the reference's acceptance tests
// for this triangle except the running-best comparison (:311, :328-335): det's
// sign is certain, detT has that sign (t > 0), detU and detV have it or vanish
// (u, v >= 0 after rounding, including -0), and u + v - 1 = b / det <
// -2^-20, so fl(fl(u) + fl(v)) <= 1 (three roundings of 2^-24 each).
__device__ __forceinline__ bool primary_covers(const RtTri &c, const PrimDet &pd)
{
    const double dT = c.detT;
    if (pd.dlo - pd.Ed > 0) {
        const double dmax = pd.dhi + pd.Ed;
        return dT > 0 && pd.ulo - pd.Eu >= 0 && pd.vlo - pd.Ev >= 0 && pd.bhi + pd.Eb < -0x1p-20 * dmax;
    }
    if (pd.dhi + pd.Ed < 0) {
        const double dmax = -(pd.dlo - pd.Ed);
        return dT < 0 && pd.uhi + pd.Eu <= 0 && pd.vhi + pd.Ev <= 0 && pd.blo - pd.Eb > 0x1p-20 * dmax;
    }
    return false;
}

// The shadow ray of a hit ON triangle k never hits k itself (:394-395): it
// starts at S = pos + n 1e-5f, off k's plane on the side of k's stored normal
// n, and the light lies on the same side.  With N = e1 x e2 (exact), X the
// exact plane point of the ray (|pos - X| <= Delta: t's relative error times
// |t d| plus two roundings, as in primary_hit_box), (S - v0).N =
// 1e-5f (n.N) + (pos - X).N + roundings, and the float det3 (s, e1, e2) adds
// at most 16 eps sum|triple products|: its sign is that of n.N when
// 1e-5 |n.N| exceeds that noise (each term is an upper bound; 5 % slack).  det = -d.N with d = L - pos:
// -(L - v0).N up to (Delta + rounding of d) |N| + its det3 error.  Opposite
// certain signs give t < 0 (|t| far from underflow): rejected at :311, for
// every hit position in the box [blo, bhi] of hits on k.  A light set (every
// light within rho of Lp) widens d by rho per component and moves -(L - v0).N
// by at most rho |N|.
__device__ static bool own_shadow_rejects(const cg_tri &T, const RtTri &c, const PrimDet &pd, double thi,
                                          const float cam[4], float x0, float x1, float y0, float y1, float f,
                                          const double Lp[3], double rho_l, const float blo[3],
                                          const float bhi[3])
{
    const double eps = 5.9604644775390625e-8;   // 2^-24
    double dmin;
    if (pd.dlo - pd.Ed > 0) dmin = pd.dlo - pd.Ed;
    else if (pd.dhi + pd.Ed < 0) dmin = -(pd.dhi + pd.Ed);
    else return false;
    const vec3 e1 = v3(c.e1x, c.e1y, c.e1z), e2 = v3(c.e2x, c.e2y, c.e2z);
    const double N[3] = {(double)e1.y * e2.z - (double)e2.y * e1.z, (double)e1.z * e2.x - (double)e2.z * e1.x,
                         (double)e1.x * e2.y - (double)e2.x * e1.y};
    const double Nn = sqrt(N[0] * N[0] + N[1] * N[1] + N[2] * N[2]) * (1.0 + 1e-12);
    const double aT = fabs((double)c.detT);
    const double ET = 16.0 * eps * det3_bound(fabs((double)c.sx), fabs((double)c.sy), fabs((double)c.sz), e1, e2);
    const double trel = ET / aT + pd.Ed / dmin + 0x1p-22;
    if (!(aT > 0.0 && isfinite(trel) && isfinite(thi))) return false;
    const double dl[3] = {(double)x0, (double)y0, (double)f}, dh[3] = {(double)x1, (double)y1, (double)f};
    const double v0[3] = {(double)T.v0.x, (double)T.v0.y, (double)T.v0.z};
    const double n[3] = {(double)T.normal.x, (double)T.normal.y, (double)T.normal.z};
    const double o = (double)0.00001f;
    double D2 = 0.0, rho2 = 0.0, S2 = 0.0, d2 = 0.0, Sa[3], da[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double td = thi * fmax(fabs(dl[k]), fabs(dh[k]));
        const double dk = trel * td + 0x1p-22 * (fabs((double)cam[k]) + td);
        D2 += dk * dk;
        const double pmax = fmax(fabs((double)blo[k]), fabs((double)bhi[k]));
        const double rk = 0x1p-23 * (pmax + o * fabs(n[k]) + 1.0) ;
        rho2 += rk * rk;
        Sa[k] = fmax(fabs((double)blo[k] - v0[k]), fabs((double)bhi[k] - v0[k])) + o * fabs(n[k]) + rk;
        S2 += Sa[k] * Sa[k];
        da[k] = fmax(fabs(Lp[k] - (double)blo[k]), fabs(Lp[k] - (double)bhi[k])) + rho_l;
        d2 += da[k] * da[k];
    }
    const double Delta = sqrt(D2), rho = sqrt(rho2);
    const double nN = n[0] * N[0] + n[1] * N[1] + n[2] * N[2];
    const double noiseT = (Delta + rho + eps * sqrt(S2)) * Nn + 16.0 * eps * det3_bound(Sa[0], Sa[1], Sa[2], e1, e2);
    if (!(o * fabs(nN) * (1.0 - 1e-9) > 1.05 * noiseT)) return false;   // every term above is an upper bound
    const double aN = (Lp[0] - v0[0]) * N[0] + (Lp[1] - v0[1]) * N[1] + (Lp[2] - v0[2]) * N[2];
    const double noiseD = (Delta + eps * sqrt(d2)) * Nn + 16.0 * eps * det3_bound(da[0], da[1], da[2], e1, e2) +
                          1e-12 * fabs(aN);
    if (!(fabs(aN) > 1.05 * noiseD + rho_l * Nn * (1.0 + 1e-9))) return false;
    return (nN > 0) != (-aN > 0);   // detT and det of opposite signs: t < 0
}

// Box of the positions of sphere hits (:345): a hit's float t carries an
// absolute error below sqrt(20 eps) |L| / |d| near tangency (the root of a
// discriminant perturbed by ~10 eps b^2), so the float position lies within
// 1.1e-3 |L| of the sphere; the box is widened by 4e-3 |L|.
// Clipped to the bundle's frustum: the exact hit X = cam + t d lies on the
// sphere, so |X - cam| is within r of |L| and the float t (1.1e-3 |L| / |d|
// from X's t, as above) lies in [(|L| - r - 4e-3 |L|) / |d|max,
// (|L| + r + 4e-3 |L|) / |d|min]; the position fl(cam + fl(t d)) then lies in
// cam + [t] x [d] (widened for its two roundings).
__device__ static void sphere_hit_box(const RtSphere &S, const float cam[4], float x0, float x1, float y0, float y1,
                                      float f, float lo[3], float hi[3])
{
    const double Lx = (double)cam[0] - S.cx, Ly = (double)cam[1] - S.cy, Lz = (double)cam[2] - S.cz;
    const double Ln = sqrt(Lx * Lx + Ly * Ly + Lz * Lz), r = sqrt((double)S.r2) * (1.0 + 1e-6);
    const double w = r + 4e-3 * Ln + 1e-6;
    const double C[3] = {(double)S.cx, (double)S.cy, (double)S.cz};
    const double dl[3] = {(double)x0, (double)y0, (double)f}, dh[3] = {(double)x1, (double)y1, (double)f};
    const double nx = x0 > 0 ? (double)x0 : (x1 < 0 ? (double)x1 : 0.0);
    const double ny = y0 > 0 ? (double)y0 : (y1 < 0 ? (double)y1 : 0.0);
    const double dmin = sqrt(nx * nx + ny * ny + (double)f * f) * (1.0 - 1e-12);
    const double ax = fmax(fabs((double)x0), fabs((double)x1)), ay = fmax(fabs((double)y0), fabs((double)y1));
    const double dmax = sqrt(ax * ax + ay * ay + (double)f * f) * (1.0 + 1e-12);
    const double tlo = fmax(0.0, (Ln - w) / dmax), thi = (Ln + w) / dmin;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double a = tlo * dl[k], b = tlo * dh[k], e = thi * dl[k], g = thi * dh[k];
        const double mn = fmin(fmin(a, b), fmin(e, g)), mx = fmax(fmax(a, b), fmax(e, g));
        const double m = 0x1p-20 * (fabs(C[k]) + w + fabs((double)cam[k]) + fmax(fabs(mn), fabs(mx)));
        const double blo = fmax(C[k] - w, cam[k] + mn) - m, bhi = fmin(C[k] + w, cam[k] + mx) + m;
        lo[k] = fminf(lo[k], (float)blo);
        hi[k] = fmaxf(hi[k], (float)bhi);
    }
}

// The sphere certainly blocks none of the shadow rays (:394-395) cast from hit
// positions in the box [lo, hi] towards the light at Lp: Sphere::intersect's
// float discriminant (TestModelH.h:27) is negative for all of them.  Exactly,
// disc / 4a = r^2 - dist(C, line)^2 for the line through the start S with
// direction d = Lp - pos; that line runs within ~3e-5 of the line through Lp
// and pos (S = pos + n 1e-5 and the roundings of d), and the float evaluation
// moves r^2 - dist^2 by < 20 eps (|S - C|^2 + r^2).  Certain when, over the box,
// dist(C, line(Lp, pos)) >= r + 2e-3 with |pos - Lp| >= 0.05 (so the 3e-5
// shifts move the distance by < 1e-3), using dist^2 = |w|^2 - (w.u)^2 / |u|^2,
// w = C - Lp, u = pos - Lp, max (w.u)^2 at a corner of the box, min |u|^2 at
// the point of the box nearest Lp.
__device__ static bool sphere_shadow_surely_missed(const RtSphere &S, const double Lp[3], const float lo[3],
                                                   const float hi[3])
{
    const double w[3] = {(double)S.cx - Lp[0], (double)S.cy - Lp[1], (double)S.cz - Lp[2]};
    double ulo[3], uhi[3], n2 = 0.0, wu = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        ulo[k] = (double)lo[k] - Lp[k];
        uhi[k] = (double)hi[k] - Lp[k];
        const double nk = ulo[k] > 0 ? ulo[k] : (uhi[k] < 0 ? uhi[k] : 0.0);
        n2 += nk * nk;
        wu += fmax(fabs(w[k] * ulo[k]), fabs(w[k] * uhi[k]));
    }
    if (!(isfinite(wu) && n2 >= 0.0025)) return false;
    const double w2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const double r = sqrt((double)S.r2) + 2e-3;
    // wu >= max |w.u| (sum of per-component maxima of |w_k u_k|)
    return w2 - (wu * wu) / n2 * (1.0 + 1e-9) > r * r * (1.0 + 1e-9) + 1e-4;
}

// The same for every light of a frame's set (each light tested on its own).
__device__ static bool sphere_shadow_surely_missed_set(const RtSphere &S, const RtFrame &F, const float lo[3],
                                                       const float hi[3])
{
    for (int l = 0; l < F.n_lights; ++l) {
        const RtLight L = F.lights[l];
        const double Lp[3] = {(double)L.x, (double)L.y, (double)L.z};
        if (!sphere_shadow_surely_missed(S, Lp, lo, hi)) return false;
    }
    return true;
}

// Wave-wide min / max (ds_bpermute butterflies; a DPP row version measured
// slower here).  Callers keep all 64 lanes alive and give lanes that do not
// contribute the identity (+-FLT_MAX).
// A wave-uniform 64-bit value (e.g. a mask read from LDS) moved to SGPRs, so
// loops over its bits are scalar.
__device__ __forceinline__ unsigned long long uniform_u64(unsigned long long v)
{
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ float uniform_f32(float v)
{
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

__device__ __forceinline__ float wave_min(float v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_max(float v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Per-wave culling certificate for DirectLight's shadow rays (skeleton.cpp:394).
//
// A shadow ray starts at S = P + n*1e-5 with direction d = L - P (the float
// vectors the reference uses).  With a = L - v0 and p = S - L + d (a few 1e-5
// at most, plus the rounding of s = S - v0), exact arithmetic gives
//   det  = -d.(e1 x e2)                      (linear in d)
//   detU = -d.(a x e2) - [d, p, e2]          (linear + |d||p||e2|)
//   detV = -d.(e1 x a) - [d, e1, p]
//   detT - det = a.(e1 x e2) + p.(e1 x e2)   (constant + |p||N|)
// so over the wave's box of d the same certificate as for camera rays holds,
// plus "the triangle lies beyond the light" (t > 1 + 1e-5, hence distance >=
// rmag: no shadow).  `pn` bounds |p| (Euclidean) over the wave.
struct ShadowBox {
    float lo[3], hi[3];   // exact float extremes of d over the casting lanes
    float pn;             // bound on |S - L + d| over the casting lanes
};

__device__ static bool cull_shadow(const RtTri &c, vec3 L, double rho, const ShadowBox &B)
{
    const double eps = 5.9604644775390625e-8;   // 2^-24
    const double g = 16.0 * eps;
    vec3 e1 = v3(c.e1x, c.e1y, c.e1z), e2 = v3(c.e2x, c.e2y, c.e2z);
    double ax = (double)L.x - c.v0x, ay = (double)L.y - c.v0y, az = (double)L.z - c.v0z;
    double Nx = (double)e1.y * e2.z - (double)e2.y * e1.z, Ny = (double)e1.z * e2.x - (double)e2.z * e1.x,
           Nz = (double)e1.x * e2.y - (double)e2.x * e1.y;
    double Ax = ay * e2.z - (double)e2.y * az, Ay = az * e2.x - (double)e2.z * ax, Az = ax * e2.y - (double)e2.x * ay;
    double Bx = (double)e1.y * az - ay * e1.z, By = (double)e1.z * ax - az * e1.x, Bz = (double)e1.x * ay - ax * e1.y;
    double cx = 0.5 * ((double)B.lo[0] + B.hi[0]), cy = 0.5 * ((double)B.lo[1] + B.hi[1]),
           cz = 0.5 * ((double)B.lo[2] + B.hi[2]);
    double hx = 0.5 * ((double)B.hi[0] - B.lo[0]), hy = 0.5 * ((double)B.hi[1] - B.lo[1]),
           hz = 0.5 * ((double)B.hi[2] - B.lo[2]);
    auto lin = [&](double X, double Y, double Z, double &lo, double &hi) {
        double m = -(cx * X + cy * Y + cz * Z);
        double h = hx * fabs(X) + hy * fabs(Y) + hz * fabs(Z);
        lo = m - h;
        hi = m + h;
    };
    double Dx = fmax(fabs((double)B.lo[0]), fabs((double)B.hi[0]));
    double Dy = fmax(fabs((double)B.lo[1]), fabs((double)B.hi[1]));
    double Dz = fmax(fabs((double)B.lo[2]), fabs((double)B.hi[2]));
    double dn = sqrt_ub(Dx * Dx + Dy * Dy + Dz * Dz);
    // |s| <= |a| + |d| + |p| componentwise; p also absorbs s's own rounding
    double Sx = fabs(ax) + rho + Dx + B.pn, Sy = fabs(ay) + rho + Dy + B.pn, Sz = fabs(az) + rho + Dz + B.pn;
    double pn = (double)B.pn + eps * sqrt_ub(Sx * Sx + Sy * Sy + Sz * Sz) + 1e-12;
    double n1 = sqrt_ub((double)e1.x * e1.x + (double)e1.y * e1.y + (double)e1.z * e1.z);
    double n2 = sqrt_ub((double)e2.x * e2.x + (double)e2.y * e2.y + (double)e2.z * e2.z);
    double nN = sqrt_ub(Nx * Nx + Ny * Ny + Nz * Nz);
    double dlo, dhi, ulo, uhi, vlo, vhi, blo, bhi;
    lin(Nx, Ny, Nz, dlo, dhi);
    lin(Ax, Ay, Az, ulo, uhi);
    lin(Bx, By, Bz, vlo, vhi);
    lin(Ax + Bx - Nx, Ay + By - Ny, Az + Bz - Nz, blo, bhi);
    // float-evaluation bounds (sum of |triple products|)
    auto M3 = [](double x0, double y0, double z0, double x1, double y1, double z1, double x2, double y2,
                 double z2) {   // |c0|,|c1|,|c2| components of det3(c0, c1, c2)
        return x0 * (y1 * z2 + y2 * z1) + x1 * (y0 * z2 + y2 * z0) + x2 * (y0 * z1 + y1 * z0);
    };
    double ae1x = fabs((double)e1.x), ae1y = fabs((double)e1.y), ae1z = fabs((double)e1.z);
    double ae2x = fabs((double)e2.x), ae2y = fabs((double)e2.y), ae2z = fabs((double)e2.z);
    double Ed = g * M3(Dx, Dy, Dz, ae1x, ae1y, ae1z, ae2x, ae2y, ae2z) + 1e-12 * (fabs(dlo) + fabs(dhi));
    double Eu = g * M3(Dx, Dy, Dz, Sx, Sy, Sz, ae2x, ae2y, ae2z) + dn * (pn + rho) * n2 + 1e-12 * (fabs(ulo) + fabs(uhi));
    double Ev = g * M3(Dx, Dy, Dz, ae1x, ae1y, ae1z, Sx, Sy, Sz) + dn * (pn + rho) * n1 + 1e-12 * (fabs(vlo) + fabs(vhi));
    double Et = g * M3(Sx, Sy, Sz, ae1x, ae1y, ae1z, ae2x, ae2y, ae2z) + (pn + rho) * nN;
    double Eb = Ed + Eu + Ev + 1e-12 * (fabs(blo) + fabs(bhi));
    double aN = ax * Nx + ay * Ny + az * Nz;
    double EaN = 1e-12 * (fabs(ax * Nx) + fabs(ay * Ny) + fabs(az * Nz));
    if (!(isfinite(dlo + dhi + ulo + uhi + vlo + vhi + blo + bhi) && isfinite(Ed + Eu + Ev + Et + Eb + aN)))
        return false;
    int sg;
    if (dlo - Ed > 0) sg = 1;
    else if (dhi + Ed < 0) sg = -1;
    else return sign_free_reject(dlo, dhi, Ed, ulo, uhi, Eu, vlo, vhi, Ev, blo, bhi, Eb);   // det may vanish
    const double dmin = sg > 0 ? dlo - Ed : -(dhi + Ed);
    const double dmax = sg > 0 ? dhi + Ed : -(dlo - Ed);
    const double tiny = 1e-20 * dmax;
    // detT = det + aN + (p.N): t = 1 + (detT - det)/det
    double tlo = aN - EaN - Et - Ed, thi = aN + EaN + Et + Ed;   // range of detT - det
    // beyond the light: t - 1 > 1e-5 certain -> distance >= rmag (:395)
    if (sg > 0 ? (tlo > 1e-5 * dmax) : (thi < -1e-5 * dmax)) return true;
    // t < 0: detT = det + (detT - det) has the opposite sign of det, i.e.
    // (detT - det)/det < -1 - margin
    if (sg > 0 ? (thi + dmax < -tiny - 1e-6 * dmax) : (tlo - dmax > tiny + 1e-6 * dmax)) return true;
    if (sg > 0 ? (uhi + Eu < -tiny) : (ulo - Eu > tiny)) return true;
    if (sg > 0 ? (vhi + Ev < -tiny) : (vlo - Ev > tiny)) return true;
    if (uv_sum_reject(sg, blo, bhi, Eb, fmax(fabs(ulo), fabs(uhi)) + Eu + fmax(fabs(vlo), fabs(vhi)) + Ev,
                      dmin, dmax))
        return true;
    return false;
}

// Triangle tests with exact pre-rejections.  Both skip the IEEE divide only
// when its outcome is certain:
//  * t < 0: det and detT of opposite signs with |detT| >= 2^-60 |det|,
//    |det| >= 2^-60 and len >= 2^-60, so t and distance = t*len are
//    strictly negative (no underflow to -0): rejected at :311;
//  * distance > bound: same signs and fl(|detT| len) >= fl(fl(|det| bound)
//    (1 + 2^-18)) with the right side finite and >= 2^-100, which implies
//    t*len >= bound (1 + 2^-20) and hence a rounded distance strictly above
//    `bound` (:313 for the closest hit, :395 for a shadow ray).
__device__ __forceinline__ bool surely_negative(float detT, float det, float len)
{
    const float adT = fabsf(detT), ad = fabsf(det);
    return ((detT < 0.0f) != (det < 0.0f)) && detT != 0.0f && ad >= 0x1p-60f && len >= 0x1p-60f &&
           adT >= ad * 0x1p-60f;
}
__device__ __forceinline__ bool surely_beyond(float detT, float det, float len, float bound)
{
    if (!((detT > 0.0f && det > 0.0f) || (detT < 0.0f && det < 0.0f))) return false;
    const float rhs = (fabsf(det) * bound) * 1.000003814697265625f;   // 1 + 2^-18
    return rhs <= FLT_MAX && rhs >= 0x1p-100f && fabsf(detT) * len >= rhs;
}

// Divide-free decisions of the reference's quotient tests.  ClosestIntersection
// (skeleton.cpp:306-335) forms t = detT/det, u = detU/det, v = detV/det with
// IEEE divides, but only the comparisons of their rounded values decide
// anything except the accepted hit's t.  Each function below returns 1 / 0
// when the comparison's outcome is certain from the operands' magnitudes
// (rounding errors bounded, margins 2^-18 against at most a few 2^-24
// relative errors) and -1 otherwise; a -1 sends the caller down the
// reference's own divide path, so results are bit-identical either way.
// Domain of the fast paths: finite operands with 2^-20 <= |det| <= 2^40,
// |detT|, |detU|, |detV| <= 2^40, 2^-20 <= len <= 2^20 -- the quotients and
// distances then stay in the normal range (no underflow, no overflow);
// anything else (NaN, det = 0, extreme scales) is undecided.
__device__ __forceinline__ bool fsign(float x) { return (__float_as_uint(x) >> 31) != 0u; }

// distance = fl(fl(detT/det) * len) against the reference's tests
// `distance < 0` (:311) and `distance >= bound || distance > FLT_MAX`
// (:313 with bound = the running best; :395 with bound = r_magnitude):
// 1 = passes both (0 <= distance < bound), 0 = fails one, -1 undecided.
//  * t < 0 certain: signs differ, detT != 0 and |detT| >= 2^-80 |det|, so
//    |t| >= 2^-80 and |distance| >= 2^-100: strictly negative (no -0).
//  * detT = +-0 or same signs: t >= 0 or t = -0; distance is then >= 0 or -0,
//    and `-0 < 0` is false, so the first test passes.
//  * X = fl(|detT| len), Y = fl(|det| bound): X <= fl(Y (1 - 2^-18)) gives
//    t len <= bound (1 - 2^-18)(1 + 2^-24)^3 < bound (1 - 2^-19), so the
//    rounded distance (two more roundings) is < bound; X >= fl(Y (1 + 2^-18))
//    gives t len > bound (1 + 2^-19) and a rounded distance >= bound.
//    bound > 2^100 is beyond any distance of the domain (< 2^81).
__device__ __forceinline__ int t_decide(float detT, float det, float len, float bound)
{
    const float ad = fabsf(det), at = fabsf(detT);
    if (!(ad >= 0x1p-20f && ad <= 0x1p40f && at <= 0x1p40f && len >= 0x1p-20f && len <= 0x1p20f &&
          bound >= 0x1p-20f))
        return -1;   // also NaN / inf operands
    if (detT != 0.0f && fsign(detT) != fsign(det)) return at >= ad * 0x1p-80f ? 0 : -1;
    if (bound > 0x1p100f) return 1;
    const float X = at * len, Y = ad * bound;
    if (X <= Y * (1.0f - 0x1p-18f)) return 1;
    if (X >= Y * (1.0f + 0x1p-18f)) return 0;
    return -1;
}

// (u >= 0) && (v >= 0) && ((u + v) <= 1) with u = fl(detU/det), v = fl(detV/det)
// (:328-335): 1 accept, 0 reject, -1 undecided.
//  * u < 0 certain: signs of detU and det differ, detU != 0, |detU| >= 2^-80 |det|
//    (|u| >= 2^-80: no rounding to -0).  u >= 0 certain: detU = +-0 or same signs.
//  * both >= 0: u + v = (|detU| + |detV|) / |det| exactly; P = fl(|detU| + |detV|)
//    <= fl(|det| (1 - 2^-18)) gives u + v < 1 - 2^-20, so fl(fl(u) + fl(v)) <= 1;
//    P >= fl(|det| (1 + 2^-18)) gives u + v > 1 + 2^-20 and a rounded sum > 1.
__device__ __forceinline__ int uv_decide(float det, float detU, float detV)
{
    const float ad = fabsf(det), au = fabsf(detU), av = fabsf(detV);
    if (!(ad >= 0x1p-20f && ad <= 0x1p40f && au <= 0x1p40f && av <= 0x1p40f)) return -1;
    const bool sd = fsign(det);
    const float tiny = ad * 0x1p-80f;
    const bool uneg = detU != 0.0f && fsign(detU) != sd, vneg = detV != 0.0f && fsign(detV) != sd;
    if ((uneg && au >= tiny) || (vneg && av >= tiny)) return 0;
    if (uneg || vneg) return -1;
    const float P = au + av;
    if (P <= ad * (1.0f - 0x1p-18f)) return 1;
    if (P >= ad * (1.0f + 0x1p-18f)) return 0;
    return -1;
}

// One triangle of ClosestIntersection (:306-335): whether it becomes the new
// closest hit, given det, detT, |d| and the running best; uvf(detU, detV)
// supplies the u / v numerators.  On acceptance t and distance are the
// reference's rounded values (one IEEE divide).  Rejections are decided
// divide-free whenever t_decide / uv_decide are certain.
template <class UV>
__device__ __forceinline__ bool tri_accept(float detT, float det, float len, float best, UV uvf, float &t_out,
                                           float &dist_out, bool wc = true)
{
    const float bound = FLT_MAX;
    float detU, detV;
    if (wc) cg_work(W_T_PRI);
    const float t = detT / det;                               // :306
    const float distance = t * len;                           // :307
    if (distance < 0.0f) return false;                        // :311
    if (distance >= best || distance > bound) return false;   // :313
    if (wc) cg_work(W_UV_PRI);
    uvf(detU, detV);
    {
        const float u = detU / det, v = detV / det;           // :317-321
        if (!((u >= 0) && (v >= 0) && ((u + v) <= 1))) return false;   // :328-335
    }
    t_out = t;
    dist_out = distance;
    return true;
}

// ClosestIntersection for camera-origin rays (skeleton.cpp:263-363).
// Returns best index: >= 0 triangle, -1 - k sphere k, INT_MIN no hit; t out.
// Triangles are visited in index order; with CULL only those whose bit is set
// in `mask` (certified-rejected ones are skipped, see cull_primary).
template <bool CULL>
__device__ __forceinline__ int closest_primary(const RtFrame &F, const RtTri *__restrict__ tc,
                                               const RtSphere *__restrict__ sph, vec3 d,
                                               float &best_t, unsigned long long mask)
{
    const float bound = FLT_MAX;
    float best = bound;
    int bi = INT_MIN;
    float bt = 0.f;
    vec3 nd = -d;
    float len = length(d);                                   // :307
    cg_work(W_RAY_PRI);
    for (int it = 0; CULL ? (mask != 0ull) : (it < F.n_tris); ++it) {
        int k = it;
        if (CULL) {
            k = __builtin_ctzll(mask);
            mask &= mask - 1ull;
        }
        const RtTri c = tc[k];
        float Q2 = nd.y * c.e2z - c.e2y * nd.z;
        float Q1 = nd.y * c.e1z - c.e1y * nd.z;
        float det = (nd.x * c.K1 - c.e1x * Q2) + c.e2x * Q1;  // det(-d, e1, e2) :289
        float t, distance;
        auto uvf = [&](float &detU, float &detV) {
            float Q3 = nd.y * c.sz - c.sy * nd.z;
            detU = (nd.x * c.K2 - c.sx * Q2) + c.e2x * Q3;    // det(-d, s, e2) :317
            detV = (nd.x * c.K3 - c.e1x * Q3) + c.sx * Q1;    // det(-d, e1, s) :320
        };
        if (tri_accept(c.detT, det, len, best, uvf, t, distance)) {
            best = distance;
            bt = t;
            bi = k;
        }
    }
    const vec3 s3 = v3(F.cam[0], F.cam[1], F.cam[2]);
    for (int k = 0; k < F.n_sph; ++k) {                       // :341-355
        float t;
        const RtSphere S = sph[k];
        const vec3 L = s3 - v3(S.cx, S.cy, S.cz);             // camera-constant (:48, :51)
        cg_work(W_SPH_PRI);
        if (sphere_intersect_pre(L, dot(L, L) - S.r2, d, t)) {
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

// ClosestIntersection for N independent camera rays of one lane (ray n: d =
// (X[n], Y[n], focal), traced iff live[n]), triangle-outer: each triangle's
// constants are loaded once for the N rays and their divides are
// independent.  Each ray's result equals closest_primary's for it.
template <int N>
__device__ __forceinline__ void closest_primary_n(const RtFrame &F, const RtTri *__restrict__ tc,
                                                  const RtSphere *__restrict__ sph, const float (&X)[N],
                                                  const float (&Y)[N], const bool (&live)[N],
                                                  unsigned long long mask, int (&bi)[N], float (&bt)[N],
                                                  bool wc = true)
{
    const float bound = FLT_MAX;
    const float fz = F.focal;
    float best[N], len[N];
#pragma unroll
    for (int n = 0; n < N; ++n) {
        if (wc && live[n]) cg_work(W_RAY_PRI);
        len[n] = length(v3(X[n], Y[n], fz));                  // :307
        best[n] = bound;
        bt[n] = 0.f;
        bi[n] = INT_MIN;
    }
    while (mask != 0ull) {
        const int k = __builtin_ctzll(mask);
        mask &= mask - 1ull;
        const RtTri c = tc[k];
#pragma unroll
        for (int n = 0; n < N; ++n) {
            if (!live[n]) continue;
            const vec3 nd = -v3(X[n], Y[n], fz);
            float Q2 = nd.y * c.e2z - c.e2y * nd.z;
            float Q1 = nd.y * c.e1z - c.e1y * nd.z;
            float det = (nd.x * c.K1 - c.e1x * Q2) + c.e2x * Q1;  // det(-d, e1, e2) :289
            float t, distance;
            auto uvf = [&](float &detU, float &detV) {
                float Q3 = nd.y * c.sz - c.sy * nd.z;
                detU = (nd.x * c.K2 - c.sx * Q2) + c.e2x * Q3;    // :317
                detV = (nd.x * c.K3 - c.e1x * Q3) + c.sx * Q1;    // :320
            };
            if (tri_accept(c.detT, det, len[n], best[n], uvf, t, distance, wc)) {
                best[n] = distance;
                bt[n] = t;
                bi[n] = k;
            }
        }
    }
    const vec3 s3 = v3(F.cam[0], F.cam[1], F.cam[2]);
    for (int q = 0; q < F.n_sph; ++q) {                           // :341-355
        const RtSphere S = sph[q];
        const vec3 L = s3 - v3(S.cx, S.cy, S.cz);                 // camera-constant (:48, :51)
        const float cq = dot(L, L) - S.r2;
#pragma unroll
        for (int n = 0; n < N; ++n) {
            float t;
            if (wc && live[n]) cg_work(W_SPH_PRI);
            if (live[n] && sphere_intersect_pre(L, cq, v3(X[n], Y[n], fz), t) && t < best[n]) {
                best[n] = t;
                bt[n] = t;
                bi[n] = -1 - q;
            }
        }
    }
#pragma unroll
    for (int n = 0; n < N; ++n)
        if (!(best[n] < bound)) bi[n] = INT_MIN;                  // :357
}

// ClosestIntersection for a group of NI x NJ camera sub-rays of one pixel
// (sub-ray (a, b) has d = (dx[a], dy[b], focal)), triangle-outer: each
// triangle's constants are loaded once per group and the terms that depend
// on one coordinate of -d only (Q1, Q2, e1x*Q2, e2x*Q1 on d.y; nd.x*K1 on
// d.x) are evaluated once -- the same float ops on the same operands as
// closest_primary, so each sub-ray's result is identical to it.  The
// per-sub-ray divides are independent, which gives the VALU ILP.
template <bool CULL, int NI, int NJ>
__device__ __forceinline__ void closest_primary_group(const RtFrame &F, const RtTri *__restrict__ tc,
                                                      const RtSphere *__restrict__ sph,
                                                      const float (&dx)[NI], const float (&dy)[NJ],
                                                      unsigned long long mask, int (&bi)[NI * NJ],
                                                      float (&bt)[NI * NJ])
{
    constexpr int NS = NI * NJ;
    const float bound = FLT_MAX;
    const float fz = F.focal, ndz = -fz;
    float ndx[NI], ndy[NJ], best[NS], len[NS];
#pragma unroll
    for (int a = 0; a < NI; ++a) ndx[a] = -dx[a];
#pragma unroll
    for (int b = 0; b < NJ; ++b) ndy[b] = -dy[b];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        cg_work(W_RAY_PRI);
        len[s] = length(v3(dx[s / NJ], dy[s % NJ], fz));      // :307
        best[s] = bound;
        bt[s] = 0.f;
        bi[s] = INT_MIN;
    }
    for (int it = 0; CULL ? (mask != 0ull) : (it < F.n_tris); ++it) {
        int k = it;
        if (CULL) {
            k = __builtin_ctzll(mask);
            mask &= mask - 1ull;
        }
        const RtTri c = tc[k];
        float A[NI], Q1[NJ], Q2[NJ], B[NJ], C[NJ];
#pragma unroll
        for (int a = 0; a < NI; ++a) A[a] = ndx[a] * c.K1;
#pragma unroll
        for (int b = 0; b < NJ; ++b) {
            Q2[b] = ndy[b] * c.e2z - c.e2y * ndz;
            Q1[b] = ndy[b] * c.e1z - c.e1y * ndz;
            B[b] = c.e1x * Q2[b];
            C[b] = c.e2x * Q1[b];
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int a = s / NJ, b = s % NJ;
            float det = (A[a] - B[b]) + C[b];                  // det(-d, e1, e2) :289
            float t, distance;
            auto uvf = [&](float &detU, float &detV) {
                float Q3 = ndy[b] * c.sz - c.sy * ndz;
                detU = (ndx[a] * c.K2 - c.sx * Q2[b]) + c.e2x * Q3;   // :317
                detV = (ndx[a] * c.K3 - c.e1x * Q3) + c.sx * Q1[b];   // :320
            };
            if (tri_accept(c.detT, det, len[s], best[s], uvf, t, distance)) {
                best[s] = distance;
                bt[s] = t;
                bi[s] = k;
            }
        }
    }
    const vec3 s3 = v3(F.cam[0], F.cam[1], F.cam[2]);
    for (int q = 0; q < F.n_sph; ++q) {                        // :341-355
        const RtSphere S = sph[q];
        const vec3 L = s3 - v3(S.cx, S.cy, S.cz);              // camera-constant (:48, :51)
        const float cq = dot(L, L) - S.r2;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            float t;
            cg_work(W_SPH_PRI);
            if (sphere_intersect_pre(L, cq, v3(dx[s / NJ], dy[s % NJ], fz), t) && t < best[s]) {
                best[s] = t;
                bt[s] = t;
                bi[s] = -1 - q;
            }
        }
    }
#pragma unroll
    for (int s = 0; s < NS; ++s)
        if (!(best[s] < bound)) bi[s] = INT_MIN;               // :357
}

// Shadow test of DirectLight (skeleton.cpp:394-398): ClosestIntersection
// from `start` towards the light, shadowed iff its distance < rmag.  The
// closest distance is < rmag iff SOME accepted hit is, so this is an
// any-hit search bounded by rmag with an early exit; triangles are tested
// with the reference's float ops (their acceptance does not depend on the
// running minimum, only on `distance < rmag` here).
// One triangle of the shadow test (skeleton.cpp:289-335 from a generic
// start): an accepted hit with distance < rmag (:394-395).
__device__ __forceinline__ bool tri_shadow_hit(const RtTri &c, vec3 start, vec3 nd, float len, float rmag)
{
    cg_work(W_T_SH);
    float sx = start.x - c.v0x, sy = start.y - c.v0y, sz = start.z - c.v0z;   // :296
    float Q2 = nd.y * c.e2z - c.e2y * nd.z;
    float Q1 = nd.y * c.e1z - c.e1y * nd.z;
    float det = (nd.x * c.K1 - c.e1x * Q2) + c.e2x * Q1;
    float K2 = sy * c.e2z - c.e2y * sz;
    float K4 = sy * c.e1z - c.e1y * sz;
    float detT = (sx * c.K1 - c.e1x * K2) + c.e2x * K4;                    // det(s, e1, e2)
    float t = detT / det;
    float distance = t * len;
    if (distance < 0.0f) return false;
    if (distance >= rmag || distance > FLT_MAX) return false;
    cg_work(W_UV_SH);
    float Q3 = nd.y * sz - sy * nd.z;
    float K3 = c.e1y * sz - sy * c.e1z;
    float detU = (nd.x * K2 - sx * Q2) + c.e2x * Q3;
    float detV = (nd.x * K3 - c.e1x * Q3) + sx * Q1;
    float u = detU / det;
    float v = detV / det;
    return (u >= 0) && (v >= 0) && ((u + v) <= 1);
}

template <bool CULL>
__device__ __forceinline__ bool shadowed(const RtFrame &F, const RtTri *__restrict__ tc,
                                         const RtSphere *__restrict__ sph, vec3 start, vec3 d,
                                         float rmag, unsigned long long mask)
{
    vec3 nd = -d;
    float len = length(d);
    cg_work(W_RAY_SH);
    for (int it = 0; CULL ? (mask != 0ull) : (it < F.n_tris); ++it) {
        int k = it;
        if (CULL) {
            k = __builtin_ctzll(mask);
            mask &= mask - 1ull;
        }
        if (tri_shadow_hit(tc[k], start, nd, len, rmag)) return true;
    }
    for (int k = 0; k < F.n_sph; ++k) {
        float t;
        cg_work(W_SPH_SH);
        if (sphere_intersect(sph[k], start, d, t) && t < rmag) return true;
    }
    return false;
}

// x / d per channel (:412's three numerators over one area), bit for bit.  The
// compiler's IEEE f32 division is v_div_scale (denominator), v_div_scale
// (numerator, VCC), v_rcp, two refinement FMAs, v_mul, three FMAs, v_div_fmas,
// v_div_fixup; here d's refined reciprocal is formed once for the three and the
// scaling and fix-up steps are dropped.  Those are identities when the operands
// and the quotient are normal and far from the range ends: div_scale rescales
// only a denormal or extreme-exponent operand or quotient (VCC then stays clear
// and div_fmas is a plain FMA), div_fixup rewrites only zero, infinite or NaN
// operands.  Taken when d is in [2^-40, 2^40], each x at least 2^-86 and their
// sum at most 2^40 (so each quotient lies in [2^-126, 2^80], no exponent gap
// reaches 96 and every numerator exceeds 2^-103); NaN fails the tests, and any
// lane outside divides as before.
// SHARED = false: the three IEEE divides.  Measured per kernel (profiles/r06_ab_session2.json):
// the light-set sweep (C4) gains 1.6 %, the one-light lattice (C2) lost 1.7 % and the large
// scenes' shading 0.7 %, so only the sweep takes it.
template <bool SHARED>
__device__ __forceinline__ vec3 div3_by(vec3 x, float d)
{
    if constexpr (SHARED) {
        const bool ok = d >= 0x1p-40f && d <= 0x1p40f && x.x >= 0x1p-86f && x.y >= 0x1p-86f &&
                        x.z >= 0x1p-86f && (x.x + x.y) + x.z <= 0x1p40f;
        if (ok) {
            const float r0 = __builtin_amdgcn_rcpf(d);
            const float r = fmaf(fmaf(-d, r0, 1.0f), r0, r0);
            auto q = [&](float n) {
                float m = n * r;
                m = fmaf(fmaf(-d, m, n), r, m);
                return fmaf(fmaf(-d, m, n), r, m);
            };
            return v3(q(x.x), q(x.y), q(x.z));
        }
    }
    return x / d;
}

// DirectLight's lit branch (skeleton.cpp:400-412): r = light - pos, rmag its
// FP64 magnitude (:370-371), normal at the hit (:377-387).
template <bool SHARED = false>
__device__ __forceinline__ vec3 direct_light_lit(const RtLight &Lt, vec3 r, float rmag, vec3 normal,
                                                 vec3 objColor)
{
    vec3 nd = normalize(r);                                              // :400
    float a = dot(nd, normal);                                           // :403
    const float b = (float)(4 * M_PI);                                   // :404
    float area = (float)((double)b * ((double)rmag * (double)rmag));     // :406
    if (a <= 0) a = 0.f;                                                 // :409
    vec3 lc = v3(Lt.r, Lt.g, Lt.b);
    return div3_by<SHARED>((objColor * lc) * a, area);                   // :412
}

// r_magnitude (skeleton.cpp:371): the norm in FP64, rounded to float.
__device__ __forceinline__ float light_rmag(vec3 r)
{
    double r0 = (double)r.x * (double)r.x, r1 = (double)r.y * (double)r.y,
           r2 = (double)r.z * (double)r.z;
    return (float)sqrt((r0 + r1) + r2);
}

// DirectLight (skeleton.cpp:366-415) for a hit at `pos` on object `bi`.
template <bool CULL>
__device__ __forceinline__ vec3 direct_light(const RtFrame &F, const RtTri *__restrict__ tc,
                                             const RtShade *__restrict__ shade,
                                             const RtSphere *__restrict__ sph, int bi, vec3 pos,
                                             vec3 objColor, int l, unsigned long long smask = ~0ull)
{
    const RtLight Lt = F.lights[l];                                      // uniform: scalar loads
    cg_work(W_DL);
    vec3 lp = v3(Lt.x, Lt.y, Lt.z);
    vec3 r = lp - pos;                                                   // :370
    float rmag = light_rmag(r);                                          // :371
    vec3 normal = hit_normal(shade, sph, bi, pos);
    vec3 origin = pos + normal * 0.00001f;                              // :394
    if (shadowed<CULL>(F, tc, sph, origin, r, rmag, smask)) return v3(0.0f, 0.0f, 0.0f);  // :394-398
    return direct_light_lit(Lt, r, rmag, normal, objColor);
}

// Shadow-ray certificate for light l: per-lane box of d = L - pos and bound
// on |S - L + d| over the hits given, reduced over the wave into one mask.
struct LaneShadowBox {
    float lo[3], hi[3], pn;
    __device__ void init()
    {
        lo[0] = lo[1] = lo[2] = FLT_MAX;
        hi[0] = hi[1] = hi[2] = -FLT_MAX;
        pn = 0.0f;
    }
};

__device__ __forceinline__ void shadow_box_add(LaneShadowBox &b, vec3 lmin, vec3 lmax, vec3 pos, vec3 normal)
{
    // d_k = fl(L_k - pos) (:370/:373) is monotone in L_k, so every light's
    // direction lies in [fl(lmin - pos), fl(lmax - pos)] componentwise.
    vec3 rlo = lmin - pos, rhi = lmax - pos;
    vec3 S = pos + normal * 0.00001f;                                    // :394
    // p_k = S - L_k + d_k = (S - pos) + rounding(d_k): |p_k| <= |S - pos|_1 + 2^-24 |d|_1.
    // Evaluated in float: at most 8 rounded ops of relative error 2^-24 each,
    // covered by the (1 + 2^-18) factor, so pb stays an upper bound.
    float sp = (fabsf(S.x - pos.x) + fabsf(S.y - pos.y)) + fabsf(S.z - pos.z);
    float dr = (fmaxf(fabsf(rlo.x), fabsf(rhi.x)) + fmaxf(fabsf(rlo.y), fabsf(rhi.y))) + fmaxf(fabsf(rlo.z), fabsf(rhi.z));
    float pb = ((sp + 5.9604644775390625e-8f * dr) * 1.000003814697265625f) + 1e-30f;
    b.lo[0] = fminf(b.lo[0], rlo.x); b.hi[0] = fmaxf(b.hi[0], rhi.x);
    b.lo[1] = fminf(b.lo[1], rlo.y); b.hi[1] = fmaxf(b.hi[1], rhi.y);
    b.lo[2] = fminf(b.lo[2], rlo.z); b.hi[2] = fmaxf(b.hi[2], rhi.z);
    b.pn = fmaxf(b.pn, pb);
}

// Cornell-box form of the shadow certificate's input: per lane only the
// extremes of the hit positions (6 min/max per hit).  The wave then derives
// the direction box -- d_k = fl(L_k - pos) is monotone in L_k and in pos, so
// every d lies in [fl(lmin - pos_max), fl(lmax - pos_min)] -- and bounds
// p = S - L + d = (S - pos) + rounding(d) without the hit normals:
//   |S_c - pos_c| <= |fl(n_c 1e-5f)| (1 + 2^-24) + 2^-24 |pos_c|,  |n_c| <= nbound
//   |rounding(d_c)| <= 2^-24 |d_c|
// (S = pos + n * 0.00001f, skeleton.cpp:394; nbound = the scene's largest
// normal component, from cg_rt_set_scene).  A non-finite position or bound
// turns the box infinite, i.e. no triangle is culled.
struct LanePosBox {
    float lo[3], hi[3];
    __device__ void init()
    {
        lo[0] = lo[1] = lo[2] = FLT_MAX;
        hi[0] = hi[1] = hi[2] = -FLT_MAX;
    }
    __device__ void add(vec3 p)
    {
        if (!isfinite((p.x + p.y) + p.z)) {
            lo[0] = lo[1] = lo[2] = -INFINITY;
            hi[0] = hi[1] = hi[2] = INFINITY;
            return;
        }
        lo[0] = fminf(lo[0], p.x); hi[0] = fmaxf(hi[0], p.x);
        lo[1] = fminf(lo[1], p.y); hi[1] = fmaxf(hi[1], p.y);
        lo[2] = fminf(lo[2], p.z); hi[2] = fmaxf(hi[2], p.z);
    }
};

// Whole wave, converged control flow.
__device__ __forceinline__ ShadowBox shadow_box_of_range(const RtFrame &F, const float (&lo)[3], const float (&hi)[3])
{
    ShadowBox B;
    float pn = 0.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float plo = lo[c], phi = hi[c];
        B.lo[c] = F.lmin[c] - phi;
        B.hi[c] = F.lmax[c] - plo;
        const float P = fmaxf(fabsf(plo), fabsf(phi)), D = fmaxf(fabsf(B.lo[c]), fabsf(B.hi[c]));
        pn += (F.nbound * 1.0001e-5f + (P + F.nbound * 1e-4f) * 0x1p-23f) + D * 0x1p-23f;
    }
    // float evaluation: < 16 rounded positive terms, covered by 1 + 2^-18
    B.pn = pn * 1.000003814697265625f + 1e-30f;
    return B;
}

__device__ __forceinline__ ShadowBox shadow_box_of_positions(const RtFrame &F, const LanePosBox &b)
{
    float lo[3], hi[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        lo[c] = wave_min(b.lo[c]);
        hi[c] = wave_max(b.hi[c]);
    }
    return shadow_box_of_range(F, lo, hi);
}

// Whole wave, converged control flow: the wave's box of its lanes' boxes.
__device__ __forceinline__ ShadowBox shadow_box_reduce(const LaneShadowBox &b)
{
    ShadowBox B;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        B.lo[c] = wave_min(b.lo[c]);
        B.hi[c] = wave_max(b.hi[c]);
    }
    B.pn = wave_max(b.pn);
    return B;
}

// Lane k certifies triangle k for every shadow ray in box B (whole wave).
__device__ __forceinline__ unsigned long long shadow_mask_box(const RtFrame &F, const RtTri *__restrict__ tc,
                                                              const ShadowBox &B, int lane)
{
    bool keep = true;
    if (lane < F.n_tris && B.lo[0] <= B.hi[0])
        keep = !cull_shadow(tc[lane], v3(F.lc[0], F.lc[1], F.lc[2]), F.lrho, B);
    return __ballot(keep && lane < F.n_tris);
}

// As shadow_mask_box, lane k holding triangle k's constants in `c`.
__device__ __forceinline__ unsigned long long shadow_mask_lane(const RtFrame &F, const RtTri &c, const ShadowBox &B,
                                                               int lane)
{
    bool keep = true;
    if (lane < F.n_tris && B.lo[0] <= B.hi[0]) keep = !cull_shadow(c, v3(F.lc[0], F.lc[1], F.lc[2]), F.lrho, B);
    return __ballot(keep && lane < F.n_tris);
}

__device__ __forceinline__ unsigned long long shadow_mask_of(const RtFrame &F, const RtTri *__restrict__ tc,
                                                             const LaneShadowBox &b, int lane)
{
    return shadow_mask_box(F, tc, shadow_box_reduce(b), lane);
}

__device__ __forceinline__ int shard_row(const RtFrame &F, int L)
{
    int k = L / F.stripe_h;
    return F.row0 + (k * F.nranks + F.rank) * F.stripe_h + (L - k * F.stripe_h);
}

}  // namespace cg
