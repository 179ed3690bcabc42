// cg_geom.h -- the rasteriser's per-frame geometry, shared by the host entry
// point (cg_rast_prepare) and the device kernel (rast_geometry_kernel), so
// both produce bit-identical triangle lists.
//
// Reference: rasteriser/Source/skeleton.cpp:205-241 (Draw's geometry),
// toCameraSpace :701-716, createShadowVolume :1676-1722, rotation :223-228,
// toClipSpace :691-699, clip :720-1673.
//
// Ordering: the reference clips the whole list plane by plane, each input
// triangle producing [modified, extra] in place.  Triangles never interact,
// so the final list is, per input triangle in order, the depth-first
// pre-order of its clip tree (modified child before extra child) -- which is
// what clip_dfs emits.
#pragma once

#include "cg_internal.h"

namespace cg {

struct GeomParams {
    int W, H;
    float focal;
    float cam[4];
    float R[16];
    float light_scene[4];
};

CG_HD vec4 V4(cg_vec4 v) { return v4(v.x, v.y, v.z, v.w); }
CG_HD cg_vec4 C4(vec4 v) { return cg_vec4{v.x, v.y, v.z, v.w}; }

// Triangle::ComputeNormal (rasteriser/Source/TestModelH.h:32-41)
CG_HD void rtri_normal(cg_rtri &t)
{
    vec3 e1 = v3(t.v1.x - t.v0.x, t.v1.y - t.v0.y, t.v1.z - t.v0.z);
    vec3 e2 = v3(t.v2.x - t.v0.x, t.v2.y - t.v0.y, t.v2.z - t.v0.z);
    vec3 n = normalize(cross(e2, e1));
    t.normal = cg_vec4{n.x, n.y, n.z, 1.0f};
}

// Triangle(v0, v1, v2, color) (TestModelH.h:26-30); texture = 0, index unset
CG_HD cg_rtri rtri_make(vec4 a, vec4 b, vec4 c, cg_vec3 col)
{
    cg_rtri t;
    t.v0 = C4(a); t.v1 = C4(b); t.v2 = C4(c);
    t.color = col;
    t.texture = 0;
    t.index = 0;
    rtri_normal(t);
    return t;
}

// a + t*(b - a) as vec4 ops (skeleton.cpp:757 and siblings)
CG_HD vec4 toward(vec4 a, vec4 b, float t) { return a + (b - a) * t; }

// lightPos as Draw computes it: camera space (:211-212), then rotated (:223)
CG_HD vec4 geom_light_camera(const GeomParams &p)
{
    vec4 l = v4(p.light_scene[0], p.light_scene[1], p.light_scene[2], p.light_scene[3]) -
             v4(p.cam[0], p.cam[1], p.cam[2], p.cam[3]);
    l.w = 1.0f;
    return l;
}

// Input triangle i of the clipper (before clipping), i in [0, n_room + 7*n_boxes):
// the room in order, then per box triangle: itself and its 6 shadow-volume
// triangles (:1686-1718), all rotated and with w = z/f.
CG_HD cg_rtri geom_input(const GeomParams &p, const cg_rtri *room, int n_room, const cg_rtri *boxes, int i)
{
    const vec4 cam = v4(p.cam[0], p.cam[1], p.cam[2], p.cam[3]);
    auto to_camera = [&](cg_rtri &t) {                 // :701-716
        vec4 a = V4(t.v0) - cam, b = V4(t.v1) - cam, c = V4(t.v2) - cam;
        a.w = 1.0f; b.w = 1.0f; c.w = 1.0f;
        t.v0 = C4(a); t.v1 = C4(b); t.v2 = C4(c);
    };
    cg_rtri t;
    if (i < n_room) {
        t = room[i];
        to_camera(t);
    } else {
        const int j = (i - n_room) / 7, k = (i - n_room) % 7;
        cg_rtri b = boxes[j];
        to_camera(b);
        if (k == 0) {
            t = b;
        } else {
            const vec4 L = geom_light_camera(p);
            vec4 v0 = V4(b.v0), v1 = V4(b.v1), v2 = V4(b.v2);
            vec4 n0 = (v0 - L) * 100.0f, n1 = (v1 - L) * 100.0f, n2 = (v2 - L) * 100.0f;   // :1695-1697
            const cg_vec3 sc{-1.0f, -1.0f, -1.0f};
            switch (k) {                                                              // :1705-1710
            case 1: t = rtri_make(v0, n0, v1, sc); break;
            case 2: t = rtri_make(n0, v1, n1, sc); break;
            case 3: t = rtri_make(v1, n1, v2, sc); break;
            case 4: t = rtri_make(n1, v2, n2, sc); break;
            case 5: t = rtri_make(v2, n2, v0, sc); break;
            default: t = rtri_make(n2, v0, n0, sc); break;
            }
        }
    }
    vec4 a = mat4_mul(p.R, V4(t.v0)), b = mat4_mul(p.R, V4(t.v1)), c = mat4_mul(p.R, V4(t.v2));  // :224-227
    a.w = a.z / p.focal; b.w = b.z / p.focal; c.w = c.z / p.focal;                    // :695-697
    t.v0 = C4(a); t.v1 = C4(b); t.v2 = C4(c);
    return t;
}

// One plane of clip() (:720-1673) on one triangle: writes 0, 1 or 2 children
// (modified, then extra) and returns their count.
CG_HD int clip_plane(const cg_rtri &in, int plane, const GeomParams &p, cg_rtri out[2])
{
    cg_rtri t = in;
    const float w[3] = {t.v0.w, t.v1.w, t.v2.w};
    if (plane == 5) {                                                 // :1497-1505
        if (t.v0.z > 0.01f && t.v1.z > 0.01f && t.v2.z > 0.01f) {
            out[0] = t;
            return 1;
        }
        return 0;
    }
    bool I[3], O[3];
    bool v02_third;
    float c[3] = {0.f, 0.f, 0.f}, h = 0.f, nh = 0.f, wl = 0.f;
    bool lower = false;
    if (plane == 6) {                                                 // :1507-1670
        wl = 5.0f / p.focal;
        for (int k = 0; k < 3; ++k) { I[k] = w[k] <= wl; O[k] = w[k] > wl; }
        v02_third = t.v2.x <= wl;                                     // :1607 quirk (v2.x)
    } else {
        const bool xplane = plane == 1 || plane == 2;
        c[0] = xplane ? t.v0.x : t.v0.y;
        c[1] = xplane ? t.v1.x : t.v1.y;
        c[2] = xplane ? t.v2.x : t.v2.y;
        const int full = xplane ? p.W : p.H;
        h = (float)(full / 2);                                        // SCREEN_*/2
        nh = (float)(-full / 2);                                      // -SCREEN_*/2 (int division)
        lower = plane == 1 || plane == 4;                             // in if strictly greater
        for (int k = 0; k < 3; ++k) {
            float d = lower ? (w[k] * (float)(-full)) / 2 : (w[k] * (float)full) / 2;
            I[k] = lower ? c[k] > d : c[k] < d;
            O[k] = lower ? c[k] <= d : c[k] >= d;
        }
        v02_third = I[2];
    }
    if (I[0] && I[1] && I[2]) { out[0] = t; return 1; }
    // edge parameter from in-vertex i towards out-vertex j (computed only when used)
    auto tp = [&](int i, int j) -> float {
        if (plane == 6) return (wl - w[i]) / (w[j] - w[i]);
        return lower ? (c[i] + h * w[i]) / ((((nh * w[j]) + (h * w[i])) - c[j]) + c[i])
                     : (c[i] - h * w[i]) / ((((h * w[j]) - (h * w[i])) - c[j]) + c[i]);
    };
    const vec4 v0 = V4(t.v0), v1 = V4(t.v1), v2 = V4(t.v2);
    auto extra = [&](vec4 a, vec4 b, vec4 cc) {                       // :838-841
        cg_rtri e = rtri_make(a, b, cc, t.color);
        e.normal = t.normal;
        e.texture = t.texture;
        e.index = t.index;
        return e;
    };
    if (I[0] && O[1] && O[2]) {
        t.v1 = C4(toward(v0, v1, tp(0, 1)));
        t.v2 = C4(toward(v0, v2, tp(0, 2)));
        out[0] = t;
        return 1;
    }
    if (O[0] && I[1] && O[2]) {
        t.v0 = C4(toward(v1, v0, tp(1, 0)));
        t.v2 = C4(toward(v1, v2, tp(1, 2)));
        out[0] = t;
        return 1;
    }
    if (O[0] && O[1] && I[2]) {
        t.v1 = C4(toward(v2, v1, tp(2, 1)));
        t.v0 = C4(toward(v2, v0, tp(2, 0)));
        out[0] = t;
        return 1;
    }
    if (I[0] && I[1] && O[2]) {
        vec4 p12 = toward(v1, v2, tp(1, 2)), p02 = toward(v0, v2, tp(0, 2));
        t.v2 = C4(p02);
        out[1] = extra(p02, p12, v1);
        out[0] = t;
        return 2;
    }
    if (I[0] && O[1] && v02_third) {
        // :1615 quirk: plane 6 divides t_21 by (w1 - w0)
        const float t21 = plane == 6 ? (wl - w[2]) / (w[1] - w[0]) : tp(2, 1);
        vec4 p01 = toward(v0, v1, tp(0, 1)), p21 = toward(v2, v1, t21);
        t.v1 = C4(p01);
        out[1] = extra(p01, p21, v2);
        out[0] = t;
        return 2;
    }
    if (O[0] && I[1] && I[2]) {
        vec4 p10 = toward(v1, v0, tp(1, 0)), p20 = toward(v2, v0, tp(2, 0));
        t.v0 = C4(p10);
        out[1] = extra(p10, p20, v2);
        out[0] = t;
        return 2;
    }
    return 0;                                                         // all out (or NaN): dropped
}

// Clip tree of one input triangle through planes 1..6, emitted in the
// reference's order (depth-first pre-order, modified child first).  Returns
// the number emitted; emit(k, tri) is called for k = 0, 1, ...
template <class Emit>
CG_HD int clip_dfs(const cg_rtri &root, const GeomParams &p, Emit emit)
{
    // The leaves of the clip tree in pre-order are its root-to-leaf paths in
    // lexicographic order of their choices at the splitting planes (0 =
    // modified child, 1 = extra child).  Bit pl of `path` is the choice at
    // plane pl; each path is walked from the root, and the next one flips the
    // deepest untaken split to 1 and clears the choices below it.  No stack:
    // one triangle in registers (the device kernel runs this per thread).
    unsigned path = 0u;
    int n = 0;
    for (;;) {
        cg_rtri cur = root;
        unsigned splits = 0u;   // planes of this path where the triangle split
        bool alive = true;
        for (int pl = 1; pl <= 6; ++pl) {
            cg_rtri ch[2];
            const int k = clip_plane(cur, pl, p, ch);
            if (k == 0) { alive = false; break; }
            if (k == 2) {
                splits |= 1u << pl;
                cur = (path >> pl) & 1u ? ch[1] : ch[0];
            } else {
                cur = ch[0];
            }
        }
        if (alive) emit(n++, cur);
        const unsigned open = splits & ~path;   // splits still to take their extra branch
        if (!open) break;
        const int d = 31 - __builtin_clz(open);   // the deepest one
        path = (path & ((1u << d) - 1u)) | (1u << d);
    }
    return n;
}

}  // namespace cg
