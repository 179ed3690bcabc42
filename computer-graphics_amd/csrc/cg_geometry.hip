// cg_geometry.hip -- host geometry of the rasteriser's Draw
// (rasteriser/Source/skeleton.cpp:205-241): camera space, shadow volumes,
// rotation, clip space and the six clip planes.  It runs on the host, as in
// the reference (a few hundred triangles, microseconds); the pixel work it
// feeds runs in cg_rast.hip.  Float ops follow the reference expression by
// expression (compiled with -ffp-contract=off).
#include <cstring>
#include <vector>

#include "cg_internal.h"

using namespace cg;

namespace {

vec4 V(cg_vec4 v) { return v4(v.x, v.y, v.z, v.w); }
cg_vec4 C(vec4 v) { return cg_vec4{v.x, v.y, v.z, v.w}; }

// rasteriser/Source/TestModelH.h:32-41
void compute_normal(cg_rtri &t)
{
    vec3 e1 = v3(t.v1.x - t.v0.x, t.v1.y - t.v0.y, t.v1.z - t.v0.z);
    vec3 e2 = v3(t.v2.x - t.v0.x, t.v2.y - t.v0.y, t.v2.z - t.v0.z);
    vec3 n = normalize(cross(e2, e1));
    t.normal = cg_vec4{n.x, n.y, n.z, 1.0f};
}

// Triangle(v0, v1, v2, color) constructor (TestModelH.h:26-30)
cg_rtri make_tri(vec4 a, vec4 b, vec4 c, cg_vec3 col)
{
    cg_rtri t;
    t.v0 = C(a); t.v1 = C(b); t.v2 = C(c);
    t.color = col;
    t.texture = 0;
    t.index = 0;
    compute_normal(t);
    return t;
}

// a + t*(b - a) as vec4 ops (skeleton.cpp:757 and siblings)
vec4 toward(vec4 a, vec4 b, float t) { return a + (b - a) * t; }

// The split cases of clip() in the reference's order: all in, one vertex in
// (v0 / v1 / v2), two in (v0v1 / v0v2 / v1v2).  I/O are the "in"/"out"
// predicates (kept separately: a NaN coordinate is neither and drops the
// triangle); tp(i, j) is the edge parameter from in-vertex i towards j.
template <class TP>
void clip_one(cg_rtri t, const bool I[3], const bool O[3], bool v02_third, TP tp, float t21_v02,
              std::vector<cg_rtri> &out)
{
    vec4 v0 = V(t.v0), v1 = V(t.v1), v2 = V(t.v2);
    auto extra = [&](vec4 a, vec4 b, vec4 c) {   // :838-841
        cg_rtri e = make_tri(a, b, c, t.color);
        e.normal = t.normal;
        e.texture = t.texture;
        e.index = t.index;
        return e;
    };
    if (I[0] && I[1] && I[2]) { out.push_back(t); return; }
    if (I[0] && O[1] && O[2]) {
        t.v1 = C(toward(v0, v1, tp(0, 1)));
        t.v2 = C(toward(v0, v2, tp(0, 2)));
        out.push_back(t);
        return;
    }
    if (O[0] && I[1] && O[2]) {
        t.v0 = C(toward(v1, v0, tp(1, 0)));
        t.v2 = C(toward(v1, v2, tp(1, 2)));
        out.push_back(t);
        return;
    }
    if (O[0] && O[1] && I[2]) {
        t.v1 = C(toward(v2, v1, tp(2, 1)));
        t.v0 = C(toward(v2, v0, tp(2, 0)));
        out.push_back(t);
        return;
    }
    if (I[0] && I[1] && O[2]) {
        vec4 p12 = toward(v1, v2, tp(1, 2)), p02 = toward(v0, v2, tp(0, 2));
        t.v2 = C(p02);
        cg_rtri e = extra(p02, p12, v1);
        out.push_back(t);
        out.push_back(e);
        return;
    }
    if (I[0] && O[1] && v02_third) {
        vec4 p01 = toward(v0, v1, tp(0, 1)), p21 = toward(v2, v1, t21_v02);
        t.v1 = C(p01);
        cg_rtri e = extra(p01, p21, v2);
        out.push_back(t);
        out.push_back(e);
        return;
    }
    if (O[0] && I[1] && I[2]) {
        vec4 p10 = toward(v1, v0, tp(1, 0)), p20 = toward(v2, v0, tp(2, 0));
        t.v0 = C(p10);
        cg_rtri e = extra(p10, p20, v2);
        out.push_back(t);
        out.push_back(e);
        return;
    }
    // every vertex out: dropped
}

// clip(triangles, plane) (skeleton.cpp:720-1673)
std::vector<cg_rtri> clip(const std::vector<cg_rtri> &in, int plane, const cg_rast_params &p)
{
    std::vector<cg_rtri> out;
    out.reserve(in.size() * 2);
    const int W = p.width, H = p.height;
    for (const cg_rtri &t : in) {
        const float w[3] = {t.v0.w, t.v1.w, t.v2.w};
        if (plane == 5) {                                     // :1497-1505
            if (t.v0.z > 0.01f && t.v1.z > 0.01f && t.v2.z > 0.01f) out.push_back(t);
            continue;
        }
        if (plane == 6) {                                     // :1507-1670
            const float wl = 5.0f / p.focal;
            bool I[3], O[3];
            for (int k = 0; k < 3; ++k) { I[k] = w[k] <= wl; O[k] = w[k] > wl; }
            auto tp = [&](int i, int j) { return (wl - w[i]) / (w[j] - w[i]); };
            // quirks: :1607 tests v2.x, :1615 divides t_21 by (w1 - w0)
            clip_one(t, I, O, t.v2.x <= wl, tp, (wl - w[2]) / (w[1] - w[0]), out);
            continue;
        }
        const bool xplane = plane == 1 || plane == 2;
        const float c[3] = {xplane ? t.v0.x : t.v0.y, xplane ? t.v1.x : t.v1.y, xplane ? t.v2.x : t.v2.y};
        const int half = xplane ? W / 2 : H / 2;           // SCREEN_WIDTH/2, SCREEN_HEIGHT/2
        const int neg = xplane ? -W / 2 : -H / 2;          // -SCREEN_WIDTH/2 (int division)
        const int full = xplane ? W : H;
        bool I[3], O[3];
        for (int k = 0; k < 3; ++k) {
            if (plane == 1 || plane == 4) {                // v.w * -SCREEN_*/2, in if strictly greater
                float d = (w[k] * (float)(-full)) / 2;
                I[k] = c[k] > d;
                O[k] = c[k] <= d;
            } else {                                       // v.w * SCREEN_*/2, in if strictly less
                float d = (w[k] * (float)full) / 2;
                I[k] = c[k] < d;
                O[k] = c[k] >= d;
            }
        }
        const float h = (float)half, nh = (float)neg;
        auto tp = [&](int i, int j) {
            if (plane == 1 || plane == 4)                  // (c_i + h w_i)/(-h w_j + h w_i - c_j + c_i)
                return (c[i] + h * w[i]) / ((((nh * w[j]) + (h * w[i])) - c[j]) + c[i]);
            return (c[i] - h * w[i]) / ((((h * w[j]) - (h * w[i])) - c[j]) + c[i]);
        };
        clip_one(t, I, O, I[2], tp, tp(2, 1), out);
    }
    return out;
}

}  // namespace

extern "C" int cg_rast_prepare(const cg_rast_params *p, const cg_rtri *room, int n_room,
                               const cg_rtri *boxes, int n_boxes, cg_rtri *out, int cap,
                               cg_vec4 *light_out)
{
    if (!p || n_room < 0 || n_boxes < 0 || (n_room && !room) || (n_boxes && !boxes) || cap < 0 ||
        (cap && !out) || p->focal == 0.0f || p->width <= 0 || p->height <= 0)
        return CG_E_INVALID;
    const vec4 cam = V(p->camera);
    // toCameraSpace (:701-716)
    auto to_camera = [&](cg_rtri &t) {
        vec4 a = V(t.v0) - cam, b = V(t.v1) - cam, c = V(t.v2) - cam;
        a.w = 1.0f; b.w = 1.0f; c.w = 1.0f;
        t.v0 = C(a); t.v1 = C(b); t.v2 = C(c);
    };
    std::vector<cg_rtri> tris(room, room + n_room);
    for (cg_rtri &t : tris) to_camera(t);
    vec4 lightPos = V(p->light_scene) - cam;                  // :211-212
    lightPos.w = 1.0f;
    // createShadowVolume (:1676-1722), appended after the room (:218-220)
    const cg_vec3 sc{-1.0f, -1.0f, -1.0f};
    for (int i = 0; i < n_boxes; ++i) {
        cg_rtri t = boxes[i];
        to_camera(t);
        tris.push_back(t);
        vec4 v0 = V(t.v0), v1 = V(t.v1), v2 = V(t.v2);
        vec4 n0 = (v0 - lightPos) * 100.0f, n1 = (v1 - lightPos) * 100.0f, n2 = (v2 - lightPos) * 100.0f;
        tris.push_back(make_tri(v0, n0, v1, sc));
        tris.push_back(make_tri(n0, v1, n1, sc));
        tris.push_back(make_tri(v1, n1, v2, sc));
        tris.push_back(make_tri(n1, v2, n2, sc));
        tris.push_back(make_tri(v2, n2, v0, sc));
        tris.push_back(make_tri(n2, v0, n0, sc));
    }
    // rotate (:223-228), toClipSpace w = z/f (:691-699)
    lightPos = mat4_mul(p->R, lightPos);
    for (cg_rtri &t : tris) {
        vec4 a = mat4_mul(p->R, V(t.v0)), b = mat4_mul(p->R, V(t.v1)), c = mat4_mul(p->R, V(t.v2));
        a.w = a.z / p->focal; b.w = b.z / p->focal; c.w = c.z / p->focal;
        t.v0 = C(a); t.v1 = C(b); t.v2 = C(c);
    }
    for (int plane = 1; plane <= 6; ++plane) tris = clip(tris, plane, *p);   // :236-241
    int n = (int)tris.size();
    if (out && cap) std::memcpy(out, tris.data(), sizeof(cg_rtri) * (size_t)(n < cap ? n : cap));
    if (light_out) *light_out = C(lightPos);
    return n;
}
