// cg_scene.hip -- LoadTestModel for both hot paths (host code).
//   raytracer/Source/TestModelH.h:121-279  (28 triangles + 1 sphere)
//   rasteriser/Source/TestModelH.h:48-312  (room 10 + boxes 20, setting = settingBoxes = 0)
// Vertex scaling and normals use the reference's float ops exactly.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "cg_internal.h"

using namespace cg;

namespace {

struct P4 { float x, y, z, w; };

// Triangle::ComputeNormal (both TestModelH.h files)
template <class T>
void compute_normal(T &t)
{
    vec3 e1 = v3(t.v1.x - t.v0.x, t.v1.y - t.v0.y, t.v1.z - t.v0.z);
    vec3 e2 = v3(t.v2.x - t.v0.x, t.v2.y - t.v0.y, t.v2.z - t.v0.z);
    vec3 n = normalize(cross(e2, e1));
    t.normal = cg_vec4{n.x, n.y, n.z, 1.0f};
}

// `v *= 2/L; v -= (1,1,1,1); v.x *= -1; v.y *= -1; v.w = 1` (RT :246-269, RAST :266-310)
cg_vec4 scale_vertex(cg_vec4 v, float L)
{
    float s = 2 / L;
    vec4 r = v4(v.x, v.y, v.z, v.w) * s;
    r = r - v4(1, 1, 1, 1);
    r.x *= -1;
    r.y *= -1;
    r.w = 1.0f;
    return cg_vec4{r.x, r.y, r.z, r.w};
}

struct Box { cg_vec4 A, B, C, D, E, F, G, H; };

Box box(float ax, float az, float bx, float bz, float cx, float cz, float dx, float dz, float h)
{
    Box b;
    b.A = cg_vec4{ax, 0, az, 1}; b.B = cg_vec4{bx, 0, bz, 1};
    b.C = cg_vec4{cx, 0, cz, 1}; b.D = cg_vec4{dx, 0, dz, 1};
    b.E = cg_vec4{ax, h, az, 1}; b.F = cg_vec4{bx, h, bz, 1};
    b.G = cg_vec4{cx, h, cz, 1}; b.H = cg_vec4{dx, h, dz, 1};
    return b;
}

const cg_vec3 kRed{0.75f, 0.15f, 0.15f}, kYellow{0.75f, 0.75f, 0.15f}, kGreen{0.15f, 0.75f, 0.15f},
    kCyan{0.15f, 0.75f, 0.75f}, kBlue{0.15f, 0.15f, 0.75f}, kPurple{0.75f, 0.15f, 0.75f},
    kWhite{0.75f, 0.75f, 0.75f};

}  // namespace

extern "C" int cg_rt_load_test_model(cg_tri *tris, int cap, cg_sphere *sphere)
{
    if (!tris || cap < 28) return CG_E_CAPACITY;
    const float L = 555;
    int n = 0;
    auto add = [&](cg_vec4 a, cg_vec4 b, cg_vec4 c, cg_vec3 col) {
        cg_tri &t = tris[n++];
        t.v0 = a; t.v1 = b; t.v2 = c; t.color = col;
        compute_normal(t);
    };
    Box r = box(L, 0, 0, 0, L, L, 0, L, L);   // room corners A..H (TestModelH.h:145-153)
    add(r.C, r.B, r.A, kGreen);  add(r.C, r.D, r.B, kGreen);     // floor
    add(r.A, r.E, r.C, kPurple); add(r.C, r.E, r.G, kPurple);    // left wall
    add(r.F, r.B, r.D, kYellow); add(r.H, r.F, r.D, kYellow);    // right wall
    add(r.E, r.F, r.G, kCyan);   add(r.F, r.H, r.G, kCyan);      // ceiling
    add(r.G, r.D, r.C, kWhite);  add(r.G, r.H, r.D, kWhite);     // back wall
    Box s = box(290, 114, 130, 65, 240, 272, 82, 225, 165);      // short block (:178-206)
    add(s.E, s.B, s.A, kRed); add(s.E, s.F, s.B, kRed);
    add(s.F, s.D, s.B, kRed); add(s.F, s.H, s.D, kRed);
    add(s.H, s.C, s.D, kRed); add(s.H, s.G, s.C, kRed);
    add(s.G, s.E, s.C, kRed); add(s.E, s.A, s.C, kRed);
    add(s.G, s.F, s.E, kRed); add(s.G, s.H, s.F, kRed);
    Box t = box(423, 247, 265, 296, 472, 406, 314, 456, 330);    // tall block (:212-240), no back face
    add(t.E, t.B, t.A, kBlue); add(t.E, t.F, t.B, kBlue);
    add(t.F, t.D, t.B, kBlue); add(t.F, t.H, t.D, kBlue);
    add(t.G, t.E, t.C, kBlue); add(t.E, t.A, t.C, kBlue);
    add(t.G, t.F, t.E, kBlue); add(t.G, t.H, t.F, kBlue);
    for (int i = 0; i < n; ++i) {
        tris[i].v0 = scale_vertex(tris[i].v0, L);
        tris[i].v1 = scale_vertex(tris[i].v1, L);
        tris[i].v2 = scale_vertex(tris[i].v2, L);
        compute_normal(tris[i]);
    }
    if (sphere) {                                                // :275-277, Sphere ctor :17-18
        float rad = 0.3f;
        sphere->radius = rad;
        sphere->radiusSquared = rad * rad;
        sphere->centre = cg_vec3{-0.45f, 0.6f, -0.6f};
        sphere->color = kWhite;
        sphere->normal = cg_vec3{0, 0, 0};
    }
    return n;
}

extern "C" int cg_rast_load_test_model(cg_rtri *room, int room_cap, int *n_room, cg_rtri *boxes,
                                       int boxes_cap, int *n_boxes)
{
    if (!room || !boxes || !n_room || !n_boxes || room_cap < 10 || boxes_cap < 20) return CG_E_CAPACITY;
    const float L = 555;
    int nr = 0, nb = 0;
    auto add = [&](cg_rtri *arr, int &n, cg_vec4 a, cg_vec4 b, cg_vec4 c, cg_vec3 col, int index) {
        cg_rtri &t = arr[n++];
        t.v0 = a; t.v1 = b; t.v2 = c; t.color = col;
        t.texture = 0;                                           // setting = settingBoxes = 0
        t.index = index;
        compute_normal(t);
    };
    const cg_vec3 back{0.03529f, 0.7843f, 0.8078f};
    Box r = box(L, 0, 0, 0, L, L, 0, L, L);
    add(room, nr, r.C, r.B, r.A, kGreen, 2);  add(room, nr, r.C, r.D, r.B, kGreen, 2);
    add(room, nr, r.A, r.E, r.C, kPurple, 3); add(room, nr, r.C, r.E, r.G, kPurple, 3);
    add(room, nr, r.F, r.B, r.D, kYellow, 4); add(room, nr, r.H, r.F, r.D, kYellow, 4);
    add(room, nr, r.E, r.F, r.G, kCyan, 1);   add(room, nr, r.F, r.H, r.G, kCyan, 1);
    add(room, nr, r.G, r.D, r.C, back, 0);    add(room, nr, r.G, r.H, r.D, back, 0);
    Box s = box(290, 114, 130, 65, 240, 272, 82, 225, 165);
    add(boxes, nb, s.E, s.B, s.A, kRed, 0); add(boxes, nb, s.E, s.F, s.B, kRed, 0);
    add(boxes, nb, s.F, s.D, s.B, kRed, 4); add(boxes, nb, s.F, s.H, s.D, kRed, 4);
    add(boxes, nb, s.H, s.C, s.D, kRed, 0); add(boxes, nb, s.H, s.G, s.C, kRed, 0);
    add(boxes, nb, s.G, s.E, s.C, kRed, 3); add(boxes, nb, s.E, s.A, s.C, kRed, 3);
    add(boxes, nb, s.G, s.F, s.E, kRed, 1); add(boxes, nb, s.G, s.H, s.F, kRed, 1);
    Box t = box(423, 247, 265, 296, 472, 406, 314, 456, 330);    // tall block incl. back face
    add(boxes, nb, t.E, t.B, t.A, kBlue, 0); add(boxes, nb, t.E, t.F, t.B, kBlue, 0);
    add(boxes, nb, t.F, t.D, t.B, kBlue, 4); add(boxes, nb, t.F, t.H, t.D, kBlue, 4);
    add(boxes, nb, t.H, t.C, t.D, kBlue, 0); add(boxes, nb, t.H, t.G, t.C, kBlue, 0);
    add(boxes, nb, t.G, t.E, t.C, kBlue, 3); add(boxes, nb, t.E, t.A, t.C, kBlue, 3);
    add(boxes, nb, t.G, t.F, t.E, kBlue, 1); add(boxes, nb, t.G, t.H, t.F, kBlue, -1); // :256 uninitialised
    for (int pass = 0; pass < 2; ++pass) {
        cg_rtri *arr = pass ? boxes : room;
        int n = pass ? nb : nr;
        for (int i = 0; i < n; ++i) {
            arr[i].v0 = scale_vertex(arr[i].v0, L);
            arr[i].v1 = scale_vertex(arr[i].v1, L);
            arr[i].v2 = scale_vertex(arr[i].v2, L);
            compute_normal(arr[i]);
        }
    }
    *n_room = nr;
    *n_boxes = nb;
    return nr + nb;
}

// ---------------------------------------------------------------------------
// Build-defined workloads (not in the reference).

// C4 area light: n x n point lights at the cell centres of a square of side
// `side` in the xz-plane centred on the given light, each carrying 1/(n*n) of
// its colour; light (i, j) is out[j*n + i].
extern "C" int cg_rt_area_lights(const cg_light *centre, float side, int n, cg_light *out, int cap)
{
    if (!centre || n <= 0 || n > 64 || !(side >= 0.0f)) return CG_E_INVALID;
    if (!out || cap < n * n) return CG_E_CAPACITY;
    const float fn = (float)n, inv = 1.0f / (float)(n * n);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            cg_light &l = out[j * n + i];
            l.position = centre->position;
            l.position.x = centre->position.x + side * (((float)i + 0.5f) / fn - 0.5f);
            l.position.z = centre->position.z + side * (((float)j + 0.5f) / fn - 0.5f);
            l.colour = cg_vec3{centre->colour.x * inv, centre->colour.y * inv, centre->colour.z * inv};
        }
    return n * n;
}

namespace {
// PCG32 (pcg32_random_r, XSH-RR 64/32), seeded like pcg32_srandom_r(seed, seq).
struct Pcg32 {
    uint64_t state = 0, inc = 0;
    Pcg32(uint64_t seed, uint64_t seq)
    {
        inc = (seq << 1u) | 1u;
        next();
        state += seed;
        next();
    }
    uint32_t next()
    {
        uint64_t old = state;
        state = old * 6364136223846793005ull + inc;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((0u - rot) & 31u));
    }
    // a + (b - a) * u, u = top 24 bits / 2^24 in [0, 1) (all float ops exact but the last two)
    float uniform(float a, float b) { return a + (b - a) * ((float)(next() >> 8) * 5.9604644775390625e-8f); }
};
}  // namespace

// C5 random scene: triangle k draws centroid (x, y, z) ~ U[-1,1], then
// v0, v1, v2 = centroid + U[-0.02,0.02]^3 each (x, y, z order), then colour
// ~ U[0.15,0.75]^3; w = 1; normal by ComputeNormal.  Stream seq 54.
extern "C" int cg_rt_random_scene(uint64_t seed, int n, cg_tri *out)
{
    if (n < 0 || (n && !out)) return CG_E_INVALID;
    Pcg32 g(seed, 54u);
    for (int k = 0; k < n; ++k) {
        cg_tri &t = out[k];
        float cx = g.uniform(-1.f, 1.f), cy = g.uniform(-1.f, 1.f), cz = g.uniform(-1.f, 1.f);
        cg_vec4 *v[3] = {&t.v0, &t.v1, &t.v2};
        for (cg_vec4 *p : v) {
            float dx = g.uniform(-0.02f, 0.02f), dy = g.uniform(-0.02f, 0.02f), dz = g.uniform(-0.02f, 0.02f);
            *p = cg_vec4{cx + dx, cy + dy, cz + dz, 1.0f};
        }
        float r = g.uniform(0.15f, 0.75f), gg = g.uniform(0.15f, 0.75f), b = g.uniform(0.15f, 0.75f);
        t.color = cg_vec3{r, gg, b};
        compute_normal(t);
    }
    return n;
}

namespace cg {
// The scene's box for the column windows: every triangle vertex and every
// sphere (radius widened by 1e-6), then widened by 0.02 (1 + max |coordinate|).
// A scene property: computed once per uploaded scene (cg_rt_set_scene), so
// the per-frame window below is O(1) for any camera.  Empty scene: lo > hi.
void rt_scene_box(const cg_tri *tris, int n_tris, const cg_sphere *spheres, int n_spheres, double lo[3],
                  double hi[3])
{
    for (int k = 0; k < 3; ++k) {
        lo[k] = 1e300;
        hi[k] = -1e300;
    }
    if (n_tris == 0 && n_spheres == 0) return;
    auto add = [&](double x, double y, double z, double r) {
        const double p[3] = {x, y, z};
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p[k] - r);
            hi[k] = std::max(hi[k], p[k] + r);
        }
    };
    for (int i = 0; i < n_tris; ++i) {
        const cg_vec4 *v[3] = {&tris[i].v0, &tris[i].v1, &tris[i].v2};
        for (const cg_vec4 *q : v) add(q->x, q->y, q->z, 0.0);
    }
    for (int i = 0; i < n_spheres; ++i)
        add(spheres[i].centre.x, spheres[i].centre.y, spheres[i].centre.z,
            std::sqrt((double)spheres[i].radiusSquared) * (1.0 + 1e-6));
    const double m = 0.02 * (1.0 + std::max({std::fabs(lo[0]), std::fabs(lo[1]), std::fabs(lo[2]), std::fabs(hi[0]),
                                               std::fabs(hi[1]), std::fabs(hi[2])}));
    for (int k = 0; k < 3; ++k) {
        lo[k] -= m;
        hi[k] += m;
    }
}

// Columns an unrotated camera can see anything in, from the scene's box
// (rt_scene_box).  A ray of image x-offset X = u - W/2 + i/2 (i = -1, 0, 1)
// meets the plane z = cz + s at x = cx + s X / f; it can reach a point of the
// box only if X lies between the extreme projections f (px - cx) / (pz - cz)
// of the box's corners (all with pz - cz > 0).  FP64, widened by two pixels.
void rt_box_columns(const double lo[3], const double hi[3], const cg_rt_camera *cam, int *col0, int *col1)
{
    const int W = cam->width;
    *col0 = 0;
    *col1 = W;
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            if (cam->R[4 * c + r] != (r == c ? 1.0f : 0.0f)) return;   // rotated: whole width
    if (lo[0] > hi[0]) {   // nothing to see
        *col1 = 0;
        return;
    }
    const double cx = cam->camera.x, cz = cam->camera.z, f = cam->focal;
    if (!(lo[2] - cz > 1e-6) || !(f > 0) || !std::isfinite(f)) return;   // box reaches behind the camera
    double xmin = 1e300, xmax = -1e300;
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
            const double X = f * ((a ? hi[0] : lo[0]) - cx) / ((b ? hi[2] : lo[2]) - cz);
            xmin = std::min(xmin, X);
            xmax = std::max(xmax, X);
        }
    if (!(std::isfinite(xmin) && std::isfinite(xmax))) return;
    // pixel u's sub-rays have X in [u - W/2 - 0.5, u - W/2 + 0.5]
    const double u0 = std::floor(xmin + W / 2 - 0.5) - 2.0, u1 = std::ceil(xmax + W / 2 + 0.5) + 3.0;
    int a = (int)std::max(0.0, std::min((double)W, u0)), b = (int)std::max(0.0, std::min((double)W, u1));
    a = (a / 16) * 16;
    b = std::min(W, ((b + 15) / 16) * 16);
    if (a >= b) {
        *col0 = *col1 = 0;
        return;
    }
    *col0 = a;
    *col1 = b;
}
}  // namespace cg

extern "C" int cg_rt_frame_columns(const cg_tri *tris, int n_tris, const cg_sphere *spheres, int n_spheres,
                                   const cg_rt_camera *cam, int *col0, int *col1)
{
    if (!cam || !col0 || !col1 || n_tris < 0 || n_spheres < 0 || (n_tris && !tris) || (n_spheres && !spheres) ||
        cam->width <= 0)
        return CG_E_INVALID;
    double lo[3], hi[3];
    cg::rt_scene_box(tris, n_tris, spheres, n_spheres, lo, hi);
    cg::rt_box_columns(lo, hi, cam, col0, col1);
    return CG_OK;
}
