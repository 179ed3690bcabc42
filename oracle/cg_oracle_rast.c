/*
 * cg_oracle_rast.c -- TEST INFRASTRUCTURE ONLY (checker + CPU baseline).
 *
 * Plain-C restatement of the reference rasteriser's Draw (texture modes
 * 0-3, colour modes 0-2): host geometry (camera space, shadow volumes, rotation,
 * clip space, six clip planes), VertexShader, ComputePolygonRows,
 * Interpolate, DrawPolygonRows, PixelShader, calculateIllumination and the
 * soft-shadow + anti-alias post-pass.  Each function cites the reference
 * file:line (rasteriser/Source/skeleton.cpp unless stated) it follows.
 * Float ops follow GLM 0.9.7.2 association; doubles where the reference
 * promotes.  Build with -O3 -ffp-contract=off, no -march.
 *
 * Pinned by the reference's own output, rasteriser/screenshot.bmp: the
 * metal-grill room after the recovered Update() key sequence matches it bit
 * for bit on all 602,987 pixels the missing marble map does not touch
 * (tests/test_rast_screenshot.py, texels from cg_oracle_jpeg.c = IJG libjpeg 9),
 * and by the reference's ComputePolygonRows KAT (skeleton.cpp:183-199).
 */
#include "cg_oracle.h"

#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

static inline cgo_v3 v3(float x, float y, float z) { cgo_v3 r = {x, y, z}; return r; }
static inline cgo_v4 v4(float x, float y, float z, float w) { cgo_v4 r = {x, y, z, w}; return r; }
static inline cgo_v4 v4_sub(cgo_v4 a, cgo_v4 b) { return v4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
static inline cgo_v4 v4_add(cgo_v4 a, cgo_v4 b) { return v4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
static inline cgo_v4 v4_muls(cgo_v4 a, float s) { return v4(a.x * s, a.y * s, a.z * s, a.w * s); }
static inline cgo_v3 v3_mul(cgo_v3 a, cgo_v3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline cgo_v3 v3_add(cgo_v3 a, cgo_v3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline float dot3(cgo_v3 a, cgo_v3 b)
{
    float px = a.x * b.x, py = a.y * b.y, pz = a.z * b.z;
    return (px + py) + pz;
}
static inline cgo_v3 normalize3(cgo_v3 v)
{
    float inv = 1.0f / sqrtf(dot3(v, v));
    return v3(v.x * inv, v.y * inv, v.z * inv);
}
static inline cgo_v3 cross3(cgo_v3 x, cgo_v3 y)
{
    return v3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
static inline cgo_v4 mat4_mul(const float *m, cgo_v4 v)
{
    float r[4];
    for (int k = 0; k < 4; ++k) {
        float a0 = m[0 * 4 + k] * v.x, a1 = m[1 * 4 + k] * v.y;
        float a2 = m[2 * 4 + k] * v.z, a3 = m[3 * 4 + k] * v.w;
        r[k] = (a0 + a1) + (a2 + a3);
    }
    return v4(r[0], r[1], r[2], r[3]);
}
/* x86-64 cvttss2si semantics for float->int (the reference's static_cast /
 * implicit conversion): out-of-range and NaN give INT_MIN. */
static inline int f2i(float f)
{
    if (f >= -2147483648.0f && f < 2147483648.0f) return (int)f;
    return INT_MIN;
}

/* rasteriser/Source/TestModelH.h:32-41 */
static void compute_normal(cgo_rast_tri *t)
{
    cgo_v3 e1 = v3(t->v1.x - t->v0.x, t->v1.y - t->v0.y, t->v1.z - t->v0.z);
    cgo_v3 e2 = v3(t->v2.x - t->v0.x, t->v2.y - t->v0.y, t->v2.z - t->v0.z);
    cgo_v3 n = normalize3(cross3(e2, e1));
    t->normal = v4(n.x, n.y, n.z, 1.0f);
}
/* TestModelH.h:26-30 (texture member-initialised to 0, index left as given) */
static cgo_rast_tri mk(cgo_v4 a, cgo_v4 b, cgo_v4 c, cgo_v3 col, int index)
{
    cgo_rast_tri t;
    t.v0 = a; t.v1 = b; t.v2 = c; t.color = col; t.texture = 0; t.index = index;
    compute_normal(&t);
    return t;
}

/* rasteriser/Source/TestModelH.h:48-312 with setting = settingBoxes = 0. */
int cgo_rast_load_scene(cgo_rast_tri *room, int *n_room, cgo_rast_tri *boxes, int *n_boxes)
{
    const cgo_v3 red = {0.75f, 0.15f, 0.15f}, yellow = {0.75f, 0.75f, 0.15f},
                 green = {0.15f, 0.75f, 0.15f}, cyan = {0.15f, 0.75f, 0.75f},
                 blue = {0.15f, 0.15f, 0.75f}, purple = {0.75f, 0.15f, 0.75f};
    const cgo_v3 back = {0.03529f, 0.7843f, 0.8078f};
    float L = 555;
    int n = 0, m = 0;
    cgo_v4 A = {L, 0, 0, 1}, B = {0, 0, 0, 1}, C = {L, 0, L, 1}, D = {0, 0, L, 1};
    cgo_v4 E = {L, L, 0, 1}, F = {0, L, 0, 1}, G = {L, L, L, 1}, H = {0, L, L, 1};
    room[n++] = mk(C, B, A, green, 2);  room[n++] = mk(C, D, B, green, 2);
    room[n++] = mk(A, E, C, purple, 3); room[n++] = mk(C, E, G, purple, 3);
    room[n++] = mk(F, B, D, yellow, 4); room[n++] = mk(H, F, D, yellow, 4);
    room[n++] = mk(E, F, G, cyan, 1);   room[n++] = mk(F, H, G, cyan, 1);
    room[n++] = mk(G, D, C, back, 0);   room[n++] = mk(G, H, D, back, 0);
    /* short block (TestModelH.h:140-200) */
    A = v4(290, 0, 114, 1); B = v4(130, 0, 65, 1); C = v4(240, 0, 272, 1); D = v4(82, 0, 225, 1);
    E = v4(290, 165, 114, 1); F = v4(130, 165, 65, 1); G = v4(240, 165, 272, 1); H = v4(82, 165, 225, 1);
    boxes[m++] = mk(E, B, A, red, 0); boxes[m++] = mk(E, F, B, red, 0);
    boxes[m++] = mk(F, D, B, red, 4); boxes[m++] = mk(F, H, D, red, 4);
    boxes[m++] = mk(H, C, D, red, 0); boxes[m++] = mk(H, G, C, red, 0);
    boxes[m++] = mk(G, E, C, red, 3); boxes[m++] = mk(E, A, C, red, 3);
    boxes[m++] = mk(G, F, E, red, 1); boxes[m++] = mk(G, H, F, red, 1);
    /* tall block (TestModelH.h:202-262), back face present here */
    A = v4(423, 0, 247, 1); B = v4(265, 0, 296, 1); C = v4(472, 0, 406, 1); D = v4(314, 0, 456, 1);
    E = v4(423, 330, 247, 1); F = v4(265, 330, 296, 1); G = v4(472, 330, 406, 1); H = v4(314, 330, 456, 1);
    boxes[m++] = mk(E, B, A, blue, 0); boxes[m++] = mk(E, F, B, blue, 0);
    boxes[m++] = mk(F, D, B, blue, 4); boxes[m++] = mk(F, H, D, blue, 4);
    boxes[m++] = mk(H, C, D, blue, 0); boxes[m++] = mk(H, G, C, blue, 0);
    boxes[m++] = mk(G, E, C, blue, 3); boxes[m++] = mk(E, A, C, blue, 3);
    boxes[m++] = mk(G, F, E, blue, 1); boxes[m++] = mk(G, H, F, blue, -1); /* :256 index uninitialised */
    float s = 2 / L;
    for (int pass = 0; pass < 2; ++pass) {                 /* TestModelH.h:266-310 */
        cgo_rast_tri *T = pass ? boxes : room;
        int cnt = pass ? m : n;
        for (int i = 0; i < cnt; ++i) {
            cgo_v4 *vs[3] = {&T[i].v0, &T[i].v1, &T[i].v2};
            for (int k = 0; k < 3; ++k) {
                cgo_v4 v = v4_muls(*vs[k], s);
                v = v4_sub(v, v4(1, 1, 1, 1));
                v.x *= -1; v.y *= -1; v.w = 1.0f;
                *vs[k] = v;
            }
            compute_normal(&T[i]);
        }
    }
    *n_room = n;
    *n_boxes = m;
    return n + m;
}

void cgo_rast_default_params(cgo_rast_params *p, int width, int height)
{
    memset(p, 0, sizeof(*p));
    p->width = width;
    p->height = height;
    p->focal = 512;                                   /* :30 */
    p->camera = v4(0, 0, -3.001f, 1);                 /* :31 */
    for (int k = 0; k < 16; ++k) p->R[k] = (k % 5 == 0) ? 1.0f : 0.0f;
    p->light_scene = v4(0, -0.5f, 0, 1);              /* :52 */
    p->light_power = v3(20.0f * 1, 20.0f * 1, 20.0f * 1); /* :53 */
    p->indirect_first = 0.2f;                         /* steady state (:585) */
}

/* ---------------------------- clipping --------------------------------- */
/* skeleton.cpp:720-1673.  Planes 1-4 share one shape: vertex k is "in" by a
 * strict compare of a coordinate against (w_k * s)/2 and "out" by the
 * complementary non-strict compare (kept separately: NaN is neither);
 * the edge parameter from in-vertex i to out-vertex j is
 *   (c_i + h*w_i) / ((((-h*w_j) + (h*w_i)) - c_j) + c_i)      (planes 1,4)
 *   (c_i - h*w_i) / (((( h*w_j) - (h*w_i)) - c_j) + c_i)      (planes 2,3)
 * with h = W/2 or H/2 as an int.  Plane 5 only rejects; plane 6 (far)
 * carries the reference's two quirks (:1607 tests v2.x, :1615 divides by
 * w1 - w0). */
typedef struct { int in[3], out[3]; float tp[3][3]; } clipinfo;

static void clip_info(const cgo_rast_tri *t, int plane, const cgo_rast_params *p, clipinfo *ci)
{
    const cgo_v4 V[3] = {t->v0, t->v1, t->v2};
    const int W = p->width, H = p->height;
    float c[3], w[3], d[3];
    for (int k = 0; k < 3; ++k) { w[k] = V[k].w; }
    if (plane == 1 || plane == 2) for (int k = 0; k < 3; ++k) c[k] = V[k].x;
    else for (int k = 0; k < 3; ++k) c[k] = V[k].y;
    for (int k = 0; k < 3; ++k) {
        switch (plane) {
        case 1: d[k] = (w[k] * (float)(-W)) / 2; ci->in[k] = c[k] > d[k]; ci->out[k] = c[k] <= d[k]; break;
        case 2: d[k] = (w[k] * (float)(W)) / 2;  ci->in[k] = c[k] < d[k]; ci->out[k] = c[k] >= d[k]; break;
        case 3: d[k] = (w[k] * (float)(H)) / 2;  ci->in[k] = c[k] < d[k]; ci->out[k] = c[k] >= d[k]; break;
        case 4: d[k] = (w[k] * (float)(-H)) / 2; ci->in[k] = c[k] > d[k]; ci->out[k] = c[k] <= d[k]; break;
        }
    }
    float h = (float)((plane == 1 || plane == 2) ? W / 2 : H / 2);
    float nh = (float)((plane == 1 || plane == 2) ? -W / 2 : -H / 2);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            if (i == j) continue;
            if (plane == 1 || plane == 4) {
                float num = c[i] + h * w[i];
                float den = (((nh * w[j]) + (h * w[i])) - c[j]) + c[i];
                ci->tp[i][j] = num / den;
            } else {
                float num = c[i] - h * w[i];
                float den = (((h * w[j]) - (h * w[i])) - c[j]) + c[i];
                ci->tp[i][j] = num / den;
            }
        }
}

static inline cgo_v4 lerp_from(cgo_v4 a, cgo_v4 b, float t)
{
    /* a + t*(b - a) (vec4 ops, skeleton.cpp:757) */
    return v4_add(a, v4_muls(v4_sub(b, a), t));
}

static int push(cgo_rast_tri *out, int n, int cap, const cgo_rast_tri *t)
{
    if (n < cap) out[n] = *t;
    return n + 1;
}

static cgo_rast_tri extra_tri(cgo_v4 a, cgo_v4 b, cgo_v4 c, const cgo_rast_tri *parent)
{
    cgo_rast_tri e = mk(a, b, c, parent->color, parent->index);   /* ctor -> ComputeNormal */
    e.normal = parent->normal;
    e.texture = parent->texture;
    e.index = parent->index;
    return e;
}

/* Apply one of the 7 reference cases given in/out predicates and edge params. */
static int clip_cases(cgo_rast_tri t, const int *I, const int *O, float tp[3][3],
                      cgo_rast_tri *out, int n, int cap, int quirk6_v02, float quirk6_t21)
{
    if (I[0] && I[1] && I[2]) return push(out, n, cap, &t);
    if (I[0] && O[1] && O[2]) {
        cgo_v4 v0 = t.v0, v1 = t.v1, v2 = t.v2;
        t.v1 = lerp_from(v0, v1, tp[0][1]);
        t.v2 = lerp_from(v0, v2, tp[0][2]);
        return push(out, n, cap, &t);
    }
    if (O[0] && I[1] && O[2]) {
        cgo_v4 v0 = t.v0, v1 = t.v1, v2 = t.v2;
        t.v0 = lerp_from(v1, v0, tp[1][0]);
        t.v2 = lerp_from(v1, v2, tp[1][2]);
        return push(out, n, cap, &t);
    }
    if (O[0] && O[1] && I[2]) {
        cgo_v4 v0 = t.v0, v1 = t.v1, v2 = t.v2;
        t.v1 = lerp_from(v2, v1, tp[2][1]);
        t.v0 = lerp_from(v2, v0, tp[2][0]);
        return push(out, n, cap, &t);
    }
    if (I[0] && I[1] && O[2]) {
        cgo_v4 p12 = lerp_from(t.v1, t.v2, tp[1][2]);
        cgo_v4 p02 = lerp_from(t.v0, t.v2, tp[0][2]);
        t.v2 = p02;
        cgo_rast_tri e = extra_tri(p02, p12, t.v1, &t);
        n = push(out, n, cap, &t);
        return push(out, n, cap, &e);
    }
    if (I[0] && O[1] && (quirk6_v02 >= 0 ? quirk6_v02 : I[2])) {
        cgo_v4 p01 = lerp_from(t.v0, t.v1, tp[0][1]);
        cgo_v4 p21 = lerp_from(t.v2, t.v1, quirk6_v02 >= 0 ? quirk6_t21 : tp[2][1]);
        t.v1 = p01;
        cgo_rast_tri e = extra_tri(p01, p21, t.v2, &t);
        n = push(out, n, cap, &t);
        return push(out, n, cap, &e);
    }
    if (O[0] && I[1] && I[2]) {
        cgo_v4 p10 = lerp_from(t.v1, t.v0, tp[1][0]);
        cgo_v4 p20 = lerp_from(t.v2, t.v0, tp[2][0]);
        t.v0 = p10;
        cgo_rast_tri e = extra_tri(p10, p20, t.v2, &t);
        n = push(out, n, cap, &t);
        return push(out, n, cap, &e);
    }
    return n;   /* all out (or NaN): dropped */
}

int cgo_rast_clip(const cgo_rast_tri *in, int cnt, int plane, const cgo_rast_params *p,
                  cgo_rast_tri *out, int cap)
{
    int n = 0;
    for (int i = 0; i < cnt; ++i) {
        const cgo_rast_tri *t = &in[i];
        if (plane == 5) {                                       /* :1497-1505 */
            if (t->v0.z > 0.01f && t->v1.z > 0.01f && t->v2.z > 0.01f) n = push(out, n, cap, t);
            continue;
        }
        if (plane == 6) {                                       /* :1507-1670 */
            float wl = 5.0f / p->focal;
            float w[3] = {t->v0.w, t->v1.w, t->v2.w};
            int I[3], O[3];
            for (int k = 0; k < 3; ++k) { I[k] = w[k] <= wl; O[k] = w[k] > wl; }
            float tp[3][3];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b)
                    tp[a][b] = (a == b) ? 0.0f : (wl - w[a]) / (w[b] - w[a]);
            float t21q = (wl - w[2]) / (w[1] - w[0]);           /* :1615 quirk */
            int q = t->v2.x <= wl;                              /* :1607 quirk */
            n = clip_cases(*t, I, O, tp, out, n, cap, q, t21q);
            continue;
        }
        clipinfo ci;
        clip_info(t, plane, p, &ci);
        n = clip_cases(*t, ci.in, ci.out, ci.tp, out, n, cap, -1, 0.0f);
    }
    return n;
}

/* ---------------------------- geometry --------------------------------- */

/* skeleton.cpp:205-241 (Draw's host part) */
int cgo_rast_geometry(const cgo_rast_params *p, cgo_rast_tri *out, int cap, cgo_v4 *light_out)
{
    cgo_rast_tri room[16], boxes[32];
    int nr, nb;
    cgo_rast_load_scene(room, &nr, boxes, &nb);
    for (int i = 0; i < nr; ++i) room[i].texture = p->setting;          /* TestModelH.h:85-129 */
    for (int i = 0; i < nb; ++i) boxes[i].texture = p->setting_boxes;   /* TestModelH.h:148-260 */
    enum { MAXT = 8192 };
    cgo_rast_tri *A = (cgo_rast_tri *)malloc(sizeof(cgo_rast_tri) * MAXT);
    cgo_rast_tri *B = (cgo_rast_tri *)malloc(sizeof(cgo_rast_tri) * MAXT);
    int n = 0;
    /* toCameraSpace (:701-716) */
    for (int i = 0; i < nr; ++i) A[n++] = room[i];
    int nbase = n;
    for (int i = 0; i < nb; ++i) A[n++] = boxes[i];
    for (int i = 0; i < n; ++i) {
        cgo_v4 *vs[3] = {&A[i].v0, &A[i].v1, &A[i].v2};
        for (int k = 0; k < 3; ++k) { *vs[k] = v4_sub(*vs[k], p->camera); vs[k]->w = 1.0f; }
    }
    cgo_v4 lightPos = v4_sub(p->light_scene, p->camera);   /* :211-212, :713-716 */
    lightPos.w = 1.0f;
    /* createShadowVolume (:1676-1722) on the boxes, appended after the room */
    int m = nbase;
    for (int i = nbase; i < n; ++i) {
        cgo_rast_tri t = A[i];
        cgo_v4 v0 = t.v0, v1 = t.v1, v2 = t.v2;
        cgo_v4 n0 = v4_muls(v4_sub(v0, lightPos), 100.0f);
        cgo_v4 n1 = v4_muls(v4_sub(v1, lightPos), 100.0f);
        cgo_v4 n2 = v4_muls(v4_sub(v2, lightPos), 100.0f);
        cgo_v3 sc = v3(-1.0f, -1.0f, -1.0f);
        cgo_rast_tri sv[7];
        sv[0] = t;
        sv[1] = mk(v0, n0, v1, sc, 0); sv[2] = mk(n0, v1, n1, sc, 0);
        sv[3] = mk(v1, n1, v2, sc, 0); sv[4] = mk(n1, v2, n2, sc, 0);
        sv[5] = mk(v2, n2, v0, sc, 0); sv[6] = mk(n2, v0, n0, sc, 0);
        for (int k = 0; k < 7; ++k) B[(m - nbase) + k] = sv[k];
        m += 7;
    }
    for (int i = 0; i < m - nbase; ++i) A[nbase + i] = B[i];
    n = m;
    /* rotate (:223-228), clip space w = z/f (:691-699) */
    lightPos = mat4_mul(p->R, lightPos);
    for (int i = 0; i < n; ++i) {
        A[i].v0 = mat4_mul(p->R, A[i].v0);
        A[i].v1 = mat4_mul(p->R, A[i].v1);
        A[i].v2 = mat4_mul(p->R, A[i].v2);
        A[i].v0.w = A[i].v0.z / p->focal;
        A[i].v1.w = A[i].v1.z / p->focal;
        A[i].v2.w = A[i].v2.z / p->focal;
    }
    /* clip planes 1..6 (:236-241) */
    for (int plane = 1; plane <= 6; ++plane) {
        int k = cgo_rast_clip(A, n, plane, p, B, MAXT);
        if (k > MAXT) k = MAXT;
        cgo_rast_tri *tmp = A; A = B; B = tmp;
        n = k;
    }
    int w = n < cap ? n : cap;
    if (out) memcpy(out, A, sizeof(cgo_rast_tri) * (size_t)w);
    if (light_out) *light_out = lightPos;
    free(A);
    free(B);
    return n;
}

/* ---------------------------- raster ----------------------------------- */

/* skeleton.cpp:510-522 */
void cgo_rast_vertex_shader(const cgo_rast_params *p, cgo_v4 v, cgo_pixel *px)
{
    float x = (p->focal * (v.x / v.z)) + (float)(p->width / 2);
    float y = (p->focal * (v.y / v.z)) + (float)(p->height / 2);
    px->x = f2i(x);
    px->y = f2i(y);
    px->zinv = 1 / v.z;
    px->pos3d = v;
}

/* skeleton.cpp:524-551 */
void cgo_rast_interpolate(cgo_pixel a, cgo_pixel b, cgo_pixel *result, int N)
{
    a.pos3d.x = a.pos3d.x * a.zinv;
    a.pos3d.y = a.pos3d.y * a.zinv;
    b.pos3d.x = b.pos3d.x * b.zinv;
    b.pos3d.y = b.pos3d.y * b.zinv;
    float den = (float)(N - 1 > 1 ? N - 1 : 1);
    float step_x = (float)(b.x - a.x) / den;
    float step_y = (float)(b.y - a.y) / den;
    float step_z = (b.zinv - a.zinv) / den;
    float sX = (b.pos3d.x - a.pos3d.x) / den;
    float sY = (b.pos3d.y - a.pos3d.y) / den;
    for (int i = 0; i < N; ++i) {
        float fi = (float)i;
        result[i].x = f2i(floorf((float)a.x + (step_x * fi)));
        result[i].y = f2i(floorf((float)a.y + (step_y * fi)));
        result[i].zinv = a.zinv + (step_z * fi);
        result[i].pos3d.z = 1 / result[i].zinv;
        result[i].pos3d.x = (a.pos3d.x + (sX * fi)) / result[i].zinv;
        result[i].pos3d.y = (a.pos3d.y + (sY * fi)) / result[i].zinv;
        result[i].pos3d.w = 1.0f;
    }
}

/* skeleton.cpp:433-498 */
int cgo_rast_polygon_rows(const cgo_pixel *vp, cgo_pixel *left, cgo_pixel *right, int cap)
{
    int mx = -INT_MAX, mn = INT_MAX;
    for (int i = 0; i < 3; ++i) {
        if (vp[i].y > mx) mx = vp[i].y;
        if (vp[i].y < mn) mn = vp[i].y;
    }
    int rows = (mx - mn) + 1;
    if (!left || !right) return rows;
    if (rows > cap || rows <= 0) return rows > 0 ? -rows : INT_MIN;
    for (int j = 0; j < rows; ++j) {
        memset(&left[j], 0, sizeof(cgo_pixel));
        memset(&right[j], 0, sizeof(cgo_pixel));
        left[j].x = INT_MAX; left[j].y = mn + j;
        right[j].x = -INT_MAX; right[j].y = mn + j;
    }
    cgo_pixel *line = 0;
    int line_cap = 0;
    for (int i = 0; i < 3; ++i) {
        cgo_pixel a = vp[i], b = vp[i == 2 ? 0 : i + 1];
        int dx = abs(a.x - b.x), dy = abs(a.y - b.y);
        int pixels = (dx > dy ? dx : dy) + 1;
        if (pixels > line_cap) {
            line_cap = pixels;
            line = (cgo_pixel *)realloc(line, sizeof(cgo_pixel) * (size_t)pixels);
        }
        cgo_rast_interpolate(a, b, line, pixels);
        for (int j = 0; j < pixels; ++j) {
            int k = line[j].y - mn;
            if (k < 0 || k >= rows) continue;   /* :485 guard (reads OOB before it in the reference) */
            if (line[j].x <= left[k].x) {
                left[k].x = line[j].x; left[k].zinv = line[j].zinv; left[k].pos3d = line[j].pos3d;
            }
            if (line[j].x >= right[k].x) {
                right[k].x = line[j].x; right[k].zinv = line[j].zinv; right[k].pos3d = line[j].pos3d;
            }
        }
    }
    free(line);
    return rows;
}

/* ---------------------------- textures --------------------------------- */

static const cgo_rast_textures *g_tex;
static uint8_t *g_grill_op, *g_woven_op;    /* thresholded gray maps (skeleton.cpp:149-155) */
static float *g_noise;                       /* normalMap_marble xyz (:158-170) */
enum { TEX_N = 1024, MARBLE_N = 2000 };

/* OpenCV 3.4 RGB2Gray<uchar> (imgproc/src/color.cpp) with blueIdx 0:
 * Y = (B*1868 + G*9617 + R*4899 + (1 << 13)) >> 14, then threshold (:154-155):
 * 255 where Y > 100, else 0. */
void cgo_rast_opacity_map(const uint8_t *bgr, int n, uint8_t *out)
{
    for (int i = 0; i < n; ++i) {
        const int y = (bgr[3 * i] * 1868 + bgr[3 * i + 1] * 9617 + bgr[3 * i + 2] * 4899 + (1 << 13)) >> 14;
        out[i] = y > 100 ? 255 : 0;
    }
}

void cgo_rast_set_textures(const cgo_rast_textures *t)
{
    free(g_grill_op); free(g_woven_op); free(g_noise);
    g_grill_op = g_woven_op = 0;
    g_noise = 0;
    g_tex = t;
    if (!t) return;
    if (t->grill_opacity) {
        g_grill_op = (uint8_t *)malloc(TEX_N * TEX_N);
        cgo_rast_opacity_map(t->grill_opacity, TEX_N * TEX_N, g_grill_op);
    }
    if (t->woven_opacity) {
        g_woven_op = (uint8_t *)malloc(TEX_N * TEX_N);
        cgo_rast_opacity_map(t->woven_opacity, TEX_N * TEX_N, g_woven_op);
    }
    if (t->marble) {   /* :158-170, the process's first rand() calls (seed 1) */
        const float LO = -0.000002f, HI = 0.000002f;
        g_noise = (float *)malloc(sizeof(float) * 3 * MARBLE_N * MARBLE_N);
        srand(1);
        for (int i = 0; i < 3 * MARBLE_N * MARBLE_N; ++i)
            g_noise[i] = LO + (float)rand() / ((float)(RAND_MAX / HI - LO));
    }
}

/* glm/detail/type_mat4x4.inl:37-90 (compute_inverse), m[4c + r] = m[c][r] */
void cgo_mat4_inverse(const float *m, float *out)
{
#define M(c, r) m[4 * (c) + (r)]
    float c00 = M(2,2) * M(3,3) - M(3,2) * M(2,3), c02 = M(1,2) * M(3,3) - M(3,2) * M(1,3);
    float c03 = M(1,2) * M(2,3) - M(2,2) * M(1,3);
    float c04 = M(2,1) * M(3,3) - M(3,1) * M(2,3), c06 = M(1,1) * M(3,3) - M(3,1) * M(1,3);
    float c07 = M(1,1) * M(2,3) - M(2,1) * M(1,3);
    float c08 = M(2,1) * M(3,2) - M(3,1) * M(2,2), c10 = M(1,1) * M(3,2) - M(3,1) * M(1,2);
    float c11 = M(1,1) * M(2,2) - M(2,1) * M(1,2);
    float c12 = M(2,0) * M(3,3) - M(3,0) * M(2,3), c14 = M(1,0) * M(3,3) - M(3,0) * M(1,3);
    float c15 = M(1,0) * M(2,3) - M(2,0) * M(1,3);
    float c16 = M(2,0) * M(3,2) - M(3,0) * M(2,2), c18 = M(1,0) * M(3,2) - M(3,0) * M(1,2);
    float c19 = M(1,0) * M(2,2) - M(2,0) * M(1,2);
    float c20 = M(2,0) * M(3,1) - M(3,0) * M(2,1), c22 = M(1,0) * M(3,1) - M(3,0) * M(1,1);
    float c23 = M(1,0) * M(2,1) - M(2,0) * M(1,1);
    const float F0[4] = {c00, c00, c02, c03}, F1[4] = {c04, c04, c06, c07}, F2[4] = {c08, c08, c10, c11};
    const float F3[4] = {c12, c12, c14, c15}, F4[4] = {c16, c16, c18, c19}, F5[4] = {c20, c20, c22, c23};
    const float V0[4] = {M(1,0), M(0,0), M(0,0), M(0,0)}, V1[4] = {M(1,1), M(0,1), M(0,1), M(0,1)};
    const float V2[4] = {M(1,2), M(0,2), M(0,2), M(0,2)}, V3[4] = {M(1,3), M(0,3), M(0,3), M(0,3)};
    float inv[4][4];
    for (int k = 0; k < 4; ++k) {
        const float sa = (k & 1) ? -1.0f : 1.0f;   /* SignA (+ - + -) */
        inv[0][k] = ((V1[k] * F0[k] - V2[k] * F1[k]) + V3[k] * F2[k]) * sa;
        inv[1][k] = ((V0[k] * F0[k] - V2[k] * F3[k]) + V3[k] * F4[k]) * -sa;   /* SignB */
        inv[2][k] = ((V0[k] * F1[k] - V1[k] * F3[k]) + V3[k] * F5[k]) * sa;
        inv[3][k] = ((V0[k] * F2[k] - V1[k] * F4[k]) + V2[k] * F5[k]) * -sa;
    }
    const float d0 = M(0,0) * inv[0][0], d1 = M(0,1) * inv[1][0], d2 = M(0,2) * inv[2][0], d3 = M(0,3) * inv[3][0];
    const float one_over = 1.0f / ((d0 + d1) + (d2 + d3));
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out[4 * c + r] = inv[c][r] * one_over;
#undef M
}

typedef struct {
    const cgo_rast_params *p;
    cgo_v4 lightPos;
    float *depth; int32_t *shadow; float *screen, *low, *high;
    float indirect;          /* the global indirectLightPowerPerArea (x component) */
    cgo_rast_counters *cnt;
    float Rinv[16];          /* glm::inverse(R) (findU/findV with yaw != 0) */
} rast_state;

/* findU / findV (skeleton.cpp:1756-1825): texel row u and column v of the
 * fragment's world position for object `index`.  A negative remainder (the
 * reference indexes the Mat out of bounds there) wraps to [0, size). */
static void find_uv(const rast_state *s, const cgo_pixel *px, int size, int index, int *u, int *v)
{
    cgo_v4 os;
    if (s->p->yaw != 0) {
        os = v4_add(mat4_mul(s->Rinv, px->pos3d), s->p->camera);
    } else {
        os = v4_add(px->pos3d, s->p->camera);
    }
    const float nh = (float)(-size / 2), h = (float)(size / 2);
    float fu = 0.0f, fv = 0.0f;
    int iu = 0, iv = 0;
    switch (index) {
    case 3: fu = (nh * os.y) + h; fv = (h * os.z) + h; break;
    case 1: fu = (nh * os.x) + h; fv = (nh * os.z) + h; break;
    case 4: fu = (nh * os.y) + h; fv = (nh * os.z) + h; break;
    case 2: fu = (nh * os.x) + h; fv = (nh * os.z) + h; break;
    case 0: fu = (nh * os.x) + h; fv = (nh * os.y) + h; break;
    default: break;
    }
    if (index >= 0 && index <= 4) { iu = f2i(fu); iv = f2i(fv); }
    iu %= size; iv %= size;
    if (iu < 0) iu += size;
    if (iv < 0) iv += size;
    *u = iu; *v = iv;
}

/* glm::normalize(vec4) = v * (1 / sqrt(dot(v, v))), dot = (x*x + y*y) + (z*z + w*w) */
static cgo_v4 normalize4(cgo_v4 v)
{
    float px = v.x * v.x, py = v.y * v.y, pz = v.z * v.z, pw = v.w * v.w;
    float inv = 1.0f / sqrtf((px + py) + (pz + pw));
    return v4(v.x * inv, v.y * inv, v.z * inv, v.w * inv);
}

/* skeleton.cpp:674-688 */
static cgo_v3 illum(const rast_state *s, const cgo_pixel *px, cgo_v4 N, float ind)
{
    cgo_v4 r = v4_sub(s->lightPos, px->pos3d);
    cgo_v3 r3 = v3(r.x, r.y, r.z);
    double a = (double)r.x * (double)r.x, b = (double)r.y * (double)r.y, c = (double)r.z * (double)r.z;
    float r_magnitude = (float)((a + b) + c);
    cgo_v3 n3 = v3(N.x, N.y, N.z);
    float vp = dot3(r3, n3);
    float m = vp > 0.0f ? vp : 0.0f;                              /* glm::max */
    float area = (float)((double)4.0f * M_PI * (double)r_magnitude);
    cgo_v3 lp = s->p->light_power;
    cgo_v3 D = v3((lp.x * m) / area, (lp.y * m) / area, (lp.z * m) / area);
    return v3_add(D, v3(ind, ind, ind));
}

void cgo_glibc_rand(uint64_t offset, int n, int32_t *out)
{
    srand(1);
    for (uint64_t k = 0; k < offset; ++k) (void)rand();
    for (int i = 0; i < n; ++i) out[i] = rand();
}

/* skeleton.cpp:563-565, 649-651: LO + rand() / (RAND_MAX/HI - LO), all float */
static inline float rand_unit(void)
{
    const float LO = 0.2f, HI = 0.5f;
    return LO + (float)rand() / ((float)(RAND_MAX / HI - LO));
}

/* skeleton.cpp:559-586, 647-671 (texture 0; colour modes 0, 1, 2) */
static void pixel_shader(rast_state *s, const cgo_pixel *px, const cgo_rast_tri *t)
{
    const int W = s->p->width, H = s->p->height;
    int x = px->x, y = px->y;
    if (!(x >= 0 && x < W && y >= 0 && y < H)) return;
    size_t o = (size_t)y * W + x;
    if (s->cnt) s->cnt->n_frags++;
    if (px->zinv >= s->depth[o] && t->color.x >= 0 && s->p->colour_mode != 0) {
        float r0 = rand_unit(), r1 = rand_unit(), r2 = rand_unit();   /* :649-651, :657-659 */
        cgo_v3 c = s->p->colour_mode == 1 ? v3(r0, r1, r2) : v3(r0 - 0.2f, 1.0f, r2 - 0.2f);
        (void)r1;
        cgo_v3 sc = v3_mul(c, illum(s, px, t->normal, s->indirect));  /* :652, :660 */
        s->screen[3 * o + 0] = sc.x; s->screen[3 * o + 1] = sc.y; s->screen[3 * o + 2] = sc.z;
        s->depth[o] = px->zinv;                                       /* :665 */
        if (s->cnt) s->cnt->n_shaded++;
    } else if (px->zinv >= s->depth[o] && t->color.x >= 0) {
        cgo_v3 c = t->color;
        cgo_v4 N = t->normal;
        float occ = 1.0f;
        const int tex = t->texture;
        if (tex == 1) {                                               /* marble :588-599 */
            int u, v;
            find_uv(s, px, MARBLE_N, t->index, &u, &v);
            const uint8_t *m = g_tex->marble + 3 * ((size_t)u * MARBLE_N + v);
            c = v3((float)m[2] / 255.0f, (float)m[1] / 255.0f, (float)m[0] / 255.0f);
            const float *nz = g_noise + 3 * ((size_t)y * MARBLE_N + x);
            N = v4_add(N, v4(nz[0], nz[1], nz[2], 0.0f));
        } else if (tex == 2 || tex == 3) {                            /* grill :600-621, woven :622-645 */
            int u, v;
            find_uv(s, px, TEX_N, t->index, &u, &v);
            const size_t k = (size_t)u * TEX_N + v;
            if ((tex == 2 ? g_grill_op : g_woven_op)[k] != 255) {
                s->depth[o] = 0.0f;                                   /* p.zinv = 0 (:619, :643), :665 */
                return;
            }
            if (tex == 3) {
                occ = (float)g_tex->woven_ao[(size_t)u * 3 * TEX_N + v];   /* at<uchar> on the BGR Mat */
                occ /= 255.0f;
            }
            const uint8_t *nm = (tex == 2 ? g_tex->grill_normal : g_tex->woven_normal) + 3 * k;
            N = normalize4(v4((float)nm[0] / 255.0f, (float)nm[1] / 255.0f, (float)nm[2] / 255.0f, 1.0f));
            const uint8_t *cm = (tex == 2 ? g_tex->grill : g_tex->woven) + 3 * k;
            c = v3((float)cm[2] / 255.0f, (float)cm[1] / 255.0f, (float)cm[0] / 255.0f);
        }
        cgo_v3 il = illum(s, px, N, s->indirect), il0 = illum(s, px, N, 0.0f * 1), il4 = illum(s, px, N, 0.4f * 1);
        if (tex == 3) {
            il = v3(il.x * occ, il.y * occ, il.z * occ);
            il0 = v3(il0.x * occ, il0.y * occ, il0.z * occ);
            il4 = v3(il4.x * occ, il4.y * occ, il4.z * occ);
        }
        cgo_v3 sc = v3_mul(c, il);
        cgo_v3 lo = v3_mul(c, il0);
        cgo_v3 hi = v3_mul(c, il4);
        s->indirect = 0.2f * 1;
        s->screen[3 * o + 0] = sc.x; s->screen[3 * o + 1] = sc.y; s->screen[3 * o + 2] = sc.z;
        s->low[3 * o + 0] = lo.x;    s->low[3 * o + 1] = lo.y;    s->low[3 * o + 2] = lo.z;
        s->high[3 * o + 0] = hi.x;   s->high[3 * o + 1] = hi.y;   s->high[3 * o + 2] = hi.z;
        s->depth[o] = px->zinv;
        if (s->cnt) s->cnt->n_shaded++;
    } else if (px->zinv > s->depth[o] && t->color.x < 0) {
        s->shadow[o] = 1;
        if (s->cnt) s->cnt->n_shadow++;
    }
}

static inline cgo_v3 ld3(const float *b, size_t o) { return v3(b[3 * o], b[3 * o + 1], b[3 * o + 2]); }

/* skeleton.cpp:203-308 */
void cgo_rast_draw(const cgo_rast_params *p, uint32_t *argb, float *depth, int32_t *shadow,
                   float *screen_buf, float *low_buf, float *high_buf, cgo_rast_counters *cnt)
{
    const int W = p->width, H = p->height;
    const size_t npx = (size_t)W * H;
    enum { CAP = 8192 };
    cgo_rast_tri *tris = (cgo_rast_tri *)malloc(sizeof(cgo_rast_tri) * CAP);
    rast_state s;
    memset(&s, 0, sizeof(s));
    s.p = p;
    s.cnt = cnt;
    cgo_mat4_inverse(p->R, s.Rinv);
    int n = cgo_rast_geometry(p, tris, CAP, &s.lightPos);
    if (n > CAP) n = CAP;
    s.depth = depth ? depth : (float *)malloc(sizeof(float) * npx);
    s.shadow = shadow ? shadow : (int32_t *)malloc(sizeof(int32_t) * npx);
    s.screen = screen_buf ? screen_buf : (float *)malloc(sizeof(float) * 3 * npx);
    s.low = low_buf ? low_buf : (float *)malloc(sizeof(float) * 3 * npx);
    s.high = high_buf ? high_buf : (float *)malloc(sizeof(float) * 3 * npx);
    uint32_t *out = argb ? argb : (uint32_t *)malloc(sizeof(uint32_t) * npx);
    memset(out, 0, sizeof(uint32_t) * npx);                  /* :244-259 */
    memset(s.depth, 0, sizeof(float) * npx);
    memset(s.screen, 0, sizeof(float) * 3 * npx);
    memset(s.low, 0, sizeof(float) * 3 * npx);
    memset(s.high, 0, sizeof(float) * 3 * npx);
    memset(s.shadow, 0, sizeof(int32_t) * npx);
    s.indirect = p->indirect_first;
    if (p->colour_mode != 0) {                                /* the frame's place in the rand() stream */
        srand(1);
        for (uint64_t k = 0; k < p->rand_offset; ++k) (void)rand();
    }
    if (cnt) cnt->n_tris += (uint64_t)n;
    cgo_pixel *left = (cgo_pixel *)malloc(sizeof(cgo_pixel) * (size_t)(H + 2) * 64);
    cgo_pixel *right = (cgo_pixel *)malloc(sizeof(cgo_pixel) * (size_t)(H + 2) * 64);
    int rcap = (H + 2) * 64;
    cgo_pixel *line = 0;
    int line_cap = 0;
    for (int i = 0; i < n; ++i) {                             /* :262-281 */
        const cgo_rast_tri *t = &tris[i];
        cgo_pixel vp[3];                                      /* DrawPolygon :420-431 */
        cgo_rast_vertex_shader(p, t->v0, &vp[0]);
        cgo_rast_vertex_shader(p, t->v1, &vp[1]);
        cgo_rast_vertex_shader(p, t->v2, &vp[2]);
        int rows = cgo_rast_polygon_rows(vp, 0, 0, 0);
        if (rows > rcap) {
            rcap = rows;
            left = (cgo_pixel *)realloc(left, sizeof(cgo_pixel) * (size_t)rows);
            right = (cgo_pixel *)realloc(right, sizeof(cgo_pixel) * (size_t)rows);
        }
        rows = cgo_rast_polygon_rows(vp, left, right, rcap);
        if (rows <= 0) continue;
        if (cnt) cnt->n_spans += (uint64_t)rows;
        for (int y = 0; y < rows; ++y) {                      /* DrawPolygonRows :500-508 */
            if (left[y].x == INT_MAX || right[y].x == -INT_MAX) continue; /* sentinel row: shades nothing */
            int N = right[y].x - left[y].x + 1;
            if (N < 1) continue;
            if (N > line_cap) {
                line_cap = N;
                line = (cgo_pixel *)realloc(line, sizeof(cgo_pixel) * (size_t)N);
            }
            cgo_rast_interpolate(left[y], right[y], line, N);
            for (int x = 0; x < N - 1; ++x) pixel_shader(&s, &line[x], t);
        }
    }
    /* post-pass (:283-307) */
    for (int y = 1; y < H - 1; ++y) {
        for (int x = 1; x < W - 1; ++x) {
            size_t o = (size_t)y * W + x;
            if (s.shadow[o] == 1) {
                /* surroundingShadowSum (:1725-1733): [y+1][x-1] twice, [y+1][x+1] never */
                int k = s.shadow[o] + s.shadow[o - W] + s.shadow[o - W - 1] + s.shadow[o - W + 1] +
                        s.shadow[o + W - 1] + s.shadow[o + W] + s.shadow[o + W - 1] + s.shadow[o - 1] +
                        s.shadow[o + 1];
                float val = (float)k;
                val /= 9.0f;
                float dk;
                if ((double)val < 0.6) dk = 0.05f;
                else if ((double)val < 0.7) dk = 0.08f;
                else if ((double)val < 0.8) dk = 0.1f;
                else if ((double)val < 0.9) dk = 0.12f;
                else dk = 0.3f;
                s.screen[3 * o + 0] -= dk; s.screen[3 * o + 1] -= dk; s.screen[3 * o + 2] -= dk;
            }
            /* antiAliasing (:1736-1753) */
            float *bufs[3] = {s.screen, s.low, s.high};
            cgo_v3 acc[3];
            for (int b = 0; b < 3; ++b) {
                cgo_v3 v = v3_add(v3_add(v3_add(v3_add(ld3(bufs[b], o), ld3(bufs[b], o - W)),
                                                ld3(bufs[b], o + W)), ld3(bufs[b], o - 1)),
                                  ld3(bufs[b], o + 1));
                acc[b] = v3(v.x / 5.0f, v.y / 5.0f, v.z / 5.0f);
            }
            cgo_v3 val = v3_add(v3_add(acc[0], acc[1]), acc[2]);
            val = v3(val.x / 3.0f, val.y / 3.0f, val.z / 3.0f);
            out[o] = cgo_put_pixel(val);
        }
    }
    free(line); free(left); free(right); free(tris);
    if (!depth) free(s.depth);
    if (!shadow) free(s.shadow);
    if (!screen_buf) free(s.screen);
    if (!low_buf) free(s.low);
    if (!high_buf) free(s.high);
    if (!argb) free(out);
}
