/*
 * cg_oracle_rt.c -- TEST INFRASTRUCTURE ONLY (checker + CPU baseline).
 *
 * Plain-C restatement of the reference raytracer's per-pixel loop.  Each
 * function cites the reference file:line it follows.  Every float op is one
 * IEEE binary32 op in the reference's association (GLM 0.9.7.2 scalar path,
 * see SURVEY.md Appendix A); doubles appear exactly where the reference
 * promotes.  Build with -O2 -ffp-contract=off and no -march (no FMA).
 *
 * Pinned bit-exactly against raytracer/screenshot.bmp (camera z = -2.9),
 * see tests/test_oracle.py.
 */
#include "cg_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <time.h>
#include <string.h>

/* ---- GLM subset (glm/detail/func_geometric.inl, func_matrix.inl) ---- */

static inline cgo_v3 v3(float x, float y, float z) { cgo_v3 r = {x, y, z}; return r; }
static inline cgo_v4 v4(float x, float y, float z, float w) { cgo_v4 r = {x, y, z, w}; return r; }
static inline cgo_v3 v3_sub(cgo_v3 a, cgo_v3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline cgo_v3 v3_mul(cgo_v3 a, cgo_v3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline cgo_v3 v3_add(cgo_v3 a, cgo_v3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline cgo_v3 v3_muls(cgo_v3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline cgo_v3 v3_divs(cgo_v3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline cgo_v4 v4_sub(cgo_v4 a, cgo_v4 b) { return v4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
static inline cgo_v4 v4_add(cgo_v4 a, cgo_v4 b) { return v4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
static inline cgo_v4 v4_muls(cgo_v4 a, float s) { return v4(a.x * s, a.y * s, a.z * s, a.w * s); }

/* func_geometric.inl:64-72: tmp = x*y; tmp.x + tmp.y + tmp.z */
static inline float dot3(cgo_v3 a, cgo_v3 b)
{
    float px = a.x * b.x, py = a.y * b.y, pz = a.z * b.z;
    return (px + py) + pz;
}
/* func_geometric.inl:94-100 */
static inline float length3(cgo_v3 v) { return sqrtf(dot3(v, v)); }
/* func_geometric.inl:153-159 + func_exponential.inl:149-153: v * (1/sqrt(dot)) */
static inline cgo_v3 normalize3(cgo_v3 v)
{
    float inv = 1.0f / sqrtf(dot3(v, v));
    return v3_muls(v, inv);
}
/* func_geometric.inl:133-142 */
static inline cgo_v3 cross3(cgo_v3 x, cgo_v3 y)
{
    return v3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
/* func_matrix.inl:230-240 with mat3(c0,c1,c2): m[i][j] = ci[j] */
static inline float det3(cgo_v3 c0, cgo_v3 c1, cgo_v3 c2)
{
    float a = c0.x * (c1.y * c2.z - c2.y * c1.z);
    float b = c1.x * (c0.y * c2.z - c2.y * c0.z);
    float c = c2.x * (c0.y * c1.z - c1.y * c0.z);
    return (a - b) + c;
}
/* type_mat4x4.inl:615-661: (m0*v.x + m1*v.y) + (m2*v.z + m3*v.w) */
static inline cgo_v4 mat4_mul(const float *m, cgo_v4 v)
{
    float r[4];
    for (int k = 0; k < 4; ++k) {
        float a0 = m[0 * 4 + k] * v.x;
        float a1 = m[1 * 4 + k] * v.y;
        float a2 = m[2 * 4 + k] * v.z;
        float a3 = m[3 * 4 + k] * v.w;
        r[k] = (a0 + a1) + (a2 + a3);
    }
    return v4(r[0], r[1], r[2], r[3]);
}
static inline cgo_v3 xyz(cgo_v4 v) { return v3(v.x, v.y, v.z); }

/* ---- Scene: raytracer/Source/TestModelH.h ---- */

/* TestModelH.h:96-105 */
static void compute_normal(cgo_rt_tri *t)
{
    cgo_v3 e1 = v3(t->v1.x - t->v0.x, t->v1.y - t->v0.y, t->v1.z - t->v0.z);
    cgo_v3 e2 = v3(t->v2.x - t->v0.x, t->v2.y - t->v0.y, t->v2.z - t->v0.z);
    cgo_v3 n = normalize3(cross3(e2, e1));
    t->normal = v4(n.x, n.y, n.z, 1.0f);
}

static cgo_rt_tri mk_tri(cgo_v4 a, cgo_v4 b, cgo_v4 c, cgo_v3 col)
{
    cgo_rt_tri t;
    t.v0 = a; t.v1 = b; t.v2 = c; t.color = col;
    compute_normal(&t);
    return t;
}

/* TestModelH.h:121-279: 28 triangles (room 10, short block 10, tall block 8) + 1 sphere. */
int cgo_rt_load_scene(cgo_rt_tri *tris, int cap, cgo_sphere *sph)
{
    if (cap < 28) return -1;
    const cgo_v3 red = {0.75f, 0.15f, 0.15f}, yellow = {0.75f, 0.75f, 0.15f},
                 green = {0.15f, 0.75f, 0.15f}, cyan = {0.15f, 0.75f, 0.75f},
                 blue = {0.15f, 0.15f, 0.75f}, purple = {0.75f, 0.15f, 0.75f},
                 white = {0.75f, 0.75f, 0.75f};
    float L = 555;
    int n = 0;
    cgo_v4 A = {L, 0, 0, 1}, B = {0, 0, 0, 1}, C = {L, 0, L, 1}, D = {0, 0, L, 1};
    cgo_v4 E = {L, L, 0, 1}, F = {0, L, 0, 1}, G = {L, L, L, 1}, H = {0, L, L, 1};
    tris[n++] = mk_tri(C, B, A, green);  tris[n++] = mk_tri(C, D, B, green);
    tris[n++] = mk_tri(A, E, C, purple); tris[n++] = mk_tri(C, E, G, purple);
    tris[n++] = mk_tri(F, B, D, yellow); tris[n++] = mk_tri(H, F, D, yellow);
    tris[n++] = mk_tri(E, F, G, cyan);   tris[n++] = mk_tri(F, H, G, cyan);
    tris[n++] = mk_tri(G, D, C, white);  tris[n++] = mk_tri(G, H, D, white);
    /* short block (:178-206) */
    A = v4(290, 0, 114, 1); B = v4(130, 0, 65, 1); C = v4(240, 0, 272, 1); D = v4(82, 0, 225, 1);
    E = v4(290, 165, 114, 1); F = v4(130, 165, 65, 1); G = v4(240, 165, 272, 1); H = v4(82, 165, 225, 1);
    tris[n++] = mk_tri(E, B, A, red); tris[n++] = mk_tri(E, F, B, red);
    tris[n++] = mk_tri(F, D, B, red); tris[n++] = mk_tri(F, H, D, red);
    tris[n++] = mk_tri(H, C, D, red); tris[n++] = mk_tri(H, G, C, red);
    tris[n++] = mk_tri(G, E, C, red); tris[n++] = mk_tri(E, A, C, red);
    tris[n++] = mk_tri(G, F, E, red); tris[n++] = mk_tri(G, H, F, red);
    /* tall block (:212-240), back face commented out in the reference */
    A = v4(423, 0, 247, 1); B = v4(265, 0, 296, 1); C = v4(472, 0, 406, 1); D = v4(314, 0, 456, 1);
    E = v4(423, 330, 247, 1); F = v4(265, 330, 296, 1); G = v4(472, 330, 406, 1); H = v4(314, 330, 456, 1);
    tris[n++] = mk_tri(E, B, A, blue); tris[n++] = mk_tri(E, F, B, blue);
    tris[n++] = mk_tri(F, D, B, blue); tris[n++] = mk_tri(F, H, D, blue);
    tris[n++] = mk_tri(G, E, C, blue); tris[n++] = mk_tri(E, A, C, blue);
    tris[n++] = mk_tri(G, F, E, blue); tris[n++] = mk_tri(G, H, F, blue);
    /* scale to [-1,1]^3 (:246-269) */
    float s = 2 / L;
    for (int i = 0; i < n; ++i) {
        cgo_v4 *vs[3] = {&tris[i].v0, &tris[i].v1, &tris[i].v2};
        for (int k = 0; k < 3; ++k) {
            cgo_v4 v = v4_muls(*vs[k], s);
            v = v4_sub(v, v4(1, 1, 1, 1));
            v.x *= -1; v.y *= -1; v.w = 1.0f;
            *vs[k] = v;
        }
        compute_normal(&tris[i]);
    }
    /* sphere (:275-277), Sphere ctor :17-18 */
    if (sph) {
        float r = 0.3f;
        sph->radius = r;
        sph->radiusSquared = r * r;
        sph->centre = v3(-0.45f, 0.6f, -0.6f);
        sph->color = white;
        sph->normal = v3(0, 0, 0);
    }
    return n;
}

void cgo_rt_default_params(cgo_rt_params *p, int width, int height)
{
    memset(p, 0, sizeof(*p));
    p->width = width;
    p->height = height;
    p->focal = 256.0f;                       /* skeleton.cpp:56 */
    p->camera = v4(0.0f, 0.0f, -3.0f, 1.0f); /* :57 */
    for (int k = 0; k < 16; ++k) p->R[k] = (k % 5 == 0) ? 1.0f : 0.0f; /* :60 */
    p->indirect = 0.5f;                      /* :110 */
    p->n_lights = 1;                         /* :86-89 */
    p->lights[0].position = v4(0.0f, -0.5f, -0.7f, 1.0f);
    p->lights[0].colour = v3(14.f * 1, 14.f * 1, 14.f * 1);
}

/* TestModelH.h:24-40 */
int cgo_sphere_solve_quadratic(float a, float b, float c, float *x0, float *x1)
{
    float fa = 4 * a;
    float discriminant = (b * b) - (fa * c);
    if (discriminant < 0) return 0;
    else if (discriminant == 0) {
        /* -0.5 * b / a in double, narrowed on assignment */
        *x1 = (float)((-0.5 * (double)b) / (double)a);
        *x0 = *x1;
    } else {
        float q;
        if (b > 0) q = (float)(-0.5 * (double)(b + sqrtf(discriminant)));
        else       q = (float)(-0.5 * (double)(b - sqrtf(discriminant)));
        *x0 = q / a;
        *x1 = c / q;
    }
    if (*x0 > *x1) { float t = *x0; *x0 = *x1; *x1 = t; }
    return 1;
}

/* TestModelH.h:43-66 */
int cgo_sphere_intersect(const cgo_sphere *s, cgo_v3 start, cgo_v3 dir, float *t)
{
    float t0, t1;
    cgo_v3 L = v3_sub(start, s->centre);
    float a = dot3(dir, dir);
    float b = 2 * dot3(dir, L);
    float c = dot3(L, L) - s->radiusSquared;
    if (!cgo_sphere_solve_quadratic(a, b, c, &t0, &t1)) return 0;
    if (t0 > t1) { float tmp = t0; t0 = t1; t1 = tmp; }
    if (t0 < 0) {
        t0 = t1;
        if (t0 < 0) return 0;
    }
    *t = t0;
    return 1;
}

/* The three per-ray functions below take an optional work counter.  Each is an
 * always-inline body plus a public wrapper that calls it with cnt or with a
 * constant NULL, so the uncounted copy (the CPU baseline) carries no counter
 * tests in its loops -- the reference has none (measured 4 % at 320x256). */
#define CGO_INLINE static inline __attribute__((always_inline))

/* raytracer/Source/skeleton.cpp:263-363 */
CGO_INLINE int rt_closest(cgo_v4 start, cgo_v4 dir, const cgo_rt_tri *tris, int n_tris,
                          const cgo_sphere *sph, int n_sph, cgo_isect *ci, cgo_rt_counters *cnt)
{
    const float bound = FLT_MAX;
    ci->distance = bound;
    cgo_v3 start3 = xyz(start);
    cgo_v3 dir3 = xyz(dir);
    cgo_v3 ndir = v3(-dir3.x, -dir3.y, -dir3.z);
    if (cnt) cnt->n_ray++;
    for (int i = 0; i < n_tris; ++i) {
        cgo_v4 v0 = tris[i].v0, v1 = tris[i].v1, v2 = tris[i].v2;
        cgo_v3 e1 = v3(v1.x - v0.x, v1.y - v0.y, v1.z - v0.z);
        cgo_v3 e2 = v3(v2.x - v0.x, v2.y - v0.y, v2.z - v0.z);
        cgo_v4 sol = v4_sub(start, v0);
        cgo_v3 sol3 = xyz(sol);
        float det = det3(ndir, e1, e2);                   /* :289, :306 */
        float t = det3(sol3, e1, e2) / det;               /* :305-306 */
        float distance = t * length3(dir3);               /* :307 */
        if (cnt) cnt->n_t++;
        if (distance < 0.0f) continue;                                   /* :311 */
        else if (distance >= ci->distance || distance > bound) continue; /* :313 */
        if (cnt) cnt->n_uv++;
        float u = det3(ndir, sol3, e2) / det;             /* :317-318 */
        float v = det3(ndir, e1, sol3) / det;             /* :320-321 */
        cgo_v3 td = v3_muls(dir3, t);
        cgo_v4 position = v4_add(start, v4(td.x, td.y, td.z, 0));        /* :326 */
        int check = (u >= 0) && (v >= 0) && ((u + v) <= 1);              /* :328 */
        if (check) {
            ci->position = position;
            ci->distance = distance;
            ci->triangleIndex = i;
            ci->sphereIndex = -1;
        }
    }
    for (int i = 0; i < n_sph; ++i) {                                    /* :341-355 */
        float t;
        if (cnt) cnt->n_sph++;
        if (cgo_sphere_intersect(&sph[i], start3, dir3, &t)) {
            cgo_v3 td = v3_muls(dir3, t);
            cgo_v4 position = v4_add(start, v4(td.x, td.y, td.z, 0));
            if (t < ci->distance) {
                ci->position = position;
                ci->distance = t;
                ci->triangleIndex = -1;
                ci->sphereIndex = i;
            }
        }
    }
    return ci->distance < bound;                                         /* :357 */
}
int cgo_rt_closest(cgo_v4 start, cgo_v4 dir, const cgo_rt_tri *tris, int n_tris,
                   const cgo_sphere *sph, int n_sph, cgo_isect *ci, cgo_rt_counters *cnt)
{
    return cnt ? rt_closest(start, dir, tris, n_tris, sph, n_sph, ci, cnt)
               : rt_closest(start, dir, tris, n_tris, sph, n_sph, ci, NULL);
}

/* raytracer/Source/skeleton.cpp:366-415 */
CGO_INLINE cgo_v3 rt_direct_light(const cgo_isect *i, const cgo_rt_tri *tris, int n_tris,
                                  const cgo_sphere *sph, int n_sph, const cgo_light *light,
                                  cgo_rt_counters *cnt)
{
    cgo_v3 objectColor;
    cgo_v4 normal;
    cgo_v4 r = v4_sub(light->position, i->position);
    /* :371 sqrt(pow(r0,2)+pow(r1,2)+pow(r2,2)) in double, narrowed */
    double r0 = (double)r.x * (double)r.x, r1 = (double)r.y * (double)r.y,
           r2 = (double)r.z * (double)r.z;
    float r_magnitude = (float)sqrt((r0 + r1) + r2);
    cgo_v4 direction = v4_sub(light->position, i->position);
    if (cnt) cnt->n_dl++;
    if (i->triangleIndex != -1) {
        objectColor = tris[i->triangleIndex].color;
        normal = tris[i->triangleIndex].normal;
    } else {
        const cgo_sphere *s = &sph[i->sphereIndex];
        objectColor = s->color;
        cgo_v3 n3 = normalize3(v3_sub(xyz(i->position), s->centre)); /* TestModelH.h:68-75 */
        normal = v4(n3.x, n3.y, n3.z, 0);
    }
    cgo_isect sh;
    cgo_v4 origin = v4_add(i->position, v4_muls(normal, 0.00001f));   /* :394 */
    if (rt_closest(origin, direction, tris, n_tris, sph, n_sph, &sh, cnt)) {
        if (sh.distance < r_magnitude) return v3(0.0f, 0.0f, 0.0f);   /* :395-396 */
    }
    cgo_v3 nd = normalize3(xyz(direction));                           /* :400 */
    float a = dot3(nd, xyz(normal));                                  /* :403 */
    float b = (float)(4 * M_PI);                                      /* :404 */
    float surfaceArea = (float)((double)b * ((double)r_magnitude * (double)r_magnitude)); /* :406 */
    if (a <= 0) a = 0.f;                                              /* :409 */
    cgo_v3 power = v3_divs(v3_muls(v3_mul(objectColor, light->colour), a), surfaceArea); /* :412 */
    return power;
}
cgo_v3 cgo_rt_direct_light(const cgo_isect *i, const cgo_rt_tri *tris, int n_tris,
                           const cgo_sphere *sph, int n_sph, const cgo_light *light,
                           cgo_rt_counters *cnt)
{
    return cnt ? rt_direct_light(i, tris, n_tris, sph, n_sph, light, cnt)
               : rt_direct_light(i, tris, n_tris, sph, n_sph, light, NULL);
}

/* raytracer/Source/SDLauxiliary.h:149-161 (glm::clamp = min(max(x,lo),hi), func_common.inl:409-456) */
static inline uint32_t chan(float c)
{
    float x = 255 * c;
    float m = x > 0.f ? x : 0.f;
    float k = m < 255.f ? m : 255.f;
    return (uint32_t)k;
}
uint32_t cgo_put_pixel(cgo_v3 c)
{
    uint32_t r = chan(c.x), g = chan(c.y), b = chan(c.z);
    return (128u << 24) + (r << 16) + (g << 8) + b;
}

/* raytracer/Source/skeleton.cpp:120-166: one pixel of Draw */
CGO_INLINE uint32_t rt_pixel(const cgo_rt_params *p, const cgo_rt_tri *tris, int n_tris,
                             const cgo_sphere *sph, int n_sph, int u, int v, cgo_rt_counters *cnt)
{
    const int W = p->width, H = p->height;
    cgo_v3 indirectLight = v3(p->indirect, p->indirect, p->indirect);
    cgo_v4 dir = v4((float)(u - W / 2), (float)(v - H / 2), p->focal, 1.0f); /* :126 */
    dir = mat4_mul(p->R, dir);                                              /* :128 */
    cgo_v3 pixelColour = v3(0.0f, 0.0f, 0.0f);
    int validRay = 0;
    for (int i = -1; i <= 1; ++i) {
        for (int j = -1; j <= 1; ++j) {
            float multiplier = 0.5f;
            cgo_v4 newDir = v4(dir.x + (multiplier * (float)i),
                               dir.y + (multiplier * (float)j), p->focal, 1.0f); /* :137 */
            cgo_isect is;
            if (rt_closest(p->camera, newDir, tris, n_tris, sph, n_sph, &is, cnt)) {
                validRay = 1;
                cgo_v3 objectColor = is.triangleIndex != -1 ? tris[is.triangleIndex].color
                                                            : sph[is.sphereIndex].color;
                for (int l = 0; l < p->n_lights; ++l)
                    pixelColour = v3_add(pixelColour,
                                         rt_direct_light(&is, tris, n_tris, sph, n_sph,
                                                             &p->lights[l], cnt));
                pixelColour = v3_add(pixelColour, v3_mul(objectColor, indirectLight)); /* :156 */
            }
        }
    }
    if (validRay) return cgo_put_pixel(v3_divs(pixelColour, 9.0f));   /* :160-163 */
    return cgo_put_pixel(v3(0.0f, 0.0f, 0.0f));                       /* :165 */
}
uint32_t cgo_rt_pixel(const cgo_rt_params *p, const cgo_rt_tri *tris, int n_tris,
                      const cgo_sphere *sph, int n_sph, int u, int v, cgo_rt_counters *cnt)
{
    return cnt ? rt_pixel(p, tris, n_tris, sph, n_sph, u, v, cnt) : rt_pixel(p, tris, n_tris, sph, n_sph, u, v, NULL);
}

/* raytracer/Source/skeleton.cpp:104-169 */
void cgo_rt_draw(const cgo_rt_params *p, const cgo_rt_tri *tris, int n_tris,
                 const cgo_sphere *sph, int n_sph, uint32_t *argb, int row0, int row1,
                 cgo_rt_counters *cnt)
{
    const int W = p->width, H = p->height;
    for (int v = row0; v < row1 && v < H; v++)
        for (int u = 0; u < W; u++)
            argb[(size_t)v * W + u] = cgo_rt_pixel(p, tris, n_tris, sph, n_sph, u, v, cnt);
}

typedef struct {
    const cgo_rt_params *p; const cgo_rt_tri *tris; int n_tris;
    const cgo_sphere *sph; int n_sph; const int *xy; int n; uint32_t *out; int stride, k;
    double cpu_s;   /* this worker's own CPU time (CLOCK_THREAD_CPUTIME_ID) */
} px_job;

static double thread_cpu_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *px_worker(void *arg)
{
    px_job *j = (px_job *)arg;
    const double c0 = thread_cpu_s();
    for (int i = j->k; i < j->n; i += j->stride)
        j->out[i] = cgo_rt_pixel(j->p, j->tris, j->n_tris, j->sph, j->n_sph, j->xy[2 * i], j->xy[2 * i + 1], 0);
    j->cpu_s = thread_cpu_s() - c0;
    return 0;
}

/* Pixels xy of the frame on n_threads threads; *worker_cpu_s (optional) = the
 * sum of the workers' own CPU times (no other thread of the process counted). */
void cgo_rt_draw_pixels_timed(const cgo_rt_params *p, const cgo_rt_tri *tris, int n_tris,
                              const cgo_sphere *sph, int n_sph, const int *xy, int n, uint32_t *out,
                              int n_threads, double *worker_cpu_s)
{
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    pthread_t th[256];
    px_job jobs[256];
    for (int k = 0; k < n_threads; ++k) {
        jobs[k] = (px_job){p, tris, n_tris, sph, n_sph, xy, n, out, n_threads, k, 0.0};
        if (k) pthread_create(&th[k], 0, px_worker, &jobs[k]);
    }
    px_worker(&jobs[0]);
    for (int k = 1; k < n_threads; ++k) pthread_join(th[k], 0);
    if (worker_cpu_s) {
        double t = 0.0;
        for (int k = 0; k < n_threads; ++k) t += jobs[k].cpu_s;
        *worker_cpu_s = t;
    }
}

void cgo_rt_draw_pixels(const cgo_rt_params *p, const cgo_rt_tri *tris, int n_tris,
                        const cgo_sphere *sph, int n_sph, const int *xy, int n, uint32_t *out,
                        int n_threads)
{
    cgo_rt_draw_pixels_timed(p, tris, n_tris, sph, n_sph, xy, n, out, n_threads, 0);
}

/* ---- build-defined workloads ---- */

/* C4: cell centres of an n x n grid over a side x side square in the xz-plane */
int cgo_rt_area_lights(cgo_light centre, float side, int n, cgo_light *out)
{
    if (n <= 0 || n * n > CGO_MAX_LIGHTS) return -1;
    float share = 1.0f / (float)(n * n);
    for (int j = 0; j < n; ++j) {
        for (int i = 0; i < n; ++i) {
            float fx = ((float)i + 0.5f) / (float)n - 0.5f;
            float fz = ((float)j + 0.5f) / (float)n - 0.5f;
            cgo_light *l = &out[j * n + i];
            l->position = centre.position;
            l->position.x = centre.position.x + side * fx;
            l->position.z = centre.position.z + side * fz;
            l->colour = v3_muls(centre.colour, share);
        }
    }
    return n * n;
}

/* C5: PCG32 XSH-RR (O'Neill's pcg32_random_r / pcg32_srandom_r) */
typedef struct { uint64_t s, inc; } pcg_t;
static uint32_t pcg_step(pcg_t *g)
{
    uint64_t x = g->s;
    g->s = x * 6364136223846793005ull + g->inc;
    uint32_t sh = (uint32_t)(((x >> 18) ^ x) >> 27), r = (uint32_t)(x >> 59);
    return (sh >> r) | (sh << ((32u - r) & 31u));
}
static float pcg_unif(pcg_t *g, float lo, float hi)
{
    float u = (float)(pcg_step(g) >> 8) / 16777216.0f;
    return lo + (hi - lo) * u;
}
int cgo_rt_random_scene(uint64_t seed, int n, cgo_rt_tri *out)
{
    pcg_t g = {0u, (54u << 1) | 1u};
    pcg_step(&g);
    g.s += seed;
    pcg_step(&g);
    for (int k = 0; k < n; ++k) {
        float c[3];
        for (int a = 0; a < 3; ++a) c[a] = pcg_unif(&g, -1.0f, 1.0f);
        cgo_v4 *vs[3] = {&out[k].v0, &out[k].v1, &out[k].v2};
        for (int q = 0; q < 3; ++q) {
            float o[3];
            for (int a = 0; a < 3; ++a) o[a] = pcg_unif(&g, -0.02f, 0.02f);
            *vs[q] = v4(c[0] + o[0], c[1] + o[1], c[2] + o[2], 1.0f);
        }
        float col[3];
        for (int a = 0; a < 3; ++a) col[a] = pcg_unif(&g, 0.15f, 0.75f);
        out[k].color = v3(col[0], col[1], col[2]);
        compute_normal(&out[k]);
    }
    return n;
}

typedef struct {
    const cgo_rt_params *p; const cgo_rt_tri *tris; int n_tris;
    const cgo_sphere *sph; int n_sph; uint32_t *argb; int row0, row1, stride, k;
} mt_job;

static void *mt_worker(void *arg)
{
    mt_job *j = (mt_job *)arg;
    /* interleaved rows: cost varies strongly by row */
    for (int v = j->row0 + j->k; v < j->row1; v += j->stride)
        cgo_rt_draw(j->p, j->tris, j->n_tris, j->sph, j->n_sph, j->argb, v, v + 1, 0);
    return 0;
}

int cgo_rt_draw_mt(const cgo_rt_params *p, const cgo_rt_tri *tris, int n_tris,
                   const cgo_sphere *sph, int n_sph, uint32_t *argb, int row0, int row1,
                   int n_threads)
{
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    pthread_t th[256];
    mt_job jobs[256];
    for (int k = 0; k < n_threads; ++k) {
        jobs[k] = (mt_job){p, tris, n_tris, sph, n_sph, argb, row0, row1, n_threads, k};
        if (k) pthread_create(&th[k], 0, mt_worker, &jobs[k]);
    }
    mt_worker(&jobs[0]);
    for (int k = 1; k < n_threads; ++k) pthread_join(th[k], 0);
    return n_threads;
}
