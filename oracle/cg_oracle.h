/*
 * cg_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's two pixel-loop hot paths
 * (fznsakib/Computer-Graphics: raytracer/Source/skeleton.cpp and
 * rasteriser/Source/skeleton.cpp), written from scratch in plain C with the
 * reference's exact IEEE operation order (GLM 0.9.7.2 association, no FMA,
 * FP64 islands where the reference promotes to double).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline.  The product
 * path (include/cg_render.h, computer-graphics_amd/) never links it.
 *
 * Pinning: the RT restatement is pinned bit-exactly by the reference's own
 * golden image raytracer/screenshot.bmp (tests/golden/rt_screenshot_320x256.bmp).
 * The RAST restatement is pinned bit-exactly by the reference's own
 * rasteriser/screenshot.bmp (tests/golden/rast_screenshot_900x720.bmp.xz):
 * at the key state that produced it (metal grill room, texels decoded as
 * OpenCV 3.4 + libjpeg 9 do, cg_oracle_jpeg.c) every pixel that does not
 * depend on the missing marble map -- 602,987 of 644,764 -- matches
 * (tests/test_rast_screenshot.py); plus the first-party ComputePolygonRows
 * KAT (rasteriser/Source/skeleton.cpp:183-199).
 */
#ifndef CG_ORACLE_H
#define CG_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float x, y, z; } cgo_v3;
typedef struct { float x, y, z, w; } cgo_v4;

/* raytracer/Source/TestModelH.h:80-115 (76 bytes, same field order). */
typedef struct { cgo_v4 v0, v1, v2, normal; cgo_v3 color; } cgo_rt_tri;
/* raytracer/Source/TestModelH.h:14-22 (44 bytes, same field order). */
typedef struct { float radius, radiusSquared; cgo_v3 centre, color, normal; } cgo_sphere;
/* raytracer/Source/skeleton.cpp:40-45 */
typedef struct { cgo_v4 position; float distance; int triangleIndex; int sphereIndex; } cgo_isect;
/* raytracer/Source/skeleton.cpp:47-50 */
typedef struct { cgo_v4 position; cgo_v3 colour; } cgo_light;

#define CGO_MAX_LIGHTS 128  /* C4: 8x8 area light; the large-scene tests: 9x9 */

/* Frame parameters = the reference's RT globals (skeleton.cpp:56-60). */
typedef struct {
    int width, height;
    float focal;
    cgo_v4 camera;
    float R[16];        /* glm::mat4, column-major: R[c*4+r] = m[c][r] */
    float indirect;     /* skeleton.cpp:110, 0.5 */
    int n_lights;
    cgo_light lights[CGO_MAX_LIGHTS];
} cgo_rt_params;

/* Work counters. */
typedef struct {
    uint64_t n_ray, n_t, n_uv, n_sph, n_dl;
} cgo_rt_counters;

int  cgo_rt_load_scene(cgo_rt_tri *tris, int cap, cgo_sphere *sph);
void cgo_rt_default_params(cgo_rt_params *p, int width, int height);
int  cgo_rt_closest(cgo_v4 start, cgo_v4 dir, const cgo_rt_tri *tris, int n_tris,
                    const cgo_sphere *sph, int n_sph, cgo_isect *out, cgo_rt_counters *cnt);
cgo_v3 cgo_rt_direct_light(const cgo_isect *i, const cgo_rt_tri *tris, int n_tris,
                           const cgo_sphere *sph, int n_sph, const cgo_light *light,
                           cgo_rt_counters *cnt);
int  cgo_sphere_solve_quadratic(float a, float b, float c, float *x0, float *x1);
int  cgo_sphere_intersect(const cgo_sphere *s, cgo_v3 start, cgo_v3 dir, float *t);
uint32_t cgo_put_pixel(cgo_v3 colour);
/* Render rows [row0,row1) of the frame into argb (full W*H buffer, row-major). */
void cgo_rt_draw(const cgo_rt_params *p, const cgo_rt_tri *tris, int n_tris,
                 const cgo_sphere *sph, int n_sph, uint32_t *argb, int row0, int row1,
                 cgo_rt_counters *cnt);
/* One pixel of Draw (skeleton.cpp:120-166). */
uint32_t cgo_rt_pixel(const cgo_rt_params *p, const cgo_rt_tri *tris, int n_tris,
                      const cgo_sphere *sph, int n_sph, int u, int v, cgo_rt_counters *cnt);
/* Pixels (xy[2k], xy[2k+1]) into out[k], k < n, over n_threads pthreads. */
void cgo_rt_draw_pixels(const cgo_rt_params *p, const cgo_rt_tri *tris, int n_tris,
                        const cgo_sphere *sph, int n_sph, const int *xy, int n, uint32_t *out,
                        int n_threads);
/* as cgo_rt_draw_pixels; *worker_cpu_s (optional) = the workers' summed own CPU time */
void cgo_rt_draw_pixels_timed(const cgo_rt_params *p, const cgo_rt_tri *tris, int n_tris,
                              const cgo_sphere *sph, int n_sph, const int *xy, int n, uint32_t *out,
                              int n_threads, double *worker_cpu_s);
/* Build-defined workloads, restated from their definition in
 * include/cg_render.h: C4 area light (n x n lights, colour/(n*n)) and the C5
 * PCG32 random scene. */
int cgo_rt_area_lights(cgo_light centre, float side, int n, cgo_light *out);
int cgo_rt_random_scene(uint64_t seed, int n, cgo_rt_tri *out);
/* Same, multithreaded by rows (pthreads); returns threads used. */
int  cgo_rt_draw_mt(const cgo_rt_params *p, const cgo_rt_tri *tris, int n_tris,
                    const cgo_sphere *sph, int n_sph, uint32_t *argb, int row0, int row1,
                    int n_threads);

/* ------------------------------- RAST --------------------------------- */

/* rasteriser/Source/TestModelH.h:13-42 (84 bytes). */
typedef struct { cgo_v4 v0, v1, v2, normal; cgo_v3 color; int texture; int index; } cgo_rast_tri;
/* rasteriser/Source/skeleton.cpp:88-94 */
typedef struct { int x, y; float zinv; cgo_v4 pos3d; } cgo_pixel;

typedef struct {
    int width, height;
    float focal;
    cgo_v4 camera;
    float R[16];
    cgo_v4 light_scene;       /* sceneCoordinatesLightPos, skeleton.cpp:52 */
    cgo_v3 light_power;       /* skeleton.cpp:53 */
    float indirect_first;     /* value of indirectLightPowerPerArea at frame start (0.15 first frame, 0.2 after) */
    int colour_mode;          /* randColourSelect (skeleton.cpp:81, :408): 0 lit colour, 1 random, 2 night vision */
    float yaw;                /* skeleton.cpp:34; findU/findV (:1756-1825) take inverse(R) when yaw != 0 */
    uint64_t rand_offset;     /* glibc rand() calls made before this frame (srand never called: seed 1) */
    int setting, setting_boxes; /* TestModelH.h:9-10: texture of the room / the boxes (0 none, 1 marble,
                                 2 metal grill, 3 woven wood); maps from cgo_rast_set_textures */
} cgo_rast_params;

/* The texture maps as the reference's cv::imread(..., CV_LOAD_IMAGE_UNCHANGED)
 * returns them (skeleton.cpp:135-146): row-major BGR, 3 bytes per texel.
 * marble 2000x2000, the rest 1024x1024; NULL = not loaded (a triangle with
 * that texture is then not renderable: the reference reads an empty Mat). */
typedef struct {
    const uint8_t *marble;
    const uint8_t *woven, *woven_ao, *woven_opacity, *woven_normal;
    const uint8_t *grill, *grill_opacity, *grill_normal;
} cgo_rast_textures;
/* Keeps the pointers (caller-owned) and builds what main() derives at start-up
 * (skeleton.cpp:148-172): the two opacity maps (cvtColor BGR2GRAY, threshold
 * 100 -> 0/255) and, with marble, the normal-noise map from the first
 * 3 * 2000 * 2000 rand() calls.  NULL clears. */
void cgo_rast_set_textures(const cgo_rast_textures *t);
/* OpenCV 3.4 cvtColor(CV_BGR2GRAY) for 8-bit BGR (fixed point, 14-bit
 * coefficients) followed by threshold(100, 255, THRESH_BINARY). */
void cgo_rast_opacity_map(const uint8_t *bgr, int n, uint8_t *out);
/* glm::inverse (glm/detail/type_mat4x4.inl:37-90), column-major m[4c + r]. */
void cgo_mat4_inverse(const float *m, float *out);

typedef struct {
    uint64_t n_tris, n_spans, n_frags, n_shaded, n_shadow;
} cgo_rast_counters;

/* n values of the process's libc rand() stream starting at call `offset`
 * (srand(1) first): the reference's own RNG, used to pin the product's
 * restatement of glibc's TYPE_3 generator. */
void cgo_glibc_rand(uint64_t offset, int n, int32_t *out);
int  cgo_rast_load_scene(cgo_rast_tri *room, int *n_room, cgo_rast_tri *boxes, int *n_boxes);
void cgo_rast_default_params(cgo_rast_params *p, int width, int height);
/* Host geometry of Draw (skeleton.cpp:205-241): returns number of clipped
 * triangles written to out (cap entries), light position (camera space,
 * rotated) to *light_out. */
int  cgo_rast_geometry(const cgo_rast_params *p, cgo_rast_tri *out, int cap, cgo_v4 *light_out);
int  cgo_rast_clip(const cgo_rast_tri *in, int n, int plane, const cgo_rast_params *p,
                   cgo_rast_tri *out, int cap);
void cgo_rast_vertex_shader(const cgo_rast_params *p, cgo_v4 v, cgo_pixel *px);
void cgo_rast_interpolate(cgo_pixel a, cgo_pixel b, cgo_pixel *result, int n);
/* Returns rows; left/right must hold >= rows entries (pass NULL to query). */
int  cgo_rast_polygon_rows(const cgo_pixel *vp, cgo_pixel *left, cgo_pixel *right, int cap);
/* Full RAST frame. Any output pointer may be NULL. Buffers W*H. screen/low/high
 * are float[3*W*H]. */
void cgo_rast_draw(const cgo_rast_params *p, uint32_t *argb, float *depth, int32_t *shadow,
                   float *screen_buf, float *low_buf, float *high_buf, cgo_rast_counters *cnt);

/* ------------------------- texture loading ----------------------------- */
/* cv::imread(path, CV_LOAD_IMAGE_UNCHANGED) of a JPEG as the reference's
 * OpenCV 3.4 + IJG libjpeg 9 build returns it (see cg_oracle_jpeg.c): BGR (or
 * gray) bytes, row-major.  0 or a negative error (-1 not a JPEG, -2 memory,
 * -3 corrupt, -4 unsupported, -5 out too small). */
int cgo_jpeg_info(const uint8_t *data, size_t n, int *w, int *h, int *nc);
int cgo_jpeg_decode(const uint8_t *data, size_t n, uint8_t *out, size_t cap);

/* ---------------------------- starfield -------------------------------- */
void cgo_starfield_init(float *stars, int n);
void cgo_starfield_update(float *stars, int n, float dt);
void cgo_starfield_draw(const float *stars, int n, int W, int H, uint32_t *argb);

#ifdef __cplusplus
}
#endif
#endif
