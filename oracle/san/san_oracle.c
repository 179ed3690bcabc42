/*
 * TEST INFRASTRUCTURE ONLY: drives the CPU restatement under
 * -fsanitize=address,undefined (oracle/Makefile `sanitize`), over the inputs
 * whose reference code paths carry undefined behaviour or edge cases:
 *  - ComputePolygonRows sentinel rows (rasteriser/Source/skeleton.cpp:456-459)
 *    and DrawPolygonRows' N = right.x - left.x + 1 (:502), which overflows on
 *    an untouched row in the reference; the restatement skips such rows;
 *  - the box face with an uninitialised `index` (TestModelH.h:256) in texture
 *    modes, and findU/findV's negative remainders (:1756-1825);
 *  - clipping near and across every frustum plane (yawed, moved cameras,
 *    the plane-6 quirks :1607/:1615);
 *  - the JPEG decoder on the reference's textures and on truncated /
 *    corrupted copies;
 *  - the raytracer at small sizes (sphere tangency, FP64 islands), glibc rand().
 * Usage: san_oracle TEXTURE_DIR    (exit 0 = clean; the sanitizers abort otherwise)
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../cg_oracle.h"

static uint8_t *slurp(const char *dir, const char *name, size_t *n)
{
    char path[1024];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long len = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *b = malloc((size_t)len);
    if (fread(b, 1, (size_t)len, f) != (size_t)len) { free(b); fclose(f); return NULL; }
    fclose(f);
    *n = (size_t)len;
    return b;
}

static uint8_t *decode(const char *dir, const char *name)
{
    size_t n = 0;
    uint8_t *jpg = slurp(dir, name, &n);
    if (!jpg) { fprintf(stderr, "missing %s\n", name); exit(2); }
    int w, h, c;
    if (cgo_jpeg_info(jpg, n, &w, &h, &c)) { fprintf(stderr, "bad %s\n", name); exit(2); }
    uint8_t *out = malloc((size_t)w * h * c);
    if (cgo_jpeg_decode(jpg, n, out, (size_t)w * h * c)) { fprintf(stderr, "decode %s\n", name); exit(2); }
    /* truncated and corrupted copies must fail or decode, never fault */
    for (size_t cut = 16; cut < n; cut = cut * 3 + 7) (void)cgo_jpeg_decode(jpg, cut, out, (size_t)w * h * c);
    uint8_t *bad = malloc(n);
    memcpy(bad, jpg, n);
    for (size_t k = n / 3; k < n; k += 997) bad[k] ^= 0x5a;
    (void)cgo_jpeg_decode(bad, n, out, (size_t)w * h * c);
    (void)cgo_jpeg_decode(jpg, n, out, 10);      /* capacity too small */
    free(bad);
    free(jpg);
    return out;
}

static void yaw_R(float yaw, float *R)
{
    for (int k = 0; k < 16; ++k) R[k] = (k % 5 == 0) ? 1.0f : 0.0f;
    R[0] = cosf(yaw); R[2] = -sinf(yaw); R[8] = sinf(yaw); R[10] = cosf(yaw);
}

int main(int argc, char **argv)
{
    const char *dir = argc > 1 ? argv[1] : "tests/golden/textures";
    /* textures: grill + woven decoded, marble synthetic */
    cgo_rast_textures tx;
    memset(&tx, 0, sizeof tx);
    tx.grill = decode(dir, "Metal_Grill_002_basecolor.jpg");
    tx.grill_opacity = decode(dir, "Metal_Grill_002_opacity.jpg");
    tx.grill_normal = decode(dir, "Metal_Grill_002_normal.jpg");
    tx.woven = decode(dir, "woven1024x1024.jpg");
    tx.woven_ao = decode(dir, "Wood_wicker_003_ambientOcclusion.jpg");
    tx.woven_opacity = decode(dir, "Wood_wicker_003_opacity.jpg");
    tx.woven_normal = decode(dir, "Wood_wicker_003_normal.jpg");
    uint8_t *marble = malloc(2000u * 2000u * 3u);
    for (size_t i = 0; i < 2000u * 2000u * 3u; ++i) marble[i] = (uint8_t)(i * 2654435761u >> 24);
    tx.marble = marble;
    cgo_rast_set_textures(&tx);

    const int W = 200, H = 150;
    uint32_t *argb = malloc(sizeof(uint32_t) * W * H);
    float *depth = malloc(sizeof(float) * W * H);
    int32_t *shadow = malloc(sizeof(int32_t) * W * H);
    long frames = 0;
    /* cameras inside, outside, grazing the room and behind the near plane; every texture pairing */
    const float cams[][3] = {{0, 0, -3.001f}, {0, 0, -1.2f}, {0.9f, 0.5f, -0.2f}, {-1.8f, 0, -1.6f},
                             {0, 0, 0.95f}, {3, -2, 2}, {0, 0, -0.99f}, {0.3f, 0.99f, -3}};
    const float yaws[] = {0.0f, 0.174533f, -0.8726650476455688f, 3.0f};
    for (size_t c = 0; c < sizeof cams / sizeof cams[0]; ++c)
        for (size_t y = 0; y < sizeof yaws / sizeof yaws[0]; ++y)
            for (int tex = 0; tex < 16; tex += 5) {
                cgo_rast_params p;
                cgo_rast_default_params(&p, W, H);
                p.focal = 120.0f;
                p.camera.x = cams[c][0]; p.camera.y = cams[c][1]; p.camera.z = cams[c][2];
                p.yaw = yaws[y];
                yaw_R(p.yaw, p.R);
                p.setting = tex & 3;
                p.setting_boxes = (tex >> 2) & 3;
                p.indirect_first = (c & 1) ? 0.15f : 0.2f;
                p.colour_mode = (int)(c % 3);
                p.rand_offset = 12000000u * (c & 1);
                cgo_rast_counters cnt;
                cgo_rast_draw(&p, argb, depth, shadow, NULL, NULL, NULL, &cnt);
                ++frames;
            }
    cgo_rast_set_textures(NULL);
    /* ComputePolygonRows on degenerate / huge triangles */
    cgo_pixel vp[3] = {{5, 5, 1, {0, 0, 0, 1}}, {5, 5, 1, {0, 0, 0, 1}}, {5, 5, 1, {0, 0, 0, 1}}};
    int rows = cgo_rast_polygon_rows(vp, NULL, NULL, 0);
    cgo_pixel L[64], R[64];
    (void)cgo_rast_polygon_rows(vp, L, R, rows < 64 ? rows : 64);
    vp[1].x = 40000; vp[2].y = 30;
    rows = cgo_rast_polygon_rows(vp, NULL, NULL, 0);
    cgo_pixel *L2 = malloc(sizeof(cgo_pixel) * (size_t)rows), *R2 = malloc(sizeof(cgo_pixel) * (size_t)rows);
    (void)cgo_rast_polygon_rows(vp, L2, R2, rows);
    free(L2); free(R2);

    /* raytracer: default scene, a yawed camera and two lights, small sizes */
    cgo_rt_tri tris[64];
    cgo_sphere sph;
    int n = cgo_rt_load_scene(tris, 64, &sph);
    const int RW = 64, RH = 48;
    uint32_t *rt = malloc(sizeof(uint32_t) * RW * RH);
    for (int k = 0; k < 3; ++k) {
        cgo_rt_params p;
        cgo_rt_default_params(&p, RW, RH);
        p.focal = 48.0f;
        yaw_R(-0.174533f * (float)k, p.R);
        p.camera.z = -3.0f + 0.9f * (float)k;
        if (k == 2) {
            p.n_lights = 2;
            p.lights[1] = p.lights[0];
            p.lights[1].position.x = 0.3f;
        }
        cgo_rt_counters cnt;
        cgo_rt_draw(&p, tris, n, &sph, 1, rt, 0, RH, &cnt);
        ++frames;
    }
    cgo_rt_tri rnd[500];
    cgo_rt_random_scene(0x5EED, 500, rnd);
    {
        cgo_rt_params p;
        cgo_rt_default_params(&p, 32, 24);
        p.focal = 24.0f;
        cgo_rt_draw(&p, rnd, 500, NULL, 0, rt, 0, 24, NULL);
    }
    cgo_light area[64];
    cgo_light centre = {{0, -0.5f, -0.7f, 1}, {14, 14, 14}};
    cgo_rt_area_lights(centre, 0.1f, 8, area);
    int32_t r[64];
    cgo_glibc_rand(0, 64, r);
    cgo_glibc_rand(12345678, 64, r);
    float *stars = malloc(sizeof(float) * 3 * 100);
    uint32_t *sf = malloc(sizeof(uint32_t) * 320 * 256);
    cgo_starfield_init(stars, 100);
    for (int k = 0; k < 50; ++k) { cgo_starfield_update(stars, 100, 16.0f); cgo_starfield_draw(stars, 100, 320, 256, sf); }
    printf("sanitized oracle: %ld frames clean\n", frames);
    free(stars); free(sf); free(rt); free(argb); free(depth); free(shadow); free(marble);
    free((void *)tx.grill); free((void *)tx.grill_opacity); free((void *)tx.grill_normal); free((void *)tx.woven);
    free((void *)tx.woven_ao); free((void *)tx.woven_opacity); free((void *)tx.woven_normal);
    return 0;
}
