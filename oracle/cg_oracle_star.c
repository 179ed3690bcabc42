/*
 * cg_oracle_star.c -- TEST INFRASTRUCTURE ONLY (checker).
 *
 * Plain-C restatement of starfield/Source/skeleton.cpp (main's star set-up
 * :41-46, Draw :66-79, Update :82-104) and its PutPixelSDL
 * (starfield/Source/SDLauxiliary.h:149-161).  Stars come from the C
 * library's own rand() (the reference's RNG, never seeded: seed 1).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "cg_oracle.h"

void cgo_starfield_init(float *stars, int n)
{
    srand(1);
    for (int i = 0; i < n; ++i) {                                   /* :42-45 */
        stars[3 * i + 0] = (float)(((float)rand() / (float)RAND_MAX - 0.5) * 2);
        stars[3 * i + 1] = (float)(((float)rand() / (float)RAND_MAX - 0.5) * 2);
        stars[3 * i + 2] = (float)rand() / (float)RAND_MAX;
    }
}

void cgo_starfield_update(float *stars, int n, float dt)
{
    for (int i = 0; i < n; ++i) {                                   /* :93-100 */
        float *z = &stars[3 * i + 2];
        if (*z <= 0) *z += 1;
        if (*z > 1) *z -= 1;
        *z = *z - (0.0005 * dt);
    }
}

/* x86 cvttss2si: out-of-range and NaN give INT_MIN */
static int f2i(float f)
{
    if (!(f > -2147483904.0f && f < 2147483648.0f)) return (int)0x80000000u;
    return (int)f;
}

void cgo_starfield_draw(const float *stars, int n, int W, int H, uint32_t *argb)
{
    memset(argb, 0, sizeof(uint32_t) * (size_t)W * H);              /* :69 */
    for (int i = 0; i < n; ++i) {                                   /* :73-78 */
        float x = stars[3 * i], y = stars[3 * i + 1], z = stars[3 * i + 2];
        float u = (W / 2) * (x / z) + (W / 2);
        float v = (H / 2) * (y / z) + (H / 2);
        int px = f2i(u), py = f2i(v);
        if (px < 0 || px >= W || py < 0 || py >= H) continue;       /* "apa" */
        cgo_v3 white = {1, 1, 1};
        argb[(size_t)py * W + px] = cgo_put_pixel(white);
    }
}
