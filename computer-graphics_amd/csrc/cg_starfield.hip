// cg_starfield.hip -- the starfield program (starfield/Source/skeleton.cpp): 1000
// stars from glibc rand() (:41-46), projected and plotted white every frame
// (Draw :66-79, PutPixelSDL SDLauxiliary.h:149-161), drifting in z (Update :82-104).
// Stars are (x, y, z) float triples; host-side init/update, device draw.
#include "cg_internal.h"

namespace cg {
void *ctx_buf(cg_ctx *c, int which, size_t bytes, hipError_t *e);
int ctx_fail(cg_ctx *c, hipError_t e, const char *what);
hipStream_t ctx_stream(cg_ctx *c);
}  // namespace cg

using namespace cg;

extern "C" int cg_glibc_rand(uint64_t offset, int n, int32_t *out);

// :41-46 -- (float(rand()) / float(RAND_MAX) - 0.5) * 2 is evaluated in double
extern "C" int cg_starfield_init(float *stars, int n)
{
    if (n < 0 || (n && !stars)) return CG_E_INVALID;
    if (n == 0) return CG_OK;
    int32_t *r = new (std::nothrow) int32_t[3 * (size_t)n];
    if (!r) return CG_E_INVALID;
    cg_glibc_rand(0, 3 * n, r);
    const float rmax = (float)2147483647;                 // float(RAND_MAX)
    for (int i = 0; i < n; ++i) {
        stars[3 * i + 0] = (float)(((double)((float)r[3 * i + 0] / rmax) - 0.5) * 2);
        stars[3 * i + 1] = (float)(((double)((float)r[3 * i + 1] / rmax) - 0.5) * 2);
        stars[3 * i + 2] = (float)r[3 * i + 2] / rmax;
    }
    delete[] r;
    return CG_OK;
}

// Update (:82-104) for a frame time dt (ms; the reference's float(t2 - t))
extern "C" int cg_starfield_update(float *stars, int n, float dt)
{
    if (n < 0 || (n && !stars)) return CG_E_INVALID;
    for (int i = 0; i < n; ++i) {
        float z = stars[3 * i + 2];
        if (z <= 0) z += 1;
        if (z > 1) z -= 1;
        stars[3 * i + 2] = (float)((double)z - (0.0005 * (double)dt));
    }
    return CG_OK;
}

namespace cg {

__global__ void star_clear_kernel(uint32_t *argb, int npx)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < npx) argb[i] = 0u;                             // :69 memset
}

// Draw (:66-79): u = (W/2)(x/z) + W/2, v likewise; PutPixelSDL truncates to int
// (x86 cvttss2si) and skips pixels off the screen.  Coinciding stars write
// the same white pixel.
__global__ void star_draw_kernel(const float *__restrict__ stars, int n, int W, int H, uint32_t *argb)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = stars[3 * i], y = stars[3 * i + 1], z = stars[3 * i + 2];
    const float u = ((float)(W / 2) * (x / z)) + (float)(W / 2);
    const float v = ((float)(H / 2) * (y / z)) + (float)(H / 2);
    const int px = f2i_x86(u), py = f2i_x86(v);
    if (px < 0 || px >= W || py < 0 || py >= H) return;   // "apa"
    argb[(size_t)py * W + px] = put_pixel(v3(1.0f, 1.0f, 1.0f));
}

}  // namespace cg

// One starfield frame into the caller's W*H ARGB buffer (Draw :66-79).
extern "C" int cg_starfield_draw(cg_ctx *c, const float *stars, int n, int width, int height, uint32_t *argb)
{
    if (!c || n < 0 || (n && !stars) || !argb || width <= 0 || height <= 0) return CG_E_INVALID;
    hipError_t e;
    const size_t npx = (size_t)width * height;
    float *d_st = (float *)ctx_buf(c, 14, (size_t)(n > 0 ? n : 1) * 3 * sizeof(float), &e);
    if (!d_st) return ctx_fail(c, e, "alloc stars");
    uint32_t *d_px = (uint32_t *)ctx_buf(c, 15, npx * sizeof(uint32_t), &e);
    if (!d_px) return ctx_fail(c, e, "alloc starfield frame");
    hipStream_t st = ctx_stream(c);
    if (n && (e = hipMemcpyAsync(d_st, stars, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice, st)) != hipSuccess)
        return ctx_fail(c, e, "upload stars");
    hipLaunchKernelGGL(star_clear_kernel, dim3((unsigned)((npx + 255) / 256)), dim3(256), 0, st, d_px, (int)npx);
    if (n) hipLaunchKernelGGL(star_draw_kernel, dim3((n + 255) / 256), dim3(256), 0, st, d_st, n, width, height, d_px);
    if ((e = hipGetLastError()) != hipSuccess) return ctx_fail(c, e, "starfield launch");
    if ((e = hipMemcpyAsync(argb, d_px, npx * sizeof(uint32_t), hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return ctx_fail(c, e, "starfield frame");
    return CG_OK;
}
