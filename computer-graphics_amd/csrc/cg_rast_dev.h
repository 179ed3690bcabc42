// cg_rast_dev.h -- rasteriser structures and device helpers shared by the
// colour-mode-0 pipeline (cg_rast.hip) and colour modes 1-2 (cg_rast_colour.hip).
// Reference: rasteriser/Source/skeleton.cpp.
#pragma once

#include <float.h>
#include <limits.h>

#include "cg_internal.h"

namespace cg {

struct RastArgs {
    int W, H, n;
    float focal;
    float light[3];
    float lp[3];            // lightPower
    float ind_first;        // indirectLightPowerPerArea at frame start
    int want_first;         // ind_first differs from the steady-state 0.2
    const cg_vec4 *d_light; // if set, the light comes from the device geometry
};

struct RastHdr {
    int ylo, yhi;           // visible rows [ylo, yhi] (ylo > yhi: none)
    int fy, fx;             // first shadeable fragment (if want_first), fy = INT_MAX none
};

// Ordered per-row records (one wave per screen row): for every triangle in
// order whose span on this row has a fragment on screen, a 64-byte record
// with everything the fill needs -- one scalar load per record, no
// dependent loads in the fill loop.
struct alignas(16) RowRec {
    int lx, rx;
    float lz, sz, lX, sX, lY, sY;
    int t, first_x;          // triangle index; x of the frame's first shaded fragment on this row, else -1
    int shadow;              // colour.x < 0 (shadow-volume triangle)
    float nx, ny, nz, pad0, pad1;
};
static_assert(sizeof(RowRec) == 64, "RowRec");

// calculateIllumination's direct term D (:674-683); the post-pass rebuilds
// screen/low/high = colour * (D + indirect) from it with the same ops.
__device__ __forceinline__ vec3 illum_D(const RastArgs &A, float zinv, float X, float Y, vec3 N)
{
    // Interpolate pos3d (:546-548)
    float pz = 1 / zinv;
    float px = X / zinv;
    float py = Y / zinv;
    vec3 r = v3(A.light[0] - px, A.light[1] - py, A.light[2] - pz);               // :675
    double a = (double)r.x * (double)r.x, b = (double)r.y * (double)r.y,
           c = (double)r.z * (double)r.z;
    float r2 = (float)((a + b) + c);                                              // :677
    float vp = dot(r, N);                                                         // :681
    float m = gmax(vp, 0.0f);
    float area = (float)((double)4.0f * M_PI * (double)r2);                       // :682
    return v3((A.lp[0] * m) / area, (A.lp[1] * m) / area, (A.lp[2] * m) / area);
}

// Shade state bit: the pixel's screen colour is stored directly in .yzw
// (colour modes 1-2; low/high buffers stay cleared), instead of a triangle
// index whose colour the post-pass multiplies by (D + k).
constexpr int kStateDirect = 1 << 29;

}  // namespace cg
