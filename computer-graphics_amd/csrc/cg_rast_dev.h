// cg_rast_dev.h -- rasteriser structures and device helpers shared by the
// colour-mode-0 pipeline (cg_rast.hip) and colour modes 1-2 (cg_rast_colour.hip).
// Reference: rasteriser/Source/skeleton.cpp.
#pragma once

#include <float.h>
#include <limits.h>

#include "cg_internal.h"

namespace cg {

// Texture maps on the device (cg_rast_set_textures): the BGR maps as
// cv::imread returns them, the opacity maps already gray + thresholded
// (skeleton.cpp:149-155), the marble normal noise as xyz floats (:158-170).
// A null pointer = not loaded.
struct RastTexMaps {
    const uint8_t *marble;                       // 2000 x 2000 x 3
    const float *marble_noise;                   // 2000 x 2000 x 3
    const uint8_t *woven, *woven_ao, *woven_op, *woven_nrm;   // 1024^2 x 3 (op: x 1)
    const uint8_t *grill, *grill_op, *grill_nrm;
};
constexpr int kTexN = 1024, kMarbleN = 2000;

struct RastArgs {
    int W, H, n;
    float focal;
    float light[3];
    float lp[3];            // lightPower
    float ind_first;        // indirectLightPowerPerArea at frame start
    int want_first;         // ind_first differs from the steady-state 0.2
    const cg_vec4 *d_light; // if set, the light comes from the device geometry
    // texture modes 1-3 (skeleton.cpp:588-645): only read by the TEX kernel variants
    int textured;           // some triangle may carry texture 1-3
    int use_inv;            // yaw != 0: findU/findV go through inverse(R) (:1761-1765)
    float cam[4];           // cameraPos
    float Rinv[16];         // glm::inverse(R), column-major
    RastTexMaps tx;
    int state16;            // colour mode 0: fill -> post state in 2 bytes per pixel (n < 32768)
    const cg_rtri *tris;    // the clipped triangles (normals for the shading)
};

struct RastHdr {
    int ylo, yhi;           // visible rows [ylo, yhi] (ylo > yhi: none)
    int fy, fx;             // first shadeable fragment (if want_first), fy = INT_MAX none
    unsigned t_sh;          // what the row records carry of the triangle: index | shadow volume << 31,
    int tex, index, pad;    // texture, object index
};

// Ordered per-row records (one wave per screen row): for every triangle in
// order whose span on this row has a fragment on screen, a 48-byte record
// with everything the fill needs -- no dependent loads in the fill loop (the
// shading reads the normal from the triangle, A.tris).
struct alignas(16) RowRec {
    int lx, rx;
    float lz, sz, lX, sX, lY, sY;
    unsigned t_sh;           // triangle index | shadow-volume triangle (colour.x < 0) << 31
    int first_x;             // x of the frame's first shaded fragment on this row, else -1
    int tex, index;          // the triangle's texture (0-3) and object index (findU/findV)
};
static_assert(sizeof(RowRec) == 48, "RowRec");
__device__ __forceinline__ int rec_t(const RowRec &r) { return (int)(r.t_sh & 0x7fffffffu); }
__device__ __forceinline__ int rec_shadow(const RowRec &r) { return (int)(r.t_sh >> 31); }

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

// findU / findV (skeleton.cpp:1756-1825) for a fragment with zinv and the
// interpolated pos3d numerators Xn, Yn (:546-548, the same ops as illum_D):
// texel row u, column v of a size x size map.  A negative remainder (the
// reference indexes the Mat out of bounds) wraps to [0, size).
__device__ __forceinline__ void rast_find_uv(const RastArgs &A, int index, int size, float zinv, float Xn, float Yn,
                                             int &u, int &v)
{
    float pz = 1 / zinv;
    float px = Xn / zinv;
    float py = Yn / zinv;
    float ox, oy, oz;
    if (A.use_inv) {   // inverse(R) * pos3d (w = 1), type_mat4x4.inl:615-661, then + cameraPos
        float r[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            float a0 = A.Rinv[k] * px, a1 = A.Rinv[4 + k] * py;
            float a2 = A.Rinv[8 + k] * pz, a3 = A.Rinv[12 + k] * 1.0f;
            r[k] = (a0 + a1) + (a2 + a3);
        }
        ox = r[0] + A.cam[0]; oy = r[1] + A.cam[1]; oz = r[2] + A.cam[2];
    } else {
        ox = px + A.cam[0]; oy = py + A.cam[1]; oz = pz + A.cam[2];
    }
    const float nh = (float)(-size / 2), h = (float)(size / 2);
    float fu = 0.0f, fv = 0.0f;
    switch (index) {
    case 3: fu = (nh * oy) + h; fv = (h * oz) + h; break;
    case 1: fu = (nh * ox) + h; fv = (nh * oz) + h; break;
    case 4: fu = (nh * oy) + h; fv = (nh * oz) + h; break;
    case 2: fu = (nh * ox) + h; fv = (nh * oz) + h; break;
    case 0: fu = (nh * ox) + h; fv = (nh * oy) + h; break;
    default: break;
    }
    int iu = 0, iv = 0;
    if (index >= 0 && index <= 4) {
        iu = f2i_x86(fu);
        iv = f2i_x86(fv);
    }
    iu %= size;
    iv %= size;
    u = iu < 0 ? iu + size : iu;
    v = iv < 0 ? iv + size : iv;
}

// Opacity test of textures 2 and 3 (:602, :624); textures 0-1 always shade.
// Whether texture tex's maps are on the device.  The host entries refuse a
// list with a texture whose maps are missing; a device list is not inspected
// (cg_rast_render_device), so the kernels never read a missing map: such a
// fragment shades as texture 0.
__device__ __forceinline__ bool rast_tex_present(const RastArgs &A, int tex)
{
    if (tex == 1) return A.tx.marble && A.tx.marble_noise;
    if (tex == 2) return A.tx.grill && A.tx.grill_op && A.tx.grill_nrm;
    if (tex == 3) return A.tx.woven && A.tx.woven_ao && A.tx.woven_op && A.tx.woven_nrm;
    return false;
}

__device__ __forceinline__ bool rast_opaque(const RastArgs &A, int tex, int index, float zinv, float Xn, float Yn)
{
    if ((tex != 2 && tex != 3) || !rast_tex_present(A, tex)) return true;
    int u, v;
    rast_find_uv(A, index, kTexN, zinv, Xn, Yn, u, v);
    return (tex == 2 ? A.tx.grill_op : A.tx.woven_op)[(size_t)u * kTexN + v] == 255;
}

// What a shading fragment of texture tex >= 1 reads (:588-645), for an opaque
// one: the normal calculateIllumination takes and the texel word
// B | G << 8 | R << 16 | occlusion << 24 (texture 3; textureColour and
// occlusion are rebuilt from the bytes as the reference forms them).
__device__ __forceinline__ vec3 rast_tex_normal(const RastArgs &A, int tex, int index, float zinv, float Xn, float Yn,
                                                int x, int y, vec3 Ntri, uint32_t &texel)
{
    int u, v;
    if (tex == 1) {
        rast_find_uv(A, index, kMarbleN, zinv, Xn, Yn, u, v);
        const uint8_t *m = A.tx.marble + 3 * ((size_t)u * kMarbleN + v);
        texel = (uint32_t)m[0] | ((uint32_t)m[1] << 8) | ((uint32_t)m[2] << 16);
        const float *nz = A.tx.marble_noise + 3 * ((size_t)y * kMarbleN + x);   // normalMap_marble[p.y*rows + p.x]
        return v3(Ntri.x + nz[0], Ntri.y + nz[1], Ntri.z + nz[2]);              // currentNormal + noise (w + 0)
    }
    rast_find_uv(A, index, kTexN, zinv, Xn, Yn, u, v);
    const size_t k = (size_t)u * kTexN + v;
    const uint8_t *nm = (tex == 2 ? A.tx.grill_nrm : A.tx.woven_nrm) + 3 * k;
    const uint8_t *cm = (tex == 2 ? A.tx.grill : A.tx.woven) + 3 * k;
    const uint32_t occ = tex == 3 ? A.tx.woven_ao[(size_t)u * 3 * kTexN + v] : 0u;   // at<uchar> on the BGR Mat
    texel = (uint32_t)cm[0] | ((uint32_t)cm[1] << 8) | ((uint32_t)cm[2] << 16) | (occ << 24);
    // normalize(vec4(valx, valy, valz, 1)) (:607-609, :631-634): v * (1 / sqrt(dot4))
    const float vx = (float)nm[0] / 255.0f, vy = (float)nm[1] / 255.0f, vz = (float)nm[2] / 255.0f, vw = 1.0f;
    const float d4 = ((vx * vx) + (vy * vy)) + ((vz * vz) + (vw * vw));
    const float inv = 1.0f / sqrtf(d4);
    return v3(vx * inv, vy * inv, vz * inv);
}

// Shade state bit: the pixel's screen colour is stored directly in .yzw
// (colour modes 1-2; low/high buffers stay cleared), instead of a triangle
// index whose colour the post-pass multiplies by (D + k).
constexpr int kStateDirect = 1 << 29;

}  // namespace cg
