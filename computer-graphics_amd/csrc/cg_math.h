// cg_math.h -- the GLM 0.9.7.2 subset the two hot paths use, restated with
// the reference's exact IEEE association for both the
// host geometry and the gfx950 kernels.  Every function is one expression
// tree per component; no FMA may be formed (all sources are compiled with
// -ffp-contract=off).  Citations are to /root/reference/glm/glm/detail/.
#pragma once

#include <hip/hip_runtime.h>

#define CG_HD __host__ __device__ __forceinline__

namespace cg {

struct float3_ { float x, y, z; };
struct float4_ { float x, y, z, w; };
using vec3 = float3_;
using vec4 = float4_;

CG_HD vec3 v3(float x, float y, float z) { return vec3{x, y, z}; }
CG_HD vec4 v4(float x, float y, float z, float w) { return vec4{x, y, z, w}; }
CG_HD vec3 xyz(vec4 v) { return vec3{v.x, v.y, v.z}; }

CG_HD vec3 operator+(vec3 a, vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
CG_HD vec3 operator-(vec3 a, vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
CG_HD vec3 operator*(vec3 a, vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
CG_HD vec3 operator*(vec3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
CG_HD vec3 operator/(vec3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
CG_HD vec3 operator-(vec3 a) { return v3(-a.x, -a.y, -a.z); }   // type_vec3.inl:557-563

// x / b for the constant divisors b = 3, 5, 9 (r = fl(1/b)) without the IEEE
// divide sequence: q0 = x r corrected by one FMA residual step.  Bit-identical
// to fl(x / b) for every float x -- all 2^32 inputs checked per divisor by
// scripts/divchk.c (a zero residual keeps q0, which also preserves -0 and
// the non-finite cases).
CG_HD float div_const(float x, float b, float r)
{
    const float q0 = x * r;
    const float e = fmaf(-q0, b, x);
    return (e == 0.0f || !isfinite(x)) ? q0 : fmaf(e, r, q0);
}
CG_HD vec3 div_const(vec3 a, float b, float r)
{
    return v3(div_const(a.x, b, r), div_const(a.y, b, r), div_const(a.z, b, r));
}
CG_HD vec4 operator+(vec4 a, vec4 b) { return v4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
CG_HD vec4 operator-(vec4 a, vec4 b) { return v4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
CG_HD vec4 operator*(vec4 a, float s) { return v4(a.x * s, a.y * s, a.z * s, a.w * s); }

// func_geometric.inl:64-72 -- products first, then (x + y) + z
CG_HD float dot(vec3 a, vec3 b)
{
    float px = a.x * b.x, py = a.y * b.y, pz = a.z * b.z;
    return (px + py) + pz;
}
// func_geometric.inl:94-100
CG_HD float length(vec3 v) { return sqrtf(dot(v, v)); }
// func_geometric.inl:153-159, func_exponential.inl:149-153: v * (1 / sqrt(dot))
CG_HD vec3 normalize(vec3 v)
{
    float inv = 1.0f / sqrtf(dot(v, v));
    return v * inv;
}
// func_geometric.inl:133-142
CG_HD vec3 cross(vec3 x, vec3 y)
{
    return v3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
// func_matrix.inl:230-240 for mat3(c0, c1, c2), m[i][j] = ci[j]:
// (c0.x*(c1.y*c2.z - c2.y*c1.z) - c1.x*(c0.y*c2.z - c2.y*c0.z)) + c2.x*(c0.y*c1.z - c1.y*c0.z)
CG_HD float det3(vec3 c0, vec3 c1, vec3 c2)
{
    float a = c0.x * (c1.y * c2.z - c2.y * c1.z);
    float b = c1.x * (c0.y * c2.z - c2.y * c0.z);
    float c = c2.x * (c0.y * c1.z - c1.y * c0.z);
    return (a - b) + c;
}
// type_mat4x4.inl:641-652, column-major m[c*4 + r]: (m0*v.x + m1*v.y) + (m2*v.z + m3*v.w)
CG_HD vec4 mat4_mul(const float *m, vec4 v)
{
    vec4 r;
    float *o = &r.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float a0 = m[0 * 4 + k] * v.x, a1 = m[1 * 4 + k] * v.y;
        float a2 = m[2 * 4 + k] * v.z, a3 = m[3 * 4 + k] * v.w;
        o[k] = (a0 + a1) + (a2 + a3);
    }
    return r;
}
// func_common.inl:409-456
CG_HD float gmin(float x, float y) { return x < y ? x : y; }
CG_HD float gmax(float x, float y) { return x > y ? x : y; }

// SDLauxiliary.h:149-161: uint32_t(clamp(255*c, 0, 255)) per channel, alpha 128.
CG_HD unsigned chan8(float c)
{
    float k = gmin(gmax(255 * c, 0.f), 255.f);
    return (unsigned)k;
}
CG_HD unsigned put_pixel(vec3 c)
{
    return (128u << 24) + (chan8(c.x) << 16) + (chan8(c.y) << 8) + chan8(c.z);
}

// x86-64 cvttss2si semantics (what the reference's float->int conversions
// compile to): out-of-range and NaN give INT_MIN.  gfx950's v_cvt_i32_f32
// saturates instead, so the kernels must use this.
CG_HD int f2i_x86(float f)
{
    return (f >= -2147483648.0f && f < 2147483648.0f) ? (int)f : (int)0x80000000u;
}

}  // namespace cg
