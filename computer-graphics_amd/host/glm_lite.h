// glm_lite.h -- the few GLM types/ops the host surface needs (vec3, vec4,
// mat4 with m[col][row], clamp), layout-identical to GLM 0.9.7.2's highp
// float types and to the C-ABI's cg_vec3/cg_vec4.  Arithmetic associates as
// GLM does (func_common.inl:409-456 for min/max/clamp).
#pragma once

#include <cmath>

namespace glm {

struct vec3 {
    float x, y, z;
    vec3() : x(0), y(0), z(0) {}
    vec3(float a, float b, float c) : x(a), y(b), z(c) {}
    vec3 &operator+=(const vec3 &o) { x += o.x; y += o.y; z += o.z; return *this; }
    vec3 &operator-=(const vec3 &o) { x -= o.x; y -= o.y; z -= o.z; return *this; }
};
inline vec3 operator*(float s, const vec3 &v) { return vec3(s * v.x, s * v.y, s * v.z); }

struct vec4 {
    float x, y, z, w;
    vec4() : x(0), y(0), z(0), w(0) {}
    vec4(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
    float &operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
    vec4 &operator+=(const vec4 &o) { x += o.x; y += o.y; z += o.z; w += o.w; return *this; }
};

struct mat4 {
    vec4 c[4];
    explicit mat4(float d = 1.0f)
    {
        for (int i = 0; i < 4; ++i) c[i] = vec4(i == 0 ? d : 0, i == 1 ? d : 0, i == 2 ? d : 0, i == 3 ? d : 0);
    }
    vec4 &operator[](int i) { return c[i]; }
    const vec4 &operator[](int i) const { return c[i]; }
    const float *data() const { return &c[0].x; }
};

inline float min(float x, float y) { return x < y ? x : y; }
inline float max(float x, float y) { return x > y ? x : y; }
inline float clamp(float x, float lo, float hi) { return min(max(x, lo), hi); }

}  // namespace glm
