// TestModelH.h -- the reference's scene types and LoadTestModel, host side.
// Triangle/Sphere keep the reference's field order and size (76 / 44 B for
// the raytracer, 84 B for the rasteriser's Triangle), so a vector of them is
// passed to the C-ABI without repacking.  The scene itself is built by the
// library (cg_rt_load_test_model / cg_rast_load_test_model) with the
// reference's float ops.
#pragma once

#include <vector>

#include "cg_render.h"
#include "glm_lite.h"

namespace rt {
// raytracer/Source/TestModelH.h:80-115
class Triangle {
public:
    glm::vec4 v0, v1, v2, normal;
    glm::vec3 color;
};
// raytracer/Source/TestModelH.h:14-22
class Sphere {
public:
    float radius, radiusSquared;
    glm::vec3 centre, color, normal;
};
static_assert(sizeof(Triangle) == sizeof(cg_tri), "Triangle layout");
static_assert(sizeof(Sphere) == sizeof(cg_sphere), "Sphere layout");

// raytracer/Source/TestModelH.h:121-279
inline void LoadTestModel(std::vector<Triangle> &triangles, std::vector<Sphere> &spheres)
{
    triangles.resize(64);
    spheres.resize(1);
    int n = cg_rt_load_test_model(reinterpret_cast<cg_tri *>(triangles.data()), 64,
                                  reinterpret_cast<cg_sphere *>(spheres.data()));
    triangles.resize(n > 0 ? n : 0);
}
}  // namespace rt

namespace rast {
// rasteriser/Source/TestModelH.h:13-42
class Triangle {
public:
    glm::vec4 v0, v1, v2, normal;
    glm::vec3 color;
    int texture = 0;
    int index = 0;
};
static_assert(sizeof(Triangle) == sizeof(cg_rtri), "Triangle layout");

// rasteriser/Source/TestModelH.h:48-312 (setting = settingBoxes = 0)
inline void LoadTestModel(std::vector<Triangle> &room, std::vector<Triangle> &boxes)
{
    room.resize(16);
    boxes.resize(32);
    int nr = 0, nb = 0;
    cg_rast_load_test_model(reinterpret_cast<cg_rtri *>(room.data()), 16, &nr,
                            reinterpret_cast<cg_rtri *>(boxes.data()), 32, &nb);
    room.resize(nr);
    boxes.resize(nb);
}
}  // namespace rast
