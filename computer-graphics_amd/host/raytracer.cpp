// raytracer.cpp -- headless drop-in for raytracer/Source/skeleton.cpp.
//
// Same globals (focalLength, cameraPos, lights, yaw, R), same main loop
// `while (Update()) { Draw(screen); SDL_Renderframe(screen); }`, same
// Draw(screen*) writing ARGB into screen->buffer, same screenshot.bmp on
// exit.  Keyboard input is replaced by a scripted key string (one key per
// frame, letters as in Update(): w s a d q e = light, U D L R = camera
// arrows, n m = yaw, i o = focal, x = ESC).  The per-pixel loop runs on the
// GPU through the C-ABI (include/cg_render.h).
//
//   raytracer [--width W] [--height H] [--focal F] [--keys KEYS] [--out FILE]
#include <chrono>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "SDLauxiliary.h"
#include "TestModelH.h"
#include "cg_render.h"

using namespace std;
using glm::mat4;
using glm::vec3;
using glm::vec4;

// skeleton.cpp:40-50
struct Intersection {
    vec4 position;
    float distance;
    int triangleIndex;
    int sphereIndex;
};
struct Light {
    vec4 position;
    vec3 colour;
};
static_assert(sizeof(Intersection) == sizeof(cg_isect), "Intersection layout");
static_assert(sizeof(Light) == sizeof(cg_light), "Light layout");

// skeleton.cpp:56-60
int SCREEN_WIDTH = 320, SCREEN_HEIGHT = 256;
float focalLength = 256;
vec4 cameraPos(0.0, 0.0, -3.0, 1.0);
vector<Light> lights;
float yaw = 0.0;
mat4 R(1.0f);

static cg_ctx *g_ctx = nullptr;
static string g_keys;
static size_t g_frame = 0;

bool Update();
void Draw(screen *screen);

static void die(int rc, const char *what)
{
    cerr << what << " failed (" << rc << "): " << (g_ctx ? cg_last_error(g_ctx) : "") << endl;
    exit(1);
}

// skeleton.cpp:104-169: the pixel loop runs in rt_pixel_kernel.
void Draw(screen *screen)
{
    memset(screen->buffer, 0, screen->height * screen->width * sizeof(uint32_t));
    // LoadTestModel every frame as the reference does (:113-116); the scene
    // is constant, so it is uploaded to the device once.
    static bool uploaded = false;
    vector<rt::Triangle> triangles;
    vector<rt::Sphere> spheres;
    rt::LoadTestModel(triangles, spheres);
    if (!uploaded) {
        int rc = cg_rt_set_scene(g_ctx, reinterpret_cast<const cg_tri *>(triangles.data()),
                                 (int)triangles.size(),
                                 reinterpret_cast<const cg_sphere *>(spheres.data()),
                                 (int)spheres.size());
        if (rc) die(rc, "cg_rt_set_scene");
        uploaded = true;
    }
    cg_rt_camera cam;
    cam.width = screen->width;
    cam.height = screen->height;
    cam.focal = focalLength;
    cam.camera = cg_vec4{cameraPos.x, cameraPos.y, cameraPos.z, cameraPos.w};
    memcpy(cam.R, R.data(), sizeof(cam.R));
    cam.indirect = 0.5f;                                              // :110
    int rc = cg_rt_render(g_ctx, reinterpret_cast<const cg_light *>(lights.data()),
                          (int)lights.size(), &cam, screen->buffer, nullptr);
    if (rc) die(rc, "cg_rt_render");
}

// skeleton.cpp:172-260 with scripted keys
bool Update()
{
    static auto t = chrono::steady_clock::now();
    auto t2 = chrono::steady_clock::now();
    float dt = chrono::duration<float, milli>(t2 - t).count();
    t = t2;
    cout << "Render time : " << dt << " ms." << endl;
    if (g_frame >= g_keys.size()) return g_frame++ == 0;   // no keys: render one frame
    char key = g_keys[g_frame++];
    switch (key) {
    case 'w': lights[0].position += vec4(0, 0, 0.1, 0); break;
    case 's': lights[0].position += vec4(0, 0, -0.1, 0); break;
    case 'a': lights[0].position += vec4(-0.1, 0, 0, 0); break;
    case 'd': lights[0].position += vec4(0.1, 0, 0, 0); break;
    case 'q': lights[0].position += vec4(0, -0.1, 0, 0); break;
    case 'e': lights[0].position += vec4(0, 0.1, 0, 0); break;
    case 'U': cameraPos += vec4(0, 0, 0.1, 0); break;
    case 'D': cameraPos += vec4(0, 0, -0.1, 0); break;
    case 'L': cameraPos += vec4(-0.1, 0, 0, 0); break;
    case 'R': cameraPos += vec4(0.1, 0, 0, 0); break;
    case 'n':
    case 'm':
        if (key == 'n') yaw -= 0.174533;   // double literal, narrowed (:235, :241)
        else yaw += 0.174533;
        R[0][0] = cos(yaw); R[0][1] = 0; R[0][2] = -sin(yaw);
        R[1][0] = 0;        R[1][1] = 1; R[1][2] = 0;
        R[2][0] = sin(yaw); R[2][1] = 0; R[2][2] = cos(yaw);
        break;
    case 'i': focalLength += 10; break;
    case 'o': focalLength -= 10; break;
    case 'x': return false;
    default: break;
    }
    return true;
}

int main(int argc, char *argv[])
{
    string out = "screenshot.bmp";
    for (int i = 1; i + 1 < argc; i += 2) {
        string a = argv[i];
        if (a == "--width") SCREEN_WIDTH = atoi(argv[i + 1]);
        else if (a == "--height") SCREEN_HEIGHT = atoi(argv[i + 1]);
        else if (a == "--focal") focalLength = (float)atof(argv[i + 1]);
        else if (a == "--keys") g_keys = argv[i + 1];
        else if (a == "--out") out = argv[i + 1];
    }
    int rc = cg_create(0, &g_ctx);
    if (rc) die(rc, "cg_create");
    screen *screen = InitializeSDL(SCREEN_WIDTH, SCREEN_HEIGHT, false);
    Light light1;                                                     // :86-89
    light1.position = vec4(0, -0.5, -0.7, 1.0);
    light1.colour = 14.f * vec3(1, 1, 1);
    lights.push_back(light1);
    while (Update()) {
        Draw(screen);
        SDL_Renderframe(screen);
    }
    SDL_SaveImage(screen, out.c_str());
    KillSDL(screen);
    cg_destroy(g_ctx);
    return 0;
}
