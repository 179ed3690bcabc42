// rasteriser.cpp -- headless drop-in for rasteriser/Source/skeleton.cpp
// (texture mode 0, colour mode 0).
//
// Same globals (focalLength, cameraPos, yaw, R, sceneCoordinatesLightPos,
// lightPower, indirectLightPowerPerArea, originalroom/originalbox), same
// main loop and Draw(screen*) -> screen->buffer, same screenshot.bmp.  The
// whole Draw runs on the GPU (cg_rast_draw): geometry (camera space, shadow
// volumes, clipping), span setup, ordered fill and post-pass.  (cg_rast_prepare
// + cg_rast_render keep the host-geometry split available.)  Scripted keys as
// in Update() (:311-417): w s a d q e =
// light, 1 2 = indirect, U D L R z x = camera, n m = yaw, f g = focal,
// ' ' (SPACE) = colour mode, ESC = 'X'.
// Texture modes (TestModelH.h:9-10 setting / settingBoxes, skeleton.cpp:135-170):
// --setting / --setting-boxes pick the room's / boxes' texture, --textures DIR
// holds the reference's JPEG maps under their own file names (Textures/ in the
// reference tree); they are decoded like cv::imread does (cg_image_decode_jpeg).
//
//   rasteriser [--width W] [--height H] [--focal F] [--keys KEYS] [--out FILE]
//              [--setting S] [--setting-boxes B] [--textures DIR]
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

int SCREEN_WIDTH = 900, SCREEN_HEIGHT = 720;                 // :21-22
float focalLength = 512;                                      // :30
vec4 cameraPos(0, 0, -3.001, 1);                              // :31
float yaw = 0.0;                                              // :34
mat4 R(1.0f);                                                 // :35
vec4 sceneCoordinatesLightPos(0, -0.5, 0, 1);                 // :52
vec3 lightPower = 20.0f * vec3(1, 1, 1);                      // :53
vec3 indirectLightPowerPerArea = 0.15f * vec3(1, 1, 1);       // :54
int randColourSelect = 0;                                     // :81
uint64_t randCalls = 0;                                       // glibc rand() calls so far (never seeded)
vector<rast::Triangle> originalroom;                          // :84
vector<rast::Triangle> originalbox;                           // :85

static cg_ctx *g_ctx = nullptr;
static string g_keys;
static size_t g_frame = 0;

static void die(int rc, const char *what)
{
    cerr << what << " failed (" << rc << "): " << (g_ctx ? cg_last_error(g_ctx) : "") << endl;
    exit(1);
}

// skeleton.cpp:203-308
void Draw(screen *screen)
{
    cg_rast_params p;
    p.width = screen->width;
    p.height = screen->height;
    p.focal = focalLength;
    p.camera = cg_vec4{cameraPos.x, cameraPos.y, cameraPos.z, cameraPos.w};
    memcpy(p.R, R.data(), sizeof(p.R));
    p.light_scene = cg_vec4{sceneCoordinatesLightPos.x, sceneCoordinatesLightPos.y,
                            sceneCoordinatesLightPos.z, sceneCoordinatesLightPos.w};
    p.light_power = cg_vec3{lightPower.x, lightPower.y, lightPower.z};
    p.indirect_first = indirectLightPowerPerArea.x;
    p.colour_mode = randColourSelect;
    p.yaw = yaw;
    p.rand_offset = randCalls;
    // geometry (shadow volumes + clip), fill and post-pass all on the GPU
    cg_stats st;
    int rc = cg_rast_draw(g_ctx, &p, screen->buffer, nullptr, nullptr, &st);
    if (rc) die(rc, "cg_rast_draw");
    if (randColourSelect == 0) {
        // PixelShader leaves the global at 0.2 after the first shaded fragment (:585)
        if (st.n_tris > 0) indirectLightPowerPerArea = 0.2f * vec3(1, 1, 1);
    } else {
        randCalls += 3 * (uint64_t)st.n_shaded;              // :649-651 / :657-659 per fragment
    }
}

// skeleton.cpp:311-417 with scripted keys
bool Update()
{
    if (g_frame >= g_keys.size()) return g_frame++ == 0;
    char key = g_keys[g_frame++];
    switch (key) {
    case 'w': sceneCoordinatesLightPos += vec4(0, 0, 0.1, 0); break;
    case 's': sceneCoordinatesLightPos += vec4(0, 0, -0.1, 0); break;
    case 'a': sceneCoordinatesLightPos += vec4(-0.1, 0, 0, 0); break;
    case 'd': sceneCoordinatesLightPos += vec4(0.1, 0, 0, 0); break;
    case 'q': sceneCoordinatesLightPos += vec4(0, -0.1, 0, 0); break;
    case 'e': sceneCoordinatesLightPos += vec4(0, 0.1, 0, 0); break;
    case '1': indirectLightPowerPerArea -= vec3(0.005f, 0.005f, 0.005f); break;
    case '2': indirectLightPowerPerArea += vec3(0.005f, 0.005f, 0.005f); break;
    case 'U': cameraPos += vec4(0, 0, 0.1, 0); break;
    case 'D': cameraPos += vec4(0, 0, -0.1, 0); break;
    case 'L': cameraPos += vec4(-0.1, 0, 0, 0); break;
    case 'R': cameraPos += vec4(0.1, 0, 0, 0); break;
    case 'z': cameraPos += vec4(0, -0.1, 0, 0); break;
    case 'x': cameraPos += vec4(0, 0.1, 0, 0); break;
    case 'n':
    case 'm':
        if (key == 'n') yaw -= 0.174533;
        else yaw += 0.174533;
        R[0][0] = cos(yaw); R[0][1] = 0; R[0][2] = -sin(yaw);
        R[1][0] = 0;        R[1][1] = 1; R[1][2] = 0;
        R[2][0] = sin(yaw); R[2][1] = 0; R[2][2] = cos(yaw);
        break;
    case ' ': randColourSelect = (randColourSelect + 1) % 3; break;   // SPACE (:406-409)
    case 'f': focalLength += 5; break;
    case 'g': focalLength -= 5; break;
    case 'X': return false;
    default: break;
    }
    return true;
}

// cv::imread(DIR/FILE, CV_LOAD_IMAGE_UNCHANGED) (:135-146) for a map of
// side n: BGR bytes, or empty if the file is absent (the reference then holds
// an empty Mat and must not render that texture).
static vector<uint8_t> read_map(const string &dir, const char *file, int n)
{
    vector<uint8_t> bytes, v;
    FILE *f = fopen((dir + "/" + file).c_str(), "rb");
    if (!f) return v;
    uint8_t chunk[1 << 16];
    size_t got;
    while ((got = fread(chunk, 1, sizeof(chunk), f)) > 0) bytes.insert(bytes.end(), chunk, chunk + got);
    fclose(f);
    int w = 0, h = 0, ch = 0;
    int rc = cg_image_jpeg_info(bytes.data(), bytes.size(), &w, &h, &ch);
    if (rc) die(rc, file);
    if (w != n || h != n || ch != 3) {
        cerr << file << ": " << w << "x" << h << "x" << ch << ", the reference indexes it as " << n << "x" << n
             << " BGR" << endl;
        exit(1);
    }
    v.resize((size_t)n * n * 3);
    rc = cg_image_decode_jpeg(g_ctx, bytes.data(), bytes.size(), v.data(), v.size());
    if (rc) die(rc, "cg_image_decode_jpeg");
    return v;
}

int main(int argc, char *argv[])
{
    string out = "screenshot.bmp", tex_dir;
    int setting = 0, setting_boxes = 0;
    for (int i = 1; i + 1 < argc; i += 2) {
        string a = argv[i];
        if (a == "--width") SCREEN_WIDTH = atoi(argv[i + 1]);
        else if (a == "--height") SCREEN_HEIGHT = atoi(argv[i + 1]);
        else if (a == "--focal") focalLength = (float)atof(argv[i + 1]);
        else if (a == "--keys") g_keys = argv[i + 1];
        else if (a == "--out") out = argv[i + 1];
        else if (a == "--setting") setting = atoi(argv[i + 1]);
        else if (a == "--setting-boxes") setting_boxes = atoi(argv[i + 1]);
        else if (a == "--textures") tex_dir = argv[i + 1];
    }
    int rc = cg_create(0, &g_ctx);
    if (rc) die(rc, "cg_create");
    screen *screen = InitializeSDL(SCREEN_WIDTH, SCREEN_HEIGHT, false);
    rast::LoadTestModel(originalroom, originalbox);          // :131
    for (auto &t : originalroom) t.texture = setting;         // TestModelH.h:85-129
    for (auto &t : originalbox) t.texture = setting_boxes;    // TestModelH.h:148-260
    vector<uint8_t> maps[8];
    if (!tex_dir.empty()) {                                   // :135-170
        const char *files[8] = {"Marble2000x2000.jpg", "woven1024x1024.jpg",
                                "Wood_wicker_003_ambientOcclusion.jpg", "Wood_wicker_003_opacity.jpg",
                                "Wood_wicker_003_normal.jpg", "Metal_Grill_002_basecolor.jpg",
                                "Metal_Grill_002_opacity.jpg", "Metal_Grill_002_normal.jpg"};
        for (int k = 0; k < 8; ++k) maps[k] = read_map(tex_dir, files[k], k ? 1024 : 2000);
        auto ptr = [&](int k) { return maps[k].empty() ? nullptr : maps[k].data(); };
        cg_rast_textures tx = {ptr(0), ptr(1), ptr(2), ptr(3), ptr(4), ptr(5), ptr(6), ptr(7)};
        rc = cg_rast_set_textures(g_ctx, &tx);
        if (rc) die(rc, "cg_rast_set_textures");
        if (tx.marble) randCalls = 3ull * 2000 * 2000;       // normalMap_marble's rand() calls (:158-170)
    }
    rc = cg_rast_set_scene(g_ctx, reinterpret_cast<const cg_rtri *>(originalroom.data()), (int)originalroom.size(),
                           reinterpret_cast<const cg_rtri *>(originalbox.data()), (int)originalbox.size());
    if (rc) die(rc, "cg_rast_set_scene");
    while (Update()) {
        Draw(screen);
        SDL_Renderframe(screen);
    }
    SDL_SaveImage(screen, out.c_str());
    KillSDL(screen);
    cg_destroy(g_ctx);
    return 0;
}
