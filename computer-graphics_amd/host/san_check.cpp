// san_check.cpp -- the library's host-side code under AddressSanitizer and
// UBSan (Makefile `sanitize`; no GPU needed): every C-ABI entry that runs on
// the host -- scene builders, the rasteriser's host geometry (camera space,
// shadow volumes, the six clip planes with the plane-6 quirks,
// rasteriser/Source/skeleton.cpp:205-241, 720-1673), the RT column window,
// the opacity maps, glibc rand(), the starfield, and the JPEG parser and
// entropy decoder on the reference's textures and on damaged copies.
//   san_check TEXTURE_DIR
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cg_render.h"

static std::vector<uint8_t> slurp(const std::string &path)
{
    std::vector<uint8_t> v;
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return v;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
    fclose(f);
    return v;
}

static void fail(const char *what, int rc)
{
    fprintf(stderr, "%s failed: %d\n", what, rc);
    exit(1);
}

// A crafted JPEG: SOI, the given segments (marker, payload), a few entropy bytes, EOI.
static std::vector<uint8_t> crafted(std::initializer_list<std::pair<int, std::vector<uint8_t>>> segs)
{
    std::vector<uint8_t> j = {0xFF, 0xD8};
    for (const auto &sg : segs) {
        j.push_back(0xFF);
        j.push_back((uint8_t)sg.first);
        const size_t len = sg.second.size() + 2;
        j.push_back((uint8_t)(len >> 8));
        j.push_back((uint8_t)len);
        j.insert(j.end(), sg.second.begin(), sg.second.end());
        if (sg.first == 0xDA)
            for (int k = 0; k < 64; ++k) j.push_back((uint8_t)(0x5A ^ k));
    }
    j.push_back(0xFF);
    j.push_back(0xD9);
    return j;
}

// Malformed headers the damaged-file loop cannot reach: each must
// be rejected (CG_E_INVALID) without reading outside the buffer or using
// undefined tables.
static int malformed_jpegs()
{
    const std::vector<uint8_t> sof1 = {8, 0, 16, 0, 16, 1, 1, 0x11, 0};                // 16x16 gray, tq 0
    std::vector<uint8_t> dqt(65, 1);
    dqt[0] = 0;                                                                        // table 0, 8-bit
    std::vector<uint8_t> dht_dc = {0x00, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};   // one 1-bit code
    std::vector<uint8_t> dht_dc_bad = dht_dc;
    dht_dc_bad[17] = 20;                                                               // DC category 20 > 15
    std::vector<uint8_t> dht_ac = {0x10, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x00};
    std::vector<uint8_t> dht_over = {0x10, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 2, 3};  // 3 1-bit codes
    std::vector<uint8_t> dht_ones = {0x10, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 2};     // '1' used
    const std::vector<uint8_t> sos1 = {1, 1, 0x00, 0, 63, 0};
    std::vector<uint8_t> dqt_short(dqt.begin(), dqt.begin() + 20);
    std::vector<uint8_t> dht_short(dht_ac.begin(), dht_ac.begin() + 10);
    std::vector<uint8_t> dht_short_syms = {0x10, 0, 0, 0, 0, 0, 0, 0, 40, 0, 0, 0, 0, 0, 0, 0, 0, 1, 2};
    const std::vector<uint8_t> sof3_short = {8, 0, 16, 0, 16, 3, 1, 0x11, 0};         // 3 components, 1 described
    const std::vector<uint8_t> adobe_short = {'A', 'd', 'o', 'b', 'e', 0, 100, 0, 0, 0};
    const std::vector<std::vector<uint8_t>> cases = {
        crafted({{0xDB, dqt}, {0xC0, sof1}, {0xC4, dht_dc_bad}, {0xC4, dht_ac}, {0xDA, sos1}}),   // DC s > 15
        crafted({{0xDB, dqt}, {0xC0, sof1}, {0xDA, sos1}}),                                        // no Huffman tables
        crafted({{0xDB, dqt}, {0xC0, sof1}, {0xC4, dht_dc}, {0xDA, sos1}}),                        // no AC table
        crafted({{0xC0, sof1}, {0xC4, dht_dc}, {0xC4, dht_ac}, {0xDA, sos1}}),                     // no quant table
        crafted({{0xDB, dqt}, {0xC0, sof1}, {0xC4, dht_dc}, {0xC4, dht_over}, {0xDA, sos1}}),      // over-subscribed
        crafted({{0xDB, dqt}, {0xC0, sof1}, {0xC4, dht_dc}, {0xC4, dht_ones}, {0xDA, sos1}}),      // all-ones code
        crafted({{0xDB, dqt_short}, {0xC0, sof1}}),                                                // DQT past its segment
        crafted({{0xC4, dht_short}, {0xC0, sof1}}),                                                // DHT counts cut off
        crafted({{0xC4, dht_short_syms}, {0xC0, sof1}}),                                           // DHT symbols cut off
        crafted({{0xDB, dqt}, {0xC0, sof3_short}}),                                                // SOF shorter than 3 comps
        crafted({{0xDB, dqt}, {0xC0, {8, 0, 16}}}),                                                // SOF cut off
        crafted({{0xDD, {}}, {0xDB, dqt}, {0xC0, sof1}}),                                          // DRI without its value
        crafted({{0xDB, dqt}, {0xC0, sof1}, {0xC0, sof1}}),                                        // two frame headers
        crafted({{0xDB, dqt}, {0xC0, sof1}, {0xC4, dht_dc}, {0xC4, dht_ac}, {0xDA, {}}}),          // empty SOS
    };
    int rejected = 0;
    for (const auto &j : cases) {
        if (cg_image_jpeg_check(j.data(), j.size()) != CG_E_INVALID) fail("malformed JPEG accepted", -1);
        ++rejected;
    }
    // an Adobe segment too short for its transform byte is ignored, not read past
    const auto ok = crafted({{0xEE, adobe_short}, {0xDB, dqt}, {0xC0, sof1}, {0xC4, dht_dc}, {0xC4, dht_ac},
                             {0xDA, sos1}});
    if (int rc = cg_image_jpeg_check(ok.data(), ok.size())) fail("well-formed crafted JPEG", rc);
    return rejected;
}

int main(int argc, char **argv)
{
    const std::string dir = argc > 1 ? argv[1] : "tests/golden/textures";
    // JPEG: the reference's maps, truncated and corrupted copies
    const char *files[] = {"Metal_Grill_002_basecolor.jpg", "Metal_Grill_002_opacity.jpg", "Metal_Grill_002_normal.jpg",
                           "woven1024x1024.jpg", "Wood_wicker_003_ambientOcclusion.jpg", "Wood_wicker_003_opacity.jpg",
                           "Wood_wicker_003_normal.jpg"};
    int checked = 0;
    for (const char *fn : files) {
        std::vector<uint8_t> j = slurp(dir + "/" + fn);
        if (j.empty()) fail(fn, -1);
        int w, h, c;
        if (int rc = cg_image_jpeg_info(j.data(), j.size(), &w, &h, &c)) fail("cg_image_jpeg_info", rc);
        if (int rc = cg_image_jpeg_check(j.data(), j.size())) fail("cg_image_jpeg_check", rc);
        for (size_t cut = 2; cut < j.size(); cut = cut * 3 + 5) (void)cg_image_jpeg_check(j.data(), cut);
        std::vector<uint8_t> bad = j;
        for (size_t k = bad.size() / 4; k < bad.size(); k += 1013) bad[k] ^= 0xa5;
        (void)cg_image_jpeg_check(bad.data(), bad.size());
        for (size_t k = 2; k + 1 < bad.size() && k < 700; k += 7) bad[k] = 0xff;   // damaged headers
        (void)cg_image_jpeg_info(bad.data(), bad.size(), &w, &h, &c);
        (void)cg_image_jpeg_check(bad.data(), bad.size());
        ++checked;
    }
    // rasteriser host geometry over cameras inside / outside / behind the near plane, yawed
    cg_rtri room[16], boxes[32];
    int nr = 0, nb = 0;
    if (int rc = cg_rast_load_test_model(room, 16, &nr, boxes, 32, &nb); rc < 0) fail("cg_rast_load_test_model", rc);
    std::vector<cg_rtri> out(32 * (nr + 7 * nb));
    const float cams[][3] = {{0, 0, -3.001f}, {0, 0, -1.2f}, {0.9f, 0.5f, -0.2f}, {-1.8f, 0, -1.6f},
                             {0, 0, 0.95f}, {3, -2, 2}, {0, 0, -0.99f}, {0.3f, 0.99f, -3}};
    long tris = 0;
    for (const auto &cam : cams)
        for (float yaw : {0.0f, 0.174533f, -0.8726650476455688f, 3.0f})
            for (int W : {3, 161, 900}) {
                cg_rast_params p{};
                p.width = W;
                p.height = W * 3 / 4 + 1;
                p.focal = 0.6f * (float)W;
                p.camera = cg_vec4{cam[0], cam[1], cam[2], 1.0f};
                for (int k = 0; k < 16; ++k) p.R[k] = (k % 5 == 0) ? 1.0f : 0.0f;
                p.R[0] = cosf(yaw); p.R[2] = -sinf(yaw); p.R[8] = sinf(yaw); p.R[10] = cosf(yaw);
                p.light_scene = cg_vec4{0, -0.5f, 0, 1};
                p.light_power = cg_vec3{20, 20, 20};
                p.indirect_first = 0.2f;
                p.yaw = yaw;
                cg_vec4 light;
                int n = cg_rast_prepare(&p, room, nr, boxes, nb, out.data(), (int)out.size(), &light);
                if (n < 0) fail("cg_rast_prepare", n);
                tris += n;
            }
    // RT scenes, column windows, lights, rand, opacity, starfield
    cg_tri t[64];
    cg_sphere sph;
    int n = cg_rt_load_test_model(t, 64, &sph);
    if (n < 0) fail("cg_rt_load_test_model", n);
    std::vector<cg_tri> rnd(5000);
    if (int rc = cg_rt_random_scene(0x5EED, 5000, rnd.data()); rc < 0) fail("cg_rt_random_scene", rc);
    for (float z : {-3.0f, -1.5f, 0.0f, 2.0f}) {
        cg_rt_camera cam{};
        cam.width = 1920; cam.height = 1080; cam.focal = 1080.0f;
        cam.camera = cg_vec4{0, 0, z, 1};
        for (int k = 0; k < 16; ++k) cam.R[k] = (k % 5 == 0) ? 1.0f : 0.0f;
        cam.indirect = 0.5f;
        int c0 = 0, c1 = 0;
        (void)cg_rt_frame_columns(t, n, &sph, 1, &cam, &c0, &c1);
        (void)cg_rt_frame_columns(rnd.data(), 5000, nullptr, 0, &cam, &c0, &c1);
        // kernel routes (host-only): identity, a yaw, NaN and huge entries, shards, large scenes
        const cg_rt_shard shards[3] = {{0, 1, 15, 0, 0, 0, 0}, {1, 3, 8, 0, 0, 0, 0}, {0, 1, 15, 135, 270, 0, 0}};
        for (int variant = 0; variant < 4; ++variant) {
            cg_rt_camera rc = cam;
            if (variant == 1) { rc.R[0] = 0.98f; rc.R[2] = -0.17f; rc.R[8] = 0.17f; rc.R[10] = 0.98f; }
            if (variant == 2) rc.R[0] = __builtin_nanf("");
            if (variant == 3) rc.R[8] = 1e30f;
            for (const cg_rt_shard &sh : shards)
                for (int nt : {28, 1000000})
                    for (int nl : {1, 64, 81})
                        if (cg_rt_route(&rc, nt, 1, nl, &sh) < 0) fail("cg_rt_route", -1);
        }
    }
    cg_light centre{{0, -0.5f, -0.7f, 1}, {14, 14, 14}}, area[64];
    if (int rc = cg_rt_area_lights(&centre, 0.1f, 8, area, 64); rc < 0) fail("cg_rt_area_lights", rc);
    std::vector<int32_t> r(4096);
    if (int rc = cg_glibc_rand(0, 4096, r.data())) fail("cg_glibc_rand", rc);
    if (int rc = cg_glibc_rand(11999000, 4096, r.data())) fail("cg_glibc_rand", rc);
    std::vector<uint8_t> bgr(3 * 4096), op(4096);
    for (size_t i = 0; i < bgr.size(); ++i) bgr[i] = (uint8_t)(i * 37);
    if (int rc = cg_rast_opacity_map(bgr.data(), 4096, op.data())) fail("cg_rast_opacity_map", rc);
    std::vector<float> stars(3 * 1000);
    if (int rc = cg_starfield_init(stars.data(), 1000)) fail("cg_starfield_init", rc);
    for (int k = 0; k < 100; ++k) cg_starfield_update(stars.data(), 1000, 16.0f);
    cg_rt_shard sh{1, 3, 15, 0, 0, 0, 0};
    (void)cg_rt_shard_rows(1080, &sh);
    const int malformed = malformed_jpegs();
    printf("sanitized host code: %d JPEGs, %d malformed JPEGs rejected, %ld clipped triangles, clean\n", checked,
           malformed, tris);
    return 0;
}
