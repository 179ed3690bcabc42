// SDLauxiliary.h -- headless version of the reference's framebuffer layer
// (raytracer/Source/SDLauxiliary.h, identical in rasteriser/).  Same `screen`
// struct and PutPixelSDL packing; there is no window, so SDL_Renderframe is a
// no-op and SDL_SaveImage writes the BMP SDL_SaveBMP would (BITMAPV4HEADER,
// BI_BITFIELDS, bottom-up, ARGB masks, CSType 'Win '), byte for byte.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>

#include "glm_lite.h"

typedef struct {
    void *window;       // SDL_Window*   (unused: headless)
    void *renderer;     // SDL_Renderer* (unused)
    void *texture;      // SDL_Texture*  (unused)
    int height;
    int width;
    uint32_t *buffer;
} screen;

inline screen *InitializeSDL(int width, int height, bool fullscreen = false)
{
    (void)fullscreen;
    screen *s = new screen;
    s->window = s->renderer = s->texture = nullptr;
    s->width = width;
    s->height = height;
    s->buffer = new uint32_t[(size_t)width * height];
    std::memset(s->buffer, 0, (size_t)width * height * sizeof(uint32_t));
    return s;
}

// SDLauxiliary.h:149-161
inline void PutPixelSDL(screen *s, int x, int y, glm::vec3 colour)
{
    if (x < 0 || x >= s->width || y < 0 || y >= s->height) {
        std::cout << "apa" << std::endl;
        return;
    }
    uint32_t r = uint32_t(glm::clamp(255 * colour.x, 0.f, 255.f));
    uint32_t g = uint32_t(glm::clamp(255 * colour.y, 0.f, 255.f));
    uint32_t b = uint32_t(glm::clamp(255 * colour.z, 0.f, 255.f));
    s->buffer[y * s->width + x] = (128 << 24) + (r << 16) + (g << 8) + b;
}

inline void SDL_Renderframe(screen *) {}

inline void KillSDL(screen *s)
{
    delete[] s->buffer;
    delete s;
}

// SDLauxiliary.h:24-53 (SDL_SaveBMP of an ARGB8888 surface)
inline void SDL_SaveImage(screen *s, const char *filename)
{
    const uint32_t W = s->width, H = s->height, img = W * H * 4, off = 14 + 108;
    unsigned char h[122];
    std::memset(h, 0, sizeof(h));
    auto u16 = [&](int o, uint32_t v) { h[o] = v & 0xff; h[o + 1] = (v >> 8) & 0xff; };
    auto u32 = [&](int o, uint32_t v) { u16(o, v & 0xffff); u16(o + 2, v >> 16); };
    h[0] = 'B'; h[1] = 'M';
    u32(2, off + img); u32(10, off);
    u32(14, 108); u32(18, W); u32(22, H); u16(26, 1); u16(28, 32); u32(30, 3); u32(34, img);
    u32(54, 0x00ff0000u); u32(58, 0x0000ff00u); u32(62, 0x000000ffu); u32(66, 0xff000000u);
    u32(70, 0x57696e20u);   // LCS_WINDOWS_COLOR_SPACE
    FILE *f = std::fopen(filename, "wb");
    if (!f) {
        std::cout << "Failed to save image: " << filename << std::endl;
        std::exit(1);
    }
    std::fwrite(h, 1, sizeof(h), f);
    for (int y = (int)H - 1; y >= 0; --y) std::fwrite(s->buffer + (size_t)y * W, 4, W, f);
    std::fclose(f);
}
