// film_io.cpp -- LDR output and the per-pixel variance image.
//
// nori_write_png: Bitmap::saveToLDR (bitmap.cpp:109-139, the hdrToLdr tool):
//   byte = (uint8_t) Clamp(255 * GammaCorrect(v) + 0.5, 0, 255) per channel,
//   GammaCorrect = the sRGB transfer curve (12.92 v below 0.0031308, else
//   1.055 v^(1/2.4) - 0.055, std::pow in float); written as an 8-bit RGB PNG
//   (the reference calls stb_image_write; here zlib deflate, filter type 0).
// nori_film_variance: variance of each pixel's mean radiance from the
//   statistics nori_gpu_render accumulates (render_desc.variance_out).
#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "host_scene.h"

namespace {

float gamma_correct(float v) {  // bitmap.cpp:109-112
    if (v <= 0.0031308f) return 12.92f * v;
    return 1.055f * std::pow(v, 1.f / 2.4f) - 0.055f;
}
float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }  // bitmap.cpp:113-120

void be32(std::vector<unsigned char> &b, uint32_t v) {
    for (int s = 24; s >= 0; s -= 8) b.push_back((unsigned char)(v >> s));
}
void chunk(std::vector<unsigned char> &out, const char *type, const std::vector<unsigned char> &data) {
    be32(out, (uint32_t)data.size());
    const size_t at = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    uLong crc = crc32(0L, Z_NULL, 0);
    crc = crc32(crc, out.data() + at, (uInt)(out.size() - at));
    be32(out, (uint32_t)crc);
}

}  // namespace

extern "C" int nori_write_png(const char *path, const float *rgb, int width, int height) {
    if (!path || !rgb || width <= 0 || height <= 0) return NORI_ERR_INVALID;
    // scanlines with a leading filter byte (0 = none)
    const size_t row = 1 + 3 * (size_t)width;
    std::vector<unsigned char> raw(row * (size_t)height);
    for (int y = 0; y < height; ++y) {
        unsigned char *d = raw.data() + row * (size_t)y;
        d[0] = 0;
        for (int x = 0; x < 3 * width; ++x)
            d[1 + x] = (uint8_t)clampf(255.f * gamma_correct(rgb[3 * (size_t)y * width + x]) + 0.5f, 0.f, 255.f);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<unsigned char> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return NORI_ERR_IO;
    z.resize(zlen);
    std::vector<unsigned char> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<unsigned char> ihdr;
    be32(ihdr, (uint32_t)width);
    be32(ihdr, (uint32_t)height);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit, truecolour, deflate, filter 0, no interlace
    chunk(out, "IHDR", ihdr);
    chunk(out, "IDAT", z);
    chunk(out, "IEND", {});
    FILE *f = std::fopen(path, "wb");
    if (!f) return NORI_ERR_IO;
    const bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
    return std::fclose(f) == 0 && ok ? NORI_OK : NORI_ERR_IO;
}

extern "C" int nori_film_variance(const nori_scene_desc *scene, const float *stats, float *out) {
    if (!scene || !stats || !out) return NORI_ERR_INVALID;
    const size_t n_px = (size_t)scene->camera.width * (size_t)scene->camera.height;
    for (size_t i = 0; i < n_px; ++i) {
        const float *s = stats + 8 * i;
        const double n = s[6];
        for (int c = 0; c < 3; ++c) {
            double v = 0.0;
            if (n >= 2.0) {
                const double s1 = s[c], s2 = s[3 + c];
                v = (s2 - s1 * s1 / n) / (n * (n - 1.0));
                if (v < 0.0) v = 0.0;  // rounding of nearly constant pixels
            }
            out[3 * i + c] = (float)v;
        }
    }
    return NORI_OK;
}
