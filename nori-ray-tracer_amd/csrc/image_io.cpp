// image_io.cpp -- OpenEXR output (Bitmap::save, bitmap.cpp:82-107).
// Writes a single-part scanline file: channels B, G, R as 32-bit float,
// no compression, increasing-Y line order.  Any OpenEXR reader opens it.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "host_scene.h"

namespace {

void put_bytes(std::vector<unsigned char> &b, const void *p, size_t n) {
    const unsigned char *c = static_cast<const unsigned char *>(p);
    b.insert(b.end(), c, c + n);
}
template <class T> void put(std::vector<unsigned char> &b, T v) { put_bytes(b, &v, sizeof(T)); }
void put_str(std::vector<unsigned char> &b, const char *s) { put_bytes(b, s, std::strlen(s) + 1); }
void attr(std::vector<unsigned char> &b, const char *name, const char *type, const std::vector<unsigned char> &val) {
    put_str(b, name);
    put_str(b, type);
    put<int32_t>(b, (int32_t)val.size());
    b.insert(b.end(), val.begin(), val.end());
}

}  // namespace

extern "C" int nori_write_exr(const char *path, const float *rgb, int width, int height) {
    if (!path || !rgb || width <= 0 || height <= 0) return NORI_ERR_INVALID;
    std::vector<unsigned char> h;
    const unsigned char magic[8] = {0x76, 0x2f, 0x31, 0x01, 2, 0, 0, 0};
    put_bytes(h, magic, 8);
    std::vector<unsigned char> v;
    for (const char *ch : {"B", "G", "R"}) {
        put_str(v, ch);
        put<int32_t>(v, 2);  // FLOAT
        put<uint8_t>(v, 0);  // pLinear
        put<uint8_t>(v, 0);
        put<uint8_t>(v, 0);
        put<uint8_t>(v, 0);
        put<int32_t>(v, 1);
        put<int32_t>(v, 1);
    }
    put<uint8_t>(v, 0);
    attr(h, "channels", "chlist", v);
    attr(h, "compression", "compression", {0});
    v.clear();
    for (int32_t x : {0, 0, width - 1, height - 1}) put<int32_t>(v, x);
    attr(h, "dataWindow", "box2i", v);
    attr(h, "displayWindow", "box2i", v);
    attr(h, "lineOrder", "lineOrder", {0});
    v.clear();
    put<float>(v, 1.0f);
    attr(h, "pixelAspectRatio", "float", v);
    v.clear();
    put<float>(v, 0.0f);
    put<float>(v, 0.0f);
    attr(h, "screenWindowCenter", "v2f", v);
    v.clear();
    put<float>(v, 1.0f);
    attr(h, "screenWindowWidth", "float", v);
    put<uint8_t>(h, 0);  // end of header
    const uint64_t line_bytes = 8 + 3 * 4 * (uint64_t)width;
    uint64_t base = h.size() + 8 * (uint64_t)height;
    for (int y = 0; y < height; ++y) put<uint64_t>(h, base + line_bytes * (uint64_t)y);
    FILE *f = std::fopen(path, "wb");
    if (!f) return NORI_ERR_IO;
    bool ok = std::fwrite(h.data(), 1, h.size(), f) == h.size();
    std::vector<float> line(3 * (size_t)width);
    for (int y = 0; y < height && ok; ++y) {
        int32_t hdr[2] = {y, (int32_t)(12 * width)};
        for (int c = 0; c < 3; ++c)  // B, G, R planes
            for (int x = 0; x < width; ++x) line[(size_t)c * width + x] = rgb[3 * ((size_t)y * width + x) + (2 - c)];
        ok = std::fwrite(hdr, 4, 2, f) == 2 && std::fwrite(line.data(), 4, line.size(), f) == line.size();
    }
    ok = (std::fclose(f) == 0) && ok;
    return ok ? NORI_OK : NORI_ERR_IO;
}
