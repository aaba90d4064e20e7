// image_io.cpp -- OpenEXR I/O.
// Output (Bitmap::save, bitmap.cpp:82-107): a single-part scanline file,
// channels B, G, R as 32-bit float, no compression, increasing-Y line order.
// Input (Bitmap::Bitmap(filename), bitmap.cpp:23-80, used by the envmap
// emitter): single-part scanline files with NONE, ZIPS or ZIP compression and
// HALF or FLOAT R, G, B channels (others ignored); the reference reads the R,
// G, B planes into a rows x cols Color3f array, rows = image height.
#include <zlib.h>

#include <cmath>
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

// ------------------------------------------------------------------ reader
namespace {

float half_to_float(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 31u, m = h & 1023u;
    uint32_t bits;
    if (e == 0) {
        if (m == 0) {
            bits = s;
        } else {  // subnormal half -> normal float
            float f = std::ldexp((float)m, -24);
            std::memcpy(&bits, &f, 4);
            bits |= s;
        }
    } else if (e == 31) {
        bits = s | 0x7F800000u | (m << 13);
    } else {
        bits = s | ((e + 112u) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}

struct ExrChannel {
    std::string name;
    int32_t type;  // 1 HALF, 2 FLOAT (0 UINT)
};

// ZIP/ZIPS block: zlib inflate, then undo the byte predictor and the
// even/odd byte split (OpenEXR ImfZip.cpp).
bool unzip_block(const unsigned char *src, size_t n, std::vector<unsigned char> &out, size_t raw) {
    std::vector<unsigned char> t(raw);
    uLongf got = (uLongf)raw;
    if (uncompress(t.data(), &got, src, (uLong)n) != Z_OK || got != raw) return false;
    for (size_t i = 1; i < raw; ++i) t[i] = (unsigned char)(t[i - 1] + t[i] - 128);
    out.resize(raw);
    const size_t half = (raw + 1) / 2;
    for (size_t i = 0; i < raw; ++i) out[i] = (i & 1) ? t[half + i / 2] : t[i / 2];
    return true;
}

int read_exr(const char *path, int &width, int &height, std::vector<float> &rgb, std::string &err) {
    FILE *f = std::fopen(path, "rb");
    if (!f) {
        err = "cannot open " + std::string(path);
        return NORI_ERR_IO;
    }
    std::vector<unsigned char> b;
    unsigned char buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
    std::fclose(f);
    size_t p = 0;
    auto need = [&](size_t k) { return p + k <= b.size(); };
    auto rd_str = [&](std::string &o) {
        o.clear();
        while (p < b.size() && b[p]) o.push_back((char)b[p++]);
        if (p >= b.size()) return false;
        ++p;
        return true;
    };
    auto rd_i32 = [&](int32_t &v) {
        if (!need(4)) return false;
        std::memcpy(&v, &b[p], 4);
        p += 4;
        return true;
    };
    if (!need(8) || b[0] != 0x76 || b[1] != 0x2f || b[2] != 0x31 || b[3] != 0x01) {
        err = "not an OpenEXR file: " + std::string(path);
        return NORI_ERR_IO;
    }
    if (b[4] != 2 || (b[5] & 0x1E)) {  // version 2, single-part scanline, no deep/tiles/long names
        err = "unsupported OpenEXR flavour (tiled, deep or multi-part): " + std::string(path);
        return NORI_ERR_UNSUPPORTED;
    }
    p = 8;
    std::vector<ExrChannel> ch;
    int32_t comp = -1, xmin = 0, ymin = 0, xmax = -1, ymax = -1;
    for (;;) {
        std::string name, type;
        if (!rd_str(name)) return err = "truncated header", NORI_ERR_IO;
        if (name.empty()) break;
        int32_t size;
        if (!rd_str(type) || !rd_i32(size) || !need((size_t)size)) return err = "truncated header", NORI_ERR_IO;
        const size_t end = p + (size_t)size;
        if (name == "channels") {
            while (p < end && b[p]) {
                ExrChannel c;
                rd_str(c.name);
                int32_t t = 0;
                rd_i32(t);
                c.type = t;
                p += 12;  // pLinear, reserved, xSampling, ySampling
                ch.push_back(c);
            }
        } else if (name == "compression") {
            comp = b[p];
        } else if (name == "dataWindow") {
            std::memcpy(&xmin, &b[p], 4);
            std::memcpy(&ymin, &b[p + 4], 4);
            std::memcpy(&xmax, &b[p + 8], 4);
            std::memcpy(&ymax, &b[p + 12], 4);
        }
        p = end;
    }
    width = xmax - xmin + 1;
    height = ymax - ymin + 1;
    if (width <= 0 || height <= 0) return err = "empty data window", NORI_ERR_IO;
    const int lines_per_block = comp == 0 || comp == 2 ? 1 : (comp == 3 ? 16 : 0);
    if (!lines_per_block) return err = "unsupported EXR compression " + std::to_string(comp), NORI_ERR_UNSUPPORTED;
    size_t pix_bytes = 0;
    int src[3] = {-1, -1, -1};  // channel index of R, G, B
    std::vector<size_t> offs;
    for (size_t i = 0; i < ch.size(); ++i) {
        if (ch[i].type != 1 && ch[i].type != 2) return err = "unsupported EXR channel type", NORI_ERR_UNSUPPORTED;
        offs.push_back(pix_bytes);
        pix_bytes += ch[i].type == 1 ? 2 : 4;
        if (ch[i].name == "R") src[0] = (int)i;
        if (ch[i].name == "G") src[1] = (int)i;
        if (ch[i].name == "B") src[2] = (int)i;
    }
    const int nblocks = (height + lines_per_block - 1) / lines_per_block;
    std::vector<uint64_t> table((size_t)nblocks);
    if (!need(8 * (size_t)nblocks)) return err = "truncated offset table", NORI_ERR_IO;
    std::memcpy(table.data(), &b[p], 8 * (size_t)nblocks);
    rgb.assign(3 * (size_t)width * height, 0.0f);
    std::vector<unsigned char> raw;
    for (int k = 0; k < nblocks; ++k) {
        size_t q = (size_t)table[(size_t)k];
        int32_t y0, sz;
        if (q + 8 > b.size()) return err = "bad scanline offset", NORI_ERR_IO;
        std::memcpy(&y0, &b[q], 4);
        std::memcpy(&sz, &b[q + 4], 4);
        q += 8;
        const int lines = std::min(lines_per_block, ymax + 1 - y0);
        const size_t want = (size_t)lines * width * pix_bytes;
        if (sz < 0 || q + (size_t)sz > b.size()) return err = "bad scanline block", NORI_ERR_IO;
        const unsigned char *data = &b[q];
        if (comp != 0 && (size_t)sz < want) {
            if (!unzip_block(data, (size_t)sz, raw, want)) return err = "zlib error", NORI_ERR_IO;
            data = raw.data();
        } else if ((size_t)sz < want) {
            return err = "short scanline block", NORI_ERR_IO;
        }
        for (int l = 0; l < lines; ++l) {
            const int y = y0 - ymin + l;
            const unsigned char *line = data + (size_t)l * width * pix_bytes;
            for (int c = 0; c < 3; ++c) {
                if (src[c] < 0) continue;
                const ExrChannel &e = ch[(size_t)src[c]];
                const unsigned char *plane = line + offs[(size_t)src[c]] * width;
                for (int x = 0; x < width; ++x) {
                    float v;
                    if (e.type == 1) {
                        uint16_t h;
                        std::memcpy(&h, plane + 2 * (size_t)x, 2);
                        v = half_to_float(h);
                    } else {
                        std::memcpy(&v, plane + 4 * (size_t)x, 4);
                    }
                    rgb[3 * ((size_t)y * width + x) + c] = v;
                }
            }
        }
    }
    return NORI_OK;
}

}  // namespace

namespace nori {
int load_exr(const std::string &path, int &width, int &height, std::vector<float> &rgb) {
    std::string err;
    int rc = read_exr(path.c_str(), width, height, rgb, err);
    if (rc != NORI_OK) throw NoriException(rc, "EXR: " + err);
    return rc;
}
}  // namespace nori

extern "C" int nori_read_exr(const char *path, int *width, int *height, float *rgb) {
    if (!path || !width || !height) return NORI_ERR_INVALID;
    std::vector<float> img;
    std::string err;
    int w = 0, h = 0;
    int rc = read_exr(path, w, h, img, err);
    if (rc != NORI_OK) return rc;
    *width = w;
    *height = h;
    if (rgb) std::memcpy(rgb, img.data(), img.size() * sizeof(float));
    return NORI_OK;
}
