// image_decode.cpp -- 8-bit image decoding for ImageTexture / NormalMap.
//
// The reference loads both textures with stbi_load(path, .., STBI_rgb)
// (src/imagetexture.cpp:75-84, src/normalmap.cpp:75-84), built against the
// stb_image v1.39 its GUI dependency vendors
// (ext/nanogui/ext/nanovg/src/stb_image.h).  That version decodes baseline
// (sequential, Huffman) JPEG and 8-bit PNG; progressive JPEG and other PNG
// depths are errors there and here.  This file restates its arithmetic so the
// texels are the same bytes:
//   * JPEG: canonical Huffman decoding (stb_image.h:1023-1159), blocks in
//     zig-zag order (:1163-1211), the integer IDCT derived from jidctint with
//     12-bit constants and its two rounding shifts (:1224-1331), component
//     planes padded to whole MCUs (:1579-1608), interleaved and single-
//     component scans with restart intervals (:1375-1445), the "fancy"
//     chroma upsamplers (:1679-1761) and the 16.16 fixed-point YCbCr->RGB
//     conversion (:1763-1790), row loop of load_jpeg_image (:1855-1919);
//   * PNG: IHDR/PLTE/tRNS/IDAT chunks, zlib inflate (the system zlib: inflate
//     is fully specified, so any correct inflater gives the same bytes), the
//     five row filters with an all-zero row before the first, Adam7
//     interlacing, palette expansion, then conversion to 3 channels (gray
//     replicated, alpha dropped) as stbi__convert_format does for STBI_rgb.
// Output: width x height x 3 bytes, row-major, top row first (stb's order).
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "host_scene.h"

namespace nori {

namespace {

// ------------------------------------------------------------------ JPEG
struct Huff {  // canonical Huffman table (JPEG Annex C)
    int count[17] = {0};   // codes of each length
    int first[17] = {0};   // first code of each length
    int offset[17] = {0};  // index of that code's symbol in `values`
    uint8_t values[256] = {0};
    bool present = false;
};

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0, hd = 0, ha = 0;
    int x = 0, y = 0;    // effective samples (stb img_comp.x/y)
    int w2 = 0, h2 = 0;  // plane size padded to whole MCUs
    int dc_pred = 0;
    std::vector<uint8_t> data;
};

struct Jpeg {
    const uint8_t *p, *end;
    int width = 0, height = 0, ncomp = 0;
    int hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    uint8_t dq[4][64];  // dequantisation tables in natural (de-zig-zagged) order
    Huff hdc[4], hac[4];
    Comp comp[4];
    int restart = 0;
    // entropy decoder state (stb_image.h:1064-1079): bits are taken MSB first,
    // 0xFF00 is a stuffed 0xFF, any other 0xFF xx is a marker after which the
    // decoder reads zero bits
    uint32_t buf = 0;
    int bits = 0;
    int marker = -1;
    bool nomore = false;

    int get8() { return p < end ? *p++ : 0; }
    int get16() { int a = get8(); return (a << 8) | get8(); }
    void fill() {
        while (bits <= 24) {
            int b = 0;
            if (!nomore) {
                b = get8();
                if (b == 0xFF) {
                    int c = get8();
                    while (c == 0xFF) c = get8();  // fill bytes
                    if (c != 0) {
                        marker = c;
                        nomore = true;
                        b = 0;
                    }
                }
            }
            buf |= (uint32_t)b << (24 - bits);
            bits += 8;
        }
    }
    int getbits(int n) {
        if (n == 0) return 0;
        if (bits < n) fill();
        const int k = (int)(buf >> (32 - n));
        buf <<= n;
        bits -= n;
        return k;
    }
    int decode(const Huff &h) {
        if (!h.present) throw NoriException(NORI_ERR_PARSE, "JPEG: missing Huffman table");
        if (bits < 16) fill();
        int code = 0;
        for (int len = 1; len <= 16; ++len) {
            code = (code << 1) | getbits(1);
            if (code - h.first[len] < h.count[len]) return h.values[h.offset[len] + code - h.first[len]];
        }
        throw NoriException(NORI_ERR_PARSE, "JPEG: bad Huffman code (Corrupt JPEG)");
    }
    int receive_extend(int n) {  // stb_image.h:1136-1159
        if (n == 0) return 0;
        const int k = getbits(n);
        return k < (1 << (n - 1)) ? k - (1 << n) + 1 : k;
    }
    void reset() {  // stb_image.h:1363-1373
        buf = 0;
        bits = 0;
        nomore = false;
        marker = -1;
        for (auto &c : comp) c.dc_pred = 0;
    }
};

const uint8_t kDezigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                               12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                               35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                               58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

inline uint8_t clamp8(int x) { return (uint8_t)(x < 0 ? 0 : (x > 255 ? 255 : x)); }

// jidctint-derived 8x8 IDCT with 12-bit fixed-point constants (stb_image.h:1224-1331)
constexpr int f2f(double x) { return (int)(x * 4096 + 0.5); }
struct Idct1D {
    int t0, t1, t2, t3, x0, x1, x2, x3;
    Idct1D(int s0, int s1, int s2, int s3, int s4, int s5, int s6, int s7) {
        int p2 = s2, p3 = s6;
        int p1 = (p2 + p3) * f2f(0.5411961f);
        t2 = p1 + p3 * f2f(-1.847759065f);
        t3 = p1 + p2 * f2f(0.765366865f);
        p2 = s0;
        p3 = s4;
        t0 = (p2 + p3) << 12;
        t1 = (p2 - p3) << 12;
        x0 = t0 + t3;
        x3 = t0 - t3;
        x1 = t1 + t2;
        x2 = t1 - t2;
        t0 = s7;
        t1 = s5;
        t2 = s3;
        t3 = s1;
        p3 = t0 + t2;
        int p4 = t1 + t3;
        p1 = t0 + t3;
        p2 = t1 + t2;
        const int p5 = (p3 + p4) * f2f(1.175875602f);
        t0 = t0 * f2f(0.298631336f);
        t1 = t1 * f2f(2.053119869f);
        t2 = t2 * f2f(3.072711026f);
        t3 = t3 * f2f(1.501321110f);
        p1 = p5 + p1 * f2f(-0.899976223f);
        p2 = p5 + p2 * f2f(-2.562915447f);
        p3 = p3 * f2f(-1.961570560f);
        p4 = p4 * f2f(-0.390180644f);
        t3 += p1 + p4;
        t2 += p2 + p3;
        t1 += p2 + p4;
        t0 += p1 + p3;
    }
};
void idct_block(uint8_t *out, int stride, const short *d, const uint8_t *dq) {
    int val[64];
    for (int i = 0; i < 8; ++i) {  // columns; an all-zero AC column is the DC term
        const short *c = d + i;
        const uint8_t *q = dq + i;
        int *v = val + i;
        if (c[8] == 0 && c[16] == 0 && c[24] == 0 && c[32] == 0 && c[40] == 0 && c[48] == 0 && c[56] == 0) {
            const int dc = c[0] * q[0] << 2;
            for (int r = 0; r < 8; ++r) v[8 * r] = dc;
        } else {
            Idct1D k(c[0] * q[0], c[8] * q[8], c[16] * q[16], c[24] * q[24], c[32] * q[32], c[40] * q[40],
                     c[48] * q[48], c[56] * q[56]);
            k.x0 += 512; k.x1 += 512; k.x2 += 512; k.x3 += 512;
            v[0] = (k.x0 + k.t3) >> 10;
            v[56] = (k.x0 - k.t3) >> 10;
            v[8] = (k.x1 + k.t2) >> 10;
            v[48] = (k.x1 - k.t2) >> 10;
            v[16] = (k.x2 + k.t1) >> 10;
            v[40] = (k.x2 - k.t1) >> 10;
            v[24] = (k.x3 + k.t0) >> 10;
            v[32] = (k.x3 - k.t0) >> 10;
        }
    }
    for (int r = 0; r < 8; ++r) {  // rows: remove 1<<17 with rounding, +128 level shift
        const int *v = val + 8 * r;
        uint8_t *o = out + r * stride;
        Idct1D k(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
        const int bias = 65536 + (128 << 17);
        k.x0 += bias; k.x1 += bias; k.x2 += bias; k.x3 += bias;
        o[0] = clamp8((k.x0 + k.t3) >> 17);
        o[7] = clamp8((k.x0 - k.t3) >> 17);
        o[1] = clamp8((k.x1 + k.t2) >> 17);
        o[6] = clamp8((k.x1 - k.t2) >> 17);
        o[2] = clamp8((k.x2 + k.t1) >> 17);
        o[5] = clamp8((k.x2 - k.t1) >> 17);
        o[3] = clamp8((k.x3 + k.t0) >> 17);
        o[4] = clamp8((k.x3 - k.t0) >> 17);
    }
}

void decode_block(Jpeg &j, Comp &c, short *data) {  // stb_image.h:1179-1211
    std::memset(data, 0, 64 * sizeof(short));
    const int t = j.decode(j.hdc[c.hd]);
    const int diff = t ? j.receive_extend(t) : 0;
    c.dc_pred += diff;
    data[0] = (short)c.dc_pred;
    int k = 1;
    do {
        const int rs = j.decode(j.hac[c.ha]);
        const int s = rs & 15, r = rs >> 4;
        if (s == 0) {
            if (rs != 0xF0) break;  // end of block
            k += 16;
        } else {
            k += r;
            const int v = j.receive_extend(s);
            data[kDezigzag[k < 64 ? k : 63]] = (short)v;  // corrupt input samples past the end land at 63
            ++k;
        }
    } while (k < 64);
}

// after `restart` MCUs: expect RSTn, then reset the entropy decoder
// (stb_image.h:1400-1406); false: not a restart marker, the scan ends here
bool restart_marker(Jpeg &j) {
    if (j.bits < 24) j.fill();
    if (!(j.marker >= 0xD0 && j.marker <= 0xD7)) return false;
    j.reset();
    return true;
}

void entropy_scan(Jpeg &j, const int *order, int n) {  // stb_image.h:1375-1445
    j.reset();
    int todo = j.restart ? j.restart : 0x7fffffff;
    short data[64];
    if (n == 1) {  // non-interleaved: blocks in raster order over the component's own extent
        Comp &c = j.comp[order[0]];
        const int w = (c.x + 7) >> 3, h = (c.y + 7) >> 3;
        for (int by = 0; by < h; ++by)
            for (int bx = 0; bx < w; ++bx) {
                decode_block(j, c, data);
                idct_block(c.data.data() + c.w2 * by * 8 + bx * 8, c.w2, data, j.dq[c.tq]);
                if (--todo <= 0) {
                    if (!restart_marker(j)) return;
                    todo = j.restart ? j.restart : 0x7fffffff;
                }
            }
        return;
    }
    for (int my = 0; my < j.mcuy; ++my)
        for (int mx = 0; mx < j.mcux; ++mx) {
            for (int k = 0; k < n; ++k) {
                Comp &c = j.comp[order[k]];
                for (int y = 0; y < c.v; ++y)
                    for (int x = 0; x < c.h; ++x) {
                        decode_block(j, c, data);
                        idct_block(c.data.data() + c.w2 * ((my * c.v + y) * 8) + (mx * c.h + x) * 8, c.w2, data,
                                   j.dq[c.tq]);
                    }
            }
            if (--todo <= 0) {
                if (!restart_marker(j)) return;
                todo = j.restart ? j.restart : 0x7fffffff;
            }
        }
}

// next marker byte after 0xFF (fill bytes skipped); -1 at the end of data
int next_marker(Jpeg &j) {
    if (j.marker >= 0) {
        const int m = j.marker;
        j.marker = -1;
        return m;
    }
    while (j.p < j.end) {
        if (j.get8() != 0xFF) continue;  // stray bytes after a scan (stb_image.h:1651-1663)
        int m = j.get8();
        while (m == 0xFF) m = j.get8();
        if (m != 0) return m;
    }
    return -1;
}

// "fancy" upsamplers and nearest-neighbour fallback (stb_image.h:1679-1761)
const uint8_t *resample(uint8_t *out, const uint8_t *near_, const uint8_t *far_, int w, int hs, int vs) {
    if (hs == 1 && vs == 1) return near_;
    if (hs == 1 && vs == 2) {
        for (int i = 0; i < w; ++i) out[i] = (uint8_t)((3 * near_[i] + far_[i] + 2) >> 2);
        return out;
    }
    if (hs == 2 && vs == 1) {
        const uint8_t *in = near_;
        if (w == 1) {
            out[0] = out[1] = in[0];
            return out;
        }
        out[0] = in[0];
        out[1] = (uint8_t)((in[0] * 3 + in[1] + 2) >> 2);
        int i = 1;
        for (; i < w - 1; ++i) {
            const int n = 3 * in[i] + 2;
            out[i * 2 + 0] = (uint8_t)((n + in[i - 1]) >> 2);
            out[i * 2 + 1] = (uint8_t)((n + in[i + 1]) >> 2);
        }
        out[i * 2 + 0] = (uint8_t)((in[w - 2] * 3 + in[w - 1] + 2) >> 2);
        out[i * 2 + 1] = in[w - 1];
        return out;
    }
    if (hs == 2 && vs == 2) {
        if (w == 1) {
            out[0] = out[1] = (uint8_t)((3 * near_[0] + far_[0] + 2) >> 2);
            return out;
        }
        int t1 = 3 * near_[0] + far_[0];
        out[0] = (uint8_t)((t1 + 2) >> 2);
        for (int i = 1; i < w; ++i) {
            const int t0 = t1;
            t1 = 3 * near_[i] + far_[i];
            out[i * 2 - 1] = (uint8_t)((3 * t0 + t1 + 8) >> 4);
            out[i * 2] = (uint8_t)((3 * t1 + t0 + 8) >> 4);
        }
        out[w * 2 - 1] = (uint8_t)((t1 + 2) >> 2);
        return out;
    }
    for (int i = 0; i < w; ++i)
        for (int k = 0; k < hs; ++k) out[i * hs + k] = near_[i];
    return out;
}

constexpr int fx16(double x) { return (int)(x * 65536 + 0.5); }  // float2fixed (stb_image.h:1763)

void decode_jpeg(const std::vector<uint8_t> &bytes, int &W, int &H, std::vector<uint8_t> &rgb) {
    Jpeg j;
    j.p = bytes.data();
    j.end = bytes.data() + bytes.size();
    std::memset(j.dq, 0, sizeof(j.dq));
    if (j.get8() != 0xFF || j.get8() != 0xD8) throw NoriException(NORI_ERR_PARSE, "JPEG: no SOI");
    bool frame = false;
    for (;;) {
        const int m = next_marker(j);
        if (m < 0) throw NoriException(NORI_ERR_PARSE, "JPEG: unexpected end of data");
        if (m == 0xD9) break;  // EOI
        if (m == 0xC2) throw NoriException(NORI_ERR_UNSUPPORTED, "progressive jpeg (JPEG format not supported)");
        if (m == 0xC0 || m == 0xC1) {  // SOF0/SOF1 (stb_image.h:1541-1611)
            const int Lf = j.get16();
            if (j.get8() != 8) throw NoriException(NORI_ERR_UNSUPPORTED, "JPEG: 8-bit only");
            j.height = j.get16();
            j.width = j.get16();
            j.ncomp = j.get8();
            if (j.height == 0 || j.width == 0) throw NoriException(NORI_ERR_UNSUPPORTED, "JPEG: delayed height / 0 width");
            if (j.ncomp != 1 && j.ncomp != 3) throw NoriException(NORI_ERR_PARSE, "JPEG: bad component count");
            if (Lf != 8 + 3 * j.ncomp) throw NoriException(NORI_ERR_PARSE, "JPEG: bad SOF length");
            for (int i = 0; i < j.ncomp; ++i) {
                Comp &c = j.comp[i];
                c.id = j.get8();
                const int q = j.get8();
                c.h = q >> 4;
                c.v = q & 15;
                c.tq = j.get8();
                if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3)
                    throw NoriException(NORI_ERR_PARSE, "JPEG: bad sampling factors");
                j.hmax = std::max(j.hmax, c.h);
                j.vmax = std::max(j.vmax, c.v);
            }
            if ((1 << 30) / j.width / j.ncomp < j.height) throw NoriException(NORI_ERR_PARSE, "JPEG: too large");
            j.mcux = (j.width + j.hmax * 8 - 1) / (j.hmax * 8);
            j.mcuy = (j.height + j.vmax * 8 - 1) / (j.vmax * 8);
            for (int i = 0; i < j.ncomp; ++i) {
                Comp &c = j.comp[i];
                c.x = (j.width * c.h + j.hmax - 1) / j.hmax;
                c.y = (j.height * c.v + j.vmax - 1) / j.vmax;
                c.w2 = j.mcux * c.h * 8;
                c.h2 = j.mcuy * c.v * 8;
                c.data.assign((size_t)c.w2 * c.h2, 0);
            }
            frame = true;
        } else if (m == 0xDA) {  // SOS (stb_image.h:1516-1539)
            if (!frame) throw NoriException(NORI_ERR_PARSE, "JPEG: scan before frame");
            const int Ls = j.get16(), n = j.get8();
            if (n < 1 || n > 4 || n > j.ncomp || Ls != 6 + 2 * n) throw NoriException(NORI_ERR_PARSE, "JPEG: bad SOS");
            int order[4];
            for (int i = 0; i < n; ++i) {
                const int id = j.get8(), q = j.get8();
                int w = 0;
                while (w < j.ncomp && j.comp[w].id != id) ++w;
                if (w == j.ncomp) throw NoriException(NORI_ERR_PARSE, "JPEG: bad component id");
                j.comp[w].hd = q >> 4;
                j.comp[w].ha = q & 15;
                if (j.comp[w].hd > 3 || j.comp[w].ha > 3) throw NoriException(NORI_ERR_PARSE, "JPEG: bad table id");
                order[i] = w;
            }
            j.get8();
            j.get8();
            j.get8();  // spectral selection / approximation: baseline 0, 63, 0
            entropy_scan(j, order, n);
        } else if (m == 0xDD) {  // DRI
            if (j.get16() != 4) throw NoriException(NORI_ERR_PARSE, "JPEG: bad DRI length");
            j.restart = j.get16();
        } else if (m == 0xDB) {  // DQT: 8-bit tables
            int L = j.get16() - 2;
            while (L > 0) {
                const int q = j.get8();
                if ((q >> 4) != 0 || (q & 15) > 3) throw NoriException(NORI_ERR_UNSUPPORTED, "JPEG: bad DQT");
                for (int i = 0; i < 64; ++i) j.dq[q & 15][kDezigzag[i]] = (uint8_t)j.get8();
                L -= 65;
            }
        } else if (m == 0xC4) {  // DHT
            int L = j.get16() - 2;
            while (L > 0) {
                const int q = j.get8(), tc = q >> 4, th = q & 15;
                if (tc > 1 || th > 3) throw NoriException(NORI_ERR_PARSE, "JPEG: bad DHT");
                Huff &h = tc ? j.hac[th] : j.hdc[th];
                h = Huff();
                int total = 0;
                for (int i = 1; i <= 16; ++i) total += h.count[i] = j.get8();
                if (total > 256) throw NoriException(NORI_ERR_PARSE, "JPEG: bad DHT");
                int code = 0, k = 0;
                for (int len = 1; len <= 16; ++len) {
                    h.first[len] = code;
                    h.offset[len] = k;
                    code += h.count[len];
                    k += h.count[len];
                    if (code - 1 >= (1 << len) && h.count[len]) throw NoriException(NORI_ERR_PARSE, "JPEG: bad code lengths");
                    code <<= 1;
                }
                for (int i = 0; i < total; ++i) h.values[i] = (uint8_t)j.get8();
                h.present = true;
                L -= 17 + total;
            }
        } else if ((m >= 0xE0 && m <= 0xEF) || m == 0xFE) {  // APPn / COM
            const int L = j.get16();
            j.p = std::min(j.end, j.p + std::max(0, L - 2));
        } else if ((m >= 0xC3 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            throw NoriException(NORI_ERR_UNSUPPORTED, "JPEG: only baseline (SOF0/SOF1) is supported");
        } else if (m >= 0xD0 && m <= 0xD7) {
            // stray restart marker between scans: nothing to do
        } else {
            throw NoriException(NORI_ERR_PARSE, "JPEG: unknown marker");
        }
    }
    if (!frame) throw NoriException(NORI_ERR_PARSE, "JPEG: no frame");
    W = j.width;
    H = j.height;
    rgb.assign((size_t)W * H * 3, 0);
    // resampling state per component (stb_image.h:1855-1897)
    struct Rs {
        int hs, vs, ystep, ypos, wl;
        const uint8_t *line0, *line1;
        std::vector<uint8_t> buf;
    } rs[3];
    for (int k = 0; k < j.ncomp; ++k) {
        Rs &r = rs[k];
        r.hs = j.hmax / j.comp[k].h;
        r.vs = j.vmax / j.comp[k].v;
        r.ystep = r.vs >> 1;
        r.wl = (W + r.hs - 1) / r.hs;
        r.ypos = 0;
        r.line0 = r.line1 = j.comp[k].data.data();
        r.buf.assign((size_t)W + 3 + (size_t)r.wl * r.hs, 0);
    }
    const uint8_t *co[3];
    for (int y = 0; y < H; ++y) {
        for (int k = 0; k < j.ncomp; ++k) {
            Rs &r = rs[k];
            const bool bot = r.ystep >= (r.vs >> 1);
            co[k] = resample(r.buf.data(), bot ? r.line1 : r.line0, bot ? r.line0 : r.line1, r.wl, r.hs, r.vs);
            if (++r.ystep >= r.vs) {
                r.ystep = 0;
                r.line0 = r.line1;
                if (++r.ypos < j.comp[k].y) r.line1 += j.comp[k].w2;
            }
        }
        uint8_t *o = rgb.data() + (size_t)y * W * 3;
        if (j.ncomp == 3) {
            for (int i = 0; i < W; ++i) {
                const int yf = (co[0][i] << 16) + 32768, cr = co[2][i] - 128, cb = co[1][i] - 128;
                const int r = (yf + cr * fx16(1.40200f)) >> 16;
                const int g = (yf - cr * fx16(0.71414f) - cb * fx16(0.34414f)) >> 16;
                const int b = (yf + cb * fx16(1.77200f)) >> 16;
                o[3 * i + 0] = clamp8(r);
                o[3 * i + 1] = clamp8(g);
                o[3 * i + 2] = clamp8(b);
            }
        } else {
            for (int i = 0; i < W; ++i) o[3 * i] = o[3 * i + 1] = o[3 * i + 2] = co[0][i];
        }
    }
}

// ------------------------------------------------------------------ PNG
uint32_t be32(const uint8_t *p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }

int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    if (pb <= pc) return b;
    return c;
}

// un-filter `h` rows of `w` pixels of `n` bytes each from `src` (filter byte + row)
void unfilter(const uint8_t *&src, const uint8_t *end, int w, int h, int n, uint8_t *out) {
    const size_t stride = (size_t)w * n;
    std::vector<uint8_t> zero(stride, 0);
    for (int y = 0; y < h; ++y) {
        if (src + 1 + stride > end) throw NoriException(NORI_ERR_PARSE, "PNG: not enough pixels (Corrupt PNG)");
        const int f = *src++;
        uint8_t *cur = out + (size_t)y * stride;
        const uint8_t *prev = y ? cur - stride : zero.data();
        for (size_t i = 0; i < stride; ++i) {
            const int a = i >= (size_t)n ? cur[i - n] : 0, b = prev[i], c = i >= (size_t)n ? prev[i - n] : 0;
            int v = src[i];
            switch (f) {
            case 0: break;
            case 1: v += a; break;
            case 2: v += b; break;
            case 3: v += (a + b) >> 1; break;
            case 4: v += paeth(a, b, c); break;
            default: throw NoriException(NORI_ERR_PARSE, "PNG: invalid filter (Corrupt PNG)");
            }
            cur[i] = (uint8_t)v;
        }
        src += stride;
    }
}

void decode_png(const std::vector<uint8_t> &bytes, int &W, int &H, std::vector<uint8_t> &rgb) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (bytes.size() < 8 || std::memcmp(bytes.data(), sig, 8) != 0) throw NoriException(NORI_ERR_PARSE, "PNG: bad signature");
    const uint8_t *p = bytes.data() + 8, *end = bytes.data() + bytes.size();
    int depth = 0, color = -1, interlace = 0;
    std::vector<uint8_t> idat, pal;  // palette as RGBA
    bool have_hdr = false;
    while (p + 8 <= end) {
        const uint32_t len = be32(p);
        const uint8_t *type = p + 4, *data = p + 8;
        if (data + len + 4 > end) throw NoriException(NORI_ERR_PARSE, "PNG: truncated chunk");
        if (!std::memcmp(type, "IHDR", 4)) {
            W = (int)be32(data);
            H = (int)be32(data + 4);
            depth = data[8];
            color = data[9];
            interlace = data[12];
            if (depth != 8) throw NoriException(NORI_ERR_UNSUPPORTED, "PNG not supported: 8-bit only");
            if (color != 0 && color != 2 && color != 3 && color != 4 && color != 6)
                throw NoriException(NORI_ERR_PARSE, "PNG: bad color type");
            if (data[10] != 0 || data[11] != 0 || interlace > 1) throw NoriException(NORI_ERR_PARSE, "PNG: bad IHDR");
            if (W <= 0 || H <= 0 || (1 << 30) / W / 4 < H) throw NoriException(NORI_ERR_PARSE, "PNG: too large");
            have_hdr = true;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            if (len > 256 * 3 || len % 3) throw NoriException(NORI_ERR_PARSE, "PNG: invalid PLTE");
            pal.assign(4 * (len / 3), 255);
            for (uint32_t i = 0; i < len / 3; ++i)
                for (int k = 0; k < 3; ++k) pal[4 * i + k] = data[3 * i + k];
        } else if (!std::memcmp(type, "tRNS", 4)) {
            // palette alpha (dropped by the conversion to 3 channels); gray/RGB keys do not change RGB
        } else if (!std::memcmp(type, "CgBI", 4)) {
            throw NoriException(NORI_ERR_UNSUPPORTED, "PNG: Apple CgBI files are not supported");
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), data, data + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        } else if (!(type[0] & 32)) {
            throw NoriException(NORI_ERR_UNSUPPORTED, "PNG: unknown critical chunk");
        }
        p = data + len + 4;  // skip CRC
    }
    if (!have_hdr || idat.empty()) throw NoriException(NORI_ERR_PARSE, "PNG: missing IHDR or IDAT");
    if (color == 3 && pal.empty()) throw NoriException(NORI_ERR_PARSE, "PNG: no PLTE");
    const int n = color == 0 ? 1 : color == 2 ? 3 : color == 3 ? 1 : color == 4 ? 2 : 4;
    // raw size: Adam7 passes or one image, one filter byte per row
    static const int ax[7] = {0, 4, 0, 2, 0, 1, 0}, ay[7] = {0, 0, 4, 0, 2, 0, 1};
    static const int sx[7] = {8, 8, 4, 4, 2, 2, 1}, sy[7] = {8, 8, 8, 4, 4, 2, 2};
    size_t raw_len = 0;
    if (!interlace) {
        raw_len = (size_t)H * (1 + (size_t)W * n);
    } else {
        for (int k = 0; k < 7; ++k) {
            const int pw = (W - ax[k] + sx[k] - 1) / sx[k], ph = (H - ay[k] + sy[k] - 1) / sy[k];
            if (pw > 0 && ph > 0) raw_len += (size_t)ph * (1 + (size_t)pw * n);
        }
    }
    std::vector<uint8_t> raw(raw_len);
    uLongf got = (uLongf)raw_len;
    const int zr = uncompress(raw.data(), &got, idat.data(), (uLong)idat.size());
    if ((zr != Z_OK && zr != Z_BUF_ERROR) || got < raw_len)
        throw NoriException(NORI_ERR_PARSE, "PNG: zlib stream too short or corrupt");
    std::vector<uint8_t> img((size_t)W * H * n);
    const uint8_t *src = raw.data(), *rend = raw.data() + raw.size();
    if (!interlace) {
        unfilter(src, rend, W, H, n, img.data());
    } else {
        for (int k = 0; k < 7; ++k) {
            const int pw = (W - ax[k] + sx[k] - 1) / sx[k], ph = (H - ay[k] + sy[k] - 1) / sy[k];
            if (pw <= 0 || ph <= 0) continue;
            std::vector<uint8_t> sub((size_t)pw * ph * n);
            unfilter(src, rend, pw, ph, n, sub.data());
            for (int y = 0; y < ph; ++y)
                for (int x = 0; x < pw; ++x)
                    std::memcpy(&img[((size_t)(ay[k] + y * sy[k]) * W + ax[k] + x * sx[k]) * n],
                                &sub[((size_t)y * pw + x) * n], n);
        }
    }
    rgb.assign((size_t)W * H * 3, 0);
    for (size_t i = 0; i < (size_t)W * H; ++i) {
        const uint8_t *s = &img[i * n];
        uint8_t *o = &rgb[3 * i];
        if (color == 3) {
            if ((size_t)s[0] * 4 + 3 >= pal.size()) throw NoriException(NORI_ERR_PARSE, "PNG: palette index out of range");
            o[0] = pal[4 * s[0]];
            o[1] = pal[4 * s[0] + 1];
            o[2] = pal[4 * s[0] + 2];
        } else if (n <= 2) {
            o[0] = o[1] = o[2] = s[0];
        } else {
            o[0] = s[0];
            o[1] = s[1];
            o[2] = s[2];
        }
    }
}

}  // namespace

// stbi_load(path, &w, &h, &c, STBI_rgb): the format is chosen by content
void decode_image_rgb8(const std::string &path, int &W, int &H, std::vector<uint8_t> &rgb) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw NoriException(NORI_ERR_IO, "No image data was loaded! (cannot open \"" + path + "\")");
    std::vector<uint8_t> bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (bytes.size() >= 2 && bytes[0] == 0xFF && bytes[1] == 0xD8)
        decode_jpeg(bytes, W, H, rgb);
    else if (bytes.size() >= 8 && bytes[0] == 137 && bytes[1] == 'P')
        decode_png(bytes, W, H, rgb);
    else
        throw NoriException(NORI_ERR_UNSUPPORTED, "No image data was loaded! (\"" + path + "\" is not a JPEG or PNG file)");
}

}  // namespace nori
