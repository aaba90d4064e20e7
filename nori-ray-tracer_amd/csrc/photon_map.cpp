// photon_map.cpp -- host side of the photon map (photonmapper integrator).
//
// The traced photons come back from k_photons as (position, direction, power)
// floats.  Each is stored the way the reference stores it, PhotonData
// (photon.h, photon.cpp:30-74): the direction quantized to 8-bit spherical
// angles and the power in Ward's RGBE, decoded through the same 256-entry
// tables -- so the density estimate sums exactly the reference's photon
// values (the device decodes the packed angles and RGBE through the same
// tables, so only 16 bytes per candidate photon are read).  The reference's kd-tree (kdtree.h) answers "every photon with
// |x - p|^2 < r^2"; here a hash grid of cell size r answers the same query
// from the 27 cells around p (kernels.hip, OneBounce::Li_pmap).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "host_scene.h"

namespace nori {
namespace {

constexpr float kPiF = 3.14159265358979323846f;  // common.h:56 (a float literal)

struct PhotonTables {  // PhotonData::initialize (photon.cpp:30-41)
    float cos_phi[256], sin_phi[256], cos_theta[256], sin_theta[256], exp_table[256];
    PhotonTables() {
        for (int i = 0; i < 256; i++) {
            const float angle = (float)i * (kPiF / 256.0f);
            cos_phi[i] = std::cos(2.0f * angle);
            sin_phi[i] = std::sin(2.0f * angle);
            cos_theta[i] = std::cos(angle);
            sin_theta[i] = std::sin(angle);
            exp_table[i] = std::ldexp(1.0f, i - (128 + 8));
        }
        exp_table[0] = 0;
    }
};

uint32_t cell_hash(const float *p, float ic) {  // == kernels.hip: (int)floorf(p * ic), photon_cell_hash
    const int x = (int)std::floor(p[0] * ic), y = (int)std::floor(p[1] * ic), z = (int)std::floor(p[2] * ic);
    return ((uint32_t)x * 73856093u) ^ ((uint32_t)y * 19349663u) ^ ((uint32_t)z * 83492791u);
}

}  // namespace

void build_photon_map(const std::vector<float> &raw, uint32_t n, float radius, std::vector<float> &photons,
                      std::vector<uint32_t> &rgbe_out, std::vector<float> &tables, std::vector<uint32_t> &start,
                      uint32_t &mask) {
    static const PhotonTables T;
    tables.assign(5 * 256, 0.0f);
    for (int i = 0; i < 256; ++i) {
        tables[i] = T.cos_phi[i], tables[256 + i] = T.sin_phi[i], tables[512 + i] = T.cos_theta[i];
        tables[768 + i] = T.sin_theta[i], tables[1024 + i] = T.exp_table[i];
    }
    // PhotonData(dir, power) (photon.cpp:43-74); the device decodes it as
    // getDirection / getPower (photon.h:44-55) through the same tables
    std::vector<float> dec(4 * (size_t)n);
    std::vector<uint32_t> code(n);
    for (uint32_t i = 0; i < n; ++i) {
        const float *r = &raw[12 * (size_t)i];
        const float dx = r[4], dy = r[5], dz = r[6];
        // all float: common.h:56 makes M_PI a float literal
        const uint8_t theta = (uint8_t)std::min(255, (int)(std::acos(dz) * (256.0f / kPiF)));
        const int tmp = std::min(255, (int)(std::atan2(dy, dx) * (256.0f / (2.0f * kPiF))));
        const uint8_t phi = (uint8_t)(tmp < 0 ? tmp + 256 : tmp);
        uint8_t rgbe[4];
        const float pr = r[8], pg = r[9], pb = r[10];
        float mx = std::max(std::max(pr, pg), pb);
        if (mx < 1e-32) {
            rgbe[0] = rgbe[1] = rgbe[2] = rgbe[3] = 0;
        } else {
            int e;
            mx = std::frexp(mx, &e) * 256.0f / mx;
            rgbe[0] = (uint8_t)(pr * mx);
            rgbe[1] = (uint8_t)(pg * mx);
            rgbe[2] = (uint8_t)(pb * mx);
            rgbe[3] = (uint8_t)(e + 128);
        }
        float *d = &dec[4 * (size_t)i];
        const uint32_t dir = (uint32_t)theta | ((uint32_t)phi << 8);
        d[0] = r[0], d[1] = r[1], d[2] = r[2];
        std::memcpy(&d[3], &dir, 4);
        code[i] = (uint32_t)rgbe[0] | ((uint32_t)rgbe[1] << 8) | ((uint32_t)rgbe[2] << 16) | ((uint32_t)rgbe[3] << 24);
    }
    // hash grid: buckets = the power of two >= 2n, photons sorted by bucket
    uint32_t buckets = 1024;
    while (buckets < 2 * n && buckets < (1u << 30)) buckets <<= 1;
    mask = buckets - 1;
    const float ic = 1.0f / radius;
    std::vector<uint32_t> key(n);
    start.assign((size_t)buckets + 2, 0);
    for (uint32_t i = 0; i < n; ++i) {
        key[i] = cell_hash(&dec[4 * (size_t)i], ic) & mask;
        ++start[key[i] + 1];
    }
    for (uint32_t b = 0; b < buckets; ++b) start[b + 1] += start[b];
    start[(size_t)buckets + 1] = start[buckets];
    std::vector<uint32_t> fill(start.begin(), start.begin() + buckets);
    photons.assign(4 * (size_t)n, 0.0f);
    rgbe_out.assign(n, 0u);
    for (uint32_t i = 0; i < n; ++i) {  // stable: emission order within a bucket
        const uint32_t at = fill[key[i]]++;
        std::memcpy(&photons[4 * (size_t)at], &dec[4 * (size_t)i], 4 * sizeof(float));
        rgbe_out[at] = code[i];
    }
}

}  // namespace nori
