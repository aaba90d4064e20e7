// photon_map.cpp -- host side of the photon map (photonmapper integrator).
//
// The traced photons come back from k_photons as (position, direction, power)
// floats.  Each is stored the way the reference stores it, PhotonData
// (photon.h, photon.cpp:30-74): the direction quantized to 8-bit spherical
// angles and the power in Ward's RGBE, decoded through the same 256-entry
// tables -- so the density estimate sums exactly the reference's photon
// values.  The reference's kd-tree (kdtree.h) answers "every photon with
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
                      std::vector<uint32_t> &start, uint32_t &mask) {
    static const PhotonTables T;
    // PhotonData(dir, power) (photon.cpp:43-74) and getDirection / getPower (photon.h:44-55)
    std::vector<float> dec(12 * (size_t)n);
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
        float *d = &dec[12 * (size_t)i];
        d[0] = r[0], d[1] = r[1], d[2] = r[2], d[3] = 0;
        d[4] = T.cos_phi[phi] * T.sin_theta[theta];
        d[5] = T.sin_phi[phi] * T.sin_theta[theta];
        d[6] = T.cos_theta[theta], d[7] = 0;
        const float s = T.exp_table[rgbe[3]];
        d[8] = (float)rgbe[0] * s, d[9] = (float)rgbe[1] * s, d[10] = (float)rgbe[2] * s, d[11] = 0;
    }
    // hash grid: buckets = the power of two >= 2n, photons sorted by bucket
    uint32_t buckets = 1024;
    while (buckets < 2 * n && buckets < (1u << 30)) buckets <<= 1;
    mask = buckets - 1;
    const float ic = 1.0f / radius;
    std::vector<uint32_t> key(n);
    start.assign((size_t)buckets + 2, 0);
    for (uint32_t i = 0; i < n; ++i) {
        key[i] = cell_hash(&dec[12 * (size_t)i], ic) & mask;
        ++start[key[i] + 1];
    }
    for (uint32_t b = 0; b < buckets; ++b) start[b + 1] += start[b];
    start[(size_t)buckets + 1] = start[buckets];
    std::vector<uint32_t> fill(start.begin(), start.begin() + buckets);
    photons.assign(12 * (size_t)n, 0.0f);
    for (uint32_t i = 0; i < n; ++i)  // stable: emission order within a bucket
        std::memcpy(&photons[12 * (size_t)fill[key[i]]++], &dec[12 * (size_t)i], 12 * sizeof(float));
}

}  // namespace nori
