// raysort.hip -- queue-wide ray reordering for the BVH walks (NORI_RAY_SORT).
//
// The BVH scenes' extension and shadow launches are latency-bound pointer
// chases ("C3's traversal"): a wave runs as long as its
// longest ray and every lane fetches its own nodes.  Before such a launch the
// queue entries of a pool part are ordered by a spatial key -- a Morton code of
// the ray origin in the scene box (b bits per axis) with the direction octant
// below it -- so that a wave holds rays that start close together and head the
// same way, and, with the XCD-aware block order, each XCD's L2 holds the part
// of the tree its range of rays visits.  Only a 4-byte slot index moves: the
// sorted walk reads each ray from its slot and writes the hit back there, so
// the path state stays where k_shade put it.  Each ray's result does not
// depend on the order the rays are traced in, so images are bit-identical.
//
// Key layout (3b + 4 bits): [morton(o) : 3b][octant(d) : 3], and the value
// 1 << (3b + 3) for empty slots, which sorts them behind every ray.
#include <hipcub/hipcub.hpp>

#include "kernels.h"

namespace nori {

static_assert(kSeg == 256, "k_ray_keys: one work-group of 256 lanes per queue segment");

ND uint32_t spread3(uint32_t v) {  // bits 0..9 of v to bits 0, 3, 6, ...
    v &= 0x3FFu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

struct RayKeyDesc {
    float lo[3], scale[3];  // origin -> [0, 2^b): (o - lo) * scale, clamped
    uint32_t cells;         // 2^b
    uint32_t empty;         // key of an empty slot
};

// Work-group g = queue segment g of the part: lane j keys slot g*kSeg + j
// (a ray when j < cnt[g]); lane 0 adds the segment's count to *n.
__global__ __launch_bounds__(256) void k_ray_keys(const float4 *ro, const float4 *rd, const uint32_t *cnt,
                                                  RayKeyDesc kd, uint32_t *keys, uint32_t *vals, uint32_t *n) {
    const uint32_t g = blockIdx.x, j = threadIdx.x, s = g * kSeg + j;
    const uint32_t c = cnt[g];
    uint32_t key = kd.empty;
    if (j < c) {
        const float4 o = ro[s], d = rd[s];
        const float fmax = (float)(kd.cells - 1);
        const uint32_t ix = (uint32_t)fminf(fmaxf((o.x - kd.lo[0]) * kd.scale[0], 0.0f), fmax);
        const uint32_t iy = (uint32_t)fminf(fmaxf((o.y - kd.lo[1]) * kd.scale[1], 0.0f), fmax);
        const uint32_t iz = (uint32_t)fminf(fmaxf((o.z - kd.lo[2]) * kd.scale[2], 0.0f), fmax);
        const uint32_t oct = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
        key = ((spread3(ix) | spread3(iy) << 1 | spread3(iz) << 2) << 3) | oct;
    }
    keys[s] = key;
    vals[s] = s;
    if (j == 0 && c) atomicAdd(n, c);
}

size_t ray_sort_temp_bytes(uint32_t slots, int bits) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                             (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)slots, 0,
                                             3 * bits + 4);
    return bytes;
}

hipError_t launch_ray_sort(const DevScene &S, const float4 *ro, const float4 *rd, const uint32_t *cnt, uint32_t G,
                           int bits, const RaySortBufs &B, hipStream_t st) {
    if (G == 0 || bits < 1 || bits > 9) return hipErrorInvalidValue;
    RayKeyDesc kd;
    kd.cells = 1u << bits;
    for (int k = 0; k < 3; ++k) {
        const float ext = S.root_max[k] - S.root_min[k];
        kd.lo[k] = S.root_min[k];
        kd.scale[k] = ext > 0.0f ? (float)kd.cells / ext : 0.0f;
    }
    kd.empty = 1u << (3 * bits + 3);
    hipError_t e = hipMemsetAsync(B.n, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_ray_keys, dim3(G), dim3(256), 0, st, ro, rd, cnt, kd, B.keys[0], B.vals[0], B.n);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t bytes = B.temp_bytes;
    return hipcub::DeviceRadixSort::SortPairs(B.temp, bytes, B.keys[0], B.keys[1], B.vals[0], B.vals[1],
                                              (int)(G * kSeg), 0, 3 * bits + 4, st);
}

}  // namespace nori
