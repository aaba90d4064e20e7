// dev_scene.h -- device-resident scene and wavefront queue layouts.
//
// HBM layout (all arrays 16-byte aligned, structure-of-arrays so a wave's
// 64 lanes read/write 64 consecutive 16-byte records = 1 KiB per access):
//   nodes      float4[8*N]   4-wide BVH, 128 B per inner node (host_scene.h)
//   prims      float4[3*P]   48 B per primitive in leaf order
//   tri_vidx   uint32[3*P]   vertex ids per global primitive (shading)
//   pos, nrm   float4[V]     vertex position + texture u / normal + texture v
//   prim_shape uint32[P]     global primitive -> shape
//   cdf        float[]       per-mesh area CDFs (DiscretePDF, dpdf.h)
// Path queues (two, ping-ponged) hold one path per entry, 52 B + the hit:
//   ray_o float4 (o.xyz, previous bsdf pdf | -1; a camera ray: 1/z of its
//                 camera-space direction, so mint = near/z, maxt = far/z)
//   ray_d float4 (d.xyz, sample record index (bits 0-28) | colour channel
//                 of a chromatic-aberration sample (bits 29-30) | bit 31:
//                 camera ray; any other ray has mint = Epsilon, maxt = inf)
//   thr   float4 (beta.rgb, pcg32 state bits 0-31)
//   rng   uint32 (pcg32 state bits 32-63; the stream increment is
//                 2 sid + 1 of the sample id, recomputed from the record index)
//   hit   float4 (t, prim, u, v)
// Shadow queue: ray_o, ray_d, payload float4 (contribution.rgb, work).
// Sample records: float4 per camera sample (L.rgb, 0).
#pragma once
#ifndef __HIPCC_RTC__  // (hipRTC: the runtime header is built in)
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>

#include "device_math.h"
#include "seg_index.h"

namespace nori {

struct DevShape {
    int32_t type, bsdf, emitter, has_normals;
    uint32_t prim_offset, prim_count, cdf_offset, has_uvs;
    float center[3], radius;
    float area_norm;     // DiscretePDF::getNormalization (mesh) or sphere pdf
    int32_t nm_w, nm_h, nm_wrap;  // NormalMap (meshes with normals, mesh.cpp:147-155)
    // sphere only: no other primitive meets the closed ball (host-checked with
    // a margin, and the ball lies inside the scene box): a ray from a point of
    // this sphere that hits it again hits nothing before (the chord is inside
    // the ball), so the tail finisher takes that hit without a scene scan
    int32_t solitary;
    const uint32_t *nmap;         // RGBX8 texels in global memory, or null
};

// 128 B.  Area: radiance.  Envmap (envmap.cpp): R x C texels (R = Bitmap rows,
// the reference's m_width), tables at float offsets into DevScene::env:
// rgb R*C*3, pdf R*C, cdf R*(C+1), marginal pdf R, marginal cdf R+1.
// Point (pointlight.cpp): position, power.  Spot (spotlight.cpp): position,
// power (= "color"), direction, cosines of falloffStart and totalWidth.
struct DevEmitter {
    int32_t type, shape;
    float radiance[3];
    float weight;
    int32_t R, C;
    uint32_t rgb_off, pdf_off, cdf_off, pmarg_off, cmarg_off;
    float position[3], power[3], direction[3], cos_fs, cos_tw;
    uint32_t pad[8];
};
static_assert(sizeof(DevEmitter) == 128, "DevEmitter layout");

struct DevScene {
    const float4 *nodes;
    const float4 *prims;
    const uint32_t *tri_vidx;
    const float4 *pos;
    const float4 *nrm;
    const uint32_t *prim_shape;
    const DevShape *shapes;
    const DevBsdf *bsdfs;
    const DevEmitter *emitters;
    const float *cdf;
    const float *env;  // envmap tables (DevEmitter offsets), global memory
    uint32_t num_emitters;
    uint32_t num_nodes;
    uint32_t num_prims;
    uint32_t num_scan_tris;  // scan mode: prims = triangles (padded to kScanGroup), then spheres
    uint32_t num_scan_real;  // scan mode: triangle records before the padding of the last group
    // scan mode: axis-plane triangle pairs (runtime.hip build_scan_list):
    // pair g = scan records 2g, 2g+1 in the plane x_a = plane_c[g], pairs of
    // axis a are [plane_end[a-1], plane_end[a])
    const float *plane_c;
    // per pair: the in-plane filter of k_extend_bin (runtime.hip plane_filters)
    const float4 *plane_f;
    uint32_t plane_end[3];
    // run-time switches of the scan's exact wall-pair skips (nori_gpu_create:
    // NORI_CAMERA_CULL, NORI_TRACE_CULL): camera_cull != 0 -- k_extend_scan
    // filters the pairs of a wave of camera rays by the in-plane test
    // (pair_candidate); trace_cull -- the trace API's scan: 0 tests every
    // pair, 1 the plane-distance skip (plane_may_hit), 2 the in-plane filter
    int32_t camera_cull, trace_cull;
    // scan-mode scenes: k_shade traces its next-event shadow rays itself
    // (kernels.hip k_shade) instead of queueing them for k_shadow_scan
    // (nori_gpu_create: NORI_NEE_INLINE=0 keeps the queue)
    int32_t nee_inline;
    float root_min[3], root_max[3];  // scene box = BVH root box (bvh.cpp:345)
    int32_t W, H;
    float invW, invH;
    float s2c[16];
    float c2w[16];
    float cam_o[3];  // cameraToWorld * (0,0,0,1) / w (perspective.cpp:104)
    float near_clip, far_clip;
    int32_t cam_type;          // NORI_CAMERA_*
    float lens_radius, focal;  // thinlens / advancedCamera
    float distortion[2];       // advancedCamera barrel distortion
    float chromatic[3];        // advancedCamera chromatic aberration (zero otherwise)
    int32_t chroma;            // chromatic != 0: three Li calls per sample, one per colour channel
    // 1: only the basic plugins (constant-albedo diffuse, mirror, dielectric;
    // area lights; perspective camera; no normal maps): the path kernels run
    // their FULL = false variants (device_math.h albedo_at)
    int32_t basic;
    int32_t W_max;             // max(W, H)
    float av_length;           // "av" integrator
    float filter[NORI_FILTER_RESOLUTION + 1];
    float filter_radius, lookup;
    int32_t border;
    // != 0 (= lookup, a power of two <= 64): a sample record's w word carries
    // the sub-pixel class of its jitter (jit_class), from which k_splat reads
    // the filter weights instead of re-deriving the jitter from pcg32
    int32_t jit_lk;
    int32_t integrator;
    // 1: next-event estimation at a mirror/dielectric vertex only draws its
    // three random numbers (deviation D10; no environment-map emitter)
    int32_t skip_discrete_nee;
    // homogeneous medium (medium.cpp)
    int32_t has_medium;
    float mbox_min[3], mbox_max[3];
    float sigma_t[3], albedo[3];
    // Small scenes: every table above packed into one blob (byte offsets),
    // which latency-bound kernels stage into LDS (blob_bytes == 0: none).
    // photonmapper: photons sorted by hash-grid bucket, bucket starts
    // (ph_mask + 2 entries), cell size r
    const float4 *ph;            // (x, y, z, theta | phi << 8 as bits): 16 B read per candidate
    const uint32_t *ph_rgbe;     // r | g << 8 | b << 16 | e << 24, read for photons inside the radius
    const float *ph_tab;         // PhotonData tables: cos phi, sin phi, cos theta, sin theta, exp (5 x 256)
    const uint32_t *ph_start;
    uint32_t ph_mask;
    float ph_inv_cell, ph_r2, ph_norm;  // 1/r, r*r, r*r*photonCount (photonmapper.cpp:177)
    const float4 *blob;
    uint32_t blob_bytes;
    uint32_t off_prims, off_vidx, off_pos, off_nrm, off_pshape, off_shapes, off_bsdfs, off_emitters, off_cdf,
        off_nodes;
};

// Photon-map hash grid: integer cell -> bucket (masked by the caller).
NHD uint32_t photon_cell_hash(int x, int y, int z) {
    return ((uint32_t)x * 73856093u) ^ ((uint32_t)y * 19349663u) ^ ((uint32_t)z * 83492791u);
}
// Stream seed of the photon-tracing pass: photon e draws from pcg32 stream
// wave_seed(kPhotonSeed, e) (deviation D8; the reference draws every photon
// from one unseeded sampler in sequence, photonmapper.cpp:47-48).
constexpr uint64_t kPhotonSeed = 0x70686f746f6e6d70ull;

// A copy of S whose small-scene tables point into `lds` (the staged blob).
ND DevScene scene_in_lds(const DevScene &S, const char *lds) {
    DevScene L = S;
    L.prims = reinterpret_cast<const float4 *>(lds + S.off_prims);
    L.tri_vidx = reinterpret_cast<const uint32_t *>(lds + S.off_vidx);
    L.pos = reinterpret_cast<const float4 *>(lds + S.off_pos);
    L.nrm = reinterpret_cast<const float4 *>(lds + S.off_nrm);
    L.prim_shape = reinterpret_cast<const uint32_t *>(lds + S.off_pshape);
    L.shapes = reinterpret_cast<const DevShape *>(lds + S.off_shapes);
    L.bsdfs = reinterpret_cast<const DevBsdf *>(lds + S.off_bsdfs);
    L.emitters = reinterpret_cast<const DevEmitter *>(lds + S.off_emitters);
    L.cdf = reinterpret_cast<const float *>(lds + S.off_cdf);
    L.nodes = reinterpret_cast<const float4 *>(lds + S.off_nodes);
    return L;
}

struct PathQueue {
    float4 *ray_o;   // (o, prev | camera ray: 1/z)
    float4 *ray_d;   // (d, work | kCameraRay)
    float4 *hit;
    float4 *thr;     // (beta, pcg32 state low word)
    uint32_t *rng;   // pcg32 state high word
};
constexpr uint32_t kCameraRay = 0x80000000u;  // ray_d.w flag: mint/maxt from the camera clip planes
constexpr uint32_t kChanShift = 29;            // ray_d.w bits 29-30: colour channel (chromatic aberration)
constexpr uint32_t kWorkMask = (1u << kChanShift) - 1u;  // record index (work ids < 2^29: runtime chunking)

struct ShadowQueue {
    float4 *ray_o;
    float4 *ray_d;
    float4 *payload;
};

// Segmented queues: shade work-group b owns queue entries [b*kSeg, (b+1)*kSeg)
// of the path queues and of the shadow queue; counts are per segment, so no
// global atomics are needed to compact.  Work ids reach a segment through a
// static stream of 256-id chunks (consecutive ids = adjacent pixels of one
// 32x32 block, so a segment traces coherent camera rays).
#ifndef NORI_SCAN_GROUP
#define NORI_SCAN_GROUP 4
#endif
constexpr uint32_t kScanGroup = NORI_SCAN_GROUP;  // triangles fetched per batch of scalar loads in the scan
struct WorkDesc {
    uint64_t total;          // work ids in this chunk of passes
    uint32_t M;              // pixels in the selected blocks
    uint32_t pass_begin;     // absolute pass of work id 0
    const uint32_t *pixels;  // M entries, y*W + x, block-major
    uint64_t seed;
    uint32_t G;              // segments
    uint32_t *done_flag;     // host-mapped: set when the last segment exhausts its stream
    uint32_t rot;            // stream rotation (stream_rotation)
    uint32_t b0;             // global id of the launch's segment 0 (pool halves on two streams)
    float *var;              // per-pixel sample statistics W x H x 8 (sum L, sum L^2, n) or null
};
// Round j hands segment b the chunk (b + j*rot) mod G of that round.  Path
// lengths vary strongly across the image, so every segment's stream must
// sample the whole image evenly or the segments run dry at very different
// times: rot = chunks per pass / rounds spreads a segment's rounds over the
// pass at equal strides (each round is a shift, so any rot is a bijection).
NHD uint64_t stream_work(const WorkDesc &wd, uint32_t b, uint32_t p) {
    uint64_t j = p / kSeg;
    uint64_t col = (b + j * wd.rot) % wd.G;
    return (j * wd.G + col) * kSeg + (p % kSeg);
}
inline uint32_t stream_rotation(uint64_t total, uint32_t M, uint32_t G) {
    uint64_t chunks_per_pass = (M + kSeg - 1) / kSeg;
    uint64_t rounds = (total + (uint64_t)G * kSeg - 1) / ((uint64_t)G * kSeg);
    uint64_t r = rounds ? chunks_per_pass / rounds : 1;
    return (uint32_t)(r ? r : 1);
}

struct SegState {
    uint32_t *cnt[2];   // paths per segment (ping-pong)
    uint32_t *shcnt;    // shadow rays per segment
    uint32_t *cursor;   // work-stream position per segment
    uint4 *stats;       // per segment: extension rays, shadow rays, samples started, finisher rays
};

// Device counters, each on its own 128-byte line.
struct Counters {
    uint32_t exhausted;            // segments whose work stream is used up
    uint32_t pad0[31];
    unsigned long long invalid;    // dropped samples (splat)
    unsigned long long prof[15];   // profiling builds only (NORI_PROF_SHADE / NORI_PROF_FINISH): phase clocks
    uint32_t finish_paths;         // paths completed by the tail finisher
    uint32_t finish_max_rays;      // most rays traced by one finisher path
    uint32_t pad2[30];
    unsigned long long direct_rays[2];  // one-bounce integrators: closest-hit, shadow rays
    unsigned long long pad3[14];
};

}  // namespace nori
