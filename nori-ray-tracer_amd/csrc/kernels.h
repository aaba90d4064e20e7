// kernels.h -- launch wrappers for the gfx950 kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "dev_scene.h"

namespace nori {

constexpr int kShadeBlock = 256;   // shade / regen work-group size
constexpr int kTraceBlock = 128;   // traversal work-group size (LDS stack columns)
constexpr int kTraceSpill = 64;    // traversal stack entries beyond the LDS part (private memory)
#ifndef NORI_STACK_KEYS
#define NORI_STACK_KEYS 1
#endif
// Stack entries held in LDS for an LDS budget of `stack` words per lane: with
// NORI_STACK_KEYS each entry is a (child ref, entry distance) pair.
constexpr int stack_lds_entries(int stack) { return NORI_STACK_KEYS ? stack / 2 : stack; }
constexpr int kSplatBlock = 256;
#ifndef NORI_SCAN_RAYS
#define NORI_SCAN_RAYS 2
#endif
constexpr int kScanRays = NORI_SCAN_RAYS;  // rays per thread of the scan-mode extension kernel
#ifndef NORI_SCAN_RAYS_SHADOW
#define NORI_SCAN_RAYS_SHADOW 1
#endif
constexpr int kScanRaysShadow = NORI_SCAN_RAYS_SHADOW;  // ... and of the scan-mode shadow kernel
#ifndef NORI_SHADE_LDS_MAX
#define NORI_SHADE_LDS_MAX 16384
#endif
constexpr uint32_t kShadeLdsMax = NORI_SHADE_LDS_MAX;  // largest scene blob the shade kernel stages in LDS
// The shade kernels of the full plugin set are compiled without the inline
// shadow rays (S.nee_inline only for basic scenes): with them, C4 3964 and
// C5 4162 against 4000 / 4308 Msamples/s, queue mode both (one box, 2 reps).
// NORI_NEE_FULL=1 compiles them in (NORI_NEE_INLINE=1 then applies there too).
#ifndef NORI_NEE_FULL
#define NORI_NEE_FULL 0
#endif
constexpr bool kNeeFull = NORI_NEE_FULL;

struct SplatDesc {
    uint32_t M;               // pixels per pass in the work list
    uint32_t passes;          // passes in this chunk
    uint32_t pass_begin;      // absolute pass of chunk pass 0
    uint32_t passes_per_wg;   // passes folded by one work-group
    const int4 *blocks;       // (ox, oy, bw | bh << 16, first list entry)
    uint64_t seed;
    float *var;               // per-pixel sample statistics W x H x 8 (sum L, sum L^2, n) or null
};

// Scene-specialised scan kernels (rtc.hip): a scan-mode scene's scan list
// compiled in as literals through hipRTC at context creation.
struct ScanRtcScene {
    const float *rec;  // 12 floats per record
    uint32_t nrec;
    const float *plane_c, *plane_f;  // per pair: 1 and 8 floats
    uint32_t pairs;
    uint32_t plane_end[3];
    uint32_t tris, real;
};
struct ScanRtc {
    hipModule_t mod = nullptr;
    hipFunction_t extend = nullptr, shadow = nullptr, trace[2] = {nullptr, nullptr};  // trace[any_hit]
    hipFunction_t both = nullptr;  // extension + shadow rays of one iteration in one launch (launch_trace_both)
    int k_extend = 0;         // rays per thread of `extend`
    double compile_ms = 0.0;  // hipRTC compile (or cache read) at context creation
    bool cached = false;      // the code object came from the process or disk cache
    size_t code_bytes = 0;
};
std::string rtc_const_scene(const ScanRtcScene &sc);
// Compiles (or finds cached) the specialised code object for target `arch`.
bool rtc_compile(const ScanRtcScene &sc, const std::string &arch, int trace_cull, std::vector<char> &code, double &ms,
                 bool &cached, std::string &why);
// ... and loads it on the current device; false (with why) leaves `out` empty.
bool scan_rtc_build(const ScanRtcScene &sc, int device, int trace_cull, ScanRtc &out, std::string &why);
void scan_rtc_release(ScanRtc &r);
int rtc_rays_per_thread();

// stack = LDS stack depth (8, 16, 32 or 64) chosen from the BVH depth.
// rtc: the scene's specialised scan kernels, used for stack 0 when present.
hipError_t launch_trace(const DevScene &S, const float4 *rays, uint32_t n, int any_hit, float4 *hits, int stack,
                        hipStream_t st, const ScanRtc *rtc = nullptr);
hipError_t launch_shade(const DevScene &S, const PathQueue &in, const PathQueue &out, const ShadowQueue &sq,
                        const SegState &seg, int in_sel, const WorkDesc &wd, float4 *rec, Counters *C,
                        uint32_t nseg, hipStream_t st);
hipError_t launch_extend(const DevScene &S, const PathQueue &q, const uint32_t *cnt, uint32_t G, int stack,
                         hipStream_t st, const ScanRtc *rtc = nullptr);
hipError_t launch_shadow(const DevScene &S, const ShadowQueue &sq, const uint32_t *shcnt, float4 *rec, uint32_t G,
                         int stack, hipStream_t st, const ScanRtc *rtc = nullptr);
// Both trace launches of an iteration as one (the BVH walks, or the
// specialised scan kernels); false: nothing launched (a scan scene without
// them), use launch_extend + launch_shadow.
bool launch_trace_both(const DevScene &S, const PathQueue &q, const uint32_t *cnt, const ShadowQueue &sq,
                       const uint32_t *shcnt, float4 *rec, uint32_t G, int stack, const ScanRtc *rtc, hipStream_t st,
                       hipError_t &err);
// Marks the record of every queued path pending (w = kRecPending, the jitter
// class bits cleared): k_splat skips it, the finisher splats it itself.
// Zeroes the counters and segment state of a chunk, Counters::exhausted = empty.
hipError_t launch_reset(Counters *C, uint32_t empty, const SegState &seg, uint32_t G, hipStream_t st);
hipError_t launch_mark(const PathQueue &Q, const SegState &seg, int sel, float4 *rec, uint32_t G, hipStream_t st);
// The prefix over the segments' path counts that numbers the tail's paths
// (pre: G + 1 words); launch_finish reads it.
hipError_t launch_tail_prefix(const SegState &seg, int sel, uint32_t G, uint32_t *pre, hipStream_t st);
// Completes every queued path and splats its sample into `film` itself.
// (after launch_tail_prefix on the same stream)
hipError_t launch_finish(const DevScene &S, const PathQueue &Q, const SegState &seg, int sel, float4 *rec,
                         const WorkDesc &wd, float *film, Counters *C, uint32_t G, int stack, uint32_t *pre,
                         hipStream_t st);
// Photon tracing (photonmapper preprocess): count pass (out == null) writes
// the photons stored by each emitted photon e0 + i into count[i]; store pass
// writes the photons of emitted photons i < n at pre[i] (3 float4 each:
// position, direction towards the light, power), `total` photons in all.
hipError_t launch_photons(const DevScene &S, uint64_t e0, uint32_t n, uint32_t *count, const uint64_t *pre,
                          uint64_t total, float4 *out, int stack, hipStream_t st);
// One-bounce integrators (normals, av, direct, direct_ems/mats/mis) and the
// photon mapper: one thread per work id of wd (pass-major, pixels in
// wd.pixels order) writes its record.
hipError_t launch_direct(const DevScene &S, const WorkDesc &wd, float4 *rec, Counters *C, int stack, hipStream_t st);
// NL-means denoiser (denoise.hip, denoiser/denoiser.py): img W x H x 3,
// var W x H, radius R (offsets), box half-width P (= the script's f - 1).
size_t denoise_lds_bytes(int R, int P);
hipError_t launch_denoise(const float *img, const float *var, int W, int H, int R, int P, float k, int mode,
                          float *out, hipStream_t st);
hipError_t launch_splat(const DevScene &S, const float4 *rec, const SplatDesc &sd, uint32_t nblocks, float *film,
                        Counters *C, hipStream_t st);

}  // namespace nori
