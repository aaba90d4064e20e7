// runtime.hip -- libnori_gpu host runtime and C ABI (include/nori_gpu.h).
//
// nori_gpu_render replaces RenderThread::renderScene's pass loop
// (render.cpp:173-250): instead of spp sequential passes of a
// tbb::parallel_for over 32x32 blocks, every (pass, pixel) sample of the
// requested blocks becomes a work id; a pool of paths stays resident in HBM
// and the shade kernel refills finished slots from a device work counter, so
// the GPU stays full until the last sample.  Radiance accumulates per sample
// record; after the pool drains, k_splat applies ImageBlock::put.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "comm.h"
#include "host_scene.h"
#include "kernels.h"

namespace nori {

static thread_local std::string g_last_error;
constexpr uint32_t kScanMaxPrims = 64;  // wave-uniform scan instead of BVH at or below this
constexpr size_t kBlobMaxBytes = 48 << 10;  // small-scene blob staged into LDS

#define HIP_TRY(x)                                                                                       \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) throw NoriException(NORI_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    void ensure(size_t n) {
        if (n <= bytes && p) return;
        release();
        hipError_t e = hipMalloc(&p, n ? n : 16);
        if (e != hipSuccess) {
            p = nullptr;
            throw NoriException(NORI_ERR_OOM, std::string("hipMalloc(") + std::to_string(n) + "): " + hipGetErrorString(e));
        }
        bytes = n;
    }
    template <class T> void upload(const std::vector<T> &v) {
        ensure(v.size() * sizeof(T));
        if (!v.empty()) HIP_TRY(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    }
    template <class T> T *as() const { return reinterpret_cast<T *>(p); }
};

// rfilter.cpp -> tabulated filter (block.cpp:54-66)
static float filter_eval(const nori_camera_desc &c, float x) {
    switch (c.filter_type) {
    case NORI_FILTER_GAUSSIAN: {
        float alpha = -1.0f / (2.0f * c.filter_p0 * c.filter_p0);
        float v = std::exp(alpha * x * x) - std::exp(alpha * c.filter_radius * c.filter_radius);
        return 0.0f < v ? v : 0.0f;
    }
    case NORI_FILTER_MITCHELL: {
        float B = c.filter_p0, C = c.filter_p1;
        x = std::fabs(2.0f * x / c.filter_radius);
        float x2 = x * x, x3 = x2 * x;
        if (x < 1) return 1.0f / 6.0f * ((12 - 9 * B - 6 * C) * x3 + (-18 + 12 * B + 6 * C) * x2 + (6 - 2 * B));
        if (x < 2) return 1.0f / 6.0f * ((-B - 6 * C) * x3 + (6 * B + 30 * C) * x2 + (-12 * B - 48 * C) * x + (8 * B + 24 * C));
        return 0.0f;
    }
    case NORI_FILTER_TENT: {
        float v = 1.0f - std::fabs(x);
        return 0.0f < v ? v : 0.0f;
    }
    case NORI_FILTER_BOX: return 1.0f;
    case NORI_FILTER_WINDOWED: {
        x = std::fabs(x);
        const float pi = 3.14159265358979323846f;
        auto sinc = [&](float y) { return y < 1e-5f ? 1.0f : std::sin(pi * y) / (pi * y); };
        return sinc(x) * sinc(x / c.filter_p0);
    }
    }
    return 0.0f;
}
static int film_border(const nori_camera_desc &c) { return (int)std::ceil(c.filter_radius - 0.5f); }
// k_splat's weights from a jitter class (kernels.hip jit_class) need every
// step of ImageBlock::put's index arithmetic exact: a power-of-two radius and
// lookup factor (radius * lookup = NORI_FILTER_RESOLUTION), lookup <= 64 so
// that a class fits 8 bits.  The reference's default radii (gaussian and
// Mitchell 2, tent 1, box 0.5) qualify; other filters keep the pcg32 jitter.
static bool pow2f(float v) {
    int e = 0;
    return v > 0.0f && std::frexp(v, &e) == 0.5f;
}
static int jit_code_lookup(float radius, float lookup) {
    if (const char *e = std::getenv("NORI_JIT_CODE"); e && e[0] == '0') return 0;  // A/B
    if (!pow2f(radius) || !pow2f(lookup) || lookup > 64.0f || radius * lookup != (float)NORI_FILTER_RESOLUTION)
        return 0;
    return (int)lookup;
}
static void filter_table(const nori_camera_desc &c, float *t) {
    for (int i = 0; i < NORI_FILTER_RESOLUTION; ++i) t[i] = filter_eval(c, (c.filter_radius * i) / NORI_FILTER_RESOLUTION);
    t[NORI_FILTER_RESOLUTION] = 0.0f;
}

// EnvironmentMap tables (envmap.cpp:13-58, 91-109), appended to `env`.
// precompute1D literally: res is the LAST value of `i + f(row, i)`, and the CDF
// accumulates pf(i - 1), a column-major linear index into the whole pf matrix
// (rows not yet computed read as 0, as from a fresh allocation).
static float env_precompute1D(int row, const float *f, int cols, float *pf, float *Pf, int pf_rows) {
    float res = 0;
    int i;
    for (i = 0; i < cols; i++) res = (float)i + f[(size_t)row * cols + i];
    if (res == 0) return res;
    for (int j = 0; j < cols; j++) pf[(size_t)row * cols + j] = f[(size_t)row * cols + j] / res;
    Pf[(size_t)row * (cols + 1)] = 0;
    for (i = 1; i < cols; i++) {
        const int k = i - 1;
        Pf[(size_t)row * (cols + 1) + i] =
            Pf[(size_t)row * (cols + 1) + i - 1] + pf[(size_t)(k % pf_rows) * cols + (k / pf_rows)];
    }
    Pf[(size_t)row * (cols + 1) + i] = 1;
    return res;
}
static void build_envmap(const nori_emitter_desc &e, DevEmitter &o, std::vector<float> &env) {
    const int R = e.env_rows, C = e.env_cols;
    if (R < 2 || C < 2 || !e.env_rgb) throw NoriException(NORI_ERR_INVALID, "EnvMap: the image needs at least 2x2 texels");
    o.weight = e.weight;
    o.R = R;
    o.C = C;
    auto grab = [&](size_t n) {
        const size_t off = env.size();
        env.resize(off + n, 0.0f);
        return (uint32_t)off;
    };
    o.rgb_off = grab(3 * (size_t)R * C);
    std::memcpy(&env[o.rgb_off], e.env_rgb, 12 * (size_t)R * C);
    o.pdf_off = grab((size_t)R * C);
    o.cdf_off = grab((size_t)R * (C + 1));
    o.pmarg_off = grab((size_t)R);
    o.cmarg_off = grab((size_t)R + 1);
    if (env.size() >= (1ull << 32)) throw NoriException(NORI_ERR_UNSUPPORTED, "EnvMap: tables above 4G floats");
    std::vector<float> lum((size_t)R * C), sum((size_t)R);
    for (int i = 0; i < R; i++)
        for (int j = 0; j < C; j++) {
            const float *c = e.env_rgb + 3 * ((size_t)i * C + j);
            lum[(size_t)i * C + j] =
                std::sqrt((e.lum_scale[0] * c[0] + e.lum_scale[1] * c[1]) + e.lum_scale[2] * c[2]) + kEps / 10000000;
        }
    for (int i = 0; i < R; ++i) sum[i] = env_precompute1D(i, lum.data(), C, &env[o.pdf_off], &env[o.cdf_off], R);
    env_precompute1D(0, sum.data(), R, &env[o.pmarg_off], &env[o.cmarg_off], 1);
}

// BlockGenerator spiral (block.cpp:140-188)
static std::vector<uint32_t> spiral_blocks(int W, int H) {
    int nx = (int)std::ceil(W / (float)NORI_BLOCK_SIZE), ny = (int)std::ceil(H / (float)NORI_BLOCK_SIZE);
    std::vector<uint32_t> out;
    int left = nx * ny, dir = 0, bx = nx / 2, by = ny / 2, steps = 1, numSteps = 1;
    while (left > 0) {
        out.push_back((uint32_t)(by * nx + bx));
        if (--left == 0) break;
        do {
            switch (dir) {
            case 0: ++bx; break;
            case 1: ++by; break;
            case 2: --bx; break;
            default: --by; break;
            }
            if (--steps == 0) {
                dir = (dir + 1) % 4;
                if (dir == 2 || dir == 0) ++numSteps;
                steps = numSteps;
            }
        } while (bx < 0 || by < 0 || bx >= nx || by >= ny);
    }
    return out;
}

}  // namespace nori

using namespace nori;

struct nori_scene {
    std::unique_ptr<HostScene> hs;
};

constexpr int kMaxParts = 4;  // pool parts on separate streams (GPU_MAX_HW_QUEUES is 4)

struct nori_gpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;       // film splat, overlapped with the tail finisher
    hipEvent_t fork = nullptr, join = nullptr;
    hipStream_t parts[kMaxParts] = {};  // parts[0] unused (part 0 runs on `stream`)
    hipEvent_t joins[kMaxParts] = {};
    DevScene S{};
    ScanRtc rtc;         // scan-mode scenes: the scan kernels specialised for this scene (rtc.hip), or empty
    // an iteration's extension and shadow rays of a part in one launch
    // (launch_trace_both); set at upload_scene (NORI_TRACE_FUSE=0 / 1 forces it)
    bool fuse_trace = true;
    // the tail's finisher enqueued before the film splat beside it (NORI_FINISH_FIRST=0: after)
    bool finish_first = true;
    nori_camera_desc cam{};
    DevBuf nodes, prims, tri_vidx, pos, nrm, prim_shape, shapes, bsdfs, emitters, cdf, env, blob, plane_c, plane_f;
    DevBuf tex;          // ImageTexture / NormalMap texels (RGBX8), global memory
    uint32_t spp = 1;    // the scene's sampleCount (default pass count)
    int stack = 8;       // traversal of extend/shadow: 0 = wave-uniform scan, else LDS stack depth
    uint32_t bvh_depth = 0, bvh_nodes = 0, num_prims = 0;
    size_t scene_bytes = 0;
    std::atomic<int> cancel{0};
    std::atomic<float> progress{1.0f};
    // render state
    DevBuf q[2][5], sq[3], seg[4], segstats, tailpre, rec, counters, pixels, blocks, film;
    DevBuf varbuf;                   // per-pixel sample statistics when variance_out is a host buffer
    DevBuf ph, ph_rgbe, ph_tab, ph_start;             // photonmapper: photon map (photon_map.cpp) and its hash-grid buckets
    uint32_t pool_cap = 0;
    uint32_t *pinned = nullptr;      // host-mapped flags: [0] done, [1] exhausted segments
    uint32_t *pinned_dev = nullptr;  // device view of `pinned`
    // the render's blocks (spiral order, block_subset applied) and their
    // block-major pixel list, with device copies in `pixels` / `blocks`:
    // rebuilt and uploaded only when the block selection changes
    std::vector<uint32_t> work_order, hpixels;
    std::vector<int4> hblocks;
    bool work_valid = false;
    // pinned staging of the end-of-render read-back (Counters + per-segment stats)
    char *readback = nullptr;
    size_t readback_bytes = 0;
    std::vector<hipEvent_t> ring[kMaxParts];
    ~nori_gpu_ctx() {
        for (auto &r : ring)
            for (auto e : r) (void)hipEventDestroy(e);
        for (int h = 1; h < kMaxParts; ++h) {
            if (joins[h]) (void)hipEventDestroy(joins[h]);
            if (parts[h]) (void)hipStreamDestroy(parts[h]);
        }
        scan_rtc_release(rtc);
        if (pinned) (void)hipHostFree(pinned);
        if (readback) (void)hipHostFree(readback);
        if (fork) (void)hipEventDestroy(fork);
        if (join) (void)hipEventDestroy(join);
        if (side) (void)hipStreamDestroy(side);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

struct nori_gpu_comm {
    void *nccl = nullptr;  // ncclComm_t (comm.cpp)
    int nranks = 1, rank = 0, device = 0;
    bool aborted = false;   // ncclCommAbort ran: every later call fails
    int *status_dev = nullptr, *status_host = nullptr;  // the per-render status exchange word
    ~nori_gpu_comm() {
        if (!aborted) comm_destroy(nccl);
        if (status_dev) (void)hipFree(status_dev);
        if (status_host) (void)hipHostFree(status_host);
    }
};

namespace {

int fail(int code, const std::string &m) {
    g_last_error = m;
    return code;
}

template <class F> int guarded(F &&f) {
    try {
        g_last_error.clear();
        return f();
    } catch (const NoriException &e) {
        return fail(e.code, e.what());
    } catch (const std::bad_alloc &) {
        return fail(NORI_ERR_OOM, "host allocation failed");
    } catch (const std::exception &e) {
        return fail(NORI_ERR_INVALID, e.what());
    }
}

// Scene box = BVH root box: every mesh vertex and every sphere's bounds.
void scene_root_box(const nori_scene_desc &d, float rmin[3], float rmax[3]) {
    for (int k = 0; k < 3; ++k) rmin[k] = __builtin_inff(), rmax[k] = -__builtin_inff();
    auto expand = [&](float x, float y, float z) {
        float p[3] = {x, y, z};
        for (int k = 0; k < 3; ++k) {
            rmin[k] = std::fmin(rmin[k], p[k]);
            rmax[k] = std::fmax(rmax[k], p[k]);
        }
    };
    for (uint32_t s = 0; s < d.num_shapes; ++s) {
        const nori_shape_desc &sd = d.shapes[s];
        if (sd.type == NORI_SHAPE_SPHERE) {
            expand(sd.center[0] - sd.radius, sd.center[1] - sd.radius, sd.center[2] - sd.radius);
            expand(sd.center[0] + sd.radius, sd.center[1] + sd.radius, sd.center[2] + sd.radius);
        } else {
            for (uint32_t v = 0; v < sd.vtx_count; ++v) {
                const float *p = d.positions + 3 * (size_t)(sd.vtx_offset + v);
                expand(p[0], p[1], p[2]);
            }
        }
    }
}

// DevShape::solitary for every sphere: no other primitive comes within a
// margin of its closed ball and the ball lies inside the scene box (rmin,
// rmax) by that margin.  Closest point of a triangle to the centre: Ericson,
// Real-Time Collision Detection 5.1.5, in double precision.
double point_triangle_dist2(const double p[3], const float *a, const float *b, const float *c) {
    double ab[3], ac[3], ap[3];
    for (int k = 0; k < 3; ++k) ab[k] = (double)b[k] - a[k], ac[k] = (double)c[k] - a[k], ap[k] = p[k] - a[k];
    auto dot = [](const double *x, const double *y) { return x[0] * y[0] + x[1] * y[1] + x[2] * y[2]; };
    auto dist2 = [&](const double q[3]) {
        double s = 0;
        for (int k = 0; k < 3; ++k) s += (p[k] - q[k]) * (p[k] - q[k]);
        return s;
    };
    double q[3];
    const double d1 = dot(ab, ap), d2 = dot(ac, ap);
    if (d1 <= 0 && d2 <= 0) { for (int k = 0; k < 3; ++k) q[k] = a[k]; return dist2(q); }
    double bp[3];
    for (int k = 0; k < 3; ++k) bp[k] = p[k] - b[k];
    const double d3 = dot(ab, bp), d4 = dot(ac, bp);
    if (d3 >= 0 && d4 <= d3) { for (int k = 0; k < 3; ++k) q[k] = b[k]; return dist2(q); }
    const double vc = d1 * d4 - d3 * d2;
    if (vc <= 0 && d1 >= 0 && d3 <= 0) {
        const double v = d1 / (d1 - d3);
        for (int k = 0; k < 3; ++k) q[k] = a[k] + v * ab[k];
        return dist2(q);
    }
    double cp[3];
    for (int k = 0; k < 3; ++k) cp[k] = p[k] - c[k];
    const double d5 = dot(ab, cp), d6 = dot(ac, cp);
    if (d6 >= 0 && d5 <= d6) { for (int k = 0; k < 3; ++k) q[k] = c[k]; return dist2(q); }
    const double vb = d5 * d2 - d1 * d6;
    if (vb <= 0 && d2 >= 0 && d6 <= 0) {
        const double w = d2 / (d2 - d6);
        for (int k = 0; k < 3; ++k) q[k] = a[k] + w * ac[k];
        return dist2(q);
    }
    const double va = d3 * d6 - d5 * d4;
    if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
        const double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        for (int k = 0; k < 3; ++k) q[k] = b[k] + w * ((double)c[k] - b[k]);
        return dist2(q);
    }
    const double den = 1.0 / (va + vb + vc), v = vb * den, w = vc * den;
    for (int k = 0; k < 3; ++k) q[k] = a[k] + ab[k] * v + ac[k] * w;
    return dist2(q);
}

void mark_solitary_spheres(const nori_scene_desc &d, const float rmin[3], const float rmax[3],
                           std::vector<DevShape> &shapes) {
    if (const char *e = std::getenv("NORI_CHORD"); e && e[0] == '0') return;  // A/B: full scans only
    for (uint32_t s = 0; s < d.num_shapes; ++s) {
        const nori_shape_desc &sp = d.shapes[s];
        if (sp.type != NORI_SHAPE_SPHERE || !(sp.radius > 0.0f)) continue;
        const double r = sp.radius, c[3] = {sp.center[0], sp.center[1], sp.center[2]};
        const double margin = 1e-4 * (std::max({std::fabs(c[0]), std::fabs(c[1]), std::fabs(c[2])}) + r);
        bool ok = true;
        for (int k = 0; k < 3 && ok; ++k) ok = c[k] - r > (double)rmin[k] + margin && c[k] + r < (double)rmax[k] - margin;
        const double reach = r + margin;
        for (uint32_t o = 0; o < d.num_shapes && ok; ++o) {
            if (o == s) continue;
            const nori_shape_desc &od = d.shapes[o];
            if (od.type == NORI_SHAPE_SPHERE) {
                double dd = 0;
                for (int k = 0; k < 3; ++k) dd += (c[k] - od.center[k]) * (c[k] - od.center[k]);
                ok = std::sqrt(dd) > reach + od.radius;
                continue;
            }
            for (uint32_t t = 0; t < od.tri_count && ok; ++t) {
                const uint32_t *f = d.indices + 3 * (size_t)(od.tri_offset + t);
                const float *p0 = d.positions + 3 * (size_t)f[0], *p1 = d.positions + 3 * (size_t)f[1],
                            *p2 = d.positions + 3 * (size_t)f[2];
                bool far = false;  // quick reject: the triangle's box misses the ball's box
                for (int k = 0; k < 3; ++k)
                    far = far || std::min({p0[k], p1[k], p2[k]}) > c[k] + reach || std::max({p0[k], p1[k], p2[k]}) < c[k] - reach;
                if (!far) ok = point_triangle_dist2(c, p0, p1, p2) > reach * reach;
            }
        }
        shapes[s].solitary = ok ? 1 : 0;
        if (std::getenv("NORI_DEBUG")) std::fprintf(stderr, "[nori] sphere shape %u: solitary %d\n", s, (int)ok);
    }
}

// The scan list of scan-mode scenes (kernels.hip scan_core).  Triangles that
// lie in an axis plane -- both edges with an exactly zero component on the
// same axis a, so every vertex has x_a = c -- come first, paired by plane:
// the kernels skip such a pair for a whole wave when no ray of the wave can
// hit it, a test that is exact only under the conditions checked here (no
// cancellation in the one remaining product difference of det and of t's
// numerator, kernels.hip plane_may_hit).  Pairs are ordered by axis (the
// kernels loop over each axis separately); a plane holding an odd number of
// triangles pads its last pair with a record no ray hits.  The remaining
// triangles follow, padded to kScanGroup, then the spheres.  Every record
// carries its leaf-order position in e2.w: among equal t the scan keeps the
// hit of the later leaf position, the reference's traversal order.
bool debug_log();
struct ScanList {
    std::vector<float> prims;   // 12 floats per record
    std::vector<float> plane_c; // per pair: the plane coordinate c
    std::vector<float> plane_f; // per pair: the in-plane filter of k_extend_bin (8 floats, plane_filters)
    uint32_t plane_end[3] = {0, 0, 0};  // pairs with axis <= a
    uint32_t tris = 0;          // triangle records (pairs + the rest, padded)
    uint32_t real = 0;          // ... of which the last real one ends here (the padding after it never hits)
};

// The in-plane filter of the binned extension kernel (kernels.hip
// pair_candidate): a ray can be accepted by the Moller-Trumbore test of a
// triangle of pair g only if its crossing with the pair's plane x_A = c lies
// within the pair's in-plane bounding rectangle widened by a margin M that
// covers every rounding error of the test.  Derivation (A the plane axis, B
// and C the other two, u = 2^-24, gamma_k = k u / (1 - k u)): with e1_A =
// e2_A = 0, the reference's u numerator tvec . (d x e2) divided by the exact
// det = -d_A n (n = e1_B e2_C - e1_C e2_B) is a sum of terms bounded by
// E (|o_B - v0_B| + |o_C - v0_C| + |t*| (|d_B| + |d_C|)) / |n| = E L / |n|
// (E the largest in-plane edge component, t* = (c - o_A) / d_A the exact
// crossing), each computed with at most 6 roundings, and det carries
// (2 kappa + 1) u (kappa <= 32, axis_plane); so the computed u and v differ
// from the exact barycentrics of the crossing by at most
// gamma_8 E L / |n| + gamma_(2 kappa + 6) each.  An accepted (u, v) lies in
// the triangle (u + v <= 1 up to one rounding), hence the exact crossing lies
// within 2 E (gamma_8 E L / |n| + gamma_(2 kappa + 6)) + 2^-23 E of the
// triangle's bounding box in B and C.  The kernel computes the crossing as
// t_f = (c - o_A) * (1 / d_A) (3 roundings of t*) and d_B = o_B + t_f d_B -
// mid_B, whose own error is below gamma_8 S + 2^-22 |mid_B| with
// S = |o_B| + |o_C| + |t_f| (|d_B| + |d_C|) >= L - V, V = |v0_B| + |v0_C|.
// Hence the test  |d_B| <= half_B + Ka S + Kb  (and the same in C) with
//     Ka = (2 gamma_8 E^2 / n_min + gamma_8) * 1.05
//     Kb = (2 gamma_8 E^2 / n_min * V + 2 E gamma_70 + 2^-23 E + 2^-22 |mid|) * 1.05
// never rejects an accepted ray (the factor 1.05 covers the roundings of the
// filter's own products).  Per pair: (mid_B, half_B + Kb, mid_C, half_C + Kb),
// (Ka, c, 0, 0).  A padding record (zero edges) never hits and is left out.
void plane_filters(ScanList &L) {
    const uint32_t npairs = (uint32_t)L.plane_c.size();
    L.plane_f.assign(8 * (size_t)npairs, 0.0f);
    const double u = std::ldexp(1.0, -24);
    auto gam = [&](double k) { return k * u / (1.0 - k * u); };
    auto up = [](double x) {  // the float >= x
        float f = (float)x;
        return (double)f < x ? std::nextafter(f, INFINITY) : f;
    };
    for (uint32_t g = 0; g < npairs; ++g) {
        const int A = g < L.plane_end[0] ? 0 : g < L.plane_end[1] ? 1 : 2, B = (A + 1) % 3, C = (A + 2) % 3;
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        double E = 0.0, nmin = INFINITY, V = 0.0;
        for (int k = 0; k < 2; ++k) {
            const float *r = &L.prims[12 * (size_t)(2 * g + k)];
            const float *v0 = r, *e1 = r + 4, *e2 = r + 8;
            const double n = std::fabs((double)e1[B] * e2[C] - (double)e1[C] * e2[B]);
            if (n == 0.0) continue;  // padding record
            for (int a : {B, C}) {
                for (double x : {(double)v0[a], (double)v0[a] + e1[a], (double)v0[a] + e2[a]}) {
                    lo[a] = std::min(lo[a], x);
                    hi[a] = std::max(hi[a], x);
                }
                E = std::max({E, std::fabs((double)e1[a]), std::fabs((double)e2[a])});
            }
            nmin = std::min(nmin, n);
            V = std::max(V, std::fabs((double)v0[B]) + std::fabs((double)v0[C]));
        }
        float *f = &L.plane_f[8 * (size_t)g];
        if (!(nmin < INFINITY)) {  // two padding records: an empty rectangle no ray passes
            f[0] = f[2] = 0.0f;
            f[1] = f[3] = -1.0f;
            f[5] = L.plane_c[g];
            continue;
        }
        const double K1 = 2.0 * gam(8) * E * E / nmin;
        const double Ka = (K1 + gam(8)) * 1.05;
        for (int k = 0; k < 2; ++k) {
            const int a = k ? C : B;
            const float mid = (float)(0.5 * (lo[a] + hi[a]));
            const double half = std::max(hi[a] - mid, mid - lo[a]);
            const double Kb = (K1 * V + 2.0 * E * gam(70) + std::ldexp(E, -23) + std::ldexp(std::fabs(mid), -22)) * 1.05;
            f[2 * k] = mid;
            f[2 * k + 1] = (float)up(up(half) + Kb);
        }
        f[4] = (float)up(Ka);
        f[5] = L.plane_c[g];
    }
}
bool axis_plane(const float *r, int a) {
    const float *e1 = r + 4, *e2 = r + 8;
    if (e1[a] != 0.0f || e2[a] != 0.0f) return false;
    const int b = (a + 1) % 3, c = (a + 2) % 3;
    for (int k : {b, c}) {  // products of normal range: nonzero components in [2^-60, 2^60]
        for (float x : {e1[k], e2[k]})
            if (x != 0.0f && !(std::fabs(x) >= 0x1p-60f && std::fabs(x) <= 0x1p60f)) return false;
    }
    // det and t's numerator are (ray component) x (P - Q) with P, Q the two
    // products below: kappa = (|P| + |Q|) / |P - Q| bounds their rounding
    const double P = (double)e1[b] * e2[c], Q = (double)e1[c] * e2[b];
    const double diff = std::fabs(P - Q);
    return diff > 0.0 && (std::fabs(P) + std::fabs(Q)) <= 32.0 * diff;
}
ScanList build_scan_list(const DeviceBvh &bvh, uint32_t n) {
    ScanList L;
    auto rec = [&](uint32_t i) { return &bvh.prims[12 * (size_t)i]; };
    auto sphere = [&](uint32_t i) {
        uint32_t f;
        std::memcpy(&f, rec(i) + 7, 4);
        return f != 0u;
    };
    auto add = [&](uint32_t i) {
        const float *r = rec(i);
        L.prims.insert(L.prims.end(), r, r + 12);
        std::memcpy(&L.prims[L.prims.size() - 1], &i, 4);  // e2.w = leaf-order position
    };
    auto add_null = [&] {
        float null_prim[12] = {0};  // zero edges: det = 0, never hit
        const uint32_t none = 0xFFFFFFFFu;
        std::memcpy(&null_prim[3], &none, 4);
        L.prims.insert(L.prims.end(), null_prim, null_prim + 12);
    };
    std::vector<int> axis(n, -1);
    for (uint32_t i = 0; i < n; ++i)
        if (!sphere(i))
            for (int a = 0; a < 3 && axis[i] < 0; ++a)
                if (axis_plane(rec(i), a)) axis[i] = a;
    for (int a = 0; a < 3; ++a) {
        // this axis's planes in order of first appearance (leaf order)
        std::vector<float> planes;
        for (uint32_t i = 0; i < n; ++i)
            if (axis[i] == a && std::find(planes.begin(), planes.end(), rec(i)[a]) == planes.end())
                planes.push_back(rec(i)[a]);
        for (float c : planes) {
            uint32_t in_pair = 0;
            for (uint32_t i = 0; i < n; ++i)
                if (axis[i] == a && rec(i)[a] == c) {
                    add(i);
                    if (++in_pair == 2) {
                        L.plane_c.push_back(c);
                        in_pair = 0;
                    }
                }
            if (in_pair) {
                add_null();
                L.plane_c.push_back(c);
            }
        }
        L.plane_end[a] = (uint32_t)L.plane_c.size();
    }
    L.tris = 2 * (uint32_t)L.plane_c.size();
    uint32_t rest = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (!sphere(i) && axis[i] < 0) add(i), ++rest;
    L.real = L.tris + rest;
    for (; rest % kScanGroup; ++rest) add_null();
    L.tris += rest;
    for (uint32_t i = 0; i < n; ++i)
        if (sphere(i)) add(i);
    plane_filters(L);
    if (const char *e = std::getenv("NORI_PLANE_CULL"); e && e[0] == '0') {  // A/B: no plane pairs
        ScanList F;
        for (uint32_t i = 0; i < n; ++i)
            if (!sphere(i)) {
                const float *r = rec(i);
                F.prims.insert(F.prims.end(), r, r + 12);
                std::memcpy(&F.prims[F.prims.size() - 1], &i, 4);
                ++F.tris;
            }
        F.real = F.tris;
        for (; F.tris % kScanGroup; ++F.tris) {
            float null_prim[12] = {0};
            const uint32_t none = 0xFFFFFFFFu;
            std::memcpy(&null_prim[3], &none, 4);
            F.prims.insert(F.prims.end(), null_prim, null_prim + 12);
        }
        for (uint32_t i = 0; i < n; ++i)
            if (sphere(i)) {
                const float *r = rec(i);
                F.prims.insert(F.prims.end(), r, r + 12);
                std::memcpy(&F.prims[F.prims.size() - 1], &i, 4);
            }
        return F;
    }
    if (debug_log())
        std::fprintf(stderr, "[nori] scan list: %zu axis-plane pairs (x %u, y %u, z %u), %u other triangle records\n",
                     L.plane_c.size(), L.plane_end[0], L.plane_end[1] - L.plane_end[0],
                     L.plane_end[2] - L.plane_end[1], rest);
    return L;
}

// The path kernels' lite variants (FULL = false) serve scenes made of the
// basic plugins only: constant-albedo diffuse, mirror and dielectric BSDFs,
// area lights, the perspective camera, no normal maps.  NORI_BASIC=0 forces
// the full variants (A/B).
bool basic_scene(const nori_scene_desc &d) {
    if (const char *e = std::getenv("NORI_BASIC"); e && e[0] == '0') return false;
    for (uint32_t i = 0; i < d.num_bsdfs; ++i) {
        const nori_bsdf_desc &b = d.bsdfs[i];
        if (b.type != NORI_BSDF_DIFFUSE && b.type != NORI_BSDF_MIRROR && b.type != NORI_BSDF_DIELECTRIC) return false;
        if (b.type == NORI_BSDF_DIFFUSE && b.albedo_texture != NORI_TEXTURE_CONSTANT) return false;
    }
    for (uint32_t i = 0; i < d.num_emitters; ++i)
        if (d.emitters[i].type != NORI_EMITTER_AREA) return false;
    for (uint32_t i = 0; i < d.num_shapes; ++i)
        if (d.shapes[i].normal_map >= 0) return false;
    return d.camera.camera_type == NORI_CAMERA_PERSPECTIVE;
}

void upload_scene(nori_gpu_ctx &c, const nori_scene_desc &d) {
    float rmin[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float rmax[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    auto expand = [&](float x, float y, float z) {
        float p[3] = {x, y, z};
        for (int k = 0; k < 3; ++k) {
            rmin[k] = std::fmin(rmin[k], p[k]);
            rmax[k] = std::fmax(rmax[k], p[k]);
        }
    };
    // image textures and normal maps: 8-bit RGB -> one RGBX word per texel, so
    // a lookup is one 4-byte load; DevBsdf/DevShape hold pointers into it
    std::vector<size_t> img_off(d.num_images);
    {
        std::vector<uint32_t> tex;
        for (uint32_t i = 0; i < d.num_images; ++i) {
            const nori_image_desc &im = d.images[i];
            if (!im.rgb || im.width <= 0 || im.height <= 0 || (im.wrap != NORI_WRAP_REPEAT && im.wrap != NORI_WRAP_CLAMP))
                throw NoriException(NORI_ERR_INVALID, "bad image description");
            img_off[i] = tex.size();
            const size_t n = (size_t)im.width * im.height;
            for (size_t t = 0; t < n; ++t)
                tex.push_back((uint32_t)im.rgb[3 * t] | ((uint32_t)im.rgb[3 * t + 1] << 8) | ((uint32_t)im.rgb[3 * t + 2] << 16));
        }
        if (tex.empty()) tex.assign(1, 0u);
        c.tex.upload(tex);
    }
    auto image_ptr = [&](int32_t i) -> const uint32_t * {
        if (i < 0) return nullptr;
        if ((uint32_t)i >= d.num_images) throw NoriException(NORI_ERR_INVALID, "image index out of range");
        return c.tex.as<uint32_t>() + img_off[i];
    };
    std::vector<DevShape> shapes(d.num_shapes);
    std::vector<uint32_t> prim_shape, tri_vidx;
    std::vector<float> cdf;
    uint32_t off = 0;
    for (uint32_t s = 0; s < d.num_shapes; ++s) {
        const nori_shape_desc &sd = d.shapes[s];
        DevShape &ds = shapes[s];
        std::memset(&ds, 0, sizeof(ds));
        ds.nmap = image_ptr(sd.normal_map);
        if (ds.nmap) {
            ds.nm_w = d.images[sd.normal_map].width;
            ds.nm_h = d.images[sd.normal_map].height;
            ds.nm_wrap = d.images[sd.normal_map].wrap;
        }
        ds.type = sd.type;
        ds.bsdf = sd.bsdf;
        ds.emitter = sd.emitter;
        ds.has_normals = sd.has_normals;
        ds.has_uvs = sd.has_uvs && d.uvs ? 1u : 0u;
        ds.prim_offset = off;
        for (int k = 0; k < 3; ++k) ds.center[k] = sd.center[k];
        ds.radius = sd.radius;
        if (sd.bsdf < 0 || (uint32_t)sd.bsdf >= d.num_bsdfs) throw NoriException(NORI_ERR_INVALID, "shape without a valid bsdf");
        if (sd.type == NORI_SHAPE_SPHERE) {
            ds.prim_count = 1;
            float inv = 1.f / sd.radius;  // sphere.cpp:99-104: pow(1/r, 2) * 1/(4 pi)
            ds.area_norm = (float)((double)inv * (double)inv * (double)(0.25f * 0.31830988618379067154f));
            prim_shape.push_back(s);
            tri_vidx.insert(tri_vidx.end(), {0u, 0u, 0u});
            expand(sd.center[0] - sd.radius, sd.center[1] - sd.radius, sd.center[2] - sd.radius);
            expand(sd.center[0] + sd.radius, sd.center[1] + sd.radius, sd.center[2] + sd.radius);
        } else if (sd.type == NORI_SHAPE_MESH) {
            if ((uint64_t)sd.tri_offset + sd.tri_count > d.num_triangles || (uint64_t)sd.vtx_offset + sd.vtx_count > d.num_vertices)
                throw NoriException(NORI_ERR_INVALID, "mesh range outside the scene arrays");
            ds.prim_count = sd.tri_count;
            ds.cdf_offset = (uint32_t)cdf.size();
            // Mesh::activate area DiscretePDF (mesh.cpp:30-38, dpdf.h:58-91)
            std::vector<float> c(sd.tri_count + 1);
            c[0] = 0.0f;
            for (uint32_t t = 0; t < sd.tri_count; ++t) {
                const uint32_t *f = d.indices + 3 * (size_t)(sd.tri_offset + t);
                for (int k = 0; k < 3; ++k)
                    if (f[k] >= d.num_vertices) throw NoriException(NORI_ERR_INVALID, "vertex index out of range");
                const float *p0 = d.positions + 3 * (size_t)f[0], *p1 = d.positions + 3 * (size_t)f[1], *p2 = d.positions + 3 * (size_t)f[2];
                float e1[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]}, e2[3] = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};
                float cx = e1[1] * e2[2] - e1[2] * e2[1], cy = e1[2] * e2[0] - e1[0] * e2[2], cz = e1[0] * e2[1] - e1[1] * e2[0];
                float area = 0.5f * std::sqrt((cx * cx + cy * cy) + cz * cz);
                c[t + 1] = c[t] + area;
                prim_shape.push_back(s);
                tri_vidx.insert(tri_vidx.end(), {f[0], f[1], f[2]});
            }
            float sum = c[sd.tri_count];
            if (sum > 0) {
                float norm = 1.0f / sum;
                for (uint32_t t = 1; t <= sd.tri_count; ++t) c[t] *= norm;
                c[sd.tri_count] = 1.0f;
                ds.area_norm = norm;
            } else {
                ds.area_norm = 0.0f;
            }
            cdf.insert(cdf.end(), c.begin(), c.end());
            for (uint32_t v = 0; v < sd.vtx_count; ++v) {
                const float *p = d.positions + 3 * (size_t)(sd.vtx_offset + v);
                expand(p[0], p[1], p[2]);
            }
        } else {
            throw NoriException(NORI_ERR_INVALID, "unknown shape type");
        }
        off += ds.prim_count;
    }
    c.num_prims = off;
    mark_solitary_spheres(d, rmin, rmax, shapes);
    std::vector<DevBsdf> bsdfs(d.num_bsdfs);
    for (uint32_t i = 0; i < d.num_bsdfs; ++i) {
        const nori_bsdf_desc &b = d.bsdfs[i];
        DevBsdf &o = bsdfs[i];
        std::memset(&o, 0, sizeof(o));
        o.type = b.type;
        for (int k = 0; k < 3; ++k) o.albedo[k] = b.albedo[k], o.kd[k] = b.kd[k], o.base[k] = b.base_color[k];
        o.int_ior = b.int_ior;
        o.ext_ior = b.ext_ior;
        o.eta_ei = b.ext_ior / b.int_ior;  // the divisions of common.cpp:296 / dielectric.cpp:57-60, done once
        o.eta_ie = b.int_ior / b.ext_ior;
        o.inv_eta_ei = 1 / o.eta_ei;
        o.alpha = b.alpha;
        float mk = b.kd[0] < b.kd[1] ? b.kd[1] : b.kd[0];
        mk = mk < b.kd[2] ? b.kd[2] : mk;
        o.ks = 1 - mk;  // microfacet.cpp:45
        o.metallic = b.metallic;
        o.specular = b.specular;
        o.roughness = b.roughness;
        o.sheen = b.sheen;
        o.sheen_tint = b.sheen_tint;
        o.spec_tint = b.specular_tint;
        double r2 = (double)b.roughness * (double)b.roughness;  // disney.cpp:59
        o.d_alpha = (float)(r2 > 1e-3 ? r2 : 1e-3);
        o.tex = b.albedo_texture;
        for (int k = 0; k < 3; ++k) o.tex_v2[k] = b.tex_value2[k];
        for (int k = 0; k < 2; ++k) o.tex_delta[k] = b.tex_delta[k], o.tex_scale[k] = b.tex_scale[k];
        if (b.albedo_texture == NORI_TEXTURE_IMAGE) {
            o.img = image_ptr(b.albedo_image);
            if (!o.img) throw NoriException(NORI_ERR_INVALID, "ImageTexture albedo without an image");
            o.img_w = d.images[b.albedo_image].width;
            o.img_h = d.images[b.albedo_image].height;
            o.img_wrap = d.images[b.albedo_image].wrap;
        } else if (b.albedo_texture != NORI_TEXTURE_CONSTANT && b.albedo_texture != NORI_TEXTURE_CHECKERBOARD) {
            throw NoriException(NORI_ERR_INVALID, "unknown albedo texture");
        }
        if (b.type < NORI_BSDF_DIFFUSE || b.type > NORI_BSDF_DISNEY) throw NoriException(NORI_ERR_INVALID, "unknown bsdf type");
    }
    std::vector<DevEmitter> emitters(d.num_emitters);
    std::vector<float> env;  // envmap tables of every envmap emitter
    for (uint32_t i = 0; i < d.num_emitters; ++i) {
        const nori_emitter_desc &e = d.emitters[i];
        if (e.type != NORI_EMITTER_AREA && e.type != NORI_EMITTER_ENVMAP && e.type != NORI_EMITTER_POINT &&
            e.type != NORI_EMITTER_SPOT)
            throw NoriException(NORI_ERR_UNSUPPORTED, "unknown emitter type");
        const bool free_standing = e.type == NORI_EMITTER_POINT || e.type == NORI_EMITTER_SPOT;
        if (!free_standing && (e.shape < 0 || (uint32_t)e.shape >= d.num_shapes))
            throw NoriException(NORI_ERR_INVALID, "emitter without a shape");
        std::memset(&emitters[i], 0, sizeof(DevEmitter));
        emitters[i].type = e.type;
        emitters[i].shape = free_standing ? -1 : e.shape;
        for (int k = 0; k < 3; ++k) {
            emitters[i].radiance[k] = e.radiance[k];
            emitters[i].position[k] = e.position[k];
            emitters[i].power[k] = e.power[k];
            emitters[i].direction[k] = e.direction[k];
        }
        emitters[i].cos_fs = e.cos_falloff_start;
        emitters[i].cos_tw = e.cos_total_width;
        if (e.type == NORI_EMITTER_ENVMAP) build_envmap(e, emitters[i], env);
    }
    if (d.integrator < NORI_INTEGRATOR_PATH_MATS || d.integrator > NORI_INTEGRATOR_PHOTONMAPPER)
        throw NoriException(NORI_ERR_UNSUPPORTED, "unknown integrator");
    if (d.num_emitters == 0 && d.integrator != NORI_INTEGRATOR_NORMALS && d.integrator != NORI_INTEGRATOR_AV)
        throw NoriException(NORI_ERR_INVALID, "the scene has no emitter");
    if (d.integrator == NORI_INTEGRATOR_PHOTONMAPPER) {
        if (d.photon_count == 0 || !(d.photon_radius > 0.0f) || !std::isfinite(d.photon_radius))
            throw NoriException(NORI_ERR_INVALID, "photonmapper: photon_count and photon_radius must be positive");
        for (uint32_t i = 0; i < d.num_emitters; ++i)  // Emitter::samplePhoton (emitter.h) throws for the others
            if (d.emitters[i].type != NORI_EMITTER_AREA)
                throw NoriException(NORI_ERR_UNSUPPORTED, "photonmapper: photons from area lights only");
    }
    if (d.camera.camera_type < NORI_CAMERA_PERSPECTIVE || d.camera.camera_type > NORI_CAMERA_ADVANCED)
        throw NoriException(NORI_ERR_UNSUPPORTED, "unknown camera type");
    // the reference leaves Scene::m_medium uninitialised without a <medium>
    // (scene.h:141): rejected here, as in the oracle
    if (d.integrator == NORI_INTEGRATOR_VOLUMETRIC && !d.medium.present)
        throw NoriException(NORI_ERR_INVALID, "the volumetric integrator needs a <medium>");

    // Traversal strategy: scenes of at most kScanMaxPrims primitives are
    // intersected by a wave-uniform scan (scalar loads, no divergence), larger
    // ones by per-lane BVH traversal.  NORI_TRAVERSAL=bvh|scan overrides.
    const char *mode = std::getenv("NORI_TRAVERSAL");
    bool scan = off <= kScanMaxPrims;
    if (mode && std::string(mode) == "bvh") scan = false;
    if (mode && std::string(mode) == "scan") scan = true;
    DeviceBvh bvh;
    build_device_bvh(d, rmin, rmax, bvh);
    c.bvh_depth = bvh.depth;
    c.bvh_nodes = bvh.num_nodes;
    // traversal stack: at most 3 entries per level of the 4-wide tree; the
    // first `stack` live in LDS, up to kTraceSpill more in private memory
    // (an 8-wide tree, 256-B nodes with a 19-comparator child order, was
    // measured 15 % slower on C3 in round 5: DESIGN_LOG.md)
    const uint32_t need = 3 * bvh.depth + 1;
    // (LDS budget 16 words: measured best on the 22.7k and 524k triangle
    // scenes -- occupancy beats a deeper LDS part; 32 only when the spill
    // area could not cover the rest)
    if (need <= (uint32_t)stack_lds_entries(8)) c.stack = 8;
    else if (need <= (uint32_t)stack_lds_entries(16) + kTraceSpill) c.stack = 16;
    else c.stack = 32;
    if (const char *e = std::getenv("NORI_BVH_STACK")) {  // tuning: 8, 16 or 32
        const int v = std::atoi(e);
        if (v == 8 || v == 16 || v == 32) c.stack = v;
    }
    if (need > (uint32_t)stack_lds_entries(c.stack) + kTraceSpill) throw NoriException(NORI_ERR_UNSUPPORTED, "BVH too deep for the traversal stack");
    if (scan) c.stack = 0;
    ScanList scan_list;
    if (scan) scan_list = build_scan_list(bvh, off);
    const std::vector<float> &prim_list = scan ? scan_list.prims : bvh.prims;

    std::vector<float> pos(4 * (size_t)d.num_vertices), nrm(4 * (size_t)d.num_vertices);
    for (uint32_t v = 0; v < d.num_vertices; ++v) {
        for (int k = 0; k < 3; ++k) {
            pos[4 * (size_t)v + k] = d.positions[3 * (size_t)v + k];
            nrm[4 * (size_t)v + k] = d.normals ? d.normals[3 * (size_t)v + k] : 0.0f;
        }
        // texture coordinates ride in the w lanes (u with the position, v with the normal)
        pos[4 * (size_t)v + 3] = d.uvs ? d.uvs[2 * (size_t)v] : 0.0f;
        nrm[4 * (size_t)v + 3] = d.uvs ? d.uvs[2 * (size_t)v + 1] : 0.0f;
    }
    if (pos.empty()) pos.assign(4, 0.0f), nrm.assign(4, 0.0f);
    if (cdf.empty()) cdf.assign(1, 0.0f);
    c.nodes.upload(bvh.nodes);
    c.prims.upload(prim_list);
    if (!scan_list.plane_c.empty()) c.plane_c.upload(scan_list.plane_c);
    if (!scan_list.plane_f.empty()) c.plane_f.upload(scan_list.plane_f);
    c.tri_vidx.upload(tri_vidx);
    c.pos.upload(pos);
    c.nrm.upload(nrm);
    c.prim_shape.upload(prim_shape);
    c.shapes.upload(shapes);
    c.bsdfs.upload(bsdfs);
    c.emitters.upload(emitters);
    c.cdf.upload(cdf);
    if (env.empty()) env.assign(4, 0.0f);
    c.env.upload(env);
    c.scene_bytes = c.nodes.bytes + c.prims.bytes;
    // small-scene blob (staged into LDS by the tail finisher)
    std::vector<char> blob;
    uint32_t offs[10] = {0};
    auto put = [&](int k, const void *p, size_t n) {
        while (blob.size() % 16) blob.push_back(0);
        offs[k] = (uint32_t)blob.size();
        const char *b = static_cast<const char *>(p);
        blob.insert(blob.end(), b, b + n);
    };
    put(0, prim_list.data(), prim_list.size() * 4);
    put(1, tri_vidx.data(), tri_vidx.size() * 4);
    put(2, pos.data(), pos.size() * 4);
    put(3, nrm.data(), nrm.size() * 4);
    put(4, prim_shape.data(), prim_shape.size() * 4);
    put(5, shapes.data(), shapes.size() * sizeof(DevShape));
    put(6, bsdfs.data(), bsdfs.size() * sizeof(DevBsdf));
    put(7, emitters.data(), emitters.size() * sizeof(DevEmitter));
    put(8, cdf.data(), cdf.size() * 4);
    put(9, bvh.nodes.data(), bvh.nodes.size() * 4);
    while (blob.size() % 16) blob.push_back(0);
    const bool use_blob = c.stack == 0 && blob.size() <= kBlobMaxBytes;
    if (use_blob) c.blob.upload(blob);

    DevScene &S = c.S;
    S.nodes = c.nodes.as<float4>();
    S.prims = c.prims.as<float4>();
    S.tri_vidx = c.tri_vidx.as<uint32_t>();
    S.pos = c.pos.as<float4>();
    S.nrm = c.nrm.as<float4>();
    S.prim_shape = c.prim_shape.as<uint32_t>();
    S.shapes = c.shapes.as<DevShape>();
    S.bsdfs = c.bsdfs.as<DevBsdf>();
    S.emitters = c.emitters.as<DevEmitter>();
    S.cdf = c.cdf.as<float>();
    S.env = c.env.as<float>();
    S.num_emitters = d.num_emitters;
    S.num_nodes = bvh.num_nodes;
    S.num_prims = (uint32_t)(prim_list.size() / 12);
    S.num_scan_tris = scan_list.tris;
    S.num_scan_real = scan_list.real;
    S.plane_c = scan_list.plane_c.empty() ? nullptr : c.plane_c.as<float>();
    S.plane_f = scan_list.plane_f.empty() ? nullptr : c.plane_f.as<float4>();
    for (int a = 0; a < 3; ++a) S.plane_end[a] = scan_list.plane_end[a];
    {
        const char *e = std::getenv("NORI_CAMERA_CULL");  // A/B and verification: 0 = no in-plane filter
        S.camera_cull = !(e && e[0] == '0');
        const char *t = std::getenv("NORI_TRACE_CULL");  // trace API: 0, 1 (default) or 2 (needs plane pairs)
        S.trace_cull = t ? std::atoi(t) : 1;
        if (S.trace_cull < 0 || S.trace_cull > 2 || (S.trace_cull == 2 && !S.plane_f)) S.trace_cull = 1;
    }
    if (scan && scan_list.prims.size() / 12 <= 2 * kScanMaxPrims) {  // the scan kernels compiled for this scene's scan list (rtc.hip); else the generic ones
        ScanRtcScene sc{scan_list.prims.data(), (uint32_t)(scan_list.prims.size() / 12), scan_list.plane_c.data(),
                        scan_list.plane_f.data(), (uint32_t)scan_list.plane_c.size(),
                        {scan_list.plane_end[0], scan_list.plane_end[1], scan_list.plane_end[2]}, scan_list.tris,
                        scan_list.real};
        std::string why;
        if (!scan_rtc_build(sc, c.device, S.trace_cull, c.rtc, why) && debug_log())
            std::fprintf(stderr, "[nori] generic scan kernels: %s\n", why.c_str());
    }
    for (int k = 0; k < 3; ++k) S.root_min[k] = rmin[k], S.root_max[k] = rmax[k];
    S.blob = use_blob ? c.blob.as<float4>() : nullptr;
    S.blob_bytes = use_blob ? (uint32_t)blob.size() : 0u;
    S.off_prims = offs[0];
    S.off_vidx = offs[1];
    S.off_pos = offs[2];
    S.off_nrm = offs[3];
    S.off_pshape = offs[4];
    S.off_shapes = offs[5];
    S.off_bsdfs = offs[6];
    S.off_emitters = offs[7];
    S.off_cdf = offs[8];
    S.off_nodes = offs[9];
    const nori_camera_desc &cam = d.camera;
    c.cam = cam;
    if (cam.width <= 0 || cam.height <= 0) throw NoriException(NORI_ERR_INVALID, "bad output size");
    S.W = cam.width;
    S.H = cam.height;
    S.invW = 1.0f / (float)cam.width;
    S.invH = 1.0f / (float)cam.height;
    std::memcpy(S.s2c, cam.sample_to_camera, sizeof(S.s2c));
    std::memcpy(S.c2w, cam.camera_to_world, sizeof(S.c2w));
    {  // perspective.cpp:104: Eigen's (c2w * (0,0,0,1)).hnormalized(), column order
        const float *c = S.c2w;
        const float w = ((c[12] * 0.0f + c[13] * 0.0f) + c[14] * 0.0f) + c[15];
        S.cam_o[0] = (((c[0] * 0.0f + c[1] * 0.0f) + c[2] * 0.0f) + c[3]) / w;
        S.cam_o[1] = (((c[4] * 0.0f + c[5] * 0.0f) + c[6] * 0.0f) + c[7]) / w;
        S.cam_o[2] = (((c[8] * 0.0f + c[9] * 0.0f) + c[10] * 0.0f) + c[11]) / w;
    }
    S.near_clip = cam.near_clip;
    S.far_clip = cam.far_clip;
    S.cam_type = cam.camera_type;
    S.lens_radius = cam.lens_radius;
    S.focal = cam.focal_distance;
    S.distortion[0] = cam.distortion[0];
    S.distortion[1] = cam.distortion[1];
    for (int k = 0; k < 3; ++k) S.chromatic[k] = cam.camera_type == NORI_CAMERA_ADVANCED ? cam.chromatic[k] : 0.0f;
    S.chroma = S.chromatic[0] != 0.0f || S.chromatic[1] != 0.0f || S.chromatic[2] != 0.0f;
    S.basic = basic_scene(d) ? 1 : 0;
    {
        // shadow rays traced inside k_shade (scan-mode scenes): on by default
        // for the basic-plugin kernels (C2 +3-7 %, its 64-spp share +3 %), off
        // for the full ones (C4 -5.7 %, C5 -4.3 %: the full k_shade holds 90-96
        // VGPRs, and the queue's shadow kernel is the scene-specialised one).
        // NORI_NEE_INLINE=0 / 1 forces it off / on for scan-mode scenes whose
        // shade kernel carries it (the basic ones; kernels.h kNeeFull).
        const char *n = std::getenv("NORI_NEE_INLINE");
        S.nee_inline = c.stack == 0 && (n ? n[0] == '1' : S.basic != 0) && (S.basic != 0 || kNeeFull);
    }
    {
        // one launch for an iteration's extension and shadow queues: on for
        // the BVH walks (C3 +10 %) and the basic scan kernels that keep the
        // queue; the full-plugin scan scenes run faster with two launches
        // (C4 3942 -> 3957, C5 4217 -> 4288 Msamples/s, 3 interleaved reps,
        // tools/gpu_fuse_ab.sh).  NORI_TRACE_FUSE=0 / 1 forces it.
        const char *f = std::getenv("NORI_TRACE_FUSE");
        c.fuse_trace = f ? f[0] != '0' : !(c.stack == 0 && S.basic == 0);
    }
    S.W_max = cam.width > cam.height ? cam.width : cam.height;
    S.av_length = d.av_length;
    filter_table(cam, S.filter);
    S.filter_radius = cam.filter_radius;
    S.lookup = NORI_FILTER_RESOLUTION / cam.filter_radius;
    S.border = film_border(cam);
    if (S.border > 4) throw NoriException(NORI_ERR_UNSUPPORTED, "filter radius above 4.5 pixels");
    S.jit_lk = jit_code_lookup(S.filter_radius, S.lookup);
    S.integrator = d.integrator;
    {  // deviation D10 (kernels.hip skip_nee); NORI_DISCRETE_NEE=1 keeps the full NEE everywhere
        bool env = false;
        for (uint32_t i = 0; i < d.num_emitters; ++i) env = env || d.emitters[i].type == NORI_EMITTER_ENVMAP;
        const char *e = std::getenv("NORI_DISCRETE_NEE");
        S.skip_discrete_nee = !env && !(e && e[0] == '1');
    }
    S.has_medium = d.medium.present;
    if (S.has_medium) {  // medium.cpp:10-20
        const nori_medium_desc &m = d.medium;
        for (int k = 0; k < 3; ++k) {
            S.mbox_min[k] = m.box_min[k];
            S.mbox_max[k] = m.box_max[k];
            S.sigma_t[k] = m.sigma_a[k] + m.sigma_s[k];
            S.albedo[k] = m.sigma_s[k] / S.sigma_t[k];
        }
    }
}

void ensure_pool(nori_gpu_ctx &c, uint32_t pool) {
    if (pool <= c.pool_cap) return;
    for (int b = 0; b < 2; ++b) {
        c.q[b][0].ensure(16 * (size_t)pool);
        c.q[b][1].ensure(16 * (size_t)pool);
        c.q[b][2].ensure(16 * (size_t)pool);
        c.q[b][3].ensure(16 * (size_t)pool);
        c.q[b][4].ensure(4 * (size_t)pool);
    }
    for (int k = 0; k < 3; ++k) c.sq[k].ensure(16 * (size_t)pool);
    for (int k = 0; k < 4; ++k) c.seg[k].ensure(4 * (size_t)(pool / kSeg));
    c.segstats.ensure(16 * (size_t)(pool / kSeg));
    c.tailpre.ensure(4 * (size_t)(pool / kSeg + 1));
    c.pool_cap = pool;
}

PathQueue queue_of(nori_gpu_ctx &c, int b) {
    PathQueue q;
    q.ray_o = c.q[b][0].as<float4>();
    q.ray_d = c.q[b][1].as<float4>();
    q.hit = c.q[b][2].as<float4>();
    q.thr = c.q[b][3].as<float4>();
    q.rng = c.q[b][4].as<uint32_t>();
    return q;
}

constexpr int kRing = 16;     // readback ring entries
constexpr int kLookahead = 6;    // iterations queued ahead of the termination check
constexpr int kLookaheadEnd = 2; // ... once work streams run dry

struct Timers {
    std::vector<hipEvent_t> ev;
    size_t used = 0;
    hipEvent_t get() {
        if (used == ev.size()) {
            hipEvent_t e;
            HIP_TRY(hipEventCreate(&e));
            ev.push_back(e);
        }
        return ev[used++];
    }
    ~Timers() {
        for (auto e : ev) (void)hipEventDestroy(e);
    }
};

bool debug_log() {
    const char *e = std::getenv("NORI_DEBUG");
    return e && e[0] == '1';
}
// NORI_POOL_PARTS: independent pool parts on their own streams (1..kMaxParts).
// Default 3: each part's launches wait for their own slowest walks / longest
// lanes, and three streams keep the chip busy in between (C3: 2 parts 619,
// 3 parts 651, 4 parts 499 Msamples/s -- 4 streams exceed the hardware
// queues; table scene 517 -> 555; C2 4563 -> 4658; 64-spp share 3026 ->
// 3089; C4 and C5 within 1 %).
uint32_t pool_parts(bool bvh) {
    (void)bvh;
    const uint32_t def = 3u;
    const char *e = std::getenv("NORI_POOL_PARTS");
    const long v = e ? std::atol(e) : (long)def;
    return (uint32_t)(v >= 1 && v <= kMaxParts ? v : def);
}
// Sample passes folded by one splat work-group.  Default: about one
// work-group per CU over the whole launch (passes x blocks / 256), so the
// splat leaves most of the chip to the tail finisher it overlaps with
// (cbox 512x512@512: 256 blocks x 512 passes per work-group, splat 3.0 ms and
// finisher 3.6 ms vs 4.7 / 5.2 ms at 32 passes).  NORI_SPLAT_PASSES overrides.
// The one-bounce integrators' splat has no finisher beside it: it targets
// 4096 work-groups instead.
uint32_t splat_passes(uint32_t np, size_t nblocks, uint32_t target_wgs = 256) {
    const char *e = std::getenv("NORI_SPLAT_PASSES");
    long v = e ? std::atol(e) : (long)(((uint64_t)np * nblocks + target_wgs - 1) / target_wgs);
    if (v < 1) v = 1;
    return (uint32_t)std::min<long>(v, np);
}
// Per-pixel sample statistics (render_desc.variance_out): the device buffer
// the kernels add into -- the caller's own when it is device memory, else a
// zeroed scratch buffer that var_finish adds into the host array.
float *var_begin(nori_gpu_ctx &c, const nori_gpu_render_desc &rd) {
    if (!rd.variance_out) return nullptr;
    if (rd.output_on_device) return rd.variance_out;
    const size_t n = 8 * (size_t)c.S.W * (size_t)c.S.H;
    c.varbuf.ensure(n * sizeof(float));
    HIP_TRY(hipMemsetAsync(c.varbuf.p, 0, n * sizeof(float), c.stream));
    return c.varbuf.as<float>();
}
void var_finish(nori_gpu_ctx &c, const nori_gpu_render_desc &rd, bool cancelled) {
    if (!rd.variance_out || rd.output_on_device || cancelled) return;
    const size_t n = 8 * (size_t)c.S.W * (size_t)c.S.H;
    std::vector<float> h(n);
    HIP_TRY(hipMemcpy(h.data(), c.varbuf.p, n * sizeof(float), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; ++i) rd.variance_out[i] += h[i];
}

// PhotonMapper::preprocess (photonmapper.cpp:41-117): photons are traced on
// the device in emission order batches (k_photons count pass) until the
// stored count reaches photonCount, then the emitted photons that contribute
// are traced again writing their photons (store pass), and the host stores
// them as the reference's PhotonData and builds the hash grid.
void photon_preprocess(nori_gpu_ctx &c, const nori_scene_desc &d) {
    const uint64_t N = d.photon_count;
    const uint32_t batch = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(N, 1u << 20), 1u << 24);
    DevBuf cnt;
    cnt.ensure(4 * (size_t)batch);
    std::vector<uint32_t> hc(batch);
    std::vector<uint64_t> pre;  // photons stored before each emitted photon
    uint64_t total = 0, e0 = 0;
    while (total < N) {
        if (e0 >= 64 * N + batch)  // the reference would loop forever
            throw NoriException(NORI_ERR_INVALID, "photonmapper: photons do not reach a diffuse surface");
        HIP_TRY(launch_photons(c.S, e0, batch, cnt.as<uint32_t>(), nullptr, 0, nullptr, c.stack, c.stream));
        HIP_TRY(hipMemcpyAsync(hc.data(), cnt.p, 4 * (size_t)batch, hipMemcpyDeviceToHost, c.stream));
        HIP_TRY(hipStreamSynchronize(c.stream));
        for (uint32_t i = 0; i < batch && total < N; ++i) {
            pre.push_back(total);
            total += hc[i];
        }
        e0 += batch;
    }
    DevBuf dpre, out;
    dpre.upload(pre);
    out.ensure(48 * (size_t)N);
    // all-ones (NaN) first: a slot the store pass leaves unwritten keeps a NaN
    // in its zero pad word and is caught below instead of entering the map
    HIP_TRY(hipMemsetAsync(out.p, 0xFF, 48 * (size_t)N, c.stream));
    HIP_TRY(launch_photons(c.S, 0, (uint32_t)pre.size(), nullptr, dpre.as<uint64_t>(), N, out.as<float4>(), c.stack,
                           c.stream));
    HIP_TRY(hipStreamSynchronize(c.stream));
    std::vector<float> raw(12 * (size_t)N), ph, tab;
    HIP_TRY(hipMemcpy(raw.data(), out.p, 48 * (size_t)N, hipMemcpyDeviceToHost));
    // the store pass must reproduce the count pass photon for photon
    // (position, 0, direction, 0, power, 0 per slot)
    for (size_t i = 0; i < (size_t)N; ++i)
        if (!(raw[12 * i + 3] == 0.0f && raw[12 * i + 7] == 0.0f && raw[12 * i + 11] == 0.0f))
            throw NoriException(NORI_ERR_INVALID, "photonmapper: the store pass left photon slot " + std::to_string(i) +
                                                      " unwritten (count and store passes disagree)");
    std::vector<uint32_t> start, rgbe;
    uint32_t mask = 0;
    build_photon_map(raw, (uint32_t)N, d.photon_radius, ph, rgbe, tab, start, mask);
    c.ph.upload(ph);
    c.ph_rgbe.upload(rgbe);
    c.ph_tab.upload(tab);
    c.ph_start.upload(start);
    c.S.ph_rgbe = c.ph_rgbe.as<uint32_t>();
    c.S.ph_tab = c.ph_tab.as<float>();
    const float r = d.photon_radius;
    c.S.ph = c.ph.as<float4>();
    c.S.ph_start = c.ph_start.as<uint32_t>();
    c.S.ph_mask = mask;
    c.S.ph_inv_cell = 1.0f / r;
    c.S.ph_r2 = r * r;                                 // kdtree.h:266
    c.S.ph_norm = (r * r) * (float)d.photon_count;     // photonmapper.cpp:177
}

// normals / av / direct*: no path pool -- per chunk of passes, k_direct runs
// every sample start to end and writes its record, then k_splat filters them.
int render_one_bounce(nori_gpu_ctx &c, const nori_gpu_render_desc &rd, const std::vector<uint32_t> &pixels,
                      const std::vector<int4> &blocks, float *rgbw_out, nori_gpu_stats *stats,
                      std::chrono::steady_clock::time_point t0) {
    const DevScene &S = c.S;
    const int W = S.W, H = S.H, B = S.border;
    const uint32_t M = (uint32_t)pixels.size(), passes = rd.pass_count;
    const size_t rec_budget = (size_t)4 << 30;
    uint32_t chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(passes, rec_budget / (16 * (size_t)M)));
    // work ids (record indices) < 2^29: the path queue keeps a chromatic
    // sample's colour channel in bits 29-30 of the same word (kWorkMask)
    chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(chunk, ((uint64_t)1 << kChanShift) / M));
    c.rec.ensure(16 * (size_t)chunk * M);
    c.counters.ensure(sizeof(Counters));
    const size_t film_elems = 4 * (size_t)(W + 2 * B) * (H + 2 * B);
    float *film = nullptr;
    if (rd.output_on_device) {
        film = rgbw_out;
    } else {
        c.film.ensure(film_elems * sizeof(float));
        film = c.film.as<float>();
        HIP_TRY(hipMemsetAsync(film, 0, film_elems * sizeof(float), c.stream));
    }
    Counters *C = c.counters.as<Counters>();
    HIP_TRY(hipMemsetAsync(C, 0, sizeof(Counters), c.stream));
    c.cancel = 0;
    c.progress = 0.0f;
    Timers tm;
    const bool timing = rd.timing != 0;
    double kms[2] = {0, 0};
    std::vector<std::array<hipEvent_t, 3>> spans;
    uint64_t done = 0;
    bool cancelled = false;
    float *var = var_begin(c, rd);
    for (uint32_t p0 = 0; p0 < passes; p0 += chunk) {
        if (c.cancel.load()) {
            cancelled = true;
            break;
        }
        const uint32_t np = std::min(chunk, passes - p0);
        WorkDesc wd{(uint64_t)np * M, M, rd.pass_begin + p0, c.pixels.as<uint32_t>(), rd.seed, 0, nullptr, 1, 0, var};
        SplatDesc sd{M, np, rd.pass_begin + p0, std::max<uint32_t>(1, splat_passes(np, blocks.size(), 4096)), c.blocks.as<int4>(),
                     rd.seed, var};
        std::array<hipEvent_t, 3> ev{};
        if (timing) {
            for (auto &e : ev) e = tm.get();
            HIP_TRY(hipEventRecord(ev[0], c.stream));
        }
        HIP_TRY(launch_direct(S, wd, c.rec.as<float4>(), C, c.stack, c.stream));
        if (timing) HIP_TRY(hipEventRecord(ev[1], c.stream));
        HIP_TRY(launch_splat(S, c.rec.as<float4>(), sd, (uint32_t)blocks.size(), film, C, c.stream));
        if (timing) {
            HIP_TRY(hipEventRecord(ev[2], c.stream));
            spans.push_back(ev);
        }
        HIP_TRY(hipStreamSynchronize(c.stream));
        done += wd.total;
        c.progress = (float)((double)(p0 + np) / passes);
    }
    Counters hc;
    HIP_TRY(hipMemcpyAsync(&hc, C, sizeof(Counters), hipMemcpyDeviceToHost, c.stream));
    HIP_TRY(hipStreamSynchronize(c.stream));
    for (const auto &e : spans) {
        float a = 0, b = 0;
        HIP_TRY(hipEventElapsedTime(&a, e[0], e[1]));
        HIP_TRY(hipEventElapsedTime(&b, e[1], e[2]));
        kms[0] += a;
        kms[1] += b;
    }
    if (!rd.output_on_device && !cancelled) {
        std::vector<float> hf(film_elems);
        HIP_TRY(hipMemcpy(hf.data(), film, film_elems * sizeof(float), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < film_elems; ++i) rgbw_out[i] += hf[i];
    }
    var_finish(c, rd, cancelled);
    c.progress = 1.0f;
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->samples = done;
        stats->invalid_samples = hc.invalid;
        stats->rays_closest = hc.direct_rays[0];
        stats->rays_shadow = hc.direct_rays[1];
        stats->iterations = 0;
        stats->scene_bytes = c.scene_bytes;
        stats->bvh_nodes = c.bvh_nodes;
        stats->bvh_depth = c.bvh_depth;
        stats->stream_parts = 1;
        stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        stats->ms_shade = kms[0];  // k_direct: the whole integrator
        stats->ms_splat = kms[1];
        stats->scan_rtc = c.rtc.extend ? 1u : 0u;  // (held for the trace API; k_direct scans generically)
        stats->scan_rtc_cached = c.rtc.cached ? 1u : 0u;
        stats->ms_scan_rtc = c.rtc.compile_ms;
    }
    if (cancelled) return fail(NORI_ERR_CANCELLED, "rendering was cancelled");
    return NORI_OK;
}

// The render's blocks in BlockGenerator order (block.cpp:140-188) with the
// block_subset applied, and the block-major pixel list (camera samples of one
// block are adjacent work ids); cached on the context with their device
// copies, so a render of the same selection neither rebuilds nor uploads them.
static void work_lists(nori_gpu_ctx &c, const nori_gpu_render_desc &rd) {
    const int W = c.S.W, H = c.S.H;
    const int nbx = (int)std::ceil(W / (float)NORI_BLOCK_SIZE), nby = (int)std::ceil(H / (float)NORI_BLOCK_SIZE);
    std::vector<uint32_t> order = spiral_blocks(W, H);
    if (rd.num_blocks) {
        std::vector<char> want((size_t)nbx * nby, 0);
        for (uint32_t i = 0; i < rd.num_blocks; ++i) {
            if (rd.block_ids[i] >= (uint32_t)(nbx * nby)) throw NoriException(NORI_ERR_INVALID, "block id out of range");
            want[rd.block_ids[i]] = 1;
        }
        std::vector<uint32_t> sel;
        for (uint32_t b : order)
            if (want[b]) sel.push_back(b);
        order.swap(sel);
    }
    if (c.work_valid && order == c.work_order) return;
    c.work_valid = false;
    c.hpixels.clear();
    c.hblocks.clear();
    for (uint32_t b : order) {
        int bx = (int)(b % (uint32_t)nbx), by = (int)(b / (uint32_t)nbx);
        int ox = bx * NORI_BLOCK_SIZE, oy = by * NORI_BLOCK_SIZE;
        int bw = std::min(NORI_BLOCK_SIZE, W - ox), bh = std::min(NORI_BLOCK_SIZE, H - oy);
        c.hblocks.push_back(make_int4(ox, oy, bw | (bh << 16), (int)c.hpixels.size()));
        for (int y = 0; y < bh; ++y)
            for (int x = 0; x < bw; ++x) c.hpixels.push_back((uint32_t)((oy + y) * W + (ox + x)));
    }
    c.pixels.upload(c.hpixels);
    c.blocks.upload(c.hblocks);
    c.work_order.swap(order);
    c.work_valid = true;
}

int render(nori_gpu_ctx &c, const nori_gpu_render_desc &rd, float *rgbw_out, nori_gpu_stats *stats) {
    auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipSetDevice(c.device));
    const DevScene &S = c.S;
    const int W = S.W, H = S.H, B = S.border;
    work_lists(c, rd);
    const std::vector<uint32_t> &pixels = c.hpixels;
    const std::vector<int4> &blocks = c.hblocks;
    const uint32_t M = (uint32_t)pixels.size();
    const uint32_t passes = rd.pass_count ? rd.pass_count : 0;
    if (passes == 0 || M == 0) throw NoriException(NORI_ERR_INVALID, "nothing to render (pass_count or blocks empty)");
    const bool one_bounce = S.integrator >= NORI_INTEGRATOR_NORMALS;
    // default pool: about 1/16 of the render's samples in flight, between
    // 1M and 4M paths (~0.9 GB of queues at 4M).  Large pools hide the shade
    // kernel's memory latency (4M measured best among 256K..4M on cbox at 512
    // spp); small renders -- the per-GPU share of a strong-scaled frame --
    // spend less time draining a smaller pool (round 2, two parts, cbox 64
    // spp: 4M 2190, 2M 2320, 1M 2400 Msamples/s; 512 spp: 4M and 2M within
    // 1 %).  With three parts (round 3) the 64-spp share peaks at 1.25-1.5M
    // (512K 2560, 1M 3030-3160, 1.25M 3320, 1.5M 3275-3296, 2M 3192, 3M 2952)
    // and the 128-spp share at 2M (3989 against 3875 at 2.5M, 3773 at 3M).
    // Since k_shade traces the shadow rays itself (round 6, nee_inline) the
    // 64-spp share peaks at 1M again (4875 against 4702 at 1.5M, 4734 at
    // 1.25M, 4555 at 768K; 3 reps), so the floor is 1M.  The BVH walks
    // (C3) want about 1/8 in flight: 4M 846-851 against 807-812 at 2M
    // (3M 796-798, 6M 796-798, 8M 839-846; 3 interleaved reps).
    if (one_bounce) return render_one_bounce(c, rd, pixels, blocks, rgbw_out, stats, t0);
    if (M > kWorkMask) throw NoriException(NORI_ERR_INVALID, "frame too large: more than 2^29 pixels per pass");
    uint32_t pool = rd.path_pool;
    if (!pool) {  // NORI_PATH_POOL: default pool size override (tuning)
        const char *e = std::getenv("NORI_PATH_POOL");
        if (e && std::atol(e) > 0) {
            pool = (uint32_t)std::min<long>(std::atol(e), 1L << 26);
        } else {
            const uint64_t want = (uint64_t)passes * M / (c.stack ? 8 : 16);
            pool = 1u << 20;
            while (pool < (1u << 22) && pool < want) pool <<= 1;
        }
    }
    pool = std::max<uint32_t>(kSeg, (pool + kSeg - 1) / kSeg * kSeg);
    ensure_pool(c, pool);
    // sample-record budget: chunks of passes, each < 2^31 records
    const size_t rec_budget = (size_t)6 << 30;
    uint32_t chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(passes, rec_budget / (16 * (size_t)M)));
    // work ids (record indices) < 2^29: the path queue keeps a chromatic
    // sample's colour channel in bits 29-30 of the same word (kWorkMask)
    chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(chunk, ((uint64_t)1 << kChanShift) / M));
    c.rec.ensure(16 * (size_t)chunk * M);
    c.counters.ensure(sizeof(Counters));
    const size_t film_elems = 4 * (size_t)(W + 2 * B) * (H + 2 * B);
    float *film = nullptr;
    if (rd.output_on_device) {
        film = rgbw_out;
    } else {
        c.film.ensure(film_elems * sizeof(float));
        film = c.film.as<float>();
        HIP_TRY(hipMemsetAsync(film, 0, film_elems * sizeof(float), c.stream));
    }
    if (!c.pinned) {
        // host-mapped, coherent: the shade kernel stores the completion flag here
        HIP_TRY(hipHostMalloc((void **)&c.pinned, 256, hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(hipHostGetDevicePointer((void **)&c.pinned_dev, c.pinned, 0));
        for (auto &r : c.ring) {
            r.resize(kRing);
            for (auto &e : r) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
    }
    Counters *C = c.counters.as<Counters>();
    ShadowQueue sq{c.sq[0].as<float4>(), c.sq[1].as<float4>(), c.sq[2].as<float4>()};
    PathQueue Q[2] = {queue_of(c, 0), queue_of(c, 1)};
    c.cancel = 0;
    c.progress = 0.0f;
    const uint64_t total_all = (uint64_t)passes * M;
    uint64_t done_before = 0, rays_c = 0, rays_s = 0, invalid = 0, iters = 0;
    Timers tm;
    struct Span {
        hipEvent_t a, b;
        int kind;
    };
    std::vector<Span> spans;
    const bool timing = rd.timing != 0;
    auto timed_on = [&](hipStream_t st, int kind, auto &&launch) {
        if (!timing) {
            HIP_TRY(launch());
            return;
        }
        Span s{tm.get(), tm.get(), kind};
        HIP_TRY(hipEventRecord(s.a, st));
        HIP_TRY(launch());
        HIP_TRY(hipEventRecord(s.b, st));
        spans.push_back(s);
    };
    auto timed = [&](int kind, auto &&launch) { timed_on(c.stream, kind, launch); };
    bool cancelled = false;
    const uint32_t parts = std::max<uint32_t>(1, std::min<uint32_t>(pool_parts(c.stack != 0), pool / kSeg));
    const uint32_t G = pool / kSeg;
    SegState seg{{c.seg[0].as<uint32_t>(), c.seg[1].as<uint32_t>()}, c.seg[2].as<uint32_t>(), c.seg[3].as<uint32_t>(),
                 c.segstats.as<uint4>()};
    std::vector<uint4> hstats(G);
    uint64_t finish_rays = 0, samples_started = 0;
    float *var = var_begin(c, rd);
    for (uint32_t p0 = 0; p0 < passes && !cancelled; p0 += chunk) {
        uint32_t np = std::min(chunk, passes - p0);
        WorkDesc wd{(uint64_t)np * M, M, rd.pass_begin + p0, c.pixels.as<uint32_t>(), rd.seed, G, c.pinned_dev, 1, 0,
                    var};
        wd.rot = stream_rotation(wd.total, M, G);
        __atomic_store_n(&c.pinned[0], 0u, __ATOMIC_RELEASE);
        __atomic_store_n(&c.pinned[1], 0u, __ATOMIC_RELEASE);
        // segments whose stream is empty from the start count as exhausted
        uint32_t empty = 0;
        for (uint32_t b = 0; b < G; ++b) empty += stream_work(wd, b, 0) >= wd.total;
        HIP_TRY(launch_reset(C, empty, seg, G, c.stream));
        int last_out = 0;
        // The pool is split into `parts` independent parts (segments never
        // interact), each driven on its own stream: the memory-bound shade
        // launch of one part overlaps the VALU-bound traversal of another.
        std::vector<uint32_t> Gp(parts), base(parts);
        for (uint32_t h = 0; h < parts; ++h) {
            base[h] = (uint32_t)((uint64_t)G * h / parts);
            Gp[h] = (uint32_t)((uint64_t)G * (h + 1) / parts) - base[h];
        }
        auto q_view = [&](const PathQueue &q, uint32_t b0) {
            const size_t e = (size_t)b0 * kSeg;
            return PathQueue{q.ray_o + e, q.ray_d + e, q.hit + e, q.thr + e, q.rng + e};
        };
        std::vector<std::array<PathQueue, 2>> Qh(parts);
        std::vector<ShadowQueue> sqh(parts);
        std::vector<SegState> segh(parts);
        std::vector<WorkDesc> wdh(parts);
        for (uint32_t h = 0; h < parts; ++h) {
            Qh[h][0] = q_view(Q[0], base[h]);
            Qh[h][1] = q_view(Q[1], base[h]);
            const size_t e = (size_t)base[h] * kSeg;
            sqh[h] = ShadowQueue{sq.ray_o + e, sq.ray_d + e, sq.payload + e};
            segh[h] = SegState{{seg.cnt[0] + base[h], seg.cnt[1] + base[h]}, seg.shcnt + base[h],
                               seg.cursor + base[h], seg.stats + base[h]};
            wdh[h] = wd;
            wdh[h].b0 = base[h];
        }
        HIP_TRY(hipEventRecord(c.fork, c.stream));  // the part streams start after the resets above
        for (uint32_t h = 1; h < parts; ++h) HIP_TRY(hipStreamWaitEvent(c.parts[h], c.fork, 0));
        uint64_t lag = kLookahead;
        // NORI_DEBUG: host time spent enqueuing vs waiting on the ring events
        // (a wait that returns at once means the device ran dry of work)
        const bool dbg = debug_log();
        double t_enq = 0.0, t_wait = 0.0;
        uint32_t idle_waits = 0;
        auto now_us = [] {
            return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
        };
        for (uint64_t it = 0;; ++it) {
            const double te0 = dbg ? now_us() : 0.0;
            int in = (int)(it & 1), out = in ^ 1;
            last_out = out;
            for (uint32_t h = 0; h < parts; ++h) {
                hipStream_t st = h ? c.parts[h] : c.stream;
                const SegState &sg = segh[h];
                timed_on(st, 2, [&] {
                    return launch_shade(S, Qh[h][in], Qh[h][out], sqh[h], sg, in, wdh[h], c.rec.as<float4>(), C,
                                        Gp[h], st);
                });
                hipError_t both_err = hipSuccess;
                if (S.nee_inline) {  // the shadow rays were traced by k_shade itself
                    timed_on(st, 0, [&] { return launch_extend(S, Qh[h][out], sg.cnt[out], Gp[h], c.stack, st, &c.rtc); });
                    continue;
                }
                if (!timing && c.fuse_trace &&
                    launch_trace_both(S, Qh[h][out], sg.cnt[out], sqh[h], sg.shcnt, c.rec.as<float4>(), Gp[h], c.stack,
                                      &c.rtc, st, both_err)) {
                    HIP_TRY(both_err);  // (the timed renders keep two launches: one event span per kernel)
                    continue;
                }
                timed_on(st, 0, [&] { return launch_extend(S, Qh[h][out], sg.cnt[out], Gp[h], c.stack, st, &c.rtc); });
                timed_on(st, 1, [&] {
                    return launch_shadow(S, sqh[h], sg.shcnt, c.rec.as<float4>(), Gp[h], c.stack, st, &c.rtc);
                });
            }
            ++iters;
            // an event per iteration; the host waits on the one from `lag`
            // iterations back
            const uint64_t ev = it;
            for (uint32_t h = 0; h < parts; ++h)
                HIP_TRY(hipEventRecord(c.ring[h][ev % kRing], h ? c.parts[h] : c.stream));
            const double te1 = dbg ? now_us() : 0.0;
            t_enq += te1 - te0;
            if (ev >= lag) {
                for (uint32_t h = 0; h < parts; ++h) HIP_TRY(hipEventSynchronize(c.ring[h][(ev - lag) % kRing]));
                if (dbg) {
                    const double w = now_us() - te1;
                    t_wait += w;
                    idle_waits += w < 5.0 ? 1u : 0u;
                }
                uint32_t exhausted = __atomic_load_n(&c.pinned[1], __ATOMIC_ACQUIRE);
                // the streams are running dry: queue fewer iterations ahead,
                // so that few drain iterations (full-grid launches over a
                // thinning pool) are already queued when the last one does
                if (exhausted) lag = std::min<uint64_t>(lag, kLookaheadEnd);
                c.progress = (float)std::min(1.0, (double)done_before / (double)total_all +
                                                      (double)np / passes * exhausted / G);
                // every work id has been handed out: finish the remaining paths in one launch
                if (__atomic_load_n(&c.pinned[0], __ATOMIC_ACQUIRE)) break;
                if (c.cancel.load()) {
                    cancelled = true;
                    break;
                }
            }
        }
        for (uint32_t h = 1; h < parts; ++h) {  // join: the tail below runs on the whole pool
            HIP_TRY(hipEventRecord(c.joins[h], c.parts[h]));
            HIP_TRY(hipStreamWaitEvent(c.stream, c.joins[h], 0));
        }
        if (cancelled) break;
        // The samples still in flight are marked pending; the film splat of all
        // the others runs on the side stream while the finisher completes the
        // pending ones and splats each itself.
        hipStream_t splat_st = c.side;
        HIP_TRY(launch_mark(Q[last_out], seg, last_out, c.rec.as<float4>(), G, c.stream));
        HIP_TRY(launch_tail_prefix(seg, last_out, G, c.tailpre.as<uint32_t>(), c.stream));
        HIP_TRY(hipEventRecord(c.fork, c.stream));
        HIP_TRY(hipStreamWaitEvent(c.side, c.fork, 0));
        SplatDesc sd{M, np, rd.pass_begin + p0, std::max<uint32_t>(1, splat_passes(np, blocks.size())),
                     c.blocks.as<int4>(), rd.seed, var};
        auto splat = [&] {
            timed_on(splat_st, 3, [&] { return launch_splat(S, c.rec.as<float4>(), sd, (uint32_t)blocks.size(), film, C, splat_st); });
        };
        auto finish = [&] {
            timed(4, [&] {
                return launch_finish(S, Q[last_out], seg, last_out, c.rec.as<float4>(), wd, film, C, G, c.stack,
                                     c.tailpre.as<uint32_t>(), c.stream);
            });
        };
        // both wait for the same fork; the finisher's waves are enqueued first
        // (c.finish_first) so that they are resident before the splat fills the CUs
        if (c.finish_first) {
            finish();
            splat();
        } else {
            splat();
            finish();
        }
        HIP_TRY(hipEventRecord(c.join, c.side));
        HIP_TRY(hipStreamWaitEvent(c.stream, c.join, 0));
        // read-back through pinned staging: both copies queue behind the
        // finisher without a host round trip each (pageable copies stage twice)
        const size_t rb = sizeof(Counters) + 16 * (size_t)G;
        if (c.readback_bytes < rb) {
            if (c.readback) HIP_TRY(hipHostFree(c.readback));
            c.readback = nullptr;
            c.readback_bytes = 0;
            HIP_TRY(hipHostMalloc((void **)&c.readback, rb, hipHostMallocDefault));
            c.readback_bytes = rb;
        }
        HIP_TRY(hipMemcpyAsync(c.readback, C, sizeof(Counters), hipMemcpyDeviceToHost, c.stream));
        HIP_TRY(hipMemcpyAsync(c.readback + sizeof(Counters), seg.stats, 16 * (size_t)G, hipMemcpyDeviceToHost, c.stream));
        HIP_TRY(hipStreamSynchronize(c.stream));
        Counters hc;
        std::memcpy(&hc, c.readback, sizeof(Counters));
        std::memcpy(hstats.data(), c.readback + sizeof(Counters), 16 * (size_t)G);
        for (const uint4 &st : hstats) {
            rays_c += st.x;
            rays_s += st.y;
            samples_started += st.z;
            finish_rays += st.w;
        }
        invalid += hc.invalid;
        if (debug_log())
        {
            std::fprintf(stderr, "[nori] chunk %u: %lu iterations, finisher %u paths, longest %u rays\n", p0,
                         (unsigned long)iters, hc.finish_paths, hc.finish_max_rays);
            std::fprintf(stderr, "[nori] host loop: %.0f us enqueuing, %.0f us waiting; %u of the waits returned at once\n",
                         t_enq, t_wait, idle_waits);
            if (hc.prof[6])  // NORI_PROF_SHADE builds
                std::fprintf(stderr, "[nori] shade clocks per wave: loads %.0f shade %.0f compact %.0f store %.0f regen %.0f drain %.0f (%llu waves)\n",
                             (double)hc.prof[0] / hc.prof[6], (double)hc.prof[1] / hc.prof[6],
                             (double)hc.prof[2] / hc.prof[6], (double)hc.prof[3] / hc.prof[6],
                             (double)hc.prof[4] / hc.prof[6], (double)hc.prof[5] / hc.prof[6], hc.prof[6]);
            else if (hc.prof[4])  // NORI_PROF_FINISH builds
                std::fprintf(stderr, "[nori] finisher clocks per wave-iteration: shade %.0f shadow %.0f splat %.0f extend %.0f (%llu); "
                             "longest wave %.3f ms over %llu iterations\n",
                             (double)hc.prof[0] / hc.prof[4], (double)hc.prof[1] / hc.prof[4],
                             (double)hc.prof[2] / hc.prof[4], (double)hc.prof[3] / hc.prof[4], hc.prof[4],
                             (double)(hc.prof[5] >> 20) * 1e-5, hc.prof[5] & 0xFFFFFull);
            if (hc.prof[14])  // NORI_PROF_GLASS builds
                std::fprintf(stderr, "[nori] lone-lane glass chains: %llu chord bounces, %.0f ns each\n", hc.prof[14],
                             10.0 * hc.prof[13] / hc.prof[14]);
            if (hc.prof[12])
                std::fprintf(stderr, "[nori] finisher late iterations (lone lanes): shade %.0f shadow %.0f splat %.0f extend %.0f ns (%llu)\n",
                             10.0 * hc.prof[8] / hc.prof[12], 10.0 * hc.prof[9] / hc.prof[12],
                             10.0 * hc.prof[10] / hc.prof[12], 10.0 * hc.prof[11] / hc.prof[12], hc.prof[12]);
        }
        done_before += wd.total;
    }
    if (samples_started != done_before && !cancelled)
        throw NoriException(NORI_ERR_INVALID, "internal: started " + std::to_string(samples_started) + " of " +
                                                  std::to_string(done_before) + " samples");
    double kms[5] = {0, 0, 0, 0, 0};
    if (timing) {
        HIP_TRY(hipStreamSynchronize(c.stream));
        for (const Span &s : spans) {
            float ms = 0.0f;
            HIP_TRY(hipEventElapsedTime(&ms, s.a, s.b));
            kms[s.kind] += ms;
        }
    }
    if (!rd.output_on_device && !cancelled) {
        std::vector<float> hf(film_elems);
        HIP_TRY(hipMemcpy(hf.data(), film, film_elems * sizeof(float), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < film_elems; ++i) rgbw_out[i] += hf[i];
    }
    var_finish(c, rd, cancelled);
    HIP_TRY(hipStreamSynchronize(c.stream));
    HIP_TRY(hipStreamSynchronize(c.side));
    for (int h = 1; h < kMaxParts; ++h) HIP_TRY(hipStreamSynchronize(c.parts[h]));
    c.progress = 1.0f;
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->samples = done_before;
        stats->invalid_samples = invalid;
        stats->rays_closest = rays_c;
        stats->rays_shadow = rays_s;
        stats->iterations = iters;
        stats->scene_bytes = c.scene_bytes;
        stats->bvh_nodes = c.bvh_nodes;
        stats->bvh_depth = c.bvh_depth;
        stats->stream_parts = parts;
        stats->path_pool = pool;
        stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        stats->ms_extend = kms[0];
        stats->ms_shadow = kms[1];
        stats->ms_shade = kms[2];
        stats->ms_splat = kms[3];
        stats->ms_finish = kms[4];
        stats->rays_finish = finish_rays;
        stats->scan_rtc = c.rtc.extend ? 1u : 0u;
        stats->scan_rtc_cached = c.rtc.cached ? 1u : 0u;
        stats->ms_scan_rtc = c.rtc.compile_ms;
        stats->nee_inline = S.nee_inline ? 1u : 0u;
    }
    if (cancelled) return fail(NORI_ERR_CANCELLED, "rendering was cancelled");
    return NORI_OK;
}

}  // namespace

// ------------------------------------------------------------------ C ABI
namespace {

// This rank's share of a whole-frame render (nori_gpu_shard_desc).  The pass
// count defaults to the scene's sampleCount (0 -> 1) in both entry points, and
// a block list is checked (range) and de-duplicated in both modes, so the
// share always fits the caller's block_buf (capacity = the frame's blocks).
nori_gpu_render_desc shard_of(int W, int H, uint32_t spp, const nori_gpu_render_desc &whole, int mode, int nranks,
                              int rank, std::vector<uint32_t> &blocks) {
    if (nranks < 1 || rank < 0 || rank >= nranks) throw NoriException(NORI_ERR_INVALID, "shard: rank out of range");
    if (mode != NORI_SHARD_PASSES && mode != NORI_SHARD_BLOCKS) throw NoriException(NORI_ERR_INVALID, "shard: unknown mode");
    nori_gpu_render_desc out = whole;
    const uint32_t P = whole.pass_count ? whole.pass_count : std::max<uint32_t>(spp, 1u);
    const uint32_t nb = (uint32_t)(((W + NORI_BLOCK_SIZE - 1) / NORI_BLOCK_SIZE) * ((H + NORI_BLOCK_SIZE - 1) / NORI_BLOCK_SIZE));
    std::vector<char> want(nb, whole.num_blocks ? 0 : 1);
    for (uint32_t i = 0; i < whole.num_blocks; ++i) {
        if (whole.block_ids[i] >= nb) throw NoriException(NORI_ERR_INVALID, "block id out of range");
        want[whole.block_ids[i]] = 1;
    }
    blocks.clear();
    if (mode == NORI_SHARD_PASSES) {
        const uint64_t a = (uint64_t)P * rank / nranks, b = (uint64_t)P * (rank + 1) / nranks;
        out.pass_begin = whole.pass_begin + (uint32_t)a;
        out.pass_count = (uint32_t)(b - a);
        if (whole.num_blocks)  // the restricted frame, each block once, in the caller's order
            for (uint32_t i = 0; i < whole.num_blocks; ++i)
                if (want[whole.block_ids[i]]) {
                    blocks.push_back(whole.block_ids[i]);
                    want[whole.block_ids[i]] = 0;
                }
    } else {
        uint32_t k = 0;  // round-robin over the spiral order (block.cpp:140-188)
        for (uint32_t b : spiral_blocks(W, H))
            if (want[b] && (k++ % (uint32_t)nranks) == (uint32_t)rank) blocks.push_back(b);
        out.pass_count = blocks.empty() ? 0 : P;  // no block of this rank: an empty share
    }
    out.num_blocks = (uint32_t)blocks.size();
    out.block_ids = blocks.empty() ? nullptr : blocks.data();
    return out;
}

// Samples of a share (pass count x pixels of its blocks, or of the image).
double share_samples(int W, int H, const nori_gpu_render_desc &s) {
    if (!s.num_blocks) return (double)s.pass_count * W * H;
    const int nx = (W + NORI_BLOCK_SIZE - 1) / NORI_BLOCK_SIZE;
    double px = 0;
    for (uint32_t i = 0; i < s.num_blocks; ++i) {
        const int bx = (int)(s.block_ids[i] % (uint32_t)nx), by = (int)(s.block_ids[i] / (uint32_t)nx);
        px += (double)std::min(NORI_BLOCK_SIZE, W - bx * NORI_BLOCK_SIZE) * std::min(NORI_BLOCK_SIZE, H - by * NORI_BLOCK_SIZE);
    }
    return px * s.pass_count;
}

// Watchdog of the collectives of a sharded render: how long a rank waits in
// the status exchange or the film sum for its peers before it aborts the
// communicator.  Only a peer that cannot join at all (its device faulted,
// its process died) is waited for: every other failure reaches the peers
// through the status exchange.  NORI_COMM_TIMEOUT_S fixes the bound;
// otherwise, for a rank that rendered its share (status NORI_OK), it scales
// with the frame: max(30 s, 20 x this rank's own render time x largest share
// / own share), since every peer renders a share of about the same size with
// the same code.  A rank whose own render failed or was cancelled, or that
// has no share, has no render time that says how long its peers need: it
// waits up to 600 s.
double comm_timeout_s(int status, double own_s, double own_samples, double max_samples) {
    if (const char *e = std::getenv("NORI_COMM_TIMEOUT_S")) {
        const double v = std::atof(e);
        if (v > 0.0) return v;
    }
    if (status != NORI_OK || !(own_samples > 0.0)) return 600.0;
    return std::max(30.0, 20.0 * own_s * std::max(1.0, max_samples / own_samples));
}

// Status word of the exchange: severity << 16 | rank, reduced by max over the
// ranks, so the worst outcome wins and names its rank (the highest of equals).
// Severity 0 rendered, 1 cancelled, 2 failed.
int comm_status_word(int rc, int rank) {
    const int sev = rc == NORI_OK ? 0 : (rc == NORI_ERR_CANCELLED ? 1 : 2);
    return (sev << 16) | (rank & 0xFFFF);
}

}  // namespace

extern "C" {

const char *nori_gpu_last_error(void) { return g_last_error.c_str(); }

// denoiser/denoiser.py (NL-means over a rendered image and its per-pixel
// variance) on device `device`: host buffers in, host buffer out.
int nori_denoise(int device, const float *rgb, const float *variance, int width, int height, int radius, int patch,
                 float k, int mode, float *out) {
    return guarded([&] {
        if (!rgb || !variance || !out || width <= 0 || height <= 0 || radius < 0 || radius > 8 || patch < 1 ||
            patch > 5 || mode < 0 || mode > 1 || !(k > 0.0f))
            return fail(NORI_ERR_INVALID, "nori_denoise: invalid arguments");
        HIP_TRY(hipSetDevice(device));
        {  // the tile + halo staging must fit one work-group's LDS
            int lds_max = 0;
            HIP_TRY(hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, device));
            const size_t need = denoise_lds_bytes(radius, patch - 1);
            if (need > (size_t)lds_max)
                return fail(NORI_ERR_INVALID, "nori_denoise: radius " + std::to_string(radius) + " / patch " +
                                                  std::to_string(patch) + " need " + std::to_string(need) +
                                                  " bytes of LDS per work-group, the device has " +
                                                  std::to_string(lds_max));
        }
        const size_t n = (size_t)width * (size_t)height;
        DevBuf di, dv, dout;
        di.ensure(12 * n);
        dv.ensure(4 * n);
        dout.ensure(12 * n);
        HIP_TRY(hipMemcpy(di.p, rgb, 12 * n, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(dv.p, variance, 4 * n, hipMemcpyHostToDevice));
        HIP_TRY(launch_denoise((const float *)di.p, (const float *)dv.p, width, height, radius, patch - 1, k, mode,
                               (float *)dout.p, nullptr));
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(hipMemcpy(out, dout.p, 12 * n, hipMemcpyDeviceToHost));
        return (int)NORI_OK;
    });
}
int nori_gpu_abi_version(void) { return NORI_GPU_ABI_VERSION; }

int nori_read_image(const char *path, int *width, int *height, uint8_t *rgb) {
    return guarded([&] {
        if (!path || !width || !height) return fail(NORI_ERR_INVALID, "null argument");
        int w = 0, h = 0;
        std::vector<uint8_t> img;
        decode_image_rgb8(path, w, h, img);
        *width = w;
        *height = h;
        if (rgb) std::memcpy(rgb, img.data(), img.size());
        return NORI_OK;
    });
}

int nori_scene_load_xml(const char *path, int width, int height, int spp, nori_scene **out) {
    return guarded([&] {
        if (!path || !out) return fail(NORI_ERR_INVALID, "null argument");
        auto *s = new nori_scene;
        s->hs.reset(load_scene_xml(path, width, height, spp));
        *out = s;
        return NORI_OK;
    });
}
const nori_scene_desc *nori_scene_get_desc(const nori_scene *s) { return s ? &s->hs->desc : nullptr; }

int nori_scene_bvh_info(const nori_scene_desc *d, nori_bvh_info *out) {
    return guarded([&] {
        if (!d || !out) return fail(NORI_ERR_INVALID, "null argument");
        if (d->abi_version != NORI_GPU_ABI_VERSION) return fail(NORI_ERR_INVALID, "ABI version mismatch");
        float rmin[3], rmax[3];
        scene_root_box(*d, rmin, rmax);
        DeviceBvh bvh;
        build_device_bvh(*d, rmin, rmax, bvh);
        std::memset(out, 0, sizeof(*out));
        out->ref_nodes = bvh.ref_nodes;
        out->device_nodes = bvh.num_nodes;
        out->depth = bvh.depth;
        out->num_prims = (uint32_t)(bvh.prims.size() / 12);
        out->sah_cost = bvh.sah_cost;
        uint64_t h = 1469598103934665603ull;
        for (size_t i = 0; i < bvh.prims.size(); i += 12) {
            uint32_t id;
            std::memcpy(&id, &bvh.prims[i + 3], 4);
            for (int k = 0; k < 4; ++k) h = (h ^ ((id >> (8 * k)) & 0xFFu)) * 1099511628211ull;
        }
        out->order_hash = h;
        return NORI_OK;
    });
}
int nori_scene_scan_rtc(const nori_scene_desc *d, const char *arch, size_t *code_bytes, double *ms) {
    return guarded([&] {
        if (!d || !arch || !code_bytes || !ms) return fail(NORI_ERR_INVALID, "null argument");
        if (d->abi_version != NORI_GPU_ABI_VERSION) return fail(NORI_ERR_INVALID, "ABI version mismatch");
        float rmin[3], rmax[3];
        scene_root_box(*d, rmin, rmax);
        DeviceBvh bvh;
        build_device_bvh(*d, rmin, rmax, bvh);
        const uint32_t n = (uint32_t)(bvh.prims.size() / 12);
        *code_bytes = 0;
        *ms = 0.0;
        if (n > kScanMaxPrims) return NORI_OK;  // a BVH scene: nothing to specialise
        const ScanList L = build_scan_list(bvh, n);
        ScanRtcScene sc{L.prims.data(), (uint32_t)(L.prims.size() / 12), L.plane_c.data(), L.plane_f.data(),
                        (uint32_t)L.plane_c.size(), {L.plane_end[0], L.plane_end[1], L.plane_end[2]}, L.tris, L.real};
        std::vector<char> code;
        bool cached = false;
        std::string why;
        if (!rtc_compile(sc, arch, 1, code, *ms, cached, why)) return fail(NORI_ERR_UNSUPPORTED, why);
        *code_bytes = code.size();
        return NORI_OK;
    });
}
int nori_scene_scan_list(const nori_scene_desc *d, nori_scan_info *info, float *records, float *plane_c,
                         float *plane_f) {
    return guarded([&] {
        if (!d || !info) return fail(NORI_ERR_INVALID, "null argument");
        if (d->abi_version != NORI_GPU_ABI_VERSION) return fail(NORI_ERR_INVALID, "ABI version mismatch");
        float rmin[3], rmax[3];
        scene_root_box(*d, rmin, rmax);
        DeviceBvh bvh;
        build_device_bvh(*d, rmin, rmax, bvh);
        const uint32_t n = (uint32_t)(bvh.prims.size() / 12);
        std::memset(info, 0, sizeof(*info));
        if (n > kScanMaxPrims) return NORI_OK;  // a BVH scene: no scan list
        const ScanList L = build_scan_list(bvh, n);
        info->records = (uint32_t)(L.prims.size() / 12);
        info->pairs = (uint32_t)L.plane_c.size();
        for (int a = 0; a < 3; ++a) info->plane_end[a] = L.plane_end[a];
        info->tris = L.tris;
        if (records) std::memcpy(records, L.prims.data(), L.prims.size() * 4);
        if (plane_c && !L.plane_c.empty()) std::memcpy(plane_c, L.plane_c.data(), L.plane_c.size() * 4);
        if (plane_f && !L.plane_f.empty()) std::memcpy(plane_f, L.plane_f.data(), L.plane_f.size() * 4);
        return NORI_OK;
    });
}
void nori_scene_free(nori_scene *s) { delete s; }

int nori_film_border(const nori_scene_desc *d) { return d ? film_border(d->camera) : NORI_ERR_INVALID; }
int nori_filter_table(const nori_scene_desc *d, float *table) {
    if (!d || !table) return fail(NORI_ERR_INVALID, "null argument");
    filter_table(d->camera, table);
    return NORI_OK;
}
int nori_film_develop(const nori_scene_desc *d, const float *rgbw, float *rgb) {
    if (!d || !rgbw || !rgb) return fail(NORI_ERR_INVALID, "null argument");
    int W = d->camera.width, H = d->camera.height, B = film_border(d->camera), FW = W + 2 * B;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const float *c = rgbw + 4 * ((size_t)(y + B) * FW + (x + B));
            float *o = rgb + 3 * ((size_t)y * W + x);
            for (int k = 0; k < 3; ++k) o[k] = c[3] != 0 ? c[k] / c[3] : 0.0f;  // color.h:113-118
        }
    return NORI_OK;
}

int nori_gpu_device_count(int *count) {
    return guarded([&] {
        if (!count) return fail(NORI_ERR_INVALID, "null argument");
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        *count = e == hipSuccess ? n : 0;
        return NORI_OK;
    });
}

int nori_gpu_create(const nori_scene_desc *d, int device, nori_gpu_ctx **out) {
    return guarded([&] {
        if (!d || !out) return fail(NORI_ERR_INVALID, "null argument");
        if (d->abi_version != NORI_GPU_ABI_VERSION) return fail(NORI_ERR_INVALID, "scene desc ABI version mismatch");
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(NORI_ERR_HIP, "no HIP device available");
        if (device < 0 || device >= n) return fail(NORI_ERR_INVALID, "device index out of range");
        HIP_TRY(hipSetDevice(device));
        std::unique_ptr<nori_gpu_ctx> c(new nori_gpu_ctx);
        c->device = device;
        c->spp = d->sample_count ? d->sample_count : 1;
        if (const char *e = std::getenv("NORI_FINISH_FIRST"); e && e[0] == '0') c->finish_first = false;
        HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
        for (int h = 1; h < kMaxParts; ++h) {
            HIP_TRY(hipStreamCreateWithFlags(&c->parts[h], hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&c->joins[h], hipEventDisableTiming));
        }
        HIP_TRY(hipEventCreateWithFlags(&c->fork, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&c->join, hipEventDisableTiming));
        upload_scene(*c, *d);
        if (d->integrator == NORI_INTEGRATOR_PHOTONMAPPER) photon_preprocess(*c, *d);
        *out = c.release();
        return NORI_OK;
    });
}

int nori_gpu_render(nori_gpu_ctx *c, const nori_gpu_render_desc *rd, float *rgbw_out, nori_gpu_stats *stats) {
    return guarded([&] {
        if (!c || !rd || !rgbw_out) return fail(NORI_ERR_INVALID, "null argument");
        if (rd->num_blocks && !rd->block_ids) return fail(NORI_ERR_INVALID, "block_ids is null");
        return render(*c, *rd, rgbw_out, stats);
    });
}

int nori_gpu_trace(nori_gpu_ctx *c, const float *rays, uint32_t n, int any_hit, nori_gpu_hit *hits) {
    return guarded([&] {
        if (!c || !rays || !hits) return fail(NORI_ERR_INVALID, "null argument");
        if (n == 0) return NORI_OK;
        HIP_TRY(hipSetDevice(c->device));
        DevBuf r, h;
        r.ensure(32 * (size_t)n);
        h.ensure(16 * (size_t)n);
        HIP_TRY(hipMemcpy(r.p, rays, 32 * (size_t)n, hipMemcpyHostToDevice));
        HIP_TRY(launch_trace(c->S, r.as<float4>(), n, any_hit, h.as<float4>(), c->stack, c->stream, &c->rtc));
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(hipMemcpy(hits, h.p, 16 * (size_t)n, hipMemcpyDeviceToHost));
        return NORI_OK;
    });
}

int nori_gpu_cancel(nori_gpu_ctx *c) {
    if (!c) return fail(NORI_ERR_INVALID, "null argument");
    c->cancel = 1;
    return NORI_OK;
}
float nori_gpu_progress(const nori_gpu_ctx *c) { return c ? c->progress.load() : 0.0f; }

int nori_gpu_comm_id(unsigned char *id) {
    return guarded([&] {
        if (!id) return fail(NORI_ERR_INVALID, "null argument");
        comm_unique_id(id);
        return (int)NORI_OK;
    });
}
int nori_gpu_comm_create(const unsigned char *id, int nranks, int rank, int device, nori_gpu_comm **out) {
    return guarded([&] {
        if (!id || !out) return fail(NORI_ERR_INVALID, "null argument");
        if (nranks < 1 || nranks > 0xFFFF || rank < 0 || rank >= nranks) return fail(NORI_ERR_INVALID, "rank out of range");
        std::unique_ptr<nori_gpu_comm> c(new nori_gpu_comm);
        // the status exchange's words, allocated here so that no allocation
        // stands between a failed share and the exchange
        HIP_TRY(hipSetDevice(device));
        HIP_TRY(hipMalloc((void **)&c->status_dev, sizeof(int)));
        HIP_TRY(hipHostMalloc((void **)&c->status_host, sizeof(int), hipHostMallocDefault));
        c->nccl = comm_create(id, nranks, rank, device);
        c->nranks = nranks;
        c->rank = rank;
        c->device = device;
        *out = c.release();
        return (int)NORI_OK;
    });
}
int nori_gpu_comm_rank(const nori_gpu_comm *c, int *nranks, int *rank) {
    if (!c || !nranks || !rank) return fail(NORI_ERR_INVALID, "null argument");
    *nranks = c->nranks;
    *rank = c->rank;
    return NORI_OK;
}
void nori_gpu_comm_destroy(nori_gpu_comm *c) { delete c; }
const char *nori_gpu_comm_library(void) { return comm_library_path(); }

int nori_gpu_shard_desc(const nori_scene_desc *d, const nori_gpu_render_desc *rd, int mode, int nranks, int rank,
                        nori_gpu_render_desc *out, uint32_t *block_buf) {
    return guarded([&] {
        if (!d || !rd || !out || (rd->num_blocks && !rd->block_ids)) return fail(NORI_ERR_INVALID, "null argument");
        std::vector<uint32_t> blocks;
        nori_gpu_render_desc s =
            shard_of(d->camera.width, d->camera.height, d->sample_count, *rd, mode, nranks, rank, blocks);
        if (!blocks.empty()) {
            if (!block_buf) return fail(NORI_ERR_INVALID, "block_buf is null");
            std::memcpy(block_buf, blocks.data(), 4 * blocks.size());
            s.block_ids = block_buf;
        } else {
            s.block_ids = nullptr;
        }
        *out = s;
        return (int)NORI_OK;
    });
}

int nori_gpu_render_sharded(nori_gpu_ctx *c, nori_gpu_comm *comm, const nori_gpu_render_desc *rd, int mode, int root,
                            float *film, nori_gpu_stats *stats) {
    return guarded([&] {
        if (!c || !comm) return fail(NORI_ERR_INVALID, "null argument");
        if (comm->aborted) return fail(NORI_ERR_HIP, "communicator was aborted by an earlier failure");
        // This rank's share.  A failure or a cancel (nori_gpu_cancel) must not
        // leave the peers blocked in the film sum: every rank joins a status
        // exchange first (max over ranks of severity << 16 | rank), and the
        // film sum runs only if every rank rendered its share.  Everything
        // fallible of the share -- argument checks, the film clear, the
        // render -- reports through the exchange.
        int rc = NORI_OK;
        std::string err;
        double own_s = 0.0, own_samples = 0.0, max_samples = 0.0;
        size_t n = 0;
        try {
            if (!rd || !film) throw NoriException(NORI_ERR_INVALID, "null argument");
            if (rd->num_blocks && !rd->block_ids) throw NoriException(NORI_ERR_INVALID, "block_ids is null");
            if (rd->variance_out)  // per-pixel statistics are not summed across ranks
                throw NoriException(NORI_ERR_INVALID, "nori_gpu_render_sharded: variance_out must be NULL");
            if (root >= comm->nranks) throw NoriException(NORI_ERR_INVALID, "root out of range");
            if (comm->device != c->device)
                throw NoriException(NORI_ERR_INVALID, "communicator and context on different devices");
            HIP_TRY(hipSetDevice(c->device));
            std::vector<uint32_t> blocks, other;
            nori_gpu_render_desc s = shard_of(c->S.W, c->S.H, c->spp, *rd, mode, comm->nranks, comm->rank, blocks);
            own_samples = share_samples(c->S.W, c->S.H, s);
            for (int r = 0; r < comm->nranks; ++r)
                max_samples = std::max(max_samples, share_samples(c->S.W, c->S.H,
                                                                  shard_of(c->S.W, c->S.H, c->spp, *rd, mode,
                                                                           comm->nranks, r, other)));
            s.output_on_device = 1;
            s.variance_out = nullptr;
            n = 4 * (size_t)(c->S.W + 2 * c->S.border) * (size_t)(c->S.H + 2 * c->S.border);
            HIP_TRY(hipMemsetAsync(film, 0, n * sizeof(float), c->stream));
            const auto t0 = std::chrono::steady_clock::now();
            if (s.pass_count) rc = render(*c, s, film, stats);
            else if (stats) std::memset(stats, 0, sizeof(*stats));
            own_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        } catch (const NoriException &e) {
            rc = e.code;
            err = e.what();
        } catch (const std::bad_alloc &) {
            rc = NORI_ERR_OOM;
            err = "out of memory";
        } catch (const std::exception &e) {
            rc = NORI_ERR_INVALID;
            err = e.what();
        }
        if (rc != NORI_OK && err.empty()) err = g_last_error;
        if (rc == NORI_ERR_HIP) {
            // A sticky error (a device fault) fails every later call on the
            // device, so this rank cannot join the exchange: abort, and the
            // peers' watchdog ends their wait.  Any other HIP error leaves
            // the stream usable and goes through the exchange.
            (void)hipGetLastError();
            if (hipSetDevice(c->device) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) {
                comm_abort(comm->nccl);
                comm->aborted = true;
                return fail(rc, err);
            }
        }
        const double timeout = comm_timeout_s(rc, own_s, own_samples, max_samples);
        const int all = comm_max_int(comm->nccl, comm->status_dev, comm->status_host,
                                     comm_status_word(rc, comm->rank), c->stream, timeout, comm->aborted);
        if (rc != NORI_OK) return fail(rc, err);
        if ((all >> 16) != 0)
            return fail((all >> 16) == 1 ? NORI_ERR_CANCELLED : NORI_ERR_INVALID,
                        "the frame is incomplete: rank " + std::to_string(all & 0xFFFF) +
                            ((all >> 16) == 1 ? " was cancelled" : " failed to render its share"));
        comm_sum(comm->nccl, film, n, root, c->stream);
        comm_wait(comm->nccl, c->stream, timeout, comm->aborted);
        return (int)NORI_OK;
    });
}
int nori_gpu_comm_status_word(int rc, int rank) { return comm_status_word(rc, rank); }
double nori_gpu_comm_timeout(int status, double own_seconds, double own_samples, double max_samples) {
    return comm_timeout_s(status, own_seconds, own_samples, max_samples);
}
void nori_gpu_destroy(nori_gpu_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    delete c;
}

}  // extern "C"
