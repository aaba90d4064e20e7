// scan.h -- the wave-uniform scan of small scenes (<= 64 primitives): the
// reference's ray-primitive tests (mesh.cpp:83-120, sphere.cpp:43-76) in
// exact fp32, the scan list's wall-pair skips, and the bodies of the scan
// trace kernels (k_extend_scan, k_shadow_scan, the trace API's scan).
//
// Compiled twice: into libnori_gpu.so (kernels.hip), reading the scan list
// from DevScene, and at context creation through hipRTC (rtc.cpp) with
// NORI_CONST_SCENE and the scene's generated const_scene.h, so that the
// records are literal operands of the tests -- no scalar loads, no waits on
// them, and the compiler folds what the records make constant.
#pragma once
#include "dev_scene.h"

namespace nori {

#define INF_F __builtin_inff()

struct TRay {
    V3 o, d, rcp;
    float mint, maxt;
};

// BoundingBox3f::rayIntersect (bbox.h:336-363) in branch-free form with the
// same result on every input, including d_i == 0 and NaN slabs.
ND bool box_test(const float4 &mn, const float4 &mx, const TRay &r, float &tnear) {
    bool ok = true;
    float nearT = -INF_F, farT = INF_F;
#define NORI_AXIS(c)                                                            \
    {                                                                           \
        float t1 = (mn.c - r.o.c) * r.rcp.c, t2 = (mx.c - r.o.c) * r.rcp.c;      \
        float lo = t1 > t2 ? t2 : t1, hi = t1 > t2 ? t1 : t2;                   \
        bool zero = r.d.c == 0.0f;                                              \
        float n2 = smax(lo, nearT), f2 = smin(hi, farT);                        \
        ok = ok && (zero ? !(r.o.c < mn.c || r.o.c > mx.c) : (n2 <= f2));       \
        nearT = zero ? nearT : n2;                                              \
        farT = zero ? farT : f2;                                                \
    }
    NORI_AXIS(x) NORI_AXIS(y) NORI_AXIS(z)
#undef NORI_AXIS
    tnear = nearT;
    return ok && r.mint <= farT && nearT <= r.maxt;
}

// 1 / det of the triangle tests, correctly rounded (== 1.0f / det, tools/rcp_check.hip).
ND float rcp_det(float x) { return rcp_rn(x); }
// Mesh::rayIntersect (mesh.cpp:83-120), edges precomputed exactly.
ND bool tri_hit(const float4 &a, const float4 &b, const float4 &c, const TRay &r, float &t, float &u, float &v) {
    V3 v0 = ld3(a), e1 = ld3(b), e2 = ld3(c);
    V3 pvec = cross(r.d, e2);
    float det = dot(e1, pvec);
    if (det > -1e-8f && det < 1e-8f) return false;
    float inv_det = rcp_rn(det);  // == 1.0f / det (tools/rcp_check.hip)
    V3 tvec = r.o - v0;
    u = dot(tvec, pvec) * inv_det;
    if (u < 0.0f || u > 1.0f) return false;
    V3 qvec = cross(tvec, e1);
    v = dot(r.d, qvec) * inv_det;
    if (v < 0.0f || u + v > 1.0f) return false;
    t = dot(e2, qvec) * inv_det;
    return t >= r.mint && t <= r.maxt;
}

// Sphere::rayIntersect (sphere.cpp:43-76).
ND bool sphere_hit(const float4 &a, const float4 &b, const TRay &r, float &t) {
    V3 oc = r.o - ld3(a);
    float rad = b.x;
    float A = dot(r.d, r.d);
    float B = 2.0f * dot(oc, r.d);
    float C = dot(oc, oc) - rad * rad;
    float disc = (B * B - 4 * A * C);
    if (!(disc > 0)) return false;
    float delta = sqrtf(B * B - 4 * A * C);
    float t1 = (-B - delta) / (2 * A), t2 = (-B + delta) / (2 * A);
    if (r.mint <= t1 && t1 <= r.maxt) { t = t1; return true; }
    if (r.mint <= t2 && t2 <= r.maxt) { t = t2; return true; }
    return false;
}

// Branch-free forms of the two tests for the wave-uniform scan: every lane
// evaluates the whole test and the acceptance predicate is the conjunction of
// the reference's early-out conditions, so the accepted (t, u, v) are the
// same values; lanes of a wave never split inside a primitive test.
ND bool tri_hit_nb(const float4 &a, const float4 &b, const float4 &c, const TRay &r, float &t, float &u, float &v) {
    V3 v0 = ld3(a), e1 = ld3(b), e2 = ld3(c);
    V3 pvec = cross(r.d, e2);
    float det = dot(e1, pvec);
    float inv_det = rcp_det(det);  // == 1.0f / det (tools/rcp_check.hip)
    V3 tvec = r.o - v0;
    u = dot(tvec, pvec) * inv_det;
    V3 qvec = cross(tvec, e1);
    v = dot(r.d, qvec) * inv_det;
    t = dot(e2, qvec) * inv_det;
    return !(det > -1e-8f && det < 1e-8f) && !(u < 0.0f || u > 1.0f) && !(v < 0.0f || u + v > 1.0f) &&
           t >= r.mint && t <= r.maxt;
}
// tri_hit_nb for a triangle whose edges both have an exactly zero
// component on axis A (the scan's axis-plane pairs): the products with those
// zeros are left out.  In cross() and dot() each of them only ever adds a
// signed zero to, or subtracts one from, a single other product, so every
// intermediate keeps its value; only the sign of an exactly zero result can
// differ, which no acceptance test sees (t = +-0 < mint; u = +-0 and v = +-0
// compare alike), so hits and t are bit-identical and u, v equal as values.
// 12 of the test's ~65 VALU instructions fewer.
template <int A>
ND bool tri_hit_plane(const float4 &a, const float4 &b, const float4 &c, const TRay &r, float &t, float &u,
                      float &v) {
    const V3 v0 = ld3(a), e1 = ld3(b), e2 = ld3(c), d = r.d;
    V3 pvec, qvec;
    float det;
    const V3 tvec = r.o - v0;
    if (A == 0) {
        pvec = V3{d.y * e2.z - d.z * e2.y, -(d.x * e2.z), d.x * e2.y};
        det = e1.y * pvec.y + e1.z * pvec.z;
        qvec = V3{tvec.y * e1.z - tvec.z * e1.y, -(tvec.x * e1.z), tvec.x * e1.y};
    } else if (A == 1) {
        pvec = V3{d.y * e2.z, d.z * e2.x - d.x * e2.z, -(d.y * e2.x)};
        det = e1.x * pvec.x + e1.z * pvec.z;
        qvec = V3{tvec.y * e1.z, tvec.z * e1.x - tvec.x * e1.z, -(tvec.y * e1.x)};
    } else {
        pvec = V3{-(d.z * e2.y), d.z * e2.x, d.x * e2.y - d.y * e2.x};
        det = e1.x * pvec.x + e1.y * pvec.y;
        qvec = V3{-(tvec.z * e1.y), tvec.z * e1.x, tvec.x * e1.y - tvec.y * e1.x};
    }
    const float inv_det = rcp_det(det);
    u = dot(tvec, pvec) * inv_det;
    v = dot(d, qvec) * inv_det;
    t = (A == 0 ? e2.y * qvec.y + e2.z * qvec.z : A == 1 ? e2.x * qvec.x + e2.z * qvec.z : e2.x * qvec.x + e2.y * qvec.y) *
        inv_det;
    return !(det > -1e-8f && det < 1e-8f) && !(u < 0.0f || u > 1.0f) && !(v < 0.0f || u + v > 1.0f) &&
           t >= r.mint && t <= r.maxt;
}
template <bool FAST = false>
ND bool sphere_hit_nb(const float4 &a, const float4 &b, const TRay &r, float &t) {
    V3 oc = r.o - ld3(a);
    float rad = b.x;
    float A = dot(r.d, r.d);
    float B = 2.0f * dot(oc, r.d);
    float C = dot(oc, oc) - rad * rad;
    float disc = (B * B - 4 * A * C);
    float delta = fsqrt<FAST>(B * B - 4 * A * C);
    float t1 = (-B - delta) / (2 * A), t2 = (-B + delta) / (2 * A);
    bool h1 = r.mint <= t1 && t1 <= r.maxt, h2 = r.mint <= t2 && t2 <= r.maxt;
    t = h1 ? t1 : t2;
    return (disc > 0) && (h1 || h2);
}

// sphere_hit_nb with its square root and its two divisions in short
// correctly rounded forms, so the same t bits for every ray: sqrt_rn's core
// (v_sqrt_f32 and one Tuckerman test each way, exhaustively exact on
// [2^-96, 2^96), device_math.h) and Markstein's quotient x / y =
// fma(fma(-y, q0, x), r, q0), q0 = x r, r = 1/y correctly rounded (rcp_rn),
// exact for |x|, |y| in [2^-60, 2^60] (tools/div_check.c: 8.2e8 quotients,
// no mismatch).  Rays with disc > 0 outside those ranges take the IEEE
// forms; rays with disc <= 0 miss either way.
#ifndef NORI_SPHERE_FAST
#define NORI_SPHERE_FAST 1
#endif
ND bool in_range60(float x) { return fabsf(x) >= 0x1p-60f && fabsf(x) <= 0x1p60f; }
ND bool sphere_hit_fast(const float4 &a, const float4 &b, const TRay &r, float &t) {
    if (!NORI_SPHERE_FAST) return sphere_hit_nb(a, b, r, t);
    V3 oc = r.o - ld3(a);
    float rad = b.x;
    float A = dot(r.d, r.d);
    float B = 2.0f * dot(oc, r.d);
    float C = dot(oc, oc) - rad * rad;
    float disc = (B * B - 4 * A * C);
    const float y = 2 * A;
#ifdef __HIP_DEVICE_COMPILE__
    const float s0 = __builtin_amdgcn_sqrtf(disc);
    const float sd = __uint_as_float(__float_as_uint(s0) - 1u), su = __uint_as_float(__float_as_uint(s0) + 1u);
    const float rd = __builtin_fmaf(-sd, s0, disc), ru = __builtin_fmaf(-su, s0, disc);
    float delta = ru > 0.0f ? su : (rd <= 0.0f ? sd : s0);
    const float ry = rcp_rn(y);
    float x1 = -B - delta, x2 = -B + delta;
    float q1 = x1 * ry, q2 = x2 * ry;
    float t1 = __builtin_fmaf(__builtin_fmaf(-y, q1, x1), ry, q1), t2 = __builtin_fmaf(__builtin_fmaf(-y, q2, x2), ry, q2);
    const bool fast = disc >= 0x1p-96f && disc < 0x1p96f && in_range60(y) && in_range60(x1) && in_range60(x2);
    if (__builtin_expect(disc > 0 && !fast, 0)) {
        delta = sqrtf(B * B - 4 * A * C);
        t1 = (-B - delta) / (2 * A);
        t2 = (-B + delta) / (2 * A);
    }
#else
    float delta = sqrtf(B * B - 4 * A * C);
    float t1 = (-B - delta) / y, t2 = (-B + delta) / y;
#endif
    bool h1 = r.mint <= t1 && t1 <= r.maxt, h2 = r.mint <= t2 && t2 <= r.maxt;
    t = h1 ? t1 : t2;
    return (disc > 0) && (h1 || h2);
}

// Small scenes: wave-uniform scan of the primitive list.  Every lane tests
// every primitive the wave needs in the same order, so the records arrive
// through scalar loads and no lane diverges; the result is the closest hit.
// Ties at equal t go to the primitive later in the reference's leaf order
// (each record's e2.w; the reference visits its leaves in that order and
// keeps a later equal hit, `t <= maxt`, mesh.cpp:119), so the result does not
// depend on the order of the list.  The list (runtime.hip build_scan_list):
// axis-plane triangle pairs by axis, the other triangles padded with
// never-hit records to a multiple of kScanGroup (one batch of scalar loads
// per group), then the spheres.  The root box test of bvh.cpp:420 is kept so
// rays missing the scene never report hits.  K rays per thread share every
// fetched record.
template <int K>
ND void scan_prologue(const DevScene &S, TRay (&r)[K], bool (&live)[K]) {
    const float4 rmn = make_float4(S.root_min[0], S.root_min[1], S.root_min[2], 0.f);
    const float4 rmx = make_float4(S.root_max[0], S.root_max[1], S.root_max[2], 0.f);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        TRay &x = r[k];
        if (x.mint == kEps) x.mint = smax(x.mint, x.mint * smax(smax(fabsf(x.o.x), fabsf(x.o.y)), fabsf(x.o.z)));
        x.rcp = V3{rcp_full(x.d.x), rcp_full(x.d.y), rcp_full(x.d.z)};
        float tn;
        live[k] = live[k] && !(x.maxt < x.mint) && box_test(rmn, rmx, x, tn);
    }
}

// Can the Moller-Trumbore test of a triangle in the plane x_A = c accept this
// ray?  `false` is exact: the test then rejects.  With e1_A = e2_A = 0 (both
// edges in the plane) every product with those zeros drops out of cross() and
// dot() exactly (device_math.h: x*0 = +-0 and y +- 0 = y), and with
// T = fl(o_A - c) (tvec_A, of exact sign) and D = d_A what remains is
//     t's numerator  fl(fl(P' T) - fl(Q' T))   = T n (1 + a),
//     det            fl(fl(P'' D) - fl(Q'' D))  = -D n (1 + b),
// where P, Q are the two edge products of the normal component n = P - Q
// (the primes mark the association; rounding is sign-symmetric) and
// |a|, |b| <= (2 kappa + 1) u for kappa = (|P| + |Q|) / |P - Q| <= 32,
// host-checked (runtime.hip axis_plane) with products in the normal range.
// inv_det = 1/det rounded once (rcp_rn), one more rounding for t, so
//     t = -(T / D)(1 + e),   |e| <= 132 u < 8e-6 < 2^-16.
// Hence t >= mint and t <= maxt need T and D of opposite signs and
// mint (1 - 2^-16) < |T / D| < maxt (1 + 2^-16); the products below carry
// their own relative rounding (one u each), far inside that margin.  Rays of
// zero D have det = +-0 (rejected: |det| < 1e-8), and give NaN or 0 here.
// The bounds assume mint > 0 and maxt > 0 (every path ray); a trace-API ray
// with mint <= 0 (Moller-Trumbore then accepts t = +-0 on the plane) or
// maxt <= 0 drops the bound on that side.
constexpr float kPlaneLo = 1.0f - 0x1p-16f, kPlaneHi = 1.0f + 0x1p-16f;
ND bool plane_may_hit(float o, float d, float c, float mint, float maxt) {
    const float T = o - c, ad = fabsf(d);
    const float s = d > 0.0f ? -T : T;  // > 0: the ray moves towards the plane
    const float lo = mint > 0.0f ? mint * kPlaneLo * ad : -INF_F, hi = maxt > 0.0f ? maxt * kPlaneHi * ad : INF_F;
    return s > lo && s < hi;
}

template <int A>
ND float comp(const V3 &v) { return A == 0 ? v.x : A == 1 ? v.y : v.z; }

// May the Moller-Trumbore test of a triangle of this pair accept the ray?
// false is exact (runtime.hip plane_filters): the crossing t_f must lie in
// [mint, maxt] up to the plane_may_hit margins (|t_f / t - 1| <= gamma_3 on
// top of its 133 u), and its in-plane point within the widened rectangle.
// NaN and infinite crossings (d_A = 0: det = 0, never accepted) fail the
// range test or pass the rectangle test, never wrongly reject.
template <int A>
ND bool pair_candidate(const TRay &r, const float4 &f0, const float4 &f1, float mlo, float mhi, float so, float sd) {
    constexpr int B = (A + 1) % 3, C = (A + 2) % 3;
    const float tf = (f1.y - comp<A>(r.o)) * comp<A>(r.rcp);
    const float dB = __builtin_fmaf(tf, comp<B>(r.d), comp<B>(r.o) - f0.x);
    const float dC = __builtin_fmaf(tf, comp<C>(r.d), comp<C>(r.o) - f0.z);
    const float S = __builtin_fmaf(fabsf(tf), sd, so);
    const float thB = __builtin_fmaf(f1.x, S, f0.y), thC = __builtin_fmaf(f1.x, S, f0.w);
    return tf > mlo && tf <= mhi && !(fabsf(dB) > thB) && !(fabsf(dC) > thC);
}

// One triangle record against K rays; the tie rule above.  PLANE 0-2: an
// axis-plane triangle of that axis (tri_hit_plane), -1: any triangle.
template <int K, bool ANY, int PLANE = -1>
ND void scan_tri(const float4 &a, const float4 &b, const float4 &c, TRay (&r)[K], const bool (&live)[K],
                 float (&tb)[K], uint32_t (&pb)[K], uint32_t (&lb)[K], float (&ub)[K], float (&vb)[K],
                 bool (&found)[K]) {
    const uint32_t pos = __float_as_uint(c.w);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        float t = 0, u = 0, v = 0;
        bool h;  // t <= r.maxt = tb
        if constexpr (PLANE >= 0) h = tri_hit_plane<PLANE>(a, b, c, r[k], t, u, v);
        else h = tri_hit_nb(a, b, c, r[k], t, u, v);
        if (h && live[k] && (ANY || t != tb[k] || pos > lb[k])) {
            found[k] = true;
            if (!ANY) {
                r[k].maxt = tb[k] = t;
                ub[k] = u;
                vb[k] = v;
                pb[k] = __float_as_uint(a.w);
                lb[k] = pos;
            }
        }
    }
}

// The axis-plane pairs of axis A: a pair is skipped for the whole wave when
// plane_may_hit is false for every live ray (the current maxt only shrinks,
// so an earlier bound is never too tight).  CULL false: every pair is tested
// -- the extension rays of a wave are too incoherent for a wave-wide skip
// (measured: the checks cost 7 % of the kernel's instructions and skip almost
// nothing), while shadow rays, short segments towards the lights, skip most
// walls.
#ifdef NORI_CONST_SCENE
// The hipRTC build of one scene (rtc.cpp): its scan list as literal operands.
#include "const_scene.h"
ND float4 crec(uint32_t i) { return make_float4(kCRec[4 * i], kCRec[4 * i + 1], kCRec[4 * i + 2], kCRec[4 * i + 3]); }
ND float4 cpf(uint32_t i) { return make_float4(kCPlaneF[4 * i], kCPlaneF[4 * i + 1], kCPlaneF[4 * i + 2], kCPlaneF[4 * i + 3]); }
#define NORI_SC_PLANE_END(a) kCPlaneEnd[a]
#define NORI_SC_PRIM(i) crec(i)
#define NORI_SC_PLANE_F(i) cpf(i)
#define NORI_SC_PLANE_C(g) kCPlaneC[g]
#define NORI_SC_TRIS kCTris
#define NORI_SC_REAL kCReal
#define NORI_SC_PRIMS kCPrims
#define NORI_SC_UNROLL _Pragma("unroll")
#else
#define NORI_SC_PLANE_END(a) S.plane_end[a]
#define NORI_SC_PRIM(i) S.prims[i]
#define NORI_SC_PLANE_F(i) S.plane_f[i]
#define NORI_SC_PLANE_C(g) S.plane_c[g]
#define NORI_SC_TRIS S.num_scan_tris
#define NORI_SC_REAL S.num_scan_real
#define NORI_SC_PRIMS S.num_prims
#define NORI_SC_UNROLL
#endif
template <int A, int K, bool ANY, int CULL, bool GEN = false>
ND void scan_planes(const DevScene &S, TRay (&r)[K], const bool (&live)[K], float (&tb)[K], uint32_t (&pb)[K],
                    uint32_t (&lb)[K], float (&ub)[K], float (&vb)[K], bool (&found)[K]) {
    const uint32_t g0 = A == 0 ? 0u : NORI_SC_PLANE_END(A - 1), g1 = NORI_SC_PLANE_END(A);
    NORI_SC_UNROLL
    for (uint32_t g = g0; g < g1; ++g) {
        if (CULL == 2) {  // the in-plane filter (pair_candidate): the whole rectangle, not only the plane
            constexpr int B = (A + 1) % 3, C = (A + 2) % 3;
            const float4 f0 = NORI_SC_PLANE_F(2 * g), f1 = NORI_SC_PLANE_F(2 * g + 1);
            bool may = false;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const float mlo = r[k].mint > 0.0f ? r[k].mint * kPlaneLo : -INF_F;
                const float mhi = r[k].maxt > 0.0f ? r[k].maxt * kPlaneHi : INF_F;
                const float so = fabsf(comp<B>(r[k].o)) + fabsf(comp<C>(r[k].o));
                const float sd = fabsf(comp<B>(r[k].d)) + fabsf(comp<C>(r[k].d));
                may = may || (live[k] && pair_candidate<A>(r[k], f0, f1, mlo, mhi, so, sd));
            }
            if (!__any(may)) continue;
        } else if (CULL) {
            const float c = NORI_SC_PLANE_C(g);
            bool may = false;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const float o = A == 0 ? r[k].o.x : A == 1 ? r[k].o.y : r[k].o.z;
                const float d = A == 0 ? r[k].d.x : A == 1 ? r[k].d.y : r[k].d.z;
                may = may || (live[k] && plane_may_hit(o, d, c, r[k].mint, r[k].maxt));
            }
            if (!__any(may)) continue;
        }
        float4 q[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) q[j] = NORI_SC_PRIM(6 * g + j);
        scan_tri<K, ANY, GEN ? -1 : A>(q[0], q[1], q[2], r, live, tb, pb, lb, ub, vb, found);
        scan_tri<K, ANY, GEN ? -1 : A>(q[3], q[4], q[5], r, live, tb, pb, lb, ub, vb, found);
    }
}

// ZMINT (the trace API, whose rays may carry mint <= 0): a wave holding such
// a ray tests the pairs with the generic test -- tri_hit_plane returns the
// same t except for the sign of an exactly zero t, which only mint <= 0 can
// accept.
template <int K, bool ANY, int CULL, bool ZMINT = false>
ND void scan_core(const DevScene &S, TRay (&r)[K], bool (&live)[K], float (&tb)[K], uint32_t (&pb)[K],
                  float (&ub)[K], float (&vb)[K], bool (&found)[K]) {
    scan_prologue<K>(S, r, live);
    uint32_t lb[K];  // leaf-order position of the closest hit so far
#pragma unroll
    for (int k = 0; k < K; ++k) {
        tb[k] = INF_F;
        pb[k] = 0xFFFFFFFFu;
        lb[k] = 0;
        ub[k] = vb[k] = 0.0f;
        found[k] = false;
    }
    auto all_done = [&]() {
        bool done = true;
#pragma unroll
        for (int k = 0; k < K; ++k) done = done && (found[k] || !live[k]);
        return __all(done);
    };
    bool gen = false;
    if constexpr (ZMINT) {
        bool z = false;
#pragma unroll
        for (int k = 0; k < K; ++k) z = z || (live[k] && !(r[k].mint > 0.0f));
        gen = __any(z);
    }
    if (NORI_SC_PLANE_END(2) && !gen) {
        scan_planes<0, K, ANY, CULL>(S, r, live, tb, pb, lb, ub, vb, found);
        scan_planes<1, K, ANY, CULL>(S, r, live, tb, pb, lb, ub, vb, found);
        scan_planes<2, K, ANY, CULL>(S, r, live, tb, pb, lb, ub, vb, found);
    } else if (ZMINT && NORI_SC_PLANE_END(2)) {
        scan_planes<0, K, ANY, CULL, true>(S, r, live, tb, pb, lb, ub, vb, found);
        scan_planes<1, K, ANY, CULL, true>(S, r, live, tb, pb, lb, ub, vb, found);
        scan_planes<2, K, ANY, CULL, true>(S, r, live, tb, pb, lb, ub, vb, found);
    }
    const uint32_t nt = NORI_SC_TRIS, n = NORI_SC_PRIMS, real = NORI_SC_REAL;
    NORI_SC_UNROLL
    for (uint32_t i = 2 * NORI_SC_PLANE_END(2); i < nt; i += kScanGroup) {
        if (ANY && all_done()) return;
        float4 q[3 * kScanGroup];
#pragma unroll
        for (uint32_t j = 0; j < 3 * kScanGroup; ++j) q[j] = NORI_SC_PRIM(3 * i + j);
#pragma unroll
        for (uint32_t g = 0; g < kScanGroup; ++g)
            if (i + g < real)  // (the padding records never hit)
                scan_tri<K, ANY>(q[3 * g], q[3 * g + 1], q[3 * g + 2], r, live, tb, pb, lb, ub, vb, found);
    }
    NORI_SC_UNROLL
    for (uint32_t i = nt; i < n; ++i) {
        if (ANY && all_done()) return;
        const float4 p0 = NORI_SC_PRIM(3 * i), p1 = NORI_SC_PRIM(3 * i + 1);
        const uint32_t pos = __float_as_uint(NORI_SC_PRIM(3 * i + 2).w);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            float t = 0;
            const bool h = sphere_hit_fast(p0, p1, r[k], t);  // t <= r.maxt = tb
            if (h && live[k] && (ANY || t != tb[k] || pos > lb[k])) {
                found[k] = true;
                if (!ANY) {
                    r[k].maxt = tb[k] = t;
                    ub[k] = vb[k] = 0.0f;
                    pb[k] = __float_as_uint(p0.w);
                    lb[k] = pos;
                }
            }
        }
    }
}

// Scan-mode traversal of K rays per thread: every primitive record is
// fetched once (scalar loads) and tested against K independent rays, which
// gives the VALU K independent dependency chains to interleave.  Results are
// those of traverse<0, ANY> ray by ray.  CULL: the wave-wide plane skips
// (every caller but the extension kernel, whose waves are incoherent).
template <int K, bool ANY, int CULL = 1, bool ZMINT = false>
ND void scan_rays(const DevScene &S, TRay (&r)[K], bool (&live)[K], float (&tb)[K], uint32_t (&pb)[K],
                  float (&ub)[K], float (&vb)[K], bool (&found)[K]) {
    scan_core<K, ANY, CULL, ZMINT>(S, r, live, tb, pb, ub, vb, found);
}

// A path queue entry's ray (dev_scene.h PathQueue): camera rays carry 1/z of
// their camera-space direction (mint = nearClip/z, maxt = farClip/z, as
// camera_sample computes them); every other path ray is (Epsilon, inf).
ND void path_ray(const DevScene &S, const float4 &a, const float4 &b, TRay &r) {
    r.o = ld3(a);
    r.d = ld3(b);
    const bool cam = (__float_as_uint(b.w) & kCameraRay) != 0u;
    r.mint = cam ? S.near_clip * a.w : kEps;
    r.maxt = cam ? S.far_clip * a.w : INF_F;
}

// Unoccluded shadow ray: record += payload (the reference's `color +=`,
// path_mis.cpp:48-60).  A record belongs to one path, which has at most one
// shadow ray per launch, so a plain read-modify-write is race free; it runs
// after the traversal, for unoccluded rays only (reading every ray's record
// before the scan fetched 2.3x the algorithmic bytes; three returnless float
// atomics measured 1.8x slower on cbox: every atomic writes its line through).
ND void shadow_add(float4 *rec, const float4 &c) {
    const uint32_t w = __float_as_uint(c.w);
    const float4 L = rec[w];
    rec[w] = make_float4(L.x + c.x, L.y + c.y, L.z + c.z, L.w);
}

// Work-group sizes of the scan-mode extension and shadow kernels: 256
// threads (C2 median 5176 against 5023 Msamples/s with 128; 512 makes the
// extension launch slower, 0.0786 against 0.0752 ms).
#ifndef NORI_EXTEND_BLOCK
#define NORI_EXTEND_BLOCK 256
#endif
#ifndef NORI_SHADOW_BLOCK
#define NORI_SHADOW_BLOCK 256
#endif
template <int K, uint32_t B>
constexpr uint32_t scan_per() {  // work-groups per group of kTraceGroup segments
    static_assert(K >= 1 && kTraceGroup * kSeg % (B * K) == 0 && kTraceGroup * kSeg / (B * K) >= 1,
                  "a scan work-group of B threads x K rays must tile the group's kTraceGroup * kSeg entries");
    return kTraceGroup * kSeg / (B * K);
}
// k_extend_scan: the closest hits of the path queue's extension rays.
template <int K>
ND void extend_scan_body(const DevScene &S, const PathQueue &pq, const uint32_t *cnt, uint32_t G, uint32_t bid) {
    const SegRange sr = seg_group(cnt, G, bid, scan_per<K, NORI_EXTEND_BLOCK>());
    // a lane's K rays are entries NORI_EXTEND_BLOCK apart (adjacent entries, so
    // that a wave covers 64 K consecutive ones, measured 1 % slower)
    constexpr uint32_t STEP = NORI_EXTEND_BLOCK;
    const uint32_t n = sr.pre[kTraceGroup], i0 = seg_first(bid, scan_per<K, NORI_EXTEND_BLOCK>(), NORI_EXTEND_BLOCK, K, threadIdx.x);
    if (i0 >= n) return;  // entries fill the slice from its start
    TRay r[K];
    bool live[K];
    uint32_t q[K];
    // lanes past the end load entry i0 again (unconditional loads: no
    // branch, so all of them are in flight together)
    bool cam = true;  // every live ray of this lane a camera ray
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t i = i0 + k * STEP;
        live[k] = i < n;
        q[k] = seg_entry(sr, live[k] ? i : i0);
        const float4 b = pq.ray_d[q[k]];
        path_ray(S, pq.ray_o[q[k]], b, r[k]);
        cam = cam && (!live[k] || (__float_as_uint(b.w) & kCameraRay) != 0u);
    }
    float t[K], u[K], v[K];
    uint32_t p[K];
    bool f[K];
    // A wave of camera rays (the tail of a segment: new samples, adjacent
    // pixels) is coherent: its rays leave through one or two walls, so the
    // in-plane filter skips the other pairs for the whole wave.  The
    // incoherent waves of bounce rays test every pair unchecked (a wave-wide
    // skip never happens there; NORI_CAMERA_CULL=0 tests every wave so).
    if (S.camera_cull && S.plane_f && __all(cam)) scan_rays<K, false, 2>(S, r, live, t, p, u, v, f);
    else scan_rays<K, false, 0>(S, r, live, t, p, u, v, f);
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (i0 + k * STEP < n) pq.hit[q[k]] = make_float4(t[k], __uint_as_float(p[k]), u[k], v[k]);
}

// k_shadow_scan: any hit of the shadow queue's rays; an unoccluded ray adds
// its payload to its sample record.
template <int K>
ND void shadow_scan_body(const DevScene &S, const ShadowQueue &sq, const uint32_t *shcnt, float4 *rec, uint32_t G,
                         uint32_t bid) {
    const SegRange sr = seg_group(shcnt, G, bid, scan_per<K, NORI_SHADOW_BLOCK>());
    const uint32_t n = sr.pre[kTraceGroup], i0 = seg_first(bid, scan_per<K, NORI_SHADOW_BLOCK>(), NORI_SHADOW_BLOCK, K, threadIdx.x);
    if (i0 >= n) return;
    TRay r[K];
    bool live[K], valid[K];
    uint32_t q[K];
    // unconditional loads (lanes past the end repeat entry i0); the payload is
    // fetched before the scan so its latency hides behind the traversal
    float4 c[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t i = i0 + k * NORI_SHADOW_BLOCK;
        valid[k] = live[k] = i < n;
        q[k] = seg_entry(sr, live[k] ? i : i0);
        float4 a = sq.ray_o[q[k]], b = sq.ray_d[q[k]];
        c[k] = sq.payload[q[k]];
        r[k].o = ld3(a);
        r[k].d = ld3(b);
        r[k].mint = a.w;
        r[k].maxt = b.w;
    }
    float t[K], u[K], v[K];
    uint32_t p[K];
    bool f[K];
    scan_rays<K, true>(S, r, live, t, p, u, v, f);
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (valid[k] && !f[k]) shadow_add(rec, c[k]);
}


// The trace API's scan (k_trace<0, ANY>): one caller ray per thread; mint may
// be <= 0 (scan_core ZMINT); S.trace_cull selects the wall-pair skips under test.
template <bool ANY>
ND void trace_scan_body(const DevScene &S, const float4 *rays, uint32_t n, float4 *hits) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const float4 a = rays[2 * (size_t)q], b = rays[2 * (size_t)q + 1];
    TRay rr[1];
    rr[0].o = ld3(a);
    rr[0].d = ld3(b);
    rr[0].mint = a.w;
    rr[0].maxt = b.w;
    bool live[1] = {true}, found[1];
    float t[1], u[1], v[1];
    uint32_t p[1];
#ifdef NORI_RTC_TRACE_CULL  // the hipRTC build: S.trace_cull compiled in
    scan_rays<1, ANY, NORI_RTC_TRACE_CULL, true>(S, rr, live, t, p, u, v, found);
#else
    if (S.trace_cull == 2) scan_rays<1, ANY, 2, true>(S, rr, live, t, p, u, v, found);
    else if (S.trace_cull == 0) scan_rays<1, ANY, 0, true>(S, rr, live, t, p, u, v, found);
    else scan_rays<1, ANY, 1, true>(S, rr, live, t, p, u, v, found);
#endif
    if (ANY) hits[q] = make_float4(found[0] ? 0.0f : INF_F, __uint_as_float(found[0] ? 0u : 0xFFFFFFFFu), 0.0f, 0.0f);
    else hits[q] = make_float4(t[0], __uint_as_float(p[0]), u[0], v[0]);
}

}  // namespace nori
