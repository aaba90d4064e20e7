// kernels.hip -- CDNA4 (gfx950) kernels of the wavefront path tracer.
//
// One iteration of the state machine (runtime.hip drives it):
//   k_shade   : per path: surface hit -> emission, next-event estimation
//               (light sample + shadow ray), Russian roulette, BSDF sample,
//               or regeneration of a finished path slot with a new camera
//               sample.  Work-group b owns queue segment b; survivors and
//               shadow rays are compacted inside the segment with 64-lane
//               ballots + an LDS prefix over the 4 waves (no global atomics).
//   k_extend  : closest-hit BVH traversal of the compacted path queue.
//   k_shadow  : any-hit traversal; unoccluded rays add their payload to the
//               sample record (the reference's `color +=`, path_mis.cpp:48-60).
// Once every segment's work stream is used up, k_finish runs the remaining
// paths to completion one thread per path (no per-bounce launches for the
// Russian-roulette tail), then k_splat filters every sample into the film.
//
// This replaces render.cpp:194-233 (pass loop + tbb::parallel_for),
// renderBlock (render.cpp:80-133), PathMisIntegrator::Li (path_mis.cpp:17-101),
// PathMatsIntegrator::Li (path_mats.cpp:17-60), BVH::rayIntersect
// (bvh.cpp:404-462) and ImageBlock::put (block.cpp:93-133).
#include "kernels.h"
#include "scan.h"

#include <cstdlib>

// The kernels are compiled in three translation units so that hipcc builds
// them in parallel: NORI_TU 0 (this file) = everything but the two largest
// groups, 1 (kernels_shade.hip) = k_shade + launch_shade, 2
// (kernels_finish.hip) = k_finish + launch_finish.  Templates are shared;
// each non-template kernel and launcher lives in exactly one unit.
#ifndef NORI_TU
#define NORI_TU 0
#endif

namespace nori {


// ------------------------------------------------------------------ wave helpers
ND uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
ND uint32_t rank_in(uint64_t mask) {  // set lanes of `mask` below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
// ------------------------------------------------------------------ traversal
// Load through the global address space: the scene tables sit in a struct
// of generic pointers, which would otherwise compile to FLAT loads (they also
// count against lgkmcnt, which the LDS traversal stack waits on).  BVH
// traversal always reads global memory (only scan-mode scenes are staged in LDS).
typedef float gfloat4 __attribute__((ext_vector_type(4)));
ND float4 gld(const float4 *p) {
    const gfloat4 v = *(const __attribute__((address_space(1))) gfloat4 *)p;
    return make_float4(v.x, v.y, v.z, v.w);
}

// One 4-wide BVH node: the child boxes in SoA form (mnx.x = child 0's min.x,
// ...) and the four child references (exact 128-byte nodes; quantized
// 64-byte nodes measured 9-12 % slower on C3 and the table scene, DESIGN_LOG.md).
ND void load_node(const DevScene &S, uint32_t ref, float4 &mnx, float4 &mny, float4 &mnz, float4 &mxx, float4 &mxy,
                  float4 &mxz, float4 &rf) {
    const float4 *nd = S.nodes + 8 * (size_t)ref;
    mnx = gld(nd), mny = gld(nd + 1), mnz = gld(nd + 2), mxx = gld(nd + 3), mxy = gld(nd + 4), mxz = gld(nd + 5);
    rf = gld(nd + 6);
}

// Primitive records fetched per memory round trip in a BVH leaf.
#ifndef NORI_LEAF_BATCH
#define NORI_LEAF_BATCH 1
#endif
constexpr int kLeafBatch = NORI_LEAF_BATCH;

// LDS words per lane of a traversal stack of depth STACK: child refs and entry distances.
// (stack_lds_entries(STACK) entries: the LDS budget stays STACK words, so the
// occupancy does not change; deeper entries spill to private memory)
constexpr int stack_words(int STACK) { return STACK ? STACK : 1; }

// BVH::rayIntersect (bvh.cpp:404-462): adaptive epsilon, closest or any hit.
// Near child first; the short stack lives in LDS, one column per lane.
template <int STACK, bool ANY>
ND bool traverse(const DevScene &S, TRay r, uint32_t *stk, float &tb, uint32_t &pb, float &ub, float &vb) {
    if constexpr (STACK == 0) {
        TRay rr[1] = {r};
        bool live[1] = {true}, found[1];
        float t1[1], u1[1], v1[1];
        uint32_t p1[1];
        scan_rays<1, ANY>(S, rr, live, t1, p1, u1, v1, found);
        tb = t1[0];
        pb = p1[0];
        ub = u1[0];
        vb = v1[0];
        return found[0];
    }
    if (r.mint == kEps) r.mint = smax(r.mint, r.mint * smax(smax(fabsf(r.o.x), fabsf(r.o.y)), fabsf(r.o.z)));
    tb = INF_F;
    pb = 0xFFFFFFFFu;
    ub = vb = 0.0f;
    r.rcp = V3{rcp_full(r.d.x), rcp_full(r.d.y), rcp_full(r.d.z)};
    if (r.maxt < r.mint) return false;
    // 4-wide nodes: test the four child boxes, enter the nearest hit child and
    // push the others farthest first.  Box tests are monotone (a child box lies
    // inside its parent's and rounding keeps the slab test monotone), so the
    // candidate primitives are exactly those of the reference's binary tree.
    // Stack entries carry the child's entry distance: a popped entry whose box
    // starts beyond the current closest hit is dropped unvisited -- exactly
    // the nearT <= maxt clause of its box test re-run at pop time (same ray,
    // same box, maxt only shrinks), without fetching the node.
    uint32_t spill[kTraceSpill];  // stack entries beyond the LDS part (rare)
    float spillk[kTraceSpill];
    constexpr int L = stack_lds_entries(STACK);
    auto push = [&](int &sp, uint32_t v, float k) {
        if (sp < L) {
            stk[sp * kTraceBlock] = v;
            if (NORI_STACK_KEYS) stk[(L + sp) * kTraceBlock] = __float_as_uint(k);
        } else {
            spill[sp - L] = v;
            if (NORI_STACK_KEYS) spillk[sp - L] = k;
        }
        ++sp;
    };
    uint32_t ref = 0;
    int sp = 0;
    bool found = false;
    for (;;) {
        if (!(ref & 0x80000000u)) {
            float4 mnx, mny, mnz, mxx, mxy, mxz, rf;
            load_node(S, ref, mnx, mny, mnz, mxx, mxy, mxz, rf);
            float k0, k1, k2, k3;
            bool h;
            h = box_test(make_float4(mnx.x, mny.x, mnz.x, 0), make_float4(mxx.x, mxy.x, mxz.x, 0), r, k0);
            k0 = h ? k0 : INF_F;
            const bool h0 = h;
            h = box_test(make_float4(mnx.y, mny.y, mnz.y, 0), make_float4(mxx.y, mxy.y, mxz.y, 0), r, k1);
            k1 = h ? k1 : INF_F;
            const bool h1 = h;
            h = box_test(make_float4(mnx.z, mny.z, mnz.z, 0), make_float4(mxx.z, mxy.z, mxz.z, 0), r, k2);
            k2 = h ? k2 : INF_F;
            const bool h2 = h;
            h = box_test(make_float4(mnx.w, mny.w, mnz.w, 0), make_float4(mxx.w, mxy.w, mxz.w, 0), r, k3);
            k3 = h ? k3 : INF_F;
            const bool h3 = h;
            const int nh = (int)h0 + (int)h1 + (int)h2 + (int)h3;
            if (nh > 0) {
                // order (key, ref) by entry distance; misses (key inf, hit false) sort last
                uint32_t c0 = __float_as_uint(rf.x), c1 = __float_as_uint(rf.y), c2 = __float_as_uint(rf.z),
                         c3 = __float_as_uint(rf.w);
                bool m0 = !h0, m1 = !h1, m2 = !h2, m3 = !h3;
                auto cs = [](float &ka, uint32_t &ca, bool &ma, float &kb, uint32_t &cb, bool &mb) {
                    const bool sw = ma > mb || (ma == mb && kb < ka);
                    const float tk = ka;
                    const uint32_t tc = ca;
                    const bool tm = ma;
                    ka = sw ? kb : ka;
                    kb = sw ? tk : kb;
                    ca = sw ? cb : ca;
                    cb = sw ? tc : cb;
                    ma = sw ? mb : ma;
                    mb = sw ? tm : mb;
                };
                cs(k0, c0, m0, k1, c1, m1);
                cs(k2, c2, m2, k3, c3, m3);
                cs(k0, c0, m0, k2, c2, m2);
                cs(k1, c1, m1, k3, c3, m3);
                cs(k1, c1, m1, k2, c2, m2);
                if (nh > 3) push(sp, c3, k3);
                if (nh > 2) push(sp, c2, k2);
                if (nh > 1) push(sp, c1, k1);
                ref = c0;
                continue;
            }
        } else {
            // leaf: the records of NORI_LEAF_BATCH primitives are fetched
            // together (every record is 48 B, so the third vector is loaded
            // unconditionally; lanes past the leaf end re-read its last
            // record) -- one memory round trip per batch instead of one or
            // two per primitive.  Tested in leaf order, as bvh.cpp:440-452.
            const uint32_t start = ref & 0x1FFFFFFu, end = start + ((ref >> 25) & 63u) + 1u;
            for (uint32_t i0 = start; i0 < end; i0 += kLeafBatch) {
                float4 q[kLeafBatch][3];
#pragma unroll
                for (int k = 0; k < kLeafBatch; ++k) {
                    const float4 *p = S.prims + 3 * (size_t)min(i0 + (uint32_t)k, end - 1u);
                    q[k][0] = gld(p);
                    q[k][1] = gld(p + 1);
                    q[k][2] = gld(p + 2);
                }
#pragma unroll
                for (int k = 0; k < kLeafBatch; ++k) {
                    if (i0 + (uint32_t)k >= end) break;
                    float t = 0, u = 0, v = 0;
                    bool h;
                    if (__float_as_uint(q[k][1].w) == 0u) {
                        h = tri_hit(q[k][0], q[k][1], q[k][2], r, t, u, v);
                    } else {
                        h = sphere_hit(q[k][0], q[k][1], r, t);
                        u = v = 0.0f;
                    }
                    if (h) {
                        if (ANY) return true;
                        found = true;
                        r.maxt = tb = t;
                        ub = u;
                        vb = v;
                        pb = __float_as_uint(q[k][0].w);
                    }
                }
            }
        }
        bool next = false;
        while (sp > 0) {
            --sp;
            ref = sp < L ? stk[sp * kTraceBlock] : spill[sp - L];
            if (!NORI_STACK_KEYS) {
                next = true;
                break;
            }
            const float key = sp < L ? __uint_as_float(stk[(L + sp) * kTraceBlock]) : spillk[sp - L];
            if (!(key > r.maxt)) {
                next = true;
                break;
            }
        }
        if (!next) break;
    }
    (void)STACK;
    return found;
}

template <int STACK, bool ANY>
__global__ __launch_bounds__(kTraceBlock) void k_trace(DevScene S, const float4 *rays, uint32_t n, float4 *hits) {
    if constexpr (STACK == 0) {  // the caller's rays: mint may be <= 0 (scan_core ZMINT)
        trace_scan_body<ANY>(S, rays, n, hits);
        return;
    }
    __shared__ uint32_t stk[stack_words(STACK) * kTraceBlock];
    uint32_t q = blockIdx.x * kTraceBlock + threadIdx.x;
    if (q >= n) return;
    float4 a = rays[2 * (size_t)q], b = rays[2 * (size_t)q + 1];
    TRay r;
    r.o = ld3(a);
    r.d = ld3(b);
    r.mint = a.w;
    r.maxt = b.w;
    float t, u, v;
    uint32_t p;
    const bool h = traverse<STACK, ANY>(S, r, stk + threadIdx.x, t, p, u, v);
    if (ANY) hits[q] = make_float4(h ? 0.0f : INF_F, __uint_as_float(h ? 0u : 0xFFFFFFFFu), 0.0f, 0.0f);
    else hits[q] = make_float4(t, __uint_as_float(p), u, v);
}

// Entry numbering of the trace launches: seg_index.h.
constexpr uint32_t kTraceSlices = kTraceGroup * kSeg / kTraceBlock;  // BVH-walk work-groups per group
ND SegRange seg_range(const uint32_t *cnt, uint32_t G, uint32_t bid) { return seg_group(cnt, G, bid, kTraceSlices); }

// Extension rays: closest hit of every queued path (work-group `bid` of the
// launch's extension part).
template <int STACK>
ND void extend_body(const DevScene &S, const PathQueue &pq, const uint32_t *cnt, uint32_t G, uint32_t bid,
                    uint32_t *stk) {
    const SegRange sr = seg_range(cnt, G, bid);
    const uint32_t i = seg_first(bid, kTraceSlices, kTraceBlock, 1, threadIdx.x);
    if (i < sr.pre[kTraceGroup]) {
        const uint32_t q = seg_entry(sr, i);
        TRay r;
        path_ray(S, pq.ray_o[q], pq.ray_d[q], r);
        float t, u, v;
        uint32_t p;
        traverse<STACK, false>(S, r, stk + threadIdx.x, t, p, u, v);
        pq.hit[q] = make_float4(t, __uint_as_float(p), u, v);
    }
}

// Shadow rays: any hit; unoccluded -> record += payload.
template <int STACK>
ND void shadow_body(const DevScene &S, const ShadowQueue &sq, const uint32_t *shcnt, float4 *rec, uint32_t G,
                    uint32_t bid, uint32_t *stk) {
    const SegRange sr = seg_range(shcnt, G, bid);
    const uint32_t i = seg_first(bid, kTraceSlices, kTraceBlock, 1, threadIdx.x);
    if (i < sr.pre[kTraceGroup]) {
        const uint32_t q = seg_entry(sr, i);
        float4 a = sq.ray_o[q], b = sq.ray_d[q];
        TRay r;
        r.o = ld3(a);
        r.d = ld3(b);
        r.mint = a.w;
        r.maxt = b.w;
        float t, u, v;
        uint32_t p;
        if (!traverse<STACK, true>(S, r, stk + threadIdx.x, t, p, u, v)) shadow_add(rec, sq.payload[q]);
    }
}

#ifdef NORI_TRACE_WAVES
#define NORI_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(NORI_TRACE_WAVES)))
#else
#define NORI_TRACE_ATTR
#endif
// XCD-aware block order for the BVH walks (NORI_XCD_REMAP): the dispatcher
// sends work-group b to XCD b % 8, each XCD with its own 4 MB L2.  Giving XCD
// x a contiguous range of queue segments (neighbouring image chunks, so
// nearby ray origins) lets each L2 hold the part of the tree its rays visit.
// A bijection of [0, nb): XCD x takes ranks [x q + min(x, r), ... + count).
#ifndef NORI_XCD_REMAP
#define NORI_XCD_REMAP 1
#endif
constexpr uint32_t kXcds = 8;
ND uint32_t xcd_block(uint32_t b, uint32_t nb) {
    if (!NORI_XCD_REMAP) return b;
    const uint32_t x = b % kXcds, k = b / kXcds, q = nb / kXcds, r = nb % kXcds;
    return x * q + min(x, r) + k;
}
template <int STACK>
__global__ __launch_bounds__(kTraceBlock) NORI_TRACE_ATTR void k_extend(DevScene S, PathQueue pq, const uint32_t *cnt, uint32_t G) {
    __shared__ uint32_t stk[stack_words(STACK) * kTraceBlock];
    extend_body<STACK>(S, pq, cnt, G, STACK ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x, stk);
}
template <int STACK>
__global__ __launch_bounds__(kTraceBlock) NORI_TRACE_ATTR void k_shadow(DevScene S, ShadowQueue sq, const uint32_t *shcnt,
                                                        float4 *rec, uint32_t G) {
    __shared__ uint32_t stk[stack_words(STACK) * kTraceBlock];
    shadow_body<STACK>(S, sq, shcnt, rec, G, STACK ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x, stk);
}
// An iteration's extension and shadow walks in one launch (launch_trace_both):
// work-groups [0, nb_ext) walk the extension rays, the rest the shadow rays
// (independent queues); nb_ext is a multiple of the 8 XCDs, so both ranges
// keep their XCD-aware order.
template <int STACK>
__global__ __launch_bounds__(kTraceBlock) NORI_TRACE_ATTR void k_trace_both(DevScene S, PathQueue pq, const uint32_t *cnt,
                                                                            ShadowQueue sq, const uint32_t *shcnt,
                                                                            float4 *rec, uint32_t G, uint32_t nb_ext) {
    __shared__ uint32_t stk[stack_words(STACK) * kTraceBlock];
    if (blockIdx.x < nb_ext) extend_body<STACK>(S, pq, cnt, G, xcd_block(blockIdx.x, nb_ext), stk);
    else shadow_body<STACK>(S, sq, shcnt, rec, G, xcd_block(blockIdx.x - nb_ext, gridDim.x - nb_ext), stk);
}
template <int K>
__global__ __launch_bounds__(NORI_EXTEND_BLOCK) void k_extend_scan(DevScene S, PathQueue pq, const uint32_t *cnt,
                                                                   uint32_t G) {
    extend_scan_body<K>(S, pq, cnt, G, blockIdx.x);
}
template <int K>
__global__ __launch_bounds__(NORI_SHADOW_BLOCK) void k_shadow_scan(DevScene S, ShadowQueue sq, const uint32_t *shcnt,
                                                                   float4 *rec, uint32_t G) {
    shadow_scan_body<K>(S, sq, shcnt, rec, G, blockIdx.x);
}

// ------------------------------------------------------------------ shading helpers
struct SurfHit {
    V3 p;
    Frame sh;
    int shape;
    V2 uv;
};

// setHitInformation: mesh.cpp:122-170, sphere.cpp:78-93 (shading frame and
// texture coordinates; a mesh without UVs keeps the barycentrics in its.uv).
template <bool FULL = true>
ND SurfHit surface(const DevScene &S, uint32_t prim, float t, float u, float v, V3 o, V3 d) {
    SurfHit h;
    h.shape = (int)S.prim_shape[prim];
    const DevShape &sh = S.shapes[h.shape];
    // only a textured albedo reads the texture coordinates (BRec.uv): the
    // sphere's atan2/acos are skipped for every other BSDF
    const bool need_uv = FULL && (S.bsdfs[sh.bsdf].tex != NORI_TEXTURE_CONSTANT || sh.nmap);
    h.uv = V2{u, v};
    if (sh.type == NORI_SHAPE_SPHERE) {
        h.p = o + d * t;
        const V3 n = normalize(h.p - V3{sh.center[0], sh.center[1], sh.center[2]});
        h.sh = frame_from(n);
        if (need_uv) {
            // sphericalCoordinates (common.cpp:264-272); 0.5 is a double literal
            float phi = atan2f(n.y, n.x);
            if (phi < 0) phi += 2 * kPi;
            h.uv.x = (float)(0.5 + (double)(acosf(n.z) / (2 * kPi)));
            h.uv.y = phi / kPi;
        }
    } else {
        const uint32_t *f = S.tri_vidx + 3 * (size_t)prim;
        uint32_t i0 = f[0], i1 = f[1], i2 = f[2];
        const float4 q0 = S.pos[i0], q1 = S.pos[i1], q2 = S.pos[i2];
        V3 p0 = ld3(q0), p1 = ld3(q1), p2 = ld3(q2);
        float bx = 1 - (u + v);
        h.p = (p0 * bx + p1 * u) + p2 * v;
        if (need_uv && sh.has_uvs)  // u in pos.w, v in nrm.w
            h.uv = V2{(bx * q0.w + u * q1.w) + v * q2.w,
                      (bx * S.nrm[i0].w + u * S.nrm[i1].w) + v * S.nrm[i2].w};
        if (sh.has_normals) {
            V3 n = (ld3(S.nrm[i0]) * bx + ld3(S.nrm[i1]) * u) + ld3(S.nrm[i2]) * v;
            h.sh = frame_from(normalize(n));
            if (FULL && sh.nmap) {  // NormalMap::eval (normalmap.cpp:95-134): 2 * byte / 255 - 1, normalized
                const V3 t = texel_rgb(texel_at(sh.nmap, sh.nm_w, sh.nm_h, sh.nm_wrap, h.uv));
                const V3 m = V3{2.0f * t.x - 1.0f, 2.0f * t.y - 1.0f, 2.0f * t.z - 1.0f};
                h.sh = frame_from(to_world(h.sh, normalize(m)));
            }
        } else {
            h.sh = frame_from(normalize(cross(p1 - p0, p2 - p0)));
        }
    }
    return h;
}

// EnvironmentMap (envmap.cpp), restated as the oracle's env_* functions.
constexpr float kEnvTFar = 100000.0f;  // envmap.cpp:9
// sphericalCoordinates (common.cpp:264-272) + mapIntersect (envmap.cpp:61-75)
ND V2 env_map(const DevEmitter &e, V3 vec) {
    float theta = acosf(vec.z), phi = atan2f(vec.y, vec.x);
    if (phi < 0) phi = (float)((double)phi + 2 * M_PI);
    V2 uv;
    uv.x = theta * (float)(e.R - 1) * kInvPi;
    uv.y = (float)((double)phi * 0.5 * (double)(e.C - 1) * (double)kInvPi);
    if (isnan(uv.x) || isnan(uv.y)) uv = V2{0, 0};
    return uv;
}
ND int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
ND V3 env_texel(const DevScene &S, const DevEmitter &e, int i, int j) {
    const float *c = S.env + e.rgb_off + 3 * ((size_t)i * e.C + j);
    return V3{c[0], c[1], c[2]};
}
// EnvironmentMap::eval (envmap.cpp:124-156): bilinear, wrapping at the edges
ND V3 env_eval(const DevScene &S, const DevEmitter &e, V3 wi) {
    const V2 uv = env_map(e, normalize(wi));
    const int u = clampi((int)uv.x, 0, e.R - 1), v = clampi((int)uv.y, 0, e.C - 1);
    const int us = (u + 1) % e.R, vs = (v + 1) % e.C;
    const V3 BL = env_texel(S, e, u, v), UL = env_texel(S, e, u, vs), BR = env_texel(S, e, us, v),
             UR = env_texel(S, e, us, vs);
    const int dusu = us - u, dvsv = vs - v;
    const float dusum = (float)us - uv.x, dumu = uv.x - (float)u, dvmv = uv.y - (float)v, dvsvm = (float)vs - uv.y;
    const V3 acc = ((((BL * dusum) * dvsvm) + ((BR * dumu) * dvsvm)) + ((UL * dusum) * dvmv)) + ((UR * dumu) * dvmv);
    const float inv = (float)(1.0 / (double)(dusu * dvsv));
    const V3 r = V3{inv * acc.x, inv * acc.y, inv * acc.z};
    return V3{e.weight * r.x, e.weight * r.y, e.weight * r.z};
}
// EnvironmentMap::pdf (envmap.cpp:184-192)
ND float env_pdf(const DevScene &S, const DevEmitter &e, V3 wi) {
    const V2 uv = env_map(e, normalize(wi));
    const int i = clampi((int)uv.x, 0, e.R - 1), j = clampi((int)uv.y, 0, e.C - 1);
    return S.env[e.pmarg_off + i] * S.env[e.pdf_off + (size_t)i * e.C + j];
}
// sample1D (envmap.cpp:112-122): the reference scans for the first i with
// P[i] <= s < P[i+1] (the oracle keeps that scan).  P[0..cols-1] is
// nondecreasing (P[0] = 0 plus non-negative pf terms; only the final
// P[cols] = 1 of the literal precompute1D can drop below P[cols-1]), so the
// first such i below cols-1 is upper_bound(P[0..cols-1], s) - 1, and every
// other case -- s >= P[cols-1], or no interval at all (all-zero rows, NaN s)
// -- ends at cols-1 in the scan too.  Binary search: O(log cols) loads
// instead of up to cols dependent pairs per environment sample.
ND void env_sample1D(const float *pf, const float *P, int cols, float s, float &x, float &prob) {
    int lo = 0, hi = cols;  // first j in [0, cols) with P[j] > s, or cols
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (P[mid] <= s) lo = mid + 1;
        else hi = mid;
    }
    const int i = (lo == 0 || lo >= cols) ? cols - 1 : lo - 1;
    const float t = (P[i + 1] - s) / (P[i + 1] - P[i]);
    x = (1 - t) * (float)i + t * (float)(i + 1);
    prob = pf[i];
}
// EnvironmentMap::sample (envmap.cpp:158-181); deviation D4: the Jacobian
// uses the sampled direction (the reference reads lRec.wi uninitialised).
ND V3 env_sample(const DevScene &S, const DevEmitter &e, V2 smp, V3 &wi) {
    float u, v, u_pdf, v_pdf;
    env_sample1D(S.env + e.pmarg_off, S.env + e.cmarg_off, e.R, smp.x, u, u_pdf);
    const int row = (int)u;
    env_sample1D(S.env + e.pdf_off + (size_t)row * e.C, S.env + e.cdf_off + (size_t)row * (e.C + 1), e.C, smp.y, v,
                 v_pdf);
    const float theta = (float)((double)u * M_PI / (double)(e.R - 1));  // invMapIntersect
    const float phi = (float)((double)(v * 2.0f) * M_PI / (double)(e.C - 1));
    wi = normalize(V3{sinf(theta) * cosf(phi), sinf(theta) * sinf(phi), cosf(theta)});
    const float st2 = 1.0f - wi.z * wi.z, st = st2 <= 0.0f ? 0.0f : sqrtf(st2);  // Frame::sinTheta
    const float jac = (float)((double)((e.C - 1) * (e.R - 1)) / (2 * (M_PI * M_PI) * (double)st));
    v_pdf = env_pdf(S, e, wi) * jac;
    const V3 c = env_eval(S, e, wi);
    return V3{c.x / v_pdf, c.y / v_pdf, c.z / v_pdf};
}

// AreaEmitter (arealight.cpp:39-76) or EnvironmentMap
template <bool FULL = true>
ND float emitter_pdf(const DevScene &S, const DevEmitter &e, V3 n, V3 wi) {
    if (FULL && e.type == NORI_EMITTER_ENVMAP) return env_pdf(S, e, wi);
    return dot(n, -wi) > 0.0f ? S.shapes[e.shape].area_norm : 0.0f;
}
template <bool FULL = true>
ND V3 emitter_eval(const DevScene &S, const DevEmitter &e, V3 n, V3 wi) {
    if (FULL && e.type == NORI_EMITTER_ENVMAP) return env_eval(S, e, wi);
    return dot(n, -wi) > 0.0f ? V3{e.radiance[0], e.radiance[1], e.radiance[2]} : V3{0, 0, 0};
}
// Shape::sampleSurface: Mesh (mesh.cpp:40-58, DiscretePDF::sampleReuse
// dpdf.h:152-157) or Sphere (sphere.cpp:95-100).
ND void sample_surface(const DevScene &S, const DevShape &sh, V2 smp, V3 &p, V3 &n) {
    if (sh.type == NORI_SHAPE_SPHERE) {
        V3 q = sq_uniform_sphere(smp);
        p = V3{sh.center[0], sh.center[1], sh.center[2]} + q * sh.radius;
        n = q;
        return;
    }
    const float *cdf = S.cdf + sh.cdf_offset;
    uint32_t lo = 0, hi = sh.prim_count + 1;
    float x = smp.x;
    while (lo < hi) {  // lower_bound
        uint32_t mid = (lo + hi) >> 1;
        if (cdf[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    uint32_t idx = lo == 0 ? 0 : lo - 1;
    if (idx > sh.prim_count - 1) idx = sh.prim_count - 1;
    float c0 = cdf[idx], c1 = cdf[idx + 1];
    x = (x - c0) / (c1 - c0);
    V3 bc = sq_uniform_triangle(V2{x, smp.y});
    const uint32_t *f = S.tri_vidx + 3 * (size_t)(sh.prim_offset + idx);
    uint32_t i0 = f[0], i1 = f[1], i2 = f[2];
    V3 p0 = ld3(S.pos[i0]), p1 = ld3(S.pos[i1]), p2 = ld3(S.pos[i2]);
    p = (p0 * bc.x + p1 * bc.y) + p2 * bc.z;
    if (sh.has_normals)
        n = normalize((ld3(S.nrm[i0]) * bc.x + ld3(S.nrm[i1]) * bc.y) + ld3(S.nrm[i2]) * bc.z);
    else
        n = normalize(cross(p1 - p0, p2 - p0));
}

// Camera::sampleRay: PerspectiveCamera (perspective.cpp:90-112), ThinLensCamera
// (thinlens.cpp:120-147) and AdvancedCamera (advancedCamera.cpp:85-157: barrel
// distortion, uniform-disk lens, per-channel focus shift with chromatic
// aberration, channel = 0..2 then; -1 otherwise).  Eigen column order.
template <bool FULL = true>
ND void camera_sample(const DevScene &S, float px, float py, V2 ap, int channel, V3 &o, V3 &d, float &mint,
                      float &maxt, float *invz_out = nullptr) {
    const float *m = S.s2c;
    const float qx = px * S.invW, qy = py * S.invH;
    const float r0 = ((m[0] * qx + m[1] * qy) + m[2] * 0.0f) + m[3];
    const float r1 = ((m[4] * qx + m[5] * qy) + m[6] * 0.0f) + m[7];
    const float r2 = ((m[8] * qx + m[9] * qy) + m[10] * 0.0f) + m[11];
    const float r3 = ((m[12] * qx + m[13] * qy) + m[14] * 0.0f) + m[15];
    V3 nearP = V3{r0 / r3, r1 / r3, r2 / r3};
    V3 dl = normalize(nearP);
    float w = 0.0f;
    bool chroma = false;
    if (FULL && S.cam_type == NORI_CAMERA_ADVANCED) {
        const float k1 = S.distortion[0], k2 = S.distortion[1];
        if (k1 != 0.0f || k2 != 0.0f) {  // Newton iterations for the undistorted radius
            const float ux = nearP.x / nearP.z, uy = nearP.y / nearP.z;
            const float y = sqrtf(ux * ux + uy * uy);
            float r = y, rr, f, df;
            int i = 0;
            for (;;) {
                rr = r * r;
                f = r * (1 + (k1 * rr) + k2 * (rr * rr)) - y;
                df = 1 + (3 * k1 * rr) + (5 * k2 * rr * rr);
                r = r - f / df;
                if ((double)fabsf(f) < 1e-6 || i++ > 4) break;
            }
            const float factor = r / y;
            nearP.x *= factor;
            nearP.y *= factor;
            dl = normalize(nearP);
        }
        chroma = S.chromatic[0] != 0.0f || S.chromatic[1] != 0.0f || S.chromatic[2] != 0.0f;
        if (chroma) w = S.chromatic[channel < 0 ? 0 : (channel > 2 ? 2 : channel)];
    }
    const float invZ = rcp_full(dl.z);
    const float *c = S.c2w;
    V3 lo = V3{0, 0, 0};
    if (FULL && S.cam_type != NORI_CAMERA_PERSPECTIVE && (S.lens_radius > 0.0f || chroma)) {
        V2 pl = S.cam_type == NORI_CAMERA_THINLENS ? sq_concentric_disk(ap) : sq_uniform_disk(ap);
        pl = V2{S.lens_radius * pl.x, S.lens_radius * pl.y};
        const float ft = S.focal / dl.z;
        V3 pf = dl * ft;  // Ray3f(0, d)(ft)
        if (S.cam_type == NORI_CAMERA_ADVANCED) {
            float spx = px - 0.5f * (float)S.W, spy = py - 0.5f * (float)S.H;
            spx /= (float)S.W_max;
            spy /= (float)S.W_max;
            const float sq = spx * spx + spy * spy;
            pf = pf + V3{-((spx * sq) * w), (spy * sq) * w, 0.0f};
        }
        lo = V3{pl.x, pl.y, 0.0f};
        dl = normalize(pf - lo);
        const float hw = ((c[12] * lo.x + c[13] * lo.y) + c[14] * lo.z) + c[15];
        o = V3{(((c[0] * lo.x + c[1] * lo.y) + c[2] * lo.z) + c[3]) / hw,
               (((c[4] * lo.x + c[5] * lo.y) + c[6] * lo.z) + c[7]) / hw,
               (((c[8] * lo.x + c[9] * lo.y) + c[10] * lo.z) + c[11]) / hw};
    } else {
        o = V3{S.cam_o[0], S.cam_o[1], S.cam_o[2]};  // cameraToWorld * (0,0,0,1), same for every ray (host)
    }
    d = V3{(c[0] * dl.x + c[1] * dl.y) + c[2] * dl.z, (c[4] * dl.x + c[5] * dl.y) + c[6] * dl.z,
           (c[8] * dl.x + c[9] * dl.y) + c[10] * dl.z};
    mint = S.near_clip * invZ;
    maxt = S.far_clip * invZ;
    if (invz_out) *invz_out = invZ;  // path queue encoding of a camera ray (path_ray)
}

// ------------------------------------------------------------------ shade + regenerate
struct PathState {
    V3 o, d;
    float mint, maxt;
    V3 beta;
    float prev;  // BSDF pdf of the last bounce; -1: w_mats = 1 (camera ray or discrete lobe)
    Pcg rng;
    uint32_t work;
    bool cam;    // the ray is a camera ray (stored with invz instead of prev)
    uint32_t chan;  // chromatic aberration: the colour channel whose Li this path computes (0 otherwise)
    float invz;  // camera ray: 1/z of its camera-space direction
    V3 L;  // finisher only: the sample's radiance so far (the record, held in registers)
};
struct ShadowOut {
    bool emit;
    V3 o, d, contrib;
    float maxt;
    uint32_t work;
    bool has_em;  // S.nee_inline: the vertex's emission (nee_em_lds) waits for k_shade's record update
};

// Sample id of work id w (render.cpp's (pass, pixel) sample; the pcg32 stream
// key of wave_seed): pass = w / M of the chunk, pixel = the work list's entry.
ND uint64_t sample_id(const DevScene &S, const WorkDesc &wd, uint32_t w) {
    const uint32_t pass = w / wd.M;
    return (uint64_t)(wd.pass_begin + pass) * ((uint64_t)S.W * (uint64_t)S.H) + wd.pixels[w - pass * wd.M];
}
ND void load_path(const DevScene &S, const WorkDesc &wd, const PathQueue &Q, uint32_t q, PathState &ps) {
    const float4 ro = Q.ray_o[q], rd = Q.ray_d[q], th = Q.thr[q];
    const uint32_t sh = Q.rng[q];
    ps.o = ld3(ro);
    ps.d = ld3(rd);
    const uint32_t wf = __float_as_uint(rd.w);
    ps.work = wf & kWorkMask;
    ps.chan = (wf >> kChanShift) & 3u;
    ps.cam = (wf & kCameraRay) != 0u;
    ps.invz = ro.w;
    ps.prev = ps.cam ? -1.0f : ro.w;
    ps.mint = ps.cam ? S.near_clip * ro.w : kEps;
    ps.maxt = ps.cam ? S.far_clip * ro.w : INF_F;
    ps.beta = ld3(th);
    ps.rng.state = ((uint64_t)sh << 32) | __float_as_uint(th.w);
    ps.rng.inc = (sample_id(S, wd, ps.work) << 1u) | 1u;  // pcg32 seed(initstate, initseq = sid)
}
ND void store_path(const PathQueue &Q, uint32_t i, const PathState &ps) {
    Q.ray_o[i] = make_float4(ps.o.x, ps.o.y, ps.o.z, ps.cam ? ps.invz : ps.prev);
    Q.ray_d[i] = make_float4(ps.d.x, ps.d.y, ps.d.z,
                             __uint_as_float(ps.work | (ps.chan << kChanShift) | (ps.cam ? kCameraRay : 0u)));
    Q.thr[i] = make_float4(ps.beta.x, ps.beta.y, ps.beta.z, __uint_as_float((uint32_t)ps.rng.state));
    Q.rng[i] = (uint32_t)(ps.rng.state >> 32);
}

// ------------------------------------------------------------------ medium
// HomogeneousMedium (medium.cpp:22-94): box = origin -/+ |size|, sigma_t =
// sigma_a + sigma_s, albedo = sigma_s / sigma_t, isotropic phase function
// (phasefunction.cpp:13-16).
// BoundingBox3f::rayIntersect(ray, nearT, farT) (bbox.h:366-393) for the ray
// (o, d) with dRcp = 1/d; a NaN direction leaves the slab test false.
ND bool mbox_range(const DevScene &S, V3 o, V3 d, float &nearT, float &farT) {
    nearT = -INF_F;
    farT = INF_F;
    const float oc[3] = {o.x, o.y, o.z}, dc[3] = {d.x, d.y, d.z};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float origin = oc[i], mn = S.mbox_min[i], mx = S.mbox_max[i];
        if (dc[i] == 0.0f) {
            if (origin < mn || origin > mx) return false;
        } else {
            const float r = rcp_full(dc[i]);
            float t1 = (mn - origin) * r, t2 = (mx - origin) * r;
            if (t1 > t2) {
                float t = t1;
                t1 = t2;
                t2 = t;
            }
            nearT = smax(t1, nearT);
            farT = smin(t2, farT);
            if (!(nearT <= farT)) return false;
        }
    }
    return true;
}
ND bool mbox_contains(const DevScene &S, V3 p) {  // bbox.h:115-123 (non-strict)
    return p.x >= S.mbox_min[0] && p.y >= S.mbox_min[1] && p.z >= S.mbox_min[2] && p.x <= S.mbox_max[0] &&
           p.y <= S.mbox_max[1] && p.z <= S.mbox_max[2];
}
// HomogeneousMedium::Tr(src, dst): transmittance over the part of [src, dst]
// inside the box.  Tr(p, p) has a NaN direction and is 1, as in the reference.
ND V3 medium_tr(const DevScene &S, V3 src, V3 dst) {
    if (!S.has_medium) return V3{1, 1, 1};
    const V3 d = normalize(dst - src);
    float nearT, farT;
    if (!mbox_range(S, src, d, nearT, farT)) return V3{1, 1, 1};
    const V3 sp = mbox_contains(S, src) ? src : src + normalize(d) * nearT;
    const V3 ep = mbox_contains(S, dst) ? dst : src + normalize(d) * farT;
    const float n = norm(ep - sp);
    return V3{expf(-S.sigma_t[0] * n), expf(-S.sigma_t[1] * n), expf(-S.sigma_t[2] * n)};
}
// HomogeneousMedium::sample: free-flight distance from the box entry point;
// true (and p) when the ray scatters before tmax.  No random number is drawn
// for a ray that misses the box.
ND bool medium_sample(const DevScene &S, V3 o, V3 d, Pcg &rng, float tmax, V3 &p) {
    if (!S.has_medium) return false;
    float nearT, farT;
    if (!mbox_range(S, o, d, nearT, farT)) return false;
    const V3 sp = mbox_contains(S, o) ? o : o + normalize(d) * nearT;
    const float st = smax(smax(S.sigma_t[0], S.sigma_t[1]), S.sigma_t[2]);
    const float distance = norm(sp - o) + (-1.0f * logf(1 - next1D(rng)) / st);  // invTr
    if (distance >= tmax) return false;
    p = o + d * distance;  // Ray3f::operator()
    return true;
}

// PointLight::sample (pointlight.cpp:17-25) and SpotLight::sample
// (spotlight.cpp:20-46, falloff by the angle to the spot direction) from x:
// returns the radiance, sets the direction and the shadow ray's maxt.
ND V3 point_sample(const DevEmitter &E, V3 x, V3 &wi, float &maxt) {
    const V3 pos = V3{E.position[0], E.position[1], E.position[2]};
    const V3 d = pos - x;
    wi = normalize(d);
    maxt = norm(d) - kEps;
    const V3 pw = V3{E.power[0], E.power[1], E.power[2]};
    if (E.type == NORI_EMITTER_POINT) return pw / (4.f * kPi * dot(d, d));
    const V3 w = -wi, dir = V3{E.direction[0], E.direction[1], E.direction[2]};
    const float cosTheta = dot(dir, normalize(w));
    float fo;
    if (cosTheta < E.cos_tw) fo = 0;
    else if (cosTheta > E.cos_fs) fo = 1;
    else fo = (acosf(E.cos_tw) - acosf(cosTheta)) / (acosf(E.cos_tw) - acosf(E.cos_fs));
    const V3 q = x - pos;
    return (pw * fo) / (4.f * kPi * dot(q, q));
}

// Next-event estimation from x (AreaEmitter::sample, arealight.cpp:52-68):
// one emitter chosen uniformly (scene.h:68-74), Li already scaled by N.
struct NeeSample {
    V3 p, wi, Li;
    float pdf_em, maxt;  // maxt: of the shadow ray from x
};
// Emitter::sample of one emitter from x with the 2D sample s2: radiance over
// pdf (not yet scaled by the emitter count), direction, area-measure pdf and
// the shadow ray's maxt.
template <bool FULL = true>
ND NeeSample emitter_sample_one(const DevScene &S, const DevEmitter &E, V3 x, V2 s2) {
    NeeSample r;
    if (FULL && (E.type == NORI_EMITTER_POINT || E.type == NORI_EMITTER_SPOT)) {
        r.Li = point_sample(E, x, r.wi, r.maxt);
        r.pdf_em = 1.0f;  // PDF_VALUE (pointlight.cpp:32-35) / lRec.pdf (spotlight.cpp:54-57)
        r.p = V3{E.position[0], E.position[1], E.position[2]};
        return r;
    }
    if (FULL && E.type == NORI_EMITTER_ENVMAP) {
        r.Li = env_sample(S, E, s2, r.wi);
        r.pdf_em = env_pdf(S, E, r.wi);
        r.maxt = kEnvTFar;               // shadow ray (ref, wi, Epsilon, T_FAR)
        r.p = x + r.wi * kEnvTFar;       // D4: lRec.p is never set by the reference
        return r;
    }
    V3 ln;
    sample_surface(S, S.shapes[E.shape], s2, r.p, ln);
    const V3 dv = r.p - x;
    r.wi = normalize(dv);
    r.pdf_em = emitter_pdf<FULL>(S, E, ln, r.wi);
    const float att = dot(ln, -r.wi) / dot(dv, dv);
    r.Li = r.pdf_em > 0.0f ? (emitter_eval<FULL>(S, E, ln, r.wi) * att) / r.pdf_em : V3{0, 0, 0};
    r.maxt = norm(dv) - kEps;
    return r;
}
// Next-event estimation of the path integrators: one emitter chosen uniformly
// (Scene::getRandomEmitter, scene.h:68-74), Li scaled by the emitter count.
// (ul, s2: the emitter-choice draw and the 2D light sample, in that order)
template <bool FULL = true>
ND NeeSample nee_sample_u(const DevScene &S, V3 x, float ul, V2 s2) {
    const uint32_t N = S.num_emitters;
    uint32_t li = (uint32_t)floorf((float)N * ul);
    if (li > N - 1) li = N - 1;
    NeeSample r = emitter_sample_one<FULL>(S, S.emitters[li], x, s2);
    r.Li = r.Li * (float)N;
    return r;
}
template <bool FULL = true>
ND NeeSample nee_sample(const DevScene &S, V3 x, Pcg &rng) {
    const float ul = next1D(rng);
    const V2 s2 = next2D(rng);
    return nee_sample_u<FULL>(S, x, ul, s2);
}

// Chromatic aberration (render.cpp:106-121): a sample's value is
// value0 + value1 + value2 with value_c = e_c * Li_c (e_c the unit colour of
// channel c), so component c of the record gets Li_c.c and the two other
// paths add 0 * Li_k.c there -- +-0, or NaN when that term is not finite,
// which the splat's validity check then drops, as the reference does.  Each
// contribution of channel c's path goes to the record through this mask.
ND V3 chan_only(const DevScene &S, uint32_t ch, const V3 &a) {
    if (!S.chroma) return a;
    return V3{ch == 0 ? a.x : 0.0f * a.x, ch == 1 ? a.y : 0.0f * a.y, ch == 2 ? a.z : 0.0f * a.z};
}

// Emission found by the shade kernel, added to the sample record.  Each record
// has one path, and the shadow kernel's read-modify-write of it runs in a later
// launch, so the adds need no atomicity -- but returnless atomics do not make
// the wave wait for the record's read (a full memory latency in most waves);
// IEEE adds in the same order, so the sums are identical.
// ATOMIC false (finisher): the sum is kept in ps.L, in registers -- a tail
// path's bounces are a serial chain, and a record read per bounce would add a
// memory latency to each.
// S.nee_inline (k_shade traces the vertex's shadow ray itself): the emission
// waits in so.em for the one read-modify-write of the record at the kernel's
// end, which adds it first and then the unoccluded NEE term -- the order of
// the adds above.
// (in LDS by thread, so that it does not hold registers through the rest of
// the vertex)
ND float *nee_em_lds() {
    __shared__ float s_emt[3 * kSeg];
    return s_emt;
}
template <bool ATOMIC, bool INL>
ND void rec_add(const DevScene &S, float4 *rec, PathState &ps, ShadowOut &so, const V3 &a0) {
    const V3 a = chan_only(S, ps.chan, a0);
    if (!ATOMIC) {
        ps.L = ps.L + a;
        return;
    }
    if (INL && S.nee_inline) {
        float *const e = nee_em_lds() + 3 * threadIdx.x;
        e[0] = a.x;
        e[1] = a.y;
        e[2] = a.z;
        so.has_em = true;
        return;
    }
    float *r = reinterpret_cast<float *>(rec + ps.work);
    atomicAdd(r + 0, a.x);
    atomicAdd(r + 1, a.y);
    atomicAdd(r + 2, a.z);
}

// Deviation D10: a mirror or dielectric BSDF evaluates to exactly zero, so
// the NEE term at such a vertex, attenuation * w_ems * 0 * theta * Li, is zero
// whenever its other factors are finite.  Then only its three random numbers
// (emitter choice, 2D light sample) are drawn and no light is sampled: RR and
// the BSDF sample read the same stream positions, the image is bit-identical.
// Kept in full when the attenuation is not finite or the scene has an
// environment map (its Li can be inf/NaN, which the reference turns into an
// invalid sample); for area/point lights Li is finite unless the vertex
// coincides exactly with the sampled light point.
ND bool skip_nee(const DevScene &S, const DevBsdf &B, const V3 &beta) {
    return S.skip_discrete_nee && (B.type == NORI_BSDF_MIRROR || B.type == NORI_BSDF_DIELECTRIC) &&
           isfinite(beta.x) && isfinite(beta.y) && isfinite(beta.z);
}

// One iteration of VolumetricIntegrator::Li (volumetric.cpp:18-156) for the
// current segment (ps.o, ps.d) and its closest hit h (prim ~0: none, t = inf).
// Free flight first: a scattering event does phase-function NEE with
// transmittance, Russian roulette at 0.8 and a uniform-sphere bounce; else
// the surface vertex does path_mis-style emission and NEE, both weighted by
// transmittance.  ps.prev carries the pdf for w_mats at the next emitter hit
// (1/4pi after a scattering event, -1 after a discrete lobe).
template <bool ATOMIC, bool FULL = true>
ND bool shade_vertex_vol(const DevScene &S, PathState &ps, const float4 &h, float4 *rec, ShadowOut &so) {
    so.emit = false;
    so.has_em = false;
    const uint32_t prim = __float_as_uint(h.y);
    const bool inter = prim != 0xFFFFFFFFu;
    SurfHit hs;
    float tmax = INF_F;
    if (inter) {
        hs = surface<FULL>(S, prim, h.x, h.z, h.w, ps.o, ps.d);
        tmax = norm(hs.p - ps.o);
    }
    V3 mp;
    if (medium_sample(S, ps.o, ps.d, ps.rng, tmax, mp)) {
        const V3 wo = sq_uniform_sphere(next2D(ps.rng));
        const float pdf_mat = kInvFourPi;
        NeeSample ne = nee_sample<FULL>(S, mp, ps.rng);
        ps.beta = ps.beta * V3{S.albedo[0], S.albedo[1], S.albedo[2]};
        const V3 tr = medium_tr(S, mp, ne.p);
        so.contrib = chan_only(S, ps.chan, ((ps.beta * tr) * ne.Li) * pdf_mat);
        so.emit = !is_zero(so.contrib);
        so.o = mp;
        so.d = ne.wi;
        so.maxt = ne.maxt;
        so.work = ps.work;
        const float q = smin(ps.beta.x, 0.80f);
        if (next1D(ps.rng) > q) return false;
        ps.beta = ps.beta / q;
        ps.o = mp;
        ps.d = normalize(wo);
        ps.mint = kEps;
        ps.maxt = INF_F;
        ps.prev = pdf_mat;
        return true;
    }
    if (!inter) return false;  // escaped (volumetric.cpp: break)
    const DevShape &sh = S.shapes[hs.shape];
    const DevBsdf &B = S.bsdfs[sh.bsdf];
    if (sh.emitter >= 0) {
        const DevEmitter &E = S.emitters[sh.emitter];
        const V3 wi = normalize(hs.p - ps.o);
        const V3 Le = emitter_eval<FULL>(S, E, hs.sh.n, wi);
        float w = 1.0f;
        if (ps.prev >= 0.0f) {
            const float pe = emitter_pdf<FULL>(S, E, hs.sh.n, wi);
            w = ps.prev + pe > 0.f ? ps.prev / (ps.prev + pe) : ps.prev;
        }
        const V3 Ladd = ((ps.beta * w) * Le) * medium_tr(S, hs.p, hs.p);
        rec_add<ATOMIC, !FULL || kNeeFull>(S, rec, ps, so, Ladd);
    }
    if (skip_nee(S, B, ps.beta)) {
        pcg_skip(ps.rng, 3);
    } else {
        NeeSample ne = nee_sample<FULL>(S, hs.p, ps.rng);
        BRec br;
        br.wi = to_local(hs.sh, -ps.d);
        br.uv = hs.uv;
        br.wo = to_local(hs.sh, ne.wi);
        br.measure = kMeasureSolidAngle;
        const float theta = smax(0.0f, br.wo.z);
        const V3 f = bsdf_eval<FULL>(B, br);
        const float pdf_mat = bsdf_pdf<FULL>(B, br);
        const float w_ems = (pdf_mat + ne.pdf_em) > 0.0f ? ne.pdf_em / (pdf_mat + ne.pdf_em) : ne.pdf_em;
        const V3 tr = medium_tr(S, hs.p, ne.p);
        so.contrib = chan_only(S, ps.chan, ((((ps.beta * w_ems) * f) * theta) * ne.Li) * tr);
        so.emit = !is_zero(so.contrib);
        so.o = hs.p;
        so.d = ne.wi;
        so.maxt = ne.maxt;
        so.work = ps.work;
    }
    const float q = smin(ps.beta.x, 0.80f);
    if (next1D(ps.rng) > q) return false;
    ps.beta = ps.beta / q;
    BRec br;
    br.wi = to_local(hs.sh, -ps.d);
    br.uv = hs.uv;
    br.wo = V3{0, 0, 1};
    br.measure = kMeasureUnknown;
    const V3 w = bsdf_sample<FULL>(B, br, next2D(ps.rng));
    if (is_zero(w)) return false;  // deviation D1
    ps.beta = ps.beta * w;
    const float pm = bsdf_pdf<FULL>(B, br);
    ps.prev = br.measure == kMeasureDiscrete ? -1.0f : pm;
    ps.o = hs.p;
    ps.d = to_world(hs.sh, br.wo);
    ps.mint = kEps;
    ps.maxt = INF_F;
    return true;
}

// One vertex of PathMisIntegrator::Li (path_mis.cpp:32-97) or
// PathMatsIntegrator::Li (path_mats.cpp:26-57) given the closest hit of the
// current ray.  Returns true if the path continues (ps holds the new ray).
template <int INTEG, bool ATOMIC, bool FULL = true>
ND bool shade_vertex(const DevScene &S, PathState &ps, const float4 &h, float4 *rec, ShadowOut &so) {
    if constexpr (INTEG == NORI_INTEGRATOR_VOLUMETRIC) return shade_vertex_vol<ATOMIC, FULL>(S, ps, h, rec, so);
    so.emit = false;
    so.has_em = false;
    uint32_t prim = __float_as_uint(h.y);
    if (prim == 0xFFFFFFFFu) return false;  // escaped: path_mis.cpp:84-85
    constexpr bool MIS = INTEG == NORI_INTEGRATOR_PATH_MIS;
    SurfHit hs = surface<FULL>(S, prim, h.x, h.z, h.w, ps.o, ps.d);
    const DevShape &sh = S.shapes[hs.shape];
    const DevBsdf &B = S.bsdfs[sh.bsdf];
    if (sh.emitter >= 0) {  // emission (path_mis.cpp:35-39, path_mats.cpp:31-35)
        const DevEmitter &E = S.emitters[sh.emitter];
        V3 wi = normalize(hs.p - ps.o);
        V3 Le = emitter_eval<FULL>(S, E, hs.sh.n, wi);
        V3 Ladd;
        if (MIS) {
            float w = 1.0f;  // w_mats (path_mis.cpp:87-97)
            if (ps.prev >= 0.0f) {
                float pe = emitter_pdf<FULL>(S, E, hs.sh.n, wi);
                w = ps.prev + pe > 0.f ? ps.prev / (ps.prev + pe) : ps.prev;
            }
            Ladd = (ps.beta * w) * Le;
        } else {
            Ladd = ps.beta * Le;
        }
        rec_add<ATOMIC, !FULL || kNeeFull>(S, rec, ps, so, Ladd);
    }
    if (MIS && skip_nee(S, B, ps.beta)) {
        pcg_skip3(ps.rng);  // deviation D10: the three NEE draws, unused
    } else if (MIS) {  // next-event estimation (path_mis.cpp:42-61)
        const NeeSample ne = nee_sample<FULL>(S, hs.p, ps.rng);
        BRec br;
        br.wi = to_local(hs.sh, -ps.d);
        br.uv = hs.uv;
        br.wo = to_local(hs.sh, ne.wi);
        br.measure = kMeasureSolidAngle;
        float theta = smax(0.0f, br.wo.z);
        V3 f = bsdf_eval<FULL>(B, br);
        float pdf_mat = bsdf_pdf<FULL>(B, br);
        float w_ems = (pdf_mat + ne.pdf_em) > 0.0f ? ne.pdf_em / (pdf_mat + ne.pdf_em) : ne.pdf_em;
        so.contrib = chan_only(S, ps.chan, (((ps.beta * w_ems) * f) * theta) * ne.Li);
        so.emit = !is_zero(so.contrib);  // a zero contribution adds nothing (NaN still goes)
        so.o = hs.p;
        so.d = ne.wi;
        so.maxt = ne.maxt;
        so.work = ps.work;
    }
    // Russian roulette on the red channel (path_mis.cpp:64-69)
    float qrr = smin(ps.beta.x, 0.99f);
    if (next1D(ps.rng) > qrr) return false;
    ps.beta = ps.beta / qrr;
    BRec br;
    br.wi = to_local(hs.sh, -ps.d);
    br.uv = hs.uv;
    br.wo = V3{0, 0, 1};
    br.measure = kMeasureUnknown;
    V3 w = bsdf_sample<FULL>(B, br, next2D(ps.rng));
    if (is_zero(w)) return false;  // deviation D1: zero-weight samples end the path
    ps.beta = ps.beta * w;
    if (MIS) {
        float pm = bsdf_pdf<FULL>(B, br);
        ps.prev = br.measure == kMeasureDiscrete ? -1.0f : pm;
    }
    ps.o = hs.p;
    ps.d = to_world(hs.sh, br.wo);
    ps.mint = kEps;
    ps.maxt = INF_F;
    return true;
}

// shade_vertex at a vertex of a solitary, non-emitting dielectric sphere
// whose next-event estimation is skipped (skip_nee: deviation D10), reduced
// to the operations that run there -- the same arithmetic in the same order
// (surface(): hit point, normal, frame; the three skipped NEE draws; Russian
// roulette; Dielectric::sample; the discrete pdf) without the plugin
// dispatch: the tail finisher's trapped glass-sphere paths run a chain of
// these.  t: the chord's closest hit.  Returns false if the path ends.
// NORI_GLASS_FAST_SQRT=1: sqrt_rn (range-checked fast sqrt) in the glass
// chain instead of the IEEE sequence -- its branch costs more than it saves
// for a lone lane (958-965 against 1026-1049 ns per chord bounce, round 6).
#ifndef NORI_GLASS_FAST_SQRT
#define NORI_GLASS_FAST_SQRT 0
#endif
constexpr bool kGlassFast = NORI_GLASS_FAST_SQRT;
#ifndef NORI_GLASS_STEP  // 0: every chord bounce through glass_bounce / chord_hit
#define NORI_GLASS_STEP 1
#endif
constexpr bool kGlassStep = NORI_GLASS_STEP;
template <int INTEG>
ND bool glass_bounce(const DevShape &sh, const DevBsdf &B, PathState &ps, float t) {
    const V3 p = ps.o + ps.d * t;
    const Frame f = frame_from<kGlassFast>(normalize<kGlassFast>(p - V3{sh.center[0], sh.center[1], sh.center[2]}));
    if (INTEG == NORI_INTEGRATOR_PATH_MIS) pcg_skip3(ps.rng);
    const float qrr = smin(ps.beta.x, 0.99f);
    if (next1D(ps.rng) > qrr) return false;
    ps.beta = ps.beta / qrr;  // (times the sample weight 1, exactly)
    const V3 wo = dielectric_wo<kGlassFast>(B, to_local(f, -ps.d), next2D(ps.rng));
    if (INTEG == NORI_INTEGRATOR_PATH_MIS) ps.prev = -1.0f;  // discrete measure
    ps.o = p;
    ps.d = to_world(f, wo);
    ps.mint = kEps;
    ps.maxt = INF_F;
    return true;
}

// One chord bounce of a path trapped in a solitary dielectric sphere, as
// straight-line code: glass_bounce at the chord's end t followed by the next
// chord (chord_hit), with every early-out of the reference's functions turned
// into a select -- the same operations in the same order on the same values
// (surface(): hit point, normal, coordinateSystem frame; the three skipped
// NEE draws; Russian roulette; fresnel; the reflected direction; the sphere
// test of the next chord with the adaptive epsilon).  A lone lane pays for
// every branch of the general code in exec-mask switches (the chain is its
// dependent latency: ~1 us per bounce), so the common case -- the ray is
// reflected back inside and hits the sphere again -- runs here; true (and
// ps, t updated) only in that case.  Otherwise nothing is changed and the
// caller runs the bounce through glass_bounce / chord_hit, which produce the
// refraction, the Russian-roulette end or the exit.  (sqrtf and the
// divisions are the IEEE sequences: the range-checked fast forms' branches
// measured slower here)
template <int INTEG>
ND bool glass_step(const DevShape &sh, const DevBsdf &B, PathState &ps, float &t) {
    const V3 c = V3{sh.center[0], sh.center[1], sh.center[2]};
    const V3 p = ps.o + ps.d * t;
    const V3 n = normalize(p - c);
    // frame_from(n) (frame.h:49-51, common.cpp:274-283) with the branch as selects
    const bool bx = fabsf(n.x) > fabsf(n.y);
    const float a = bx ? n.x : n.y;
    const float invLen = 1.0f / sqrtf(a * a + n.z * n.z);  // == rcp_full(), without its range branch
    Frame f;
    f.n = n;
    f.t = bx ? V3{n.z * invLen, 0.0f, -n.x * invLen} : V3{0.0f, n.z * invLen, -n.y * invLen};
    f.s = cross(f.t, n);
    Pcg rng = ps.rng;
    if (INTEG == NORI_INTEGRATOR_PATH_MIS) pcg_skip3(rng);
    const float qrr = smin(ps.beta.x, 0.99f);
    const bool survive = !(next1D(rng) > qrr);
    const V3 beta = ps.beta / qrr;
    const V3 wi = to_local(f, -ps.d);
    const V2 s2 = next2D(rng);
    // fresnel(wi.z, ext, int) (common.cpp:285-314) with its branches as selects
    const bool inside = wi.z < 0.0f;
    const float etaI = inside ? B.int_ior : B.ext_ior, etaT = inside ? B.ext_ior : B.int_ior;
    const float eta = inside ? B.eta_ie : B.eta_ei, ci = inside ? -wi.z : wi.z;
    const float sin2 = eta * eta * (1 - ci * ci);
    const float ct = sqrtf(1.0f - sin2);
    const float Rs = (etaI * ci - etaT * ct) / (etaI * ci + etaT * ct);
    const float Rp = (etaT * ci - etaI * ct) / (etaT * ci + etaI * ct);
    const float F = B.ext_ior == B.int_ior ? 0.0f : (sin2 > 1.0f ? 1.0f : (Rs * Rs + Rp * Rp) / 2.0f);
    const bool reflect = F > s2.x;  // Dielectric::sample's reflection: wo = (-wi.x, -wi.y, wi.z)
    const V3 d = to_world(f, V3{-wi.x, -wi.y, wi.z});
    // the next chord: chord_hit (sphere_hit_nb with the adaptive epsilon, bvh.cpp:412-418)
    TRay r;
    r.o = p;
    r.d = d;
    r.mint = smax(kEps, kEps * smax(smax(fabsf(p.x), fabsf(p.y)), fabsf(p.z)));
    r.maxt = INF_F;
    float tn;
    const bool hit = sphere_hit_nb(make_float4(c.x, c.y, c.z, 0.0f), make_float4(sh.radius, 0.0f, 0.0f, 0.0f), r, tn);
    // path_mis: the next vertex's NEE must still be skippable (skip_nee: a
    // finite throughput), else the caller's general bounce takes over
    const bool fin = INTEG != NORI_INTEGRATOR_PATH_MIS || (isfinite(beta.x) && isfinite(beta.y) && isfinite(beta.z));
    if (!(survive && reflect && hit && fin)) return false;
    ps.rng = rng;
    ps.beta = beta;
    if (INTEG == NORI_INTEGRATOR_PATH_MIS) ps.prev = -1.0f;  // discrete measure
    ps.o = p;
    ps.d = d;
    ps.mint = kEps;
    ps.maxt = INF_F;
    t = tn;
    return true;
}

// New camera sample for work id w (render.cpp:98-126 + independent.cpp).
// pix = wd.pixels[w mod M], loaded by the caller (early: a load issued
// after the path stores would wait for them too -- vmcnt counts in order)
template <bool FULL = true>
ND void regen_path(const DevScene &S, const WorkDesc &wd, uint32_t w, uint32_t pix, PathState &ps, float4 *rec) {
    uint32_t pass = w / wd.M;
    uint32_t W = (uint32_t)S.W;
    uint32_t y = pix / W, x = pix - y * W;
    uint64_t sid = (uint64_t)(wd.pass_begin + pass) * ((uint64_t)S.W * (uint64_t)S.H) + pix;
    wave_seed(ps.rng, wd.seed, sid);
    V2 jit = next2D(ps.rng);
    const V2 ap = next2D(ps.rng);  // apertureSample (render.cpp:99)
    camera_sample<FULL>(S, (float)x + jit.x, (float)y + jit.y, ap, -1, ps.o, ps.d, ps.mint, ps.maxt, &ps.invz);
    ps.cam = true;
    ps.chan = 0;
    ps.beta = V3{1, 1, 1};
    ps.prev = -1.0f;
    ps.work = w;
    rec[w] = make_float4(0, 0, 0, rec_code(S.jit_lk, S.border, x, y, jit));
}

// Chromatic aberration: channel ps.chan's Li has ended, so the sample goes on
// with the next channel's camera ray (render.cpp:106-121: the three rays share
// the pixel and aperture samples, their Li calls consume the sampler in turn,
// so the pcg32 state simply continues).
template <bool FULL = true>
ND void next_channel(const DevScene &S, const WorkDesc &wd, PathState &ps) {
    const uint32_t pass = ps.work / wd.M, pix = wd.pixels[ps.work - pass * wd.M];
    const uint32_t W = (uint32_t)S.W, y = pix / W, x = pix - y * W;
    Pcg r;
    wave_seed(r, wd.seed, (uint64_t)(wd.pass_begin + pass) * ((uint64_t)S.W * (uint64_t)S.H) + pix);
    const V2 jit = next2D(r);
    const V2 ap = next2D(r);
    ps.chan += 1;
    camera_sample<FULL>(S, (float)x + jit.x, (float)y + jit.y, ap, (int)ps.chan, ps.o, ps.d, ps.mint, ps.maxt, &ps.invz);
    ps.cam = true;
    ps.beta = V3{1, 1, 1};
    ps.prev = -1.0f;
}

#ifndef NORI_SHADE_WAVES
#define NORI_SHADE_WAVES 5
#endif
// S.nee_inline: one LDS slot per vertex that adds to its record (a shadow ray
// and/or emission), over the blob: (o, maxt), (d, work | flags),
// (contrib, the owner thread, whose emission is in nee_em_lds)
constexpr uint32_t kNeeSlotBytes = kSeg * 3 * 16;
constexpr uint32_t kSlotEmit = 1u << 31, kSlotEm = 1u << 30;  // above kWorkMask
#ifndef NORI_SORT_OCTANT
#define NORI_SORT_OCTANT 1
#endif
// lds_bytes != 0: the scene blob is staged into LDS first, so the chains of
// dependent table reads of a vertex (shape -> bsdf -> vertices -> light CDF)
// run at LDS instead of L2 latency.
// LDS is a template parameter, not a run-time choice: with the scene pointers
// known to point into LDS the compiler emits ds_read for the table reads; a
// run-time select between the LDS and the global tables leaves generic
// pointers, i.e. flat loads (vector-memory latency, both wait counters).
template <int INTEG, bool LDS, int VAR>
__global__ __launch_bounds__(kShadeBlock) __attribute__((amdgpu_waves_per_eu(NORI_SHADE_WAVES)))
void k_shade(DevScene Sg, PathQueue in, PathQueue out, ShadowQueue sq, SegState seg, int in_sel, WorkDesc wd,
             float4 *rec, Counters *C, uint32_t lds_bytes) {
    static_assert(kShadeBlock == kSeg, "one shade thread per segment slot");
    // VAR: 0 basic plugins only (FULL = false), 1 full, 2 full + chromatic
    // aberration (the per-channel continuation is compiled in only then)
    constexpr bool FULL = VAR != 0, CHROMA = VAR == 2;
    __shared__ uint32_t s_sh[kShadeBlock / 64], s_al[kShadeBlock / 64], s_em[kShadeBlock / 64], s_w[kSeg], s_pix[kSeg];
#if NORI_SORT_OCTANT
    __shared__ uint32_t s_oc[8 * (kShadeBlock / 64)];
    const bool sort_octant = Sg.num_nodes > 0 && Sg.blob_bytes == 0;  // BVH-traversed scenes only
#endif
    extern __shared__ __attribute__((aligned(16))) float4 blob_lds[];
    const uint32_t b = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, q = b * kSeg + tid;
#ifdef NORI_PROF_SHADE  // profiling build: clocks of the kernel's phases, summed over waves
    uint64_t pt[6] = {0, 0, 0, 0, 0, 0}, pc = __builtin_amdgcn_s_memtime();
#define NORI_SPHASE(i)                                       \
    {                                                        \
        const uint64_t now = __builtin_amdgcn_s_memtime();   \
        pt[i] += now - pc;                                   \
        pc = now;                                            \
    }
#else
#define NORI_SPHASE(i)
#endif
    // every load the work-group needs is issued up front, so their latencies
    // overlap instead of adding up: the segment's bookkeeping (scalar), and
    // the path entries whether or not they hold a path (a queue slot beyond
    // the count is stale but allocated; nothing reads its values)
    const uint32_t n_in = seg.cnt[in_sel][b];
    const uint32_t cursor = seg.cursor[b];
    const uint4 st0 = seg.stats[b];
    PathState ps;
    load_path(Sg, wd, in, q, ps);
    const float4 hit = in.hit[q];
    // The next kSeg positions of the segment's work stream and their pixels:
    // slot j of the free slots regenerates position cursor + j.  Looked up
    // here, beside the path loads, and parked in LDS; a lookup after the
    // compaction would wait for every store and atomic issued before it
    // (vmcnt counts in issue order).  Work ids < 2^31 (runtime chunking).
    const uint64_t wspec = stream_work(wd, wd.b0 + b, cursor + tid);
    const uint32_t pspec = wspec < wd.total ? wd.pixels[(uint32_t)wspec % wd.M] : 0u;
    DevScene S = Sg;
    if constexpr (LDS) {
        for (uint32_t i = tid; i < lds_bytes / 16; i += kShadeBlock) blob_lds[i] = Sg.blob[i];
        __syncthreads();
        S = scene_in_lds(Sg, reinterpret_cast<const char *>(blob_lds));
    }
    NORI_SPHASE(0)
    ShadowOut so;
    so.emit = false;
    so.has_em = false;
    bool alive = false;
#ifdef NORI_PROF_SHADE
    __builtin_amdgcn_s_waitcnt(0);  // path loads landed: phase 1 is the shading proper
    NORI_SPHASE(0)
#endif
    if (tid < n_in) {
        alive = shade_vertex<INTEG, true, FULL>(S, ps, hit, rec, so);
        ps.cam = false;  // a survivor carries its BSDF-sampled ray (Epsilon, inf)
        if (CHROMA && !alive && ps.chan < 2) {  // the sample's next colour channel
            next_channel<FULL>(Sg, wd, ps);
            alive = true;
        }
    }
    NORI_SPHASE(1)
    s_w[tid] = wspec < wd.total ? (uint32_t)wspec : ~0u;
    s_pix[tid] = pspec;
    // ---- compaction: survivors first (in lane order), shadow rays likewise
    // (S.nee_inline: the vertices that add to their record -- a shadow ray
    // and/or emission -- into the LDS slots)
    const bool nee_in = (!FULL || kNeeFull) && Sg.nee_inline != 0;
    const bool key = so.emit || so.has_em;  // (has_em only with nee_in)
    const uint64_t mal = __ballot(alive), msh = __ballot(key), mem = __ballot(so.emit);
    if (lane_id() == 0) {
        s_al[wave] = (uint32_t)__popcll(mal);
        s_sh[wave] = (uint32_t)__popcll(msh);
        s_em[wave] = (uint32_t)__popcll(mem);
    }
    __syncthreads();
    NORI_SPHASE(2)
    uint32_t al_off = rank_in(mal), sh_off = rank_in(msh), al_tot = 0, sh_tot = 0, em_tot = 0;
    for (uint32_t w = 0; w < kShadeBlock / 64; ++w) {
        al_off += w < wave ? s_al[w] : 0u;
        sh_off += w < wave ? s_sh[w] : 0u;
        al_tot += s_al[w];
        sh_tot += s_sh[w];
        em_tot += s_em[w];
    }
#if NORI_SORT_OCTANT
    // survivors grouped by the octant of their new direction (then lane
    // order), so the waves of the BVH extension kernel get rays that visit
    // a node's children in the same order
    if (sort_octant) {
        const uint32_t oct = (ps.d.x < 0.0f ? 1u : 0u) | (ps.d.y < 0.0f ? 2u : 0u) | (ps.d.z < 0.0f ? 4u : 0u);
        uint32_t mine = 0;
        for (uint32_t o = 0; o < 8; ++o) {
            const uint64_t m = __ballot(alive && oct == o);
            if (lane_id() == 0) s_oc[o * (kShadeBlock / 64) + wave] = (uint32_t)__popcll(m);
            if (alive && oct == o) mine = rank_in(m);
        }
        __syncthreads();
        if (alive) {
            uint32_t off = mine;
            for (uint32_t o = 0; o < 8; ++o)
                for (uint32_t w = 0; w < kShadeBlock / 64; ++w)
                    off += (o < oct || (o == oct && w < wave)) ? s_oc[o * (kShadeBlock / 64) + w] : 0u;
            al_off = off;
        }
    }
#endif
    const uint32_t need_tot = kSeg - al_tot;
    // (the slots overlay the blob: the compaction's barrier above ends every
    // read of it -- regeneration and the scan below read the global tables)
    float4 *const s_sa = blob_lds, *const s_sb = s_sa + kSeg, *const s_sc = s_sb + kSeg;
    if (nee_in && key) {
        s_sa[sh_off] = make_float4(so.o.x, so.o.y, so.o.z, so.maxt);
        s_sb[sh_off] = make_float4(so.d.x, so.d.y, so.d.z,
                                   __uint_as_float(ps.work | (so.emit ? kSlotEmit : 0u) | (so.has_em ? kSlotEm : 0u)));
        s_sc[sh_off] = make_float4(so.contrib.x, so.contrib.y, so.contrib.z, __uint_as_float(tid));
    } else if (so.emit) {
        uint32_t i = b * kSeg + sh_off;
        sq.ray_o[i] = make_float4(so.o.x, so.o.y, so.o.z, kEps);
        sq.ray_d[i] = make_float4(so.d.x, so.d.y, so.d.z, so.maxt);
        sq.payload[i] = make_float4(so.contrib.x, so.contrib.y, so.contrib.z, __uint_as_float(so.work));
    }
    if (alive) store_path(out, b * kSeg + al_off, ps);
    NORI_SPHASE(3)
    // ---- regeneration: the free slots [al_tot, kSeg) take the next work ids of
    // the segment's stream, so only the tail waves run the camera-ray code and
    // a wave's new samples are adjacent pixels (stream_work increases with p)
    if (tid >= al_tot) {
        const uint32_t wn = s_w[tid - al_tot];
        if (wn != ~0u) {
            PathState np;
            regen_path<FULL>(Sg, wd, wn, s_pix[tid - al_tot], np, rec);
            store_path(out, q, np);
        }
    }
    if (nee_in) {
        // slot j = thread j (dense waves): the record is read first, so its
        // latency hides behind the scan; the shadow ray's any hit through the
        // wave-uniform scan, as k_shadow_scan; then the record += emission,
        // += the unoccluded NEE term, in the order of the separate kernels
        __syncthreads();
        if (wave * 64u < sh_tot) {
            const bool mine = tid < sh_tot;
            const uint32_t j = mine ? tid : 0u;
            const float4 a = s_sa[j], d = s_sb[j], c = s_sc[j];
            const uint32_t bits = __float_as_uint(d.w), work = bits & kWorkMask;
            const bool emit = mine && (bits & kSlotEmit) != 0u, hem = mine && (bits & kSlotEm) != 0u;
            float4 L = make_float4(0.f, 0.f, 0.f, 0.f);
            if (mine) L = rec[work];
            bool f[1] = {false};
            if (__any(emit)) {
                TRay r[1];
                r[0].o = ld3(a);
                r[0].d = ld3(d);
                r[0].mint = kEps;
                r[0].maxt = a.w;
                bool live[1] = {emit};
                float t[1], u[1], v[1];
                uint32_t p[1];
                scan_rays<1, true>(Sg, r, live, t, p, u, v, f);
            }
            bool add = false;
            if (hem) {
                const float *e = nee_em_lds() + 3 * __float_as_uint(c.w);
                L.x += e[0];
                L.y += e[1];
                L.z += e[2];
                add = true;
            }
            if (emit && !f[0]) {
                L.x += c.x;
                L.y += c.y;
                L.z += c.z;
                add = true;
            }
            if (add) rec[work] = L;
        }
    }
    NORI_SPHASE(4)
#ifdef NORI_PROF_SHADE
    __builtin_amdgcn_s_waitcnt(0);
    NORI_SPHASE(5)
    if (lane_id() == 0 && (b & 15) == 0) {  // a sample of the waves (atomics on one line)
        for (int i = 0; i < 6; ++i) atomicAdd(&C->prof[i], (unsigned long long)pt[i]);
        atomicAdd(&C->prof[6], 1ull);
    }
#endif
#undef NORI_SPHASE
    if (tid == 0) {
        // new samples = the prefix of [cursor, cursor + need_tot) still inside the stream
        uint32_t lo = 0, hi = need_tot;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (stream_work(wd, wd.b0 + b, cursor + mid) < wd.total) lo = mid + 1;
            else hi = mid;
        }
        const uint32_t fresh_tot = lo;
        seg.cnt[in_sel ^ 1][b] = al_tot + fresh_tot;
        seg.shcnt[b] = nee_in ? 0u : sh_tot;  // (inline: traced above)
        seg.cursor[b] = cursor + need_tot;
        seg.stats[b] = make_uint4(st0.x + al_tot + fresh_tot, st0.y + em_tot, st0.z + fresh_tot, st0.w);
        if (stream_work(wd, wd.b0 + b, cursor) < wd.total && stream_work(wd, wd.b0 + b, cursor + need_tot) >= wd.total) {
            // the last segment to run dry tells the host (system-scope store to
            // host-mapped memory) -- no per-iteration readback is needed
            uint32_t n = atomicAdd(&C->exhausted, 1u) + 1u;
            // progress hint: plain system-scope store (no PCIe atomics needed),
            // every 64th exhausted segment only (a store to host memory per
            // segment slowed the last iterations measurably)
            if ((n & 63u) == 0u) __hip_atomic_store(wd.done_flag + 1, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (n == wd.G) __hip_atomic_store(wd.done_flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// ImageBlock::put(pos, val) (block.cpp:93-122) of one sample straight into
// the film, with the block-relative coordinates of the sample's own block so
// the filter weights round exactly as in k_splat.
ND void splat_sample(const DevScene &S, float *film, Counters *C, uint32_t x, uint32_t y, V2 jit, float4 L,
                     float *var) {
    if (L.x < 0 || !isfinite(L.x) || L.y < 0 || !isfinite(L.y) || L.z < 0 || !isfinite(L.z)) {
        atomicAdd(&C->invalid, 1ull);
        return;
    }
    if (var) {  // the pixel's sample statistics (nori_gpu_render_desc.variance_out)
        float *v = var + 8 * ((size_t)y * S.W + x);
        atomicAdd(v + 0, L.x);
        atomicAdd(v + 1, L.y);
        atomicAdd(v + 2, L.z);
        atomicAdd(v + 3, L.x * L.x);
        atomicAdd(v + 4, L.y * L.y);
        atomicAdd(v + 5, L.z * L.z);
        atomicAdd(v + 6, 1.0f);
    }
    const int B = S.border, TS = NORI_BLOCK_SIZE + 2 * B, FW = S.W + 2 * B;
    const int ox = (int)(x / NORI_BLOCK_SIZE) * NORI_BLOCK_SIZE, oy = (int)(y / NORI_BLOCK_SIZE) * NORI_BLOCK_SIZE;
    const float rad = S.filter_radius, lk = S.lookup;
    float px = ((float)x + jit.x) - 0.5f - (float)(ox - B), py = ((float)y + jit.y) - 0.5f - (float)(oy - B);
    int x0 = max((int)ceilf(px - rad), 0), y0 = max((int)ceilf(py - rad), 0);
    int x1 = min((int)floorf(px + rad), TS - 1), y1 = min((int)floorf(py + rad), TS - 1);
    for (int cy = y0; cy <= y1; ++cy) {
        float wy = S.filter[min((int)(fabsf((float)cy - py) * lk), NORI_FILTER_RESOLUTION)];
        for (int cx = x0; cx <= x1; ++cx) {
            float wx = S.filter[min((int)(fabsf((float)cx - px) * lk), NORI_FILTER_RESOLUTION)];
            float *f = film + 4 * ((size_t)(oy + cy) * FW + (ox + cx));
            float a = (L.x * wx) * wy, b = (L.y * wx) * wy, c = (L.z * wx) * wy, w = (1.0f * wx) * wy;
            if (w != 0.0f || a != 0.0f || b != 0.0f || c != 0.0f) {
                atomicAdd(f + 0, a);
                atomicAdd(f + 1, b);
                atomicAdd(f + 2, c);
                atomicAdd(f + 3, w);
            }
        }
    }
}

#if NORI_TU == 0
// Pending marker for the samples the finisher will splat itself.
__global__ __launch_bounds__(kTraceBlock) void k_mark(PathQueue Q, SegState seg, int sel, float4 *rec) {
    const uint32_t sg = blockIdx.x >> 1, idx = (blockIdx.x & 1) * kTraceBlock + threadIdx.x;
    if (idx >= seg.cnt[sel][sg]) return;
    rec[__float_as_uint(Q.ray_d[sg * kSeg + idx].w) & kWorkMask].w = __uint_as_float(kRecPending);
}

#endif
// Cooperative scan (scan-mode scenes, n <= 64 primitives): the rays of the
// lanes in `want` are traced one after another by the whole wave, lane l
// testing primitive l against the broadcast ray.  The result is exactly that
// of traverse<0, ANY> for the ray: every candidate passes the test against the
// ray's own maxt, the closest wins, and among equal t the last primitive in
// scan order wins (the `t <= maxt` update).  A lone tail path then pays one
// primitive test per ray instead of n.
struct CoopPrim {  // lane l's primitive, loaded once per finisher wave
    float4 p0, p1, p2;  // p2.w: leaf-order position (the tie rule of scan_core)
    bool has, tri;
};
ND CoopPrim coop_load(const DevScene &S) {
    CoopPrim c;
    const uint32_t lane = lane_id();
    c.has = lane < S.num_prims;
    c.p0 = c.p1 = c.p2 = make_float4(0, 0, 0, 0);
    if (c.has) {
        const float4 *pp = S.prims + 3 * (size_t)lane;
        c.p0 = pp[0];
        c.p1 = pp[1];
        c.p2 = pp[2];
    }
    c.tri = __float_as_uint(c.p1.w) == 0u;
    return c;
}
template <bool ANY>
ND bool coop_scan(const DevScene &S, const CoopPrim &cp, const TRay &mine, bool want, float &t, uint32_t &p, float &u,
                  float &v) {
    const uint32_t lane = lane_id();
    const float4 rmn = make_float4(S.root_min[0], S.root_min[1], S.root_min[2], 0.f);
    const float4 rmx = make_float4(S.root_max[0], S.root_max[1], S.root_max[2], 0.f);
    bool res = false;
    t = INF_F;
    p = 0xFFFFFFFFu;
    u = v = 0.0f;
    auto bcast = [](float x, int j) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), j)); };
    uint64_t m = __ballot(want);
    while (m) {
        const int j = __builtin_ctzll(m);
        m &= m - 1;
        TRay r;
        r.o = V3{bcast(mine.o.x, j), bcast(mine.o.y, j), bcast(mine.o.z, j)};
        r.d = V3{bcast(mine.d.x, j), bcast(mine.d.y, j), bcast(mine.d.z, j)};
        r.mint = bcast(mine.mint, j);
        r.maxt = bcast(mine.maxt, j);
        if (r.mint == kEps) r.mint = smax(r.mint, r.mint * smax(smax(fabsf(r.o.x), fabsf(r.o.y)), fabsf(r.o.z)));
        r.rcp = V3{rcp_full(r.d.x), rcp_full(r.d.y), rcp_full(r.d.z)};
        float tn;
        const bool live = !(r.maxt < r.mint) && box_test(rmn, rmx, r, tn);
        float tl = 0, ul = 0, vl = 0;
        bool hl = false;
        if (cp.has) hl = cp.tri ? tri_hit_nb(cp.p0, cp.p1, cp.p2, r, tl, ul, vl) : sphere_hit_nb(cp.p0, cp.p1, r, tl);
        uint64_t hm = __ballot(hl && live);
        if (ANY) {
            if ((int)lane == j) res = hm != 0ull;
            continue;
        }
        if (!hm) continue;
        // closest hit over the (few) hitting lanes, the later leaf-order
        // position among equal t (scan_core's rule); t > 0, so its bits order
        // like the value and the comparison stays scalar
        uint32_t best = 0xFFFFFFFFu, best_pos = 0;
        int w = 0;
        do {
            const int l = __builtin_ctzll(hm);
            hm &= hm - 1;
            const uint32_t tb = (uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(tl + 0.0f), l);
            const uint32_t pos = (uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(cp.p2.w), l);
            if (tb < best || (tb == best && pos >= best_pos)) {
                best = tb;
                best_pos = pos;
                w = l;
            }
        } while (hm);
        const float tw = __uint_as_float(best), uw = bcast(cp.tri ? ul : 0.0f, w), vw = bcast(cp.tri ? vl : 0.0f, w);
        const uint32_t pw = (uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(cp.p0.w), w);
        if ((int)lane == j) {
            res = true;
            t = tw;
            p = pw;
            u = uw;
            v = vw;
        }
    }
    return res;
}

// The chord of a solitary sphere (DevShape::solitary): a ray leaving a point
// of sphere `sh` that hits the sphere again at t hits nothing else before t,
// and for a ray that starts on the sphere the root box test of the scan
// passes (the ball lies inside the scene box by a margin).  Same arithmetic
// as the scan's sphere test (sphere_hit_nb, the adaptive epsilon of
// bvh.cpp:412-418), so t is the scan's; false: the caller scans as usual.
template <bool FAST = false>
ND bool chord_hit(const DevShape &sh, const PathState &ps, float &t) {
    TRay r;
    r.o = ps.o;
    r.d = ps.d;
    r.mint = ps.mint;
    r.maxt = ps.maxt;
    if (r.mint == kEps) r.mint = smax(r.mint, r.mint * smax(smax(fabsf(r.o.x), fabsf(r.o.y)), fabsf(r.o.z)));
    if (r.maxt < r.mint) return false;
    return sphere_hit_nb<FAST>(make_float4(sh.center[0], sh.center[1], sh.center[2], 0.0f),
                               make_float4(sh.radius, 0.0f, 0.0f, 0.0f), r, t);
}

// At most this many tracing lanes use the cooperative scan (each costs one
// primitive test per lane and a reduction; the per-lane scan costs n tests).
#ifndef NORI_COOP_MAX
#define NORI_COOP_MAX 4
#endif
constexpr int kCoopMax = NORI_COOP_MAX;

// Runs every path still queued to completion, one thread per path: the
// Russian-roulette tail (a glass-sphere path survives with q = 0.99 per
// bounce) would otherwise cost three launches per bounce.  Waves loop while
// any lane's path is alive so that the lanes can trace cooperatively.
// Exclusive prefix of the queued-path counts of the G segments (pre[G] = total).
#if NORI_TU == 2
__global__ __launch_bounds__(1024) void k_tail_prefix(const uint32_t *cnt, uint32_t G, uint32_t *pre) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x, per = (G + 1023) / 1024, b = t * per, e = min(G, b + per);
    uint32_t sum = 0;
    for (uint32_t i = b; i < e; ++i) sum += cnt[i];
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {  // inclusive scan (Hillis-Steele)
        const uint32_t v = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = t ? part[t - 1] : 0u;
    for (uint32_t i = b; i < e; ++i) {
        pre[i] = run;
        run += cnt[i];
    }
    if (t == 1023) pre[G] = part[1023];
}

#endif
#ifndef NORI_FINISH_PRIO
#define NORI_FINISH_PRIO 1
#endif
#ifndef NORI_FINISH_WAVES  // 0: 64 paths per wave
// 2048 since the glass-sphere chain (round 3): fewer finisher waves leave the
// film splat beside it more of the chip; 64-spp share 3446 -> 3550 (4096) ->
// 3652 (2048) Msamples/s, 512 spp 4737 -> 4753 / 4744 (one box, interleaved).
// 1024 since round 6's shorter glass chain: 64-spp share 4677 -> 4725 (4
// reps, every 1024 run above every 2048 run), 512 spp 5843 / 5834 (noise)
#define NORI_FINISH_WAVES 1024
#endif
constexpr uint32_t kFinishWaves = NORI_FINISH_WAVES;
#ifndef NORI_FINISH_GLASS  // 0: the tail finisher shades glass-sphere vertices generically
#define NORI_FINISH_GLASS 1
#endif
constexpr bool kFinishGlass = NORI_FINISH_GLASS;
template <int STACK, int INTEG, bool LDS, int VAR>  // LDS: the scene blob is staged (scan-mode scenes); VAR: see k_shade
__global__ __launch_bounds__(kTraceBlock) void k_finish(DevScene Sg, PathQueue Q, SegState seg, int sel,
                                                        float4 *rec, WorkDesc wd, float *film, Counters *C,
                                                        const uint32_t *pre, uint32_t G) {
    __shared__ uint32_t stk[stack_words(STACK) * kTraceBlock];
    extern __shared__ __attribute__((aligned(16))) float4 blob_lds[];
    // the queued paths of all segments, numbered through the prefix `pre`
    // (k_tail_prefix), K consecutive ones per wave: K = n / kFinishWaves
    // rounded up, so the tail spreads over about kFinishWaves waves.  The
    // render waits for the longest path, and a lane's bounce costs the sum of
    // the branches its wave-mates take: few paths per wave keep that chain
    // close to the lone-lane latency from its first bounce on.
    constexpr bool FULL = VAR != 0, CHROMA = VAR == 2;
    const uint32_t n = pre[G];
    const uint32_t K = kFinishWaves ? min(64u, max(1u, (n + kFinishWaves - 1) / kFinishWaves)) : 64u;
    if (blockIdx.x * (kTraceBlock / 64) * K >= n) return;  // whole block idle
    // Each bounce of a tail path is a chain of dependent reads of small
    // tables; for small scenes they are staged into LDS first so the chain
    // runs at LDS latency instead of L2 latency.
    DevScene S = Sg;
    if constexpr (LDS) {  // the BVH path reads global memory (gld)
        for (uint32_t i = threadIdx.x; i < Sg.blob_bytes / 16; i += kTraceBlock) blob_lds[i] = Sg.blob[i];
        __syncthreads();
        S = scene_in_lds(Sg, reinterpret_cast<const char *>(blob_lds));
    }
    const uint32_t first = (blockIdx.x * kTraceBlock + threadIdx.x) / 64 * K, gid = first + lane_id();
    if (first >= n) return;  // whole wave idle
#if NORI_FINISH_PRIO
    // the film splat runs beside the finisher: its waves must not take the
    // issue slots of these few latency-bound ones
    __builtin_amdgcn_s_setprio(3);
#endif
    bool active = lane_id() < K && gid < n;
    uint32_t sg = 0;
    if (active) {  // segment of path gid: last s with pre[s] <= gid
        uint32_t lo = 0, hi = G;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pre[mid] <= gid) lo = mid;
            else hi = mid;
        }
        sg = lo;
    }
    const uint32_t q = sg * kSeg + (active ? gid - pre[sg] : 0u);
    PathState ps;
    float4 h = make_float4(0, 0, 0, 0);
    if (active) {
        load_path(Sg, wd, Q, q, ps);
        h = Q.hit[q];
        ps.L = ld3(rec[ps.work]);
    }
    uint32_t rays = 0;
    const bool coop = STACK == 0 && S.num_prims <= 64;
    CoopPrim cp;
    if (coop) cp = coop_load(S);
    auto trace = [&](const TRay &r, bool want, bool any_hit, float &t, uint32_t &p, float &u, float &v) -> bool {
        if (coop && __popcll(__ballot(want)) <= kCoopMax)
            return any_hit ? coop_scan<true>(S, cp, r, want, t, p, u, v) : coop_scan<false>(S, cp, r, want, t, p, u, v);
        if (!want) return false;
        return any_hit ? traverse<STACK, true>(S, r, stk + threadIdx.x, t, p, u, v)
                       : traverse<STACK, false>(S, r, stk + threadIdx.x, t, p, u, v);
    };
#ifdef NORI_PROF_FINISH  // profiling build: clocks of the loop's phases, summed over waves
    // pt: shader clocks (s_memtime) of every iteration; p1: wall time (s_memrealtime,
    // 100 MHz) of the late iterations (index >= NORI_PROF_LATE) of long-running
    // waves, when the device runs little else: the lone-lane bounce
#ifndef NORI_PROF_LATE
#define NORI_PROF_LATE 200
#endif
    uint64_t pt[4] = {0, 0, 0, 0}, pc = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime(), wit = 0;
    uint64_t p1[4] = {0, 0, 0, 0}, n1 = 0, rc = rt0;
    bool solo = false;
#define NORI_PHASE(i)                                        \
    {                                                        \
        const uint64_t now = __builtin_amdgcn_s_memtime();   \
        pt[i] += now - pc;                                   \
        pc = now;                                            \
        const uint64_t rnow = __builtin_amdgcn_s_memrealtime(); \
        if (solo) p1[i] += rnow - rc;                        \
        rc = rnow;                                           \
    }
#else
#define NORI_PHASE(i)
#endif
    while (__ballot(active)) {
#ifdef NORI_PROF_FINISH
        solo = wit >= NORI_PROF_LATE;
        n1 += solo ? 1 : 0;
        rc = __builtin_amdgcn_s_memrealtime();
#endif
        ShadowOut so;
        so.emit = false;
        bool alive = false;
        // the shape of the vertex being shaded, if it is a solitary sphere (its
        // table reads issued before the shading, off the dependency chain)
        int sol = -1;  // (volumetric: a scattering event moves the origin off the surface)
        if (INTEG != NORI_INTEGRATOR_VOLUMETRIC && active && __float_as_uint(h.y) != 0xFFFFFFFFu) {
            const int s0 = (int)S.prim_shape[__float_as_uint(h.y)];
            sol = S.shapes[s0].solitary ? s0 : -1;
        }
        // a vertex on a solitary glass sphere: the chain of its chord bounces
        // runs here (glass_bounce, chord_hit) until the path leaves the
        // sphere or ends, or its NEE could no longer be skipped
        bool shaded = false;  // this iteration's vertex is shaded, ps holds the next ray
        if (INTEG != NORI_INTEGRATOR_VOLUMETRIC && kFinishGlass && active && sol >= 0) {
            // copies: the chain's constants are read from LDS once, before
            // the loop, and kept in registers (not re-read per bounce)
            const DevShape gs = S.shapes[sol];
            const DevBsdf gb = S.bsdfs[gs.bsdf];
            if (gb.type == NORI_BSDF_DIELECTRIC && gs.emitter < 0) {
#ifdef NORI_PROF_GLASS  // diagnostic build: wall time of lone-lane chains per chord bounce
                const bool lone = __popcll(__ballot(active)) == 1;
                const uint64_t g0 = __builtin_amdgcn_s_memrealtime();
                const uint32_t r0 = rays;
#endif
                while (INTEG != NORI_INTEGRATOR_PATH_MIS || skip_nee(S, gb, ps.beta)) {
                    if (kGlassStep)  // reflected into the next chord, as long as it lasts
                        while (glass_step<INTEG>(gs, gb, ps, h.x)) ++rays;
                    alive = glass_bounce<INTEG>(gs, gb, ps, h.x);
                    shaded = true;
                    if (!alive) break;
                    float tc;
                    if (!chord_hit<kGlassFast>(gs, ps, tc)) {
                        sol = -1;  // it leaves the sphere: traced below
                        break;
                    }
                    h = make_float4(tc, __uint_as_float(gs.prim_offset), 0.0f, 0.0f);
                    ++rays;
                    shaded = false;
                }
#ifdef NORI_PROF_GLASS
                if (lone && rays - r0 >= 8) {
                    atomicAdd(&C->prof[13], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - g0));
                    atomicAdd(&C->prof[14], (unsigned long long)(rays - r0));
                }
#endif
            }
        }
        if (active && !shaded) alive = shade_vertex<INTEG, false, FULL>(S, ps, h, rec, so);
        NORI_PHASE(0)
        {
            TRay r{so.o, so.d, V3{0, 0, 0}, kEps, so.maxt};
            float t, u, v;
            uint32_t p;
            rays += so.emit ? 1u : 0u;
            bool occluded = trace(r, so.emit, true, t, p, u, v);
            if (so.emit && !occluded) ps.L = ps.L + so.contrib;  // so.work == ps.work
        }
        NORI_PHASE(1)
        if (CHROMA && active && !alive && ps.chan < 2) {  // the sample's next colour channel
            next_channel<FULL>(Sg, wd, ps);
            alive = true;
            sol = -1;  // a camera ray
        }
        if (active && !alive) {
            active = false;
            // the sample is complete: splat it (k_splat skipped it as pending)
            const uint32_t w = ps.work, pass = w / wd.M, e = w - pass * wd.M, pix = wd.pixels[e];
            const uint32_t y = pix / (uint32_t)S.W, x = pix - y * (uint32_t)S.W;
            Pcg rg;
            wave_seed(rg, wd.seed, (uint64_t)(wd.pass_begin + pass) * ((uint64_t)S.W * (uint64_t)S.H) + pix);
            V2 jit = next2D(rg);
            // Sg: kernarg filter table (no local copy)
            splat_sample(Sg, film, C, x, y, jit, make_float4(ps.L.x, ps.L.y, ps.L.z, 0.0f), wd.var);
            atomicAdd(&seg.stats[sg].w, rays);
            atomicAdd(&C->finish_paths, 1u);
            atomicMax(&C->finish_max_rays, rays);
        }
        TRay r{ps.o, ps.d, V3{0, 0, 0}, ps.mint, ps.maxt};
        float t, u, v;
        uint32_t p;
        rays += active ? 1u : 0u;
        NORI_PHASE(2)
        // a path leaving a solitary sphere: its chord, if it has one, is the
        // closest hit (the glass-sphere paths of the tail bounce inside)
        bool want = active;
        if (active && sol >= 0) {
            float tc;
            if (chord_hit(S.shapes[sol], ps, tc)) {
                h = make_float4(tc, __uint_as_float(S.shapes[sol].prim_offset), 0.0f, 0.0f);
                want = false;
            }
        }
        trace(r, want, false, t, p, u, v);
        if (want) h = make_float4(t, __uint_as_float(p), u, v);
        NORI_PHASE(3)
#ifdef NORI_PROF_FINISH
        if (lane_id() == 0) atomicAdd(&C->prof[4], 1ull);
        ++wit;
#endif
    }
#ifdef NORI_PROF_FINISH
    if (lane_id() == 0) {
        for (int i = 0; i < 4; ++i) atomicAdd(&C->prof[i], (unsigned long long)pt[i]);
        for (int i = 0; i < 4; ++i) atomicAdd(&C->prof[8 + i], (unsigned long long)p1[i]);
        atomicAdd(&C->prof[12], (unsigned long long)n1);
        // the longest-running wave: its span in 100 MHz ticks (high bits) and loop iterations
        const uint64_t span = __builtin_amdgcn_s_memrealtime() - rt0;
        atomicMax(&C->prof[5], (unsigned long long)((span << 20) | (wit & 0xFFFFFu)));
    }
#endif
#undef NORI_PHASE
}

// ------------------------------------------------------------------ one-bounce integrators
// normals (normals.cpp:16-24), av (averagevisibility.cpp:16-27), direct
// (direct.cpp:17-45), direct_ems (direct_ems.cpp:17-51), direct_mats
// (direct_mats.cpp:17-44), direct_mis (direct_mis.cpp:17-85).  They trace a
// fixed, small number of rays per camera sample (1 + lights + 1 at most), so
// there is no path state to keep: one thread runs one sample start to end and
// writes its record; k_splat filters the records as for the path integrators.
template <int STACK>
struct OneBounce {
    const DevScene &S;
    uint32_t *stk;
    uint32_t rc = 0, rs = 0;  // rays traced: closest, shadow
    ND bool closest(V3 o, V3 d, float mint, float maxt, SurfHit &hs) {
        ++rc;
        TRay r{o, d, V3{0, 0, 0}, mint, maxt};
        float t, u, v;
        uint32_t p;
        if (!traverse<STACK, false>(S, r, stk, t, p, u, v)) return false;
        hs = surface(S, p, t, u, v, o, d);
        return true;
    }
    ND bool occluded(V3 o, V3 d, float maxt) {
        ++rs;
        TRay r{o, d, V3{0, 0, 0}, kEps, maxt};
        float t, u, v;
        uint32_t p;
        return traverse<STACK, true>(S, r, stk, t, p, u, v);
    }
    // emission of the hit surface seen from `from` (EmitterQueryRecord(from, its.p, n))
    ND V3 emission(const SurfHit &hs, V3 from) {
        const DevShape &sh = S.shapes[hs.shape];
        if (sh.emitter < 0) return V3{0, 0, 0};
        return emitter_eval(S, S.emitters[sh.emitter], hs.sh.n, normalize(hs.p - from));
    }
    // PhotonMapper::Li (photonmapper.cpp:119-196): emission at every hit, the
    // photon density estimate at the first diffuse surface, Russian roulette
    // and BSDF sampling at the others.  The kd-tree search (kdtree.h:260-316:
    // every photon with |x - p|^2 < r^2) is a 27-cell lookup in a hash grid of
    // cell size r: a bucket may hold photons of colliding cells, so each
    // photon is counted only from its own cell.
    ND V3 Li_pmap(Pcg &rng, V3 o, V3 d, float mint, float maxt) {
        V3 color{0, 0, 0}, att{1, 1, 1};
        for (;;) {
            SurfHit hs;
            if (!closest(o, d, mint, maxt, hs)) return color;
            color = color + att * emission(hs, o);
            const DevBsdf &B = S.bsdfs[S.shapes[hs.shape].bsdf];
            if (B.type == NORI_BSDF_DIFFUSE) {  // Diffuse::isDiffuse (diffuse.cpp:122)
                const float ic = S.ph_inv_cell;
                const int cx = (int)floorf(hs.p.x * ic), cy = (int)floorf(hs.p.y * ic), cz = (int)floorf(hs.p.z * ic);
                const V3 wi = to_local(hs.sh, -d);
                V3 pc{0, 0, 0};
                for (int dz = -1; dz <= 1; ++dz)
                    for (int dy = -1; dy <= 1; ++dy)
                        for (int dx = -1; dx <= 1; ++dx) {
                            const int gx = cx + dx, gy = cy + dy, gz = cz + dz;
                            const uint32_t h = photon_cell_hash(gx, gy, gz) & S.ph_mask;
                            const uint32_t j1 = S.ph_start[h + 1];
#ifndef NORI_PMAP_BATCH
#define NORI_PMAP_BATCH 4  // candidate photons whose positions are loaded together
#endif
                            for (uint32_t j0 = S.ph_start[h]; j0 < j1; j0 += NORI_PMAP_BATCH) {
                              float4 qb[NORI_PMAP_BATCH];
#pragma unroll
                              for (int u = 0; u < NORI_PMAP_BATCH; ++u)
                                  qb[u] = j0 + u < j1 ? gld(S.ph + j0 + u) : make_float4(0, 0, 0, 0);
#pragma unroll
                              for (int u = 0; u < NORI_PMAP_BATCH; ++u) {
                                const uint32_t j = j0 + u;
                                if (j >= j1) break;
                                const float4 pp = qb[u];
                                const V3 dd = ld3(pp) - hs.p;
                                if (!(dot(dd, dd) < S.ph_r2)) continue;
                                // own cell only (a bucket may hold colliding cells)
                                if ((int)floorf(pp.x * ic) != gx || (int)floorf(pp.y * ic) != gy ||
                                    (int)floorf(pp.z * ic) != gz)
                                    continue;
                                BRec br;
                                br.wi = wi;
                                // PhotonData::getDirection / getPower (photon.h:44-55)
                                const uint32_t dir = __float_as_uint(pp.w), rgbe = S.ph_rgbe[j];
                                const float *T = S.ph_tab;
                                const float st = T[768 + (dir & 255u)];
                                const V3 wd{T[(dir >> 8) & 255u] * st, T[256 + ((dir >> 8) & 255u)] * st,
                                            T[512 + (dir & 255u)]};
                                const float sc = T[1024 + (rgbe >> 24)];
                                const V3 pw{(float)(rgbe & 255u) * sc, (float)((rgbe >> 8) & 255u) * sc,
                                            (float)((rgbe >> 16) & 255u) * sc};
                                br.wo = to_local(hs.sh, wd);
                                br.measure = kMeasureSolidAngle;
                                br.uv = hs.uv;
                                pc = pc + bsdf_eval(B, br) * pw;
                              }
                            }
                        }
                return color + att * ((pc * kInvPi) / S.ph_norm);
            }
            const float q = smin(att.x, 0.99f);
            if (next1D(rng) > q) return color;
            att = att / q;
            BRec br;
            br.wi = to_local(hs.sh, -d);
            br.wo = V3{0, 0, 1};
            br.measure = kMeasureUnknown;
            br.uv = hs.uv;
            const V3 w = bsdf_sample(B, br, next2D(rng));
            if (is_zero(w)) return color;  // deviation D1
            att = att * w;
            o = hs.p;
            d = to_world(hs.sh, br.wo);
            mint = kEps;
            maxt = INF_F;
        }
    }
    template <int INTEG>
    ND V3 Li(Pcg &rng, V3 o, V3 d, float mint, float maxt) {
        if constexpr (INTEG == NORI_INTEGRATOR_PHOTONMAPPER) return Li_pmap(rng, o, d, mint, maxt);
        SurfHit hs;
        if (!closest(o, d, mint, maxt, hs)) return INTEG == NORI_INTEGRATOR_AV ? V3{1, 1, 1} : V3{0, 0, 0};
        if (INTEG == NORI_INTEGRATOR_NORMALS) return V3{fabsf(hs.sh.n.x), fabsf(hs.sh.n.y), fabsf(hs.sh.n.z)};
        if (INTEG == NORI_INTEGRATOR_AV) {
            // Warp::sampleUniformHemisphere (warp.cpp:25-42): rejection in the cube
            V3 w;
            do {
                w.x = 1.f - 2.f * next1D(rng);
                w.y = 1.f - 2.f * next1D(rng);
                w.z = 1.f - 2.f * next1D(rng);
            } while (dot(w, w) > 1.f);
            if (dot(w, hs.sh.n) < 0.f) w = -w;
            w = w / norm(w);
            ++rs;
            TRay r{hs.p, w, V3{0, 0, 0}, kEps, S.av_length};
            float t, u, v;
            uint32_t p;
            return traverse<STACK, true>(S, r, stk, t, p, u, v) ? V3{0, 0, 0} : V3{1, 1, 1};
        }
        const DevBsdf &B = S.bsdfs[S.shapes[hs.shape].bsdf];
        V3 color = INTEG == NORI_INTEGRATOR_DIRECT ? V3{0, 0, 0} : emission(hs, o);
        if (INTEG == NORI_INTEGRATOR_DIRECT || INTEG == NORI_INTEGRATOR_DIRECT_EMS ||
            INTEG == NORI_INTEGRATOR_DIRECT_MIS) {
            // every light, one shadow ray each; `direct` passes an unset sample
            // (its lights ignore it): (0, 0) here, nothing drawn
            for (uint32_t i = 0; i < S.num_emitters; ++i) {
                const V2 s2 = INTEG == NORI_INTEGRATOR_DIRECT ? V2{0, 0} : next2D(rng);
                const NeeSample ne = emitter_sample_one(S, S.emitters[i], hs.p, s2);
                if (occluded(hs.p, ne.wi, ne.maxt)) continue;
                const V3 wi = to_local(hs.sh, ne.wi), dv = to_local(hs.sh, -d);
                BRec br;
                br.measure = kMeasureSolidAngle;
                br.uv = hs.uv;
                br.wi = INTEG == NORI_INTEGRATOR_DIRECT ? wi : dv;  // direct.cpp builds (light, view)
                br.wo = INTEG == NORI_INTEGRATOR_DIRECT ? dv : wi;
                const V3 f = bsdf_eval(B, br);
                if (INTEG == NORI_INTEGRATOR_DIRECT_MIS) {
                    const float pdf_mat = bsdf_pdf(B, br);
                    const float w_em = pdf_mat + ne.pdf_em > 0.f ? ne.pdf_em / (pdf_mat + ne.pdf_em) : ne.pdf_em;
                    color = color + ((f * w_em) * ne.Li) * wi.z;
                } else {
                    color = color + (f * wi.z) * ne.Li;
                }
            }
        }
        if (INTEG == NORI_INTEGRATOR_DIRECT_MATS || INTEG == NORI_INTEGRATOR_DIRECT_MIS) {
            BRec br;
            br.wi = to_local(hs.sh, -d);
            br.wo = V3{0, 0, 1};
            br.measure = kMeasureUnknown;
            br.uv = hs.uv;
            const V3 w = bsdf_sample(B, br, next2D(rng));
            if (is_zero(w)) return color;  // deviation D1: no ray along an unset direction
            const float pdf_mat = INTEG == NORI_INTEGRATOR_DIRECT_MIS ? bsdf_pdf(B, br) : 0.0f;
            SurfHit nh;
            if (!closest(hs.p, to_world(hs.sh, br.wo), kEps, INF_F, nh)) return color;
            const DevShape &ns = S.shapes[nh.shape];
            if (ns.emitter < 0) return color;
            const DevEmitter &E = S.emitters[ns.emitter];
            const V3 wl = normalize(nh.p - hs.p);
            const V3 Le = emitter_eval(S, E, nh.sh.n, wl);
            if (INTEG == NORI_INTEGRATOR_DIRECT_MATS) return color + w * Le;
            const float pdf_em = emitter_pdf(S, E, nh.sh.n, wl);
            const float w_mat = pdf_mat + pdf_em > 0.f ? pdf_mat / (pdf_mat + pdf_em) : 0.0f;
            return color + (w * w_mat) * Le;
        }
        return color;
    }
};

#ifndef NORI_DIRECT_XCD
#define NORI_DIRECT_XCD 1
#endif
template <int STACK, int INTEG>
__global__ __launch_bounds__(kTraceBlock) void k_direct(DevScene S, WorkDesc wd, float4 *rec, Counters *C) {
    __shared__ uint32_t stk[stack_words(STACK) * kTraceBlock];
    // XCD-aware order (NORI_DIRECT_XCD): each XCD sweeps its own contiguous
    // eighth of the work ids, so at any moment it shades one band of image
    // rows and its L2 holds the photons / tree nodes of that band
    const uint32_t bid = NORI_DIRECT_XCD ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint64_t w = (uint64_t)bid * kTraceBlock + threadIdx.x;
    OneBounce<STACK> ob{S, stk + threadIdx.x};
    if (w < wd.total) {
        const uint32_t pass = (uint32_t)(w / wd.M), e = (uint32_t)(w - (uint64_t)pass * wd.M), pix = wd.pixels[e];
        const uint32_t y = pix / (uint32_t)S.W, x = pix - y * (uint32_t)S.W;
        Pcg rng;
        wave_seed(rng, wd.seed, (uint64_t)(wd.pass_begin + pass) * ((uint64_t)S.W * (uint64_t)S.H) + pix);
        const V2 jit = next2D(rng);
        const V2 ap = next2D(rng);  // apertureSample (render.cpp:99)
        const float px = (float)x + jit.x, py = (float)y + jit.y;
        V3 L;
        if (S.chromatic[0] != 0.0f || S.chromatic[1] != 0.0f || S.chromatic[2] != 0.0f) {
            // render.cpp:106-121: one ray per colour channel, Li calls in turn,
            // each weighted by its channel's unit colour
            V3 o[3], d[3];
            float mn[3], mx[3];
            for (int ch = 0; ch < 3; ++ch) camera_sample(S, px, py, ap, ch, o[ch], d[ch], mn[ch], mx[ch]);
            V3 v[3];
            for (int ch = 0; ch < 3; ++ch) {
                const V3 l = ob.template Li<INTEG>(rng, o[ch], d[ch], mn[ch], mx[ch]);
                v[ch] = V3{ch == 0 ? 1.f : 0.f, ch == 1 ? 1.f : 0.f, ch == 2 ? 1.f : 0.f} * l;
            }
            L = (v[0] + v[1]) + v[2];
        } else {
            V3 o, d;
            float mn, mx;
            camera_sample(S, px, py, ap, -1, o, d, mn, mx);
            L = V3{1, 1, 1} * ob.template Li<INTEG>(rng, o, d, mn, mx);
        }
        rec[w] = make_float4(L.x, L.y, L.z, rec_code(S.jit_lk, S.border, x, y, jit));
    }
    // ray counts: one atomic per wave
    uint32_t rc = ob.rc, rs = ob.rs;
    for (int off = 32; off > 0; off >>= 1) {
        rc += __shfl_xor(rc, off);
        rs += __shfl_xor(rs, off);
    }
    if (lane_id() == 0 && (rc | rs)) {
        atomicAdd(&C->direct_rays[0], (unsigned long long)rc);
        atomicAdd(&C->direct_rays[1], (unsigned long long)rs);
    }
}

// ------------------------------------------------------------------ photon tracing
// PhotonMapper::preprocess (photonmapper.cpp:41-117), one thread per emitted
// photon e (pcg32 stream wave_seed(kPhotonSeed, e), deviation D8): a light
// chosen uniformly, AreaEmitter::samplePhoton (arealight.cpp:78-95: surface
// point, cosine-weighted direction, power = Le * pi / pdf * lights), then
// bounces with a stored photon at every diffuse hit, Russian roulette on the
// red channel and BSDF sampling.  COUNT pass: photons stored per emitted
// photon.  STORE pass (photons e < n): they go to pre[e].. in emission order,
// and the map ends after `total` photons -- the reference's "return if the
// map is full" (photonmapper.cpp:92-94) over the emission order.
template <int STACK, bool STORE>
__global__ __launch_bounds__(kTraceBlock) void k_photons(DevScene S, uint64_t e0, uint32_t n, uint32_t *count,
                                                         const uint64_t *pre, uint64_t total, float4 *out) {
    __shared__ uint32_t stk[stack_words(STACK) * kTraceBlock];
    const uint32_t i = blockIdx.x * kTraceBlock + threadIdx.x;
    if (i >= n) return;
    Pcg rng;
    wave_seed(rng, kPhotonSeed, e0 + i);
    const uint32_t ne = S.num_emitters;
    uint32_t li = (uint32_t)floorf((float)ne * next1D(rng));  // Scene::getRandomEmitter (scene.h:68-74)
    if (li > ne - 1) li = ne - 1;
    const DevEmitter &E = S.emitters[li];
    const V2 s1 = next2D(rng), s2 = next2D(rng);
    const DevShape &esh = S.shapes[E.shape];
    V3 p, nrm;
    sample_surface(S, esh, s1, p, nrm);
    const float pdf = esh.area_norm;
    uint64_t stored = 0;
    const uint64_t base = STORE ? pre[i] : 0;
    const uint64_t limit = STORE ? (total > base ? total - base : 0) : ~0ull;
    if (pdf > 0) {  // (a light of zero area: no photon)
        const V3 cs = to_world(frame_from(nrm), sq_cosine_hemisphere(s2));
        const V3 ref = p + cs;  // EmitterQueryRecord(sRec.p + cosine_sample, sRec.p, sRec.n)
        V3 power = ((emitter_eval(S, E, nrm, normalize(p - ref)) * kPi) / pdf) * (float)ne;
        V3 o = p, d = cs;
        uint32_t *lstk = stk + threadIdx.x;
        for (;;) {
            TRay r{o, d, V3{0, 0, 0}, kEps, INF_F};
            float t, u, v;
            uint32_t prim;
            if (!traverse<STACK, false>(S, r, lstk, t, prim, u, v)) break;
            const SurfHit hs = surface(S, prim, t, u, v, o, d);
            const DevBsdf &B = S.bsdfs[S.shapes[hs.shape].bsdf];
            if (B.type == NORI_BSDF_DIFFUSE) {
                if (STORE) {
                    if (stored >= limit) break;
                    float4 *q = out + 3 * (size_t)(base + stored);
                    q[0] = make_float4(hs.p.x, hs.p.y, hs.p.z, 0.0f);
                    q[1] = make_float4(-d.x, -d.y, -d.z, 0.0f);
                    q[2] = make_float4(power.x, power.y, power.z, 0.0f);
                }
                ++stored;
            }
            const float q = smin(power.x, 0.99f);
            if (next1D(rng) > q) break;
            power = power / q;
            BRec br;
            br.wi = to_local(hs.sh, -d);
            br.wo = V3{0, 0, 1};
            br.measure = kMeasureUnknown;
            br.uv = hs.uv;
            const V3 w = bsdf_sample(B, br, next2D(rng));
            if (is_zero(w)) break;  // deviation D1
            power = power * w;
            o = hs.p;
            d = to_world(hs.sh, br.wo);
        }
    }
    if (!STORE) count[i] = (uint32_t)(stored < 0xFFFFFFFFull ? stored : 0xFFFFFFFFull);
}

#if NORI_TU == 0
template <bool STORE>
static void photons_dispatch(const DevScene &S, uint64_t e0, uint32_t n, uint32_t *count, const uint64_t *pre,
                             uint64_t total, float4 *out, int stack, hipStream_t st) {
    const dim3 g((n + kTraceBlock - 1) / kTraceBlock), b(kTraceBlock);
    switch (stack) {
    case 0: hipLaunchKernelGGL((k_photons<0, STORE>), g, b, 0, st, S, e0, n, count, pre, total, out); break;
    case 8: hipLaunchKernelGGL((k_photons<8, STORE>), g, b, 0, st, S, e0, n, count, pre, total, out); break;
    case 16: hipLaunchKernelGGL((k_photons<16, STORE>), g, b, 0, st, S, e0, n, count, pre, total, out); break;
    default: hipLaunchKernelGGL((k_photons<32, STORE>), g, b, 0, st, S, e0, n, count, pre, total, out); break;
    }
}
hipError_t launch_photons(const DevScene &S, uint64_t e0, uint32_t n, uint32_t *count, const uint64_t *pre,
                          uint64_t total, float4 *out, int stack, hipStream_t st) {
    if (n == 0) return hipSuccess;
    if (out) photons_dispatch<true>(S, e0, n, count, pre, total, out, stack, st);
    else photons_dispatch<false>(S, e0, n, count, pre, total, out, stack, st);
    return hipGetLastError();
}

#endif
// ------------------------------------------------------------------ film splat
#ifndef NORI_SPLAT_DEPTH
#define NORI_SPLAT_DEPTH 1  // sample records in flight per thread (prefetch depth)
#endif
// ImageBlock::put(pos, val) (block.cpp:93-122) for every sample of one 32x32
// block and a range of passes, then ImageBlock::put(block) (block.cpp:124-133)
// into the film.  A thread owns one pixel: all samples of that pixel fall in
// the same (2B+1)^2 window around it, so the thread sums the filtered samples
// of all its passes in registers and touches the LDS tile once per window
// cell instead of once per sample and cell.
// CODED (S.jit_lk != 0): the sample's window weights come from the jitter
// class its record carries (device_math.h jit_class), one row of a class
// table built per work-group -- the same weights as re-deriving the jitter
// from the sample's pcg32 stream (CODED = false), without the stream.
// SPLIT: two lanes per pixel (adjacent lanes, the same record), the first
// summing the R, G and the second the B, W windows -- half the registers per
// lane (more waves per SIMD hide the record loads), each lane redoing only the
// record's decode and weight reads (CODED).
// 768 threads (3 waves per SIMD) with 4 records in flight per lane: 108
// VGPRs, so that a 144-VGPR finisher wave still fits beside three splat
// waves on a SIMD (3 x 112 + 144 <= 512).  Measured (C2): splat 1.14-1.18 ms
// and finisher 1.15-1.17 ms against 1.26-1.33 / 1.10-1.15 ms for 512 threads
// with 8 records; 768 threads with 8 records (136 VGPRs) splat in 0.83 ms
// but starve the finisher (1.75 ms), DESIGN_LOG.md (round 5).
#ifndef NORI_SPLAT_SPLIT_BLOCK
#define NORI_SPLAT_SPLIT_BLOCK 768
#endif
#ifndef NORI_SPLAT_SPLIT_DEPTH
#define NORI_SPLAT_SPLIT_DEPTH 4
#endif
#ifndef NORI_SPLAT_NB
#define NORI_SPLAT_NB 0
#endif
constexpr int kSplatSplitBlock = NORI_SPLAT_SPLIT_BLOCK;
template <int B, bool CODED, bool SPLIT = false>
__global__ __launch_bounds__(SPLIT ? kSplatSplitBlock : kSplatBlock) void k_splat(DevScene S, const float4 *rec,
                                                                                  SplatDesc sd, float *film,
                                                                                  Counters *C) {
    constexpr int NT = SPLIT ? kSplatSplitBlock : kSplatBlock, NH = SPLIT ? 1 : 2;  // threads; pairs per lane
    constexpr int D = SPLIT ? NORI_SPLAT_SPLIT_DEPTH : NORI_SPLAT_DEPTH;           // records in flight per lane
    constexpr bool NB = CODED && NORI_SPLAT_NB;  // per-sample checks as selects, not branches
    constexpr int TS = NORI_BLOCK_SIZE + 2 * B, K = 2 * B + 1, KP = (K + 3) / 4;  // float4s per weight row
    __shared__ float tile[TS * TS * 4];
    __shared__ float ftab[NORI_FILTER_RESOLUTION + 1];
    __shared__ float4 wtab[CODED ? 256 * KP : 1];  // CODED: the window weights of every jitter class
    int4 bi = sd.blocks[blockIdx.x];
    const int ox = bi.x, oy = bi.y, bw = bi.z & 0xFFFF, bh = bi.z >> 16;
    const uint32_t off = (uint32_t)bi.w;
    const uint32_t p0 = blockIdx.y * sd.passes_per_wg, p1 = min(sd.passes, p0 + sd.passes_per_wg);
    for (int i = threadIdx.x; i < TS * TS * 4; i += NT) tile[i] = 0.0f;
    if (threadIdx.x <= NORI_FILTER_RESOLUTION) ftab[threadIdx.x] = S.filter[threadIdx.x];
    __syncthreads();
    const int npix = bw * bh;
    const float rad = S.filter_radius, lk = S.lookup;
    if constexpr (CODED) {
        // class (floor(P) - lx - B + 1, [f lk integer], q) -> the K weights of the window
        // cells d = 0..K-1 (tile column lx + d), computed by the formula of
        // the direct path below on a representative sub-pixel offset f of the
        // class (q / lk or (q + 1/2) / lk: the same indices and box ends,
        // device_math.h jit_class); P = lx + m + f with m = B + n - 1
        float *wt = reinterpret_cast<float *>(wtab);
        for (int i = threadIdx.x; i < 16 * S.jit_lk * KP; i += NT) {
            const int c = i / (4 * KP), d = i - c * (4 * KP);
            const int m = B + (c & 1) - 1, q = c >> 2;
            const float f = (c & 2) ? (float)q / lk : ((float)q + 0.5f) / lk;
            float wv = 0.0f;
            if (d < K) {
                const int lo = m + (int)ceilf(f - rad), hi = m + (int)floorf(f + rad);
                const int k = min((int)(fabsf((float)(d - m) - f) * lk), NORI_FILTER_RESOLUTION);
                wv = (d >= lo && d <= hi) ? ftab[k] : 0.0f;
            }
            wt[i] = wv;
        }
        __syncthreads();
    }
    const uint64_t WH = (uint64_t)S.W * (uint64_t)S.H;
    uint32_t inval = 0;
    for (int jj = threadIdx.x; jj < (SPLIT ? 2 : 1) * npix; jj += NT) {
        const int j = SPLIT ? jj >> 1 : jj, h = SPLIT ? jj & 1 : 0;  // h: the lane's channel pair (SPLIT)
        const int ly = j / bw, lx = j - ly * bw, x = ox + lx, y = oy + ly;
        // the window's RGBW sums as two packed pairs per cell (RG, BW; SPLIT:
        // the lane's pair): each half of a v_pk_mul_f32 / v_pk_add_f32 rounds
        // as the scalar op does
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 acc[K][K][NH];
#pragma unroll
        for (int a = 0; a < K; ++a)
#pragma unroll
            for (int c = 0; c < K; ++c)
#pragma unroll
                for (int e = 0; e < NH; ++e) acc[a][c][e] = f2{0.0f, 0.0f};
        bool any = false;
        float vs[7] = {0, 0, 0, 0, 0, 0, 0};  // sample statistics of the pixel (sd.var)
        auto put = [&](const float4 &L0, uint32_t p) {
            const uint32_t code = __float_as_uint(L0.w);
            // pending: the finisher splats this sample; Color3f::isValid
            // (common.cpp:224-231): invalid samples are dropped
            const bool pend = (code & kRecPending) != 0u;
            const bool valid = !(L0.x < 0 || !isfinite(L0.x) || L0.y < 0 || !isfinite(L0.y) || L0.z < 0 || !isfinite(L0.z));
            const bool ok = !pend && valid;
            if constexpr (!NB) {
                if (!ok) {
                    inval += (!pend && h == 0) ? 1u : 0u;
                    return;
                }
            } else {
                inval += (!pend && !valid && h == 0) ? 1u : 0u;
            }
            // NB: a skipped sample adds exact zeros -- radiance 0 and weights
            // 0 -- so the window sums keep their values bit for bit
            const float4 L = make_float4(ok ? L0.x : 0.0f, ok ? L0.y : 0.0f, ok ? L0.z : 0.0f, 0.0f);
            any = any || ok;
            vs[0] += L.x;
            vs[1] += L.y;
            vs[2] += L.z;
            vs[3] += L.x * L.x;
            vs[4] += L.y * L.y;
            vs[5] += L.z * L.z;
            vs[6] += ok ? 1.0f : 0.0f;
            float wx[K], wy[K];
            if constexpr (CODED) {
                const float4 *tx = wtab + (code & 255u) * KP, *ty = wtab + ((code >> 8) & 255u) * KP;
#pragma unroll
                for (int e = 0; e < KP; ++e) {
                    const float4 a = tx[e], b = ty[e];
                    const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
                    for (int c4 = 0; c4 < 4; ++c4)
                        if (4 * e + c4 < K) {
                            wx[4 * e + c4] = av[c4];
                            wy[4 * e + c4] = ok ? bv[c4] : 0.0f;
                        }
                }
            } else {
                uint64_t sid = (uint64_t)(sd.pass_begin + p) * WH + (uint64_t)y * S.W + x;
                Pcg r;
                wave_seed(r, sd.seed, sid);
                V2 jit = next2D(r);
                float px = ((float)x + jit.x) - 0.5f - (float)(ox - B), py = ((float)y + jit.y) - 0.5f - (float)(oy - B);
                int x0 = max((int)ceilf(px - rad), 0), y0 = max((int)ceilf(py - rad), 0);
                int x1 = min((int)floorf(px + rad), TS - 1), y1 = min((int)floorf(py + rad), TS - 1);
#pragma unroll
                for (int d = 0; d < K; ++d) {
                    int cx = lx + d, cy = ly + d;  // tile column / row of window cell d
                    int kx = min((int)(fabsf((float)cx - px) * lk), NORI_FILTER_RESOLUTION);
                    int ky = min((int)(fabsf((float)cy - py) * lk), NORI_FILTER_RESOLUTION);
                    const float fx = ftab[kx], fy = ftab[ky];  // unconditional: no branch per cell
                    wx[d] = (cx >= x0 && cx <= x1) ? fx : 0.0f;
                    wy[d] = (cy >= y0 && cy <= y1) ? fy : 0.0f;
                }
            }
            // Color4f(value) * wx (the row factor is shared by all rows); (1 * wx) = wx exactly
            f2 lp[NH][K];
            const f2 rg{L.x, L.y}, bw1{L.z, 1.0f};
#pragma unroll
            for (int c = 0; c < K; ++c)
#pragma unroll
                for (int e = 0; e < NH; ++e) lp[e][c] = (SPLIT ? (h ? bw1 : rg) : (e ? bw1 : rg)) * wx[c];
#pragma unroll
            for (int a = 0; a < K; ++a)
#pragma unroll
                for (int c = 0; c < K; ++c)
#pragma unroll
                    for (int e = 0; e < NH; ++e) acc[a][c][e] += lp[e][c] * wy[a];
        };
        // the records of the next D passes are in flight while one is splatted
        // (a ring of D registers, the pass loop unrolled by D: no moves)
        float4 Lq[D];
#pragma unroll
        for (int d = 0; d < D; ++d)
            Lq[d] = p0 + d < p1 ? rec[(size_t)(p0 + d) * sd.M + off + j] : make_float4(0, 0, 0, __uint_as_float(kRecPending));
        for (uint32_t p = p0; p < p1; p += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const float4 L = Lq[d];
                if (p + D + d < p1) Lq[d] = rec[(size_t)(p + D + d) * sd.M + off + j];
                if (p + d < p1) put(L, p + d);
            }
        }
        if (any && sd.var && h == 0) {
            float *v = sd.var + 8 * ((size_t)y * S.W + x);
            for (int k = 0; k < 7; ++k) atomicAdd(v + k, vs[k]);
        }
        if (any) {
#pragma unroll
            for (int a = 0; a < K; ++a)
#pragma unroll
                for (int c = 0; c < K; ++c) {
                    float *t = tile + 4 * ((ly + a) * TS + (lx + c)) + 2 * h;
                    const f2 u = acc[a][c][0], v = acc[a][c][NH - 1];
                    if (SPLIT ? (u.x != 0.0f || u.y != 0.0f) : (v.y != 0.0f || u.x != 0.0f || u.y != 0.0f || v.x != 0.0f)) {
                        atomicAdd(t + 0, u.x);
                        atomicAdd(t + 1, u.y);
                        if (!SPLIT) {
                            atomicAdd(t + 2, v.x);
                            atomicAdd(t + 3, v.y);
                        }
                    }
                }
        }
    }
    if (inval) atomicAdd(&C->invalid, (unsigned long long)inval);
    __syncthreads();
    const int rows = bh + 2 * B, cols = bw + 2 * B, FW = S.W + 2 * B;
    for (int i = threadIdx.x; i < rows * cols; i += NT) {
        int yy = i / cols, xx = i - yy * cols;
        const float *c = tile + 4 * (yy * TS + xx);
        float *f = film + 4 * ((size_t)(oy + yy) * FW + (ox + xx));
        if (c[3] != 0.0f || c[0] != 0.0f || c[1] != 0.0f || c[2] != 0.0f) {
            atomicAdd(f + 0, c[0]);
            atomicAdd(f + 1, c[1]);
            atomicAdd(f + 2, c[2]);
            atomicAdd(f + 3, c[3]);
        }
    }
}

// ------------------------------------------------------------------ launchers
#if NORI_TU == 0
template <bool ANY>
static hipError_t trace_dispatch(const DevScene &S, const float4 *rays, uint32_t n, float4 *hits, int stack,
                                 hipStream_t st) {
    dim3 g((n + kTraceBlock - 1) / kTraceBlock), b(kTraceBlock);
    switch (stack) {
    case 0: hipLaunchKernelGGL((k_trace<0, ANY>), g, b, 0, st, S, rays, n, hits); break;
    case 8: hipLaunchKernelGGL((k_trace<8, ANY>), g, b, 0, st, S, rays, n, hits); break;
    case 16: hipLaunchKernelGGL((k_trace<16, ANY>), g, b, 0, st, S, rays, n, hits); break;
    case 32: hipLaunchKernelGGL((k_trace<32, ANY>), g, b, 0, st, S, rays, n, hits); break;
    default: hipLaunchKernelGGL((k_trace<64, ANY>), g, b, 0, st, S, rays, n, hits); break;
    }
    return hipGetLastError();
}
hipError_t launch_trace(const DevScene &S, const float4 *rays, uint32_t n, int any_hit, float4 *hits, int stack,
                        hipStream_t st, const ScanRtc *rtc) {
    if (n == 0) return hipSuccess;
    if (stack == 0 && rtc && rtc->trace[any_hit ? 1 : 0]) {
        void *args[] = {(void *)&S, (void *)&rays, (void *)&n, (void *)&hits};
        return hipModuleLaunchKernel(rtc->trace[any_hit ? 1 : 0], (n + kTraceBlock - 1) / kTraceBlock, 1, 1, kTraceBlock,
                                     1, 1, 0, st, args, nullptr);
    }
    return any_hit ? trace_dispatch<true>(S, rays, n, hits, stack, st)
                   : trace_dispatch<false>(S, rays, n, hits, stack, st);
}

#endif
#if NORI_TU == 1
template <int INTEG, int VAR>
static void shade_dispatch(const DevScene &S, const PathQueue &in, const PathQueue &out, const ShadowQueue &sq,
                           const SegState &seg, int in_sel, const WorkDesc &wd, float4 *rec, Counters *C,
                           uint32_t lds, uint32_t nseg, hipStream_t st) {
    dim3 g(nseg), b(kShadeBlock);  // nseg segments from wd.b0 (wd.G counts the whole pool)
    // the shadow-ray slots overlay the blob, dead once the vertices are shaded
    const uint32_t dyn = S.nee_inline ? std::max(lds, kNeeSlotBytes) : lds;
    if (lds)
        hipLaunchKernelGGL((k_shade<INTEG, true, VAR>), g, b, dyn, st, S, in, out, sq, seg, in_sel, wd, rec, C, lds);
    else
        hipLaunchKernelGGL((k_shade<INTEG, false, VAR>), g, b, dyn, st, S, in, out, sq, seg, in_sel, wd, rec, C, 0u);
}
template <int INTEG>
static void shade_dispatch(const DevScene &S, const PathQueue &in, const PathQueue &out, const ShadowQueue &sq,
                           const SegState &seg, int in_sel, const WorkDesc &wd, float4 *rec, Counters *C,
                           uint32_t lds, uint32_t nseg, hipStream_t st) {
    if (S.basic) shade_dispatch<INTEG, 0>(S, in, out, sq, seg, in_sel, wd, rec, C, lds, nseg, st);
    else if (S.chroma) shade_dispatch<INTEG, 2>(S, in, out, sq, seg, in_sel, wd, rec, C, lds, nseg, st);
    else shade_dispatch<INTEG, 1>(S, in, out, sq, seg, in_sel, wd, rec, C, lds, nseg, st);
}
hipError_t launch_shade(const DevScene &S, const PathQueue &in, const PathQueue &out, const ShadowQueue &sq,
                        const SegState &seg, int in_sel, const WorkDesc &wd, float4 *rec, Counters *C,
                        uint32_t nseg, hipStream_t st) {
    if (nseg == 0 || wd.b0 + nseg > wd.G) return hipErrorInvalidValue;
    const uint32_t lds = S.blob_bytes <= kShadeLdsMax ? S.blob_bytes : 0u;
    switch (S.integrator) {
    case NORI_INTEGRATOR_PATH_MATS:
        shade_dispatch<NORI_INTEGRATOR_PATH_MATS>(S, in, out, sq, seg, in_sel, wd, rec, C, lds, nseg, st);
        break;
    case NORI_INTEGRATOR_VOLUMETRIC:
        shade_dispatch<NORI_INTEGRATOR_VOLUMETRIC>(S, in, out, sq, seg, in_sel, wd, rec, C, lds, nseg, st);
        break;
    default: shade_dispatch<NORI_INTEGRATOR_PATH_MIS>(S, in, out, sq, seg, in_sel, wd, rec, C, lds, nseg, st); break;
    }
    return hipGetLastError();
}

#endif
#if NORI_TU == 0
hipError_t launch_extend(const DevScene &S, const PathQueue &q, const uint32_t *cnt, uint32_t G, int stack,
                         hipStream_t st, const ScanRtc *rtc) {
    dim3 g(seg_grid(G, kTraceSlices)), b(kTraceBlock);
    if (stack == 0) {
        const dim3 gk(seg_grid(G, scan_per<kScanRays, NORI_EXTEND_BLOCK>())), bk(NORI_EXTEND_BLOCK);
        if (rtc && rtc->extend) {
            void *args[] = {(void *)&S, (void *)&q, (void *)&cnt, (void *)&G};
            const uint32_t per = kTraceGroup * kSeg / (NORI_EXTEND_BLOCK * (uint32_t)rtc->k_extend);
            return hipModuleLaunchKernel(rtc->extend, seg_grid(G, per), 1, 1, bk.x, 1, 1, 0, st, args, nullptr);
        }
        hipLaunchKernelGGL(k_extend_scan<kScanRays>, gk, bk, 0, st, S, q, cnt, G);
        return hipGetLastError();
    }
    switch (stack) {
    case 8: hipLaunchKernelGGL(k_extend<8>, g, b, 0, st, S, q, cnt, G); break;
    case 16: hipLaunchKernelGGL(k_extend<16>, g, b, 0, st, S, q, cnt, G); break;
    case 32: hipLaunchKernelGGL(k_extend<32>, g, b, 0, st, S, q, cnt, G); break;
    default: hipLaunchKernelGGL(k_extend<64>, g, b, 0, st, S, q, cnt, G); break;
    }
    return hipGetLastError();
}

bool launch_trace_both(const DevScene &S, const PathQueue &q, const uint32_t *cnt, const ShadowQueue &sq,
                       const uint32_t *shcnt, float4 *rec, uint32_t G, int stack, const ScanRtc *rtc, hipStream_t st,
                       hipError_t &err) {
    static_assert(NORI_EXTEND_BLOCK == NORI_SHADOW_BLOCK, "one work-group size for both roles");
    if (stack != 0) {  // BVH walks
        static_assert(kTraceSlices % kXcds == 0, "the shadow range starts on an XCD boundary");
        const uint32_t nbe = seg_grid(G, kTraceSlices), nbt = 2 * nbe;
        switch (stack) {
        case 8: hipLaunchKernelGGL(k_trace_both<8>, dim3(nbt), dim3(kTraceBlock), 0, st, S, q, cnt, sq, shcnt, rec, G, nbe); break;
        case 16: hipLaunchKernelGGL(k_trace_both<16>, dim3(nbt), dim3(kTraceBlock), 0, st, S, q, cnt, sq, shcnt, rec, G, nbe); break;
        case 32: hipLaunchKernelGGL(k_trace_both<32>, dim3(nbt), dim3(kTraceBlock), 0, st, S, q, cnt, sq, shcnt, rec, G, nbe); break;
        default: hipLaunchKernelGGL(k_trace_both<64>, dim3(nbt), dim3(kTraceBlock), 0, st, S, q, cnt, sq, shcnt, rec, G, nbe); break;
        }
        err = hipGetLastError();
        return true;
    }
    if (!rtc || !rtc->both) return false;
    uint32_t nb_ext = seg_grid(G, kTraceGroup * kSeg / (NORI_EXTEND_BLOCK * (uint32_t)rtc->k_extend));
    const uint32_t nb = nb_ext + seg_grid(G, scan_per<kScanRaysShadow, NORI_SHADOW_BLOCK>());
    void *args[] = {(void *)&S, (void *)&q, (void *)&cnt, (void *)&sq, (void *)&shcnt, (void *)&rec, (void *)&G, (void *)&nb_ext};
    err = hipModuleLaunchKernel(rtc->both, nb, 1, 1, NORI_EXTEND_BLOCK, 1, 1, 0, st, args, nullptr);
    return true;
}
hipError_t launch_shadow(const DevScene &S, const ShadowQueue &sq, const uint32_t *shcnt, float4 *rec, uint32_t G,
                         int stack, hipStream_t st, const ScanRtc *rtc) {
    dim3 g(seg_grid(G, kTraceSlices)), b(kTraceBlock);
    if (stack == 0) {
        const dim3 gk(seg_grid(G, scan_per<kScanRaysShadow, NORI_SHADOW_BLOCK>())), bk(NORI_SHADOW_BLOCK);
        if (rtc && rtc->shadow) {
            void *args[] = {(void *)&S, (void *)&sq, (void *)&shcnt, (void *)&rec, (void *)&G};
            return hipModuleLaunchKernel(rtc->shadow, gk.x, 1, 1, bk.x, 1, 1, 0, st, args, nullptr);
        }
        hipLaunchKernelGGL(k_shadow_scan<kScanRaysShadow>, gk, bk, 0, st, S, sq, shcnt, rec, G);
        return hipGetLastError();
    }
    switch (stack) {
    case 8: hipLaunchKernelGGL(k_shadow<8>, g, b, 0, st, S, sq, shcnt, rec, G); break;
    case 16: hipLaunchKernelGGL(k_shadow<16>, g, b, 0, st, S, sq, shcnt, rec, G); break;
    case 32: hipLaunchKernelGGL(k_shadow<32>, g, b, 0, st, S, sq, shcnt, rec, G); break;
    default: hipLaunchKernelGGL(k_shadow<64>, g, b, 0, st, S, sq, shcnt, rec, G); break;
    }
    return hipGetLastError();
}

// Start of a chunk of passes: zero the counters, the segments' path counts,
// work cursors and statistics, and preset the count of segments whose work
// stream is empty from the start (one launch instead of five copies/fills).
__global__ __launch_bounds__(256) void k_reset(Counters *C, uint32_t empty, SegState seg, uint32_t G) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    constexpr uint32_t nw = sizeof(Counters) / 4;
    if (i < nw) reinterpret_cast<uint32_t *>(C)[i] = i == 0 ? empty : 0u;  // word 0: exhausted
    if (i < G) {
        seg.cnt[0][i] = 0u;
        seg.cursor[i] = 0u;
        seg.stats[i] = make_uint4(0u, 0u, 0u, 0u);
    }
}
hipError_t launch_reset(Counters *C, uint32_t empty, const SegState &seg, uint32_t G, hipStream_t st) {
    static_assert(offsetof(Counters, exhausted) == 0, "Counters layout");
    const uint32_t n = std::max<uint32_t>(G, sizeof(Counters) / 4);
    hipLaunchKernelGGL(k_reset, dim3((n + 255) / 256), dim3(256), 0, st, C, empty, seg, G);
    return hipGetLastError();
}

hipError_t launch_mark(const PathQueue &Q, const SegState &seg, int sel, float4 *rec, uint32_t G, hipStream_t st) {
    hipLaunchKernelGGL(k_mark, dim3(2 * G), dim3(kTraceBlock), 0, st, Q, seg, sel, rec);
    return hipGetLastError();
}

#endif
#if NORI_TU == 2
template <int INTEG, int VAR>
static void finish_dispatch(const DevScene &S, const PathQueue &Q, const SegState &seg, int sel, float4 *rec,
                            const WorkDesc &wd, float *film, Counters *C, uint32_t G, int stack, uint32_t *pre,
                            hipStream_t st) {
    // enough waves for any path count n <= 256 G (kFinishWaves, or n / 64 <= 4 G when
    // K = 64); the idle blocks exit at once
    constexpr uint32_t wpb = kTraceBlock / 64;  // waves per block
    dim3 g(std::max<uint32_t>(2 * G, (kFinishWaves + wpb - 1) / wpb)), b(kTraceBlock);
    switch (stack) {
    case 0:  // LDS-staged when the scene has a blob
        if (S.blob_bytes)
            hipLaunchKernelGGL((k_finish<0, INTEG, true, VAR>), g, b, S.blob_bytes, st, S, Q, seg, sel, rec, wd, film, C, pre, G);
        else
            hipLaunchKernelGGL((k_finish<0, INTEG, false, VAR>), g, b, 0, st, S, Q, seg, sel, rec, wd, film, C, pre, G);
        break;
    case 8: hipLaunchKernelGGL((k_finish<8, INTEG, false, VAR>), g, b, 0, st, S, Q, seg, sel, rec, wd, film, C, pre, G); break;
    case 16: hipLaunchKernelGGL((k_finish<16, INTEG, false, VAR>), g, b, 0, st, S, Q, seg, sel, rec, wd, film, C, pre, G); break;
    case 32: hipLaunchKernelGGL((k_finish<32, INTEG, false, VAR>), g, b, 0, st, S, Q, seg, sel, rec, wd, film, C, pre, G); break;
    default: hipLaunchKernelGGL((k_finish<64, INTEG, false, VAR>), g, b, 0, st, S, Q, seg, sel, rec, wd, film, C, pre, G); break;
    }
}
template <int INTEG>
static void finish_dispatch(const DevScene &S, const PathQueue &Q, const SegState &seg, int sel, float4 *rec,
                            const WorkDesc &wd, float *film, Counters *C, uint32_t G, int stack, uint32_t *pre,
                            hipStream_t st) {
    if (S.basic) finish_dispatch<INTEG, 0>(S, Q, seg, sel, rec, wd, film, C, G, stack, pre, st);
    else if (S.chroma) finish_dispatch<INTEG, 2>(S, Q, seg, sel, rec, wd, film, C, G, stack, pre, st);
    else finish_dispatch<INTEG, 1>(S, Q, seg, sel, rec, wd, film, C, G, stack, pre, st);
}
hipError_t launch_tail_prefix(const SegState &seg, int sel, uint32_t G, uint32_t *pre, hipStream_t st) {
    hipLaunchKernelGGL(k_tail_prefix, dim3(1), dim3(1024), 0, st, seg.cnt[sel], G, pre);
    return hipGetLastError();
}
hipError_t launch_finish(const DevScene &S, const PathQueue &Q, const SegState &seg, int sel, float4 *rec,
                         const WorkDesc &wd, float *film, Counters *C, uint32_t G, int stack, uint32_t *pre,
                         hipStream_t st) {
    if (S.integrator == NORI_INTEGRATOR_PATH_MATS)
        finish_dispatch<NORI_INTEGRATOR_PATH_MATS>(S, Q, seg, sel, rec, wd, film, C, G, stack, pre, st);
    else if (S.integrator == NORI_INTEGRATOR_VOLUMETRIC)
        finish_dispatch<NORI_INTEGRATOR_VOLUMETRIC>(S, Q, seg, sel, rec, wd, film, C, G, stack, pre, st);
    else
        finish_dispatch<NORI_INTEGRATOR_PATH_MIS>(S, Q, seg, sel, rec, wd, film, C, G, stack, pre, st);
    return hipGetLastError();
}

#endif
#if NORI_TU == 0
template <int INTEG>
static void direct_dispatch(const DevScene &S, const WorkDesc &wd, float4 *rec, Counters *C, int stack,
                            hipStream_t st) {
    const dim3 g((uint32_t)((wd.total + kTraceBlock - 1) / kTraceBlock)), b(kTraceBlock);
    switch (stack) {
    case 0: hipLaunchKernelGGL((k_direct<0, INTEG>), g, b, 0, st, S, wd, rec, C); break;
    case 8: hipLaunchKernelGGL((k_direct<8, INTEG>), g, b, 0, st, S, wd, rec, C); break;
    case 16: hipLaunchKernelGGL((k_direct<16, INTEG>), g, b, 0, st, S, wd, rec, C); break;
    default: hipLaunchKernelGGL((k_direct<32, INTEG>), g, b, 0, st, S, wd, rec, C); break;
    }
}
hipError_t launch_direct(const DevScene &S, const WorkDesc &wd, float4 *rec, Counters *C, int stack, hipStream_t st) {
    if (wd.total == 0) return hipSuccess;
    switch (S.integrator) {
    case NORI_INTEGRATOR_NORMALS: direct_dispatch<NORI_INTEGRATOR_NORMALS>(S, wd, rec, C, stack, st); break;
    case NORI_INTEGRATOR_AV: direct_dispatch<NORI_INTEGRATOR_AV>(S, wd, rec, C, stack, st); break;
    case NORI_INTEGRATOR_DIRECT: direct_dispatch<NORI_INTEGRATOR_DIRECT>(S, wd, rec, C, stack, st); break;
    case NORI_INTEGRATOR_DIRECT_EMS: direct_dispatch<NORI_INTEGRATOR_DIRECT_EMS>(S, wd, rec, C, stack, st); break;
    case NORI_INTEGRATOR_DIRECT_MATS: direct_dispatch<NORI_INTEGRATOR_DIRECT_MATS>(S, wd, rec, C, stack, st); break;
    case NORI_INTEGRATOR_DIRECT_MIS: direct_dispatch<NORI_INTEGRATOR_DIRECT_MIS>(S, wd, rec, C, stack, st); break;
    case NORI_INTEGRATOR_PHOTONMAPPER: direct_dispatch<NORI_INTEGRATOR_PHOTONMAPPER>(S, wd, rec, C, stack, st); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// NORI_SPLAT_SPLIT=0: one lane per pixel in the coded splat too.
#ifndef NORI_SPLAT_SPLIT
#define NORI_SPLAT_SPLIT 1
#endif
static bool splat_split() {
    static const bool on = [] {
        const char *e = std::getenv("NORI_SPLAT_SPLIT");
        return e ? e[0] != '0' : NORI_SPLAT_SPLIT != 0;
    }();
    return on;
}
hipError_t launch_splat(const DevScene &S, const float4 *rec, const SplatDesc &sd, uint32_t nblocks, float *film,
                        Counters *C, hipStream_t st) {
    if (nblocks == 0 || sd.passes == 0) return hipSuccess;
    dim3 g(nblocks, (sd.passes + sd.passes_per_wg - 1) / sd.passes_per_wg), b(kSplatBlock);
    const bool coded = S.jit_lk != 0, split = coded && splat_split();
    const dim3 b2(kSplatSplitBlock);
#define NORI_SPLAT_CASE(b_)                                                                          \
    case b_:                                                                                         \
        if (split) hipLaunchKernelGGL((k_splat<b_, true, true>), g, b2, 0, st, S, rec, sd, film, C); \
        else if (coded) hipLaunchKernelGGL((k_splat<b_, true>), g, b, 0, st, S, rec, sd, film, C);  \
        else hipLaunchKernelGGL((k_splat<b_, false>), g, b, 0, st, S, rec, sd, film, C);            \
        break;
    switch (S.border) {
    NORI_SPLAT_CASE(0)
    NORI_SPLAT_CASE(1)
    NORI_SPLAT_CASE(2)
    NORI_SPLAT_CASE(3)
    NORI_SPLAT_CASE(4)
    default: return hipErrorInvalidValue;
    }
#undef NORI_SPLAT_CASE
    return hipGetLastError();
}

#endif
}  // namespace nori
