// kernels.hip -- CDNA4 (gfx950) kernels of the wavefront path tracer.
//
// One iteration of the state machine (runtime.hip drives it):
//   k_shade   : per path: surface hit -> emission, next-event estimation
//               (light sample + shadow ray), Russian roulette, BSDF sample,
//               or regeneration of a finished path slot with a new camera
//               sample.  Output paths and shadow rays are compacted with a
//               64-lane ballot + mbcnt prefix and one atomic per wave.
//   k_extend  : closest-hit BVH traversal of the compacted path queue.
//   k_shadow  : any-hit traversal; unoccluded rays add their payload to the
//               sample record (the reference's `color +=`, path_mis.cpp:48-60).
// After the queue drains, k_splat filters every sample into the RGBW film.
//
// This replaces render.cpp:194-233 (pass loop + tbb::parallel_for),
// renderBlock (render.cpp:80-133), PathMisIntegrator::Li (path_mis.cpp:17-101),
// PathMatsIntegrator::Li (path_mats.cpp:17-60), BVH::rayIntersect
// (bvh.cpp:404-462) and ImageBlock::put (block.cpp:93-133).
#include "kernels.h"

namespace nori {

#define INF_F __builtin_inff()

// ------------------------------------------------------------------ wave helpers
ND uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
ND uint32_t rank_in(uint64_t mask) {  // set lanes of `mask` below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
// Reserve `popc(mask)` slots on a device counter with one atomic per wave.
// Must be called by all 64 lanes of the wave (uniform control flow).
ND uint32_t wave_reserve(uint32_t *counter, uint64_t mask) {
    uint32_t base = 0;
    if (lane_id() == 0 && mask) base = atomicAdd(counter, (uint32_t)__popcll(mask));
    return __shfl(base, 0);
}
ND unsigned long long wave_reserve64(unsigned long long *counter, uint64_t mask) {
    unsigned long long base = 0;
    if (lane_id() == 0 && mask) base = atomicAdd(counter, (unsigned long long)__popcll(mask));
    uint32_t lo = __shfl((uint32_t)base, 0), hi = __shfl((uint32_t)(base >> 32), 0);
    return ((unsigned long long)hi << 32) | lo;
}

// ------------------------------------------------------------------ traversal
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

// Mesh::rayIntersect (mesh.cpp:83-120), edges precomputed exactly.
ND bool tri_hit(const float4 &a, const float4 &b, const float4 &c, const TRay &r, float &t, float &u, float &v) {
    V3 v0 = ld3(a), e1 = ld3(b), e2 = ld3(c);
    V3 pvec = cross(r.d, e2);
    float det = dot(e1, pvec);
    if (det > -1e-8f && det < 1e-8f) return false;
    float inv_det = 1.0f / det;
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

// BVH::rayIntersect (bvh.cpp:404-462): adaptive epsilon, closest or any hit.
// Near child first; the short stack lives in LDS, one column per lane.
template <int STACK, bool ANY>
ND bool traverse(const DevScene &S, TRay r, uint32_t *stk, float &tb, uint32_t &pb, float &ub, float &vb) {
    if (r.mint == kEps) r.mint = smax(r.mint, r.mint * smax(smax(fabsf(r.o.x), fabsf(r.o.y)), fabsf(r.o.z)));
    tb = INF_F;
    pb = 0xFFFFFFFFu;
    ub = vb = 0.0f;
    if (r.maxt < r.mint) return false;
    r.rcp = V3{1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z};
    uint32_t ref = 0;
    int sp = 0;
    bool found = false;
    for (;;) {
        if (!(ref & 0x80000000u)) {
            const float4 *nd = S.nodes + 4 * (size_t)ref;
            float4 a = nd[0], b = nd[1], c = nd[2], e = nd[3];
            float tl, tr;
            bool hl = box_test(a, b, r, tl), hr = box_test(c, e, r, tr);
            uint32_t lref = __float_as_uint(a.w), rref = __float_as_uint(b.w);
            if (hl && hr) {
                bool lf = tl <= tr;
                stk[sp * kTraceBlock] = lf ? rref : lref;
                ++sp;
                ref = lf ? lref : rref;
                continue;
            }
            if (hl || hr) {
                ref = hl ? lref : rref;
                continue;
            }
        } else {
            uint32_t start = ref & 0x1FFFFFFu, end = start + ((ref >> 25) & 63u) + 1u;
            for (uint32_t i = start; i < end; ++i) {
                const float4 *p = S.prims + 3 * (size_t)i;
                float4 p0 = p[0], p1 = p[1];
                float t = 0, u = 0, v = 0;
                bool h;
                if (__float_as_uint(p1.w) == 0u) {
                    float4 p2 = p[2];
                    h = tri_hit(p0, p1, p2, r, t, u, v);
                } else {
                    h = sphere_hit(p0, p1, r, t);
                    u = v = 0.0f;
                }
                if (h) {
                    if (ANY) return true;
                    found = true;
                    r.maxt = tb = t;
                    ub = u;
                    vb = v;
                    pb = __float_as_uint(p0.w);
                }
            }
        }
        if (sp == 0) break;
        --sp;
        ref = stk[sp * kTraceBlock];
    }
    (void)STACK;
    return found;
}

template <int STACK, bool ANY>
__global__ __launch_bounds__(kTraceBlock) void k_trace(DevScene S, const float4 *rays, uint32_t n, float4 *hits) {
    __shared__ uint32_t stk[STACK * kTraceBlock];
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
    bool h = traverse<STACK, ANY>(S, r, stk + threadIdx.x, t, p, u, v);
    if (ANY) hits[q] = make_float4(h ? 0.0f : INF_F, __uint_as_float(h ? 0u : 0xFFFFFFFFu), 0.0f, 0.0f);
    else hits[q] = make_float4(t, __uint_as_float(p), u, v);
}

// Extension rays: closest hit of every queued path.  Thread 0 also clears the
// counters the next shade launch appends to (placed here so that no extra
// launch is needed: they were last read by the previous shade / shadow).
template <int STACK>
__global__ __launch_bounds__(kTraceBlock) void k_extend(DevScene S, PathQueue pq, Counters *C, int q_sel, int reset_q,
                                                        int reset_sh) {
    __shared__ uint32_t stk[STACK * kTraceBlock];
    uint32_t q = blockIdx.x * kTraceBlock + threadIdx.x;
    if (q == 0) {
        C->qcount[reset_q] = 0;
        C->shadow_count[reset_sh] = 0;
    }
    uint32_t n = C->qcount[q_sel];
    if (q >= n) return;
    float4 a = pq.ray_o[q], b = pq.ray_d[q];
    TRay r;
    r.o = ld3(a);
    r.d = ld3(b);
    r.mint = a.w;
    r.maxt = b.w;
    float t, u, v;
    uint32_t p;
    traverse<STACK, false>(S, r, stk + threadIdx.x, t, p, u, v);
    pq.hit[q] = make_float4(t, __uint_as_float(p), u, v);
}

// Shadow rays: any hit; unoccluded -> record += payload.
template <int STACK>
__global__ __launch_bounds__(kTraceBlock) void k_shadow(DevScene S, ShadowQueue sq, Counters *C, int sh_sel,
                                                        float4 *rec) {
    __shared__ uint32_t stk[STACK * kTraceBlock];
    uint32_t q = blockIdx.x * kTraceBlock + threadIdx.x;
    uint32_t n = C->shadow_count[sh_sel];
    if (q >= n) return;
    float4 a = sq.ray_o[q], b = sq.ray_d[q];
    TRay r;
    r.o = ld3(a);
    r.d = ld3(b);
    r.mint = a.w;
    r.maxt = b.w;
    float t, u, v;
    uint32_t p;
    if (!traverse<STACK, true>(S, r, stk + threadIdx.x, t, p, u, v)) {
        float4 c = sq.payload[q];
        uint32_t w = __float_as_uint(c.w);
        float4 L = rec[w];
        rec[w] = make_float4(L.x + c.x, L.y + c.y, L.z + c.z, 0.0f);
    }
}

// ------------------------------------------------------------------ shading helpers
struct SurfHit {
    V3 p;
    Frame sh;
    int shape;
};

// setHitInformation: mesh.cpp:122-170, sphere.cpp:78-93 (shading frame only).
ND SurfHit surface(const DevScene &S, uint32_t prim, float t, float u, float v, V3 o, V3 d) {
    SurfHit h;
    h.shape = (int)S.prim_shape[prim];
    const DevShape &sh = S.shapes[h.shape];
    if (sh.type == NORI_SHAPE_SPHERE) {
        h.p = o + d * t;
        h.sh = frame_from(normalize(h.p - V3{sh.center[0], sh.center[1], sh.center[2]}));
    } else {
        const uint32_t *f = S.tri_vidx + 3 * (size_t)prim;
        uint32_t i0 = f[0], i1 = f[1], i2 = f[2];
        V3 p0 = ld3(S.pos[i0]), p1 = ld3(S.pos[i1]), p2 = ld3(S.pos[i2]);
        float bx = 1 - (u + v);
        h.p = (p0 * bx + p1 * u) + p2 * v;
        if (sh.has_normals) {
            V3 n = (ld3(S.nrm[i0]) * bx + ld3(S.nrm[i1]) * u) + ld3(S.nrm[i2]) * v;
            h.sh = frame_from(normalize(n));
        } else {
            h.sh = frame_from(normalize(cross(p1 - p0, p2 - p0)));
        }
    }
    return h;
}

// AreaEmitter (arealight.cpp:39-76)
ND float emitter_pdf(const DevScene &S, const DevEmitter &e, V3 n, V3 wi) {
    return dot(n, -wi) > 0.0f ? S.shapes[e.shape].area_norm : 0.0f;
}
ND V3 emitter_eval(const DevEmitter &e, V3 n, V3 wi) {
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

ND void camera_ray(const DevScene &S, float px, float py, V3 &o, V3 &d, float &mint, float &maxt) {
    // PerspectiveCamera::sampleRay (perspective.cpp:90-112); Eigen column order.
    const float *m = S.s2c;
    float qx = px * S.invW, qy = py * S.invH;
    float r0 = ((m[0] * qx + m[1] * qy) + m[2] * 0.0f) + m[3];
    float r1 = ((m[4] * qx + m[5] * qy) + m[6] * 0.0f) + m[7];
    float r2 = ((m[8] * qx + m[9] * qy) + m[10] * 0.0f) + m[11];
    float r3 = ((m[12] * qx + m[13] * qy) + m[14] * 0.0f) + m[15];
    V3 nearP = V3{r0 / r3, r1 / r3, r2 / r3};
    V3 dl = normalize(nearP);
    float invZ = 1.0f / dl.z;
    const float *c = S.c2w;
    float w = ((c[12] * 0.0f + c[13] * 0.0f) + c[14] * 0.0f) + c[15];
    o = V3{(((c[0] * 0.0f + c[1] * 0.0f) + c[2] * 0.0f) + c[3]) / w,
           (((c[4] * 0.0f + c[5] * 0.0f) + c[6] * 0.0f) + c[7]) / w,
           (((c[8] * 0.0f + c[9] * 0.0f) + c[10] * 0.0f) + c[11]) / w};
    d = V3{(c[0] * dl.x + c[1] * dl.y) + c[2] * dl.z, (c[4] * dl.x + c[5] * dl.y) + c[6] * dl.z,
           (c[8] * dl.x + c[9] * dl.y) + c[10] * dl.z};
    mint = S.near_clip * invZ;
    maxt = S.far_clip * invZ;
}

// ------------------------------------------------------------------ shade + regenerate
// INTEG: NORI_INTEGRATOR_PATH_MIS or NORI_INTEGRATOR_PATH_MATS.
template <int INTEG>
__global__ __launch_bounds__(kShadeBlock) void k_shade(DevScene S, PathQueue in, PathQueue out, ShadowQueue sq,
                                                       Counters *C, int in_sel, int sh_sel, WorkDesc wd,
                                                       float4 *rec) {
    const uint32_t q = blockIdx.x * kShadeBlock + threadIdx.x;
    const uint32_t n_in = C->qcount[in_sel];

    bool alive = false, shadow = false;
    V3 no = {0, 0, 0}, nd = {0, 0, 1}, beta = {1, 1, 1};
    float prev = -1.0f;
    Pcg rng = {0, 1};
    uint32_t work = 0, swork = 0;
    V3 so = {0, 0, 0}, sdir = {0, 0, 1}, contrib = {0, 0, 0};
    float smaxt = 0.0f;

    if (q < n_in) {
        float4 h = in.hit[q];
        uint32_t prim = __float_as_uint(h.y);
        work = in.work[q];
        if (prim != 0xFFFFFFFFu) {
            float4 ro = in.ray_o[q], rd = in.ray_d[q], th = in.thr[q];
            uint4 rs = in.rng[q];
            rng.state = ((uint64_t)rs.y << 32) | rs.x;
            rng.inc = ((uint64_t)rs.w << 32) | rs.z;
            V3 o = ld3(ro), d = ld3(rd);
            beta = ld3(th);
            prev = th.w;
            SurfHit hs = surface(S, prim, h.x, h.z, h.w, o, d);
            const DevShape &sh = S.shapes[hs.shape];
            const DevBsdf &B = S.bsdfs[sh.bsdf];
            V3 Ladd = {0, 0, 0};
            bool add = false;
            if (sh.emitter >= 0) {  // emission (path_mis.cpp:35-39, path_mats.cpp:31-35)
                const DevEmitter &E = S.emitters[sh.emitter];
                V3 wi = normalize(hs.p - o);
                V3 Le = emitter_eval(E, hs.sh.n, wi);
                if (INTEG == NORI_INTEGRATOR_PATH_MIS) {
                    float w = 1.0f;  // w_mats (path_mis.cpp:87-97)
                    if (prev >= 0.0f) {
                        float pe = emitter_pdf(S, E, hs.sh.n, wi);
                        w = prev + pe > 0.f ? prev / (prev + pe) : prev;
                    }
                    Ladd = (beta * w) * Le;
                } else {
                    Ladd = beta * Le;
                }
                add = true;
            }
            if (INTEG == NORI_INTEGRATOR_PATH_MIS) {  // next-event estimation (path_mis.cpp:42-61)
                float ul = next1D(rng);
                uint32_t N = S.num_emitters;
                uint32_t li = (uint32_t)floorf((float)N * ul);
                if (li > N - 1) li = N - 1;
                const DevEmitter &E = S.emitters[li];
                V2 s2 = next2D(rng);
                V3 lp, ln;
                sample_surface(S, S.shapes[E.shape], s2, lp, ln);
                V3 dv = lp - hs.p;
                V3 wi = normalize(dv);
                float pdf_em = emitter_pdf(S, E, ln, wi);
                float att = dot(ln, -wi) / dot(dv, dv);
                V3 Li = pdf_em > 0.0f ? (emitter_eval(E, ln, wi) * att) / pdf_em : V3{0, 0, 0};
                Li = Li * (float)N;
                BRec br;
                br.wi = to_local(hs.sh, -d);
                br.wo = to_local(hs.sh, wi);
                br.measure = kMeasureSolidAngle;
                float theta = smax(0.0f, br.wo.z);
                V3 f = bsdf_eval(B, br);
                float pdf_mat = bsdf_pdf(B, br);
                float w_ems = (pdf_mat + pdf_em) > 0.0f ? pdf_em / (pdf_mat + pdf_em) : pdf_em;
                contrib = (((beta * w_ems) * f) * theta) * Li;
                shadow = !is_zero(contrib);
                swork = work;
                so = hs.p;
                sdir = wi;
                smaxt = norm(dv) - kEps;
            }
            if (add) {
                float4 L = rec[work];
                rec[work] = make_float4(L.x + Ladd.x, L.y + Ladd.y, L.z + Ladd.z, 0.0f);
            }
            // Russian roulette on the red channel (path_mis.cpp:64-69)
            float qrr = smin(beta.x, 0.99f);
            if (!(next1D(rng) > qrr)) {
                beta = beta / qrr;
                BRec br;
                br.wi = to_local(hs.sh, -d);
                br.wo = V3{0, 0, 1};
                br.measure = kMeasureUnknown;
                V3 w = bsdf_sample(B, br, next2D(rng));
                if (!is_zero(w)) {  // deviation D1: zero-weight samples end the path
                    beta = beta * w;
                    if (INTEG == NORI_INTEGRATOR_PATH_MIS) {
                        float pm = bsdf_pdf(B, br);
                        prev = br.measure == kMeasureDiscrete ? -1.0f : pm;
                    }
                    no = hs.p;
                    nd = to_world(hs.sh, br.wo);
                    alive = true;
                }
            }
        }
    }

    // ---- regenerate finished slots from the work counter (one atomic per wave)
    bool need = !alive;
    uint64_t mneed = __ballot(need);
    unsigned long long base = wave_reserve64(&C->next_work, mneed);
    float nmint = kEps, nmaxt = INF_F;
    if (need) {
        unsigned long long w = base + rank_in(mneed);
        if (w < wd.total) {
            work = (uint32_t)w;
            uint32_t pass = work / wd.M, e = work - pass * wd.M;
            uint32_t pix = wd.pixels[e];
            uint32_t W = (uint32_t)S.W;
            uint32_t y = pix / W, x = pix - y * W;
            uint64_t sid = (uint64_t)(wd.pass_begin + pass) * ((uint64_t)S.W * (uint64_t)S.H) + pix;
            wave_seed(rng, wd.seed, sid);
            V2 jit = next2D(rng);
            (void)next2D(rng);  // apertureSample (render.cpp:99)
            camera_ray(S, (float)x + jit.x, (float)y + jit.y, no, nd, nmint, nmaxt);
            beta = V3{1, 1, 1};
            prev = -1.0f;
            rec[work] = make_float4(0, 0, 0, 0);
            alive = true;
        }
    }

    // ---- compact shadow rays and surviving paths
    uint64_t msh = __ballot(shadow);
    uint32_t sbase = wave_reserve(&C->shadow_count[sh_sel], msh);
    if (shadow) {
        uint32_t i = sbase + rank_in(msh);
        sq.ray_o[i] = make_float4(so.x, so.y, so.z, kEps);
        sq.ray_d[i] = make_float4(sdir.x, sdir.y, sdir.z, smaxt);
        sq.payload[i] = make_float4(contrib.x, contrib.y, contrib.z, __uint_as_float(swork));
    }
    uint64_t mal = __ballot(alive);
    uint32_t obase = wave_reserve(&C->qcount[in_sel ^ 1], mal);
    if (lane_id() == 0 && (mal | msh)) {
        if (mal) atomicAdd(&C->rays_closest, (unsigned long long)__popcll(mal));
        if (msh) atomicAdd(&C->rays_shadow, (unsigned long long)__popcll(msh));
    }
    if (alive) {
        uint32_t i = obase + rank_in(mal);
        out.ray_o[i] = make_float4(no.x, no.y, no.z, nmint);
        out.ray_d[i] = make_float4(nd.x, nd.y, nd.z, nmaxt);
        out.thr[i] = make_float4(beta.x, beta.y, beta.z, prev);
        out.rng[i] = make_uint4((uint32_t)rng.state, (uint32_t)(rng.state >> 32), (uint32_t)rng.inc, (uint32_t)(rng.inc >> 32));
        out.work[i] = work;
    }
}

// ------------------------------------------------------------------ film splat
// ImageBlock::put(pos, val) (block.cpp:93-122) into an LDS tile per 32x32
// block, then ImageBlock::put(block) (block.cpp:124-133) into the film.
__global__ __launch_bounds__(kSplatBlock) void k_splat(DevScene S, const float4 *rec, SplatDesc sd, float *film,
                                                      Counters *C) {
    extern __shared__ float tile[];
    __shared__ float ftab[NORI_FILTER_RESOLUTION + 1];
    const int B = S.border, TS = NORI_BLOCK_SIZE + 2 * B;
    int4 bi = sd.blocks[blockIdx.x];
    int ox = bi.x, oy = bi.y, bw = bi.z & 0xFFFF, bh = bi.z >> 16;
    uint32_t off = (uint32_t)bi.w;
    uint32_t p0 = blockIdx.y * sd.passes_per_wg, p1 = min(sd.passes, p0 + sd.passes_per_wg);
    for (int i = threadIdx.x; i < TS * TS * 4; i += kSplatBlock) tile[i] = 0.0f;
    if (threadIdx.x <= NORI_FILTER_RESOLUTION) ftab[threadIdx.x] = S.filter[threadIdx.x];
    __syncthreads();
    const uint32_t npix = (uint32_t)(bw * bh);
    const uint32_t n = (p1 - p0) * npix;
    const float rad = S.filter_radius, lk = S.lookup;
    const uint64_t WH = (uint64_t)S.W * (uint64_t)S.H;
    uint32_t inval = 0;
    for (uint32_t i = threadIdx.x; i < n; i += kSplatBlock) {
        uint32_t pl = i / npix, j = i - pl * npix;
        uint32_t p = p0 + pl;
        int ly = (int)(j / (uint32_t)bw), lx = (int)(j - (uint32_t)ly * (uint32_t)bw);
        float4 L = rec[(size_t)p * sd.M + off + j];
        int x = ox + lx, y = oy + ly;
        uint64_t sid = (uint64_t)(sd.pass_begin + p) * WH + (uint64_t)y * S.W + x;
        Pcg r;
        wave_seed(r, sd.seed, sid);
        V2 jit = next2D(r);
        float psx = (float)x + jit.x, psy = (float)y + jit.y;
        // Color3f::isValid (common.cpp:224-231)
        bool valid = !(L.x < 0 || !isfinite(L.x) || L.y < 0 || !isfinite(L.y) || L.z < 0 || !isfinite(L.z));
        if (!valid) {
            ++inval;
            continue;
        }
        float px = psx - 0.5f - (float)(ox - B), py = psy - 0.5f - (float)(oy - B);
        int x0 = max((int)ceilf(px - rad), 0), y0 = max((int)ceilf(py - rad), 0);
        int x1 = min((int)floorf(px + rad), TS - 1), y1 = min((int)floorf(py + rad), TS - 1);
        for (int yy = y0; yy <= y1; ++yy) {
            float wy = ftab[(int)(fabsf((float)yy - py) * lk)];
            for (int xx = x0; xx <= x1; ++xx) {
                float wx = ftab[(int)(fabsf((float)xx - px) * lk)];
                float *c = tile + 4 * (yy * TS + xx);
                atomicAdd(c + 0, (L.x * wx) * wy);
                atomicAdd(c + 1, (L.y * wx) * wy);
                atomicAdd(c + 2, (L.z * wx) * wy);
                atomicAdd(c + 3, (1.0f * wx) * wy);
            }
        }
    }
    if (inval) atomicAdd(&C->invalid, (unsigned long long)inval);
    __syncthreads();
    const int rows = bh + 2 * B, cols = bw + 2 * B, FW = S.W + 2 * B;
    for (int i = threadIdx.x; i < rows * cols; i += kSplatBlock) {
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
template <bool ANY>
static hipError_t trace_dispatch(const DevScene &S, const float4 *rays, uint32_t n, float4 *hits, int stack,
                                 hipStream_t st) {
    dim3 g((n + kTraceBlock - 1) / kTraceBlock), b(kTraceBlock);
    switch (stack) {
    case 8: hipLaunchKernelGGL((k_trace<8, ANY>), g, b, 0, st, S, rays, n, hits); break;
    case 16: hipLaunchKernelGGL((k_trace<16, ANY>), g, b, 0, st, S, rays, n, hits); break;
    case 32: hipLaunchKernelGGL((k_trace<32, ANY>), g, b, 0, st, S, rays, n, hits); break;
    default: hipLaunchKernelGGL((k_trace<64, ANY>), g, b, 0, st, S, rays, n, hits); break;
    }
    return hipGetLastError();
}
hipError_t launch_trace(const DevScene &S, const float4 *rays, uint32_t n, int any_hit, float4 *hits, int stack,
                        hipStream_t st) {
    if (n == 0) return hipSuccess;
    return any_hit ? trace_dispatch<true>(S, rays, n, hits, stack, st)
                   : trace_dispatch<false>(S, rays, n, hits, stack, st);
}

hipError_t launch_shade(const DevScene &S, const PathQueue &in, const PathQueue &out, const ShadowQueue &sq,
                        Counters *C, int in_sel, int sh_sel, const WorkDesc &wd, float4 *rec, uint32_t pool,
                        hipStream_t st) {
    dim3 g(pool / kShadeBlock), b(kShadeBlock);
    if (S.integrator == NORI_INTEGRATOR_PATH_MATS)
        hipLaunchKernelGGL((k_shade<NORI_INTEGRATOR_PATH_MATS>), g, b, 0, st, S, in, out, sq, C, in_sel, sh_sel, wd, rec);
    else
        hipLaunchKernelGGL((k_shade<NORI_INTEGRATOR_PATH_MIS>), g, b, 0, st, S, in, out, sq, C, in_sel, sh_sel, wd, rec);
    return hipGetLastError();
}

hipError_t launch_extend(const DevScene &S, const PathQueue &q, Counters *C, int q_sel, int reset_q, int reset_sh,
                         uint32_t pool, int stack, hipStream_t st) {
    dim3 g(pool / kTraceBlock), b(kTraceBlock);
    switch (stack) {
    case 8: hipLaunchKernelGGL(k_extend<8>, g, b, 0, st, S, q, C, q_sel, reset_q, reset_sh); break;
    case 16: hipLaunchKernelGGL(k_extend<16>, g, b, 0, st, S, q, C, q_sel, reset_q, reset_sh); break;
    case 32: hipLaunchKernelGGL(k_extend<32>, g, b, 0, st, S, q, C, q_sel, reset_q, reset_sh); break;
    default: hipLaunchKernelGGL(k_extend<64>, g, b, 0, st, S, q, C, q_sel, reset_q, reset_sh); break;
    }
    return hipGetLastError();
}

hipError_t launch_shadow(const DevScene &S, const ShadowQueue &sq, Counters *C, int sh_sel, float4 *rec,
                         uint32_t pool, int stack, hipStream_t st) {
    dim3 g(pool / kTraceBlock), b(kTraceBlock);
    switch (stack) {
    case 8: hipLaunchKernelGGL(k_shadow<8>, g, b, 0, st, S, sq, C, sh_sel, rec); break;
    case 16: hipLaunchKernelGGL(k_shadow<16>, g, b, 0, st, S, sq, C, sh_sel, rec); break;
    case 32: hipLaunchKernelGGL(k_shadow<32>, g, b, 0, st, S, sq, C, sh_sel, rec); break;
    default: hipLaunchKernelGGL(k_shadow<64>, g, b, 0, st, S, sq, C, sh_sel, rec); break;
    }
    return hipGetLastError();
}

hipError_t launch_splat(const DevScene &S, const float4 *rec, const SplatDesc &sd, uint32_t nblocks, float *film,
                        Counters *C, hipStream_t st) {
    if (nblocks == 0 || sd.passes == 0) return hipSuccess;
    int TS = NORI_BLOCK_SIZE + 2 * S.border;
    size_t lds = sizeof(float) * 4 * (size_t)TS * TS;
    dim3 g(nblocks, (sd.passes + sd.passes_per_wg - 1) / sd.passes_per_wg), b(kSplatBlock);
    hipLaunchKernelGGL(k_splat, g, b, lds, st, S, rec, sd, film, C);
    return hipGetLastError();
}

}  // namespace nori
