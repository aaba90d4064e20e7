// device_math.h -- fp32 vector math, pcg32, warps, frames, BSDFs and the area
// emitter for the gfx950 kernels.  Each routine restates the reference function
// cited beside it (paths relative to the reference checkout).  The file is
// compiled with -ffp-contract=off so +,-,*,/ and sqrt round exactly as in the
// reference's x86-64 build; transcendentals come from the ROCm device library
// and may differ from glibc by a few ulp.
#pragma once
#ifndef __HIPCC_RTC__  // (hipRTC: the runtime header is built in)
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>

#include "../../include/nori_gpu.h"

#define ND __device__ __forceinline__
#define NHD __host__ __device__ __forceinline__

namespace nori {

constexpr float kPi = 3.14159265358979323846f;      // common.h:56 (float literal)
constexpr float kInvPi = 0.31830988618379067154f;   // common.h:57
constexpr float kInvFourPi = 0.07957747154594766788f;
constexpr float kEps = NORI_EPSILON;                // common.h:52

struct V3 {
    float x, y, z;
};
NHD V3 v3(float x, float y, float z) { return V3{x, y, z}; }
NHD V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
NHD V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
NHD V3 operator-(V3 a) { return V3{-a.x, -a.y, -a.z}; }
NHD V3 operator*(V3 a, float s) { return V3{a.x * s, a.y * s, a.z * s}; }
NHD V3 operator*(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
NHD V3 operator/(V3 a, float s) { return V3{a.x / s, a.y / s, a.z / s}; }
// Eigen's redux order for 3-vectors: (a0 + a1) + a2
NHD float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
NHD V3 cross(V3 a, V3 b) {
    return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// sqrtf, correctly rounded, in a shorter dependent chain: v_sqrt_f32 (about
// 1 ulp) then one Tuckerman test each way (29 instead of 52 ns of lone-lane
// latency, tools/latency_probe.hip).  Bit-identical to the IEEE sqrtf for
// every float in [2^-96, 2^96) (tools/sqrt_check.hip, exhaustive); the IEEE
// sequence runs outside that range.  FAST = true selects it in the templates
// below (the tail finisher's glass-sphere chain, kernels.hip glass_bounce).
NHD float sqrt_rn(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    if (__builtin_expect(!(x >= 0x1p-96f && x < 0x1p96f), 0)) return sqrtf(x);
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    const float rd = __builtin_fmaf(-sd, s, x), ru = __builtin_fmaf(-su, s, x);
    const float r = rd <= 0.0f ? sd : s;
    return ru > 0.0f ? su : r;
#else
    return sqrtf(x);
#endif
}
template <bool FAST = false>
NHD float fsqrt(float x) {
    if constexpr (FAST) return sqrt_rn(x);
    else return sqrtf(x);
}
NHD float norm(V3 a) { return sqrtf(dot(a, a)); }
template <bool FAST = false>
NHD V3 normalize(V3 a) { return a / fsqrt<FAST>(dot(a, a)); }  // MatrixBase::normalized()
NHD float smax(float a, float b) { return (a < b) ? b : a; }  // std::max
NHD float smin(float a, float b) { return (b < a) ? b : a; }  // std::min
NHD float maxc(V3 a) { return smax(smax(a.x, a.y), a.z); }
NHD bool is_zero(V3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
NHD float luminance(V3 c) {  // common.cpp:233-235
    return c.x * 0.212671f + c.y * 0.715160f + c.z * 0.072169f;
}
NHD float clampf_(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
ND V3 ld3(const float4 &f) { return V3{f.x, f.y, f.z}; }
// 1.0f / x, correctly rounded: v_rcp_f32 (~1 ulp) and one FMA Newton step
// (3 VALU instead of the 9 of the IEEE division sequence).  Verified
// bit-identical to the IEEE quotient for every float with |x| in
// [2^-125, 2^125] by tools/rcp_check.hip; outside that range (and for
// inf/NaN) the IEEE division runs.  Below 2^-125 the triangle test never
// uses the value (|det| < 1e-8 is rejected, mesh.cpp:96).
ND float rcp_rn(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    if (__builtin_expect(!(__builtin_fabsf(x) <= 0x1p125f), 0)) return 1.0f / x;
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
#else
    return 1.0f / x;
#endif
}

// 1.0f / x for every float x: rcp_rn inside the verified range, the IEEE
// division outside it (zero, denormals, |x| > 2^125, inf, NaN) -- so the
// result is always the IEEE quotient.  Used where x may be zero (ray
// direction components: the slab test's d_i == 0 case, bbox.h:344-346).
NHD float rcp_full(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    const float a = __builtin_fabsf(x);
    if (__builtin_expect(!(a >= 0x1p-125f && a <= 0x1p125f), 0)) return 1.0f / x;
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
#else
    return 1.0f / x;
#endif
}

// ---------------------------------------------------------------- pcg32
// ext/pcg32/pcg32.h:51-110.  The increment of a WAVE stream is derived from
// its sample id, so a path only carries the 64-bit state.
constexpr uint64_t kPcgMult = 0x5851f42d4c957f2dULL;
struct Pcg {
    uint64_t state, inc;
};
NHD uint32_t pcg_next(Pcg &r) {
    uint64_t old = r.state;
    r.state = old * kPcgMult + r.inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((-rot) & 31));
}
NHD void pcg_seed(Pcg &r, uint64_t initstate, uint64_t initseq) {
    r.state = 0u;
    r.inc = (initseq << 1u) | 1u;
    pcg_next(r);
    r.state += initstate;
    pcg_next(r);
}
NHD void pcg_skip(Pcg &r, int n) {  // n draws whose values are not needed
    for (int i = 0; i < n; ++i) r.state = r.state * kPcgMult + r.inc;
}
// Three draws skipped in one step: s3 = A^3 s + (A^2 + A + 1) inc (mod 2^64),
// the same state as pcg_skip(r, 3); the increment term does not depend on
// the state, so the dependent chain is one 64-bit multiply-add instead of three.
constexpr uint64_t kPcgMult3 = kPcgMult * kPcgMult * kPcgMult;
constexpr uint64_t kPcgInc3 = kPcgMult * kPcgMult + kPcgMult + 1u;
NHD void pcg_skip3(Pcg &r) { r.state = r.state * kPcgMult3 + r.inc * kPcgInc3; }
NHD float pcg_float(Pcg &r) {
    uint32_t u = (pcg_next(r) >> 9) | 0x3f800000u;
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f - 1.0f;
}
NHD uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
// WAVE stream of camera sample `sample_id` (same definition as the oracle).
NHD void wave_seed(Pcg &r, uint64_t seed, uint64_t sample_id) {
    pcg_seed(r, splitmix64(sample_id ^ seed), sample_id);
}
struct V2 {
    float x, y;
};
// Sampler::next1D / next2D (independent.cpp:58-67): x drawn first.
NHD float next1D(Pcg &r) { return pcg_float(r); }
NHD V2 next2D(Pcg &r) {
    V2 s;
    s.x = pcg_float(r);
    s.y = pcg_float(r);
    return s;
}

// ---------------------------------------------------------------- jitter classes
// ImageBlock::put (block.cpp:93-122) places a sample of pixel x in block
// offset ox at P = fl(fl(fl(x + jit) - 0.5) - (ox - border)) and weighs tile
// cell c by filter[(int)(|c - P| * lookup)] when
// ceil(P - r) <= c <= floor(P + r).  With a power-of-two radius r and lookup
// factor every later step is exact -- c - P and f = P - floor(P) share P's grid
// and are no larger, the products are by powers of two -- except
// fl(P +- r), which can round across an integer only where |c - P| >= r,
// i.e. at index NORI_FILTER_RESOLUTION, whose weight is 0.  So the weights of
// the window cells depend only on (floor(P) - (x - ox) - border + 1 in {0, 1},
// [f * lookup integer], q = floor(f * lookup)): for j = c - floor(P) >= 1
// the index is j * lookup - ceil(f * lookup), for j <= 0 it is
// |j| * lookup + q, and the box's ends are floor(P) + ceil(f - r) and
// floor(P) + floor(f + r).  jit_class packs that triple into 8 bits
// (lookup <= 64); k_splat expands a class into its weights with a
// representative f of the same triple (tests/test_jit_class.py checks the
// weights against the direct formula on every pixel column).
constexpr uint32_t kRecPending = 0x80000000u;  // sample record w bit 31: the finisher splats it
NHD uint32_t jit_class(uint32_t x, float jit, float lk, int border) {
    const int ox = (int)(x / NORI_BLOCK_SIZE) * NORI_BLOCK_SIZE;
    const float P = ((float)x + jit) - 0.5f - (float)(ox - border);
    const float n = floorf(P), f = P - n, qf = f * lk, q = floorf(qf);
    return (uint32_t)((int)n - ((int)x - ox) - border + 1) | (q == qf ? 2u : 0u) | (uint32_t)q << 2;
}
// The w word of a new sample record: both classes (S.jit_lk != 0) or 0.
NHD float rec_code(int lk, int border, uint32_t x, uint32_t y, V2 jit) {
    if (!lk) return 0.0f;
    const uint32_t c = jit_class(x, jit.x, (float)lk, border) | jit_class(y, jit.y, (float)lk, border) << 8;
    float w;
    __builtin_memcpy(&w, &c, 4);
    return w;
}

// ---------------------------------------------------------------- frames
struct Frame {
    V3 s, t, n;
};
template <bool FAST = false>
NHD Frame frame_from(V3 a) {  // frame.h:49-51 + coordinateSystem common.cpp:274-283
    Frame f;
    f.n = a;
    if (fabsf(a.x) > fabsf(a.y)) {
        float invLen = rcp_full(fsqrt<FAST>(a.x * a.x + a.z * a.z));
        f.t = V3{a.z * invLen, 0.0f, -a.x * invLen};
    } else {
        float invLen = rcp_full(fsqrt<FAST>(a.y * a.y + a.z * a.z));
        f.t = V3{0.0f, a.z * invLen, -a.y * invLen};
    }
    f.s = cross(f.t, a);
    return f;
}
NHD V3 to_local(const Frame &f, V3 v) { return V3{dot(v, f.s), dot(v, f.t), dot(v, f.n)}; }
NHD V3 to_world(const Frame &f, V3 v) { return (f.s * v.x + f.t * v.y) + f.n * v.z; }
NHD float tan_theta(V3 v) {  // frame.h:77-82
    float temp = 1 - v.z * v.z;
    if (temp <= 0.0f) return 0.0f;
    return sqrtf(temp) / v.z;
}

// fresnel (common.cpp:285-314) with etaI / etaT taken from the precomputed
// quotients (eta_ei = extIOR / intIOR, eta_ie = intIOR / extIOR)
template <bool FAST = false>
NHD float fresnel(float cosThetaI, float extIOR, float intIOR, float eta_ei, float eta_ie) {
    float etaI = extIOR, etaT = intIOR, eta = eta_ei;
    if (extIOR == intIOR) return 0.0f;
    if (cosThetaI < 0.0f) {
        float t = etaI;
        etaI = etaT;
        etaT = t;
        eta = eta_ie;
        cosThetaI = -cosThetaI;
    }
    float sinThetaTSqr = eta * eta * (1 - cosThetaI * cosThetaI);
    if (sinThetaTSqr > 1.0f) return 1.0f;
    float cosThetaT = fsqrt<FAST>(1.0f - sinThetaTSqr);
    float Rs = (etaI * cosThetaI - etaT * cosThetaT) / (etaI * cosThetaI + etaT * cosThetaT);
    float Rp = (etaT * cosThetaI - etaI * cosThetaT) / (etaT * cosThetaI + etaI * cosThetaT);
    return (Rs * Rs + Rp * Rp) / 2.0f;
}

// ---------------------------------------------------------------- warps
NHD V3 sq_cosine_hemisphere(V2 s) {  // warp.cpp:110-115
    float theta = acosf(sqrtf(1 - (1 - s.x)));
    float phi = 2.f * kPi * s.y;
    float st = sinf(theta);
    return V3{st * cosf(phi), st * sinf(phi), cosf(theta)};
}
NHD V3 sq_uniform_sphere(V2 s) {  // warp.cpp:86-91
    float theta = acosf(1 - 2 * (1 - s.x));
    float phi = 2.f * kPi * s.y;
    float st = sinf(theta);
    return V3{st * cosf(phi), st * sinf(phi), cosf(theta)};
}
NHD float sq_uniform_sphere_pdf(V3 v) {  // warp.cpp:93-96
    return fabsf(norm(v) - 1.0f) < kEps ? 0.25f * kInvPi : 0.0f;
}
NHD V3 sq_beckmann(V2 s, float alpha) {  // warp.cpp:122-127 (pow(alpha,2) is double)
    double a2 = (double)alpha * (double)alpha;
    float theta = (float)atan(sqrt(-a2 * (double)logf(1 - s.x)));
    float phi = 2 * kPi * s.y;
    float st = sinf(theta);
    return V3{st * cosf(phi), st * sinf(phi), cosf(theta)};
}
// Warp::squareToConcentricDisk (warp.cpp:143-162), squareToUniformDisk (warp.cpp:53-58)
NHD V2 sq_concentric_disk(V2 s) {
    const V2 o = V2{2.f * s.x - 1.f, 2.f * s.y - 1.f};
    if (o.x == 0.0f && o.y == 0.0f) return V2{0, 0};
    float theta, r;
    if (fabsf(o.x) > fabsf(o.y)) {
        r = o.x;
        theta = kPi * 0.25f * (o.y / o.x);
    } else {
        r = o.y;
        theta = kPi * 0.5f - kPi * 0.25f * (o.x / o.y);
    }
    return V2{r * cosf(theta), r * sinf(theta)};
}
NHD V2 sq_uniform_disk(V2 s) {
    const float angle = 2 * s.x * kPi, size = sqrtf(s.y);
    return V2{cosf(angle) * size, sinf(angle) * size};
}
NHD V3 sq_uniform_triangle(V2 s) {  // warp.cpp:135-140
    float su1 = sqrtf(s.x);
    float u = 1.f - su1, v = s.y * su1;
    return V3{u, v, 1.f - u - v};
}
NHD V3 sq_gtr2(V2 s, float alpha) {  // warp.cpp:180-185
    float a2 = alpha * alpha;  // (float)pow(alpha,2): exact product rounded once
    float theta = acosf(sqrtf((1.0f - s.x) / (1.0f + (a2 - 1.0f) * s.x)));
    float phi = 2 * kPi * s.y;
    float st = sinf(theta);
    return V3{st * cosf(phi), st * sinf(phi), cosf(theta)};
}
NHD float sq_gtr2_pdf(V3 m, float alpha) {  // warp.cpp:187-193
    float a2 = alpha * alpha;
    float cosTheta = m.z;
    double base = 1.0 + (double)(a2 - 1.0f) * ((double)cosTheta * (double)cosTheta);
    float pdf = (float)((double)(a2 * cosTheta * kInvPi) / (base * base));
    return (cosTheta >= 0 && fabsf(dot(m, m) - 1.0f) < 1.0f) ? pdf : 0.0f;
}

// ---------------------------------------------------------------- BSDFs
enum { kMeasureUnknown = 0, kMeasureSolidAngle = 1, kMeasureDiscrete = 2 };  // common.h:199-203

// Device BSDF record: desc values plus derived constants.
struct DevBsdf {
    int32_t type;
    float albedo[3];
    float int_ior, ext_ior, alpha, ks;
    float kd[3];
    float base[3];
    float metallic, specular, roughness, sheen, sheen_tint, spec_tint, d_alpha;
    int32_t tex;  // diffuse albedo: NORI_TEXTURE_CONSTANT (albedo), _CHECKERBOARD (albedo = value1) or _IMAGE
    float tex_v2[3], tex_delta[2], tex_scale[2];
    int32_t img_w, img_h, img_wrap;  // NORI_TEXTURE_IMAGE: RGBX8 texels in global memory
    const uint32_t *img;
    // the IOR quotients fresnel() and Dielectric::sample compute per call,
    // computed once on the host with the same float divisions:
    // ext/int, int/ext and 1.0f / (ext/int)
    float eta_ei, eta_ie, inv_eta_ei;
};

// ImageTexture::getData / NormalMap::getData (imagetexture.cpp:95-115): the
// texel (int)(u W), (int)(v H), repeated (C++ %) or clamped.  eval's bilinear
// weights are uv*W - (float)(uv*W) = 0 (imagetexture.cpp:118-134), so eval is
// this one texel.  A negative coordinate under "repeat" indexes before the
// image in the reference (undefined); it is wrapped into range here.
ND uint32_t texel_at(const uint32_t *img, int W, int H, int wrap, V2 uv) {
    const float x = uv.x * (float)W, y = uv.y * (float)H;
    int ix, iy;
    if (wrap == NORI_WRAP_REPEAT) {
        ix = (int)x % W;
        iy = (int)y % H;
        ix += ix < 0 ? W : 0;
        iy += iy < 0 ? H : 0;
    } else {
        ix = min(max((int)x, 0), W - 1);
        iy = min(max((int)y, 0), H - 1);
    }
    return img[(size_t)iy * W + ix];
}
// static_cast<float>(byte) / UCHAR_MAX per channel
ND V3 texel_rgb(uint32_t t) {
    return V3{(float)(t & 255u) / 255.0f, (float)((t >> 8) & 255u) / 255.0f, (float)((t >> 16) & 255u) / 255.0f};
}

struct BRec {
    V3 wi, wo;
    int measure;
    V2 uv;  // bsdf.h:55, the hit's texture coordinates
};

// Texture<Color3f>::eval: constant (consttexture.cpp), Checkerboard::eval
// (checkerboard.cpp:22-27) or ImageTexture::eval (imagetexture.cpp:118-134)
// FULL = false: the "basic" plugin set of the path kernels' lite variants
// (scenes with constant-albedo diffuse, mirror and dielectric BSDFs only,
// area lights, the perspective camera; runtime.hip basic_scene): the code of
// the other plugins is not compiled in, so the kernels stay small (their
// instruction working set fits the instruction cache, which the lone-lane
// tail paths of k_finish are bound by).
template <bool FULL = true>
ND V3 albedo_at(const DevBsdf &b, V2 uv) {
    if (!FULL) return V3{b.albedo[0], b.albedo[1], b.albedo[2]};
    if (b.tex == NORI_TEXTURE_IMAGE) return texel_rgb(texel_at(b.img, b.img_w, b.img_h, b.img_wrap, uv));
    if (b.tex != NORI_TEXTURE_CHECKERBOARD) return V3{b.albedo[0], b.albedo[1], b.albedo[2]};
    const int x = (int)fabsf(floorf(uv.x / b.tex_scale[0] - b.tex_delta[0]));
    const int y = (int)fabsf(floorf(uv.y / b.tex_scale[1] - b.tex_delta[1]));
    return x % 2 == y % 2 ? V3{b.albedo[0], b.albedo[1], b.albedo[2]} : V3{b.tex_v2[0], b.tex_v2[1], b.tex_v2[2]};
}

ND float beckmann_D(const DevBsdf &b, V3 m) {  // microfacet.cpp:47-53
    float temp = tan_theta(m) / b.alpha, ct = m.z, ct2 = ct * ct;
    return expf(-temp * temp) / (kPi * b.alpha * b.alpha * ct2 * ct2);
}
ND float smith_G1(const DevBsdf &b, V3 v, V3 m) {  // microfacet.cpp:56-76
    float tanTheta = tan_theta(v);
    if (tanTheta == 0.0f) return 1.0f;
    if (dot(m, v) * v.z <= 0) return 0.0f;
    float a = rcp_full(b.alpha * tanTheta);
    if (a >= 1.6f) return 1.0f;
    float a2 = a * a;
    return (3.535f * a + 2.181f * a2) / (1.0f + 2.276f * a + 2.577f * a2);
}
ND float schlick(float u) {  // disney.cpp:25-29: pow(m, 5) in double
    double m = (double)clampf_(1 - u, 0.0f, 1.0f);
    double m2 = m * m;
    return (float)(m2 * m2 * m);
}
ND float ggx(float NdotV, float alphaG) {  // disney.cpp:31-36
    float a = alphaG * alphaG, b = NdotV * NdotV;
    return rcp_full(NdotV + sqrtf(a + b - a * b));
}
ND V3 lerp3(float t, V3 a, V3 c) { return a * (1.0f - t) + c * t; }  // disney.cpp:40-42

template <bool FULL = true>
ND V3 bsdf_eval(const DevBsdf &b, const BRec &r) {
    switch (b.type) {
    case NORI_BSDF_DIFFUSE:  // diffuse.cpp:72-82
        if (r.measure != kMeasureSolidAngle || r.wi.z <= 0 || r.wo.z <= 0) return V3{0, 0, 0};
        return albedo_at<FULL>(b, r.uv) * kInvPi;
    case NORI_BSDF_MICROFACET: {  // microfacet.cpp:79-90
        if constexpr (!FULL) return V3{0, 0, 0};
        V3 n = normalize(r.wi + r.wo);
        float D = beckmann_D(b, n);
        float F = fresnel(dot(n, r.wi), b.ext_ior, b.int_ior, b.eta_ei, b.eta_ie);
        float G = smith_G1(b, r.wi, n) * smith_G1(b, r.wo, n);
        float den = 4.0f * r.wi.z * r.wo.z;
        float spec = b.ks * D * F * G / den;
        V3 d = V3{b.kd[0], b.kd[1], b.kd[2]} * kInvPi;
        return V3{d.x + spec, d.y + spec, d.z + spec};
    }
    case NORI_BSDF_DISNEY: {  // disney.cpp:63-114
        if constexpr (!FULL) return V3{0, 0, 0};
        float NdotV = r.wi.z, NdotL = r.wo.z;
        if (NdotV < 0 || NdotL < 0) return V3{0, 0, 0};
        V3 wh = normalize(r.wi + r.wo);
        float LdotH = dot(r.wo, wh), VdotH = dot(r.wi, wh);
        V3 base = V3{b.base[0], b.base[1], b.base[2]};
        float l = luminance(base);
        V3 white = V3{1, 1, 1};
        V3 ctint = (l > 0.f) ? V3{base.x / l, base.y / l, base.z / l} : white;
        float smix = (float)((double)b.specular * 0.08);
        V3 cspec = lerp3(b.metallic, lerp3(b.spec_tint, white, ctint) * smix, base);
        float fd90 = (float)(0.5 + (double)(2 * b.roughness) * ((double)VdotH * (double)VdotH));
        float fl = schlick(NdotL), fv = schlick(NdotV);
        V3 diffuse = ((base * kInvPi) * (1.f + (fd90 - 1.f) * fl)) * (1.f + (fd90 - 1.f) * fv);
        float alpha = smax(0.001f, b.roughness * b.roughness);
        float Ds = sq_gtr2_pdf(wh, alpha);
        float FH = schlick(LdotH);
        V3 Fs = lerp3(FH, cspec, white);
        float Gs = ggx(NdotL, alpha) * ggx(NdotV, alpha);
        V3 specular = (Fs * Gs) * Ds;
        V3 fsheen = lerp3(b.sheen_tint, white, ctint) * (FH * b.sheen);
        return (diffuse + fsheen) * (1 - b.metallic) + specular;
    }
    default:  // mirror / dielectric: discrete lobes evaluate to zero
        return V3{0, 0, 0};
    }
}

template <bool FULL = true>
ND float bsdf_pdf(const DevBsdf &b, const BRec &r) {
    switch (b.type) {
    case NORI_BSDF_DIFFUSE:  // diffuse.cpp:85-98
        if (r.measure != kMeasureSolidAngle || r.wi.z <= 0 || r.wo.z <= 0) return 0.0f;
        return kInvPi * r.wo.z;
    case NORI_BSDF_MICROFACET: {  // microfacet.cpp:93-106
        if constexpr (!FULL) return 0.0f;
        float c = r.wo.z;
        if (c <= 0.0f) return 0.0f;
        V3 n = normalize(r.wi + r.wo);
        float mt = beckmann_D(b, n) * n.z / (4.0f * fabsf(dot(n, r.wo)));
        return b.ks * mt + (1 - b.ks) * (c * kInvPi);
    }
    case NORI_BSDF_DISNEY: {  // disney.cpp:117-129
        if constexpr (!FULL) return 0.0f;
        float c = r.wo.z;
        if (c <= 0.0f) return 0.0f;
        V3 n = normalize(r.wi + r.wo);
        float mt = sq_gtr2_pdf(n, b.d_alpha) * n.z / (4.0f * fabsf(dot(n, r.wo)));
        return (1 - b.metallic) * (c * kInvPi) + b.metallic * mt;
    }
    default:
        return 0.0f;
    }
}

// Dielectric::sample's direction (dielectric.cpp:45-73; weight 1, discrete)
template <bool FAST = false>
ND V3 dielectric_wo(const DevBsdf &b, V3 wi, V2 s) {
    float theta = wi.z;
    V3 nv = V3{0, 0, 1.0f};
    if (fresnel<FAST>(theta, b.ext_ior, b.int_ior, b.eta_ei, b.eta_ie) > s.x) return V3{-wi.x, -wi.y, wi.z};
    float factor = b.eta_ei;  // ext / int
    if (theta < 0.0f) {
        factor = b.inv_eta_ei;  // 1 / factor
        nv.z *= -1;
    }
    V3 part1 = (wi - nv * dot(wi, nv)) * (-factor);
    double wn = (double)dot(wi, nv);
    double rad = 1.0 - (double)factor * (double)factor * (1.0 - wn * wn);
    V3 part2 = (-nv) * (float)sqrt(rad);
    return normalize<FAST>(part1 + part2);
}

// Returns the sample weight; r.wo / r.measure are set as the reference sets them.
template <bool FULL = true>
ND V3 bsdf_sample(const DevBsdf &b, BRec &r, V2 s) {
    switch (b.type) {
    case NORI_BSDF_DIFFUSE:  // diffuse.cpp:101-116
        if (r.wi.z <= 0) return V3{0, 0, 0};
        r.measure = kMeasureSolidAngle;
        r.wo = sq_cosine_hemisphere(s);
        return albedo_at<FULL>(b, r.uv);
    case NORI_BSDF_MIRROR:  // mirror.cpp:39-55
        if (r.wi.z <= 0) return V3{0, 0, 0};
        r.wo = V3{-r.wi.x, -r.wi.y, r.wi.z};
        r.measure = kMeasureDiscrete;
        return V3{1, 1, 1};
    case NORI_BSDF_DIELECTRIC:  // dielectric.cpp:45-73
        r.wo = dielectric_wo(b, r.wi, s);
        r.measure = kMeasureDiscrete;
        return V3{1, 1, 1};
    case NORI_BSDF_MICROFACET: {  // microfacet.cpp:109-131
        if constexpr (!FULL) return V3{0, 0, 0};
        if (r.wi.z <= 0.0f) return V3{0, 0, 0};
        if (s.x < b.ks) {
            V3 n = sq_beckmann(V2{s.x / b.ks, s.y}, b.alpha);
            r.wo = normalize(n * (2.0f * dot(r.wi, n)) - r.wi);
        } else {
            r.wo = sq_cosine_hemisphere(V2{(s.x - b.ks) / (1.f - b.ks), s.y});
        }
        float c = r.wo.z;
        if (c <= 0.f) return V3{0, 0, 0};
        return (bsdf_eval<FULL>(b, r) * c) / bsdf_pdf<FULL>(b, r);
    }
    case NORI_BSDF_DISNEY: {  // disney.cpp:132-155
        if constexpr (!FULL) return V3{0, 0, 0};
        if (r.wi.z <= 0.0f) return V3{0, 0, 0};
        if (s.x <= b.metallic) {
            V3 n = sq_gtr2(V2{s.x / b.metallic, s.y}, b.d_alpha);
            r.wo = normalize(n * (2.0f * dot(r.wi, n)) - r.wi);
        } else {
            r.wo = sq_cosine_hemisphere(V2{(s.x - b.metallic) / (1 - b.metallic), s.y});
        }
        float c = r.wo.z;
        if (c <= 0.0f) return V3{0, 0, 0};
        return (bsdf_eval<FULL>(b, r) * c) / bsdf_pdf<FULL>(b, r);
    }
    }
    return V3{0, 0, 0};
}

}  // namespace nori
