// sqrt_check.hip -- exhaustive check of short correctly-rounded sqrt
// sequences against the IEEE sqrtf the compiler emits, over every positive
// float in [2^-120, 2^120) (diagnostic for device_math.h sqrt_rn).
// build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/sqrt_check.hip -o tools/sqrt_check
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ float seq_raw(float x) { return __builtin_amdgcn_sqrtf(x); }
// hardware sqrt + one Tuckerman test in each direction (no denormal scaling)
__device__ float seq_tuck(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    const float rd = __builtin_fmaf(-sd, s, x), ru = __builtin_fmaf(-su, s, x);
    float r = rd <= 0.0f ? sd : s;
    return ru > 0.0f ? su : r;
}
// rsqrt-based: y = x * rsq, one FMA correction
__device__ float seq_rsq(float x) {
    const float r = __builtin_amdgcn_rsqf(x);
    const float s = x * r;
    const float e = __builtin_fmaf(-s, s, x);
    return __builtin_fmaf(e, 0.5f * r, s);
}

__global__ void k_check(unsigned base, unsigned long long *bad) {
    const unsigned bits = base + blockIdx.x * blockDim.x + threadIdx.x;
    const float x = __uint_as_float(bits);
    const float ref = sqrtf(x);
    unsigned b0 = seq_raw(x) != ref, b1 = seq_tuck(x) != ref, b2 = seq_rsq(x) != ref;
    if (b0) atomicAdd(&bad[0], 1ull);
    if (b1) atomicAdd(&bad[1], 1ull);
    if (b2) atomicAdd(&bad[2], 1ull);
}

int main() {
    unsigned long long *d, h[3];
    hipMalloc(&d, sizeof(h));
    hipMemset(d, 0, sizeof(h));
    const unsigned lo = 0x0f800000u, hi = 0x6f800000u;  // 2^-96 .. 2^96 (no scaling branch in the IEEE expansion)
    const unsigned step = 1u << 24;
    for (unsigned b = lo; b < hi; b += step) hipLaunchKernelGGL(k_check, dim3(step / 256), dim3(256), 0, 0, b, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    std::printf("mismatches vs IEEE sqrtf over [2^-96, 2^96): raw v_sqrt %llu, v_sqrt+Tuckerman %llu, rsq+FMA %llu\n", h[0],
                h[1], h[2]);
    return 0;
}
