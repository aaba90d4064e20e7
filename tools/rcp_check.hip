// Exhaustive check of the reciprocal used by the triangle test
// (device_math.h rcp_rn): v_rcp_f32 followed by one FMA Newton step must
// equal the correctly rounded IEEE quotient 1.0f / x for every float x whose
// magnitude lies in [2^-125, 2^125] (the triangle test rejects |det| < 1e-8
// before dividing, and larger determinants than 2^125 take the IEEE path).
// Build: hipcc -O3 --offload-arch=gfx950 tools/rcp_check.hip -o tools/rcp_check
// Prints the number of mismatching inputs (0 expected) and the first few.
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ float rcp_newton(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}

__global__ void check(uint32_t base, unsigned long long *bad, uint32_t *first) {
    const uint32_t bits = base + blockIdx.x * blockDim.x + threadIdx.x;
    const float x = __uint_as_float(bits);
    const uint32_t ex = (bits >> 23) & 0xFFu;
    if (ex < 127 - 125 || ex > 127 + 125) return;  // outside the fast path's range
    const float a = 1.0f / x;  // IEEE division (div_scale / div_fmas / div_fixup)
    const float b = rcp_newton(x);
    if (__float_as_uint(a) != __float_as_uint(b)) {
        const unsigned long long n = atomicAdd(bad, 1ull);
        if (n < 8) first[n] = bits;
    }
}

int main() {
    unsigned long long *bad;
    uint32_t *first;
    hipMalloc(&bad, sizeof(*bad));
    hipMalloc(&first, 8 * sizeof(uint32_t));
    hipMemset(bad, 0, sizeof(*bad));
    hipMemset(first, 0, 8 * sizeof(uint32_t));
    const uint32_t block = 256, chunk = 1u << 28;  // 4 launches of 2^28 inputs each cover all 2^32 patterns
    for (uint64_t base = 0; base < (1ull << 32); base += chunk)
        hipLaunchKernelGGL(check, dim3(chunk / block), dim3(block), 0, 0, (uint32_t)base, bad, first);
    unsigned long long h = 0;
    uint32_t f[8];
    hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost);
    hipMemcpy(f, first, sizeof(f), hipMemcpyDeviceToHost);
    const hipError_t e = hipDeviceSynchronize();
    std::printf("rcp_check: %s, mismatches %llu\n", hipGetErrorString(e), h);
    for (unsigned long long i = 0; i < h && i < 8; ++i) std::printf("  x bits 0x%08x\n", f[i]);
    return e == hipSuccess && h == 0 ? 0 : 1;
}
