// latency_probe.hip -- dependent-chain latency of one wave with ONE active
// lane on gfx950 (diagnostic for the tail finisher's lone-lane bounce):
// n iterations of a chain of the operation under test, timed with HIP events.
// build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/latency_probe.hip -o tools/latency_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_fmul(float *out, int n, float a) {
    if (threadIdx.x != 0) return;
    float x = out[0];
    for (int i = 0; i < n; ++i) {
        x = x * a;
        x = x * a;
        x = x * a;
        x = x * a;
    }
    out[0] = x;
}
__global__ void k_div(float *out, int n, float a) {
    if (threadIdx.x != 0) return;
    float x = out[0];
    for (int i = 0; i < n; ++i) {
        x = a / x;
        x = a / x;
        x = a / x;
        x = a / x;
    }
    out[0] = x;
}
__global__ void k_sqrt(float *out, int n, float a) {
    if (threadIdx.x != 0) return;
    float x = out[0];
    for (int i = 0; i < n; ++i) {
        x = sqrtf(x) * a;
        x = sqrtf(x) * a;
        x = sqrtf(x) * a;
        x = sqrtf(x) * a;
    }
    out[0] = x;
}
__device__ float tuck(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    const float rd = __builtin_fmaf(-sd, s, x), ru = __builtin_fmaf(-su, s, x);
    float r = rd <= 0.0f ? sd : s;
    return ru > 0.0f ? su : r;
}
__global__ void k_sqrt_tuck(float *out, int n, float a) {
    if (threadIdx.x != 0) return;
    float x = out[0];
    for (int i = 0; i < n; ++i) {
        x = tuck(x) * a;
        x = tuck(x) * a;
        x = tuck(x) * a;
        x = tuck(x) * a;
    }
    out[0] = x;
}
__global__ void k_sqrt_raw(float *out, int n, float a) {
    if (threadIdx.x != 0) return;
    float x = out[0];
    for (int i = 0; i < n; ++i) {
        x = __builtin_amdgcn_sqrtf(x) * a;
        x = __builtin_amdgcn_sqrtf(x) * a;
        x = __builtin_amdgcn_sqrtf(x) * a;
        x = __builtin_amdgcn_sqrtf(x) * a;
    }
    out[0] = x;
}
__global__ void k_rcp_rn(float *out, int n, float a) {
    if (threadIdx.x != 0) return;
    float x = out[0];
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float r = __builtin_amdgcn_rcpf(x);
            const float e = __builtin_fmaf(-x, r, 1.0f);
            x = __builtin_fmaf(e, r, r) * a;
        }
    }
    out[0] = x;
}
__global__ void k_lds(float *out, int n, float a) {
    __shared__ int idx[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) idx[i] = (i * 7 + 3) & 255;
    __syncthreads();
    if (threadIdx.x != 0) return;
    int j = (int)out[1];
    for (int i = 0; i < n; ++i) {
        j = idx[j];
        j = idx[j];
        j = idx[j];
        j = idx[j];
    }
    out[0] = (float)j;
}
__global__ void k_u64(float *out, int n, float a) {
    if (threadIdx.x != 0) return;
    unsigned long long s = (unsigned long long)out[1];
    for (int i = 0; i < n; ++i) {
        s = s * 0x5851f42d4c957f2dULL + 7;
        s = s * 0x5851f42d4c957f2dULL + 7;
        s = s * 0x5851f42d4c957f2dULL + 7;
        s = s * 0x5851f42d4c957f2dULL + 7;
    }
    out[0] = (float)(s >> 40);
}
__global__ void k_readlane(float *out, int n, float a) {
    // the cooperative scan's broadcast: a VALU result read back as a scalar
    float x = out[threadIdx.x];
    for (int i = 0; i < n; ++i) {
        x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x * a), 0));
        x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x * a), 0));
        x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x * a), 0));
        x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x * a), 0));
    }
    if (threadIdx.x == 0) out[0] = x;
}

int main() {
    float *d;
    hipMalloc(&d, 1024);
    float init[2] = {1.5f, 5.0f};
    hipMemcpy(d, init, 8, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int n = 200000;
    struct K {
        const char *name;
        void (*f)(float *, int, float);
    } ks[] = {{"fmul", k_fmul}, {"div", k_div}, {"sqrt*", k_sqrt}, {"sqrt_tuck*", k_sqrt_tuck}, {"v_sqrt*", k_sqrt_raw}, {"rcp_rn*", k_rcp_rn}, {"lds", k_lds}, {"u64 mad", k_u64}, {"mul+readlane", k_readlane}};
    for (auto &k : ks) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k.f, dim3(1), dim3(64), 0, 0, d, n, 1.0000001f);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (rep) std::printf("%-14s %.2f ns per dependent op (%.1f cycles at 2.4 GHz)\n", k.name, ms * 1e6 / (4.0 * n),
                                 ms * 1e6 / (4.0 * n) * 2.4);
        }
    }
    return 0;
}
