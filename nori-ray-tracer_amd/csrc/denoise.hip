// denoise.hip -- the NL-means denoiser (denoiser/denoiser.py) as one kernel.
//
// The reference script runs, for each of the (2r+1)^2 neighbour offsets s,
// whole-image numpy passes (denoiser.py:55-66):
//   ngb      = roll(img, s)                 (periodic shift, :41-44)
//   d2pixel  = (sum_c (ngb - img)^2 - v1) / (eps + k^2 v2)     (:32-37)
//   d2patch  = box(d2pixel)                 (convolve2d 'same', zero fill)
//   wgt      = box(exp(-max(0, d2patch)))
//   out     += wgt * ngb,  wsum += wgt;     out /= wsum at the end.
// Here one work-group owns a kDnTX x kDnTY output tile: it stages the image
// and variance around the tile (halo r + 2p, periodic like np.roll) in LDS
// once, then for every offset computes d2pixel on the tile +- 2p, the first
// box on the tile +- p and the second box on the tile, accumulating the
// weighted neighbours in registers -- the 49 full-image passes of the
// script become one read of the image and one write.
//
// Variances (denoiser.py:32-37): the script's d2() names its third
// parameter img_variance but is called with the shifted variance, and reads
// the global ngb_variance for the other term, so both v1 and v2 come out as
// 2 * var(ngb) (mode 0, what the script computes).  Mode 1 is the textbook
// form the script spells out (v1 = var_p + min(var_p, var_q),
// v2 = var_p + var_q).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace nori {

namespace {

constexpr int kDnTX = 32, kDnTY = 16;  // output tile (256 threads, 2 pixels each)
constexpr float kDnEps = 1e-3f;        // denoiser.py:23

__device__ inline int wrap(int v, int n) {
    v %= n;
    return v < 0 ? v + n : v;
}

__global__ __launch_bounds__(256) void k_nlmeans(const float *__restrict__ img, const float *__restrict__ var, int W,
                                                 int H, int R, int P, float k, int mode, float *__restrict__ out) {
    extern __shared__ float lds[];
    const int halo = R + 2 * P;
    const int AW = kDnTX + 2 * halo, AH = kDnTY + 2 * halo;  // staged image/variance region
    const int DW = kDnTX + 4 * P, DH = kDnTY + 4 * P;        // d2pixel region (tile +- 2p)
    const int GW = kDnTX + 2 * P, GH = kDnTY + 2 * P;        // weight region (tile +- p)
    float *A = lds;                   // AW x AH x 4 (r, g, b, variance)
    float *D = A + 4 * AW * AH;       // DW x DH
    float *G = D + DW * DH;           // GW x GH
    float *Hs = G + GW * GH;          // DH x GW: row sums of D (first box, separable)
    float *Hg = D;                    // GH x kDnTX: row sums of G (second box; D is free by then)
    const int x0 = blockIdx.x * kDnTX, y0 = blockIdx.y * kDnTY, tid = threadIdx.x;
    for (int i = tid; i < AW * AH; i += 256) {
        const int ay = i / AW, ax = i - ay * AW;
        const int gy = wrap(y0 - halo + ay, H), gx = wrap(x0 - halo + ax, W);
        const size_t g = (size_t)gy * W + gx;
        A[4 * i + 0] = img[3 * g + 0];
        A[4 * i + 1] = img[3 * g + 1];
        A[4 * i + 2] = img[3 * g + 2];
        A[4 * i + 3] = var[g];
    }
    __syncthreads();
    const float inv_box = 1.0f / (float)((2 * P + 1) * (2 * P + 1));
    const float k2 = k * k;
    float acc[2][3] = {{0, 0, 0}, {0, 0, 0}}, wsum[2] = {0, 0};
    for (int sr = -R; sr <= R; ++sr)      // axis 0 (rows): np.roll(data, dx, 0)
        for (int sc = -R; sc <= R; ++sc) {  // axis 1 (columns)
            // d2pixel on the tile +- 2p; zero outside the image (convolve2d fill)
            for (int i = tid; i < DW * DH; i += 256) {
                const int dy = i / DW, dx = i - dy * DW;
                const int y = y0 - 2 * P + dy, x = x0 - 2 * P + dx;
                float d2 = 0.0f;
                if (y >= 0 && y < H && x >= 0 && x < W) {
                    const int ay = dy - 2 * P + halo, ax = dx - 2 * P + halo;
                    const float *p = A + 4 * (ay * AW + ax);
                    const float *q = A + 4 * ((ay - sr) * AW + (ax - sc));  // ngb = img[y - sr, x - sc]
                    const float e0 = q[0] - p[0], e1 = q[1] - p[1], e2 = q[2] - p[2];
                    const float sq = (e0 * e0 + e1 * e1) + e2 * e2;
                    const float nv = q[3];
                    float v1, v2;
                    if (mode == 0) {
                        v1 = nv + nv;
                        v2 = nv + nv;
                    } else {
                        v1 = p[3] + fminf(p[3], nv);
                        v2 = p[3] + nv;
                    }
                    d2 = (sq - v1) / (kDnEps + k2 * v2);
                }
                D[i] = d2;
            }
            __syncthreads();
            // box means as row sums then column sums (separable, zero outside the image)
            for (int i = tid; i < DH * GW; i += 256) {
                const int y = i / GW, x = i - y * GW;
                float r = 0.0f;
                for (int l = 0; l <= 2 * P; ++l) r += D[y * DW + x + l];
                Hs[i] = r;
            }
            __syncthreads();
            // wgt = exp(-max(0, box(d2pixel))) on the tile +- p
            for (int i = tid; i < GW * GH; i += 256) {
                const int gy = i / GW, gx = i - gy * GW;
                const int y = y0 - P + gy, x = x0 - P + gx;
                float w = 0.0f;
                if (y >= 0 && y < H && x >= 0 && x < W) {
                    float c = 0.0f;
                    for (int j = 0; j <= 2 * P; ++j) c += Hs[(gy + j) * GW + gx];
                    w = expf(-fmaxf(0.0f, c * inv_box));
                }
                G[i] = w;
            }
            __syncthreads();
            for (int i = tid; i < GH * kDnTX; i += 256) {
                const int y = i / kDnTX, x = i - y * kDnTX;
                float r = 0.0f;
                for (int l = 0; l <= 2 * P; ++l) r += G[y * GW + x + l];
                Hg[i] = r;
            }
            __syncthreads();
            for (int h = 0; h < 2; ++h) {
                const int t = tid + 256 * h, ty = t / kDnTX, tx = t - ty * kDnTX;
                float c = 0.0f;
                for (int j = 0; j <= 2 * P; ++j) c += Hg[(ty + j) * kDnTX + tx];
                const float w = c * inv_box;
                const float *q = A + 4 * ((ty + halo - sr) * AW + (tx + halo - sc));
                acc[h][0] += w * q[0];
                acc[h][1] += w * q[1];
                acc[h][2] += w * q[2];
                wsum[h] += w;
            }
            __syncthreads();
        }
    for (int h = 0; h < 2; ++h) {
        const int t = tid + 256 * h, ty = t / kDnTX, tx = t - ty * kDnTX;
        const int y = y0 + ty, x = x0 + tx;
        if (y < H && x < W) {
            const size_t g = (size_t)y * W + x;
            out[3 * g + 0] = acc[h][0] / wsum[h];
            out[3 * g + 1] = acc[h][1] / wsum[h];
            out[3 * g + 2] = acc[h][2] / wsum[h];
        }
    }
}

}  // namespace

size_t denoise_lds_bytes(int R, int P) {
    const int halo = R + 2 * P;
    return sizeof(float) * ((size_t)4 * (kDnTX + 2 * halo) * (kDnTY + 2 * halo) +
                            (size_t)(kDnTX + 4 * P) * (kDnTY + 4 * P) + (size_t)(kDnTX + 2 * P) * (kDnTY + 2 * P) +
                            (size_t)(kDnTY + 4 * P) * (kDnTX + 2 * P));
}

hipError_t launch_denoise(const float *img, const float *var, int W, int H, int R, int P, float k, int mode,
                          float *out, hipStream_t st) {
    const dim3 g((W + kDnTX - 1) / kDnTX, (H + kDnTY - 1) / kDnTY), b(256);
    hipLaunchKernelGGL(k_nlmeans, g, b, denoise_lds_bytes(R, P), st, img, var, W, H, R, P, k, mode, out);
    return hipGetLastError();
}

}  // namespace nori
