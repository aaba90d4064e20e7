/* Checks the division used by the scan's sphere test (kernels.hip div_rn):
 * q = x / y correctly rounded from r = RN(1 / y), q0 = RN(x r),
 * e = fma(-y, q0, x) (exact), q = RN(q0 + e r) -- Markstein's theorem -- for
 * 2^-100 <= |x| <= 2^100 and y in the reciprocal's verified range.  Random
 * x over those binades against every y of a binade sample, and every
 * significand of x against random y.  CPU float arithmetic with fmaf rounds
 * like the GPU's v_fma_f32 / v_mul_f32 (IEEE, round to nearest even).
 * build: gcc -O2 -mfma tools/div_check.c -o /tmp/div_check -lm ; run: /tmp/div_check [n] */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static uint64_t s = 88172645463325252ull;
static uint32_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)(s >> 16); }

static float div_rn(float x, float y) {
    volatile float r = 1.0f / y;  /* rcp_rn: correctly rounded 1/y */
    float q0 = x * r;
    float e = fmaf(-y, q0, x);
    return fmaf(e, r, q0);
}

int main(int argc, char **argv) {
    long n = argc > 1 ? atol(argv[1]) : 200000000L;
    long bad = 0, done = 0;
    for (long i = 0; i < n; ++i) {
        /* y: random significand, exponent in [-60, 60]; x: random significand, |x| in [2^-100, 2^100] */
        float y = f_of((rnd() & 0x807FFFFFu) | ((uint32_t)(127 - 60 + rnd() % 121) << 23));
        float x = f_of((rnd() & 0x807FFFFFu) | ((uint32_t)(127 - 100 + rnd() % 201) << 23));
        float q = x / y;
        if (!(fabsf(q) >= 0x1p-126f) || isinf(q)) continue;
        ++done;
        if (u_of(div_rn(x, y)) != u_of(q)) {
            if (bad++ < 5) printf("mismatch x=%a y=%a q=%a got %a\n", x, y, q, div_rn(x, y));
        }
    }
    /* every significand of x against 64 random y near 2 (the sphere test's 2 A, A = |d|^2 ~ 1) */
    for (int k = 0; k < 64; ++k) {
        float y = f_of(u_of(2.0f) + (rnd() % 65) - 32);
        for (uint32_t m = 0; m < (1u << 23); ++m) {
            float x = f_of(m | (uint32_t)(127 + (int)(k % 7) - 3) << 23);
            ++done;
            if (u_of(div_rn(x, y)) != u_of(x / y)) {
                if (bad++ < 10) printf("mismatch x=%a y=%a\n", x, y);
            }
        }
    }
    printf("%ld quotients checked, %ld mismatches\n", done, bad);
    return bad != 0;
}
