/* Verifies the exact-division identity used by the traversal's slab test:
 *   y = RN(1/d) (= (float)(1.0/(double)d)), q = RN(a*y), r = fma(-q, d, a), q' = fma(r, y, q)
 *   q' == RN(a/d) bit for bit (an exact zero may come out +0 for -0: the slab test only compares), for 2^-64 <= |d| <= 2 and a == +-0 or 2^-90 <= |a| <= 2^61.
 * (Markstein's theorem: y within 1/2 ulp of 1/d, q within 1 ulp of a/d, no under/overflow.)
 * gcc -O2 -ffp-contract=off scripts/verify_fastdiv.c -lm && ./a.out [samples] */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static float fbits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float rand_in(int emin, int emax) { /* random sign, exponent in [emin, emax), random significand */
    uint64_t r = rnd();
    int e = emin + (int)(r % (uint64_t)(emax - emin));
    uint32_t mant = (uint32_t)(r >> 20) & 0x7FFFFF;
    int mode = (int)((r >> 50) & 7);
    if (mode == 0) mant = 0; else if (mode == 1) mant = 0x7FFFFF; else if (mode == 2) mant = 1; else if (mode == 3) mant = 0x7FFFFE;
    uint32_t u = ((uint32_t)(e + 127) << 23) | mant | ((r >> 63) ? 0x80000000u : 0);
    return fbits(u);
}
static inline float fastdiv(float a, float d, float y) {
    float q = a * y;
    float r = fmaf(-q, d, a);
    return fmaf(r, y, q);
}
int main(int argc, char** argv) {
    long n = argc > 1 ? atol(argv[1]) : 200000000L;
    long bad = 0;
    for (long i = 0; i < n; ++i) {
        float d = rand_in(-64, 2);
        float a = (i % 97 == 0) ? ((i & 1) ? -0.0f : 0.0f) : rand_in(-90, 61);
        float y = (float)(1.0 / (double)d);
        float q1 = fastdiv(a, d, y), q0 = a / d;
        if (bits(q1) != bits(q0) && !(q1 == 0.0f && q0 == 0.0f)) {  /* only the sign of an exact zero may differ */
            if (bad < 10) printf("MISMATCH a=%a d=%a fast=%a exact=%a\n", a, d, q1, q0);
            ++bad;
        }
    }
    printf("%ld samples, %ld mismatches\n", n, bad);
    return bad != 0;
}
