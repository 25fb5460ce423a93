/*
 * lgs_detmath.h — deterministic fp32 transcendentals shared by the HIP env step
 * (leggedsim.hip, device code) and the CPU oracle (oracle/lgs_oracle.c, plain C).
 *
 * Why: libm (glibc) and the ROCm device library (ocml) round sinf/cosf/expf/
 * atan2f/asinf differently in the last bit, and one ulp in a joint rotation or a
 * contact distance is enough for a contact to switch on in one implementation and
 * not the other.  Both sides compile THIS code with -ffp-contract=off: every
 * multiply-add below is an explicit fmaf (a correctly rounded fused op on x86-64-v3
 * and on gfx950 alike), every other operation is a single IEEE op (division and
 * sqrt are correctly rounded in HIP by default), so the two builds produce the
 * same bits for the same input.
 *
 * Accuracy (tests/test_detmath.py, against double-precision libm): sin/cos/exp
 * within 2 ulp, atan2/asin within 3 ulp over the ranges the env uses.  The
 * polynomials are the Cephes single-precision minimax sets (public domain).
 */
#ifndef LGS_DETMATH_H
#define LGS_DETMATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define LGS_DM __host__ __device__ static inline __attribute__((always_inline))
#else
#define LGS_DM static inline
#endif

#define LGS_DM_PI 3.14159274101257324f    /* fp32(pi)   */
#define LGS_DM_PIO2 1.57079637050628662f  /* fp32(pi/2) */
#define LGS_DM_PIO4 0.785398185253143311f /* fp32(pi/4) */

LGS_DM float lgs_dm_i2f(int32_t i) {
    float f;
    memcpy(&f, &i, 4);
    return f;
}

/* sin and cos of x (|x| < 1e4): x = k pi/2 + r, |r| <= pi/4, three-part pi/2 */
LGS_DM void lgs_sincosf(float x, float* s_out, float* c_out) {
    const float k = rintf(x * 0.636619747f);
    float r = fmaf(-k, 1.57079637050628662f, x);
    r = fmaf(-k, -4.37113882867379300e-08f, r);
    r = fmaf(-k, -1.71512451000588190e-15f, r);
    const float z = r * r;
    /* sin r = r + r^3 (S1 + z (S2 + z S3)) */
    float ps = fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f);
    ps = fmaf(ps, z, -1.6666654611e-1f);
    const float sn = fmaf(ps * z, r, r);
    /* cos r = 1 - z/2 + z^2 (C1 + z (C2 + z C3)) */
    float pc = fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f);
    pc = fmaf(pc, z, 4.166664568298827e-2f);
    const float cs = fmaf(pc * z, z, fmaf(-0.5f, z, 1.0f));
    const int q = ((int)k) & 3;
    float s, c;
    if (q == 0) { s = sn; c = cs; }
    else if (q == 1) { s = cs; c = -sn; }
    else if (q == 2) { s = -sn; c = -cs; }
    else { s = -cs; c = sn; }
    *s_out = s;
    *c_out = c;
}
LGS_DM float lgs_sinf(float x) {
    float s, c;
    lgs_sincosf(x, &s, &c);
    return s;
}
LGS_DM float lgs_cosf(float x) {
    float s, c;
    lgs_sincosf(x, &s, &c);
    return c;
}

/* e^x: x = k ln2 + r (two-part ln2), e^r by the Cephes polynomial, times 2^k built
 * from its exponent bits (exact).  x < -87 returns 0 (the true value is < 2e-38). */
LGS_DM float lgs_expf(float x) {
    if (x < -87.0f) return 0.0f;
    if (x > 88.0f) x = 88.0f;
    const float k = rintf(x * 1.44269502f);
    float r = fmaf(-k, 0.693359375f, x);
    r = fmaf(-k, -2.12194440e-4f, r);
    float p = fmaf(1.9875691500e-4f, r, 1.3981999507e-3f);
    p = fmaf(p, r, 8.3334519073e-3f);
    p = fmaf(p, r, 4.1665795894e-2f);
    p = fmaf(p, r, 1.6666665459e-1f);
    p = fmaf(p, r, 5.0000001201e-1f);
    const float y = fmaf(p, r * r, r) + 1.0f;
    return y * lgs_dm_i2f(((int32_t)k + 127) << 23);
}

/* atan(x) for x >= 0 (Cephes atanf reduction: x > tan 3pi/8 -> pi/2 - atan(1/x),
 * x > tan pi/8 -> pi/4 + atan((x-1)/(x+1))) */
LGS_DM float lgs_atan_pos(float x) {
    float y0 = 0.0f;
    if (x > 2.41421356f) {
        y0 = LGS_DM_PIO2;
        x = -1.0f / x;
    } else if (x > 0.414213562f) {
        y0 = LGS_DM_PIO4;
        x = (x - 1.0f) / (x + 1.0f);
    }
    const float z = x * x;
    float p = fmaf(8.05374449538e-2f, z, -1.38776856032e-1f);
    p = fmaf(p, z, 1.99777106478e-1f);
    p = fmaf(p, z, -3.33329491539e-1f);
    return fmaf(p * z, x, x) + y0;
}

/* atan2(y, x) with C's signed-zero conventions */
LGS_DM float lgs_atan2f(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    float a = (ax == 0.0f && ay == 0.0f) ? 0.0f : lgs_atan_pos(ay / ax);
    if (signbit(x)) a = LGS_DM_PI - a;
    return copysignf(a, y);
}

/* asin(x), |x| <= 1 (Cephes asinf: |x| > 0.5 via asin = pi/2 - 2 asin(sqrt((1-|x|)/2))) */
LGS_DM float lgs_asinf(float x) {
    const float a = fabsf(x);
    const int big = a > 0.5f;
    const float z = big ? 0.5f * (1.0f - a) : a * a;
    const float s = big ? sqrtf(z) : a;
    float p = fmaf(4.2163199048e-2f, z, 2.4181311049e-2f);
    p = fmaf(p, z, 4.5470025998e-2f);
    p = fmaf(p, z, 7.4953002686e-2f);
    p = fmaf(p, z, 1.6666752422e-1f);
    float r = fmaf(p * z, s, s);
    if (big) r = LGS_DM_PIO2 - (r + r);
    return copysignf(r, x);
}

#endif /* LGS_DETMATH_H */
