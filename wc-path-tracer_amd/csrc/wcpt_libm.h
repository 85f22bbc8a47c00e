/*
 * wcpt_libm.h — deterministic single-precision log / cos / exp for the path-tracing kernel.
 *
 * Why this exists: pathTracer.comp calls the GLSL built-ins log, cos and exp (Random.glsl:45-47 via
 * RandomDirection, pathTracer.comp:278). Their precision is driver-defined in Vulkan, so the reference
 * itself is not bit-reproducible. To make "GPU image == CPU oracle image" a bit-exact statement we define
 * these three functions ourselves, using only IEEE-754 binary32 +, -, *, / (correctly rounded on gfx950 by
 * hipcc's default and on x86-64 SSE), floorf, fabsf and integer bit manipulation, and NO fused multiply-add
 * (everything that includes this file is compiled with -ffp-contract=off). The same source therefore yields
 * bit-identical results on the GPU kernel and in the C oracle (oracle/pt_oracle.c includes this header).
 * Accuracy is checked against float64 libm in tests/test_libm.py (<= 2 ulp over the kernel's domains).
 *
 * The algorithms are the textbook ones: logf via the atanh series in s = f/(2+f) with a degree-4 minimax
 * tail; cosf via Cody-Waite reduction by pi/2 and minimax sin/cos kernels on [-pi/4, pi/4]; expf via
 * reduction by ln2 and a degree-6 polynomial with exact power-of-two scaling.
 *
 * The quotient f/(2+f) of logf is evaluated as f * RN(1/(2+f)) with a correctly rounded reciprocal (wcpt_rcp1_2:
 * v_rcp_f32 + one FMA Newton step on the GPU, exact for every divisor in [1, 4) -- 2+f lies in [1.29, 2.42] --
 * and the IEEE quotient 1.0f/x on the host; the device's exhaustive reciprocal check covers this range): 4 VALU
 * instead of the ~11 of a correctly rounded division, the same bits on both sides.
 *
 * The kernel calls logf and cosf only on its own domains -- log(rand()) with rand() in {0} U [2^-32, 1]
 * (Random.glsl:46) and cos(2*PI*rand()) in [0, 2*pi] (:45,47) -- so it uses wcpt_logf_rand / wcpt_cosf_2pi: the
 * same main path as wcpt_logf / wcpt_cosf without the special-case tests that cannot fire there (NaN, negative,
 * subnormal and infinite arguments, huge reductions). On those domains they return the same bits by construction
 * (tests/test_libm.py checks it).
 */
#ifndef WCPT_LIBM_H
#define WCPT_LIBM_H

#include <stdint.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define WCPT_HD __host__ __device__ static inline
#else
#include <math.h>
#define WCPT_HD static inline
#endif

WCPT_HD uint32_t wcpt_f2u(float f) { union { float f; uint32_t u; } c; c.f = f; return c.u; }
WCPT_HD float    wcpt_u2f(uint32_t u) { union { float f; uint32_t u; } c; c.u = u; return c.f; }

/* 2^e for e in [-126, 127], exact. */
WCPT_HD float wcpt_pow2i(int e) { return wcpt_u2f((uint32_t)(e + 127) << 23); }

/* Correctly rounded 1/x for x in [1, 4) (the divisor 2+f of wcpt_logf's series). */
#if defined(__HIP_DEVICE_COMPILE__)
__device__ static inline float wcpt_rcp1_2(float x)
{
    const float y = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y, 1.0f);
    return __builtin_fmaf(e, y, y);
}
#else
static inline float wcpt_rcp1_2(float x) { return 1.0f / x; }
#endif

/* Main path of wcpt_logf for a positive normal finite x (x already scaled by 2^-k0 for a subnormal argument). */
WCPT_HD float wcpt_logf_core(float x, int k0)
{
    const float ln2_hi = 6.9313812256e-01f;   /* 0x3f317180: 16 trailing zero bits, k*ln2_hi exact */
    const float ln2_lo = 9.0580006145e-06f;   /* 0x3717f7d1 */
    const float Lg1 = 0.66666662693f;          /* 0x3f2aaaaa */
    const float Lg2 = 0.40000972152f;          /* 0x3ecccce1 */
    const float Lg3 = 0.28498786688f;          /* 0x3e91e9ee */
    const float Lg4 = 0.24279078841f;          /* 0x3e789e26 */
    uint32_t ix = wcpt_f2u(x);
    /* Split x = 2^k * m with m in [sqrt(2)/2, sqrt(2)). */
    ix = ix + (0x3f800000u - 0x3f3504f3u);
    const int k = k0 + (int)(ix >> 23) - 127;
    ix = (ix & 0x007fffffu) + 0x3f3504f3u;
    const float m = wcpt_u2f(ix);
    const float f = m - 1.0f;                          /* exact (Sterbenz) */
    const float s = f * wcpt_rcp1_2(2.0f + f);         /* f / (2 + f), reciprocal correctly rounded */
    const float z = s * s;
    const float w = z * z;
    const float t1 = w * (Lg2 + w * Lg4);
    const float t2 = z * (Lg1 + w * Lg3);
    const float R = t2 + t1;
    const float hfsq = 0.5f * f * f;
    const float dk = (float)k;
    return s * (hfsq + R) + dk * ln2_lo - hfsq + f + dk * ln2_hi;
}

/* Natural logarithm, every binary32 argument. */
WCPT_HD float wcpt_logf(float x)
{
    const uint32_t ix = wcpt_f2u(x);
    if (x != x) return x;                                  /* NaN */
    if (ix >= 0x80000000u) {
        if (ix == 0x80000000u) return wcpt_u2f(0xff800000u); /* log(-0) = -inf */
        return wcpt_u2f(0x7fc00000u);                     /* log(<0) = NaN */
    }
    if (ix == 0u) return wcpt_u2f(0xff800000u);           /* log(+0) = -inf */
    if (ix == 0x7f800000u) return x;                       /* log(+inf) = +inf */
    if (ix < 0x00800000u) return wcpt_logf_core(x * 33554432.0f, -25); /* subnormal: scale by 2^25 (exact) */
    return wcpt_logf_core(x, 0);
}

/* log of a rand() value (Random.glsl:27-32,46): x = n * 2^-32 for an integer n, so x is 0 or in [2^-32, 1]: equal
 * to wcpt_logf there (the other special cases cannot occur). */
WCPT_HD float wcpt_logf_rand(float x)
{
    return x == 0.0f ? wcpt_u2f(0xff800000u) : wcpt_logf_core(x, 0);
}

/* Main path of wcpt_cosf for a finite ax = |x| <= 2^23. */
WCPT_HD float wcpt_cosf_core(float ax)
{
    const float two_over_pi = 0.63661977236758134f;
    const float pio2_1 = 1.5703125f;                       /* 0x3fc90000, 8 significant bits   */
    const float pio2_2 = 4.837512969970703125e-4f;         /* 0x39fd8000, 13 significant bits  */
    const float pio2_3 = 7.5497899548e-8f;                 /* remainder of pi/2                */
    const float S1 = -1.6666654611e-1f, S2 = 8.3321608736e-3f, S3 = -1.9515295891e-4f;
    const float C1 = 4.166664568298827e-2f, C2 = -1.388731625493765e-3f, C3 = 2.443315711809948e-5f;
    const float jf = floorf(ax * two_over_pi + 0.5f);
    const int j = (int)jf;
    const float r = ((ax - jf * pio2_1) - jf * pio2_2) - jf * pio2_3;
    const float z = r * r;
    float c = ((C3 * z + C2) * z + C1) * z * z;
    c = c - 0.5f * z;
    c = c + 1.0f;
    float s = ((S3 * z + S2) * z + S1) * z * r;
    s = s + r;
    switch (j & 3) {
    case 0: return c;
    case 1: return -s;
    case 2: return -c;
    default: return s;
    }
}

/* Cosine, every binary32 argument. Accurate reduction for |x| < ~1e5; larger arguments still return a
 * deterministic value in [-1, 1]. */
WCPT_HD float wcpt_cosf(float x)
{
    if (x != x) return x;
    float ax = fabsf(x);
    if (wcpt_f2u(ax) == 0x7f800000u) return wcpt_u2f(0x7fc00000u);
    if (ax > 8388608.0f) ax = ax - floorf(ax * 0.25f) * 4.0f; /* keep j representable; deterministic */
    return wcpt_cosf_core(ax);
}

/* cos(2*PI*rand()) (Random.glsl:45,47): the argument lies in [0, 2*pi], where this equals wcpt_cosf. */
WCPT_HD float wcpt_cosf_2pi(float x) { return wcpt_cosf_core(x); }

/* Exponential. Domain used by the kernel: -absorption*strength*t (pathTracer.comp:278). */
WCPT_HD float wcpt_expf(float x)
{
    const float log2e = 1.44269504088896341f;
    const float ln2_hi = 0.693359375f;                     /* 0x3f318000 */
    const float ln2_lo = -2.12194440e-4f;
    const float P0 = 1.9875691500e-4f, P1 = 1.3981999507e-3f, P2 = 8.3334519073e-3f;
    const float P3 = 4.1665795894e-2f, P4 = 1.6666665459e-1f, P5 = 5.0000001201e-1f;
    float kf, r, z, p;
    int k;
    if (x != x) return x;
    if (x > 88.72283905f) return wcpt_u2f(0x7f800000u);
    if (x < -103.97208405f) return 0.0f;
    kf = floorf(x * log2e + 0.5f);
    r = (x - kf * ln2_hi) - kf * ln2_lo;
    z = r * r;
    p = (((((P0 * r + P1) * r + P2) * r + P3) * r + P4) * r + P5) * z + r + 1.0f;
    k = (int)kf;
    if (k > 127) {
        p = p * wcpt_pow2i(127);
        k = k - 127;
        return p * wcpt_pow2i(k);
    }
    if (k < -125) {
        p = p * wcpt_pow2i(k + 100);                       /* exact: stays normal */
        return p * wcpt_pow2i(-100);                       /* single rounding into the subnormal range */
    }
    return p * wcpt_pow2i(k);
}

#endif /* WCPT_LIBM_H */
