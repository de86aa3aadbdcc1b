/*
 * detmath_ref.h -- ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * Deterministic float32 elementary functions used by the CPU oracle.
 *
 * Why this exists: the reference (ACMMP.cu) is built with nvcc --use_fast_math
 * (CMakeLists.txt:39-46), so its expf/sinf/asinf/atan2f/rsqrtf/division are
 * vendor approximations that cannot be reproduced bit-for-bit anywhere else.
 * The oracle therefore fixes ONE concrete definition of every elementary
 * function, built only from IEEE-754 binary32 operations that are
 * correctly rounded on both x86-64 and gfx950 (+ - * / sqrt fma floor rint,
 * exact power-of-two scaling).  The product kernels carry their own,
 * independently written copy of the same definitions
 * (acmmp-spherical_amd/csrc/detmath.h); parity tests then compare the two
 * bit-for-bit, and tests/test_detmath.py checks the accuracy of these
 * definitions against float64 numpy (<= a few ulp).
 *
 * Polynomial coefficients: oracle/tools/fit_detmath.py (Lawson minimax fit).
 *
 * Contraction rule: nothing here is fused unless written as fmaf(); the oracle
 * is compiled with -ffp-contract=off.
 */
#ifndef ACMMP_ORACLE_DETMATH_REF_H
#define ACMMP_ORACLE_DETMATH_REF_H

#include <math.h>
#include <stdint.h>
#include <string.h>

#define DM_PI_HI    3.14159274101257324f   /* float(pi)              */
#define DM_PI_LO   (-8.74227765734758577e-08f)
#define DM_PIO2_HI  1.57079637050628662f   /* float(pi/2)            */
#define DM_PIO2_LO (-4.37113882867379300e-08f)

static inline float dm_bits2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t dm_f2bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* 2^n for n in [-126, 127], built exactly from the exponent field. */
static inline float dm_pow2i(int n) { return dm_bits2f((uint32_t)(n + 127) << 23); }

/* float -> int32, truncating toward zero, saturating, NaN -> 0.
 * (the behaviour of CUDA cvt.rzi.s32.f32 and of gfx950 v_cvt_i32_f32) */
static inline int dm_f2i_sat(float x)
{
    if (x != x) return 0;
    if (x >= 2147483648.0f) return 2147483647;
    if (x < -2147483648.0f) return (-2147483647 - 1);
    return (int)x;
}

/* e^x.  Cody-Waite reduction by ln2, degree-6 polynomial, exact 2^k scaling in
 * two steps so that sub-normal results are rounded exactly once. */
static inline float dm_expf(float x)
{
    if (x != x) return x;
    if (x > 88.7228393554688f) return INFINITY;
    if (x < -103.972084045410f) return 0.0f;
    const float k = rintf(x * 1.44269502162933350f);
    float r = fmaf(k, -0.693145751953125f, x);
    r = fmaf(k, -1.42860676533018700e-06f, r);
    float q = 0.00139012828003615141f;
    q = fmaf(q, r, 0.00836314447224140167f);
    q = fmaf(q, r, 0.0416668541729450226f);
    q = fmaf(q, r, 0.166665777564048767f);
    q = fmaf(q, r, 0.5f);
    const float p = 1.0f + fmaf(r * r, q, r);
    const int ki = (int)k;
    const int k1 = ki / 2;
    const int k2 = ki - k1;
    return (p * dm_pow2i(k1)) * dm_pow2i(k2);
}

/* sin and cos together: reduction by pi/2 (3-part Cody-Waite), quadrant select. */
static inline void dm_sincosf(float x, float *s, float *c)
{
    if (!(fabsf(x) < 1.0e30f)) { *s = NAN; *c = NAN; return; }
    const float k = rintf(x * 0.636619746685028076f);
    float r = fmaf(k, -1.5703125f, x);
    r = fmaf(k, -4.83870506286621094e-04f, r);
    r = fmaf(k, 4.37113882867379300e-08f, r);
    const float z = r * r;
    float ps = 2.72494116870802827e-06f;
    ps = fmaf(ps, z, -1.98400826775468886e-04f);
    ps = fmaf(ps, z, 8.33333190530538559e-03f);
    ps = fmaf(ps, z, -0.166666671633720398f);
    const float sr = fmaf(r * z, ps, r);
    float pc = -2.73006861561953e-07f;
    pc = fmaf(pc, z, 2.48005981120513752e-05f);
    pc = fmaf(pc, z, -1.38888880610466003e-03f);
    pc = fmaf(pc, z, 0.0416666679084300995f);
    const float cr = fmaf(z * z, pc, fmaf(-0.5f, z, 1.0f));
    const float kq = k - 4.0f * floorf(k * 0.25f);
    const int q = (int)kq & 3;
    switch (q) {
    case 0: *s = sr; *c = cr; break;
    case 1: *s = cr; *c = -sr; break;
    case 2: *s = -sr; *c = -cr; break;
    default: *s = -cr; *c = sr; break;
    }
}
static inline float dm_sinf(float x) { float s, c; dm_sincosf(x, &s, &c); return s; }
static inline float dm_cosf(float x) { float s, c; dm_sincosf(x, &s, &c); return c; }

/* asin core on [0, 0.5]: x + x*z*P(z), z = x*x (passed in). */
static inline float dm_asin_core(float x, float z)
{
    float p = 0.0337996557354927063f;
    p = fmaf(p, z, 0.0170816909521818161f);
    p = fmaf(p, z, 0.0311153121292591095f);
    p = fmaf(p, z, 0.0445981100201606750f);
    p = fmaf(p, z, 0.0750009864568710327f);
    p = fmaf(p, z, 0.166666656732559204f);
    return fmaf(x * z, p, x);
}

static inline float dm_asinf(float x)
{
    if (x != x) return x;
    const float a = fabsf(x);
    if (a > 1.0f) return NAN;
    float r;
    if (a <= 0.5f) {
        r = dm_asin_core(a, a * a);
    } else {
        const float z = (1.0f - a) * 0.5f;
        const float s = sqrtf(z);
        r = fmaf(-2.0f, dm_asin_core(s, z), DM_PIO2_HI) + DM_PIO2_LO;
    }
    return copysignf(r, x);
}

static inline float dm_acosf(float x)
{
    if (x != x) return x;
    if (fabsf(x) > 1.0f) return NAN;
    if (x > 0.5f) {
        const float z = (1.0f - x) * 0.5f;
        const float s = sqrtf(z);
        return 2.0f * dm_asin_core(s, z);
    }
    if (x < -0.5f) {
        const float z = (1.0f + x) * 0.5f;
        const float s = sqrtf(z);
        return fmaf(-2.0f, dm_asin_core(s, z), DM_PI_HI) + DM_PI_LO;
    }
    const float a = fabsf(x);
    const float r = copysignf(dm_asin_core(a, a * a), x);
    return (DM_PIO2_HI - r) + DM_PIO2_LO;
}

/* atan2 with C99 special cases for zeros / infinities. */
static inline float dm_atan2f(float y, float x)
{
    if (x != x || y != y) return x + y;
    const float ax = fabsf(x), ay = fabsf(y);
    const int xneg = signbit(x) != 0;
    if (ay == 0.0f) {
        return xneg ? copysignf(DM_PI_HI, y) : copysignf(0.0f, y);
    }
    if (ax == 0.0f) return copysignf(DM_PIO2_HI, y);
    if (isinf(ax) || isinf(ay)) {
        float r;
        if (isinf(ax) && isinf(ay)) r = xneg ? 2.35619449615478516f : 0.785398185253143311f;
        else if (isinf(ax)) r = xneg ? DM_PI_HI : 0.0f;
        else r = DM_PIO2_HI;
        return copysignf(r, y);
    }
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float t = mn / mx;
    const float z = t * t;
    float p = -9.51492460444569588e-04f;
    p = fmaf(p, z, 6.28401106223464012e-03f);
    p = fmaf(p, z, -1.94261018186807632e-02f);
    p = fmaf(p, z, 3.85241769254207611e-02f);
    p = fmaf(p, z, -5.77491596341133118e-02f);
    p = fmaf(p, z, 7.42385536432266235e-02f);
    p = fmaf(p, z, -9.03848111629486084e-02f);
    p = fmaf(p, z, 0.111049808561801910f);
    p = fmaf(p, z, -0.142853394150733948f);
    p = fmaf(p, z, 0.199999913573265076f);
    p = fmaf(p, z, -0.333333343267440796f);
    float r = fmaf(t * z, p, t);
    if (ay > ax) r = (DM_PIO2_HI - r) + DM_PIO2_LO;
    if (xneg) r = (DM_PI_HI - r) + DM_PI_LO;
    return copysignf(r, y);
}

/* rsqrtf as used by NormalizeVec3 (ACMMP.cu:113): one IEEE sqrt, one IEEE divide. */
static inline float dm_rsqrtf(float x) { return 1.0f / sqrtf(x); }

#endif
