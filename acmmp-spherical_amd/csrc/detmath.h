// detmath.h -- deterministic binary32 elementary functions for the gfx950 kernels.
//
// The reference compiles with nvcc --use_fast_math (CMakeLists.txt:39-46), whose
// expf/sinf/asinf/atan2f/rsqrtf are vendor approximations.  This engine instead fixes
// one definition of each function, built only from operations that are correctly
// rounded on gfx950 (v_fma_f32, v_floor_f32, v_rndne_f32, the IEEE div/sqrt
// sequences hipcc emits by default, exact power-of-two scaling).  The definitions
// are documented in DESIGN.md §2.3; the test oracle restates them independently,
// and parity is checked bit-for-bit.  Every function here is a few dozen VALU ops
// and runs only per pixel / per hypothesis, except asin/atan2, which sit in the
// SPHERE projection of every sample (the price of exact parity).
//
// Compiled with -ffp-contract=off: only the fmaf() written here fuse.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ACMMP_HD __host__ __device__ __forceinline__

namespace acmmp {

constexpr float kPiHi = 3.14159274101257324f;
constexpr float kPiLo = -8.74227765734758577e-08f;
constexpr float kPio2Hi = 1.57079637050628662f;
constexpr float kPio2Lo = -4.37113882867379300e-08f;
constexpr float kCudartPiF = 3.141592654f;         // CUDART_PI_F
constexpr double kMPi = 3.14159265358979323846;    // M_PI
constexpr float kInv2Pi = 0.159154936671257019f;
constexpr float kInvPi = 0.318309873342514038f;

ACMMP_HD float bits_to_f(uint32_t u) { return __builtin_bit_cast(float, u); }
ACMMP_HD uint32_t f_to_bits(float f) { return __builtin_bit_cast(uint32_t, f); }
ACMMP_HD float pow2i(int n) { return bits_to_f(static_cast<uint32_t>(n + 127) << 23); }

// float -> int32: truncate toward zero, saturate, NaN -> 0 (v_cvt_i32_f32 semantics), branch-free:
// the clamp bounds are exact binary32 values inside the int32 range.
ACMMP_HD int f2i_sat(float x) {
    int r = static_cast<int>(fminf(fmaxf(x, -2147483648.0f), 2147483520.0f));
    r = x >= 2147483648.0f ? 2147483647 : r;
    return x != x ? 0 : r;
}

ACMMP_HD float det_exp(float x) {
    if (x != x) return x;
    if (x > 88.7228393554688f) return __builtin_inff();
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
    const int ki = static_cast<int>(k);
    const int k1 = ki / 2;
    const int k2 = ki - k1;
    return (p * pow2i(k1)) * pow2i(k2);
}

ACMMP_HD void det_sincos(float x, float* s, float* c) {
    if (!(fabsf(x) < 1.0e30f)) { *s = __builtin_nanf(""); *c = __builtin_nanf(""); return; }
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
    const int q = static_cast<int>(kq) & 3;
    const float ss = (q & 1) ? cr : sr;
    const float cc = (q & 1) ? sr : cr;
    *s = (q & 2) ? -ss : ss;
    *c = ((q + 1) & 2) ? -cc : cc;
}
ACMMP_HD float det_sin(float x) { float s, c; det_sincos(x, &s, &c); return s; }
ACMMP_HD float det_cos(float x) { float s, c; det_sincos(x, &s, &c); return c; }

ACMMP_HD float det_asin_core(float x, float z) {
    float p = 0.0337996557354927063f;
    p = fmaf(p, z, 0.0170816909521818161f);
    p = fmaf(p, z, 0.0311153121292591095f);
    p = fmaf(p, z, 0.0445981100201606750f);
    p = fmaf(p, z, 0.0750009864568710327f);
    p = fmaf(p, z, 0.166666656732559204f);
    return fmaf(x * z, p, x);
}

// asin with one data-dependent branch (|x| <= 0.5).  |x| > 1 and NaN need no test: they take
// the second path, where sqrt of a negative / NaN argument yields the NaN.
ACMMP_HD float det_asin(float x) {
    const float a = fabsf(x);
    float r;
    if (a <= 0.5f) {
        r = det_asin_core(a, a * a);
    } else {
        const float z = (1.0f - a) * 0.5f;
        r = fmaf(-2.0f, det_asin_core(sqrtf(z), z), kPio2Hi) + kPio2Lo;
    }
    return copysignf(r, x);
}

ACMMP_HD float det_acos(float x) {
    if (x != x) return x;
    if (fabsf(x) > 1.0f) return __builtin_nanf("");
    if (x > 0.5f) {
        const float z = (1.0f - x) * 0.5f;
        return 2.0f * det_asin_core(sqrtf(z), z);
    }
    if (x < -0.5f) {
        const float z = (1.0f + x) * 0.5f;
        return fmaf(-2.0f, det_asin_core(sqrtf(z), z), kPiHi) + kPiLo;
    }
    const float a = fabsf(x);
    const float r = copysignf(det_asin_core(a, a * a), x);
    return (kPio2Hi - r) + kPio2Lo;
}

// C99 special cases of atan2: NaN, zero and infinite arguments.
ACMMP_HD float det_atan2_special(float y, float x) {
    if (x != x || y != y) return x + y;
    const float ax = fabsf(x), ay = fabsf(y);
    const bool xneg = (f_to_bits(x) >> 31) != 0;
    if (ay == 0.0f) return xneg ? copysignf(kPiHi, y) : copysignf(0.0f, y);
    if (ax == 0.0f) return copysignf(kPio2Hi, y);
    float r;
    if (ax == __builtin_inff() && ay == __builtin_inff()) r = xneg ? 2.35619449615478516f : 0.785398185253143311f;
    else if (ax == __builtin_inff()) r = xneg ? kPiHi : 0.0f;
    else r = kPio2Hi;
    return copysignf(r, y);
}

// atan2: branch-free main path for finite non-zero arguments; the rare special arguments are
// re-evaluated by det_atan2_special in a branch that a wave only takes when one of its lanes needs it.
// t = min(|x|,|y|) / max(|x|,|y|) computed by the caller (the kernels' projection divides with
// div_proj, kernels.hip).
ACMMP_HD float det_atan2_ratio(float y, float x, float t) {
    const float ax = fabsf(x), ay = fabsf(y);
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
    const float rs = (kPio2Hi - r) + kPio2Lo;
    r = ay > ax ? rs : r;
    const float rn = (kPiHi - r) + kPiLo;
    r = (f_to_bits(x) >> 31) ? rn : r;
    r = copysignf(r, y);
    const bool regular = ay != 0.0f && ax != 0.0f && ax < __builtin_inff() && ay < __builtin_inff();
    if (!regular) r = det_atan2_special(y, x);
    return r;
}

ACMMP_HD float det_atan2(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    return det_atan2_ratio(y, x, fminf(ax, ay) / fmaxf(ax, ay));
}

ACMMP_HD float det_rsqrt(float x) { return 1.0f / sqrtf(x); }

// hypotf (SimpleFusionKernel, ACMMP.cu:1750, 1790): sqrt(x*x + y*y) with the contraction rule.
ACMMP_HD float det_hypot(float x, float y) { return sqrtf(fmaf(y, y, x * x)); }

ACMMP_HD float dot3(float a0, float a1, float a2, float b0, float b1, float b2) {
    return fmaf(a2, b2, fmaf(a1, b1, a0 * b0));
}

}  // namespace acmmp
