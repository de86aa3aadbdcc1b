// kernels.hip -- gfx950 kernels of the ACMMP-Spherical PatchMatch hot path.
//
// Reference: /root/reference/ACMMP.cu:14-1649 (RandomInitialization,
// Black/RedPixelUpdate -> CheckerboardPropagation, GetDepthandNormal,
// Black/RedPixelFilter, JBU_cu).  Semantics are those of DESIGN.md §2 (the
// reference's algorithm with its undefined / non-reproducible parts fixed), and the
// output is bit-identical to the CPU oracle (oracle/acmmp_oracle.c).
//
// Structure:
//  * one lane per pixel of the colour being updated, 64x4 workgroups over the
//    colour-split grid, so a wave owns 64 consecutive same-colour pixels of a row;
//  * the 36-sample bilateral NCC is evaluated sample-outer / view-inner: the
//    view-independent part of a sample (ray, plane depth, world point) is computed
//    once and projected into a chunk of VB source views held in registers;
//  * bilateral weights, w*ref and ref texels are per-pixel tables built once per
//    run (they depend only on the reference image), so no exp() runs per sample;
//  * current-hypothesis and refinement costs are evaluated only for views some
//    lane of the wave selected (zero-weight views add exactly +0 in the reference).
#include <algorithm>
#include <cstdlib>

#include "detmath.h"
#include "engine.h"
#include "planar.h"

// Translation-unit split: build.py compiles this file once per ACMMP_TU value (0..kTUs-1), in
// parallel, and every kernel instance and host launcher lands in exactly one of those objects.  With
// ACMMP_TU unset the whole file is one unit.
#ifndef ACMMP_TU
#define ACMMP_TU -1
#endif
#define ACMMP_IN_TU(n) (ACMMP_TU < 0 || ACMMP_TU == (n))

namespace acmmp {

// Two-lane f32 vectors: arithmetic on them issues as the packed VALU forms (v_pk_fma_f32 / v_pk_mul_f32 /
// v_pk_add_f32: two IEEE single-precision operations per lane in one issue slot, scripts/micro/pk_rate.hip:
// 123 TFLOP/s against 71 for v_fma_f32), with scalar operands broadcast through op_sel.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 splat2(float x) { return (f32x2){x, x}; }

// ------------------------------------------------------------------ RNG

__device__ __forceinline__ uint4 philox10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                          uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
}

// curand_init(seed, subsequence = row-major pixel, 0) on a Philox4_32_10 state; uniform() = curand_uniform
struct Rng {
    uint32_t k0, k1, sub, n, blk_id;
    uint4 blk;
    __device__ __forceinline__ void init(uint32_t seed_lo, uint32_t seed_hi, uint32_t pixel, uint32_t count) {
        k0 = seed_lo; k1 = seed_hi; sub = pixel; n = count; blk_id = 0xFFFFFFFFu;
    }
    __device__ __forceinline__ float uniform() {
        const uint32_t b = n >> 2;
        if (b != blk_id) { blk = philox10(b, 0u, sub, 0u, k0, k1); blk_id = b; }
        const uint32_t w = n & 3u;
        const uint32_t x = w == 0 ? blk.x : (w == 1 ? blk.y : (w == 2 ? blk.z : blk.w));
        ++n;
        return fmaf(static_cast<float>(x), 2.3283064365386963e-10f, 1.1641532182693481e-10f);
    }
};

// ------------------------------------------------------------------ camera model

__device__ __forceinline__ void normalize3(float& x, float& y, float& z) {
    const float inv = det_rsqrt(dot3(x, y, z, x, y, z));
    x *= inv; y *= inv; z *= inv;
}

// PixelToDir, ACMMP.cu:119-134
__device__ __forceinline__ float3 pixel_to_dir(const DevCam& c, int px, int py) {
    float3 d;
    if (c.model == kPinhole) {
        d.x = (static_cast<float>(px) - c.K[2]) / c.K[0];
        d.y = (static_cast<float>(py) - c.K[5]) / c.K[4];
        d.z = 1.f;
        normalize3(d.x, d.y, d.z);
    } else {
        const float lon = (static_cast<float>(px) - c.cx) / static_cast<float>(c.W) * 2.0f * kCudartPiF;
        const float lat = -(static_cast<float>(py) - c.cy) / static_cast<float>(c.H) * kCudartPiF;
        float sl, cl, sa, ca;
        det_sincos(lon, &sl, &cl);
        det_sincos(lat, &sa, &ca);
        d.x = ca * sl;
        d.y = -sa;
        d.z = ca * cl;
    }
    return d;
}

template <typename Cam>
__device__ __forceinline__ float3 rotate_to_world(Cam& c, float x, float y, float z) {
    float3 r;
    r.x = dot3(c.R[0], c.R[3], c.R[6], x, y, z) + c.C[0];
    r.y = dot3(c.R[1], c.R[4], c.R[7], x, y, z) + c.C[1];
    r.z = dot3(c.R[2], c.R[5], c.R[8], x, y, z) + c.C[2];
    return r;
}

// Get3DPointonWorld_cu (ACMMP.cu:565-600) at arbitrary float coordinates.
template <int MODEL>
__device__ __forceinline__ float3 world_point(const DevCam& c, float x, float y, float depth) {
    if (MODEL == kSphere) {
        const float lon = (x - c.cx) / static_cast<float>(c.W) * 2.0f * kCudartPiF;
        const float lat = -(y - c.cy) / static_cast<float>(c.H) * kCudartPiF;
        float sl, cl, sa, ca;
        det_sincos(lon, &sl, &cl);
        det_sincos(lat, &sa, &ca);
        return rotate_to_world(c, (ca * sl) * depth, (-sa) * depth, (ca * cl) * depth);
    } else {
        return rotate_to_world(c, (depth * (x - c.K[2])) * c.inv_fx, (depth * (y - c.K[5])) * c.inv_fy, depth);
    }
}

// The same at an integer reference pixel whose ray `d` is already known (SPHERE's
// camera-frame point is ray * depth exactly as Get3DPointonWorld_cu rounds it).
template <int MODEL, typename Cam>
__device__ __forceinline__ float3 world_point_ray(Cam& c, int x, int y, float depth, float4 d) {
    if (MODEL == kSphere) {
        return rotate_to_world(c, d.x * depth, d.y * depth, d.z * depth);
    } else {
        return rotate_to_world(c, (depth * (static_cast<float>(x) - c.K[2])) * c.inv_fx,
                               (depth * (static_cast<float>(y) - c.K[5])) * c.inv_fy, depth);
    }
}

// Single-instruction helpers with the hardware's own semantics (inline asm, so the compiler neither
// canonicalises operands nor widens them): v_cvt_i32_f32 truncates, saturates and maps NaN to 0
// (= f2i_sat); v_med3_i32 clamps; v_mad_u32_u24 multiplies 24-bit operands.  None of them may read a
// transcendental's result directly (see max_abs below); scripts/hazard_scan.py checks the built code.
__device__ __forceinline__ int cvt_i32(float x) {
    int r;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ int cvt_flr_i32(float x) {             // cvt_i32(floorf(x)) in one instruction
    int r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ int clamp_m1(int x, int hi) {          // clampi(x, -1, hi), hi wave-uniform
    int r;
    asm("v_med3_i32 %0, %1, -1, %2" : "=v"(r) : "v"(x), "s"(hi));
    return r;
}
__device__ __forceinline__ unsigned mad_u24(unsigned a, unsigned b, unsigned c) {  // a, b < 2^24, b uniform
    unsigned r;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    return r;
}
// |a| vs |b| for the atan2 range reductions.  gfx950 wants one wait state between a VALU transcendental
// (v_sqrt, v_rcp, ...) and the first instruction reading its result; the compiler's hazard recognizer inserts
// it for the instructions it can see, not for inline asm.  Round 6 found an inline-asm v_max_f32 scheduled
// directly after the v_sqrt of hypot(x, z): it read a half-written register (wrong costs in lane groups 0-3 of
// every 8 in k_eval_ref's instances, found by a paired-sample loop whose schedule put the two together; the
// round-5 tree had the pair in its V = 1 k_eval_ref instances only).  So:
//   max_abs / min_abs      the builtins (general operands; never signalling NaNs, so no canonicalisation)
//   max_abs_nt / min_abs_nt inline asm, operands never a transcendental's result (the rigid transform's fmas)
//   max_abs_h / min_abs_h  inline asm behind an s_nop 0, for the hypot operand
// The asm forms keep the scheduler's round-5 order in the fast SPHERE projections: both pairs on the builtins
// measured k_eval_nb 1.444 ms against 1.428 ms this way (profiles/r06_ab8_hazard_ab.txt).
// scripts/hazard_scan.py checks the device assembly for (transcendental, immediate reader) pairs.
__device__ __forceinline__ float max_abs(float a, float b) { return __builtin_fmaxf(fabsf(a), fabsf(b)); }
__device__ __forceinline__ float min_abs(float a, float b) { return __builtin_fminf(fabsf(a), fabsf(b)); }
__device__ __forceinline__ float max_abs_nt(float a, float b) {
    float r;
    asm("v_max_f32_e64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float min_abs_nt(float a, float b) {
    float r;
    asm("v_min_f32_e64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float max_abs_h(float a, float b) {
    float r;
    asm("s_nop 0\n\tv_max_f32_e64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float min_abs_h(float a, float b) {
    float r;
    asm("s_nop 0\n\tv_min_f32_e64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float clamp0(float x, float hi) {        // fminf(fmaxf(x, 0), hi), hi uniform
    float r;
    asm("v_max_f32_e32 %0, 0, %1\n\tv_min_f32_e32 %0, %2, %0" : "=&v"(r) : "v"(x), "s"(hi));
    return r;
}

// sqrtf for the SPHERE projection: LLVM's IEEE f32 sqrt lowering (v_sqrt_f32, then the +-1 ulp
// fma fix-up) without its small-argument rescale and its +-0/inf class select.  Bit-identical to
// sqrtf for every x >= 2^-96, +inf and NaN; for smaller x the result is still < 1e-6 and the
// projection replaces it by the principal point (d < 1e-6 select), and the depth it returns is
// unused by every caller, so outputs never differ.
__device__ __forceinline__ float sqrt_proj(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __builtin_bit_cast(float, __builtin_bit_cast(int, s) - 1);
    const float sup = __builtin_bit_cast(float, __builtin_bit_cast(int, s) + 1);
    const float r = fmaf(-sdn, s, x) <= 0.0f ? sdn : s;
    return fmaf(-sup, s, x) > 0.0f ? sup : r;
}

// a / b for the SPHERE projection: LLVM's IEEE f32 division sequence (v_rcp_f32, one Newton step
// on the reciprocal, two residual corrections, the last one fused) without v_div_scale's exponent
// pre-scaling and v_div_fixup's special-case pass.  Bit-identical to a / b whenever |b| lies in
// [2^-125, 2^125] and |a| >= 2^-102 or a == 0 (the sign of a zero quotient may differ); the two
// projection callers (ty / d and the atan2 ratio min / max) only leave that range for a point
// closer than 2^-102 to the camera centre (replaced by the principal point) or a quotient below
// 2^-80, whose contribution to the pixel coordinate is absorbed by cx / cy.
__device__ __forceinline__ float div_proj(float a, float b) {
    float y = __builtin_amdgcn_rcpf(b);
    y = fmaf(fmaf(-b, y, 1.0f), y, y);
    float q = a * y;
    q = fmaf(fmaf(-b, q, a), y, q);
    return fmaf(fmaf(-b, q, a), y, q);
}

__device__ __forceinline__ float atan2_proj(float y, float x) {
    return det_atan2_ratio(y, x, div_proj(min_abs(x, y), max_abs(x, y)));
}

// det_asin with its large-argument square root through sqrt_proj: there z = (1 - |x|) / 2 is 0, NaN,
// negative (|x| > 1 by rounding) or >= 2^-25 (1 - |x| is exact and at least 2^-24), where sqrt_proj
// equals sqrtf bit for bit.
__device__ __forceinline__ float asin_proj(float x) {
    // straight-line: one polynomial on selected arguments (no divergent branch, so the compiler can
    // interleave the views of a chunk; r01_v25 A/B +0.5%)
    const float a = fabsf(x);
    const bool small = a <= 0.5f;
    const float zl = (1.0f - a) * 0.5f;
    const float c = det_asin_core(small ? a : sqrt_proj(zl), small ? a * a : zl);
    return copysignf(small ? c : fmaf(-2.0f, c, kPio2Hi) + kPio2Lo, x);
}

// ProjectonCamera_cu, ACMMP.cu:602-644 (Cam: DevCam in any address space)
template <int MODEL, typename Cam, bool EXACT_DEPTH = false>
__device__ __forceinline__ void project(Cam& c, float3 P, float& ox, float& oy, float& depth) {
    const float tx = dot3(c.R[0], c.R[1], c.R[2], P.x, P.y, P.z) + c.t[0];
    const float ty = dot3(c.R[3], c.R[4], c.R[5], P.x, P.y, P.z) + c.t[1];
    const float tz = dot3(c.R[6], c.R[7], c.R[8], P.x, P.y, P.z) + c.t[2];
    if (MODEL == kSphere) {
        // sqrt_proj differs from sqrtf only below 2^-96, where the point is replaced by the principal
        // point; callers that use the returned depth (fusion) ask for the IEEE square root
        const float d = EXACT_DEPTH ? sqrtf(dot3(tx, ty, tz, tx, ty, tz)) : sqrt_proj(dot3(tx, ty, tz, tx, ty, tz));
        depth = d;
        const float neg_lat = asin_proj(EXACT_DEPTH ? ty / d : div_proj(ty, d));
        const float lon = EXACT_DEPTH ? det_atan2(tx, tz) : atan2_proj(tx, tz);
        ox = fmaf(lon * kInv2Pi, c.Wf, c.cx);
        oy = fmaf(neg_lat * kInvPi, c.Hf, c.cy);
        if (d < 1e-6f) { ox = c.cx; oy = c.cy; }        // (:618-622) selected, not branched around
    } else {
        depth = tz;
        const float inv = 1.0f / tz;
        ox = dot3(c.K[0], c.K[1], c.K[2], tx, ty, tz) * inv;
        oy = dot3(c.K[3], c.K[4], c.K[5], tx, ty, tz) * inv;
    }
}

// ComputeDepthfromPlaneHypothesis, ACMMP.cu:187-193
__device__ __forceinline__ float depth_from_plane(float4 ph, float4 d) {
    const float denom = dot3(ph.x, ph.y, ph.z, d.x, d.y, d.z);
    return (fabsf(denom) < 1e-6f) ? 1e6f : (-ph.w / denom);
}

// ------------------------------------------------------------------ fast-math sample projection
//
// KParams::fast (acmmp_set_math): the per-sample arithmetic of ComputeBilateralNCC
// (ACMMP.cu:456-476) as the reference's --use_fast_math build (CMakeLists.txt:42) treats it --
// hardware v_rsq / v_sqrt / v_rcp (<= 1 ulp) instead of the IEEE division and square-root
// sequences, the translation folded into the rotation's fma chain, W / 2pi and H / pi folded into
// one constant, and the asin / atan2 polynomials without their special-argument paths (a point on
// the source camera's vertical axis, tx = tz = 0, has no defined longitude; the reference's atan2f
// returns 0 there, this returns NaN and the sample's cost is 2.0).  Not bit-identical to the
// oracle: parity is the tolerance of SURVEY.md §8c (tests/test_gpu_fastmath.py).

// Chunks whose VB views are all present compile without per-view guards (one basic block per sample):
// every pinhole chunk (+17% at C2, V = 10: its 8-view chunk) and SPHERE chunks of at most 2 views
// (k_eval_ref's 2-view chunks at V = 15 +4.7%; SPHERE's 4-view k_eval_nb chunks lose 1-3% that way,
// longer live ranges -- r02 A/B profiles/r02_full_chunk_ab.txt).  The fast mode has no |t| < 1e-6 test
// per view-sample (3 VALU; r02 A/B profiles/r02_micro_ab.txt: metric +2%, C3 +1.8%).

// atan(t) on [0, 1]: t + t^3 P(t^2), 7-term minimax, max |error| 1.1e-7 rad
__device__ __forceinline__ float atan_core_fast(float t) {
    const float z = t * t;
    float p = -0.004355291370302439f;
    p = fmaf(p, z, 0.023039722815155983f);
    p = fmaf(p, z, -0.05777300149202347f);
    p = fmaf(p, z, 0.09794192016124725f);
    p = fmaf(p, z, -0.139765664935112f);
    p = fmaf(p, z, 0.19962701201438904f);
    p = fmaf(p, z, -0.3333165943622589f);
    return fmaf(t * z, p, t);
}

// The same for two arguments at once, in packed VALU operations.
__device__ __forceinline__ f32x2 atan_core_fast2(f32x2 t) {
    const f32x2 z = t * t;
    f32x2 p = splat2(-0.004355291370302439f);
    p = pk_fma(p, z, splat2(0.023039722815155983f));
    p = pk_fma(p, z, splat2(-0.05777300149202347f));
    p = pk_fma(p, z, splat2(0.09794192016124725f));
    p = pk_fma(p, z, splat2(-0.139765664935112f));
    p = pk_fma(p, z, splat2(0.19962701201438904f));
    p = pk_fma(p, z, splat2(-0.3333165943622589f));
    return pk_fma(t * z, p, t);
}

// SPHERE: the source pixel of the direction (t.x, t.y, tz) in the source camera's frame.  Longitude =
// atan2(tx, tz) (ProjectonCamera_cu :631) and -latitude = asin(ty / |t|) (:626-630) = atan2(ty, hypot(tx, tz)):
// both through ONE packed atan over y = (tx, ty), x = (tz, h) -- the minimax atan of atan_core_fast
// (1.1e-7 rad) for the latitude too, in place of the asin polynomial with its range reduction and square
// root.  Invariant under a positive scale of the direction.
template <typename Cam>
__device__ __forceinline__ void sphere_pixel_fast(Cam& c, f32x2 t, float tz, float& ox, float& oy) {
    const float h = __builtin_amdgcn_sqrtf(fmaf(tz, tz, t.x * t.x));
    const f32x2 mn = (f32x2){min_abs_nt(tz, t.x), min_abs_h(h, t.y)};
    const f32x2 rc = (f32x2){__builtin_amdgcn_rcpf(max_abs_nt(tz, t.x)), __builtin_amdgcn_rcpf(max_abs_h(h, t.y))};
    f32x2 r = atan_core_fast2(mn * rc);
    const f32x2 rq = splat2(kPio2Hi) - r;                          // |y| > |x|: pi/2 - atan(|x| / |y|)
    r.x = fabsf(t.x) > fabsf(tz) ? rq.x : r.x;
    r.y = fabsf(t.y) > h ? rq.y : r.y;
    r.x = __builtin_bit_cast(int, tz) < 0 ? kPiHi - r.x : r.x;   // x < 0 (h >= 0 never is)
    const f32x2 ang = (f32x2){copysignf(r.x, t.x), copysignf(r.y, t.y)};
    const f32x2 o = pk_fma(ang, (f32x2){c.fkx, c.fky}, (f32x2){c.cx, c.cy});
    ox = o.x;
    oy = o.y;
}

// P: the sample's point in the REFERENCE camera's frame (depth * ray); FR / Ft map it into the source
// camera (DevCam::FRxy / FRz / Ft, set per problem), so no world point is formed per sample.  Rows 0
// and 1 of FR are interleaved in DevCam so (x, y) of the mapped point is one packed fma chain (the same
// fma order per row as three separate rows), with the pair of constants as one SGPR pair.
// ft: the translation Ft, from the camera (nullptr) or from registers the caller holds (a VOP3 fma reads
// one SGPR, so a translation in SGPRs costs a move per row and view-sample)
// Two directions at once, their two atan polynomials as interleaved packed chains (a chain of dependent
// v_pk_fma_f32 waits a hazard cycle between steps, s_nop; two chains fill each other's), the same operations per
// direction as sphere_pixel_fast, so the same bits
template <typename Cam>
__device__ __forceinline__ void sphere_pixel_fast_x2(Cam& c, f32x2 ta, float tza, f32x2 tb, float tzb, float& oxa,
                                                     float& oya, float& oxb, float& oyb) {
    const float ha = __builtin_amdgcn_sqrtf(fmaf(tza, tza, ta.x * ta.x));
    const float hb = __builtin_amdgcn_sqrtf(fmaf(tzb, tzb, tb.x * tb.x));
    const f32x2 mna = (f32x2){min_abs_nt(tza, ta.x), min_abs_h(ha, ta.y)};
    const f32x2 mnb = (f32x2){min_abs_nt(tzb, tb.x), min_abs_h(hb, tb.y)};
    const f32x2 rca = (f32x2){__builtin_amdgcn_rcpf(max_abs_nt(tza, ta.x)), __builtin_amdgcn_rcpf(max_abs_h(ha, ta.y))};
    const f32x2 rcb = (f32x2){__builtin_amdgcn_rcpf(max_abs_nt(tzb, tb.x)), __builtin_amdgcn_rcpf(max_abs_h(hb, tb.y))};
    const f32x2 ua = mna * rca, ub = mnb * rcb;
    const f32x2 za = ua * ua, zb = ub * ub;
    f32x2 pa = splat2(-0.004355291370302439f), pb = pa;
    pa = pk_fma(pa, za, splat2(0.023039722815155983f));
    pb = pk_fma(pb, zb, splat2(0.023039722815155983f));
    pa = pk_fma(pa, za, splat2(-0.05777300149202347f));
    pb = pk_fma(pb, zb, splat2(-0.05777300149202347f));
    pa = pk_fma(pa, za, splat2(0.09794192016124725f));
    pb = pk_fma(pb, zb, splat2(0.09794192016124725f));
    pa = pk_fma(pa, za, splat2(-0.139765664935112f));
    pb = pk_fma(pb, zb, splat2(-0.139765664935112f));
    pa = pk_fma(pa, za, splat2(0.19962701201438904f));
    pb = pk_fma(pb, zb, splat2(0.19962701201438904f));
    pa = pk_fma(pa, za, splat2(-0.3333165943622589f));
    pb = pk_fma(pb, zb, splat2(-0.3333165943622589f));
    f32x2 ra = pk_fma(ua * za, pa, ua);
    f32x2 rb = pk_fma(ub * zb, pb, ub);
    const f32x2 rqa = splat2(kPio2Hi) - ra, rqb = splat2(kPio2Hi) - rb;
    ra.x = fabsf(ta.x) > fabsf(tza) ? rqa.x : ra.x;
    rb.x = fabsf(tb.x) > fabsf(tzb) ? rqb.x : rb.x;
    ra.y = fabsf(ta.y) > ha ? rqa.y : ra.y;
    rb.y = fabsf(tb.y) > hb ? rqb.y : rb.y;
    ra.x = __builtin_bit_cast(int, tza) < 0 ? kPiHi - ra.x : ra.x;
    rb.x = __builtin_bit_cast(int, tzb) < 0 ? kPiHi - rb.x : rb.x;
    const f32x2 anga = (f32x2){copysignf(ra.x, ta.x), copysignf(ra.y, ta.y)};
    const f32x2 angb = (f32x2){copysignf(rb.x, tb.x), copysignf(rb.y, tb.y)};
    const f32x2 oa = pk_fma(anga, (f32x2){c.fkx, c.fky}, (f32x2){c.cx, c.cy});
    const f32x2 ob = pk_fma(angb, (f32x2){c.fkx, c.fky}, (f32x2){c.cx, c.cy});
    oxa = oa.x; oya = oa.y; oxb = ob.x; oyb = ob.y;
}

template <typename Cam>
__device__ __forceinline__ void rigid_fast(Cam& c, float3 P, f32x2& t, float& tz, const float* ft = nullptr) {
    const f32x2 fxy = ft ? (f32x2){ft[0], ft[1]} : (f32x2){c.Ft[0], c.Ft[1]};
    const float fz = ft ? ft[2] : c.Ft[2];
    t = pk_fma((f32x2){c.FRxy[0], c.FRxy[1]}, splat2(P.x), fxy);
    t = pk_fma((f32x2){c.FRxy[2], c.FRxy[3]}, splat2(P.y), t);
    t = pk_fma((f32x2){c.FRxy[4], c.FRxy[5]}, splat2(P.z), t);
    tz = fmaf(c.FRz[2], P.z, fmaf(c.FRz[1], P.y, fmaf(c.FRz[0], P.x, fz)));
}

template <int MODEL, typename Cam>
__device__ __forceinline__ void project_fast(Cam& c, float3 P, float& ox, float& oy, const float* ft = nullptr) {
    f32x2 t;
    float tz;
    rigid_fast(c, P, t, tz, ft);
    if (MODEL == kSphere) {
        sphere_pixel_fast(c, t, tz, ox, oy);
        // |t| < 1e-6 (:618-622), a sample on a source camera's centre, is not tested: such a sample
        // projects to NaN and its view's cost is 2.0 (the NCC clamp) -- the reference's tex2D of
        // (cx, cy) there is as meaningless, and no real geometry reaches it
    } else {
        // K (R_rel P + b) rows 0-1; the perspective divide by its row 2
        const f32x2 o = t * splat2(__builtin_amdgcn_rcpf(tz));
        ox = o.x;
        oy = o.y;
    }
}

// The fast path's sample point in the reference camera's frame (project_fast maps it onward):
// SPHERE depth * ray, PINHOLE depth-as-z (Get3DPointonWorld_cu's pinhole branch, :579-581)
template <int MODEL, typename Cam>
__device__ __forceinline__ float3 cam_point_fast(Cam& c, int x, int y, float depth, float4 d) {
    if (MODEL == kSphere) return make_float3(d.x * depth, d.y * depth, d.z * depth);
    return make_float3((depth * (static_cast<float>(x) - c.K[2])) * c.inv_fx,
                       (depth * (static_cast<float>(y) - c.K[5])) * c.inv_fy, depth);
}

// ComputeDepthfromPlaneHypothesis with the hardware reciprocal
__device__ __forceinline__ float depth_from_plane_fast(float4 ph, float4 d) {
    const float denom = dot3(ph.x, ph.y, ph.z, d.x, d.y, d.z);
    return (fabsf(denom) < 1e-6f) ? 1e6f : (-ph.w * __builtin_amdgcn_rcpf(denom));
}

// GetDistance2Origin, ACMMP.cu:168-173
__device__ __forceinline__ float dist_to_origin(float4 d, float depth, float4 n) {
    return -dot3(n.x, n.y, n.z, d.x * depth, d.y * depth, d.z * depth);
}

// TransformNormal / TransformNormal2RefCam, ACMMP.cu:378-396
__device__ __forceinline__ float4 to_world(const DevCam& c, float4 n) {
    return make_float4(dot3(c.R[0], c.R[3], c.R[6], n.x, n.y, n.z), dot3(c.R[1], c.R[4], c.R[7], n.x, n.y, n.z),
                       dot3(c.R[2], c.R[5], c.R[8], n.x, n.y, n.z), n.w);
}
__device__ __forceinline__ float4 to_ref(const DevCam& c, float4 n) {
    return make_float4(dot3(c.R[0], c.R[1], c.R[2], n.x, n.y, n.z), dot3(c.R[3], c.R[4], c.R[5], n.x, n.y, n.z),
                       dot3(c.R[6], c.R[7], c.R[8], n.x, n.y, n.z), n.w);
}

__device__ __forceinline__ float dot3n(float4 a, float4 b) { return dot3(a.x, a.y, a.z, b.x, b.y, b.z); }

// ------------------------------------------------------------------ texture fetches

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// tex2D(img, ix+0.5, iy+0.5): exact texel with clamp addressing (padded image base = texel (-1,-1))
__device__ __forceinline__ float texel_padded(const float* img, int pitch, int W, int H, int ix, int iy) {
    return img[static_cast<long long>(clampi(iy, 0, H - 1) + 1) * pitch + clampi(ix, 0, W - 1) + 1];
}

__device__ __forceinline__ float texel_plain(const float* img, int W, int H, int ix, int iy) {
    return img[static_cast<long long>(clampi(iy, 0, H - 1)) * W + clampi(ix, 0, W - 1)];
}

// ------------------------------------------------------------------ helpers over KParams

// Reference-camera ray of pixel (x, y), |x - px|, |y - py| <= R (PixelToDir, ACMMP.cu:119-134).
// SPHERE: (cos lat * sin lon, -sin lat, cos lat * cos lon) from the separable tables -- the same
// two products PixelToDir rounds.  PINHOLE: the precomputed table.
template <int MODEL>
__device__ __forceinline__ float4 ray_at(const KParams& kp, int x, int y) {
    if (MODEL == kSphere) {
        const float2 r = kp.sph_row[y + kp.R];
        const float2 c = kp.sph_col[x + kp.R];
        return make_float4(r.y * c.x, -r.x, r.y * c.y, 0.0f);
    }
    return kp.dirs[static_cast<long long>(y + kp.R) * kp.dpitch + (x + kp.R)];
}
__device__ __forceinline__ long long cs_index(const KParams& kp, int x, int y) {
    return static_cast<long long>(y) * kp.Wh + (x >> 1);
}
__device__ __forceinline__ int uniform_int(int v) { return __builtin_amdgcn_readfirstlane(v); }

// ------------------------------------------------------------------ NCC over a chunk of views

// Per-pixel patch, staged in LDS once per launch: for every sample s of the 6x6 stride-2 window
// (ACMMP.cu:450-451) the reference ray (PixelToDir of the sample pixel), the bilateral weight
// w_s (ACMMP.cu:398-403, 482-486) and the reference texel.  SPHERE's weight sums are
// hypothesis- and view-independent (no sample is ever skipped there).
struct Patch {
    const float4* rw;               // [s * stride] = (ray.x, ray.y, ray.z, w); null when not staged
    const float* rr;                // [s * stride] = reference texel
    const float2* wr;               // lite staging: [s * stride] = (w, texel); rays re-read from the tables
    const float2* row;              // separable SPHERE staging (STAGED 4): (sin, cos) latitude per patch row
    const float2* col;              //   and (sin, cos) longitude per patch column; wr holds (w, texel)
    int stride;
    float center;                   // reference texel at the pixel
    float sbw, sref, srr;
};

typedef float float2u __attribute__((ext_vector_type(2), aligned(4)));

// tex2D(img, x+0.5, y+0.5) with fp32 bilinear weights and clamp addressing.  The one-texel
// replicated border makes (ix, ix+1) valid for ix in [-1, W-1], which equals clamping both,
// and lets each row of the footprint be one 8-byte load.
__device__ __forceinline__ float bilinear_pair(const float* img, int pitch, int W, int H, float x, float y) {
    const float fx = floorf(x), fy = floorf(y);
    const float a = x - fx, b = y - fy;
    const int ix = clampi(f2i_sat(fx), -1, W - 1);
    const int iy = clampi(f2i_sat(fy), -1, H - 1);
    const float* p0 = img + static_cast<long long>(iy + 1) * pitch + (ix + 1);
    const float2u top = *reinterpret_cast<const float2u*>(p0);
    const float2u bot = *reinterpret_cast<const float2u*>(p0 + pitch);
    const float r0 = fmaf(a, top.y - top.x, top.x);
    const float r1 = fmaf(a, bot.y - bot.x, bot.x);
    return fmaf(b, r1 - r0, r0);
}

// The same fetch through a buffer descriptor of the view's padded image (32-bit texel offsets,
// 24-bit multiply), split into issue (Tap) and use (lerp_tap) so a caller can put the loads of
// several views in flight before consuming any.  SPHERE callers pass x already wrapped and y
// clamped to [0, H-1] (never NaN), so y needs no clamp; x keeps clampi(f2i_sat(floor x), -1, W-1):
// the float clamp below is the same map for every non-NaN value, and NaN -> 0 as f2i_sat does.
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
struct Tap {
    float a, b;
    f32x2 top, bot;
    u32x2 pw;                       // binary16: the footprint's two row-pair words
};

// ix = clampi(f2i_sat(floor x), -1, W-1), iy likewise (SPHERE: y already in [0, H-1], so iy = (int)floor y
// >= 0); the footprint's top-left texel sits at byte (iy+1)*pitch4 + (ix+1)*4 of the padded image.
// SPHERE moves the +1 row into the scalar offsets (top row soffset = pitch4, bottom = 2*pitch4).
//
// TEX = 1 reads the binary16 copy instead (DevCam::img16_base, row-pair layout: word (X, Y) =
// (t(X, Y), t(X, Y + 1)), 4 B per texel position, the fp32 image's offsets): the footprint is the two
// words at (ix + 1, iy + 1) and (ix + 2, iy + 1), one 8-byte load (r02 A/B against two 4-byte row
// loads: +1% exact, +3.6% fast at the metric, neutral at C2/C3).
template <int TEX, bool Y_IN_RANGE, typename Cam>
__device__ __forceinline__ Tap fetch_tap(__amdgpu_buffer_rsrc_t rs, Cam& c, float x, float y) {
    const float fx = floorf(x), fy = floorf(y);
    Tap t;
    t.a = x - fx;
    t.b = y - fy;
    if (TEX == 1) {
        // the same footprint with v_fract_f32 / v_cvt_flr_i32_f32 (one instruction each instead of floor
        // + sub / floor + cvt).  fract(x) = min(x - floor(x), 1 - 2^-24) equals x - floor(x) unless x is
        // in (-2^-24, 0): a SPHERE x is wrapped (a negative one is sx - k W, a multiple of ulp(W) >= 2^-23)
        // and y clamped to [0, H-1]; a pinhole sample outside [0, W) x [0, H) is never accumulated.
        t.a = __builtin_amdgcn_fractf(x);
        t.b = __builtin_amdgcn_fractf(y);
        const unsigned ix4 = (static_cast<unsigned>(clamp_m1(cvt_flr_i32(x), c.Wm1)) << 2) + 4u;
        if (Y_IN_RANGE) {
            const unsigned off = mad_u24(static_cast<unsigned>(cvt_flr_i32(y)), c.pitch4, ix4);
            t.pw = __builtin_amdgcn_raw_buffer_load_b64(rs, off, c.pitch4, 0);
        } else {
            const unsigned off = mad_u24(static_cast<unsigned>(clamp_m1(cvt_flr_i32(y), c.Hm1) + 1), c.pitch4, ix4);
            t.pw = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
        }
        return t;
    }
    const unsigned ix4 = (static_cast<unsigned>(clamp_m1(cvt_i32(fx), c.Wm1)) << 2) + 4u;
    if (Y_IN_RANGE) {
        const unsigned off = mad_u24(static_cast<unsigned>(cvt_i32(fy)), c.pitch4, ix4);
        t.top = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, c.pitch4, 0));
        t.bot = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 2 * c.pitch4, 0));
    } else {
        const unsigned off = mad_u24(static_cast<unsigned>(clamp_m1(cvt_i32(fy), c.Hm1) + 1), c.pitch4, ix4);
        t.top = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
        t.bot = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, c.pitch4, 0));
    }
    return t;
}

// Pinhole: ix = cvt_flr_i32(x), iy = cvt_flr_i32(y) of the sample; the sample is in the source image
// (ProjectonCamera's caller, ACMMP.cu:470-473: !(x < 0 || x >= W || y < 0 || y >= H)) exactly when both are
// in [0, W-1] / [0, H-1] as unsigned compares -- the same verdict for every float, NaN included (the float
// compares pass a NaN coordinate, and v_cvt_flr_i32_f32 maps NaN to 0) and +-inf / out-of-int-range values
// (saturated).  Two compares against the integers the fetch needs anyway, instead of four float ones.
template <typename Cam>
__device__ __forceinline__ bool pin_in_image(Cam& c, int ix, int iy) {
    return (static_cast<unsigned>(ix) <= static_cast<unsigned>(c.Wm1)) &
           (static_cast<unsigned>(iy) <= static_cast<unsigned>(c.Hm1));
}

// The pinhole footprint at (ix, iy) = floor(x, y) without fetch_tap's clamps: an in-image sample's
// footprint is inside the padded image, and an out-of-image one is never accumulated (its weight and
// texel are selected to zero), so its offset may be anything -- the buffer descriptor's range check
// returns 0 for an offset past the image, and one inside it reads some texel that is discarded.  The
// row +1 of the padding goes into the scalar offsets.  Same addresses and weights as fetch_tap for
// every in-image sample.
template <int TEX>
__device__ __forceinline__ Tap fetch_tap_pin_p(__amdgpu_buffer_rsrc_t rs, int pitch4, float x, float y, int ix, int iy) {
    Tap t;
    const unsigned off = mad_u24(static_cast<unsigned>(iy), pitch4, (static_cast<unsigned>(ix) << 2) + 4u);
    if (TEX == 1) {
        t.a = __builtin_amdgcn_fractf(x);           // = x - floor(x) for x >= 0 (fetch_tap's note)
        t.b = __builtin_amdgcn_fractf(y);
        t.pw = __builtin_amdgcn_raw_buffer_load_b64(rs, off, pitch4, 0);
        return t;
    }
    t.a = x - floorf(x);
    t.b = y - floorf(y);
    t.top = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, pitch4, 0));
    t.bot = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 2 * pitch4, 0));
    return t;
}
template <int TEX, typename Cam>
__device__ __forceinline__ Tap fetch_tap_pin(__amdgpu_buffer_rsrc_t rs, Cam& c, float x, float y, int ix, int iy) {
    return fetch_tap_pin_p<TEX>(rs, c.pitch4, x, y, ix, iy);
}

// fmaf(a, d, (float)lo(v)) in one v_fma_mix_f32
__device__ __forceinline__ float f16_fma_lo(float a, float d, unsigned v) {
    float r;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,0,1]" : "=v"(r) : "v"(a), "v"(d), "v"(v));
    return r;
}

// row-pair words w0 = (t00, t01), w1 = (t10, t11): t10 - t00 and t11 - t01, each rounded once
__device__ __forceinline__ float f16_lo_diff(unsigned w1, unsigned w0) {
    float r;
    asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(w1), "v"(w0));
    return r;
}
__device__ __forceinline__ float f16_hi_diff(unsigned w1, unsigned w0) {
    float r;
    asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[1,0,1] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(w1), "v"(w0));
    return r;
}
// fmaf(a, d, (float)hi(v)) in one v_fma_mix_f32
__device__ __forceinline__ float f16_fma_hi(float a, float d, unsigned v) {
    float r;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r) : "v"(a), "v"(d), "v"(v));
    return r;
}

template <int TEX = 0>
__device__ __forceinline__ float lerp_tap(const Tap& t) {
    if (TEX == 1) {
        // (the words stay in the load's own vector type: a round trip through f32x2 lanes was folded
        // into one lane by this compiler)
        const unsigned w0 = t.pw[0], w1 = t.pw[1];
        const float r0 = f16_fma_lo(t.a, f16_lo_diff(w1, w0), w0);
        const float r1 = f16_fma_hi(t.a, f16_hi_diff(w1, w0), w0);
        return fmaf(t.b, r1 - r0, r0);
    }
    const float r0 = fmaf(t.a, t.top.y - t.top.x, t.top.x);
    const float r1 = fmaf(t.a, t.bot.y - t.bot.x, t.bot.x);
    return fmaf(t.b, r1 - r0, r0);
}

// Sample s = (i, j) of pixel (px, py): ray, bilateral weight and reference texel.
template <int MODEL>
__device__ __forceinline__ float4 patch_sample(const KParams& kp, int px, int py, int s, int i, int j, float center,
                                               float& r) {
    const DevCam& rc = kp.cams[0];
    r = texel_padded(rc.img_base, rc.img_pitch, rc.W, rc.H, px + i, py + j);
    const float sp = kp.spatial[(MODEL == kSphere ? static_cast<long long>(py) * kp.S : 0) + s];
    const float w = det_exp(sp - fabsf(r - center) / kp.color_den);
    const float4 d = ray_at<MODEL>(kp, px + i, py + j);
    return make_float4(d.x, d.y, d.z, w);
}

// one sample's terms of SPHERE's patch sums (sum w, sum w r, sum w r r), in the sums' order
__device__ __forceinline__ void patch_fold_sample(float w, float r, Patch& pt) {
    pt.sbw += w;
    pt.sref = fmaf(w, r, pt.sref);
    pt.srr = fmaf(w * r, r, pt.srr);
}

// SPHERE's hypothesis- and view-independent weight sums of an unstaged patch (the staged layouts
// form them in coop_patch_nb / coop_patch_sep, in the same order).
template <int MODEL>
__device__ __forceinline__ void patch_sums(const KParams& kp, Patch& pt, int px, int py) {
    pt.sbw = 0.f; pt.sref = 0.f; pt.srr = 0.f;
    if (MODEL == kSphere) {
        for (int s = 0; s < kp.S; ++s) {
            float r;
            const float w = patch_sample<MODEL>(kp, px, py, s, -kp.R + (s / kp.nside) * kp.inc,
                                                -kp.R + (s % kp.nside) * kp.inc, pt.center, r).w;
            patch_fold_sample(w, r, pt);
        }
    }
}

// Unstaged patch of one lane's pixel: samples are recomputed inside the NCC loop (init / debug
// kernels, which evaluate one or two hypotheses per pixel).
template <int MODEL>
__device__ __forceinline__ Patch make_patch(const KParams& kp, int px, int py) {
    const DevCam& rc = kp.cams[0];
    Patch pt;
    pt.rw = nullptr; pt.rr = nullptr; pt.wr = nullptr; pt.row = pt.col = nullptr; pt.stride = 0;
    pt.center = texel_padded(rc.img_base, rc.img_pitch, rc.W, rc.H, px, py);
    patch_sums<MODEL>(kp, pt, px, py);
    return pt;
}

// STAGED: 0 = samples recomputed here, 3 = the k_eval_nb layout of coop_patch_nb, 4 = the separable
// SPHERE layout of coop_patch_sep.  PIPE: every view's texels of a sample in flight before the first
// is used (~6 VGPRs per view); otherwise each view's sample is consumed as soon as it arrives
// (pipelined fetch groups of 2 and 4 views measured neutral to -2%, r01_v29).  PIPE callers keep the
// reference camera in registers across the loop (read per sample through the constant address space
// instead: -3%, r01_v27).

// The NCC of one view from its weighted sums (ACMMP.cu:500-516): sbw = sum w, srrr = (sum w r, sum w r r),
// ssrs = (sum w s, sum w r s), sss = sum w s s
__device__ __forceinline__ float ncc_cost(float sbw, f32x2 srrr, f32x2 ssrs, float sss) {
    // sbw and the reference sums through an opaque copy: their reciprocal, mean and variance are the same for
    // every view and hypothesis, and hoisted to the prologue they were kept (and spilled) across the view loop
    asm volatile("" : "+v"(sbw), "+v"(srrr));
    float out = 2.0f;
    if (!(sbw < 1e-6f)) {
        const float inv = 1.0f / sbw;
        const float m_ref = srrr.x * inv, m_src = ssrs.x * inv;
        const float e_rr = srrr.y * inv, e_ss = sss * inv, e_rs = ssrs.y * inv;
        const float var_ref = fmaf(-m_ref, m_ref, e_rr);
        const float var_src = fmaf(-m_src, m_src, e_ss);
        if (!(var_ref < 1e-5f || var_src < 1e-5f)) {
            const float covar = fmaf(-m_ref, m_src, e_rs);
            const float ncc = 1.0f - covar / sqrtf(var_ref * var_src);
            out = fmaxf(0.0f, fminf(2.0f, ncc));
        }
    }
    return out;
}

// The interpolated loop's fallback (k_nb_fix): a SPHERE view's sums with every one of the 36 samples
// projected in the fast arithmetic, in patch order (ACMMP.cu:456-498) -- the per-sample fast loop's values
// and order, so its bits.  sphere_sample_texel: one sample's source texel; sphere_fold_sample: its terms.
template <int TEX, typename Cam>
__device__ __forceinline__ float sphere_sample_texel(Cam& c, float4 ph, __amdgpu_buffer_rsrc_t rs, float4 rw) {
    const float dep = depth_from_plane_fast(ph, rw);
    float x, y;
    project_fast<kSphere>(c, cam_point_fast<kSphere>(c, 0, 0, dep, rw), x, y);
    x = fmaf(-floorf(x * c.invW), c.Wf, x);
    y = __builtin_amdgcn_fmed3f(y, 0.0f, c.Hm1f);
    return lerp_tap<TEX>(fetch_tap<TEX, true>(rs, c, x, y));
}

__device__ __forceinline__ void sphere_fold_sample(float w, float r, float sp, f32x2& ssrs, float& sss) {
    const f32x2 wwr = (f32x2){w, w * r};
    ssrs = pk_fma(wwr, splat2(sp), ssrs);
    const float ws = w * sp;
    sss = fmaf(ws, sp, sss);
}

// Where the interpolation's nodes spread too far (below) the (pixel, hypothesis, view) must take the per-sample
// arithmetic instead; the chunk hands those entries on, and interpolates only when it has somewhere to hand
// them:
//  * fixkey = the wave's first colour-grid pixel (k_eval_nb's 8-lanes-per-pixel layout: lane l of the wave takes
//    pixel fixkey + l / 8 and hypothesis l % 8): the entry (pixel << 8 | hypothesis << 5 | view) is queued for
//    k_nb_fix, which recomputes it after the launch.  The key is formed at the queue from the lane id, so
//    nothing per lane stays live across the view loop for it (a per-lane key spilled at the 7-wave budget);
//  * kFixNan: the refinement's k_eval_ref (V > 4) gets those costs as NaN (an NCC cost is never NaN: the
//    clamp of ACMMP.cu:513 maps a NaN ratio to 2.0) and leaves them to k_eval_ref_tail (inline fallbacks there
//    cost C3 6.6 ms per half-sweep: random candidates, profiles/r04_prof_ab.txt).  (A bitmask handed back
//    through a pointer instead took k_eval_ref from 120 to 256 VGPRs.)
// With kFixNone every sample is projected.
constexpr uint32_t kFixNone = ~0u, kFixNan = ~0u - 1u;

// The lane's index in its wave, read where it is used: an asm volatile statement is neither hoisted nor merged
// with another read, so a value derived from it is not kept live from the prologue (k_eval_nb spilled its lane
// id, output pointer and queue key at the 7-wave budget: 4 of its 5 spilled dwords).
__device__ __forceinline__ int lane_id_here() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
template <int MODEL, int VB, int STAGED, bool PIPE, int TEX, int FM = 0, bool FULL = false, bool NB = false>
__device__ __forceinline__ void ncc_chunk(const KParams& kp, int px, int py, const Patch& pt, float4 ph,
                                          const int (&vlist)[VB], int nv_rt, float (&cost)[VB],
                                          uint32_t fixkey = kFixNone) {
    // FULL: every view of the chunk present (compile-time); otherwise a wave-uniform count, kept in an
    // SGPR so the per-view guards are scalar branches (without it they were lane masks round-tripped
    // through a VGPR: two VALU per view-sample)
    const int nv = FULL ? VB : uniform_int(nv_rt);
    // per-view guard inside the sample loop: `v < nv` hoisted out of the loop is an i1 live across it,
    // which the backend keeps as a lane mask and re-tests through a VGPR (v_cndmask + v_cmp per
    // view-sample); re-reading nv into an SGPR at the use keeps the test a scalar compare.  Applied to
    // fast-mode SPHERE k_eval_nb-layout chunks: k_eval_nb -1.5..-2% there,
    // while the pinhole refinement (+2.7%), k_select (+3%) and the exact-mode k_eval_nb (+0.7%) lose
    // (r02 A/B profiles/r02_nv_guard_ab.txt)
    constexpr bool kScalarGuard = MODEL == kSphere && STAGED == 3 && FM;
    auto has = [&](int v) -> bool {
        if (FULL) return true;
        if constexpr (kScalarGuard) {
            int n;
            asm volatile("s_mov_b32 %0, %1" : "=s"(n) : "s"(nv));
            return v < n;
        }
        return v < nv;
    };
    // SPHERE: the weight sum of every view is the pixel's patch sum (hypothesis- and view-independent);
    // below 1e-6 each cost is 2.0 (ACMMP.cu:501-503) whatever the samples, so they are not evaluated.
    // (The SPHERE sigma-in-radians band of SURVEY.md §0.5 puts ~40% of a 2000x1500 view here.)
    if (MODEL == kSphere && pt.sbw < 1e-6f) {
#pragma unroll
        for (int v = 0; v < VB; ++v) cost[v] = 2.0f;
        return;
    }
    const DevCam& rc = kp.cams[0];
    // (sum w s, sum w r s) and pinhole's (sum w r, sum w r r) per view as packed pairs: one v_pk_fma_f32
    // per view-sample for each pair (the same fma per sum as separate registers, so the same bits)
    float sbw[VB], sss[VB];
    f32x2 ssrs[VB], srrr[VB];
    bool cval[VB];
    int cv[VB];
#pragma unroll
    for (int v = 0; v < VB; ++v) cv[v] = uniform_int(v < nv ? vlist[v] : vlist[0]);
    // camera table is read-only for the whole launch: view it through the constant address space so
    // every field becomes a scalar (SMEM) load of a wave-uniform address
    typedef const __attribute__((address_space(4))) DevCam ConstCam;
    ConstCam* ccams = (ConstCam*)(kp.cams);
#define PCV(v) ccams[cv[v]]
    const float4 dc = ray_at<MODEL>(kp, px, py);
    const float3 Pc3 = FM ? cam_point_fast<MODEL>(rc, px, py, depth_from_plane_fast(ph, dc), dc)
                          : world_point_ray<MODEL>(rc, px, py, depth_from_plane(ph, dc), dc);
#pragma unroll
    for (int v = 0; v < VB; ++v) {
        sbw[v] = pt.sbw;
        srrr[v] = (f32x2){pt.sref, pt.srr};
        sss[v] = 0.f;
        ssrs[v] = splat2(0.f);
        cval[v] = true;
        if (MODEL == kPinhole && v < nv) {
            float ox, oy, od;
            if (FM) project_fast<MODEL>(PCV(v), Pc3, ox, oy);
            else project<MODEL>(PCV(v), Pc3, ox, oy, od);
            cval[v] = !(ox < 0.0f || ox >= PCV(v).Wf || oy < 0.0f || oy >= PCV(v).Hf);
        }
    }
    // fast-mode SPHERE k_eval_nb chunks hold each view's Ft in VGPRs across the loop (a VOP3 fma reads
    // one SGPR, so a translation in SGPRs costs a move per view-sample): k_eval_nb -1.3..-1.7%, metric +1%
    // (profiles/r02_ft_vgpr_ab.txt)
    constexpr bool kFtV = FM && MODEL == kSphere && STAGED == 3 && !(TEX == 1);
    float ftv[VB][3];
#pragma unroll
    for (int v = 0; v < VB; ++v) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            ftv[v][k] = 0.f;
            if (kFtV) asm volatile("v_mov_b32 %0, %1" : "=v"(ftv[v][k]) : "s"(PCV(v).Ft[k]));
        }
    }
    const int R = kp.R, inc = kp.inc;
    constexpr int G = PIPE ? VB : 1;
    // accumulate view v's sample (ACMMP.cu:488-498): texel tap T of a sample with weight W_,
    // (w, w r) = WWR_ and reference texel R_
// Pinhole: a sample outside the source image (ok false) adds nothing (ACMMP.cu:470-473); instead of a
// branch per view-sample its weight and texel are selected to zero -- fma(0, 0, s) and s + 0 return s
// for the non-negative sums, so the same bits as skipping it
#define ACMMP_ACCUMULATE_T(v, T, W_, WWR_, R_, OK_)                          \
    do {                                                             \
        const float sp = lerp_tap<TEX>(T);                           \
        if (MODEL == kPinhole) {                                     \
            const bool ok_ = (OK_);                                  \
            const f32x2 wwr_ = ok_ ? (WWR_) : splat2(0.f);           \
            const float sp_ = ok_ ? sp : 0.f;                        \
            sbw[v] += wwr_.x;                                        \
            srrr[v] = pk_fma(wwr_, splat2(R_), srrr[v]);             \
            ssrs[v] = pk_fma(wwr_, splat2(sp_), ssrs[v]);            \
            const float ws = wwr_.x * sp_;                           \
            sss[v] = fmaf(ws, sp_, sss[v]);                          \
        } else if (has(v)) {                                         \
            ssrs[v] = pk_fma(WWR_, splat2(sp), ssrs[v]);             \
            const float ws = (W_) * sp;                              \
            sss[v] = fmaf(ws, sp, sss[v]);                           \
        }                                                            \
    } while (0)
#define ACMMP_ACCUMULATE(v) ACMMP_ACCUMULATE_T(v, tap[v], w, wwr, r, ok[v])
    // Fast SPHERE k_eval_nb chunks with 6x6 samples: per view, the source coordinates come from 16 exact
    // projections at the samples of patch columns / rows {0, 2, 3, 5} and, for the others, the 4-point
    // Lagrange interpolation through them (columns 1 and 4 from the node columns, then rows 1 and 4 from
    // the node rows): 16 projections instead of 36 per hypothesis and view.  x is interpolated as the
    // offset from the first node (unwrapped across the seam; small numbers, little rounding) and wrapped
    // per sample as usual.  In float64 the interpolated NCC is within 4.5e-5 of the projected one for
    // every query tried at the metric (near-surface and random planes, profiles/r03_interp_feasibility.json),
    // far inside the binary32 noise floor of DESIGN.md §2.4; the fast-mode gates of
    // tests/test_gpu_fastmath.py hold unchanged (k_eval_nb 1.75 -> 1.51 ms, profiles/r03_interp_ab.txt).
    // Views are the outer loop here, and a view's patch columns are taken 0, 2, 3, 5, 1, 4.
    constexpr bool kInterp = FM && MODEL == kSphere && STAGED == 3 && TEX == 1;
    int interp_done = 0;                            // (an int: a bool phi became a 0/1 VGPR)
    uint32_t rough_nan = 0u;                        // kFixNan: views whose cost becomes NaN
    if constexpr (kInterp) {
        // two uniform branches: the condition as one i1 was kept as a 0/1 VGPR across the view loop (spilled)
        if (kp.interp) if (fixkey != kFixNone) {
            interp_done = 1;
            // Lagrange weights of patch column / row 1 and 4 on the node columns / rows 0, 2, 3, 5
            constexpr float kL1[4] = {0.26666667f, 1.3333334f, -0.6666667f, 0.06666667f};
            constexpr float kL4[4] = {0.06666667f, -0.6666667f, 1.3333334f, 0.26666667f};
            constexpr int kNode[4] = {0, 2, 3, 5};
            const float spread_max = kp.spread_max;     // source pixels spanned by the corner nodes (see below)
            uint32_t rough = 0u;                        // views whose nodes spread too far (below)
            // A node's source direction through the plane's homography (round 6): the node's point in the
            // reference frame is d r with d = -w / (n . r), so its source-frame point is
            //     t = d FR r + Ft = d (FR - Ft n^T / w) r = d M r,
            // and longitude / latitude are invariant under the positive scale d: the node projects as M r --
            // one 3x3 product per node and view (M formed once per view) instead of the ray-plane depth, the
            // point and the rigid map (k_eval_nb's node part 22 -> 9 VALU slots per node-view).  That holds
            // where every node's depth is positive and not at the fast depth's |n . r| < 1e-6 clamp (1e6):
            // a hypothesis with a node outside it (a plane through the reference centre, or one so near
            // grazing that its depth changes sign inside the patch -- whose nodes spread past spread_max in
            // the per-sample arithmetic anyway) sends all its views to the per-sample fallback.  Checked once
            // per hypothesis over the 16 node rays: depth > 0 <=> sign(w) (n . r) < 0.
            {
                const float sg = copysignf(1.0f, ph.w);
                const float nx = ph.x * sg, ny = ph.y * sg, nz = ph.z * sg;
                float emax = -3.0f;
#pragma unroll
                for (int a = 0; a < 4; ++a) {
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const float4 q = pt.rw[(kNode[a] * 6 + kNode[b]) * pt.stride];
                        emax = fmaxf(emax, dot3(nx, ny, nz, q.x, pt.rr[kNode[b] * pt.stride], q.y));
                    }
                }
                if (!(emax <= -1e-6f) || ph.w == 0.0f) rough = 0xffffffffu;
            }
            const float kw = -__builtin_amdgcn_rcpf(ph.w);   // -1 / w
#pragma unroll
            for (int v = 0; v < VB; ++v) {
                if (!has(v)) continue;
                ConstCam& c = PCV(v);
                const __amdgpu_buffer_rsrc_t rs =
                    __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(c.img16_base), 0, c.img16_bytes, 0x00020000);
                // M = FR - Ft n^T / w, rows 0 and 1 interleaved per column as FRxy is
                f32x2 Mxy[3];
                float Mz[3];
                {
                    // scalar fmas: packed ones with splat operands had the splats hoisted out of the view loop as
                    // register pairs and spilled
                    const float fkx = c.Ft[0] * kw, fky = c.Ft[1] * kw, fkz = c.Ft[2] * kw;
                    const float n3[3] = {ph.x, ph.y, ph.z};
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        Mxy[k] = (f32x2){fmaf(fkx, n3[k], c.FRxy[2 * k]), fmaf(fky, n3[k], c.FRxy[2 * k + 1])};
                        Mz[k] = fmaf(fkz, n3[k], c.FRz[k]);
                    }
                }
                float x00 = 0.f;                            // the first node's x (set below)
                // one patch column's six samples from its four row nodes (x, y): the bilinear tap and the
                // sums of ACMMP.cu:488-498
                // (x, y) of a sample as one packed pair: the interpolation's x and y share their Lagrange
                // weights, so each term is one v_pk_fma_f32 (the same fma order per coordinate as the
                // scalar chains, so the same bits)
#ifndef ACMMP_COL_GROUP
#define ACMMP_COL_GROUP 6
#endif
                // the samples in groups of ACMMP_COL_GROUP: the group's texel loads issued before any of its
                // sums (one sample at a time, the interpolated columns' loads were each waited for before the
                // next issued); the sums still run in sample order, so the same bits.  Round 6: the whole column
                // (6 loads in flight; 92 -> 96 VGPRs, 2 spilled) against round 5's pairs: k_eval_nb 1.414 -> 1.396 ms,
                // metric +0.5%, C3 +0.4%; groups of 3 lost 1.3% (profiles/r06_ab15_colgroup_ab.txt)
                auto column = [&](int ci, const f32x2 (&nd)[4]) {
                    asm volatile("" ::: "memory");
                    // (k_eval_nb's instances only, NB: k_eval_ref's interpolating instance measured 1.3% slower)
                    constexpr int G = NB ? ACMMP_COL_GROUP : 1;
#pragma unroll
                    for (int c0 = 0; c0 < 6; c0 += G) {
                        Tap tg[G];
                        float wg[G], rg[G];
#pragma unroll
                        for (int k = 0; k < G; ++k) {
                            const int cj = c0 + k;
                            f32x2 xy;
                            if (cj == 0 || cj == 2 || cj == 3 || cj == 5) {
                                xy = nd[cj == 0 ? 0 : (cj == 2 ? 1 : (cj == 3 ? 2 : 3))];
                            } else {
                                const float* L = cj == 1 ? kL1 : kL4;
                                xy = pk_fma(splat2(L[3]), nd[3], pk_fma(splat2(L[2]), nd[2],
                                            pk_fma(splat2(L[1]), nd[1], splat2(L[0]) * nd[0])));
                            }
                            float x = xy.x, y = xy.y;
                            const float4 q = pt.rw[(ci * 6 + cj) * pt.stride];
                            wg[k] = q.z;
                            rg[k] = q.w;
                            x += x00;
                            x = fmaf(-floorf(x * c.invW), c.Wf, x);
                            y = __builtin_amdgcn_fmed3f(y, 0.0f, c.Hm1f);
                            tg[k] = fetch_tap<TEX, true>(rs, c, x, y);
                        }
#pragma unroll
                        for (int k = 0; k < G; ++k) {
                            const float w = wg[k];
                            const f32x2 wwr = (f32x2){w, w * rg[k]};
                            // unguarded: the view loop skips absent views (`has` re-read per sample kept the
                            // sums behind a scalar select, 3 v_cndmask per view-sample)
                            const float sp = lerp_tap<TEX>(tg[k]);
                            ssrs[v] = pk_fma(wwr, splat2(sp), ssrs[v]);
                            const float ws = w * sp;
                            sss[v] = fmaf(ws, sp, sss[v]);
                        }
                    }
                };
                // Node column by node column (patch columns 0, 2, 3, 5): its 4 nodes projected, its samples taken,
                // its share of the interpolated columns 1 and 4 at the node rows accumulated -- so one node column
                // (8 VGPRs) and the two interpolated columns (16) are live instead of all 16 nodes (32; the whole
                // view's nodes first spilled at the 7-wave budget once the view loop's other values grew).  x is
                // the offset from the first node, unwrapped across the seam: small numbers, so the interpolation's
                // rounding stays far below the positions' own.  The same values in the same sample order as
                // projecting all nodes first (round 3's form), so the same bits.
                f32x2 c1[4], c4[4];
#pragma unroll
                for (int b = 0; b < 4; ++b) c1[b] = c4[b] = splat2(0.f);
                // The interpolation holds where the source mapping is smooth over the patch.  Where the four
                // corner nodes spread over more than kp.spread_max (256) source pixels in x or y -- a patch
                // landing next to a source pole (longitude stretches as 1 / cos(latitude)) or a near-grazing
                // plane whose depth flips sign inside the patch -- the (pixel, hypothesis, view) goes to
                // k_nb_fix, which projects all 36 samples in the per-sample loop's order and arithmetic (so
                // those costs are the per-sample fast ones bit for bit).  float64 study (tests/np_interp.py,
                // tests/test_interp_design.py): with the test, the interpolated NCC stays within 1e-4 of the
                // projected one on every query tried from 2000x1000 up (capi.cpp's size gate), pole-adjacent
                // and random planes included; without it the tail reached 0.6.  Corner terms of node column 0
                // are kept until column 3's (x03, and the y pair's max / min in the same grouping).
                float x03 = 0.f, y0max = 0.f, y0min = 0.f;
                bool smooth = true;
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    f32x2 nd[4];                            // (x - x00 unwrapped, y) per node of this column
                    // node b of this column at source (x, y): x as the offset from the first node, unwrapped
                    auto put_node = [&](int b, float x, float y) {
                        if (a == 0 && b == 0) {
                            x00 = x;
                            nd[b].x = 0.0f;
                        } else {
                            const float dx = x - x00;
                            nd[b].x = fmaf(-rintf(dx * c.invW), c.Wf, dx);
                        }
                        nd[b].y = y;
                    };
                    // two nodes at a time: their atan polynomials interleave (a lone chain of dependent v_pk_fma_f32
                    // waits a hazard cycle between steps: 929 s_nop in k_eval_nb<11,4,1,1>, 348 paired; the same
                    // bits, scripts/ab_bitident.py)
#pragma unroll
                    for (int b = 0; b < 4; b += 2) {
                        f32x2 hxy[2];
                        float hz[2];
#pragma unroll
                        for (int k = 0; k < 2; ++k) {
                            const float4 q = pt.rw[(kNode[a] * 6 + kNode[b + k]) * pt.stride];
                            const float rwy = pt.rr[kNode[b + k] * pt.stride];
                            hxy[k] = pk_fma(Mxy[2], splat2(q.y), pk_fma(Mxy[1], splat2(rwy), Mxy[0] * splat2(q.x)));
                            hz[k] = fmaf(Mz[2], q.y, fmaf(Mz[1], rwy, Mz[0] * q.x));
                        }
                        float x0, y0, x1, y1;
                        sphere_pixel_fast_x2(c, hxy[0], hz[0], hxy[1], hz[1], x0, y0, x1, y1);
                        put_node(b, x0, y0);
                        put_node(b + 1, x1, y1);
                    }
                    if (a == 0) {
                        x03 = nd[3].x;
                        y0max = fmaxf(nd[0].y, nd[3].y);
                        y0min = fminf(nd[0].y, nd[3].y);
                    }
                    if (a == 3) {
                        const float sx_ = fmaxf(fmaxf(x03, nd[0].x), fmaxf(nd[3].x, 0.0f)) -
                                          fminf(fminf(x03, nd[0].x), fminf(nd[3].x, 0.0f));
                        const float sy_ = fmaxf(y0max, fmaxf(nd[0].y, nd[3].y)) - fminf(y0min, fminf(nd[0].y, nd[3].y));
                        smooth = fmaxf(sx_, sy_) <= spread_max;
                    }
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        c1[b] = pk_fma(splat2(kL1[a]), nd[b], c1[b]);
                        c4[b] = pk_fma(splat2(kL4[a]), nd[b], c4[b]);
                    }
                    // the samples re-read (w, r) from LDS rather than keep the nodes' reads live across the
                    // projections (merged, they spilled 210 VGPRs)
                    column(kNode[a], nd);
                    __builtin_amdgcn_sched_barrier(0);       // one node column live at a time
                }
                column(1, c1);
                column(4, c4);
                rough |= smooth ? 0u : (1u << v);
                __builtin_amdgcn_sched_barrier(0);           // one view's nodes live at a time
            }
            // Lanes whose corners spread too far go to k_nb_fix's queue (fixkey set: k_eval_nb and its test
            // hook), which recomputes those (pixel, hypothesis, view) costs with every sample projected --
            // the per-sample fast arithmetic bit for bit -- after the launch.  Done here, one such lane made its
            // whole wave run the 36 projections (3-6% of lanes, so most waves: k_eval_nb +28%).  After the
            // view loop (inside it the queue's code spilled, both before and after the node-column form).
            // The queue holds every entry a launch can produce (capi.cpp sizes it per k_eval_nb launch, and
            // launch_eval_nb runs k_nb_fix after each), so none is dropped; k_nb_fix flags an overflow, which
            // fails the run.  k_eval_ref (kFixNan) gets those costs as NaN instead.
            if (fixkey == kFixNan) {
                rough_nan = rough;
            } else {
#pragma unroll
                for (int v = 0; v < VB; ++v) {
                    if (!has(v)) continue;
                    const bool redo = (rough >> v) & 1u;
                    const unsigned long long b = __ballot(redo);
                    if (b) {
                        const int lane = lane_id_here();
                        const int leader = __ffsll(static_cast<long long>(b)) - 1;
                        unsigned base = 0u;
                        // one of kNbFixRegions counters per block (a single one serialised the atomics:
                        // k_eval_nb +0.35 ms at the metric)
                        const unsigned region = blockIdx.x % kNbFixRegions;
                        if (lane == leader) base = atomicAdd(kp.nbfix_count + region, static_cast<unsigned>(__popcll(b)));
                        base = __builtin_amdgcn_readlane(base, leader);      // (__shfl needs a lane id of its own)
                        const unsigned slot = base + static_cast<unsigned>(__popcll(b & ((1ull << lane) - 1ull)));
                        const uint32_t key = ((fixkey + static_cast<uint32_t>(lane >> 3)) << 8) |
                                             (static_cast<uint32_t>(lane & 7) << 5) | static_cast<uint32_t>(cv[v] - 1);
                        if (redo && slot < kp.nbfix_cap) kp.nbfix[static_cast<long long>(region) * kp.nbfix_cap + slot] = key;
                    }
                }
            }
        }
    }
    // Fast pinhole chunks of the staged layouts: the source point of sample (i, j) as one homogeneous
    // vector per view.  The reference's point is depth_s * v_s with v_s = ((x+i - cx) / fx, (y+j - cy) / fy, 1)
    // (Get3DPointonWorld_cu's pinhole branch, ACMMP.cu:579-581) and depth_s = -w / D_s, D_s = n . r_s for the
    // normalised table ray r_s (ACMMP.cu:187-193); its source image point FR (depth_s v_s) + Ft, scaled by
    // w / depth_s (a projective scale: the same x / z and y / z), is
    //     h(i, j) = w FR v_s + S_s Ft,   S_s = -D_s (w 1e-6 where |D_s| < 1e-6: the reference's depth 1e6),
    // and w FR v_s = w FR v_0 + i w FR e_x / fx + j w FR e_y / fy is affine in (i, j).  It is taken relative
    // to the pixel's own source point (X0, Y0) = h_c.xy / h_c.z, h_c = h(0, 0) formed in binary64 from the
    // binary32 inputs: x(i, j) = X0 + N_x / h_z with N_x = h_x - X0 h_z affine in (i, j) and S_s - S_c, all its
    // terms small -- so the per-sample arithmetic rounds at the scale of the patch's pixel offsets, not of
    // the image coordinates.  Per view-sample 6 VALU for the point (project_fast: 8 plus 2 moves of Ft, plus
    // the depth division and the point per sample) and no FR in scalar registers across the loop; in
    // binary32 emulation (C5 / C2 cameras, near-surface planes) the coordinates are ~2x closer to float64
    // than the per-sample form's (q99 8e-5 vs 1.7e-4 px).
// fast pinhole sample loop: two samples' loads in flight (ACMMP_PIN_PAIRS: k_eval_nb's, _REF: k_eval_ref's instances)
#ifndef ACMMP_PIN_PAIRS
#define ACMMP_PIN_PAIRS 1
#endif
#ifndef ACMMP_PIN_PAIRS_REF
#define ACMMP_PIN_PAIRS_REF 1
#endif
    constexpr bool kHomog = FM && MODEL == kPinhole && STAGED == 3;
    if constexpr (kHomog) if (kp.homog) {
        interp_done = 1;
        ConstCam& c0 = ccams[0];
        const float v0x = (static_cast<float>(px) - c0.K[2]) * c0.inv_fx;
        const float v0y = (static_cast<float>(py) - c0.K[5]) * c0.inv_fy;
        const float w_clamp = ph.w * 1e-6f;
        const float D0 = dot3(ph.x, ph.y, ph.z, dc.x, dc.y, dc.z);
        const float s0 = fabsf(D0) < 1e-6f ? w_clamp : -D0;
        // per view: N = (N0 + i hi' + j hj' + dS Ft') relative to (X0, Y0), z = hz + i hi.z + j hj.z + dS Ft.z
        f32x2 n0[VB], hi2[VB], hj2[VB], ft2[VB], xy0[VB];
        float z0[VB], hiz[VB], hjz[VB];
#pragma unroll
        for (int v = 0; v < VB; ++v) {
            n0[v] = hi2[v] = hj2[v] = ft2[v] = xy0[v] = splat2(0.f);
            z0[v] = hiz[v] = hjz[v] = 0.f;
            if (has(v)) {
                ConstCam& c = PCV(v);
                double hc[3];
                float hi[3], hj[3];
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const float f0 = r < 2 ? c.FRxy[r] : c.FRz[0];        // FR[r][0]
                    const float f1 = r < 2 ? c.FRxy[2 + r] : c.FRz[1];    // FR[r][1]
                    const float f2 = r < 2 ? c.FRxy[4 + r] : c.FRz[2];    // FR[r][2]
                    const double g = fma(static_cast<double>(f1), static_cast<double>(v0y),
                                         fma(static_cast<double>(f0), static_cast<double>(v0x), static_cast<double>(f2)));
                    hc[r] = fma(static_cast<double>(s0), static_cast<double>(c.Ft[r]), static_cast<double>(ph.w) * g);
                    hi[r] = ph.w * (f0 * c0.inv_fx);
                    hj[r] = ph.w * (f1 * c0.inv_fy);
                }
                const float hz = static_cast<float>(hc[2]);
                const float rz = __builtin_amdgcn_rcpf(hz);
                const float X0 = static_cast<float>(hc[0]) * rz, Y0 = static_cast<float>(hc[1]) * rz;
                xy0[v] = (f32x2){X0, Y0};
                n0[v] = (f32x2){static_cast<float>(fma(-static_cast<double>(X0), hc[2], hc[0])),
                                static_cast<float>(fma(-static_cast<double>(Y0), hc[2], hc[1]))};
                hi2[v] = (f32x2){fmaf(-X0, hi[2], hi[0]), fmaf(-Y0, hi[2], hi[1])};
                hj2[v] = (f32x2){fmaf(-X0, hj[2], hj[0]), fmaf(-Y0, hj[2], hj[1])};
                ft2[v] = (f32x2){fmaf(-X0, c.Ft[2], c.Ft[0]), fmaf(-Y0, c.Ft[2], c.Ft[1])};
                z0[v] = hz;
                hiz[v] = hi[2];
                hjz[v] = hj[2];
            }
        }
        // each view's image descriptor and bounds formed once, before the loop (built at their use, the
        // compiler re-read their fields through scalar loads per sample)
        __amdgpu_buffer_rsrc_t rsv[VB];
        int wm1[VB], hm1[VB], p4[VB];
        float ftz[VB];
#pragma unroll
        for (int v = 0; v < VB; ++v) {
            ConstCam& c = PCV(v);
            rsv[v] = TEX == 1
                ? __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(c.img16_base), 0, c.img16_bytes, 0x00020000)
                : __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(c.img_base), 0, c.img_bytes, 0x00020000);
            wm1[v] = uniform_int(c.Wm1);
            hm1[v] = uniform_int(c.Hm1);
            p4[v] = uniform_int(c.pitch4);
            ftz[v] = c.Ft[2];
        }
        int s = 0;
        for (int i = -R; i <= R; i += inc) {
            const float fi = static_cast<float>(i);
            f32x2 nr[VB];
            float zr[VB];
#pragma unroll
            for (int v = 0; v < VB; ++v) {
                nr[v] = pk_fma(splat2(fi), hi2[v], n0[v]);
                zr[v] = fmaf(fi, hiz[v], z0[v]);
            }
            // one sample's source points and texel loads (its sums after)
            auto issue = [&](int jv, int sv, Tap (&tp)[VB], bool (&okv)[VB], float& w_o, float& r_o, f32x2& wwr_o) {
                const float fj = static_cast<float>(jv);
                const float4 q = pt.rw[sv * pt.stride];     // (r_s, w_s)
                r_o = pt.rr[sv * pt.stride];
                const float D = dot3(ph.x, ph.y, ph.z, q.x, q.y, q.z);
                const float dS = (fabsf(D) < 1e-6f ? w_clamp : -D) - s0;
                w_o = q.w;
                wwr_o = (f32x2){w_o, w_o * r_o};
#pragma unroll
                for (int v = 0; v < VB; ++v) {
                    okv[v] = false;
                    if (has(v)) {
                        f32x2 nn = pk_fma(splat2(fj), hj2[v], nr[v]);
                        float tz = fmaf(fj, hjz[v], zr[v]);
                        nn = pk_fma(splat2(dS), ft2[v], nn);
                        tz = fmaf(dS, ftz[v], tz);
                        const f32x2 o = pk_fma(nn, splat2(__builtin_amdgcn_rcpf(tz)), xy0[v]);
                        const int ix = cvt_flr_i32(o.x), iy = cvt_flr_i32(o.y);
                        okv[v] = (static_cast<unsigned>(ix) <= static_cast<unsigned>(wm1[v])) &
                                 (static_cast<unsigned>(iy) <= static_cast<unsigned>(hm1[v]));   // pin_in_image
                        tp[v] = fetch_tap_pin_p<TEX>(rsv[v], p4[v], o.x, o.y, ix, iy);
                    }
                }
            };
            int j = -R;
            if constexpr (NB ? ACMMP_PIN_PAIRS : ACMMP_PIN_PAIRS_REF) {
                // k_eval_nb: two samples' loads in flight before either's sums (the sums in sample order, so the
                // same bits).  Round 6, at the 5-wave budget (96 VGPRs, 2 spilled; 44 spilled at 6 waves): C2 k_eval_nb
                // 3.05 -> 2.93 ms, C2 +2.3%, 1920x1080 V=20 +1.8% (profiles/r06_ab17_pinpairs_ab.txt); in k_eval_ref's
                // fast pinhole chunks (100 -> 117 VGPRs, 5 -> 4 waves) C2 k_eval_ref 1.78 -> 1.71 ms, C2 +1.6% more
                // (profiles/r06_ab18_pinpairs_ref_ab.txt)
                for (; j + inc <= R; j += 2 * inc, s += 2) {
                    Tap ta[VB], tb[VB];
                    bool oka[VB], okb[VB];
                    float wa, ra, wb, rb;
                    f32x2 wwra, wwrb;
                    issue(j, s, ta, oka, wa, ra, wwra);
                    issue(j + inc, s + 1, tb, okb, wb, rb, wwrb);
#pragma unroll
                    for (int v = 0; v < VB; ++v)
                        if (has(v)) ACMMP_ACCUMULATE_T(v, ta[v], wa, wwra, ra, oka[v]);
#pragma unroll
                    for (int v = 0; v < VB; ++v)
                        if (has(v)) ACMMP_ACCUMULATE_T(v, tb[v], wb, wwrb, rb, okb[v]);
                }
            }
            for (; j <= R; j += inc, ++s) {
                Tap tap[VB];
                bool ok[VB];
                float w, r;
                f32x2 wwr;
                issue(j, s, tap, ok, w, r, wwr);
#pragma unroll
                for (int v = 0; v < VB; ++v)
                    if (has(v)) ACMMP_ACCUMULATE(v);
            }
        }
    }
    if (!interp_done) {
        int s = 0, ii = 0;
        for (int i = -R; i <= R; i += inc, ++ii) {
            int jj = 0;                                      // s % nside without a division per sample
            const float2 cs = STAGED == 4 ? pt.col[ii] : make_float2(0.f, 0.f);
            for (int j = -R; j <= R; j += inc, ++s, ++jj) {
                float r;
                float4 rw;
                if (STAGED == 4) {                           // coop_patch_sep layout (SPHERE): ray_at's products
                    const float2 rs = pt.row[jj];
                    const float2 q = pt.wr[s];
                    rw = make_float4(rs.y * cs.x, -rs.x, rs.y * cs.y, q.x);
                    r = q.y;
                } else if (STAGED == 3) {                    // coop_patch_nb layout
                    const float4 q = pt.rw[s * pt.stride];
                    if (MODEL == kSphere) {
                        rw = make_float4(q.x, pt.rr[jj * pt.stride], q.y, q.z);
                        r = q.w;
                    } else {
                        rw = q;
                        r = pt.rr[s * pt.stride];
                    }
                } else {
                    rw = patch_sample<MODEL>(kp, px, py, s, i, j, pt.center, r);
                }
                const float w = rw.w;
                // reference camera through the constant address space too: scalar loads per sample
                // instead of 12 wave-uniform VGPRs held across the loop
                float3 P;
                const float dep = FM ? depth_from_plane_fast(ph, rw) : depth_from_plane(ph, rw);
                if (FM)
                    P = cam_point_fast<MODEL>(ccams[0], px + i, py + j, dep, rw);
                else if (!PIPE)
                    P = world_point_ray<MODEL>(ccams[0], px + i, py + j, dep, rw);
                else
                    P = world_point_ray<MODEL>(rc, px + i, py + j, dep, rw);
                const float wr = w * r;
                const f32x2 wwr = (f32x2){w, wr};
                Tap tap[VB];
                bool ok[VB];
#pragma unroll
                for (int v = 0; v < VB; ++v) {
                    ok[v] = false;
                    if (has(v)) {
                        ConstCam& c = PCV(v);
                        float sx, sy, sd;
                        if (FM) project_fast<MODEL>(c, P, sx, sy, kFtV ? ftv[v] : nullptr);
                        else project<MODEL>(c, P, sx, sy, sd);
                        ok[v] = true;
                        const __amdgpu_buffer_rsrc_t rs = TEX == 1
                            ? __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(c.img16_base), 0, c.img16_bytes, 0x00020000)
                            : __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(c.img_base), 0, c.img_bytes, 0x00020000);
                        if (MODEL == kSphere) {
                            sx = fmaf(-floorf(sx * c.invW), c.Wf, sx);
                            sy = FM ? __builtin_amdgcn_fmed3f(sy, 0.0f, c.Hm1f) : clamp0(sy, c.Hm1f);
                            tap[v] = fetch_tap<TEX, true>(rs, c, sx, sy);
                        } else {
                            const int ix = cvt_flr_i32(sx), iy = cvt_flr_i32(sy);
                            ok[v] = pin_in_image(c, ix, iy);
                            tap[v] = fetch_tap_pin<TEX>(rs, c, sx, sy, ix, iy);
                        }
                        if (G == 1) ACMMP_ACCUMULATE(v);
                    }
                    // a full SPHERE chunk has no per-view branches; keep its views' code in view order
                    // (interleaved, their live ranges overlap and the 7-wave register budget spills)
                    if (FULL && MODEL == kSphere) __builtin_amdgcn_sched_barrier(0);
                    // G > 1: views are consumed in groups of G, a group's texels all in flight before the
                    // first is used (PIPE: the whole chunk; ~6 VGPRs per view in flight)
                    if (G > 1 && ((v + 1) % G == 0 || v == VB - 1)) {
#pragma unroll
                        for (int u = v - (v % G); u <= v; ++u)
                            if (has(u)) ACMMP_ACCUMULATE(u);
                    }
                }
            }
        }
    }
#undef ACMMP_ACCUMULATE
#undef ACMMP_ACCUMULATE_T
#pragma unroll
    for (int v = 0; v < VB; ++v) {
        cost[v] = cval[v] ? ncc_cost(sbw[v], srrr[v], ssrs[v], sss[v]) : 2.0f;
        if (kInterp && ((rough_nan >> v) & 1u)) cost[v] = __builtin_nanf("");
    }
#undef PCV
}

// ComputeGeomConsistencyCost, ACMMP.cu:646-671 (sv = source camera index 1..N-1)
template <int MODEL>
__device__ __forceinline__ float geom_cost(const KParams& kp, int sv, float4 ph, int px, int py, float4 dc) {
    const DevCam& rc = kp.cams[0];
    const DevCam& sc = kp.cams[sv];
    const float depth = depth_from_plane(ph, dc);
    const float3 fwd = world_point_ray<MODEL>(rc, px, py, depth, dc);
    float sx, sy, sd;
    project<MODEL>(sc, fwd, sx, sy, sd);
    const float src_depth = texel_plain(kp.dep + sc.dep_off, sc.dep_w, sc.dep_h, f2i_sat(sx), f2i_sat(sy));
    if (src_depth == 0.0f) return 3.0f;
    const float3 s3 = world_point<MODEL>(sc, sx, sy, src_depth);
    float bx, by, bd;
    project<MODEL>(rc, s3, bx, by, bd);
    const float dcol = static_cast<float>(px) - bx, drow = static_cast<float>(py) - by;
    return fminf(3.0f, sqrtf(fmaf(drow, drow, dcol * dcol)));
}

// Views that at least one ACTIVE lane of the wave needs (mask = per-lane bitmask of views 0..V-1).
// Ballots only see active lanes, so lanes that already returned cannot drop bits (a shuffle
// butterfly would route partial results through inactive lanes).
__device__ __forceinline__ uint32_t wave_or(uint32_t mask, int V) {
    uint32_t r = 0u;
    for (int v = 0; v < V; ++v)
        if (__ballot((mask >> v) & 1u)) r |= 1u << v;
    return uniform_int(static_cast<int>(r));
}

// ------------------------------------------------------------------ random hypotheses

// SampleDepthInv, ACMMP.cu:14-22
__device__ __forceinline__ float sample_depth_inv(Rng& rs, float dmin, float dmax) {
    dmin = fmaxf(dmin, 1e-6f);
    dmax = fmaxf(dmax, dmin + 1e-6f);
    const float inv_min = 1.0f / dmax;
    const float inv_max = 1.0f / dmin;
    const float u = rs.uniform();
    const float inv = fmaf(u, inv_max - inv_min, inv_min);
    return 1.0f / inv;
}

// GenerateRandomNormal, ACMMP.cu:194-220 (view ray supplied)
__device__ __forceinline__ float4 random_normal(float4 v, Rng& rs) {
    float q1 = 1.0f, q2 = 1.0f, s = 2.0f;
    while (s >= 1.0f) {
        q1 = fmaf(2.0f, rs.uniform(), -1.0f);
        q2 = fmaf(2.0f, rs.uniform(), -1.0f);
        s = fmaf(q2, q2, q1 * q1);
    }
    const float sq = sqrtf(1.0f - s);
    float4 n = make_float4((2.0f * q1) * sq, (2.0f * q2) * sq, fmaf(-2.0f, s, 1.0f), 0.0f);
    if (dot3n(n, v) > 0.0f) { n.x = -n.x; n.y = -n.y; n.z = -n.z; }
    normalize3(n.x, n.y, n.z);
    return n;
}

// GeneratePerturbedNormal, ACMMP.cu:222-257
__device__ __forceinline__ float4 perturbed_normal(float4 v, float4 n, Rng& rs, float perturbation) {
    const float a1 = (rs.uniform() - 0.5f) * perturbation;
    const float a2 = (rs.uniform() - 0.5f) * perturbation;
    const float a3 = (rs.uniform() - 0.5f) * perturbation;
    float s1, c1, s2, c2, s3, c3;
    det_sincos(a1, &s1, &c1);
    det_sincos(a2, &s2, &c2);
    det_sincos(a3, &s3, &c3);
    const float R0 = c2 * c3;
    const float R1 = fmaf(-c1, s3, (c3 * s1) * s2);
    const float R2 = fmaf(c1 * c3, s2, s1 * s3);
    const float R3 = c2 * s3;
    const float R4 = fmaf(s1 * s2, s3, c1 * c3);
    const float R5 = fmaf(-c3, s1, (c1 * s2) * s3);
    const float R6 = -s2;
    const float R7 = c2 * s1;
    const float R8 = c1 * c2;
    float4 p = make_float4(dot3(R0, R1, R2, n.x, n.y, n.z), dot3(R3, R4, R5, n.x, n.y, n.z),
                           dot3(R6, R7, R8, n.x, n.y, n.z), n.w);
    if (dot3n(p, v) >= 0.0f) p = n;
    normalize3(p.x, p.y, p.z);
    return p;
}

// ------------------------------------------------------------------ cost-vector helpers

// Evaluate all source views of plane `ph` and hand each cost to f(view0, cost) in view order.
template <int MODEL, int VB, int STAGED, bool PIPE, int TEX, int FM, bool NOFULL = false, typename F>
__device__ __forceinline__ void for_all_views_t(const KParams& kp, int px, int py, const Patch& pt, float4 ph,
                                                uint32_t wave_mask, F&& f, uint32_t fixkey = kFixNone) {
    int v = 0;
    const int V = kp.V;
    while (true) {
        int vlist[VB];
        int nv = 0;
        // next VB views present in wave_mask (wave-uniform)
#pragma unroll
        for (int k = 0; k < VB; ++k) vlist[k] = 1;
        while (v < V && nv < VB) {
            if ((wave_mask >> v) & 1u) {
#pragma unroll
                for (int k = 0; k < VB; ++k)
                    if (k == nv) vlist[k] = v + 1;
                ++nv;
            }
            ++v;
        }
        if (nv == 0) break;
        float cost[VB];
        // (NOFULL: not in k_eval_nb's interpolating instances, whose views are a loop anyway -- the second copy
        // of the chunk took the 2-view one, V = 2, to 371 spilled dwords at its 6-wave budget)
        constexpr bool kFullCopy = (MODEL == kSphere ? VB <= 2 : true) && VB > 1 &&
                                   !(NOFULL && MODEL == kSphere && STAGED == 3 && FM && TEX == 1);
        if (kFullCopy && nv == VB)
            ncc_chunk<MODEL, VB, STAGED, PIPE, TEX, FM, true, NOFULL>(kp, px, py, pt, ph, vlist, nv, cost, fixkey);
        else
            ncc_chunk<MODEL, VB, STAGED, PIPE, TEX, FM, false, NOFULL>(kp, px, py, pt, ph, vlist, nv, cost, fixkey);
#pragma unroll
        for (int k = 0; k < VB; ++k)
            if (k < nv) f(vlist[k] - 1, cost[k]);
        if (v >= V) break;
    }
}

// The same over the binary16 images when the context has them, with the fast-math projection when
// the context asks for it (launch-uniform branches).
template <int MODEL, int VB, int STAGED, bool PIPE, bool PIPE_FM = PIPE, typename F>
__device__ __forceinline__ void for_all_views(const KParams& kp, int px, int py, const Patch& pt, float4 ph,
                                              uint32_t wave_mask, F&& f) {
    if (kp.fast) {
        if (kp.tex16) for_all_views_t<MODEL, VB, STAGED, PIPE_FM, 1, 1>(kp, px, py, pt, ph, wave_mask, f);
        else for_all_views_t<MODEL, VB, STAGED, PIPE_FM, 0, 1>(kp, px, py, pt, ph, wave_mask, f);
    } else {
        if (kp.tex16) for_all_views_t<MODEL, VB, STAGED, PIPE, 1, 0>(kp, px, py, pt, ph, wave_mask, f);
        else for_all_views_t<MODEL, VB, STAGED, PIPE, 0, 0>(kp, px, py, pt, ph, wave_mask, f);
    }
}

// TF: the texel format and math mode as one compile-time choice, so each kernel instance gets its own
// register allocation (k_eval_nb's r02 A/B: a run-time branch between them sized every path for the
// largest).  0 = fp32 texels, math mode at run time (images that are not binary16-exact); 1 = binary16
// texels, exact; 2 = binary16 texels, fast math.
template <int MODEL, int VB, int STAGED, bool PIPE, int TF, bool PIPE_FM = PIPE, typename F>
__device__ __forceinline__ void for_all_views_tf(const KParams& kp, int px, int py, const Patch& pt, float4 ph,
                                                 uint32_t wave_mask, F&& f, uint32_t fixkey = kFixNone) {
    if constexpr (TF == 0) {
        if (kp.fast) for_all_views_t<MODEL, VB, STAGED, PIPE_FM, 0, 1>(kp, px, py, pt, ph, wave_mask, f);
        else for_all_views_t<MODEL, VB, STAGED, PIPE, 0, 0>(kp, px, py, pt, ph, wave_mask, f);
    } else {
        for_all_views_t<MODEL, VB, STAGED, TF == 2 ? PIPE_FM : PIPE, 1, TF == 2 ? 1 : 0>(kp, px, py, pt, ph, wave_mask, f,
                                                                                       fixkey);
    }
}
static inline int tf_of(const KParams& kp) { return kp.tex16 ? (kp.fast ? 2 : 1) : 0; }

__device__ __forceinline__ float vw_get(const uint32_t (&vwp)[4], int v) {
    const uint32_t word = v < 8 ? vwp[0] : (v < 16 ? vwp[1] : (v < 24 ? vwp[2] : vwp[3]));
    return static_cast<float>((word >> ((v & 7) * 4)) & 15u);
}

// XCD-aware block order (k_init).  Blocks are dealt round-robin over the 8 XCDs (b and b + 8 share
// one L2, MI355X_MICROARCH.md "Workgroup dispatch"); launch order gives every XCD every 8th tile of
// the same rows, so each L2 caches the source-image footprint of all rows in flight.  Instead XCD
// (b % 8) walks strips x, x + 8, x + 16, ... of kXcdStrip consecutive logical blocks: its
// resident blocks cover 1/8 of the rows in flight, and the strips interleave finely enough that every
// XCD gets the same mix of short-circuited and evaluated rows.  The grid is padded to whole strips
// per XCD (xcd_grid); surplus blocks find no pixel.  Measured (r01_v23): k_init -10% at 3200x1600
// V=15 and -16% at 1600x1200 pinhole V=10, neutral at the metric; the same order made k_eval_nb /
// k_eval_ref 2-9% SLOWER (their lanes of one pixel already share a footprint; r01_v23,
// r02_eval_xcd_strip_ab.txt), so they keep launch order.
constexpr unsigned kXcdStrip = 256;
__device__ __forceinline__ long long xcd_block(unsigned b) {
    const unsigned x = b & 7u, k = b >> 3;
    const unsigned j = k / kXcdStrip, r = k - j * kXcdStrip;
    return (static_cast<long long>(j) * 8 + x) * kXcdStrip + r;
}

static inline unsigned xcd_grid(long long nblocks) {
    const long long strips = (nblocks + kXcdStrip - 1) / kXcdStrip;
    return static_cast<unsigned>((strips + 7) / 8 * 8 * kXcdStrip);
}

// ------------------------------------------------------------------ kernels: setup

#if ACMMP_IN_TU(0)
// Row-pair binary16 layout of one padded view: word (X, Y) = (h(I[Y][X]), h(I[Y+1][X])) for Y in [0, H].
__global__ void k_to_f16_pairs(const float* __restrict__ src, int W2, int rows, uint32_t* __restrict__ dst,
                               int* __restrict__ inexact) {
    const long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= static_cast<long long>(W2) * rows) return;
    uint32_t out = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const float x = src[i + k * W2];
        const _Float16 h = static_cast<_Float16>(x);
        if (!(static_cast<float>(h) == x) || (x != 0.0f && !(fabsf(x) >= 6.103515625e-05f)) || fabsf(x) > 65504.0f)
            atomicOr(inexact, 1);
        out |= static_cast<uint32_t>(__builtin_bit_cast(uint16_t, h)) << (16 * k);
    }
    dst[i] = out;
}

__global__ void k_pad_image(const float* __restrict__ src, size_t pitch, int W, int H, float* __restrict__ dst,
                            int dpitch) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x - 1;
    const int y = blockIdx.y * blockDim.y + threadIdx.y - 1;
    if (x > W || y > H) return;
    dst[static_cast<long long>(y + 1) * dpitch + (x + 1)] =
        src[static_cast<long long>(clampi(y, 0, H - 1)) * pitch + clampi(x, 0, W - 1)];
}

// PixelToDir tables of the reference camera (ACMMP.cu:119-134), evaluated once per view.
__global__ void k_ray_tables(const KParams kp, float4* __restrict__ dirs, float2* __restrict__ sph_row,
                             float2* __restrict__ sph_col) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y * blockDim.y + threadIdx.y;
    const int TW = kp.W + 2 * kp.R, TH = kp.H + 2 * kp.R;
    const DevCam& c = kp.cams[0];
    if (kp.model == kSphere) {
        if (y == 0 && x < TW) {
            const float lon = (static_cast<float>(x - kp.R) - c.cx) / static_cast<float>(c.W) * 2.0f * kCudartPiF;
            float sl, cl;
            det_sincos(lon, &sl, &cl);
            sph_col[x] = make_float2(sl, cl);
        }
        if (y == 1 && x < TH) {
            const float lat = -(static_cast<float>(x - kp.R) - c.cy) / static_cast<float>(c.H) * kCudartPiF;
            float sa, ca;
            det_sincos(lat, &sa, &ca);
            sph_row[x] = make_float2(sa, ca);
        }
        return;
    }
    if (x >= TW || y >= TH) return;
    const float3 d = pixel_to_dir(c, x - kp.R, y - kp.R);
    dirs[static_cast<long long>(y) * kp.dpitch + x] = make_float4(d.x, d.y, d.z, 0.0f);
}

// Spatial half of ComputeBilateralWeight (ACMMP.cu:398-403, 436-486): -|d| / (2 sigma_s^2) per
// sample, per row for SPHERE (angular distances depend on the latitude).
__global__ void k_spatial(const KParams kp, float* __restrict__ spatial) {
    const int y = blockIdx.x * blockDim.x + threadIdx.x;
    const int rows = kp.model == kSphere ? kp.H : 1;
    if (y >= rows) return;
    const DevCam& rc = kp.cams[0];
    float scale_x = 1.0f, scale_y = 1.0f, sig = kp.sigma_spatial;
    if (kp.model == kSphere) {
        const float lat_c = -(static_cast<float>(y) - rc.cy) / static_cast<float>(rc.H) * kCudartPiF;
        scale_x = (2.0f * kCudartPiF / static_cast<float>(rc.W)) * det_cos(lat_c);
        scale_y = (kCudartPiF / static_cast<float>(rc.H));
        sig = kp.sigma_spatial * (kCudartPiF / static_cast<float>(rc.H));
    }
    int s = 0;
    for (int i = -kp.R; i <= kp.R; i += kp.inc) {
        for (int j = -kp.R; j <= kp.R; j += kp.inc, ++s) {
            const float dx = kp.model == kSphere ? static_cast<float>(i) * scale_x : static_cast<float>(i);
            const float dy = kp.model == kSphere ? static_cast<float>(j) * scale_y : static_cast<float>(j);
            const float sd = sqrtf(fmaf(dy, dy, dx * dx));
            spatial[static_cast<long long>(y) * kp.S + s] = (-sd) / (2.0f * sig * sig);
        }
    }
}

#endif  // ACMMP_IN_TU(0)

// ------------------------------------------------------------------ initial cost

__device__ __forceinline__ void sort_small(float* d, int n) {
    int j;
    for (int i = 1; i < n; i++) {
        const float tmp = d[i];
        for (j = i; j >= 1 && tmp < d[j - 1]; j--) d[j] = d[j - 1];
        d[j] = tmp;
    }
}

// ComputeMultiViewInitialCostandSelectedViews, ACMMP.cu:519-556
template <int MODEL, int VB, int VMAXB, int TF>
__device__ float initial_cost(const KParams& kp, int px, int py, const Patch& pt, float4 ph, uint32_t* sel,
                              float* cvec = nullptr) {
    constexpr int VMAX = VMAXB < 8 ? VMAXB : kMaxViews;      // pick_vb: V <= VMAXB when VMAXB < 8
    float cv[VMAX], cvc[VMAX];
    int nvalid = 0;
    const uint32_t all = kp.V >= 32 ? 0xFFFFFFFFu : ((1u << kp.V) - 1u);
    for_all_views_tf<MODEL, VB, 0, true, TF>(kp, px, py, pt, ph, all, [&](int v, float c) {
        cv[v] = c;
        cvc[v] = c;
        if (c < 2.0f) nvalid++;
    });
    if (cvec)                                                   // current-plane cost cache
        for (int v = 0; v < kp.V; ++v) cvec[v * kp.Pc] = cvc[v];
    sort_small(cv, kp.V);
    *sel = 0;
    const int top_k = nvalid < kp.top_k ? nvalid : kp.top_k;
    if (top_k > 0) {
        float cost = 0.0f;
        for (int i = 0; i < top_k; ++i) cost += cv[i];
        const float thr = cv[top_k - 1];
        for (int i = 0; i < kp.V; ++i)
            if (cvc[i] <= thr) *sel |= (1u << i);
        return cost / static_cast<float>(top_k);
    }
    return 2.0f;
}

// SpatialGauss / RangeGauss, ACMMP.cu:175-185 (float exponent)
__device__ __forceinline__ float spatial_gauss(float x1, float y1, float x2, float y2, float sigma) {
    const float dx = x1 - x2, dy = y1 - y2;
    const float dis = (dx * dx + dy * dy) - 0.0f;
    return det_exp(-dis / (2.0f * sigma * sigma));
}
__device__ __forceinline__ float range_gauss(float x, float sigma) {
    const float xp = x - 0.0f;
    return det_exp(-(xp * xp) / (2.0f * sigma * sigma));
}

// ------------------------------------------------------------------ kernel: RandomInitialization

// ACMMP.cu:673-795.  Reads the persistent row-major state, writes the colour-split working state.
// RandomInitialization branch, uniform over a launch (ACMMP.cu:686-793): one kernel per branch so
// the common random branch does not carry the JBU loop's registers.
enum InitBranch { kInitRandom = 0, kInitPlanar = 1, kInitUpsample = 2, kInitReuse = 3 };

// k_init evaluates its (unstaged) NCCs four views at a time: each chunk recomputes the samples' weights
// and rays, and with the fast-math projection the wider chunk wins (r02 A/B profiles/r02_init_vb_ab.txt:
// 2 -> 4 views: 0.95 -> 0.92 ms at the metric, 2.46 -> 2.15 ms at C2, 8.27 -> 6.97 ms at C3; round 1,
// exact mode only: 1 view 1.55, 2 views 1.36, 4 views 1.41 ms at the metric).
[[maybe_unused]] constexpr int kInitVB = 4;

template <int MODEL, int VB, int BR, int VMAXB, int TF>
__global__ __launch_bounds__(256) void k_init(const KParams kp) {
    // 16x16 tiles in XCD-aware order (xcd_block) over a row-major grid of ceil(W/16) tiles per row
    const long long tile = xcd_block(blockIdx.x);
    const int tiles_x = (kp.W + 15) >> 4;
    const int x = static_cast<int>(tile % tiles_x) * 16 + threadIdx.x;
    const int y = kp.init_lo + static_cast<int>(tile / tiles_x) * 16 + threadIdx.y;
    if (x >= kp.W || y >= kp.init_hi) return;
    const DevCam& rc = kp.cams[0];
    const long long center = static_cast<long long>(y) * kp.W + x;
    const int colour = (x + y) & 1;
    const long long ci = cs_index(kp, x, y);
    const Patch pt = make_patch<MODEL>(kp, x, y);
    float* cvec = kp.cvec[colour] + ci;
    Rng rs;
    rs.init(kp.seed_lo, kp.seed_hi, static_cast<uint32_t>(center), 0u);
    const float4 dc = ray_at<MODEL>(kp, x, y);
    float4 ph;
    float cost;
    uint32_t sel = 0;
    if (BR == kInitRandom) {
        const float depth = fmaf(rs.uniform(), kp.depth_max - kp.depth_min, kp.depth_min);
        ph = random_normal(dc, rs);
        ph.w = dist_to_origin(dc, depth, ph);
        cost = initial_cost<MODEL, VB, VMAXB, TF>(kp, x, y, pt, ph, &sel, cvec);
    } else if (BR == kInitPlanar) {
        if (kp.mask[center] > 0 && kp.costs_rm[center] >= 0.1f) {
            const float perturbation = 0.02f;
            const float4 prior = kp.prior[center];
            float dp = prior.w;
            const float dmin_p = (1 - 3 * perturbation) * dp;
            const float dmax_p = (1 + 3 * perturbation) * dp;
            dp = fmaf(rs.uniform(), dmax_p - dmin_p, dmin_p);
            ph = perturbed_normal(dc, prior, rs, static_cast<float>(3 * perturbation * kMPi));
            ph.w = dp;
        } else {
            ph = kp.planes_rm[center];
            const float depth = ph.w;
            ph.w = dist_to_origin(dc, depth, ph);
        }
        cost = initial_cost<MODEL, VB, VMAXB, TF>(kp, x, y, pt, ph, &sel, cvec);
    } else if (BR == kInitUpsample) {
        const float scale = static_cast<float>(1.0 * static_cast<double>(kp.scaled_cols) / static_cast<double>(kp.W));
        const float sigmad = 0.50f, sigmar = 25.5f;
        const int Imagescale = f2i_sat(fmaxf(static_cast<float>(kp.W) / kp.scaled_cols,
                                             static_cast<float>(kp.H) / kp.scaled_rows));
        const int nn = (Imagescale * Imagescale + 1) / 2;
        const float o_y = static_cast<float>(y) * scale, o_x = static_cast<float>(x) * scale;
        const float* ref = rc.img_base;
        const float refPix = texel_padded(ref, rc.img_pitch, rc.W, rc.H, x, y);
        float nf = 0.0f;
        float nx = 0.f, ny = 0.f, nz = 0.f;
        for (int j = -nn; j <= nn; ++j) {
            int r_y = f2i_sat(o_y + static_cast<float>(j));
            r_y = (r_y > 0 ? (static_cast<float>(r_y) < kp.scaled_rows ? r_y : f2i_sat(kp.scaled_rows - 1)) : 0);
            const int r_ys = y + j;
            for (int i = -nn; i <= nn; ++i) {
                int r_x = f2i_sat(o_x + static_cast<float>(i));
                r_x = (r_x > 0 ? (static_cast<float>(r_x) < kp.scaled_cols ? r_x : f2i_sat(kp.scaled_cols - 1)) : 0);
                const int s_center = f2i_sat(static_cast<float>(r_y) * kp.scaled_cols + static_cast<float>(r_x));
                const float4 sn = kp.scaled[s_center];
                const float nbPix = texel_padded(ref, rc.img_pitch, rc.W, rc.H, x + i, r_ys);
                const float tg = spatial_gauss(o_x, o_y, static_cast<float>(r_x), static_cast<float>(r_y), sigmad) *
                                 range_gauss(fabsf(refPix - nbPix), sigmar);
                nf += tg;
                nx = nx + sn.x * tg;
                ny = ny + sn.y * tg;
                nz = nz + sn.z * tg;
            }
        }
        nx = nx / nf; ny = ny / nf; nz = nz / nf;
        normalize3(nx, ny, nz);
        const float4 cur = kp.planes_rm[center];
        uint32_t sel0;
        kp.pre_rm[center] = initial_cost<MODEL, VB, VMAXB, TF>(kp, x, y, pt, cur, &sel0);
        ph = to_ref(rc, make_float4(nx, ny, nz, 0.0f));
        ph.w = dist_to_origin(dc, cur.w, ph);
        cost = initial_cost<MODEL, VB, VMAXB, TF>(kp, x, y, pt, ph, &sel, cvec);
    } else {
        ph = kp.hier ? kp.scaled[center] : kp.planes_rm[center];
        ph = to_ref(rc, ph);
        const float depth = ph.w;
        ph.w = dist_to_origin(dc, depth, ph);
        cost = initial_cost<MODEL, VB, VMAXB, TF>(kp, x, y, pt, ph, &sel, cvec);
    }
    kp.plane_cs[colour][ci] = ph;
    kp.cost_cs[colour][ci] = cost;
    kp.sel_cs[colour][ci] = sel;
    kp.rng_cs[colour][ci] = rs.n;
}

// ------------------------------------------------------------------ kernels: CheckerboardPropagation
//
// One half-sweep of CheckerboardPropagation (ACMMP.cu:938-1325, launched by Black/RedPixelUpdate
// :1327-1349) runs as four launches over the pixels of one colour:
//   k_eval_nb   one lane per (pixel, hypothesis): adaptive neighbour pick of direction h (h < 8)
//               or the pixel's own plane (h == 8), then its cost vector over all source views
//   k_select    one lane per pixel: joint view selection, aggregated costs, acceptance, and the
//               five refinement candidates of PlaneHypothesisRefinement (all RNG draws, in order)
//   k_eval_ref  one lane per (pixel, candidate): aggregated cost of each valid candidate
//   k_finish    one lane per pixel: refinement acceptance in candidate order, hierarchy gate, store
// Intermediate per-pixel state goes through the scratch slab (engine.h).  Same-colour reads see the
// kernel-entry snapshot: neighbour planes/costs come from the colour's current buffer, the result
// goes to its other buffer.

// (the colour's buffer chosen by a select between the two kernel-argument pointers: indexed by the lane's parity,
// the pointer itself was loaded from the argument block first -- a second dependent round trip per access)
__device__ __forceinline__ float cost_at(const KParams& kp, int x, int y) {
    const float* b = ((x + y) & 1) ? kp.cost_cs[1] : kp.cost_cs[0];
    return b[cs_index(kp, x, y)];
}
__device__ __forceinline__ float4 plane_at(const KParams& kp, int pos) {
    const int x = pos & 0xFFFF, y = pos >> 16;
    const float4* b = ((x + y) & 1) ? kp.plane_cs[1] : kp.plane_cs[0];
    return b[cs_index(kp, x, y)];
}
__device__ __forceinline__ int packpos(int x, int y) { return x | (y << 16); }

// Adaptive checkerboard sampling of one direction (ACMMP.cu:965-1143); returns the packed position
// or -1 when the direction is unavailable (flag[d] == false).
__device__ __forceinline__ int pick_neighbour(const KParams& kp, int d, int px, int py) {
    // Branch-free: every candidate's cost is loaded (an out-of-image one from the first candidate's position, not
    // taken) and the strict-< scan in the reference's order runs on selects -- behind the bounds branches each
    // load was waited for before the next issued (k_pick: 7-11 serial round trips per pixel)
    const int width = kp.W, height = kp.H;
    float cmin;
    int cpos;
    auto take = [&](bool ok, int x, int y) {
        const float c = cost_at(kp, x, y);
        const bool better = ok && c < cmin;
        cmin = better ? c : cmin;
        cpos = better ? packpos(x, y) : cpos;
    };
    switch (d) {
    case 1:                                                   // up_far
        if (!(py > 2)) return -1;
        cmin = cost_at(kp, px, py - 3); cpos = packpos(px, py - 3);
#pragma unroll
        for (int i = 1; i < 11; ++i) {
            const bool ok = py > 2 + 2 * i;
            take(ok, px, ok ? py - 3 - 2 * i : py - 3);
        }
        return cpos;
    case 3:                                                   // down_far
        if (!(py < height - 3)) return -1;
        cmin = cost_at(kp, px, py + 3); cpos = packpos(px, py + 3);
#pragma unroll
        for (int i = 1; i < 11; ++i) {
            const bool ok = py < height - 3 - 2 * i;
            take(ok, px, ok ? py + 3 + 2 * i : py + 3);
        }
        return cpos;
    case 5:                                                   // left_far
        if (!(px > 2)) return -1;
        cmin = cost_at(kp, px - 3, py); cpos = packpos(px - 3, py);
#pragma unroll
        for (int i = 1; i < 11; ++i) {
            const bool ok = px > 2 + 2 * i;
            take(ok, ok ? px - 3 - 2 * i : px - 3, py);
        }
        return cpos;
    case 7:                                                   // right_far
        if (!(px < width - 3)) return -1;
        cmin = cost_at(kp, px + 3, py); cpos = packpos(px + 3, py);
#pragma unroll
        for (int i = 1; i < 11; ++i) {
            const bool ok = px < width - 3 - 2 * i;
            take(ok, ok ? px + 3 + 2 * i : px + 3, py);
        }
        return cpos;
    case 0:                                                   // up_near (V shape, same colour)
        if (!(py > 0)) return -1;
        cmin = cost_at(kp, px, py - 1); cpos = packpos(px, py - 1);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const bool a = py > 1 + i && px > i, b = py > 1 + i && px < width - 1 - i;
            take(a, a ? px - i : px, a ? py - 2 - i : py - 1);
            take(b, b ? px + i : px, b ? py - 2 - i : py - 1);
        }
        return cpos;
    case 2:                                                   // down_near
        if (!(py < height - 1)) return -1;
        cmin = cost_at(kp, px, py + 1); cpos = packpos(px, py + 1);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const bool a = py < height - 2 - i && px > i, b = py < height - 2 - i && px < width - 1 - i;
            take(a, a ? px - i : px, a ? py + 2 + i : py + 1);
            take(b, b ? px + i : px, b ? py + 2 + i : py + 1);
        }
        return cpos;
    case 4:                                                   // left_near
        if (!(px > 0)) return -1;
        cmin = cost_at(kp, px - 1, py); cpos = packpos(px - 1, py);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const bool a = px > 1 + i && py > i, b = px > 1 + i && py < height - 1 - i;
            take(a, a ? px - 2 - i : px - 1, a ? py - i : py);
            take(b, b ? px - 2 - i : px - 1, b ? py + i : py);
        }
        return cpos;
    default:                                                  // 6: right_near
        if (!(px < width - 1)) return -1;
        cmin = cost_at(kp, px + 1, py); cpos = packpos(px + 1, py);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const bool a = px < width - 2 - i && py > i, b = px < width - 2 - i && py < height - 1 - i;
            take(a, a ? px + 2 + i : px + 1, a ? py - i : py);
            take(b, b ? px + 2 + i : px + 1, b ? py + i : py);
        }
        return cpos;
    }
}

// Pixel q of the colour grid (row-major over rows x Wh); false when it does not exist.
__device__ __forceinline__ bool colour_pixel(const KParams& kp, int colour, long long q, int& px, int& py) {
    const int r = static_cast<int>(q / kp.Wh);
    const int k = static_cast<int>(q - static_cast<long long>(r) * kp.Wh);
    py = kp.row_lo + r;
    px = 2 * k + ((py + colour) & 1);
    return py < kp.row_hi && px < kp.W;
}

// k_eval_nb staging, 16 B per sample + 4 B per patch row: SPHERE stores (ray.x, ray.z, w, texel)
// per sample and ray.y = -sin(lat) once per patch row (it depends on the row only); PINHOLE stores
// (ray, w) per sample and the texels after them.  32 pixels x 36 samples = 19.2 KB per block for
// SPHERE (8 blocks per CU).
// views per NCC chunk in the evaluation kernels (more views than this run as several chunks:
// the per-sample world point is recomputed per chunk, the accumulators stay in registers)
constexpr int kEvalVB = 4;
// k_eval_nb keeps every view's texels of a sample in flight (PIPE) in fast-math mode only, whose shorter
// projection leaves the registers for it (r02 A/B: k_eval_nb 2.19 -> 2.06 ms; the exact mode -4%)
constexpr bool kNbPipeExact = false, kNbPipeFast = true;
// fast pinhole chunks (the homogeneous sample points of ncc_chunk): views per chunk (ACMMP_NB_PIN_VB
// overrides at build time for A/B builds)
#ifndef ACMMP_NB_PIN_VB
#define ACMMP_NB_PIN_VB 2
#endif
template <int MODEL, int VB, int FM>
constexpr int nb_vb() {
    constexpr int cap = (MODEL == kPinhole && FM) ? ACMMP_NB_PIN_VB : kEvalVB;
    return VB > cap ? cap : VB;
}
constexpr int kNbLanes = 8;                 // the 8 neighbour directions (the current plane's costs are cached)

static inline size_t nb_lds_bytes(int model, int S, int nside, int npix = kNbPix) {
    return model == kSphere ? (sizeof(float4) * S + sizeof(float) * nside) * npix
                            : (sizeof(float4) + sizeof(float)) * S * npix;
}

// Sample-major: entry s of pixel slot lp sits at [s * NPIX + lp], so lanes of consecutive pixel slots
// reading one sample read consecutive 16-byte words (no bank conflicts).
template <int MODEL, int NPIX = kNbPix, int NLANES = kNbLanes>
__device__ __forceinline__ Patch coop_patch_nb(const KParams& kp, bool valid, int px, int py, int lp, int h,
                                               float4* lds) {
    float4* rw = lds + lp;
    float* tail = reinterpret_cast<float*>(lds + NPIX * kp.S);
    float* rr = tail + lp;
    if (valid) {
        const DevCam& rc = kp.cams[0];
        const float center = texel_padded(rc.img_base, rc.img_pitch, rc.W, rc.H, px, py);
        for (int s = h; s < kp.S; s += NLANES) {
            const int i = -kp.R + (s / kp.nside) * kp.inc, j = -kp.R + (s % kp.nside) * kp.inc;
            float r;
            const float4 q = patch_sample<MODEL>(kp, px, py, s, i, j, center, r);
            if (MODEL == kSphere) {
                rw[s * NPIX] = make_float4(q.x, q.z, q.w, r);
                if (s < kp.nside) rr[s * NPIX] = q.y;   // samples 0..nside-1 cover every patch row j
            } else {
                rw[s * NPIX] = q;
                rr[s * NPIX] = r;
            }
        }
    }
    __syncthreads();
    Patch pt;
    pt.rw = rw; pt.rr = rr; pt.wr = nullptr; pt.row = pt.col = nullptr; pt.stride = NPIX;
    pt.center = 0.f;
    pt.sbw = 0.f; pt.sref = 0.f; pt.srr = 0.f;
    if (MODEL == kSphere && valid) {
        for (int s = 0; s < kp.S; ++s) {                // patch_sums order (ACMMP.cu:482-486)
            patch_fold_sample(rw[s * NPIX].z, rw[s * NPIX].w, pt);
        }
    }
    return pt;
}

// Separable SPHERE staging (STAGED 4): (w, texel) per sample, (sin, cos) of the latitude per patch row
// and of the longitude per patch column -- a sample's ray is ray_at's two products of them, the same
// bits.  8 S + 16 nside bytes per pixel (384 B at 36 samples, vs 600 B for coop_patch_nb), so
// k_eval_ref's 51-pixel block fits 8 times in a CU's LDS instead of 5.
static inline size_t sep_lds_bytes(int S, int nside, int npix) { return (8 * static_cast<size_t>(S) + 16 * nside) * npix; }

template <int NPIX, int NLANES>
__device__ __forceinline__ Patch coop_patch_sep(const KParams& kp, bool valid, int px, int py, int lp, int h,
                                                float4* lds) {
    float2* base = reinterpret_cast<float2*>(lds);
    float2* wr = base + lp * kp.S;
    float2* row = base + NPIX * kp.S + lp * 2 * kp.nside;
    float2* col = row + kp.nside;
    if (valid) {
        const DevCam& rc = kp.cams[0];
        const float center = texel_padded(rc.img_base, rc.img_pitch, rc.W, rc.H, px, py);
        for (int s = h; s < kp.S; s += NLANES) {
            const int i = -kp.R + (s / kp.nside) * kp.inc, j = -kp.R + (s % kp.nside) * kp.inc;
            float r;
            const float4 q = patch_sample<kSphere>(kp, px, py, s, i, j, center, r);
            wr[s] = make_float2(q.w, r);
        }
        for (int k = h; k < kp.nside; k += NLANES) {
            row[k] = kp.sph_row[py - kp.R + k * kp.inc + kp.R];
            col[k] = kp.sph_col[px - kp.R + k * kp.inc + kp.R];
        }
    }
    __syncthreads();
    Patch pt;
    pt.rw = nullptr; pt.rr = nullptr; pt.wr = wr; pt.row = row; pt.col = col; pt.stride = 1;
    pt.center = 0.f;
    pt.sbw = 0.f; pt.sref = 0.f; pt.srr = 0.f;
    if (valid) {
        for (int s = 0; s < kp.S; ++s) {                // patch_sums order (ACMMP.cu:482-486)
            patch_fold_sample(wr[s].x, wr[s].y, pt);
        }
    }
    return pt;
}

// k_eval_ref / tail: every view's texels of a sample in flight (two-phase fetch); no register budget
// (SPHERE's non-geom instance: 80 VGPRs at 6 waves, no spills).  SPHERE launches with V <= 4 stage the
// patch separably (coop_patch_sep: 8 blocks per CU instead of 5; r02 A/B: metric +0.8%, exact +0.9%,
// V = 15 -0.5%, so not there; (w, texel)-only staging with the rays re-read from the tables measured
// no better, r01_v40).  NCC chunks of 2 views where the launch has 4-view ones (r01_v40 A/B +1.7%),
// and for SPHERE launches with V > 4 too (r02 A/B: V = 15 +1.4%; pinhole V = 10 -4%, so not pinhole).
constexpr bool kRefPipe = true;
template <int MODEL, int VB>
constexpr int ref_vb() { return (VB == 4 || (VB > 4 && MODEL == kSphere)) ? 2 : (VB > kEvalVB ? kEvalVB : VB); }
// k_eval_ref's chunk: the fast pinhole chunks' homogeneous points hold ~12 VGPRs per view across the sample
// loop, so 4-view chunks took 162 VGPRs (3 waves per SIMD) and 2-view ones take 100 (5 waves): C2 k_eval_ref
// 1.90 -> 1.85 ms, +1% (profiles/r04_ab4_ab.txt).  (Capping the SPHERE V > 4 instance at 5 waves instead,
// 120 -> 96 VGPRs, lost 5% of C3's k_eval_ref there.)
template <int MODEL, int VB, int TF>
constexpr int ref_vb_eval() {
    return (MODEL == kPinhole && TF == 2 && ref_vb<MODEL, VB>() > 2) ? 2 : ref_vb<MODEL, VB>();
}
// kRefLanes / kRefPix / kRefSlots: engine.h (capi.cpp sizes the survivor and fallback queues from them)

// Adaptive checkerboard sampling of every pixel of the colour, one direction per grid row: the
// direction is wave-uniform here, where inside k_eval_nb (lane = direction) a wave walks all eight
// of pick_neighbour's cases one after the other (k_eval_nb 2.84 -> 2.60 ms, r01_v38).
#if ACMMP_IN_TU(0)
__global__ __launch_bounds__(256) void k_pick(const KParams kp, const int colour) {
    const long long q = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int d = blockIdx.y;
    // the fallback queue's region counters emptied for k_eval_nb's first view chunk (in place of a memset launch
    // between this kernel and k_eval_nb: 4 us of GPU time per half-sweep)
    static_assert(kNbFixRegions == 256, "one counter per thread of block (0, 0)");
    if (kp.nbfix && blockIdx.x == 0 && d == 0) kp.nbfix_count[threadIdx.x] = 0u;
    int px = 0, py = 0;
    if (!colour_pixel(kp, colour, q, px, py)) return;
    const long long ci = static_cast<long long>(py) * kp.Wh + (px >> 1);
    kp.nbpos[d * kp.Pc + ci] = pick_neighbour(kp, d, px, py);
}

#endif  // ACMMP_IN_TU(0)

// k_eval_nb register budgets (minimum waves per SIMD): SPHERE exact 8, SPHERE fast 6 (below), pinhole fast 6.
// TEX (binary16 texels) and FM (fast math) are compile-time here, so each of the four variants gets its
// own register allocation (a runtime branch between them sized every variant for the largest: 23
// VGPRs spilled at the 64-VGPR budget; r02 A/B profiles/r02_split_nb_ab.txt: fast 388 -> 394, exact
// 316.6 -> 320 Mpixel-iterations/s)
// fast pinhole: 6 waves (80 VGPRs, 5 dwords spilled outside the sample loops) against 5 unconstrained (90):
// C2 k_eval_nb 3.233 -> 3.212 ms (profiles/r04_ab5_ab.txt).  A software-pipelined form of its sample loop (the
// next sample's gathers issued before the current one is accumulated: 96 VGPRs, 5 waves) measured 3.17 -> 3.30 ms
// (round 5, profiles/r05_ab3_ab.txt): not kept.  Round 6: two samples' loads issued before either's sums (the sums
// in order, not a pipeline across iterations) at 5 waves (96 VGPRs, 2 spilled) -- C2 k_eval_nb 3.05 -> 2.93 ms
// (profiles/r06_ab17_pinpairs_ab.txt); at 6 waves the pair spilled 44 dwords.
template <int MODEL, int VB, int TEX, int FM>
#ifndef ACMMP_NB_PIN_WAVES
#define ACMMP_NB_PIN_WAVES 5
#endif
#ifndef ACMMP_NB_SPH_WAVES
// fast SPHERE: 5 waves (92 VGPRs, no spills).  Round 4's form (all 16 nodes of a view live at once) spilled 9 dwords at
// 7 waves and was 3% slower at 6; with the node-column form and no prologue values kept across the view loop
// (ncc_chunk), 6 waves beat 7: k_eval_nb 1.545 -> 1.511 ms at the metric, C3 15.69 -> 15.30 ms
// (profiles/r05_ab3_ab.txt).  Round 6's node pairs (sphere_pixel_fast_x2) hold two nodes' chains at once: 20 dwords
// spilled at 6 waves (metric -1.2% against unpaired nodes), none at 5, where k_eval_nb takes 1.429 against 1.436 ms
// unpaired at 6 (C3 13.62 / 13.78 ms; profiles/r06_ab5_pairs_ab.txt)
#define ACMMP_NB_SPH_WAVES 5
#endif
__global__ __launch_bounds__(256, MODEL == kSphere ? (FM ? ACMMP_NB_SPH_WAVES : 8) : (FM ? ACMMP_NB_PIN_WAVES : 1)) void k_eval_nb(
    const KParams kp, const int colour) {
    extern __shared__ float4 lds4[];
    const int t = threadIdx.x;
    // 8 lanes per pixel, one per neighbour direction (a pixel-major map -- a wave = 32 pixels x 2
    // directions -- measured 3% slower, profiles/r03_eval_nb_ab.txt)
    const int lp = t / kNbLanes, h = t - lp * kNbLanes;
    // the block's 32 pixels: a run of one colour-grid row, or (nb_tile) an 8 x 4 tile, a wave per tile row --
    // either way a wave's 8 pixels are consecutive in the grid (wrow, wcol + 0..7)
    long long wrow = 0, wcol = 0;
    if (kp.nb_tile) {
        const int tpr = (kp.Wh + 7) >> 3;
        const int tr = static_cast<int>(blockIdx.x) / tpr;
        wrow = tr * 4 + (t >> 6);
        wcol = (static_cast<int>(blockIdx.x) - tr * tpr) * 8;
    }
    const long long q = kp.nb_tile ? wrow * kp.Wh + wcol + (lp & 7) : static_cast<long long>(blockIdx.x) * kNbPix + lp;
    int px = 0, py = 0;
    const bool valid = (!kp.nb_tile || wcol + (lp & 7) < kp.Wh) && colour_pixel(kp, colour, q, px, py);
    const Patch pt = coop_patch_nb<MODEL>(kp, valid, px, py, lp, h, lds4);
    // work accounting for the roofline: pixels whose NCCs are evaluated (not short-circuited)
    const int busy = __syncthreads_count(valid && h == 0 && !(MODEL == kSphere && pt.sbw < 1e-6f));
    if (t == 0 && busy && kp.nb_count_work) atomicAdd(kp.work + (blockIdx.x & 255u), static_cast<unsigned long long>(busy));
    if (!valid) return;
    const long long Pc = kp.Pc;
    const long long ci = static_cast<long long>(py) * kp.Wh + (px >> 1);
    const int pos = kp.nbpos[h * Pc + ci];                  // k_pick
    if (pos < 0) return;
    const float4 ph = plane_at(kp, pos);
    const uint32_t all = kp.nb_views;
    // the wave's first pixel ci = row_lo * Wh + q (colour_pixel): lane l holds pixel base + l / 8, hypothesis l % 8.
    // The output address and the fallback key are formed from it and the lane id where they are used.
    const uint32_t wbase = static_cast<uint32_t>(uniform_int(static_cast<int>(
        kp.nb_tile ? (kp.row_lo + wrow) * kp.Wh + wcol : kp.row_lo * kp.Wh + blockIdx.x * kNbPix + (t >> 6) * 8)));
    const uint32_t fixkey = kp.nbfix ? wbase : kFixNone;
    for_all_views_t<MODEL, nb_vb<MODEL, VB, FM>(), 3, FM ? kNbPipeFast : kNbPipeExact, TEX, FM, true>(
        kp, px, py, pt, ph, all, [&](int v, float c) {
            const int l = lane_id_here();
            kp.hyp_cost[(static_cast<long long>(l & 7) * kp.V + v) * Pc + (wbase + (l >> 3))] = c;
        }, fixkey);
}

// The interpolation fallbacks k_eval_nb queued (ncc_chunk): each (pixel, hypothesis, view) cost with every
// sample projected, the patch recomputed (its samples, weights and sums: the same bits as the staged
// ones), over the same hyp_cost entry k_eval_nb wrote; after every k_eval_nb launch of the half-sweep and
// before k_select.  kFixLanes lanes per entry: lane j takes patch row j's samples (reference texel, weight,
// ray, source texel) into LDS, then lane 0 folds the 36 in patch order with patch_fold_sample /
// sphere_fold_sample -- the inline fallback's values in its order, so its bits.  One lane per entry, each
// running 72 dependent sample chains (the patch sums, then the view sums), took 0.10 ms per launch at
// the metric, latency-bound (profiles/r04_ab3_kernel_stats.csv).
constexpr int kFixLanes = 6, kFixPerWave = 64 / kFixLanes, kFixPerBlock = 4 * kFixPerWave;

// Lane j (< kFixLanes) of a fallback entry: patch row j's samples into smp[s] = (w, r, source texel)
template <int TEX>
__device__ __forceinline__ void fix_row(const KParams& kp, int px, int py, float4 ph, int v, int j, float4* smp) {
    typedef const __attribute__((address_space(4))) DevCam ConstCam;
    const DevCam& rc = kp.cams[0];
    const float center = texel_padded(rc.img_base, rc.img_pitch, rc.W, rc.H, px, py);
    ConstCam& c = ((ConstCam*)(kp.cams))[v + 1];
    const __amdgpu_buffer_rsrc_t rs = TEX == 1
        ? __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(c.img16_base), 0, c.img16_bytes, 0x00020000)
        : __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(c.img_base), 0, c.img_bytes, 0x00020000);
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int s = j * 6 + k;
        float r;
        const float4 rw = patch_sample<kSphere>(kp, px, py, s, -kp.R + j * kp.inc, -kp.R + k * kp.inc, center, r);
        smp[s] = make_float4(rw.w, r, sphere_sample_texel<TEX>(c, ph, rs, rw), 0.f);
    }
}

// Lane 0 of a fallback entry: the NCC from the 36 staged samples
__device__ __forceinline__ float fix_fold(const float4* smp) {
    Patch pt;
    pt.sbw = 0.f; pt.sref = 0.f; pt.srr = 0.f;
    f32x2 ssrs = splat2(0.f);
    float sss = 0.f;
#pragma unroll 6
    for (int s = 0; s < 36; ++s) {
        const float4 q = smp[s];
        patch_fold_sample(q.x, q.y, pt);
        sphere_fold_sample(q.x, q.y, q.z, ssrs, sss);
    }
    return ncc_cost(pt.sbw, (f32x2){pt.sref, pt.srr}, ssrs, sss);
}

// block b of the fix grid takes region b % kNbFixRegions, its (b / kNbFixRegions)-th stripe of entries.
// REF: the refinement's entries (k_eval_ref's queue, the same buffer after k_eval_nb's is drained): hypothesis h is
// candidate h (kp.cand), the cost goes to its cost vector (kp.cand_vcost).
template <int TEX, bool REF = false>
__global__ __launch_bounds__(256) void k_nb_fix(const KParams kp, const int colour) {
    __shared__ float4 smp[kFixPerBlock][36];
    const int t = threadIdx.x, l = t & 63;
    const int ew = l / kFixLanes, j = l - ew * kFixLanes, e = (t >> 6) * kFixPerWave + ew;
    const unsigned region = blockIdx.x % kNbFixRegions, stripes = gridDim.x / kNbFixRegions;
    const unsigned n = min(kp.nbfix_count[region], kp.nbfix_cap);
    // sized for every entry a launch can queue (capi.cpp), so this never fires; if it did, the run fails
    if (t == 0 && blockIdx.x < kNbFixRegions && kp.nbfix_count[region] > kp.nbfix_cap) atomicOr(kp.status, kStatusFixOverflow);
    const uint32_t* q = kp.nbfix + static_cast<long long>(region) * kp.nbfix_cap;
    const long long Pc = kp.Pc;
    for (unsigned i0 = (blockIdx.x / kNbFixRegions) * kFixPerBlock; i0 < n; i0 += stripes * kFixPerBlock) {
        const unsigned i = i0 + static_cast<unsigned>(e);
        const bool act = ew < kFixPerWave && i < n;
        long long ci = 0;
        int h = 0, v = 0;
        if (act) {
            const uint32_t key = q[i];
            ci = key >> 8;
            h = static_cast<int>((key >> 5) & 7u);
            v = static_cast<int>(key & 31u);
            const int py = static_cast<int>(ci / kp.Wh);
            const int px = 2 * static_cast<int>(ci - static_cast<long long>(py) * kp.Wh) + ((py + colour) & 1);
            fix_row<TEX>(kp, px, py, REF ? kp.cand[h * Pc + ci] : plane_at(kp, kp.nbpos[h * Pc + ci]), v, j, smp[e]);
        }
        __syncthreads();
        if (act && j == 0) (REF ? kp.cand_vcost : kp.hyp_cost)[(static_cast<long long>(h) * kp.V + v) * Pc + ci] = fix_fold(smp[e]);
        __syncthreads();
    }
}

// Joint view selection, aggregation, acceptance and refinement candidates (ACMMP.cu:1146-1311,
// 797-874).  `iter` selects the view-selection threshold 0.8 exp(-iter^2 / 90) (:1163).
// k_select: 5 waves per SIMD (96 VGPRs; r01_v24 A/B: 1 -> 5 waves -5%, 6 waves spills)
#ifndef ACMMP_SELECT_WAVES
#define ACMMP_SELECT_WAVES 5
#endif
template <int MODEL, int VB, bool GEOM>
__global__ __launch_bounds__(256, ACMMP_SELECT_WAVES) void k_select(const KParams kp, const int colour, const int iter) {
    const long long q = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
    // k_eval_ref's per-block survivor counters, emptied here for the launch that follows (launch_eval_ref's grid:
    // one per kRefPix of the npix work items this grid covers; in place of a memset launch)
    if (kp.ref_split > 0 && q < (static_cast<long long>(kp.row_hi - kp.row_lo) * kp.Wh + kRefPix - 1) / kRefPix)
        kp.surv_count[q] = 0u;
    int px = 0, py = 0;
    if (!colour_pixel(kp, colour, q, px, py)) return;
    const int V = kp.V;
    const long long Pc = kp.Pc;
    const long long ci = static_cast<long long>(py) * kp.Wh + (px >> 1);
    const long long center = static_cast<long long>(py) * kp.W + px;
    const float4 dc = ray_at<MODEL>(kp, px, py);
    Rng rs;
    rs.init(kp.seed_lo, kp.seed_hi, static_cast<uint32_t>(center), kp.rng_cs[colour][ci]);

    int pos[8];
    bool flag[8];
#pragma unroll
    for (int d = 0; d < 8; ++d) {
        pos[d] = kp.nbpos[d * Pc + ci];
        flag[d] = pos[d] >= 0;
    }
    // cost_array[8][32] = {2.0f}: unavailable directions read as 0, element [0][0] as 2 (:957)
    // (the load is unconditional and the value selected after it: a load behind the flag's branch was waited for
    // before the next one issued -- 128 serial L2 / HBM round trips per pixel at V = 15; every slab entry exists)
    auto cost_arr = [&](int d, int v) -> float {
        bool f = flag[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) if (k == d) f = flag[k];
        const float raw = kp.hyp_cost[(static_cast<long long>(d) * V + v) * Pc + ci];
        return f ? raw : ((d == 0 && v == 0) ? 2.0f : 0.0f);
    };

    // ---- joint view selection :1146-1208
    constexpr int VMAX = VB;                                 // launch_select: V <= VB (1, 2, 4, 8, 16 or 32)
    // up to 4 views the 8 x V cost matrix is read once into registers (all loads in flight together)
    // and both passes over it below use it; wider launches re-read it from L2
    constexpr bool kRegCost = VMAX <= 4;
    float ca[8][kRegCost ? VMAX : 1];
    if constexpr (kRegCost) {
#pragma unroll
        for (int d = 0; d < 8; ++d)
#pragma unroll
            for (int v = 0; v < VMAX; ++v) ca[d][v] = v < V ? cost_arr(d, v) : 0.0f;
    }
    auto cost_at_dv = [&](int d, int v) -> float {
        if constexpr (kRegCost) return ca[d][v];
        else return cost_arr(d, v);
    };
    // loops over views run to the compile-time VMAX with a guard, so the per-view arrays stay in
    // registers (statically indexed) instead of scratch
    float vsp[VMAX];
#pragma unroll
    for (int j = 0; j < VMAX; ++j) vsp[j] = 0.0f;
    {
        const int nbx[4] = {px, px, px - 1, px + 1};
        const int nby[4] = {py - 1, py + 1, py, py};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (flag[2 * i]) {
                const uint32_t* sb = ((nbx[i] + nby[i]) & 1) ? kp.sel_cs[1] : kp.sel_cs[0];
                const uint32_t sv = sb[cs_index(kp, nbx[i], nby[i])];
#pragma unroll
                for (int j = 0; j < VMAX; ++j)
                    if (j < V) vsp[j] += ((sv >> j) & 1u) ? 0.9f : 0.1f;
            }
        }
    }
    const float cost_threshold = static_cast<float>(0.8 * static_cast<double>(
        det_exp(static_cast<float>(iter * iter) / (-90.0f))));
    float probs[VMAX];
    // (wide launches: the next view's 8 costs are loaded before this view's are used, so one view's loads are in
    // flight while the previous view computes)
    float nxt[kRegCost ? 1 : 8];
    if constexpr (!kRegCost) {
#pragma unroll
        for (int j = 0; j < 8; j++) nxt[j] = cost_arr(j, 0);
    }
#pragma unroll
    for (int i = 0; i < VMAX; i++) {
        probs[i] = 0.0f;
        if (i >= V) continue;
        float count = 0.0f;
        int count_false = 0;
        float tmpw = 0.0f;
        if constexpr (kRegCost) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const float c = cost_at_dv(j, i);
                if (c < cost_threshold) { tmpw += det_exp(c * c / (-0.18f)); count++; }
                if (c > 1.2f) count_false++;
            }
        } else {
            // branch-free over the 8 directions (the exponential taken for every cost, added only below the
            // threshold: + 0.0f leaves the non-negative sum's bits as they are): no branch between the loads, so
            // they issue together instead of one L2 / HBM round trip each (k_select waited on memory for 73% of
            // its wave cycles at C3)
            float cs[8];
#pragma unroll
            for (int j = 0; j < 8; j++) cs[j] = nxt[j];
            if (i + 1 < V) {
#pragma unroll
                for (int j = 0; j < 8; j++) nxt[j] = cost_arr(j, i + 1);
            }
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const float c = cs[j];
                const bool lt = c < cost_threshold;
                const float e = det_exp(c * c / (-0.18f));
                tmpw += lt ? e : 0.0f;
                count += lt ? 1.0f : 0.0f;
                count_false += c > 1.2f ? 1 : 0;
            }
        }
        float pr = 0.0f;
        if (count > 2 && count_false < 3) pr = tmpw / count;
        else if (count_false < 3) pr = det_exp(cost_threshold * cost_threshold / (-0.32f));
        probs[i] = pr * vsp[i];
    }
    {
        float prob_sum = 0.0f;
#pragma unroll
        for (int i = 0; i < VMAX; ++i) if (i < V) prob_sum += probs[i];
        const float inv = 1.0f / prob_sum;
        float cum = 0.0f;
#pragma unroll
        for (int i = 0; i < VMAX; ++i) if (i < V) { cum = fmaf(probs[i], inv, cum); probs[i] = cum; }
    }
    uint32_t vwp[4] = {0u, 0u, 0u, 0u};
    for (int sample = 0; sample < 15; ++sample) {
        const float rp = rs.uniform() - 1.1920928955078125e-07f;
        // first view whose cumulative probability exceeds the draw (TransformPDFToCDF + :1190-1196)
        int hit = -1;
#pragma unroll
        for (int k = VMAX - 1; k >= 0; --k)
            if (k < V && probs[k] > rp) hit = k;
        if (hit >= 0) {
            const uint32_t inc = 1u << ((hit & 7) * 4);
            if (hit < 8) vwp[0] += inc; else if (hit < 16) vwp[1] += inc; else if (hit < 24) vwp[2] += inc;
            else vwp[3] += inc;
        }
    }
    uint32_t temp_sel = 0u;
    float weight_norm = 0.0f;
    for (int i = 0; i < V; ++i) {
        const float w = vw_get(vwp, i);
        if (w > 0) { temp_sel |= (1u << i); weight_norm += w; }
    }

    // ---- aggregated costs :1210-1228
    float final_costs[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        float fc = 0.0f;
        float4 nb = make_float4(0.f, 0.f, 0.f, 0.f);
        if (GEOM && flag[i]) nb = plane_at(kp, pos[i]);
        auto add_view = [&](int j, float c) {
            const float w = vw_get(vwp, j);
            if (w > 0) {
                if (GEOM) {
                    if (flag[i]) fc = fmaf(w, fmaf(0.2f, geom_cost<MODEL>(kp, j + 1, nb, px, py, dc), c), fc);
                    else fc = fmaf(w, c + 0.1f * 3.0f, fc);
                } else {
                    fc = fmaf(w, c, fc);
                }
            }
        };
        if constexpr (kRegCost) {
#pragma unroll
            for (int j = 0; j < VMAX; ++j)
                if (j < V) add_view(j, ca[i][j]);
        } else {
            // only the selected views' costs are read (a zero-weight view adds nothing): at V = 15 about
            // a quarter of the 8 x V matrix, which k_eval_nb's slab holds in HBM at C3 sizes.  Branch-free: an
            // unselected view loads the pixel's own first entry (cached) and adds nothing, so the loads issue
            // together
            const bool fi = flag[i];
            if (GEOM || VMAX > 16) {                         // (at 32 views the unrolled form spilled 29 dwords)
                for (int j = 0; j < V; ++j)
                    if ((temp_sel >> j) & 1u) add_view(j, cost_arr(i, j));
            } else {
                // branch-free, views beyond V included as never taken (temp_sel has no bit there): one basic block,
                // so the loads issue together.  (take <=> weight > 0: add_view's own test, as a select)
#pragma unroll
                for (int j = 0; j < VMAX; ++j) {
                    const bool take = (temp_sel >> j) & 1u;
                    const float raw = kp.hyp_cost[take ? (static_cast<long long>(i) * V + j) * Pc + ci : ci];
                    const float c = fi ? raw : ((i == 0 && j == 0) ? 2.0f : 0.0f);
                    const float nf = fmaf(vw_get(vwp, j), c, fc);
                    fc = take ? nf : fc;
                }
            }
        }
        final_costs[i] = fc / weight_norm;
    }
    int min_idx = 0;
    {
        float m = final_costs[0];
#pragma unroll
        for (int i = 1; i < 8; ++i) if (final_costs[i] <= m) { m = final_costs[i]; min_idx = i; }
    }

    // ---- current hypothesis :1232-1245 (zero-weight views add +0: skipped)
    float4 cur_plane = kp.plane_cs[colour][ci];
    // the current plane's NCC cost vector is cached from when it was evaluated (k_init, or as the
    // neighbour hypothesis / refinement candidate that won the last sweep).  Views the cache lacks
    // (a candidate whose wave skipped a view) are evaluated here; that is rare and only for them.
    float* cvec = kp.cvec[colour] + ci;
    uint32_t miss = 0u;
    float cost_now = 0.0f;
    constexpr bool kCvecLoop = GEOM || VMAX > 16;
    if (kCvecLoop) {
        for (int v = 0; v < V; ++v)
            if (vw_get(vwp, v) > 0.0f && cvec[v * Pc] != cvec[v * Pc]) miss |= 1u << v;
    } else {
        // branch-free: the selected views' cached costs loaded together (an unselected or absent view reads the
        // first entry, cached, and is not used), folded in view order as below unless one is missing
#pragma unroll
        for (int v = 0; v < VMAX; ++v) {
            const bool take = (temp_sel >> v) & 1u;
            const float c = cvec[take ? static_cast<long long>(v) * Pc : 0];
            miss |= (take && c != c) ? (1u << v) : 0u;
            const float nc = fmaf(vw_get(vwp, v), c, cost_now);
            cost_now = take ? nc : cost_now;
        }
    }
    if (miss) {
        const Patch pt = make_patch<MODEL>(kp, px, py);
        for_all_views<MODEL, 1, 0, true>(kp, px, py, pt, cur_plane, wave_or(miss, V), [&](int v, float c) {
            if ((miss >> v) & 1u) cvec[v * Pc] = c;
        });
    }
    if (kCvecLoop || miss) {
        cost_now = 0.0f;
        for (int v = 0; v < V; ++v) {
            const float w = vw_get(vwp, v);
            if (w > 0.0f) {
                const float c = cvec[v * Pc];
                if (GEOM) cost_now = fmaf(w, fmaf(0.2f, geom_cost<MODEL>(kp, v + 1, cur_plane, px, py, dc), c), cost_now);
                else cost_now = fmaf(w, c, cost_now);
            }
        }
    }
    cost_now /= weight_norm;
    float cur_cost = cost_now;
    uint32_t cur_sel = kp.sel_cs[colour][ci];
    float depth_now = depth_from_plane(cur_plane, dc);
    float restricted_cost = 0.0f;
    const bool use_prior = kp.planar && kp.mask[center] > 0;
    int src_cur = 8;                                        // hypothesis ids, see PixState::src

    // a[i] for a runtime i as a chain of bitwise selects: written as `if (k == i) r = a[k]` the optimiser turned the
    // chain back into an indexed load and put the array in scratch (48 B per lane), and a kernel with a scratch
    // segment runs slowly (k_filter's border array: 0.19 -> 0.07 ms without it)
    auto sel_bits = [](uint32_t r, uint32_t x, bool take) -> uint32_t {
        const uint32_t m = 0u - static_cast<uint32_t>(take);
        return (x & m) | (r & ~m);
    };
    // (up to 4 views; the 16-view instances spilled 230 VGPRs with the array in registers, so they keep the load)
    auto sel_pos = [&](int i) -> int {
        if constexpr (VMAX <= 4) {
            uint32_t r = static_cast<uint32_t>(pos[0]);
#pragma unroll
            for (int k = 1; k < 8; ++k) r = sel_bits(r, static_cast<uint32_t>(pos[k]), k == i);
            return static_cast<int>(r);
        }
        int r = pos[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) if (k == i) r = pos[k];
        return r;
    };
    auto sel_f = [&](const float (&a)[8], int i) -> float {
        if constexpr (VMAX <= 4) {
            uint32_t r = __builtin_bit_cast(uint32_t, a[0]);
#pragma unroll
            for (int k = 1; k < 8; ++k) r = sel_bits(r, __builtin_bit_cast(uint32_t, a[k]), k == i);
            return __builtin_bit_cast(float, r);
        }
        float r = a[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) if (k == i) r = a[k];
        return r;
    };

    if (kp.planar) {                                        // :1247-1299
        const float gamma = 0.5f;
        const float depth_sigma = (kp.depth_max - kp.depth_min) / 64.0f;
        const float two_dss = 2 * depth_sigma * depth_sigma;
        const float angle_sigma = static_cast<float>(kMPi * (5.0f / 180.0f));
        const float two_ass = 2 * angle_sigma * angle_sigma;
        const float4 prior = kp.prior[center];
        const float depth_prior = depth_from_plane(prior, dc);
        const float beta = 0.18f;
        if (use_prior) {
            // the 8 neighbour planes loaded before any of them is tested (an unavailable direction reads this
            // pixel's own plane, unused): behind `flag[i]` each load was waited for before the next
            float4 nbs[8];
#pragma unroll
            for (int i = 0; i < 8; i++) nbs[i] = plane_at(kp, flag[i] ? pos[i] : packpos(px, py));
            float rfc[8];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                rfc[i] = 0.0f;
                if (flag[i]) {
                    const float4 nb = nbs[i];
                    const float ddiff = depth_from_plane(nb, dc) - depth_prior;
                    const float ad = det_acos(dot3n(prior, nb));
                    const float pr = fmaf(det_exp((-ddiff) * ddiff / two_dss), det_exp((-ad) * ad / two_ass), gamma);
                    rfc[i] = det_exp((-final_costs[i]) * final_costs[i] / beta) * pr;
                }
            }
            int max_idx = 0;
            {
                float m = rfc[0];
#pragma unroll
                for (int i = 1; i < 8; ++i) if (rfc[i] >= m) { m = rfc[i]; max_idx = i; }
            }
            const float ddiff = depth_from_plane(cur_plane, dc) - depth_prior;
            const float ad = det_acos(dot3n(prior, cur_plane));
            const float pr = fmaf(det_exp((-ddiff) * ddiff / two_dss), det_exp((-ad) * ad / two_ass), gamma);
            const float rc_now = det_exp((-cost_now) * cost_now / beta) * pr;
            const int mpos = sel_pos(max_idx);
            if (mpos >= 0) {
                const float4 nb = plane_at(kp, mpos);
                const float db = depth_from_plane(nb, dc);
                const float rmax = sel_f(rfc, max_idx);
                if (db >= kp.depth_min && db <= kp.depth_max && rmax > rc_now) {
                    depth_now = db;
                    cur_plane = nb;
                    cur_cost = sel_f(final_costs, max_idx);
                    restricted_cost = rmax;
                    cur_sel = temp_sel;
                    src_cur = max_idx;
                }
            }
        } else {
            const int mpos = sel_pos(min_idx);
            if (mpos >= 0) {
                const float4 nb = plane_at(kp, mpos);
                const float db = depth_from_plane(nb, dc);
                const float fmin = sel_f(final_costs, min_idx);
                if (db >= kp.depth_min && db <= kp.depth_max && fmin < cost_now) {
                    depth_now = db;
                    cur_plane = nb;
                    cur_cost = fmin;
                    src_cur = min_idx;
                }
            }
        }
    }

    float4 plane_now = cur_plane;                           // fix A (:1301)
    int src_now = src_cur;
    if (!kp.planar) {                                       // :1302-1311
        const int mpos = sel_pos(min_idx);
        if (mpos >= 0) {
            const float4 nb = plane_at(kp, mpos);
            const float db = depth_from_plane(nb, dc);
            const float fmin = sel_f(final_costs, min_idx);
            if (db >= kp.depth_min && db <= kp.depth_max && fmin < cost_now) {
                depth_now = db;
                plane_now = nb;
                cost_now = fmin;
                cur_sel = temp_sel;
                src_now = min_idx;
            }
        }
    }

    // ---- PlaneHypothesisRefinement candidates :813-874
    uint32_t flags = use_prior ? 1u : 0u;
    if (weight_norm > 0.0f) {
        flags |= 2u;
        const float perturbation = 0.02f;
        const float depth_sigma = (kp.depth_max - kp.depth_min) / 64.0f;
        const float angle_sigma = kCudartPiF * (5.0f / 180.0f);
        float depth_rand;
        float4 n_rand;
        if (use_prior) {
            const float4 prior = kp.prior[center];
            const float dprior = depth_from_plane(prior, dc);
            depth_rand = sample_depth_inv(rs, fmaxf(dprior - 3 * depth_sigma, kp.depth_min),
                                          fminf(dprior + 3 * depth_sigma, kp.depth_max));
            n_rand = perturbed_normal(dc, prior, rs, angle_sigma);
        } else {
            depth_rand = sample_depth_inv(rs, kp.depth_min, kp.depth_max);
            n_rand = random_normal(dc, rs);
        }
        float lo = fmaxf((1.0f - perturbation) * depth_now, kp.depth_min);
        float hi = fminf((1.0f + perturbation) * depth_now, kp.depth_max);
        if (!(hi > lo)) { lo = kp.depth_min; hi = kp.depth_max; }
        float depth_perturbed = depth_now;
        bool ok = false;
        for (int k = 0; k < 32; ++k) {
            const float cand = sample_depth_inv(rs, lo, hi);
            if (cand >= kp.depth_min && cand <= kp.depth_max) { depth_perturbed = cand; ok = true; break; }
        }
        if (!ok) depth_perturbed = fminf(fmaxf(depth_now, kp.depth_min), kp.depth_max);
        const float4 n_pert = perturbed_normal(dc, plane_now, rs, perturbation * kCudartPiF);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const float dep = (i == 0 || i == 2) ? depth_rand : (i == 4 ? depth_perturbed : depth_now);
            float4 tp = (i == 1 || i == 2) ? n_rand : (i == 3 ? n_pert : plane_now);
            tp.w = dist_to_origin(dc, dep, tp);
            kp.cand[i * Pc + ci] = tp;
            kp.cand_dep[i * Pc + ci] = dep;
        }
    }
    PixState st;
    st.plane_now = plane_now;
    st.cur_plane = cur_plane;
    st.vw = make_uint4(vwp[0], vwp[1], vwp[2], vwp[3]);
    st.cost_now = cost_now;
    st.depth_now = depth_now;
    st.cur_cost = cur_cost;
    st.restricted_cost = restricted_cost;
    st.cur_sel = cur_sel;
    st.flags = flags;
    st.weight_norm = weight_norm;
    st.src = static_cast<uint32_t>(src_now) | (static_cast<uint32_t>(src_cur) << 8);
    kp.pst[ci] = st;
    kp.rng_cs[colour][ci] = rs.n;
}

// Aggregated cost of each valid refinement candidate (ACMMP.cu:876-906).
// the interpolated instance (SPHERE V > 4, fast, binary16) is held to 4 waves per SIMD (its geom form took 129
// VGPRs, 3 waves, once the fallback views are marked)
#ifndef ACMMP_REF_INTERP_WAVES
#define ACMMP_REF_INTERP_WAVES 4
#endif
template <int MODEL, int VB, bool GEOM, int TF>
__global__ __launch_bounds__(256, (MODEL == kSphere && VB > 4 && TF == 2) ? ACMMP_REF_INTERP_WAVES : 1) void k_eval_ref(const KParams kp, const int colour) {
    extern __shared__ float4 lds4[];
    const int t = threadIdx.x;
    const int lp = t / kRefLanes, h = t - lp * kRefLanes;
    const long long q = static_cast<long long>(blockIdx.x) * kRefPix + lp;
    int px = 0, py = 0;
    bool valid = t < kRefPix * kRefLanes && colour_pixel(kp, colour, q, px, py);
    const long long Pc = kp.Pc;
    const long long ci = valid ? static_cast<long long>(py) * kp.Wh + (px >> 1) : 0;
    uint4 vw = make_uint4(0u, 0u, 0u, 0u);
    float weight_norm = 0.0f;
    if (valid) {
        const PixState& st = kp.pst[ci];
        valid = (st.flags & 2u) != 0u;
        vw = st.vw;
        weight_norm = st.weight_norm;
    }
    constexpr int kStaged = (MODEL == kSphere && VB <= 4) ? 4 : 3;
    Patch pt;
    if constexpr (kStaged == 4) pt = coop_patch_sep<kRefPix, kRefLanes>(kp, valid, px, py, lp, h, lds4);
    else pt = coop_patch_nb<MODEL, kRefPix, kRefLanes>(kp, valid, px, py, lp, h, lds4);
    constexpr int VBA = ref_vb_eval<MODEL, VB, TF>();
    if (!valid) return;
    if (kp.ref_split > 0 && h == 0) {                        // the tail's patch, without re-summing it
        const DevCam& rc = kp.cams[0];
        kp.psum[ci] = make_float4(pt.sbw, pt.sref, pt.srr,
                                  texel_padded(rc.img_base, rc.img_pitch, rc.W, rc.H, px, py));
    }
    const float4 dc = ray_at<MODEL>(kp, px, py);
    const float4 tp = kp.cand[h * Pc + ci];
    const float depth_before = depth_from_plane(tp, dc);
    if (depth_before < kp.depth_min || depth_before > kp.depth_max || depth_before >= 1e6f) return;  // :903-906
    const uint32_t vwp[4] = {vw.x, vw.y, vw.z, vw.w};
    uint32_t mask = 0u;
    for (int v = 0; v < kp.V; ++v) if (vw_get(vwp, v) > 0.0f) mask |= 1u << v;
    float temp_cost = 0.0f;
    const uint32_t umask = wave_or(mask, kp.V);
    // split: this kernel takes views [0, S) only, unless the whole wave sits in the SPHERE degenerate
    // band (every cost 2.0 without a sample: nothing to save)
    const int S = kp.ref_split;
    const bool split = S > 0 && __any(!(MODEL == kSphere && pt.sbw < 1e-6f));
    const uint32_t amask = split ? (umask & ((1u << S) - 1u)) : umask;
    float* vcost = kp.cand_vcost + static_cast<long long>(h) * kp.V * Pc + ci;
    for (int v = 0; v < kp.V; ++v)
        if (!((amask >> v) & 1u)) vcost[v * Pc] = __builtin_nanf("");
    // The fast SPHERE V > 4 instance interpolates sample coordinates (ncc_chunk) and gets back the views whose
    // interpolation nodes spread too far (`rough`): those costs are not taken here -- vcost NaN (not evaluated),
    // no term in the chain -- and k_eval_ref_tail recomputes them with every sample projected (the per-sample
    // fast bits).  The chain over the other views is still a lower bound of the final one (below), so the
    // pruning stays exact; a survivor with rough selected views restarts its chain in the tail.
    constexpr bool kRefInterp = MODEL == kSphere && kStaged == 3 && TF == 2;
    uint32_t rough = 0u;
    for_all_views_tf<MODEL, VBA, kStaged, kRefPipe, TF>(kp, px, py, pt, tp, amask, [&](int v, float c) {
        vcost[v * Pc] = c;
        const bool r = kRefInterp && c != c;
        if (r) rough |= 1u << v;
        const float w = vw_get(vwp, v);
        if (w > 0.0f && !r) {
            if (GEOM) temp_cost = fmaf(w, fmaf(0.1f, geom_cost<MODEL>(kp, v + 1, tp, px, py, dc), c), temp_cost);
            else temp_cost = fmaf(w, c, temp_cost);
        }
    }, kRefInterp ? kFixNan : kFixNone);
    const float partial = temp_cost / weight_norm;
    // no split: the whole wave sits in the degenerate band (no sample taken, so nothing rough) or the launch has
    // no tail (launch_eval_ref turns the interpolation off then)
    if (!split) { kp.cand_cost[h * Pc + ci] = partial; return; }
    // Every remaining term w * (c [+ 0.1 geom]) is >= 0 (c in [0, 2], geom in [0, 3]), so the fma chain
    // only grows and, divided by weight_norm > 0, the final cost is >= `partial`: when
    // !(partial < cost_now) the candidate cannot pass k_finish's `temp_cost < cost_now` (cost_now
    // only decreases there), and `partial` stands in for its cost.  Prior-restricted pixels accept by
    // restricted cost instead and always finish.  A survivor that selected no view >= S still goes to
    // the tail: the views >= S its wave evaluates complete its cost vector, which the current-plane
    // cost cache takes over if it wins (a NaN entry there costs k_select a divergent re-evaluation).
    // With rough views left out the chain skips some non-negative terms; fma is monotone in its addend and
    // each skipped step never lowers the full chain, so the partial chain still bounds the final cost from
    // below bit for bit, and the pruning stays exact.
    const PixState& st = kp.pst[ci];
    const bool done = !(st.flags & 1u) && !(partial < st.cost_now);
    kp.cand_cost[h * Pc + ci] = done ? partial : temp_cost;
    if constexpr (kRefInterp) {
        // a survivor's selected views that fell back: queued (pixel << 8 | candidate << 5 | view, the buffer and
        // regions of k_eval_nb's queue, drained before) for k_nb_fix<TEX, true>, which writes their per-sample
        // costs into the candidate's cost vector before the tail runs; the tail restarts the chain
        // (round 5's first form evaluated them in the tail itself: every lane of a tail wave then took every
        // other lane's fallback views, and the tail moved 20 GB per launch at C3 with 48% L2 hits)
        const uint32_t need = done ? 0u : (rough & mask);
        if (!done) kp.cand_rough[h * Pc + ci] = need;
        const unsigned long long any = __ballot(need != 0u);
        if (any) {
            const int lane = lane_id_here();
            const unsigned region = blockIdx.x % kNbFixRegions;
            for (int v = 0; v < S; ++v) {
                const bool redo = (need >> v) & 1u;
                const unsigned long long b = __ballot(redo);
                if (!b) continue;
                const int leader = __ffsll(static_cast<long long>(b)) - 1;
                unsigned base = 0u;
                if (lane == leader) base = atomicAdd(kp.nbfix_count + region, static_cast<unsigned>(__popcll(b)));
                base = __builtin_amdgcn_readlane(base, leader);
                const unsigned slot = base + static_cast<unsigned>(__popcll(b & ((1ull << lane) - 1ull)));
                if (redo && slot < kp.nbfix_cap)
                    kp.nbfix[static_cast<long long>(region) * kp.nbfix_cap + slot] =
                        (static_cast<uint32_t>(ci) << 8) | (static_cast<uint32_t>(h) << 5) | static_cast<uint32_t>(v);
            }
        }
    }
    const unsigned long long b = __ballot(!done);
    if (b) {                                                 // queue the wave's survivors in the block's slots
        const int lane = __lane_id();
        const int leader = __ffsll(static_cast<long long>(b)) - 1;
        unsigned base = 0u;
        if (lane == leader) base = atomicAdd(kp.surv_count + blockIdx.x, static_cast<unsigned>(__popcll(b)));
        base = __shfl(base, leader);
        if (!done)
            kp.surv[static_cast<long long>(blockIdx.x) * kRefSlots + base + __popcll(b & ((1ull << lane) - 1ull))] =
                static_cast<uint32_t>(ci * 8 + h);
    }
}

#if ACMMP_IN_TU(4)
// k_eval_ref's per-block survivor counts -> their exclusive prefix surv_pre[0 .. nref] (surv_pre[nref] =
// all survivors): one block, each thread a contiguous run of k_eval_ref blocks.
__global__ __launch_bounds__(1024) void k_tail_scan(const KParams kp, const int nref) {
    // 8192 counts per pass staged in LDS with coalesced loads (a contiguous run per thread read straight from
    // HBM kept one load in flight per thread: 39 us at the metric, profiles/r04_final_kernel_stats.csv)
    constexpr int kPass = 8192, kPer = kPass / 1024;
    __shared__ unsigned cnt[kPass];
    __shared__ unsigned part[1024];
    const int t = threadIdx.x;
    unsigned carry = 0u;
    for (int base = 0; base < nref; base += kPass) {
        const int m = min(kPass, nref - base);
        for (int i = t; i < m; i += 1024) cnt[i] = kp.surv_count[base + i];
        __syncthreads();
        unsigned v[kPer], sum = 0u;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            v[k] = t * kPer + k < m ? cnt[t * kPer + k] : 0u;
            sum += v[k];
        }
        part[t] = sum;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {           // inclusive scan of the 1024 run sums
            const unsigned add = t >= off ? part[t - off] : 0u;
            __syncthreads();
            part[t] += add;
            __syncthreads();
        }
        unsigned acc = carry + part[t] - sum;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {                     // exclusive prefix, in place
            cnt[t * kPer + k] = acc;
            acc += v[k];
        }
        carry += part[1023];
        __syncthreads();
        for (int i = t; i < m; i += 1024) kp.surv_pre[base + i] = cnt[i];
        __syncthreads();
    }
    if (t == 0) kp.surv_pre[nref] = carry;
}

// The survivors in k_eval_ref block order, dense: block b's slots to surv_dense[surv_pre[b] ...].
__global__ __launch_bounds__(256) void k_tail_compact(const KParams kp) {
    const int b = blockIdx.x, r = threadIdx.x;
    if (r < static_cast<int>(kp.surv_count[b]))
        kp.surv_dense[kp.surv_pre[b] + r] = kp.surv[static_cast<long long>(b) * kRefSlots + r];
}
#endif  // ACMMP_IN_TU(4)

// The queued candidates' views [ref_split, V) (one lane per candidate, patch samples recomputed),
// continuing the aggregate's fma chain in view order from k_eval_ref's partial sum.
// The survivors, in k_eval_ref block order (slots + surv_pre), are dealt to the XCDs as 8 contiguous
// segments (blocks b and b + 8 share an XCD's L2): each XCD's resident blocks walk a window of a few
// rows, so the source footprints its L2 holds are those rows' (a queue shared by all blocks, filled in
// wave completion order, gave C3 a 58% L2 hit rate and 36 GB per launch), and every lane has a survivor
// (per-k_eval_ref-block tail blocks left half their lanes idle; a binary search of surv_pre per 256 survivors
// serialised each block: the metric's tail 0.34 -> 1.2 ms).
template <int MODEL, int VB, bool GEOM, int TF>
__global__ __launch_bounds__(256) void k_eval_ref_tail(const KParams kp, const int colour, const int nref) {
    const unsigned total = kp.surv_pre[nref];
    const unsigned x = blockIdx.x & 7u, k = blockIdx.x >> 3, nk = gridDim.x >> 3;
    const unsigned seg0 = static_cast<unsigned>(static_cast<unsigned long long>(total) * x / 8u);
    const unsigned seg1 = static_cast<unsigned>(static_cast<unsigned long long>(total) * (x + 1u) / 8u);
    const long long Pc = kp.Pc;
    const int S = kp.ref_split;
    for (unsigned i = seg0 + k * 256u + threadIdx.x; i < seg1; i += nk * 256u) {
        const uint32_t rec = kp.surv_dense[i];
        const long long ci = rec >> 3;
        const int h = static_cast<int>(rec & 7u);
        const int py = static_cast<int>(ci / kp.Wh);
        const int px = 2 * static_cast<int>(ci - static_cast<long long>(py) * kp.Wh) + ((py + colour) & 1);
        const PixState& st = kp.pst[ci];
        const uint4 vw = st.vw;
        const float weight_norm = st.weight_norm;
        const uint32_t vwp[4] = {vw.x, vw.y, vw.z, vw.w};
        // k_eval_ref's interpolated instance (SPHERE V > 4, fast, binary16) left out the selected views of
        // [0, S) whose interpolation nodes spread too far (`need`); k_nb_fix<TEX, true> has since written their
        // per-sample costs into the cost vector, so such a candidate's chain restarts from view 0 over the stored
        // costs of [0, S) in view order -- the chain k_eval_ref would have formed with the per-sample costs there
        constexpr bool kRefInterp = MODEL == kSphere && VB > 4 && TF == 2;
        const uint32_t need = kRefInterp ? kp.cand_rough[h * Pc + ci] : 0u;
        uint32_t mask = 0u;
        for (int v = S; v < kp.V; ++v) if (vw_get(vwp, v) > 0.0f) mask |= 1u << v;
        const uint32_t umask = wave_or(mask, kp.V);
        const float4 dc = ray_at<MODEL>(kp, px, py);
        const float4 tp = kp.cand[h * Pc + ci];
        Patch pt;                                            // make_patch's values, from k_eval_ref
        const float4 ps = kp.psum[ci];
        pt.rw = nullptr; pt.rr = nullptr; pt.wr = nullptr; pt.row = pt.col = nullptr; pt.stride = 0;
        pt.sbw = ps.x; pt.sref = ps.y; pt.srr = ps.z; pt.center = ps.w;
        float temp_cost = need ? 0.0f : kp.cand_cost[h * Pc + ci];
        float* vcost = kp.cand_vcost + static_cast<long long>(h) * kp.V * Pc + ci;
        auto add_term = [&](int v, float c) {
            const float w = vw_get(vwp, v);
            if (w > 0.0f) {
                if (GEOM) temp_cost = fmaf(w, fmaf(0.1f, geom_cost<MODEL>(kp, v + 1, tp, px, py, dc), c), temp_cost);
                else temp_cost = fmaf(w, c, temp_cost);
            }
        };
        if (kRefInterp && need)
            for (int v = 0; v < S; ++v) add_term(v, vcost[v * Pc]);
        // SPHERE V > 4: 4-view chunks (87 VGPRs, 5 waves) -- each chunk recomputes the 36 samples' rays,
        // weights and reference texels, so fewer chunks save that work: C3 k_eval_ref + tail 10.52 -> 9.03 ms
        // against 2-view chunks (74 VGPRs, 6 waves), +5.4% (profiles/r04_ab6_ab.txt)
#ifndef ACMMP_TAIL_SPH_VB
#define ACMMP_TAIL_SPH_VB 4
#endif
#ifndef ACMMP_TAIL_PIN_VB
#define ACMMP_TAIL_PIN_VB 4
#endif
        constexpr int VBT = (MODEL == kSphere && VB > 4) ? ACMMP_TAIL_SPH_VB
                          : (MODEL == kPinhole && VB > 4) ? ACMMP_TAIL_PIN_VB : ref_vb<MODEL, VB>();
        for_all_views_tf<MODEL, VBT, 0, kRefPipe, TF>(kp, px, py, pt, tp, umask, [&](int v, float c) {
            vcost[v * Pc] = c;
            add_term(v, c);
        });
        kp.cand_cost[h * Pc + ci] = temp_cost / weight_norm;
    }
}

// Refinement acceptance in candidate order (ACMMP.cu:902-935), hierarchy gate (:1315-1324), store.
template <int MODEL>
__global__ __launch_bounds__(256) void k_finish(const KParams kp, const int colour, const SweepOut out) {
    const long long q = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
    int px = 0, py = 0;
    if (!colour_pixel(kp, colour, q, px, py)) return;
    const long long Pc = kp.Pc;
    const long long ci = static_cast<long long>(py) * kp.Wh + (px >> 1);
    const long long center = static_cast<long long>(py) * kp.W + px;
    const float4 dc = ray_at<MODEL>(kp, px, py);
    const PixState st = kp.pst[ci];
    float4 plane_now = st.plane_now;
    float cost_now = st.cost_now;
    float restricted_cost = st.restricted_cost;
    int src_now = static_cast<int>(st.src & 255u);
    const int src_cur = static_cast<int>((st.src >> 8) & 255u);
    if (st.flags & 2u) {
        const bool use_prior = (st.flags & 1u) != 0u;
        const float gamma = 0.5f;
        const float depth_sigma = (kp.depth_max - kp.depth_min) / 64.0f;
        const float two_dss = 2 * depth_sigma * depth_sigma;
        const float angle_sigma = kCudartPiF * (5.0f / 180.0f);
        const float two_ass = 2 * angle_sigma * angle_sigma;
        const float beta = 0.18f;
        float4 prior = make_float4(0.f, 0.f, 0.f, 0.f);
        float dprior = 0.f;
        if (use_prior) {
            prior = kp.prior[center];
            dprior = depth_from_plane(prior, dc);
        }
        for (int i = 0; i < 5; ++i) {
            const float4 tp = kp.cand[i * Pc + ci];
            const float depth_before = depth_from_plane(tp, dc);
            if (depth_before < kp.depth_min || depth_before > kp.depth_max || depth_before >= 1e6f) continue;
            const float temp_cost = kp.cand_cost[i * Pc + ci];
            if (use_prior) {
                const float ddiff = kp.cand_dep[i * Pc + ci] - dprior;
                const float ac = fminf(fmaxf(dot3n(prior, tp), -1.0f), 1.0f);
                const float ad = det_acos(ac);
                const float pr = fmaf(det_exp((-ddiff) * ddiff / two_dss), det_exp((-ad) * ad / two_ass), gamma);
                const float rtc = det_exp((-temp_cost) * temp_cost / beta) * pr;
                if (rtc > restricted_cost) {
                    plane_now = tp; cost_now = temp_cost; restricted_cost = rtc; src_now = 9 + i;
                }
            } else if (temp_cost < cost_now) {
                plane_now = tp;
                cost_now = temp_cost;
                src_now = 9 + i;
            }
        }
    }
    float4 cur_plane = st.cur_plane;
    float cur_cost = st.cur_cost;
    int src = src_cur;
    if (kp.hier) {
        if (cost_now < kp.pre_rm[center] - 0.1f) { cur_cost = cost_now; cur_plane = plane_now; src = src_now; }
    } else {
        cur_cost = cost_now;
        cur_plane = plane_now;
        src = src_now;
    }
    if (src != 8) {                                          // keep the cost-vector cache in step
        const float* from = src < 8 ? kp.hyp_cost + static_cast<long long>(src) * kp.V * Pc + ci
                                    : kp.cand_vcost + static_cast<long long>(src - 9) * kp.V * Pc + ci;
        float* to = kp.cvec[colour] + ci;
        for (int v = 0; v < kp.V; ++v) to[v * Pc] = from[v * Pc];
    }
    out.plane[ci] = cur_plane;
    out.cost[ci] = cur_cost;
    kp.sel_cs[colour][ci] = st.cur_sel;
}

// ------------------------------------------------------------------ kernels: post

// GetDepthandNormal (ACMMP.cu:1351-1364) fused with the colour-split -> row-major merge.
template <int MODEL>
__global__ void k_merge(const KParams kp, const int do_post) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = kp.merge_lo + static_cast<int>(blockIdx.y * blockDim.y + threadIdx.y);
    if (x >= kp.W || y >= kp.merge_hi) return;
    const int colour = (x + y) & 1;
    const long long ci = cs_index(kp, x, y);
    const long long center = static_cast<long long>(y) * kp.W + x;
    float4 ph = kp.plane_cs[colour][ci];
    if (do_post) {
        ph.w = depth_from_plane(ph, ray_at<MODEL>(kp, x, y));
        ph = to_world(kp.cams[0], ph);
    }
    kp.planes_rm[center] = ph;
    if (do_post) kp.w_rm[center] = ph.w;                    // k_filter's taps (4-byte loads, not float4 lanes)
    kp.costs_rm[center] = kp.cost_cs[colour][ci];
    kp.sel_rm[center] = kp.sel_cs[colour][ci];
}

// Median of 21 values by a selection network where none is NaN or a zero: Batcher's odd-even merge sort on 32
// wires with 11 padded by +inf, cut to the 91 compare-exchanges that reach output 10 and to the min / max halves
// that are read (162 v_min / v_max; scripts/median_net.py generates and checks it).  Without NaNs and signed
// zeros any selection returns the median's bits, so this equals the insertion sort's d[10] (ACMMP.cu:1388-1401).
// Entries {a, b, m}: m & 1 keeps min(v[a], v[b]) in v[a], m & 2 keeps the max in v[b].
__constant__ constexpr unsigned char kMed21[91][3] = {
    {0, 1, 3}, {2, 3, 3}, {0, 2, 3}, {1, 3, 3}, {1, 2, 3}, {4, 5, 3}, {6, 7, 3}, {4, 6, 3}, {5, 7, 3}, {5, 6, 3},
    {0, 4, 3}, {2, 6, 3}, {2, 4, 3}, {1, 5, 3}, {3, 7, 3}, {3, 5, 3}, {1, 2, 3}, {3, 4, 3}, {5, 6, 3}, {8, 9, 3},
    {10, 11, 3}, {8, 10, 3}, {9, 11, 3}, {9, 10, 3}, {12, 13, 3}, {14, 15, 3}, {12, 14, 3}, {13, 15, 3},
    {13, 14, 3}, {8, 12, 3}, {10, 14, 3}, {10, 12, 3}, {9, 13, 3}, {11, 15, 3}, {11, 13, 3}, {9, 10, 3},
    {11, 12, 3}, {13, 14, 3}, {0, 8, 3}, {4, 12, 3}, {4, 8, 3}, {2, 10, 3}, {6, 14, 1}, {6, 10, 3}, {2, 4, 3},
    {6, 8, 3}, {10, 12, 3}, {1, 9, 3}, {5, 13, 3}, {5, 9, 3}, {3, 11, 3}, {7, 15, 1}, {7, 11, 3}, {3, 5, 3},
    {7, 9, 3}, {11, 13, 1}, {1, 2, 3}, {3, 4, 3}, {5, 6, 3}, {7, 8, 3}, {9, 10, 3}, {11, 12, 3}, {16, 17, 3},
    {18, 19, 3}, {16, 18, 3}, {17, 19, 3}, {17, 18, 3}, {16, 20, 3}, {18, 20, 3}, {17, 18, 3}, {19, 20, 3},
    {18, 20, 3}, {17, 18, 3}, {19, 20, 3}, {0, 16, 2}, {8, 16, 2}, {4, 20, 2}, {12, 20, 1}, {12, 16, 1},
    {2, 18, 2}, {10, 18, 1}, {6, 10, 2}, {10, 12, 1}, {1, 17, 2}, {9, 17, 1}, {5, 9, 2}, {3, 19, 2}, {11, 19, 1},
    {7, 11, 1}, {7, 9, 2}, {9, 10, 2}};
__device__ __forceinline__ float median21(float (&v)[21]) {
#pragma unroll
    for (int k = 0; k < 91; ++k) {
        const int a = kMed21[k][0], b = kMed21[k][1], m = kMed21[k][2];
        const float lo = fminf(v[a], v[b]), hi = fmaxf(v[a], v[b]);
        if (m & 1) v[a] = lo;
        if (m & 2) v[b] = hi;
    }
    return v[10];
}

// CheckerboardFilter, ACMMP.cu:1366-1480 (in place; reads only the other colour)
#if ACMMP_IN_TU(0)
__global__ void k_filter(const KParams kp, const int colour) {
    const int kx = blockIdx.x * blockDim.x + threadIdx.x;
    const int py = kp.filt_lo[colour] + static_cast<int>(blockIdx.y * blockDim.y + threadIdx.y);
    const int px = 2 * kx + ((py + colour) & 1);
    if (py >= kp.filt_hi[colour] || px >= kp.W) return;
    const int width = kp.W, height = kp.H;
    const long long center = static_cast<long long>(py) * width + px;
    const float cost = kp.costs_rm[center];                 // (tested after an interior pixel's taps are issued)
    // the taps from k_merge's copy of the depth channel: a wave's 21 tap loads then span 8-byte strides instead of
    // the float4 rows' 32 (every other pixel of a row per lane); the result goes to both (the red pass reads the
    // black pass's results, ACMMP.cu:1549-1552)
    const float* P = kp.w_rm;
    auto wv = [&](long long i) { return P[i]; };
    auto put = [&](float m) { kp.planes_rm[center].w = m; kp.w_rm[center] = m; };
    const int width_ = kp.W, height_ = kp.H;
    if (py > 4 && py < height_ - 5 && px > 4 && px < width_ - 5) {
        // interior: all 21 taps exist; the same insertion sort, unrolled over registers (the
        // early-exit inner loop becomes a "still moving" flag, so NaN orders exactly as :1396)
        const long long w = width_;
        float d[21] = {wv(center), wv(center - w), wv(center - 3 * w), wv(center - 5 * w), wv(center + w),
                       wv(center + 3 * w), wv(center + 5 * w), wv(center - 1), wv(center - 3), wv(center - 5),
                       wv(center + 1), wv(center + 3), wv(center + 5), wv(center - w + 2), wv(center + w + 2),
                       wv(center - w - 2), wv(center + w - 2), wv(center - 1 - 2 * w), wv(center + 1 - 2 * w),
                       wv(center - 1 + 2 * w), wv(center + 1 + 2 * w)};
        if (cost < 0.001f) return;                           // ACMMP.cu:1397; the taps' loads already in flight
        bool plain = true;                                   // no NaN, no signed zero among the taps
#pragma unroll
        for (int i = 0; i < 21; ++i) plain = plain && d[i] == d[i] && d[i] != 0.0f;
        if (plain) {
            put(median21(d));
            return;
        }
#pragma unroll
        for (int i = 1; i < 21; ++i) {
            const float tmp = d[i];
            bool moving = true;
#pragma unroll
            for (int j = i; j >= 1; --j) {
                const bool c = moving && tmp < d[j - 1];
                const float nd = c ? d[j - 1] : (moving ? tmp : d[j]);
                moving = c;
                d[j] = nd;
            }
            if (moving) d[0] = tmp;
        }
        put(d[10]);
        return;
    }
    if (cost < 0.001f) return;
    // border pixels: the taps that exist, in the reference's order (ACMMP.cu:1366-1450), insertion-sorted as sort_small
    // does -- in registers: each tap k is inserted into the sorted first n (<= k) with the interior's "still moving" flag
    // and the slots past n left alone, and the median read by a select over the slots.  (A private array indexed by the
    // running count lived in scratch, and a kernel with a scratch segment gets few waves per CU: k_filter took 0.19 ms
    // per launch at the metric.)
    const long long up = center - width, down = center + width;
    const long long tap[21] = {center, up, center - 3 * width, center - 5 * width, down, center + 3 * width,
                               center + 5 * width, center - 1, center - 3, center - 5, center + 1, center + 3, center + 5,
                               up + 2, down + 2, up - 2, down - 2, center - 1 - 2 * width, center + 1 - 2 * width,
                               center - 1 + 2 * width, center + 1 + 2 * width};
    const bool has[21] = {true, py > 0, py > 2, py > 4, py < height - 1, py < height - 3, py < height - 5, px > 0,
                          px > 2, px > 4, px < width - 1, px < width - 3, px < width - 5,
                          py > 0 && px < width - 2, py < height - 1 && px < width - 2, py > 0 && px > 1,
                          py < height - 1 && px > 1, px > 0 && py > 2, px < width - 1 && py > 2,
                          px > 0 && py < height - 2, px < width - 1 && py < height - 2};
    float v[21];
    int n = 0;
#pragma unroll
    for (int k = 0; k < 21; ++k) {
        v[k] = 0.0f;
        if (!has[k]) continue;
        const float tmp = wv(tap[k]);
        bool moving = true;
#pragma unroll
        for (int j = k; j >= 1; --j) {
            if (j > n) continue;                             // past the sorted prefix and the new slot
            const bool c = moving && tmp < v[j - 1];
            v[j] = c ? v[j - 1] : (moving ? tmp : v[j]);
            moving = c;
        }
        if (moving) v[0] = tmp;
        ++n;
    }
    const int mi = n / 2;
    float lo = 0.0f, hi = 0.0f;
#pragma unroll
    for (int k = 0; k < 21; ++k) {
        if (k == mi - 1) lo = v[k];
        if (k == mi) hi = v[k];
    }
    const float med = (n % 2 == 0) ? (lo + hi) / 2 : hi;
    put(med);
}

// JBU_cu, ACMMP.cu:1558-1616
__global__ void k_jbu(const float* __restrict__ ref, int W, int H, const float* __restrict__ coarse, int sw, int sh,
                      int imagescale, float* __restrict__ out) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y * blockDim.y + threadIdx.y;
    if (x >= W || y >= H) return;
    const float scale = static_cast<float>(1.0 * static_cast<double>(sw) / static_cast<double>(W));
    const float sigmad = 0.50f, sigmar = 25.5f;
    const int nn = (imagescale * imagescale + 1) / 2;
    const float o_y = static_cast<float>(y) * scale, o_x = static_cast<float>(x) * scale;
    const float refPix = texel_plain(ref, W, H, x, y);
    float total = 0.0f, nf = 0.0f;
    for (int j = -nn; j <= nn; ++j) {
        int r_y = f2i_sat(o_y + static_cast<float>(j));
        r_y = (r_y > 0 ? (r_y < sh ? r_y : sh - 1) : 0);
        int r_ys = y + j;
        r_ys = (r_ys > 0 ? (r_ys < H ? r_ys : H - 1) : 0);
        for (int i = -nn; i <= nn; ++i) {
            int r_x = f2i_sat(o_x + static_cast<float>(i));
            r_x = (r_x > 0 ? (r_x < sw ? r_x : sw - 1) : 0);
            const float srcPix = texel_plain(coarse, sw, sh, r_x, r_y);
            int r_xs = x + i;
            r_xs = (r_xs > 0 ? (r_xs < W ? r_xs : W - 1) : 0);
            const float nbPix = texel_plain(ref, W, H, r_xs, r_ys);
            const float tg = spatial_gauss(o_x, o_y, static_cast<float>(r_x), static_cast<float>(r_y), sigmad) *
                             range_gauss(fabsf(refPix - nbPix), sigmar);
            nf += tg;
            total = fmaf(srcPix, tg, total);
        }
    }
    out[static_cast<long long>(y) * W + x] = total / nf;
}

#endif  // ACMMP_IN_TU(0)

// Test hooks: NCC / geom cost of arbitrary (pixel, plane) queries against every source view.
template <int MODEL, int VB>
__global__ void k_debug(const KParams kp, int which, int n, const int* __restrict__ qx, const int* __restrict__ qy,
                        const float4* __restrict__ planes, float* __restrict__ out) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const int x = qx[q], y = qy[q];
    const float4 ph = planes[q];
    const int colour = (x + y) & 1;
    (void)colour;
    const uint32_t all = kp.V >= 32 ? 0xFFFFFFFFu : ((1u << kp.V) - 1u);
    if (which == 0) {
        const Patch pt = make_patch<MODEL>(kp, x, y);
        for_all_views<MODEL, VB, 0, true>(kp, x, y, pt, ph, all,
                                 [&](int v, float c) { out[static_cast<long long>(q) * kp.V + v] = c; });
    } else {
        const float4 dc = ray_at<MODEL>(kp, x, y);
        for (int v = 0; v < kp.V; ++v)
            out[static_cast<long long>(q) * kp.V + v] = geom_cost<MODEL>(kp, v + 1, ph, x, y, dc);
    }
}

// ------------------------------------------------------------------ host launchers

static inline int cdiv(long long a, int b) { return static_cast<int>((a + b - 1) / b); }

#if ACMMP_IN_TU(0)
hipError_t launch_to_f16_pairs(const float* src, int W, int H, uint32_t* dst, int* inexact, hipStream_t s) {
    const long long n = static_cast<long long>(W + 2) * (H + 1);
    k_to_f16_pairs<<<static_cast<unsigned>((n + 255) / 256), 256, 0, s>>>(src, W + 2, H + 1, dst, inexact);
    return hipGetLastError();
}


hipError_t launch_pad_image(const float* src, size_t pitch_floats, int W, int H, float* dst, int dst_pitch,
                            hipStream_t s) {
    dim3 blk(64, 4), grd(cdiv(W + 2, 64), cdiv(H + 2, 4));
    k_pad_image<<<grd, blk, 0, s>>>(src, pitch_floats, W, H, dst, dst_pitch);
    return hipGetLastError();
}

hipError_t launch_ray_tables(const KParams& kp, float4* dirs, float2* sph_row, float2* sph_col, hipStream_t s) {
    if (kp.model == kSphere) {
        const int n = std::max(kp.W, kp.H) + 2 * kp.R;
        k_ray_tables<<<dim3(cdiv(n, 256), 2), dim3(256, 1), 0, s>>>(kp, dirs, sph_row, sph_col);
    } else {
        dim3 blk(64, 4), grd(cdiv(kp.W + 2 * kp.R, 64), cdiv(kp.H + 2 * kp.R, 4));
        k_ray_tables<<<grd, blk, 0, s>>>(kp, dirs, sph_row, sph_col);
    }
    return hipGetLastError();
}

hipError_t launch_spatial_table(const KParams& kp, float* spatial, hipStream_t s) {
    const int rows = kp.model == kSphere ? kp.H : 1;
    k_spatial<<<cdiv(rows, 64), 64, 0, s>>>(kp, spatial);
    return hipGetLastError();
}

#endif  // ACMMP_IN_TU(0)

// View-chunk width: the per-view accumulators live in registers (6 per view).
static inline int pick_vb(int V) { return V <= 1 ? 1 : (V <= 2 ? 2 : (V <= 4 ? 4 : 8)); }

#define ACMMP_DISPATCH(MODEL_RT, V_RT, BODY)                                             \
    do {                                                                                \
        const int vb_ = pick_vb(V_RT);                                                  \
        if ((MODEL_RT) == kSphere) {                                                    \
            constexpr int M = kSphere;                                                  \
            if (vb_ == 1) { constexpr int VBC = 1; BODY; }                              \
            else if (vb_ == 2) { constexpr int VBC = 2; BODY; }                         \
            else if (vb_ == 4) { constexpr int VBC = 4; BODY; }                         \
            else { constexpr int VBC = 8; BODY; }                                       \
        } else {                                                                        \
            constexpr int M = kPinhole;                                                 \
            if (vb_ == 1) { constexpr int VBC = 1; BODY; }                              \
            else if (vb_ == 2) { constexpr int VBC = 2; BODY; }                         \
            else if (vb_ == 4) { constexpr int VBC = 4; BODY; }                         \
            else { constexpr int VBC = 8; BODY; }                                       \
        }                                                                               \
    } while (0)

#define ACMMP_DISPATCH_TF(KP, BODY)                                                     \
    do {                                                                                \
        const int tf_ = tf_of(KP);                                                      \
        if (tf_ == 2) { constexpr int TF = 2; BODY; }                                   \
        else if (tf_ == 1) { constexpr int TF = 1; BODY; }                              \
        else { constexpr int TF = 0; BODY; }                                            \
    } while (0)

#if ACMMP_IN_TU(1)
hipError_t launch_init(const KParams& kp, hipStream_t s) {
    if (kp.init_hi <= kp.init_lo) return hipSuccess;
    dim3 blk(16, 16), grd(xcd_grid(static_cast<long long>(cdiv(kp.W, 16)) * cdiv(kp.init_hi - kp.init_lo, 16)));
    // branch order of ACMMP.cu:686-793
    const int br = (!kp.geom && !kp.hier) ? kInitRandom : kp.planar ? kInitPlanar : kp.upsample ? kInitUpsample
                                                                                                 : kInitReuse;
    if (br == kInitRandom) ACMMP_DISPATCH_TF(kp, ACMMP_DISPATCH(kp.model, kp.V, (k_init<M, kInitVB, kInitRandom, VBC, TF><<<grd, blk, 0, s>>>(kp))));
    else if (br == kInitPlanar)
        ACMMP_DISPATCH_TF(kp, ACMMP_DISPATCH(kp.model, kp.V, (k_init<M, kInitVB, kInitPlanar, VBC, TF><<<grd, blk, 0, s>>>(kp))));
    else if (br == kInitUpsample)
        ACMMP_DISPATCH_TF(kp, ACMMP_DISPATCH(kp.model, kp.V, (k_init<M, kInitVB, kInitUpsample, VBC, TF><<<grd, blk, 0, s>>>(kp))));
    else ACMMP_DISPATCH_TF(kp, ACMMP_DISPATCH(kp.model, kp.V, (k_init<M, kInitVB, kInitReuse, VBC, TF><<<grd, blk, 0, s>>>(kp))));
    return hipGetLastError();
}

hipError_t launch_debug(const KParams& kp, int which, int n, const int* px, const int* py, const float4* planes,
                        float* out, hipStream_t s) {
    dim3 blk(64), grd(cdiv(n, 64));
    ACMMP_DISPATCH(kp.model, kp.V, (k_debug<M, VBC><<<grd, blk, 0, s>>>(kp, which, n, px, py, planes, out)));
    return hipGetLastError();
}

#endif  // ACMMP_IN_TU(1)

// The half-sweep's launches, each in its own translation unit (their kernels are the bulk of the
// template instances); launch_propagate strings them together.
hipError_t launch_eval_nb(const KParams& kp, int colour, hipStream_t s);
hipError_t launch_eval_nb_views(const KParams& kp, int colour, hipStream_t s);
hipError_t launch_select(const KParams& kp, int colour, int iter, hipStream_t s);
hipError_t launch_eval_ref(const KParams& kp, int colour, hipStream_t s);

// The hooks' deferred fallbacks: k_nb_fix's entry code (fix_row, fix_fold) for query pixels and planes.  LANES:
// hypotheses per query (8: acmmp_debug_ncc_nb, k_eval_nb's layout; 5: acmmp_debug_ncc_ref, the refinement's
// candidates, whose production fallbacks run k_nb_fix<1, true>).  out[(q * LANES + h) * V + v].
template <int TEX, int LANES>
__global__ __launch_bounds__(256) void k_debug_nb_fix(const KParams kp, const int* __restrict__ qx,
                                                      const int* __restrict__ qy, const float4* __restrict__ planes,
                                                      float* __restrict__ out) {
    __shared__ float4 smp[kFixPerBlock][36];
    const int t = threadIdx.x, l = t & 63;
    const int ew = l / kFixLanes, j = l - ew * kFixLanes, e = (t >> 6) * kFixPerWave + ew;
    const unsigned region = blockIdx.x % kNbFixRegions, stripes = gridDim.x / kNbFixRegions;
    const unsigned n = min(kp.nbfix_count[region], kp.nbfix_cap);
    const uint32_t* qu = kp.nbfix + static_cast<long long>(region) * kp.nbfix_cap;
    for (unsigned i0 = (blockIdx.x / kNbFixRegions) * kFixPerBlock; i0 < n; i0 += stripes * kFixPerBlock) {
        const unsigned i = i0 + static_cast<unsigned>(e);
        const bool act = ew < kFixPerWave && i < n;
        long long k = 0;
        int v = 0;
        if (act) {
            const uint32_t key = qu[i];
            const int qq = static_cast<int>(key >> 8), h = static_cast<int>((key >> 5) & 7u);
            v = static_cast<int>(key & 31u);
            k = static_cast<long long>(qq) * LANES + h;
            fix_row<TEX>(kp, qx[qq], qy[qq], planes[k], v, j, smp[e]);
        }
        __syncthreads();
        if (act && j == 0) out[k * kp.V + v] = fix_fold(smp[e]);
        __syncthreads();
    }
}

#if ACMMP_IN_TU(2)
// View-chunked k_eval_nb: one launch per chunk of 8 source views when the sources' texels outgrow the
// 256 MB Infinity Cache, so all waves in flight sample the same few images (r02 A/B
// profiles/r02_view_chunk_ab.txt: SPHERE V = 15 at 3200x1600 +3.7%, at 4096x2048 +6.4%; pinhole V = 10
// at 1600x1200, 77 MB of texels, -1% -- not chunked; round 4 with the deferred fallbacks, C3: 8 views 90.2,
// 5 89.6, one launch 89.4 Mpix-it/s, profiles/r04_chunk_ab.txt).  ACMMP_NB_VIEW_CHUNK=c overrides (c <= 0: one
// launch over all views); read per half-sweep.
int nb_view_chunk(const KParams& kp) {
    const char* e = std::getenv("ACMMP_NB_VIEW_CHUNK");
    int c = e ? std::atoi(e) : 0;
    if (!e) {
        // texel bytes of the sources at the reference's size (row-pair binary16 or fp32: 4 B per texel)
        const double bytes = 4.0 * (kp.W + 2) * (kp.H + 2) * kp.V;
        c = (kp.V > 8 && bytes > 160e6) ? 8 : 0;
    }
    return (c <= 0 || c >= kp.V) ? kp.V : c;
}

// k_eval_nb's block shape (KParams::nb_tile): 8 x 4 tiles of the colour grid (a block's 32 pixels then span
// 4 rows, so their patches and source footprints overlap in the CU's L1): k_eval_nb -3% at C2 (3.17 -> 3.07 ms),
// -2.5% at C3, neutral at the metric against 32-pixel row runs (profiles/r05_ab7_ab.txt).  ACMMP_NB_TILE=0: row runs.
int nb_tile_order(const KParams& kp) {
    (void)kp;
    const char* e = std::getenv("ACMMP_NB_TILE");
    return e ? (std::atoi(e) != 0) : 1;
}

hipError_t launch_eval_nb(const KParams& kp0, int colour, hipStream_t s) {
    KParams kp = kp0;
    // interpolation fallbacks deferred to k_nb_fix: fast SPHERE with interpolated coordinates only
    const bool fix = kp.nbfix && kp.model == kSphere && kp.fast && kp.tex16 && kp.interp;
    if (!fix) kp.nbfix = nullptr;
    const int chunk = kp.nb_chunk;                          // nb_view_chunk, fixed when the run's KParams were built
    for (int v0 = 0; v0 < kp.V; v0 += chunk) {
        const int v1 = std::min(kp.V, v0 + chunk);
        const uint32_t hi = v1 >= 32 ? 0xFFFFFFFFu : ((1u << v1) - 1u);
        kp.nb_views = hi & ~((1u << v0) - 1u);
        kp.nb_count_work = v0 == 0;
        // the queue holds one launch's entries (a region's lanes x the chunk's views): emptied before and
        // drained after every view chunk
        hipError_t e = hipSuccess;
        // (k_pick empties them for the first chunk)
        if (fix && v0 > 0 && (e = hipMemsetAsync(kp.nbfix_count, 0, sizeof(unsigned) * kNbFixRegions, s)) != hipSuccess) return e;
        if ((e = launch_eval_nb_views(kp, colour, s)) != hipSuccess) return e;
        if (fix) {
            k_nb_fix<1><<<16 * kNbFixRegions, 256, 0, s>>>(kp, colour);   // 16 stripes per region
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

// Test hook (acmmp_debug_ncc_nb): k_eval_nb's NCC code on given queries of one pixel and 8 planes (the 8
// neighbour hypotheses of k_eval_nb) -- the same coop_patch_nb staging and the same for_all_views_t
// instance (view chunk, STAGED 3, PIPE, TEX, FM), so in the fast SPHERE mode of views >= 1600x800 the
// interpolated source coordinates of DESIGN.md §2.4, which acmmp_debug_ncc (per-sample projection) does
// not run.  out[(q * 8 + h) * V + v].
template <int MODEL, int VB, int TEX, int FM>
__global__ __launch_bounds__(256) void k_debug_nb(const KParams kp, int n, const int* __restrict__ qx,
                                                  const int* __restrict__ qy, const float4* __restrict__ planes,
                                                  float* __restrict__ out) {
    extern __shared__ float4 lds4[];
    const int t = threadIdx.x;
    const int lp = t / kNbLanes, h = t - lp * kNbLanes;
    const int q = blockIdx.x * kNbPix + lp;
    const bool valid = q < n;
    const int px = valid ? qx[q] : 0, py = valid ? qy[q] : 0;
    const Patch pt = coop_patch_nb<MODEL>(kp, valid, px, py, lp, h, lds4);
    if (!valid) return;
    const long long k = static_cast<long long>(q) * kNbLanes + h;
    const float4 ph = planes[k];
    float* o = out + k * kp.V;
    const uint32_t all = kp.V >= 32 ? 0xFFFFFFFFu : ((1u << kp.V) - 1u);
    const uint32_t fixkey = kp.nbfix ? static_cast<uint32_t>(uniform_int(static_cast<int>(blockIdx.x * kNbPix + (t >> 6) * 8))) : kFixNone;
    for_all_views_t<MODEL, nb_vb<MODEL, VB, FM>(), 3, FM ? kNbPipeFast : kNbPipeExact, TEX, FM, true>(
        kp, px, py, pt, ph, all, [&](int v, float c) { o[v] = c; }, fixkey);
}

hipError_t launch_debug_nb(const KParams& kp0, int n, const int* px, const int* py, const float4* planes, float* out,
                           hipStream_t s) {
    // the hook takes k_eval_nb's path, deferred fallbacks included
    KParams kp = kp0;
    const bool fix = kp.nbfix && kp.model == kSphere && kp.fast && kp.tex16 && kp.interp && n < (1 << 24);
    if (!fix) kp.nbfix = nullptr;                           // (ncc_chunk then projects every sample)
    // the queue holds every entry: a region's blocks x 256 lanes x all V views (one launch here)
    if (fix && static_cast<long long>(cdiv(cdiv(n, kNbPix), kNbFixRegions)) * 256 * kp.V > kp.nbfix_cap)
        return hipErrorInvalidValue;
    hipError_t e0 = hipSuccess;
    if (fix && (e0 = hipMemsetAsync(kp.nbfix_count, 0, sizeof(unsigned) * kNbFixRegions, s)) != hipSuccess) return e0;
    const size_t lds_nb = nb_lds_bytes(kp.model, kp.S, kp.nside);
    const dim3 grd = static_cast<unsigned>(cdiv(n, kNbPix));
    if (kp.fast) {
        if (kp.tex16) ACMMP_DISPATCH(kp.model, kp.V, (k_debug_nb<M, VBC, 1, 1><<<grd, 256, lds_nb, s>>>(kp, n, px, py, planes, out)));
        else ACMMP_DISPATCH(kp.model, kp.V, (k_debug_nb<M, VBC, 0, 1><<<grd, 256, lds_nb, s>>>(kp, n, px, py, planes, out)));
    } else {
        if (kp.tex16) ACMMP_DISPATCH(kp.model, kp.V, (k_debug_nb<M, VBC, 1, 0><<<grd, 256, lds_nb, s>>>(kp, n, px, py, planes, out)));
        else ACMMP_DISPATCH(kp.model, kp.V, (k_debug_nb<M, VBC, 0, 0><<<grd, 256, lds_nb, s>>>(kp, n, px, py, planes, out)));
    }
    if (fix) k_debug_nb_fix<1, kNbLanes><<<kNbFixRegions, 256, 0, s>>>(kp, px, py, planes, out);
    return hipGetLastError();
}

hipError_t launch_eval_nb_views(const KParams& kp, int colour, hipStream_t s) {
    const long long npix = static_cast<long long>(kp.row_hi - kp.row_lo) * kp.Wh;
    const size_t lds_nb = nb_lds_bytes(kp.model, kp.S, kp.nside);
    const dim3 grd = static_cast<unsigned>(nb_block_count(kp.row_hi - kp.row_lo, kp.Wh, kp.nb_tile));
    (void)npix;
    if (kp.fast) {
        if (kp.tex16) ACMMP_DISPATCH(kp.model, kp.V, (k_eval_nb<M, VBC, 1, 1><<<grd, 256, lds_nb, s>>>(kp, colour)));
        else ACMMP_DISPATCH(kp.model, kp.V, (k_eval_nb<M, VBC, 0, 1><<<grd, 256, lds_nb, s>>>(kp, colour)));
    } else {
        if (kp.tex16) ACMMP_DISPATCH(kp.model, kp.V, (k_eval_nb<M, VBC, 1, 0><<<grd, 256, lds_nb, s>>>(kp, colour)));
        else ACMMP_DISPATCH(kp.model, kp.V, (k_eval_nb<M, VBC, 0, 0><<<grd, 256, lds_nb, s>>>(kp, colour)));
    }
    return hipGetLastError();
}
#endif  // ACMMP_IN_TU(2)

#if ACMMP_IN_TU(3)
hipError_t launch_select(const KParams& kp, int colour, int iter, hipStream_t s) {
    const long long npix = static_cast<long long>(kp.row_hi - kp.row_lo) * kp.Wh;
    // the per-view arrays of k_select are sized to the next power of two of V: a 32-entry bound for every V
    // above 4 kept C3's (V = 15) probabilities in 384 B of scratch per lane
    const int vs = kp.V <= 4 ? pick_vb(kp.V) : (kp.V <= 8 ? 8 : (kp.V <= 16 ? 16 : 32));
#define ACMMP_SELECT(MV)                                                                                              \
    do {                                                                                                              \
        if (kp.model == kSphere) {                                                                                    \
            if (kp.geom) k_select<kSphere, MV, true><<<cdiv(npix, 256), 256, 0, s>>>(kp, colour, iter);               \
            else k_select<kSphere, MV, false><<<cdiv(npix, 256), 256, 0, s>>>(kp, colour, iter);                      \
        } else {                                                                                                      \
            if (kp.geom) k_select<kPinhole, MV, true><<<cdiv(npix, 256), 256, 0, s>>>(kp, colour, iter);              \
            else k_select<kPinhole, MV, false><<<cdiv(npix, 256), 256, 0, s>>>(kp, colour, iter);                     \
        }                                                                                                             \
    } while (0)
    switch (vs) {
        case 1: ACMMP_SELECT(1); break;
        case 2: ACMMP_SELECT(2); break;
        case 4: ACMMP_SELECT(4); break;
        case 8: ACMMP_SELECT(8); break;
        case 16: ACMMP_SELECT(16); break;
        default: ACMMP_SELECT(32); break;
    }
#undef ACMMP_SELECT
    return hipGetLastError();
}
#endif  // ACMMP_IN_TU(3)

#if ACMMP_IN_TU(4)
hipError_t launch_eval_ref(const KParams& kp0, int colour, hipStream_t s) {
    // the interpolated refinement leaves its rough views to k_eval_ref_tail: none without a split
    KParams kp = kp0;
    if (kp.ref_split <= 0) kp.interp = 0;
    const long long npix = static_cast<long long>(kp.row_hi - kp.row_lo) * kp.Wh;
    const size_t lds_ref = (kp.model == kSphere && pick_vb(kp.V) <= 4) ? sep_lds_bytes(kp.S, kp.nside, kRefPix)
                                                                       : nb_lds_bytes(kp.model, kp.S, kp.nside, kRefPix);
    hipError_t e = hipSuccess;
    const dim3 grd_ref = static_cast<unsigned>(cdiv(npix, kRefPix));
    // (surv_count[0 .. grd_ref.x) is emptied by k_select, which runs right before)
    // the interpolated instance (fast SPHERE, V > 4) queues its survivors' fallback views on k_eval_nb's queue
    // (drained by then): a region's k_eval_ref blocks x 255 candidates x S views fit its room (Pc S / 51 against
    // k_eval_nb's Pc x chunk / 32, S <= chunk)
    const bool ref_fix = kp.interp && kp.nbfix && kp.model == kSphere && kp.fast && kp.tex16 && kp.V > 4;
    if (ref_fix && (e = hipMemsetAsync(kp.nbfix_count, 0, sizeof(unsigned) * kNbFixRegions, s)) != hipSuccess) return e;
    if (kp.geom) ACMMP_DISPATCH_TF(kp, ACMMP_DISPATCH(kp.model, kp.V, (k_eval_ref<M, VBC, true, TF><<<grd_ref, 256, lds_ref, s>>>(kp, colour))));
    else ACMMP_DISPATCH_TF(kp, ACMMP_DISPATCH(kp.model, kp.V, (k_eval_ref<M, VBC, false, TF><<<grd_ref, 256, lds_ref, s>>>(kp, colour))));
    if (ref_fix) k_nb_fix<1, true><<<16 * kNbFixRegions, 256, 0, s>>>(kp, colour);
    if (kp.ref_split > 0) {
        // the survivors' prefix over k_eval_ref blocks, then 8 x nk tail blocks (the queue's length is
        // known on the device only: nk covers the largest possible queue, up to ACMMP_TAIL_NK blocks per XCD; blocks
        // past the queue's end return at once).  Round 5 capped nk at 256: 8192 waves for the metric's ~640k
        // survivors, so most waves took a second, mostly idle pass over the grid-stride loop (the tail's VALU count
        // was 2.4x one pass's).
#ifndef ACMMP_TAIL_NK
#define ACMMP_TAIL_NK 2048
#endif
        const int nref = static_cast<int>(grd_ref.x);
        k_tail_scan<<<1, 1024, 0, s>>>(kp, nref);
        k_tail_compact<<<static_cast<unsigned>(nref), 256, 0, s>>>(kp);
        const unsigned grd = 8u * static_cast<unsigned>(std::min<long long>(ACMMP_TAIL_NK, std::max<long long>(1, cdiv(static_cast<long long>(nref) * kRefSlots, 8 * 256))));
        if (kp.geom) ACMMP_DISPATCH_TF(kp, ACMMP_DISPATCH(kp.model, kp.V, (k_eval_ref_tail<M, VBC, true, TF><<<grd, 256, 0, s>>>(kp, colour, nref))));
        else ACMMP_DISPATCH_TF(kp, ACMMP_DISPATCH(kp.model, kp.V, (k_eval_ref_tail<M, VBC, false, TF><<<grd, 256, 0, s>>>(kp, colour, nref))));
    }
    return hipGetLastError();
}

// Test hook (acmmp_debug_ncc_ref): the refinement's NCC on given queries of one pixel and 5 planes (the 5
// candidates of PlaneHypothesisRefinement, ACMMP.cu:797-936) -- k_eval_ref's staging and NCC instance over
// all views; the views whose interpolation fell back (fast SPHERE, V > 4) are queued as k_eval_ref queues a
// survivor's (candidate << 5 | view keys on the fallback queue) and recomputed by k_debug_nb_fix<1, 5>, whose
// per-entry code (fix_row, fix_fold) is k_nb_fix<1, true>'s.  out[(q * 5 + h) * V + v].
template <int MODEL, int VB, int TF>
__global__ __launch_bounds__(256) void k_debug_ref(const KParams kp, int n, const int* __restrict__ qx,
                                                   const int* __restrict__ qy, const float4* __restrict__ planes,
                                                   float* __restrict__ out) {
    extern __shared__ float4 lds4[];
    const int t = threadIdx.x;
    const int lp = t / kRefLanes, h = t - lp * kRefLanes;
    const int q = blockIdx.x * kRefPix + lp;
    const bool valid = t < kRefPix * kRefLanes && q < n;
    const int px = valid ? qx[q] : 0, py = valid ? qy[q] : 0;
    constexpr int kStaged = (MODEL == kSphere && VB <= 4) ? 4 : 3;
    Patch pt;
    if constexpr (kStaged == 4) pt = coop_patch_sep<kRefPix, kRefLanes>(kp, valid, px, py, lp, h, lds4);
    else pt = coop_patch_nb<MODEL, kRefPix, kRefLanes>(kp, valid, px, py, lp, h, lds4);
    constexpr int VBA = ref_vb_eval<MODEL, VB, TF>();
    if (!valid) return;
    const long long k = static_cast<long long>(q) * kRefLanes + h;
    const float4 ph = planes[k];
    float* o = out + k * kp.V;
    const uint32_t all = kp.V >= 32 ? 0xFFFFFFFFu : ((1u << kp.V) - 1u);
    constexpr bool kRefInterp = MODEL == kSphere && kStaged == 3 && TF == 2;
    uint32_t rough = 0u;
    for_all_views_tf<MODEL, VBA, kStaged, kRefPipe, TF>(kp, px, py, pt, ph, all, [&](int v, float c) {
        o[v] = c;
        if (kRefInterp && c != c) rough |= 1u << v;
    }, kRefInterp && kp.nbfix ? kFixNan : kFixNone);
    if (kRefInterp && kp.nbfix) {
        const unsigned long long any = __ballot(rough != 0u);
        if (any) {
            const int lane = lane_id_here();
            const unsigned region = blockIdx.x % kNbFixRegions;
            for (int v = 0; v < kp.V; ++v) {
                const bool redo = (rough >> v) & 1u;
                const unsigned long long b = __ballot(redo);
                if (!b) continue;
                const int leader = __ffsll(static_cast<long long>(b)) - 1;
                unsigned base = 0u;
                if (lane == leader) base = atomicAdd(kp.nbfix_count + region, static_cast<unsigned>(__popcll(b)));
                base = __builtin_amdgcn_readlane(base, leader);
                const unsigned slot = base + static_cast<unsigned>(__popcll(b & ((1ull << lane) - 1ull)));
                if (redo && slot < kp.nbfix_cap)
                    kp.nbfix[static_cast<long long>(region) * kp.nbfix_cap + slot] =
                        (static_cast<uint32_t>(q) << 8) | (static_cast<uint32_t>(h) << 5) | static_cast<uint32_t>(v);
            }
        }
    }
}

hipError_t launch_debug_ref(const KParams& kp0, int n, const int* px, const int* py, const float4* planes, float* out,
                            hipStream_t s) {
    KParams kp = kp0;
    if (kp.ref_split <= 0) kp.interp = 0;                   // launch_eval_ref's rule
    const size_t lds_ref = (kp.model == kSphere && pick_vb(kp.V) <= 4) ? sep_lds_bytes(kp.S, kp.nside, kRefPix)
                                                                       : nb_lds_bytes(kp.model, kp.S, kp.nside, kRefPix);
    const dim3 grd = static_cast<unsigned>(cdiv(n, kRefPix));
    // the interpolated instance's fallbacks on the context's queue: room for every entry (a region's blocks x
    // 255 candidates x V views), else the hook refuses
    const bool fix = kp.interp && kp.nbfix && kp.model == kSphere && kp.fast && kp.tex16 && kp.V > 4 && n < (1 << 24);
    if (!fix) kp.nbfix = nullptr;
    if (fix && static_cast<long long>(cdiv(grd.x, kNbFixRegions)) * kRefSlots * kp.V > kp.nbfix_cap) return hipErrorInvalidValue;
    hipError_t e0 = hipSuccess;
    if (fix && (e0 = hipMemsetAsync(kp.nbfix_count, 0, sizeof(unsigned) * kNbFixRegions, s)) != hipSuccess) return e0;
    ACMMP_DISPATCH_TF(kp, ACMMP_DISPATCH(kp.model, kp.V, (k_debug_ref<M, VBC, TF><<<grd, 256, lds_ref, s>>>(kp, n, px, py, planes, out))));
    if (fix) k_debug_nb_fix<1, kRefLanes><<<kNbFixRegions, 256, 0, s>>>(kp, px, py, planes, out);
    return hipGetLastError();
}
#endif  // ACMMP_IN_TU(4)

#if ACMMP_IN_TU(0)
hipError_t launch_propagate(const KParams& kp, int colour, int iter, SweepOut out, hipStream_t s, hipEvent_t* ev,
                            bool all_marks) {
    const long long npix = static_cast<long long>(kp.row_hi - kp.row_lo) * kp.Wh;
    hipError_t e = hipSuccess;
#define ACMMP_MARK(i) if (ev && (i < 2 || all_marks) && (e = hipEventRecord(ev[i], s)) != hipSuccess) return e
    // k_pick sits outside the four timed buckets (rocprof lists it): the k_eval_nb bucket the bench's
    // roofline prices is that kernel alone
    k_pick<<<dim3(cdiv(npix, 256), 8), 256, 0, s>>>(kp, colour);
    ACMMP_MARK(0);
    if ((e = launch_eval_nb(kp, colour, s)) != hipSuccess) return e;
    ACMMP_MARK(1);
    if ((e = launch_select(kp, colour, iter, s)) != hipSuccess) return e;
    ACMMP_MARK(2);
    if ((e = launch_eval_ref(kp, colour, s)) != hipSuccess) return e;
    ACMMP_MARK(3);
    if (kp.model == kSphere) k_finish<kSphere><<<cdiv(npix, 256), 256, 0, s>>>(kp, colour, out);
    else k_finish<kPinhole><<<cdiv(npix, 256), 256, 0, s>>>(kp, colour, out);
    ACMMP_MARK(4);
#undef ACMMP_MARK
    return hipGetLastError();
}

hipError_t launch_post(const KParams& kp, int do_post, hipStream_t s) {
    if (kp.merge_hi > kp.merge_lo) {
        dim3 blk(64, 4), grd(cdiv(kp.W, 64), cdiv(kp.merge_hi - kp.merge_lo, 4));
        if (kp.model == kSphere) k_merge<kSphere><<<grd, blk, 0, s>>>(kp, do_post);
        else k_merge<kPinhole><<<grd, blk, 0, s>>>(kp, do_post);
    }
    if (do_post) {
        for (int colour = 0; colour < 2; ++colour) {           // black, then red (ACMMP.cu:1549-1552)
            if (kp.filt_hi[colour] <= kp.filt_lo[colour]) continue;
            dim3 blk(64, 4), grd(cdiv(kp.Wh, 64), cdiv(kp.filt_hi[colour] - kp.filt_lo[colour], 4));
            k_filter<<<grd, blk, 0, s>>>(kp, colour);
        }
    }
    return hipGetLastError();
}


// ------------------------------------------------------------------ kernels: planar prior (device half)
//
// ProcessProblem's triangle rasterisation and prior-depth mask (main.cpp:138-181) with the triangles,
// planes and steps the host computed (planar.h).  One thread per (triangle, p step): the p values are
// the reference's running float sums 0, step, 2 step, ... (recomputed by the same additions), the q
// loop runs as in the reference; the reference overwrites labels in triangle order, so a pixel keeps
// the largest label that reaches it -- atomicMax gives that whatever the schedule.  Same float and
// double arithmetic as the reference's C++ (no contraction): the same pixels, bit for bit.
__global__ __launch_bounds__(256) void k_planar_raster(const PlanarDev pd, uint32_t* mask) {
    const long long t = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= pd.n_steps) return;
    int lo = 0, hi = pd.n_tri - 1;                       // triangle k with first[k] <= t < first[k + 1]
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pd.first[mid] <= t) lo = mid;
        else hi = mid - 1;
    }
    const int k = lo;
    const long long i = t - pd.first[k];
    const float step = pd.step[k];
    float p = 0.f;
    for (long long a = 0; a < i; ++a) p += step;
    const int* tr = pd.tri + 6 * static_cast<long long>(k);
    const uint32_t label = static_cast<uint32_t>(k) + 1u;
    const double rest = 1.0 - static_cast<double>(p);
    for (float q = 0.f; static_cast<double>(q) < rest; q += step) {
        const double w3 = rest - static_cast<double>(q);
        const int x = static_cast<int>(static_cast<double>(p * static_cast<float>(tr[0]) + q * static_cast<float>(tr[2])) +
                                       w3 * static_cast<double>(tr[4]));
        const int y = static_cast<int>(static_cast<double>(p * static_cast<float>(tr[1]) + q * static_cast<float>(tr[3])) +
                                       w3 * static_cast<double>(tr[5]));
        if (x >= 0 && x < pd.W && y >= 0 && y < pd.H) atomicMax(mask + static_cast<long long>(y) * pd.W + x, label);
    }
}

// GetDepthFromPlaneParam (ACMMP.cpp:991-1011) per labelled pixel; out-of-range prior depths drop the
// label (main.cpp:168-180); CudaPlanarPriorInitialization's expansion (ACMMP.cpp:855-862).
__global__ __launch_bounds__(256) void k_planar_mask(const PlanarDev pd, uint32_t* mask, float4* prior) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
    if (i >= pd.W) return;
    const long long c = static_cast<long long>(j) * pd.W + i;
    uint32_t l = mask[c];
    float4 pl = make_float4(0.f, 0.f, 0.f, 0.f);
    if (l > 0) {
        pl = pd.plane[l - 1];
        float d;
        if (pd.model == kSphere) {
            const float2 lat = pd.row_trig[j], lon = pd.col_trig[i];
            const float dx = lat.y * lon.x, dy = -lat.x, dz = lat.y * lon.y;
            const float denom = pl.x * dx + pl.y * dy + pl.z * dz;
            d = (fabsf(denom) < 1e-6f) ? 1e6f : (-pl.w / denom);
        } else {
            d = -pl.w * pd.K0 / ((static_cast<float>(i) - pd.K2) * pl.x +
                                 (pd.K0 / pd.K4) * (static_cast<float>(j) - pd.K5) * pl.y + pd.K0 * pl.z);
        }
        if (!(d <= pd.depth_max && d >= pd.depth_min)) {
            l = 0;
            pl = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    mask[c] = l;
    prior[c] = pl;
}

hipError_t launch_planar_raster(const PlanarDev& pd, uint32_t* mask, hipStream_t s) {
    if (pd.n_steps > 0) k_planar_raster<<<static_cast<unsigned>(cdiv(pd.n_steps, 256)), 256, 0, s>>>(pd, mask);
    return hipGetLastError();
}

hipError_t launch_planar_mask(const PlanarDev& pd, uint32_t* mask, float4* prior, hipStream_t s) {
    k_planar_mask<<<dim3(cdiv(pd.W, 256), pd.H), 256, 0, s>>>(pd, mask, prior);
    return hipGetLastError();
}

// GetSupportPoints (ACMMP.cpp:904-929) on the context's last RunPatchMatch output: one thread per 5x5
// block, scanned column by column with the reference's strict '>' (the first minimum-cost pixel, costs
// 2.0 and above skipped), kept when the minimum is < 0.1.  out[strip * bh + block row] = (kept, x, y,
// depth bits) -- the reference's point order is strip-major, block rows within a strip.
__global__ __launch_bounds__(256) void k_support_points(const float* __restrict__ costs, const float4* __restrict__ planes,
                                                        int W, int H, int bh, int4* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int bw = (W + 4) / 5;
    if (t >= bw * bh) return;
    const int strip = t / bh, rb = t - strip * bh;
    const int col = strip * 5, row = rb * 5;
    const int cb = min(W, col + 5), rbe = min(H, row + 5);
    float min_cost = 2.0f;
    int tx = 0, ty = 0;
    for (int c = col; c < cb; ++c)
        for (int r = row; r < rbe; ++r) {
            const float v = costs[static_cast<long long>(r) * W + c];
            if (v < 2.0f && min_cost > v) { tx = c; ty = r; min_cost = v; }
        }
    const bool keep = min_cost < 0.1f;
    const float d = keep ? planes[static_cast<long long>(ty) * W + tx].w : 0.0f;
    out[t] = make_int4(keep ? 1 : 0, tx, ty, __float_as_int(d));
}

hipError_t launch_support_points(const float* costs, const float4* planes, int W, int H, int4* out, hipStream_t s) {
    const int bh = (H + 4) / 5, n = ((W + 4) / 5) * bh;
    k_support_points<<<cdiv(n, 256), 256, 0, s>>>(costs, planes, W, H, bh, out);
    return hipGetLastError();
}


// ------------------------------------------------------------------ kernel: fusion

// tex2D<float4>(linear filter, unnormalised (c, r)) at an integer texel index WITHOUT the +0.5
// (ACMMP.cu:1690, 1768): the footprint is texels (c-1, c) x (r-1, r), both weights 0.5, clamped
// (wrap is undefined for unnormalised coordinates and acts as clamp).  fp32 fused lerps.
__device__ __forceinline__ float4 fuse_colour(const float* rgba, int W, int H, int c, int r) {
    const int x0 = c - 1 < 0 ? 0 : c - 1, x1 = c > W - 1 ? W - 1 : c;
    const int y0 = r - 1 < 0 ? 0 : r - 1, y1 = r > H - 1 ? H - 1 : r;
    const float4 t00 = reinterpret_cast<const float4*>(rgba)[static_cast<long long>(y0) * W + x0];
    const float4 t10 = reinterpret_cast<const float4*>(rgba)[static_cast<long long>(y0) * W + x1];
    const float4 t01 = reinterpret_cast<const float4*>(rgba)[static_cast<long long>(y1) * W + x0];
    const float4 t11 = reinterpret_cast<const float4*>(rgba)[static_cast<long long>(y1) * W + x1];
    auto lerp = [](float a, float b) { return fmaf(0.5f, b - a, a); };
    const float4 top = make_float4(lerp(t00.x, t10.x), lerp(t00.y, t10.y), lerp(t00.z, t10.z), lerp(t00.w, t10.w));
    const float4 bot = make_float4(lerp(t01.x, t11.x), lerp(t01.y, t11.y), lerp(t01.z, t11.z), lerp(t01.w, t11.w));
    return make_float4(lerp(top.x, bot.x), lerp(top.y, bot.y), lerp(top.z, bot.z), lerp(top.w, bot.w));
}

// SimpleFusionKernel, ACMMP.cu:1662-1814: per reference pixel, the source views whose depth
// reprojects within 1 px, 1% depth and 0.149 rad of normal; >= 3 consistent (the reference
// included) -> averaged point, normal and colour.  out: 9 floats per pixel (x y z nx ny nz c0 c1 c2,
// c0 = 255 * texture .z as the reference stores it).
template <int MODEL>
__global__ void k_fuse(const DevCam* __restrict__ cams, const FuseView* __restrict__ views, int ref, int W, int H,
                       const int* __restrict__ srcs, int n_src, float* __restrict__ out, int* __restrict__ flags) {
    const int c = blockIdx.x * 16 + (threadIdx.x & 15);
    const int r = blockIdx.y * 16 + (threadIdx.x >> 4);
    const bool inside = c < W && r < H;
    int valid = 0;
    const long long idx = static_cast<long long>(r) * W + c;
    if (inside) {
        const DevCam& rc = cams[ref];
        const FuseView rv = views[ref];
        const float ref_depth = rv.depth[idx];
        if (!(ref_depth <= 0.0f)) {
            const float3 X = world_point<MODEL>(rc, static_cast<float>(c), static_cast<float>(r), ref_depth);
            const float rn0 = rv.normal[3 * idx], rn1 = rv.normal[3 * idx + 1], rn2 = rv.normal[3 * idx + 2];
            const float4 rcol = fuse_colour(rv.rgba, W, H, c, r);
            float ps0 = X.x, ps1 = X.y, ps2 = X.z;
            float ns0 = rn0, ns1 = rn1, ns2 = rn2;
            float cs0 = rcol.z * 255.0f, cs1 = rcol.y * 255.0f, cs2 = rcol.x * 255.0f;
            int n = 1;
            for (int j = 0; j < n_src; ++j) {
                const int si = srcs[j];
                if (si < 0) continue;
                const DevCam& sc = cams[si];
                const FuseView sv = views[si];
                float px, py, pd;
                project<MODEL, const DevCam, true>(sc, X, px, py, pd);
                const int src_c = f2i_sat(px + 0.5f), src_r = f2i_sat(py + 0.5f);
                if (src_c < 0 || src_c >= sc.W || src_r < 0 || src_r >= sc.H) continue;
                const long long sidx = static_cast<long long>(src_r) * sv.W + src_c;
                const float sd = sv.depth[sidx];
                if (sd <= 0.0f) continue;
                const float3 Xs = world_point<MODEL>(sc, static_cast<float>(src_c), static_cast<float>(src_r), sd);
                float qx, qy, qd;
                project<MODEL, const DevCam, true>(rc, Xs, qx, qy, qd);
                const float err = det_hypot(static_cast<float>(c) - qx, static_cast<float>(r) - qy);
                const float rel = fabsf(pd - sd) / sd;
                const float sn0 = sv.normal[3 * sidx], sn1 = sv.normal[3 * sidx + 1], sn2 = sv.normal[3 * sidx + 2];
                float dp = dot3(rn0, rn1, rn2, sn0, sn1, sn2);
                dp = fmaxf(-1.0f, fminf(1.0f, dp));
                const float ang = det_acos(dp);
                if (err < 1.0f && rel < 0.01f && ang < 0.149f) {
                    ps0 += Xs.x; ps1 += Xs.y; ps2 += Xs.z;
                    ns0 += sn0; ns1 += sn1; ns2 += sn2;
                    const float4 scol = fuse_colour(sv.rgba, sv.W, sv.H, src_c, src_r);
                    cs0 = fmaf(scol.z, 255.0f, cs0);
                    cs1 = fmaf(scol.y, 255.0f, cs1);
                    cs2 = fmaf(scol.x, 255.0f, cs2);
                    ++n;
                }
            }
            if (n >= 3) {
                const float fn = static_cast<float>(n);
                float* o = out + 9 * idx;
                o[0] = ps0 / fn; o[1] = ps1 / fn; o[2] = ps2 / fn;
                float a0 = ns0 / fn, a1 = ns1 / fn, a2 = ns2 / fn;
                const float len = det_hypot(det_hypot(a0, a1), a2);
                if (len > 0.0f) { a0 /= len; a1 /= len; a2 /= len; }
                o[3] = a0; o[4] = a1; o[5] = a2;
                o[6] = cs0 / fn; o[7] = cs1 / fn; o[8] = cs2 / fn;
                valid = 1;
            }
        }
        flags[idx] = valid;
    }
}

// counts of valid pixels per 256-pixel chunk of the row-major image
__global__ void k_fuse_count(const int* __restrict__ flags, long long P, int* __restrict__ counts) {
    const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
    const int f = i < P ? flags[i] : 0;
    const int n = __syncthreads_count(f);
    if (threadIdx.x == 0) counts[blockIdx.x] = n;
}

// scatter the valid pixels of each chunk to offsets[chunk] + rank within the chunk (pixel order)
__global__ void k_fuse_scatter(const float* __restrict__ dense, const int* __restrict__ flags, long long P,
                               const int* __restrict__ offsets, float* __restrict__ out) {
    __shared__ int wave_tot[4];
    const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
    const int f = i < P ? flags[i] : 0;
    const unsigned long long b = __ballot(f);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int below = __popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0) wave_tot[wave] = __popcll(b);
    __syncthreads();
    int base = offsets[blockIdx.x];
    for (int w = 0; w < wave; ++w) base += wave_tot[w];
    if (f) {
        float* o = out + 9ll * (base + below);
        const float* d = dense + 9 * i;
#pragma unroll
        for (int k = 0; k < 9; ++k) o[k] = d[k];
    }
}

__global__ void k_export_depth(const float4* __restrict__ planes, long long P, float* __restrict__ dst) {
    const long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < P) dst[i] = planes[i].w;
}

hipError_t launch_fuse(int model, const DevCam* cams, const FuseView* views, int ref, int W, int H, const int* srcs,
                       int n_src, float* out_dense, int* flags, int* block_counts, hipStream_t s) {
    dim3 grd(cdiv(W, 16), cdiv(H, 16));
    if (model == kSphere) k_fuse<kSphere><<<grd, 256, 0, s>>>(cams, views, ref, W, H, srcs, n_src, out_dense, flags);
    else k_fuse<kPinhole><<<grd, 256, 0, s>>>(cams, views, ref, W, H, srcs, n_src, out_dense, flags);
    const long long P = static_cast<long long>(W) * H;
    k_fuse_count<<<static_cast<unsigned>((P + 255) / 256), 256, 0, s>>>(flags, P, block_counts);
    return hipGetLastError();
}

hipError_t launch_fuse_compact(int W, int H, const float* out_dense, const int* flags, const int* block_offsets,
                               float* out, hipStream_t s) {
    const long long P = static_cast<long long>(W) * H;
    k_fuse_scatter<<<static_cast<unsigned>((P + 255) / 256), 256, 0, s>>>(out_dense, flags, P, block_offsets, out);
    return hipGetLastError();
}

// A plain copy of n 16-byte words on the compute queue (the state export / restart of a geom pass: at HBM
// rate, where a device-to-device hipMemcpyAsync of the same 38 MB measured ~9 ms inside the pipeline's
// overlapped passes)
__global__ void k_copy16(const uint4* __restrict__ src, long long n, uint4* __restrict__ dst) {
    for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<long long>(gridDim.x) * blockDim.x)
        dst[i] = src[i];
}
__global__ void k_copy4(const uint32_t* __restrict__ src, long long n, uint32_t* __restrict__ dst) {
    for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<long long>(gridDim.x) * blockDim.x)
        dst[i] = src[i];
}

hipError_t launch_copy(const void* src, void* dst, size_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    const bool wide = bytes % 16 == 0 && reinterpret_cast<uintptr_t>(src) % 16 == 0 && reinterpret_cast<uintptr_t>(dst) % 16 == 0;
    const long long n = static_cast<long long>(wide ? bytes / 16 : bytes / 4);
    const unsigned grd = static_cast<unsigned>(std::min<long long>((n + 255) / 256, 8192));
    if (wide) k_copy16<<<grd, 256, 0, s>>>(static_cast<const uint4*>(src), n, static_cast<uint4*>(dst));
    else k_copy4<<<grd, 256, 0, s>>>(static_cast<const uint32_t*>(src), n, static_cast<uint32_t*>(dst));
    return hipGetLastError();
}

hipError_t launch_export_depth(const float4* planes, long long P, float* dst, hipStream_t s) {
    k_export_depth<<<static_cast<unsigned>((P + 255) / 256), 256, 0, s>>>(planes, P, dst);
    return hipGetLastError();
}

hipError_t launch_jbu(const float* ref, int W, int H, const float* coarse, int sw, int sh, int imagescale,
                      float* out, hipStream_t s) {
    dim3 blk(16, 16), grd(cdiv(W, 16), cdiv(H, 16));
    k_jbu<<<grd, blk, 0, s>>>(ref, W, H, coarse, sw, sh, imagescale, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------ diagnostic: the shader clock under load
//
// Not on the PatchMatch path (acmmp_clock_probe, bench.py's `clock`).  The chip lowers its clock under load,
// by different amounts on different devices (MI355X_MICROARCH.md "DVFS give-back" (5): 1.51-1.69 GHz across
// devices for issue-dense bodies), and k_eval_nb is issue-dense: its time tracks that clock.  Eight independent
// chains per lane of the logistic map x <- r x (1 - x) at r = 3.99 (a multiply and an fma per step): a
// VALU-dense body whose operands stay chaotic, so their bits keep toggling as k_eval_nb's data does (an fma
// chain converging to a fixed point draws less power and holds a higher clock, ibid. item 1); the first lane
// of each workgroup reads the shader-cycle counter and the constant 100 MHz counter around the loop (ibid.
// item 6), and the host takes the median of the per-workgroup ratios.
__global__ __launch_bounds__(256) void k_clock_probe(const float* __restrict__ rnd, int iters, ClockStamp* stamps,
                                                     float* __restrict__ sink) {
    const unsigned gid = blockIdx.x * 256u + threadIdx.x;
    float x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = 0.25f + 0.5f * fabsf(rnd[(gid * 8u + k) & 65535u]);
    constexpr float r = 3.99f;
    unsigned long long t0 = 0, r0 = 0;
    if (stamps) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float t = r * x[k];
            x[k] = fmaf(-t, x[k], t);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += x[k];
    if (stamps) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) {
            ClockStamp c;
            c.cycles = t1 - t0;
            c.ticks = r1 - r0;
            stamps[blockIdx.x] = c;
        }
    }
    sink[gid] = s;
}

hipError_t launch_clock_probe(const float* rnd, int iters, int blocks, ClockStamp* stamps, float* sink, hipStream_t s) {
    k_clock_probe<<<blocks, 256, 0, s>>>(rnd, iters, stamps, sink);
    return hipGetLastError();
}

// ------------------------------------------------------------------ exchange check: checksum of a device buffer
//
// sum over the buffer's 32-bit words w_i of mix64((i << 32) | w_i) mod 2^64 (acmmp_device_checksum): a word's
// value and position both enter, and the sum does not depend on the order it is formed in.  The pipeline
// compares every rank's checksum of each map a pass exchanged (acmmp/pipeline.py RcclExchange), so a wrong
// root, buffer or ordering in the grouped broadcast fails the run instead of feeding a wrong map on.
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_checksum(const uint32_t* __restrict__ w, long long n, unsigned long long* out) {
    unsigned long long acc = 0;
    for (long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x; i < n;
         i += static_cast<long long>(gridDim.x) * 256)
        acc += mix64((static_cast<unsigned long long>(i) << 32) | w[i]);
    __shared__ unsigned long long part[256];
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h) part[threadIdx.x] += part[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicAdd(out, part[0]);
}

hipError_t launch_checksum(const void* ptr, size_t bytes, unsigned long long* out, hipStream_t s) {
    const long long n = static_cast<long long>(bytes / 4);
    const unsigned grd = static_cast<unsigned>(std::max<long long>(1, std::min<long long>((n + 255) / 256, 2048)));
    k_checksum<<<grd, 256, 0, s>>>(static_cast<const uint32_t*>(ptr), n, out);
    return hipGetLastError();
}

#endif  // ACMMP_IN_TU(0)

}  // namespace acmmp
