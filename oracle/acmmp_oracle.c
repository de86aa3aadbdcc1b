/*
 * acmmp_oracle.c -- ORACLE / TEST INFRASTRUCTURE ONLY.  PARITY UNPINNED
 * (see acmmp_oracle.h for what pins it instead).
 *
 * A literal, per-pixel CPU restatement of the reference hot path,
 * /root/reference/ACMMP.cu.  Every function cites the reference lines it
 * follows.  It deliberately keeps the reference's structure (one pixel at a
 * time, recompute everything) so it is easy to audit against ACMMP.cu; the
 * product kernels are restructured for gfx950 and must agree with this file
 * bit-for-bit.  OpenMP over pixels inside a half-sweep is deterministic because
 * of the snapshot read rule.
 */
#include "acmmp_oracle.h"
#include "detmath_ref.h"
#include "philox_ref.h"

#include <float.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define CUDART_PI_F 3.141592654f
#define OR_M_PI 3.14159265358979323846
#define INV_2PI_F 0.159154936671257019f
#define INV_PI_F 0.318309873342514038f

typedef struct { float x, y, z, w; } f4;
typedef struct { float x, y, z; } f3;
typedef struct { float x, y; } f2;

typedef struct {
    const or_problem *pb;
    const or_params *pp;
    int W, H, V;
    uint64_t seed;
} Ctx;

static inline f4 ld4(const float *p, size_t i) { f4 r = { p[4 * i], p[4 * i + 1], p[4 * i + 2], p[4 * i + 3] }; return r; }
static inline void st4(float *p, size_t i, f4 v) { p[4 * i] = v.x; p[4 * i + 1] = v.y; p[4 * i + 2] = v.z; p[4 * i + 3] = v.w; }

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* ---- texture fetches (ACMMP.cpp:689-706: float cudaArray, Linear filter,
 *      unnormalised coordinates; Wrap on unnormalised coords degrades to clamp) ---- */

/* tex2D(img, ix + 0.5f, iy + 0.5f): exact texel, clamp-to-edge */
static inline float tex_texel(const float *img, int W, int H, int ix, int iy)
{
    return img[(size_t)clampi(iy, 0, H - 1) * (size_t)W + (size_t)clampi(ix, 0, W - 1)];
}

/* tex2D(img, x + 0.5f, y + 0.5f) with fp32 bilinear weights, clamp-to-edge */
static inline float tex_bilinear(const float *img, int W, int H, float x, float y)
{
    const float fx = floorf(x), fy = floorf(y);
    const float a = x - fx, b = y - fy;
    const int ix = dm_f2i_sat(fx), iy = dm_f2i_sat(fy);
    const int x0 = clampi(ix, 0, W - 1), x1 = (ix >= W - 1) ? W - 1 : clampi(ix + 1, 0, W - 1);
    const int y0 = clampi(iy, 0, H - 1), y1 = (iy >= H - 1) ? H - 1 : clampi(iy + 1, 0, H - 1);
    const float t00 = img[(size_t)y0 * W + x0], t10 = img[(size_t)y0 * W + x1];
    const float t01 = img[(size_t)y1 * W + x0], t11 = img[(size_t)y1 * W + x1];
    const float r0 = fmaf(a, t10 - t00, t00);
    const float r1 = fmaf(a, t11 - t01, t01);
    return fmaf(b, r1 - r0, r0);
}

/* ---- small vector helpers (ACMMP.cu:98-117) ---- */

static inline float dot3(float a0, float a1, float a2, float b0, float b1, float b2)
{
    return fmaf(a2, b2, fmaf(a1, b1, a0 * b0));
}

/* NormalizeVec3, ACMMP.cu:110-117 */
static inline void normalize3(float *x, float *y, float *z)
{
    const float n2 = dot3(*x, *y, *z, *x, *y, *z);
    const float inv = dm_rsqrtf(n2);
    *x *= inv; *y *= inv; *z *= inv;
}

/* ---- camera model ---- */

/* PixelToDir, ACMMP.cu:119-134 */
static f3 pixel_to_dir(const or_camera *c, int px, int py)
{
    f3 d;
    if (c->model == OR_PINHOLE) {
        d.x = ((float)px - c->K[2]) / c->K[0];
        d.y = ((float)py - c->K[5]) / c->K[4];
        d.z = 1.f;
        normalize3(&d.x, &d.y, &d.z);
    } else {
        const float lon = ((float)px - c->params[1]) / (float)c->width * 2.0f * CUDART_PI_F;
        const float lat = -((float)py - c->params[2]) / (float)c->height * CUDART_PI_F;
        float sl, cl, sa, ca;
        dm_sincosf(lon, &sl, &cl);
        dm_sincosf(lat, &sa, &ca);
        d.x = ca * sl;
        d.y = -sa;
        d.z = ca * cl;
    }
    return d;
}

/* Get3DPointonWorld_cu, ACMMP.cu:565-600.  Pinhole treats depth as z (:579-581);
 * the division by fx/fy is the multiplication by the IEEE reciprocal (what
 * nvcc --use_fast_math compiles it to, modulo its approximate reciprocal). */
static f3 world_point(const or_camera *c, float x, float y, float depth)
{
    f3 pc;
    if (c->model == OR_SPHERE) {
        const float lon = (x - c->params[1]) / (float)c->width * 2.0f * CUDART_PI_F;
        const float lat = -(y - c->params[2]) / (float)c->height * CUDART_PI_F;
        float sl, cl, sa, ca;
        dm_sincosf(lon, &sl, &cl);
        dm_sincosf(lat, &sa, &ca);
        pc.x = (ca * sl) * depth;
        pc.y = (-sa) * depth;
        pc.z = (ca * cl) * depth;
    } else {
        pc.x = (depth * (x - c->K[2])) * (1.0f / c->K[0]);
        pc.y = (depth * (y - c->K[5])) * (1.0f / c->K[4]);
        pc.z = depth;
    }
    const float *R = c->R, *t = c->t;
    f3 tmp;
    tmp.x = dot3(R[0], R[3], R[6], pc.x, pc.y, pc.z);
    tmp.y = dot3(R[1], R[4], R[7], pc.x, pc.y, pc.z);
    tmp.z = dot3(R[2], R[5], R[8], pc.x, pc.y, pc.z);
    const float Cx = -dot3(R[0], R[3], R[6], t[0], t[1], t[2]);
    const float Cy = -dot3(R[1], R[4], R[7], t[0], t[1], t[2]);
    const float Cz = -dot3(R[2], R[5], R[8], t[0], t[1], t[2]);
    f3 r = { tmp.x + Cx, tmp.y + Cy, tmp.z + Cz };
    return r;
}

/* ProjectonCamera_cu, ACMMP.cu:602-644.  Pinhole: no depth guard (unlike the host
 * version ACMMP.cpp:342); one IEEE reciprocal of z and two multiplies.
 * Sphere: radial depth, asin/atan2, x/(2pi) and x/pi as multiplications. */
static void project(const or_camera *c, f3 P, f2 *pt, float *depth)
{
    const float *R = c->R, *t = c->t;
    const float tx = dot3(R[0], R[1], R[2], P.x, P.y, P.z) + t[0];
    const float ty = dot3(R[3], R[4], R[5], P.x, P.y, P.z) + t[1];
    const float tz = dot3(R[6], R[7], R[8], P.x, P.y, P.z) + t[2];
    if (c->model == OR_SPHERE) {
        const float d = sqrtf(dot3(tx, ty, tz, tx, ty, tz));
        *depth = d;
        if (d < 1e-6f) {
            pt->x = c->params[1];
            pt->y = c->params[2];
            return;
        }
        const float neg_lat = dm_asinf(ty / d);       /* latitude = -asin(y/d); -latitude */
        const float lon = dm_atan2f(tx, tz);
        pt->x = fmaf(lon * INV_2PI_F, (float)c->width, c->params[1]);
        pt->y = fmaf(neg_lat * INV_PI_F, (float)c->height, c->params[2]);
    } else {
        *depth = tz;
        const float inv = 1.0f / tz;
        pt->x = dot3(c->K[0], c->K[1], c->K[2], tx, ty, tz) * inv;
        pt->y = dot3(c->K[3], c->K[4], c->K[5], tx, ty, tz) * inv;
    }
}

/* ComputeDepthfromPlaneHypothesis, ACMMP.cu:187-193 */
static inline float depth_from_plane(const or_camera *c, f4 ph, int px, int py)
{
    const f3 d = pixel_to_dir(c, px, py);
    const float denom = dot3(ph.x, ph.y, ph.z, d.x, d.y, d.z);
    return (fabsf(denom) < 1e-6f) ? 1e6f : (-ph.w / denom);
}

/* GetDistance2Origin, ACMMP.cu:153-173 */
static inline float dist_to_origin(const or_camera *c, int px, int py, float depth, f4 n)
{
    const f3 d = pixel_to_dir(c, px, py);
    const float X0 = d.x * depth, X1 = d.y * depth, X2 = d.z * depth;
    return -dot3(n.x, n.y, n.z, X0, X1, X2);
}

/* TransformNormal (cam -> world), ACMMP.cu:378-386 */
static inline f4 to_world(const or_camera *c, f4 n)
{
    const float *R = c->R;
    f4 r;
    r.x = dot3(R[0], R[3], R[6], n.x, n.y, n.z);
    r.y = dot3(R[1], R[4], R[7], n.x, n.y, n.z);
    r.z = dot3(R[2], R[5], R[8], n.x, n.y, n.z);
    r.w = n.w;
    return r;
}

/* TransformNormal2RefCam (world -> cam), ACMMP.cu:388-396 */
static inline f4 to_ref(const or_camera *c, f4 n)
{
    const float *R = c->R;
    f4 r;
    r.x = dot3(R[0], R[1], R[2], n.x, n.y, n.z);
    r.y = dot3(R[3], R[4], R[5], n.x, n.y, n.z);
    r.z = dot3(R[6], R[7], R[8], n.x, n.y, n.z);
    r.w = n.w;
    return r;
}

/* ---- random hypotheses (ACMMP.cu:14-22, 194-265) ---- */

/* SampleDepthInv, ACMMP.cu:14-22 */
static inline float sample_depth_inv(or_rng *rs, float dmin, float dmax)
{
    dmin = fmaxf(dmin, 1e-6f);
    dmax = fmaxf(dmax, dmin + 1e-6f);
    const float inv_min = 1.0f / dmax;
    const float inv_max = 1.0f / dmin;
    const float u = or_rng_uniform(rs);
    const float inv = fmaf(u, inv_max - inv_min, inv_min);
    return 1.0f / inv;
}

/* GenerateRandomNormal, ACMMP.cu:194-220 */
static f4 random_normal(const or_camera *c, int px, int py, or_rng *rs)
{
    float q1 = 1.0f, q2 = 1.0f, s = 2.0f;
    while (s >= 1.0f) {
        q1 = fmaf(2.0f, or_rng_uniform(rs), -1.0f);
        q2 = fmaf(2.0f, or_rng_uniform(rs), -1.0f);
        s = fmaf(q2, q2, q1 * q1);
    }
    const float sq = sqrtf(1.0f - s);
    f4 n;
    n.x = (2.0f * q1) * sq;
    n.y = (2.0f * q2) * sq;
    n.z = fmaf(-2.0f, s, 1.0f);
    n.w = 0.0f;
    const f3 v = pixel_to_dir(c, px, py);
    const float dp = dot3(n.x, n.y, n.z, v.x, v.y, v.z);
    if (dp > 0.0f) { n.x = -n.x; n.y = -n.y; n.z = -n.z; }
    normalize3(&n.x, &n.y, &n.z);
    return n;
}

/* GeneratePerturbedNormal, ACMMP.cu:222-257 */
static f4 perturbed_normal(const or_camera *c, int px, int py, f4 n, or_rng *rs, float perturbation)
{
    const f3 v = pixel_to_dir(c, px, py);
    const float a1 = (or_rng_uniform(rs) - 0.5f) * perturbation;
    const float a2 = (or_rng_uniform(rs) - 0.5f) * perturbation;
    const float a3 = (or_rng_uniform(rs) - 0.5f) * perturbation;
    float s1, c1, s2, c2, s3, c3;
    dm_sincosf(a1, &s1, &c1);
    dm_sincosf(a2, &s2, &c2);
    dm_sincosf(a3, &s3, &c3);
    float R[9];
    R[0] = c2 * c3;
    R[1] = fmaf(-c1, s3, (c3 * s1) * s2);
    R[2] = fmaf(c1 * c3, s2, s1 * s3);
    R[3] = c2 * s3;
    R[4] = fmaf(s1 * s2, s3, c1 * c3);
    R[5] = fmaf(-c3, s1, (c1 * s2) * s3);
    R[6] = -s2;
    R[7] = c2 * s1;
    R[8] = c1 * c2;
    f4 p;
    p.x = dot3(R[0], R[1], R[2], n.x, n.y, n.z);
    p.y = dot3(R[3], R[4], R[5], n.x, n.y, n.z);
    p.z = dot3(R[6], R[7], R[8], n.x, n.y, n.z);
    p.w = n.w;                                  /* Mat33DotVec3 leaves .w untouched */
    if (dot3(p.x, p.y, p.z, v.x, v.y, v.z) >= 0.0f) p = n;
    normalize3(&p.x, &p.y, &p.z);
    return p;
}

/* GenerateRandomPlaneHypothesis, ACMMP.cu:259-265 (linear depth) */
static f4 random_plane(const or_camera *c, int px, int py, or_rng *rs, float dmin, float dmax)
{
    const float depth = fmaf(or_rng_uniform(rs), dmax - dmin, dmin);
    f4 ph = random_normal(c, px, py, rs);
    ph.w = dist_to_origin(c, px, py, depth, ph);
    return ph;
}

/* ---- photometric cost ---- */

/* ComputeBilateralWeight, ACMMP.cu:398-403 */
static inline float bilateral_weight(float dx, float dy, float pix, float center, float ss, float sc)
{
    const float sd = sqrtf(fmaf(dy, dy, dx * dx));
    const float cd = fabsf(pix - center);
    return dm_expf((-sd) / (2.0f * ss * ss) - cd / (2.0f * sc * sc));
}

/* ComputeBilateralNCC, ACMMP.cu:405-516; `s` = source image index (1..N-1) */
static float bilateral_ncc(const Ctx *cx, int s, int px, int py, f4 ph)
{
    const or_camera *rc = &cx->pb->cams[0], *sc = &cx->pb->cams[s];
    const float *ref = cx->pb->images[0], *src = cx->pb->images[s];
    const int RW = rc->width, RH = rc->height, SW = sc->width, SH = sc->height;
    const float cost_max = 2.0f;
    const int radius = cx->pp->patch_size / 2;

    const float depth_ref = depth_from_plane(rc, ph, px, py);
    const f3 Pwc = world_point(rc, (float)px, (float)py, depth_ref);
    f2 ptc; float dd;
    project(sc, Pwc, &ptc, &dd);
    if (sc->model != OR_SPHERE) {               /* SPHERE's wrapped centre is unused (:425-427) */
        if (ptc.x < 0.0f || ptc.x >= (float)SW || ptc.y < 0.0f || ptc.y >= (float)SH) return cost_max;
    }

    float scale_x = 1.0f, scale_y = 1.0f, sig = cx->pp->sigma_spatial;
    const int rsph = rc->model == OR_SPHERE;
    if (rsph) {
        const float lat_c = -((float)py - rc->params[2]) / (float)RH * CUDART_PI_F;
        scale_x = (2.0f * CUDART_PI_F / (float)RW) * dm_cosf(lat_c);
        scale_y = (CUDART_PI_F / (float)RH);
        sig = cx->pp->sigma_spatial * (CUDART_PI_F / (float)RH);
    }
    const float invSW = 1.0f / (float)SW;

    const float center = tex_texel(ref, RW, RH, px, py);
    float sum_ref = 0.0f, sum_rr = 0.0f, sum_src = 0.0f, sum_ss = 0.0f, sum_rs = 0.0f, sum_bw = 0.0f;
    for (int i = -radius; i <= radius; i += cx->pp->radius_increment) {
        for (int j = -radius; j <= radius; j += cx->pp->radius_increment) {
            const int rx = px + i, ry = py + j;
            const float rpix = tex_texel(ref, RW, RH, rx, ry);
            const float dn = depth_from_plane(rc, ph, rx, ry);
            const f3 Pw = world_point(rc, (float)rx, (float)ry, dn);
            f2 sp; float sd;
            project(sc, Pw, &sp, &sd);
            if (sc->model == OR_SPHERE) {
                sp.x = fmaf(-floorf(sp.x * invSW), (float)SW, sp.x);      /* wrap lon  (:467) */
                sp.y = fminf(fmaxf(sp.y, 0.0f), (float)SH - 1.0f);        /* clamp lat (:468) */
            } else if (sp.x < 0.0f || sp.x >= (float)SW || sp.y < 0.0f || sp.y >= (float)SH) {
                continue;
            }
            const float spix = tex_bilinear(src, SW, SH, sp.x, sp.y);
            const float dx = rsph ? (float)i * scale_x : (float)i;
            const float dy = rsph ? (float)j * scale_y : (float)j;
            const float w = bilateral_weight(dx, dy, rpix, center, rsph ? sig : cx->pp->sigma_spatial,
                                             cx->pp->sigma_color);
            sum_bw += w;
            sum_ref = fmaf(w, rpix, sum_ref);
            const float wr = w * rpix;
            sum_rr = fmaf(wr, rpix, sum_rr);
            sum_src = fmaf(w, spix, sum_src);
            const float ws = w * spix;
            sum_ss = fmaf(ws, spix, sum_ss);
            sum_rs = fmaf(wr, spix, sum_rs);
        }
    }
    if (sum_bw < 1e-6f) return cost_max;
    const float inv_bw = 1.0f / sum_bw;
    const float m_ref = sum_ref * inv_bw, m_src = sum_src * inv_bw;
    const float e_rr = sum_rr * inv_bw, e_ss = sum_ss * inv_bw, e_rs = sum_rs * inv_bw;
    const float var_ref = fmaf(-m_ref, m_ref, e_rr);
    const float var_src = fmaf(-m_src, m_src, e_ss);
    if (var_ref < 1e-5f || var_src < 1e-5f) return cost_max;
    const float covar = fmaf(-m_ref, m_src, e_rs);
    const float ncc = 1.0f - covar / sqrtf(var_ref * var_src);
    return fmaxf(0.0f, fminf(cost_max, ncc));
}

/* sort_small, ACMMP.cu:36-45 */
static void sort_small(float *d, int n)
{
    int j;
    for (int i = 1; i < n; i++) {
        const float tmp = d[i];
        for (j = i; j >= 1 && tmp < d[j - 1]; j--) d[j] = d[j - 1];
        d[j] = tmp;
    }
}

/* ComputeMultiViewInitialCostandSelectedViews, ACMMP.cu:519-556 */
static float initial_cost(const Ctx *cx, int px, int py, f4 ph, uint32_t *sel)
{
    float cv[32], cvc[32];
    memset(cv, 0, sizeof cv); memset(cvc, 0, sizeof cvc);
    cv[0] = 2.0f; cvc[0] = 2.0f;
    int count = 0, nvalid = 0;
    const int N = cx->pp->num_images;
    for (int i = 1; i < N; ++i) {
        const float c = bilateral_ncc(cx, i, px, py, ph);
        cv[i - 1] = c; cvc[i - 1] = c;
        count++;
        if (c < 2.0f) nvalid++;
    }
    sort_small(cv, count);
    *sel = 0;
    const int top_k = nvalid < cx->pp->top_k ? nvalid : cx->pp->top_k;
    if (top_k > 0) {
        float cost = 0.0f;
        for (int i = 0; i < top_k; ++i) cost += cv[i];
        const float thr = cv[top_k - 1];
        for (int i = 0; i < N - 1; ++i)
            if (cvc[i] <= thr) *sel |= (uint32_t)(1u << i);
        return cost / (float)top_k;
    }
    return 2.0f;
}

/* ComputeGeomConsistencyCost, ACMMP.cu:646-671; `s` = source index (1..N-1) */
static float geom_cost(const Ctx *cx, int s, f4 ph, int px, int py)
{
    const or_camera *rc = &cx->pb->cams[0], *sc = &cx->pb->cams[s];
    const float depth = depth_from_plane(rc, ph, px, py);
    const f3 fwd = world_point(rc, (float)px, (float)py, depth);
    f2 sp; float sd;
    project(sc, fwd, &sp, &sd);
    const float src_depth = tex_texel(cx->pb->depths[s], cx->pb->depth_w[s], cx->pb->depth_h[s],
                                      dm_f2i_sat(sp.x), dm_f2i_sat(sp.y));
    if (src_depth == 0.0f) return 3.0f;
    const f3 s3 = world_point(sc, sp.x, sp.y, src_depth);
    f2 bp; float rd;
    project(rc, s3, &bp, &rd);
    const float dc = (float)px - bp.x, dr = (float)py - bp.y;
    return fminf(3.0f, sqrtf(fmaf(dr, dr, dc * dc)));
}

/* SpatialGauss / RangeGauss, ACMMP.cu:175-185.  Evaluated in float (the reference
 * promotes the exponent to double): see DESIGN.md §2.3. */
static inline float spatial_gauss(float x1, float y1, float x2, float y2, float sigma)
{
    const float dx = x1 - x2, dy = y1 - y2;
    const float dis = (dx * dx + dy * dy) - 0.0f;
    return dm_expf(-dis / (2.0f * sigma * sigma));
}
static inline float range_gauss(float x, float sigma)
{
    const float xp = x - 0.0f;
    return dm_expf(-(xp * xp) / (2.0f * sigma * sigma));
}

/* ---- RandomInitialization, ACMMP.cu:673-795 ---- */
static void init_pixel(const Ctx *cx, or_state *st, int x, int y, or_rng *rs)
{
    const or_params *pp = cx->pp;
    const or_problem *pb = cx->pb;
    const or_camera *rc = &pb->cams[0];
    const int W = cx->W;
    const size_t center = (size_t)y * W + x;
    or_rng_init(rs, cx->seed, center);

    if (!pp->geom_consistency && !pp->hierarchy) {
        const f4 ph = random_plane(rc, x, y, rs, pp->depth_min, pp->depth_max);
        st4(st->planes, center, ph);
        st->costs[center] = initial_cost(cx, x, y, ph, &st->selected_views[center]);
    } else if (pp->planar_prior) {
        if (pb->plane_masks[center] > 0 && st->costs[center] >= 0.1f) {
            const float perturbation = 0.02f;
            const f4 prior = ld4(pb->prior_planes, center);
            float dp = prior.w;
            const float dmin_p = (1 - 3 * perturbation) * dp;
            const float dmax_p = (1 + 3 * perturbation) * dp;
            dp = fmaf(or_rng_uniform(rs), dmax_p - dmin_p, dmin_p);
            f4 php = perturbed_normal(rc, x, y, prior, rs, (float)(3 * perturbation * OR_M_PI));
            php.w = dp;                                       /* quirk: w holds a depth (:700) */
            st4(st->planes, center, php);
            st->costs[center] = initial_cost(cx, x, y, php, &st->selected_views[center]);
        } else {
            f4 ph = ld4(st->planes, center);                  /* normal NOT moved to the ref frame (:704-710) */
            const float depth = ph.w;
            ph.w = dist_to_origin(rc, x, y, depth, ph);
            st4(st->planes, center, ph);
            st->costs[center] = initial_cost(cx, x, y, ph, &st->selected_views[center]);
        }
    } else if (pp->upsample) {
        const float scale = (float)(1.0 * (double)pp->scaled_cols / (double)W);
        const float sigmad = 0.50f, sigmar = 25.5f;
        const int Imagescale = dm_f2i_sat(fmaxf((float)W / pp->scaled_cols, (float)cx->H / pp->scaled_rows));
        const int WinWidth = Imagescale * Imagescale + 1;
        const int nn = WinWidth / 2;
        const float o_y = (float)y * scale, o_x = (float)x * scale;
        const float *ref = pb->images[0];
        const float refPix = tex_texel(ref, W, cx->H, x, y);
        float nf = 0.0f, c_total = 0.0f;
        f4 n_total = { 0.0f, 0.0f, 0.0f, 0.0f };
        for (int j = -nn; j <= nn; ++j) {
            int r_y = dm_f2i_sat(o_y + (float)j);
            r_y = (r_y > 0 ? ((float)r_y < pp->scaled_rows ? r_y : dm_f2i_sat(pp->scaled_rows - 1)) : 0);
            const int r_ys = y + j;
            for (int i = -nn; i <= nn; ++i) {
                int r_x = dm_f2i_sat(o_x + (float)i);
                r_x = (r_x > 0 ? ((float)r_x < pp->scaled_cols ? r_x : dm_f2i_sat(pp->scaled_cols - 1)) : 0);
                const int s_center = dm_f2i_sat((float)r_y * pp->scaled_cols + (float)r_x);
                f4 srcNorm = ld4(pb->scaled_planes, (size_t)s_center);
                const float srcPix = srcNorm.w;
                const int r_xs = x + i;
                const float nbPix = tex_texel(ref, W, cx->H, r_xs, r_ys);
                const float sg = spatial_gauss(o_x, o_y, (float)r_x, (float)r_y, sigmad);
                const float rg = range_gauss(fabsf(refPix - nbPix), sigmar);
                const float tg = sg * rg;
                nf += tg;
                c_total = fmaf(srcPix, tg, c_total);
                srcNorm.x = srcNorm.x * tg; srcNorm.y = srcNorm.y * tg; srcNorm.z = srcNorm.z * tg;
                n_total.x = n_total.x + srcNorm.x;
                n_total.y = n_total.y + srcNorm.y;
                n_total.z = n_total.z + srcNorm.z;
            }
        }
        (void)c_total;                                        /* costs[center] = c_total/nf is overwritten (:766) */
        n_total.x = n_total.x / nf; n_total.y = n_total.y / nf; n_total.z = n_total.z / nf;
        normalize3(&n_total.x, &n_total.y, &n_total.z);
        const f4 cur = ld4(st->planes, center);               /* host-initialised (0,0,0,depth) (ACMMP.cpp:833-840) */
        float c0 = initial_cost(cx, x, y, cur, &st->selected_views[center]);
        st->pre_costs[center] = c0;
        f4 ph = to_ref(rc, n_total);
        const float depth = cur.w;
        ph.w = dist_to_origin(rc, x, y, depth, ph);
        st4(st->planes, center, ph);
        st->costs[center] = initial_cost(cx, x, y, ph, &st->selected_views[center]);
    } else {
        f4 ph = pp->hierarchy ? ld4(pb->scaled_planes, center) : ld4(st->planes, center);
        ph = to_ref(rc, ph);
        const float depth = ph.w;
        ph.w = dist_to_origin(rc, x, y, depth, ph);
        st4(st->planes, center, ph);
        st->costs[center] = initial_cost(cx, x, y, ph, &st->selected_views[center]);
    }
}

static or_trace *g_trace = NULL;
void or_set_trace(or_trace *trace) { g_trace = trace; }

/* ---- PlaneHypothesisRefinement, ACMMP.cu:797-936 (*which <- 9 + accepted candidate) ---- */
static void refine(const Ctx *cx, f4 *plane, float *depth, float *cost, or_rng *rs,
                   const float *vw, float weight_norm, float *restricted_cost, int px, int py, int *which)
{
    if (weight_norm <= 0.0f) return;
    const or_params *pp = cx->pp;
    const or_problem *pb = cx->pb;
    const or_camera *rc = &pb->cams[0];
    const float perturbation = 0.02f;
    const size_t center = (size_t)py * cx->W + px;
    const float gamma = 0.5f;
    const float depth_sigma = (pp->depth_max - pp->depth_min) / 64.0f;
    const float two_dss = 2 * depth_sigma * depth_sigma;
    const float angle_sigma = CUDART_PI_F * (5.0f / 180.0f);
    const float two_ass = 2 * angle_sigma * angle_sigma;
    const float beta = 0.18f;
    const int use_prior = pp->planar_prior && pb->plane_masks[center] > 0;

    float depth_rand;
    f4 n_rand;
    if (use_prior) {
        const f4 prior = ld4(pb->prior_planes, center);
        const float dp = depth_from_plane(rc, prior, px, py);
        depth_rand = sample_depth_inv(rs, fmaxf(dp - 3 * depth_sigma, pp->depth_min),
                                      fminf(dp + 3 * depth_sigma, pp->depth_max));
        n_rand = perturbed_normal(rc, px, py, prior, rs, angle_sigma);
    } else {
        depth_rand = sample_depth_inv(rs, pp->depth_min, pp->depth_max);
        n_rand = random_normal(rc, px, py, rs);
    }

    float lo = fmaxf((1.0f - perturbation) * (*depth), pp->depth_min);
    float hi = fminf((1.0f + perturbation) * (*depth), pp->depth_max);
    if (!(hi > lo)) { lo = pp->depth_min; hi = pp->depth_max; }
    float depth_perturbed = *depth;
    int ok = 0;
    for (int k = 0; k < 32; ++k) {
        const float cand = sample_depth_inv(rs, lo, hi);
        if (cand >= pp->depth_min && cand <= pp->depth_max) { depth_perturbed = cand; ok = 1; break; }
    }
    if (!ok) depth_perturbed = fminf(fmaxf(*depth, pp->depth_min), pp->depth_max);

    const f4 n_pert = perturbed_normal(rc, px, py, *plane, rs, perturbation * CUDART_PI_F);

    const float depths[5] = { depth_rand, *depth, depth_rand, *depth, depth_perturbed };
    const f4 normals[5] = { *plane, n_rand, n_rand, n_pert, *plane };
    const int N = pp->num_images;
    for (int i = 0; i < 5; ++i) {
        f4 tp = normals[i];
        tp.w = dist_to_origin(rc, px, py, depths[i], tp);
        float temp_cost = 0.0f;
        for (int j = 0; j < N - 1; ++j) {
            if (vw[j] > 0.0f) {             /* zero-weight views contribute nothing: skipped */
                const float c = bilateral_ncc(cx, j + 1, px, py, tp);
                if (pp->geom_consistency)
                    temp_cost = fmaf(vw[j], fmaf(0.1f, geom_cost(cx, j + 1, tp, px, py), c), temp_cost);
                else
                    temp_cost = fmaf(vw[j], c, temp_cost);
            }
        }
        if (weight_norm > 0.0f) temp_cost /= weight_norm;
        const float depth_before = depth_from_plane(rc, tp, px, py);
        if (depth_before < pp->depth_min || depth_before > pp->depth_max || depth_before >= 1e6f) continue;
        if (use_prior) {
            const f4 prior = ld4(pb->prior_planes, center);
            const float dp = depth_from_plane(rc, prior, px, py);
            const float ddiff = depths[i] - dp;
            float ac = dot3(prior.x, prior.y, prior.z, tp.x, tp.y, tp.z);
            ac = fminf(fmaxf(ac, -1.0f), 1.0f);
            const float ad = dm_acosf(ac);
            const float prior_w = fmaf(dm_expf((-ddiff) * ddiff / two_dss), dm_expf((-ad) * ad / two_ass), gamma);
            const float rtc = dm_expf((-temp_cost) * temp_cost / beta) * prior_w;
            if (rtc > *restricted_cost) {
                *depth = depth_before; *plane = tp; *cost = temp_cost; *restricted_cost = rtc; *which = 9 + i;
            }
        } else if (temp_cost < *cost) {
            *depth = depth_before; *plane = tp; *cost = temp_cost; *which = 9 + i;
        }
    }
}

/* FindMinCostIndex / FindMaxCostIndex, ACMMP.cu:62-86 (last index wins ties) */
static int find_min_idx(const float *c, int n)
{
    float m = c[0]; int k = 0;
    for (int i = 1; i < n; ++i) if (c[i] <= m) { m = c[i]; k = i; }
    return k;
}
static int find_max_idx(const float *c, int n)
{
    float m = c[0]; int k = 0;
    for (int i = 1; i < n; ++i) if (c[i] >= m) { m = c[i]; k = i; }
    return k;
}

/* ---- CheckerboardPropagation, ACMMP.cu:938-1325.
 * Snapshot rule: every read of another pixel's plane/cost/selected_views sees
 * `in`; the pixel's own running values live in locals; only [center] of `out`
 * is written.  Fix A: plane_hypotheses_now starts as the pixel's own plane. */
static void propagate_pixel(const Ctx *cx, const or_state *in, or_state *out, or_rng *rs,
                            int px, int py, int iter)
{
    const or_params *pp = cx->pp;
    const or_problem *pb = cx->pb;
    const or_camera *rc = &pb->cams[0];
    const int width = cx->W, height = cx->H;
    const int N = pp->num_images;
    const int center = py * width + px;
    const float *costs = in->costs;
    const uint32_t draws_before = rs->n;
    int up_near = center - width, up_far = center - 3 * width;
    int down_near = center + width, down_far = center + 3 * width;
    int left_near = center - 1, left_far = center - 3;
    int right_near = center + 1, right_far = center + 3;

    float cost_array[8][32];
    memset(cost_array, 0, sizeof cost_array);
    cost_array[0][0] = 2.0f;                    /* `= {2.0f}` initialises element [0][0] only */
    int flag[8] = { 0 };
    float costMin; int costMinPoint;

#define EVAL_DIR(D, POS) do { const f4 nb = ld4(in->planes, (size_t)(POS)); \
        for (int v = 1; v < N; ++v) cost_array[D][v - 1] = bilateral_ncc(cx, v, px, py, nb); } while (0)

    if (py > 2) {                                                        /* up_far :966-982 */
        flag[1] = 1; costMin = costs[up_far]; costMinPoint = up_far;
        for (int i = 1; i < 11; ++i) if (py > 2 + 2 * i) {
            const int t = up_far - 2 * i * width;
            if (costs[t] < costMin) { costMin = costs[t]; costMinPoint = t; }
        }
        up_far = costMinPoint; EVAL_DIR(1, up_far);
    }
    if (py < height - 3) {                                               /* down_far :985-1001 */
        flag[3] = 1; costMin = costs[down_far]; costMinPoint = down_far;
        for (int i = 1; i < 11; ++i) if (py < height - 3 - 2 * i) {
            const int t = down_far + 2 * i * width;
            if (costs[t] < costMin) { costMin = costs[t]; costMinPoint = t; }
        }
        down_far = costMinPoint; EVAL_DIR(3, down_far);
    }
    if (px > 2) {                                                        /* left_far :1004-1020 */
        flag[5] = 1; costMin = costs[left_far]; costMinPoint = left_far;
        for (int i = 1; i < 11; ++i) if (px > 2 + 2 * i) {
            const int t = left_far - 2 * i;
            if (costs[t] < costMin) { costMin = costs[t]; costMinPoint = t; }
        }
        left_far = costMinPoint; EVAL_DIR(5, left_far);
    }
    if (px < width - 3) {                                                /* right_far :1023-1039 */
        flag[7] = 1; costMin = costs[right_far]; costMinPoint = right_far;
        for (int i = 1; i < 11; ++i) if (px < width - 3 - 2 * i) {
            const int t = right_far + 2 * i;
            if (costs[t] < costMin) { costMin = costs[t]; costMinPoint = t; }
        }
        right_far = costMinPoint; EVAL_DIR(7, right_far);
    }
    if (py > 0) {                                                        /* up_near :1042-1065 */
        flag[0] = 1; costMin = costs[up_near]; costMinPoint = up_near;
        for (int i = 0; i < 3; ++i) {
            if (py > 1 + i && px > i) {
                const int t = up_near - (1 + i) * width - i;
                if (costs[t] < costMin) { costMin = costs[t]; costMinPoint = t; }
            }
            if (py > 1 + i && px < width - 1 - i) {
                const int t = up_near - (1 + i) * width + i;
                if (costs[t] < costMin) { costMin = costs[t]; costMinPoint = t; }
            }
        }
        up_near = costMinPoint; EVAL_DIR(0, up_near);
    }
    if (py < height - 1) {                                               /* down_near :1068-1091 */
        flag[2] = 1; costMin = costs[down_near]; costMinPoint = down_near;
        for (int i = 0; i < 3; ++i) {
            if (py < height - 2 - i && px > i) {
                const int t = down_near + (1 + i) * width - i;
                if (costs[t] < costMin) { costMin = costs[t]; costMinPoint = t; }
            }
            if (py < height - 2 - i && px < width - 1 - i) {
                const int t = down_near + (1 + i) * width + i;
                if (costs[t] < costMin) { costMin = costs[t]; costMinPoint = t; }
            }
        }
        down_near = costMinPoint; EVAL_DIR(2, down_near);
    }
    if (px > 0) {                                                        /* left_near :1094-1117 */
        flag[4] = 1; costMin = costs[left_near]; costMinPoint = left_near;
        for (int i = 0; i < 3; ++i) {
            if (px > 1 + i && py > i) {
                const int t = left_near - (1 + i) - i * width;
                if (costs[t] < costMin) { costMin = costs[t]; costMinPoint = t; }
            }
            if (px > 1 + i && py < height - 1 - i) {
                const int t = left_near - (1 + i) + i * width;
                if (costs[t] < costMin) { costMin = costs[t]; costMinPoint = t; }
            }
        }
        left_near = costMinPoint; EVAL_DIR(4, left_near);
    }
    if (px < width - 1) {                                                /* right_near :1120-1143 */
        flag[6] = 1; costMin = costs[right_near]; costMinPoint = right_near;
        for (int i = 0; i < 3; ++i) {
            if (px < width - 2 - i && py > i) {
                const int t = right_near + (1 + i) - i * width;
                if (costs[t] < costMin) { costMin = costs[t]; costMinPoint = t; }
            }
            if (px < width - 2 - i && py < height - 1 - i) {
                const int t = right_near + (1 + i) + i * width;
                if (costs[t] < costMin) { costMin = costs[t]; costMinPoint = t; }
            }
        }
        right_near = costMinPoint; EVAL_DIR(6, right_near);
    }
#undef EVAL_DIR
    const int positions[8] = { up_near, up_far, down_near, down_far, left_near, left_far, right_near, right_far };

    /* joint view selection :1146-1208 */
    float vw[32], vsp[32];
    memset(vw, 0, sizeof vw); memset(vsp, 0, sizeof vsp);
    const int nbpos[4] = { center - width, center + width, center - 1, center + 1 };
    for (int i = 0; i < 4; ++i) {
        if (flag[2 * i]) {
            const uint32_t sv = in->selected_views[nbpos[i]];
            for (int j = 0; j < N - 1; ++j) {
                if (((sv >> j) & 1u) == 1u) vsp[j] += 0.9f;
                else vsp[j] += 0.1f;
            }
        }
    }
    float probs[32];
    memset(probs, 0, sizeof probs);
    const float cost_threshold = (float)(0.8 * (double)dm_expf((float)(iter * iter) / (-90.0f)));
    for (int i = 0; i < N - 1; i++) {
        float count = 0.0f; int count_false = 0; float tmpw = 0.0f;
        for (int j = 0; j < 8; j++) {
            const float c = cost_array[j][i];
            if (c < cost_threshold) { tmpw += dm_expf(c * c / (-0.18f)); count++; }
            if (c > 1.2f) count_false++;
        }
        if (count > 2 && count_false < 3) probs[i] = tmpw / count;
        else if (count_false < 3) probs[i] = dm_expf(cost_threshold * cost_threshold / (-0.32f));
        probs[i] = probs[i] * vsp[i];
    }
    {   /* TransformPDFToCDF :137-151 */
        float prob_sum = 0.0f;
        for (int i = 0; i < N - 1; ++i) prob_sum += probs[i];
        const float inv = 1.0f / prob_sum;
        float cum = 0.0f;
        for (int i = 0; i < N - 1; ++i) { cum = fmaf(probs[i], inv, cum); probs[i] = cum; }
    }
    for (int sample = 0; sample < 15; ++sample) {
        const float rp = or_rng_uniform(rs) - FLT_EPSILON;
        for (int k = 0; k < N - 1; ++k) {
            if (probs[k] > rp) { vw[k] += 1.0f; break; }
        }
    }
    uint32_t temp_sel = 0; float weight_norm = 0.0f;
    for (int i = 0; i < N - 1; ++i) {
        if (vw[i] > 0) { temp_sel |= (uint32_t)(1u << i); weight_norm += vw[i]; }
    }

    /* aggregated costs :1210-1228 */
    float final_costs[8];
    for (int i = 0; i < 8; ++i) {
        float fc = 0.0f;
        for (int j = 0; j < N - 1; ++j) {
            if (vw[j] > 0) {
                if (pp->geom_consistency) {
                    if (flag[i]) {
                        const f4 nb = ld4(in->planes, (size_t)positions[i]);
                        fc = fmaf(vw[j], fmaf(0.2f, geom_cost(cx, j + 1, nb, px, py), cost_array[i][j]), fc);
                    } else {
                        fc = fmaf(vw[j], cost_array[i][j] + 0.1f * 3.0f, fc);
                    }
                } else {
                    fc = fmaf(vw[j], cost_array[i][j], fc);
                }
            }
        }
        final_costs[i] = fc / weight_norm;
    }
    const int min_idx = find_min_idx(final_costs, 8);

    /* current hypothesis :1232-1245 */
    f4 cur_plane = ld4(in->planes, (size_t)center);
    float cost_now = 0.0f;
    for (int i = 0; i < N - 1; ++i) {
        if (vw[i] > 0.0f) {                 /* 0 * finite cost == +0: skipping is exact */
            const float c = bilateral_ncc(cx, i + 1, px, py, cur_plane);
            if (pp->geom_consistency)
                cost_now = fmaf(vw[i], fmaf(0.2f, geom_cost(cx, i + 1, cur_plane, px, py), c), cost_now);
            else
                cost_now = fmaf(vw[i], c, cost_now);
        }
    }
    cost_now /= weight_norm;
    float cur_cost = cost_now;                                  /* costs[center] = cost_now (:1244) */
    uint32_t cur_sel = in->selected_views[center];
    float depth_now = depth_from_plane(rc, cur_plane, px, py);
    float restricted_cost = 0.0f;
    int max_idx_tr = -1, accepted = 8;

    if (pp->planar_prior) {                                     /* :1247-1299 */
        float rfc[8] = { 0 };
        const float gamma = 0.5f;
        const float depth_sigma = (pp->depth_max - pp->depth_min) / 64.0f;
        const float two_dss = 2 * depth_sigma * depth_sigma;
        const float angle_sigma = (float)(OR_M_PI * (5.0f / 180.0f));
        const float two_ass = 2 * angle_sigma * angle_sigma;
        const f4 prior = ld4(pb->prior_planes, (size_t)center);
        const float depth_prior = depth_from_plane(rc, prior, px, py);
        const float beta = 0.18f;
        if (pb->plane_masks[center] > 0) {
            for (int i = 0; i < 8; i++) {
                if (flag[i]) {
                    const f4 nb = ld4(in->planes, (size_t)positions[i]);
                    const float dn = depth_from_plane(rc, nb, px, py);
                    const float ddiff = dn - depth_prior;
                    const float ac = dot3(prior.x, prior.y, prior.z, nb.x, nb.y, nb.z);
                    const float ad = dm_acosf(ac);
                    const float pr = fmaf(dm_expf((-ddiff) * ddiff / two_dss), dm_expf((-ad) * ad / two_ass), gamma);
                    rfc[i] = dm_expf((-final_costs[i]) * final_costs[i] / beta) * pr;
                }
            }
            const int max_idx = find_max_idx(rfc, 8);
            max_idx_tr = max_idx;
            const float dn = depth_from_plane(rc, cur_plane, px, py);
            const float ddiff = dn - depth_prior;
            const float ac = dot3(prior.x, prior.y, prior.z, cur_plane.x, cur_plane.y, cur_plane.z);
            const float ad = dm_acosf(ac);
            const float pr = fmaf(dm_expf((-ddiff) * ddiff / two_dss), dm_expf((-ad) * ad / two_ass), gamma);
            const float rc_now = dm_expf((-cost_now) * cost_now / beta) * pr;
            if (flag[max_idx]) {
                const f4 nb = ld4(in->planes, (size_t)positions[max_idx]);
                const float db = depth_from_plane(rc, nb, px, py);
                if (db >= pp->depth_min && db <= pp->depth_max && rfc[max_idx] > rc_now) {
                    depth_now = db;
                    cur_plane = nb;
                    cur_cost = final_costs[max_idx];
                    restricted_cost = rfc[max_idx];
                    cur_sel = temp_sel;
                    accepted = max_idx;
                }
            }
        } else if (flag[min_idx]) {
            const f4 nb = ld4(in->planes, (size_t)positions[min_idx]);
            const float db = depth_from_plane(rc, nb, px, py);
            if (db >= pp->depth_min && db <= pp->depth_max && final_costs[min_idx] < cost_now) {
                depth_now = db;
                cur_plane = nb;
                cur_cost = final_costs[min_idx];
                accepted = min_idx;
            }
        }
    }

    f4 plane_now = cur_plane;                                   /* fix A at :1301 */
    if (!pp->planar_prior && flag[min_idx]) {                   /* :1302-1311 */
        const f4 nb = ld4(in->planes, (size_t)positions[min_idx]);
        const float db = depth_from_plane(rc, nb, px, py);
        if (db >= pp->depth_min && db <= pp->depth_max && final_costs[min_idx] < cost_now) {
            depth_now = db;
            plane_now = nb;
            cost_now = final_costs[min_idx];
            cur_sel = temp_sel;
            accepted = min_idx;
        }
    }
    const float cost_now_cur = cost_now;

    refine(cx, &plane_now, &depth_now, &cost_now, rs, vw, weight_norm, &restricted_cost, px, py, &accepted);
    if (g_trace) {
        or_trace *t = &g_trace[center];
        for (int d = 0; d < 8; ++d) { t->pos[d] = flag[d] ? positions[d] : -1; t->final_costs[d] = final_costs[d]; }
        t->cost_now = cost_now_cur;
        t->min_idx = min_idx;
        t->max_idx = max_idx_tr;
        t->accepted = accepted;
        t->temp_selected_views = temp_sel;
        t->draws_before = draws_before;
        t->draws_after = rs->n;
        for (int v = 0; v < 32; ++v) t->view_weights[v] = (uint8_t)vw[v];
    }

    if (pp->hierarchy) {                                        /* :1315-1324 */
        if (cost_now < in->pre_costs[center] - 0.1f) {
            cur_cost = cost_now;
            cur_plane = plane_now;
        }
    } else {
        cur_cost = cost_now;
        cur_plane = plane_now;
    }
    out->costs[center] = cur_cost;
    st4(out->planes, (size_t)center, cur_plane);
    out->selected_views[center] = cur_sel;
}

/* ---- GetDepthandNormal :1351-1364 and CheckerboardFilter :1366-1480 ---- */
static void depth_and_normal(const Ctx *cx, or_state *st, int x, int y)
{
    const or_camera *rc = &cx->pb->cams[0];
    const size_t center = (size_t)y * cx->W + x;
    f4 ph = ld4(st->planes, center);
    ph.w = depth_from_plane(rc, ph, x, y);
    ph = to_world(rc, ph);
    st4(st->planes, center, ph);
}

static void filter_pixel(const Ctx *cx, or_state *st, int px, int py)
{
    const int width = cx->W, height = cx->H;
    const int center = py * width + px;
    float *P = st->planes;
#define WV(i) P[4 * (size_t)(i) + 3]
    float filter[21];
    int index = 0;
    filter[index++] = WV(center);
    const int left = center - 1, leftleft = center - 3;
    const int up = center - width, upup = center - 3 * width;
    const int down = center + width, downdown = center + 3 * width;
    const int right = center + 1, rightright = center + 3;
    if (st->costs[center] < 0.001f) return;
    if (py > 0) filter[index++] = WV(up);
    if (py > 2) filter[index++] = WV(upup);
    if (py > 4) filter[index++] = WV(upup - width * 2);
    if (py < height - 1) filter[index++] = WV(down);
    if (py < height - 3) filter[index++] = WV(downdown);
    if (py < height - 5) filter[index++] = WV(downdown + width * 2);
    if (px > 0) filter[index++] = WV(left);
    if (px > 2) filter[index++] = WV(leftleft);
    if (px > 4) filter[index++] = WV(leftleft - 2);
    if (px < width - 1) filter[index++] = WV(right);
    if (px < width - 3) filter[index++] = WV(rightright);
    if (px < width - 5) filter[index++] = WV(rightright + 2);
    if (py > 0 && px < width - 2) filter[index++] = WV(up + 2);
    if (py < height - 1 && px < width - 2) filter[index++] = WV(down + 2);
    if (py > 0 && px > 1) filter[index++] = WV(up - 2);
    if (py < height - 1 && px > 1) filter[index++] = WV(down - 2);
    if (px > 0 && py > 2) filter[index++] = WV(left - width * 2);
    if (px < width - 1 && py > 2) filter[index++] = WV(right - width * 2);
    if (px > 0 && py < height - 2) filter[index++] = WV(left + width * 2);
    if (px < width - 1 && py < height - 2) filter[index++] = WV(right + width * 2);
    sort_small(filter, index);
    const int mi = index / 2;
    if (index % 2 == 0) WV(center) = (filter[mi - 1] + filter[mi]) / 2;
    else WV(center) = filter[mi];
#undef WV
}

/* rows the reference's checkerboard grid actually covers (ACMMP.cu:1525, :1331-1333) */
static inline int checker_rows(int H) { int r = 32 * (((H / 2) + 15) / 16); return r < H ? r : H; }

static int run_rows(const or_problem *pb, const or_params *pp, or_state *st, uint64_t seed,
                    int32_t n_half_sweeps, int32_t do_post, int32_t nthreads, int row0, int row1);

int or_run_patchmatch(const or_problem *pb, const or_params *pp, or_state *st,
                      uint64_t seed, int32_t n_half_sweeps, int32_t do_post, int32_t nthreads)
{
    return run_rows(pb, pp, st, seed, n_half_sweeps, do_post, nthreads, 0, pb->cams[0].height);
}

/* Bounded CPU-baseline sample and full-size parity bands: the same per-pixel work restricted to
   rows [row0, row1); rows outside keep the state they came in with. */
int or_run_band(const or_problem *pb, const or_params *pp, or_state *st, uint64_t seed,
                int32_t n_half_sweeps, int32_t nthreads, int32_t row0, int32_t row1, int32_t do_post)
{
    return run_rows(pb, pp, st, seed, n_half_sweeps, do_post, nthreads, row0, row1);
}

static int run_rows(const or_problem *pb, const or_params *pp, or_state *st, uint64_t seed,
                    int32_t n_half_sweeps, int32_t do_post, int32_t nthreads, int row0, int row1)
{
    Ctx cx = { pb, pp, pb->cams[0].width, pb->cams[0].height, pp->num_images - 1, seed };
    const int W = cx.W, H = cx.H;
    const size_t P = (size_t)W * H;
    if (pp->num_images < 2 || pp->num_images > 33) return 1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    or_rng *rng = (or_rng *)malloc(sizeof(or_rng) * P);
    float *planes2 = (float *)malloc(sizeof(float) * 4 * P);
    float *costs2 = (float *)malloc(sizeof(float) * P);
    uint32_t *sel2 = (uint32_t *)malloc(sizeof(uint32_t) * P);
    if (!rng || !planes2 || !costs2 || !sel2) { free(rng); free(planes2); free(costs2); free(sel2); return 2; }

    if (row0 < 0) row0 = 0;
    if (row1 > H) row1 = H;
    /* pixels are independent within a step: parallel over pixels, not rows, so a few-row band
       (the bench's CPU sample) still spreads over every thread */
#pragma omp parallel for schedule(dynamic, 256)
    for (long i = (long)row0 * W; i < (long)row1 * W; ++i) {
        const int y = (int)(i / W), x = (int)(i % W);
        init_pixel(&cx, st, x, y, &rng[(size_t)i]);
    }

    if (n_half_sweeps < 0) n_half_sweeps = 2 * pp->max_iterations;
    const int rows = checker_rows(H) < row1 ? checker_rows(H) : row1;
    for (int s = 0; s < n_half_sweeps; ++s) {
        const int iter = s / 2, colour = s & 1;
        memcpy(planes2, st->planes, sizeof(float) * 4 * P);
        memcpy(costs2, st->costs, sizeof(float) * P);
        memcpy(sel2, st->selected_views, sizeof(uint32_t) * P);
        or_state in = { planes2, costs2, st->pre_costs, sel2 };
        const int Wh = (W + 1) / 2;     /* pixels of this colour per row, at most */
#pragma omp parallel for schedule(dynamic, 64)
        for (long i = (long)row0 * Wh; i < (long)rows * Wh; ++i) {
            const int y = (int)(i / Wh), x = (int)(i % Wh) * 2 + ((y + colour) & 1);
            if (x < W) propagate_pixel(&cx, &in, st, &rng[(size_t)y * W + x], x, y, iter);
        }
    }

    if (do_post) {
#pragma omp parallel for schedule(static)
        for (int y = row0; y < row1; ++y)
            for (int x = 0; x < W; ++x) depth_and_normal(&cx, st, x, y);
        for (int colour = 0; colour < 2; ++colour) {
#pragma omp parallel for schedule(static)
            for (int y = row0; y < rows; ++y)
                for (int x = (y + colour) & 1; x < W; x += 2) filter_pixel(&cx, st, x, y);
        }
    }
    free(rng); free(planes2); free(costs2); free(sel2);
    return 0;
}

/* ---- JBU_cu, ACMMP.cu:1558-1616 ---- */
void or_jbu(const float *ref, int32_t W, int32_t H, const float *coarse, int32_t sw, int32_t sh,
            int32_t imagescale, float *out, int32_t nthreads)
{
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            const float scale = (float)(1.0 * (double)sw / (double)W);
            const float sigmad = 0.50f, sigmar = 25.5f;
            const int WinWidth = imagescale * imagescale + 1;
            const int nn = WinWidth / 2;
            const float o_y = (float)y * scale, o_x = (float)x * scale;
            const float refPix = tex_texel(ref, W, H, x, y);
            float total = 0.0f, nf = 0.0f;
            for (int j = -nn; j <= nn; ++j) {
                int r_y = dm_f2i_sat(o_y + (float)j);
                r_y = (r_y > 0 ? (r_y < sh ? r_y : sh - 1) : 0);
                int r_ys = y + j;
                r_ys = (r_ys > 0 ? (r_ys < H ? r_ys : H - 1) : 0);
                for (int i = -nn; i <= nn; ++i) {
                    int r_x = dm_f2i_sat(o_x + (float)i);
                    r_x = (r_x > 0 ? (r_x < sw ? r_x : sw - 1) : 0);
                    const float srcPix = tex_texel(coarse, sw, sh, r_x, r_y);
                    int r_xs = x + i;
                    r_xs = (r_xs > 0 ? (r_xs < W ? r_xs : W - 1) : 0);
                    const float nbPix = tex_texel(ref, W, H, r_xs, r_ys);
                    const float sg = spatial_gauss(o_x, o_y, (float)r_x, (float)r_y, sigmad);
                    const float rg = range_gauss(fabsf(refPix - nbPix), sigmar);
                    const float tg = sg * rg;
                    nf += tg;
                    total = fmaf(srcPix, tg, total);
                }
            }
            out[(size_t)y * W + x] = total / nf;
        }
    }
}

/* ---- unit entry points ---- */
static Ctx mkctx(const or_problem *pb, const or_params *pp)
{
    Ctx c = { pb, pp, pb->cams[0].width, pb->cams[0].height, pp->num_images - 1, 0 };
    return c;
}
float or_bilateral_ncc(const or_problem *pb, const or_params *pp, int32_t src, int32_t px, int32_t py,
                       const float plane[4])
{
    Ctx c = mkctx(pb, pp);
    f4 ph = { plane[0], plane[1], plane[2], plane[3] };
    return bilateral_ncc(&c, src, px, py, ph);
}
float or_geom_cost(const or_problem *pb, const or_params *pp, int32_t src, int32_t px, int32_t py,
                   const float plane[4])
{
    Ctx c = mkctx(pb, pp);
    f4 ph = { plane[0], plane[1], plane[2], plane[3] };
    return geom_cost(&c, src, ph, px, py);
}
float or_initial_cost(const or_problem *pb, const or_params *pp, int32_t px, int32_t py,
                      const float plane[4], uint32_t *selected)
{
    Ctx c = mkctx(pb, pp);
    f4 ph = { plane[0], plane[1], plane[2], plane[3] };
    return initial_cost(&c, px, py, ph, selected);
}
void or_pixel_to_dir(const or_camera *cam, int32_t px, int32_t py, float out[3])
{
    const f3 d = pixel_to_dir(cam, px, py);
    out[0] = d.x; out[1] = d.y; out[2] = d.z;
}
void or_project(const or_camera *cam, const float X[3], float pt[2], float *depth)
{
    f3 P = { X[0], X[1], X[2] };
    f2 p;
    project(cam, P, &p, depth);
    pt[0] = p.x; pt[1] = p.y;
}
void or_world_point(const or_camera *cam, float x, float y, float depth, float out[3])
{
    const f3 r = world_point(cam, x, y, depth);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

/* ---- fusion: SimpleFusionKernel, ACMMP.cu:1662-1814 ------------------------------------- */

/* hypotf as a fixed definition: sqrt(x*x + y*y) under the contraction rule */
static inline float fuse_hypot(float x, float y) { return sqrtf(fmaf(y, y, x * x)); }

/* tex2D<float4>(linear, unnormalised) at integer (c, r) -- no +0.5 (ACMMP.cu:1690): texels
 * (c-1, c) x (r-1, r), weights 0.5, clamped; fused fp32 lerps */
static void fuse_colour(const float *rgba, int W, int H, int c, int r, float out[4])
{
    const int x0 = c - 1 < 0 ? 0 : c - 1, x1 = c > W - 1 ? W - 1 : c;
    const int y0 = r - 1 < 0 ? 0 : r - 1, y1 = r > H - 1 ? H - 1 : r;
    for (int k = 0; k < 4; ++k) {
        const float t00 = rgba[4 * ((size_t)y0 * W + x0) + k], t10 = rgba[4 * ((size_t)y0 * W + x1) + k];
        const float t01 = rgba[4 * ((size_t)y1 * W + x0) + k], t11 = rgba[4 * ((size_t)y1 * W + x1) + k];
        const float top = fmaf(0.5f, t10 - t00, t00), bot = fmaf(0.5f, t11 - t01, t01);
        out[k] = fmaf(0.5f, bot - top, top);
    }
}

int32_t or_fuse(int32_t n, const or_camera *cams, const float *const *depths, const float *const *normals,
                const float *const *rgba, int32_t ref, int32_t n_src, const int32_t *srcs, float *out)
{
    (void)n;
    const or_camera *rc = &cams[ref];
    const int W = rc->width, H = rc->height;
    int32_t count = 0;
    for (int r = 0; r < H; ++r) {
        for (int c = 0; c < W; ++c) {
            const size_t idx = (size_t)r * W + c;
            const float ref_depth = depths[ref][idx];
            if (ref_depth <= 0.0f) continue;                                      /* :1685 */
            const f3 X = world_point(rc, (float)c, (float)r, ref_depth);
            const float *rn = &normals[ref][3 * idx];
            float rcol[4];
            fuse_colour(rgba[ref], W, H, c, r, rcol);
            float ps0 = X.x, ps1 = X.y, ps2 = X.z;
            float ns0 = rn[0], ns1 = rn[1], ns2 = rn[2];
            float cs0 = rcol[2] * 255.0f, cs1 = rcol[1] * 255.0f, cs2 = rcol[0] * 255.0f;   /* :1705-1709 */
            int num = 1;
            for (int j = 0; j < n_src; ++j) {                                    /* :1713-1772 */
                const int si = srcs[j];
                if (si < 0) continue;
                const or_camera *sc = &cams[si];
                f2 pp;
                float pd;
                project(sc, X, &pp, &pd);
                const int src_c = dm_f2i_sat(pp.x + 0.5f), src_r = dm_f2i_sat(pp.y + 0.5f);
                if (src_c < 0 || src_c >= sc->width || src_r < 0 || src_r >= sc->height) continue;
                const size_t sidx = (size_t)src_r * sc->width + src_c;
                const float sd = depths[si][sidx];
                if (sd <= 0.0f) continue;
                const f3 Xs = world_point(sc, (float)src_c, (float)src_r, sd);
                f2 q;
                float qd;
                project(rc, Xs, &q, &qd);
                const float err = fuse_hypot((float)c - q.x, (float)r - q.y);
                const float rel = fabsf(pd - sd) / sd;
                const float *sn = &normals[si][3 * sidx];
                float dp = dot3(rn[0], rn[1], rn[2], sn[0], sn[1], sn[2]);
                dp = fmaxf(-1.0f, fminf(1.0f, dp));
                const float ang = dm_acosf(dp);
                if (err < 1.0f && rel < 0.01f && ang < 0.149f) {
                    ps0 += Xs.x; ps1 += Xs.y; ps2 += Xs.z;
                    ns0 += sn[0]; ns1 += sn[1]; ns2 += sn[2];
                    float scol[4];
                    fuse_colour(rgba[si], sc->width, sc->height, src_c, src_r, scol);
                    cs0 = fmaf(scol[2], 255.0f, cs0);
                    cs1 = fmaf(scol[1], 255.0f, cs1);
                    cs2 = fmaf(scol[0], 255.0f, cs2);
                    ++num;
                }
            }
            if (num >= 3) {                                                       /* :1775-1810 */
                if (out) {
                    const float fn = (float)num;
                    float *o = out + 9 * (size_t)count;
                    o[0] = ps0 / fn; o[1] = ps1 / fn; o[2] = ps2 / fn;
                    float a0 = ns0 / fn, a1 = ns1 / fn, a2 = ns2 / fn;
                    const float len = fuse_hypot(fuse_hypot(a0, a1), a2);
                    if (len > 0.0f) { a0 /= len; a1 /= len; a2 /= len; }
                    o[3] = a0; o[4] = a1; o[5] = a2;
                    o[6] = cs0 / fn; o[7] = cs1 / fn; o[8] = cs2 / fn;
                }
                ++count;
            }
        }
    }
    return count;
}

void or_detmath_eval(int32_t fn, const float *x, const float *y, float *out, int64_t n)
{
    for (int64_t i = 0; i < n; ++i) {
        switch (fn) {
        case 0: out[i] = dm_expf(x[i]); break;
        case 1: out[i] = dm_sinf(x[i]); break;
        case 2: out[i] = dm_cosf(x[i]); break;
        case 3: out[i] = dm_asinf(x[i]); break;
        case 4: out[i] = dm_acosf(x[i]); break;
        case 5: out[i] = dm_atan2f(x[i], y[i]); break;
        case 6: out[i] = dm_rsqrtf(x[i]); break;
        case 7: out[i] = (float)dm_f2i_sat(x[i]); break;
        default: out[i] = NAN; break;
        }
    }
}

void or_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) { or_philox4x32_10(ctr, key, out); }

float or_uniform_draw(uint64_t seed, uint64_t subsequence, uint32_t n)
{
    or_rng r;
    or_rng_init(&r, seed, subsequence);
    r.n = n;
    return or_rng_uniform(&r);
}
