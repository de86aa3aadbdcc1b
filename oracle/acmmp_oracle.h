/*
 * acmmp_oracle.h -- ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the ACMMP-Spherical PatchMatch hot path
 * (/root/reference/ACMMP.cu:14-1649).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this; the product never links it.
 *
 * PARITY UNPINNED: the reference has no tests, fixtures or golden outputs
 * (SURVEY.md §4), and it cannot be built here (nvcc/CUDA/OpenCV absent; a
 * build through stand-in headers is not allowed), so this restatement is not
 * pinned to reference outputs.  It is pinned instead to (a) Random123 known-answer
 * vectors for the RNG, (b) float64 numpy accuracy checks of the elementary
 * functions, (c) an independent float64 numpy restatement of the NCC / geometry
 * functions, and (d) ground-truth depth on synthetic scenes.  See DESIGN.md §3.
 *
 * Semantics fixed where the reference is undefined or non-reproducible
 * (DESIGN.md §2.3): fix A at ACMMP.cu:1301; snapshot (Jacobi) reads inside a
 * colour half-sweep; Philox4x32-10 seeded stream instead of clock64 XORWOW;
 * clamp-to-edge texture addressing with fp32 bilinear weights; deterministic
 * elementary functions (detmath_ref.h); the contraction rule "a product whose only
 * use is one operand of a +/- is fused into it (right-most product first)".
 */
#ifndef ACMMP_ORACLE_H
#define ACMMP_ORACLE_H
#include <stdint.h>
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_PINHOLE = 0, OR_SPHERE = 11 };

/* Same layout as the reference's Camera (main.h:40-54), 120 bytes. */
typedef struct or_camera {
    int32_t model;
    float params[4];
    float R[9];
    float t[3];
    float K[9];
    int32_t width, height;
    float depth_min, depth_max;
} or_camera;

/* Same layout as the reference's PatchMatchParams (ACMMP.h:32-55), 68 bytes. */
typedef struct or_params {
    int32_t max_iterations;
    int32_t patch_size;
    int32_t num_images;
    int32_t max_image_size;
    int32_t radius_increment;
    float sigma_spatial;
    float sigma_color;
    int32_t top_k;
    float baseline;
    float depth_min;
    float depth_max;
    float disparity_min;
    float disparity_max;
    float scaled_cols;
    float scaled_rows;
    bool geom_consistency;
    bool planar_prior;
    bool multi_geometry;
    bool hierarchy;
    bool upsample;
} or_params;

typedef struct or_problem {
    int32_t num_images;                 /* ref + sources */
    const or_camera *cams;              /* num_images cameras (already rescaled) */
    const float *const *images;         /* num_images row-major images, cams[i].height x cams[i].width */
    const float *const *depths;         /* geom: num_images depth maps (may be NULL otherwise) */
    const int32_t *depth_w;
    const int32_t *depth_h;
    const float *scaled_planes;         /* hierarchy: scaled_w*scaled_h float4 */
    int32_t scaled_w, scaled_h;
    const float *prior_planes;          /* planar: P float4 */
    const uint32_t *plane_masks;        /* planar: P */
} or_problem;

typedef struct or_state {
    float *planes;                      /* P float4, in/out */
    float *costs;                       /* P, in/out */
    float *pre_costs;                   /* P, in/out (hierarchy) */
    uint32_t *selected_views;           /* P, in/out */
} or_state;

/* ACMMP::RunPatchMatch (ACMMP.cu:1506-1556).
 * n_half_sweeps < 0 -> 2*max_iterations (the reference schedule).
 * do_post = 0 skips GetDepthandNormal + the two filters (raw working state). */
int or_run_patchmatch(const or_problem *pb, const or_params *pp, or_state *st,
                      uint64_t seed, int32_t n_half_sweeps, int32_t do_post, int32_t nthreads);

/* CPU-baseline sample and full-size parity bands: init + sweeps (+ post when do_post) restricted to rows
   [row0, row1) of the same problem. */
int or_run_band(const or_problem *pb, const or_params *pp, or_state *st, uint64_t seed,
                int32_t n_half_sweeps, int32_t nthreads, int32_t row0, int32_t row1, int32_t do_post);

/* Unit entry points (T1 tests). */
float or_bilateral_ncc(const or_problem *pb, const or_params *pp, int32_t src, int32_t px, int32_t py,
                       const float plane[4]);
float or_geom_cost(const or_problem *pb, const or_params *pp, int32_t src, int32_t px, int32_t py,
                   const float plane[4]);
float or_initial_cost(const or_problem *pb, const or_params *pp, int32_t px, int32_t py,
                      const float plane[4], uint32_t *selected);
void or_pixel_to_dir(const or_camera *cam, int32_t px, int32_t py, float out[3]);
void or_project(const or_camera *cam, const float X[3], float pt[2], float *depth);
void or_world_point(const or_camera *cam, float x, float y, float depth, float out[3]);

/* JBU_cu (ACMMP.cu:1558-1616): joint bilateral upsampling of a coarse depth map. */
void or_jbu(const float *ref, int32_t W, int32_t H, const float *coarse, int32_t sw, int32_t sh,
            int32_t imagescale, float *out, int32_t nthreads);

/* SimpleFusionKernel (ACMMP.cu:1662-1814) for one reference view + RunFusionCuda's in-order
 * collection (ACMMP.cu:2064-2071).  cams: n views rescaled to their depth maps; depths[v] (H x W),
 * normals[v] (3 per pixel), rgba[v] (4 floats per pixel: the reference's colour texture, /255).
 * out: 9 floats per consistent pixel, pixel order; returns the count (out may be NULL to count). */
int32_t or_fuse(int32_t n, const or_camera *cams, const float *const *depths, const float *const *normals,
                const float *const *rgba, int32_t ref, int32_t n_src, const int32_t *srcs, float *out);

/* Per-pixel trace of the half-sweeps of the next or_run_patchmatch / or_run_band (tests only):
 * trace[center] is (over)written by every half-sweep that updates the pixel, so after a run it
 * holds the pixel's last update.  NULL disables tracing (the default). */
typedef struct or_trace {
    int32_t pos[8];                     /* picked neighbour (row-major index) per direction, -1 = flag false */
    float final_costs[8];               /* aggregated cost per direction (:1210-1228) */
    float cost_now;                     /* aggregated cost of the current plane (:1232-1244) */
    int32_t min_idx, max_idx;           /* FindMinCostIndex; FindMaxCostIndex of the prior branch or -1 */
    int32_t accepted;                   /* hypothesis left in plane_hypotheses_now: 0-7 neighbour, 8 own plane
                                           (after the prior branch), 9+k refinement candidate k */
    uint32_t temp_selected_views;
    uint32_t draws_before, draws_after; /* RNG draw counter around the pixel's update */
    uint8_t view_weights[32];           /* the 15 draws' counts per view */
} or_trace;
void or_set_trace(or_trace *trace);

/* elementary functions and RNG, exported for tests */
void or_detmath_eval(int32_t fn, const float *x, const float *y, float *out, int64_t n);
void or_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
float or_uniform_draw(uint64_t seed, uint64_t subsequence, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif
