/*
 * acmmp.h -- C ABI of the MI355X-native ACMMP-Spherical PatchMatch engine.
 *
 * Drop-in boundary for the depth/normal inference path of the reference
 * (/root/reference, contineu-ai/ACMMP-Spherical @ 2025-11-21).  The reference's only
 * caller of the hot path is ProcessProblem (main.cpp:73-210), which drives the
 * ACMMP class (ACMMP.h:57-111).  Every entry point below names the reference
 * member it replaces.  Plain C types only: pointers and sizes, no torch/HIP types.
 *
 * Threading: one context = one GPU = one host thread at a time (the reference is
 * single-threaded and not re-entrant either).  All host pointers are borrowed for
 * the duration of the call.  Errors are returned as acmmp_status codes; the C++
 * facade (acmmp-spherical_amd/host/ACMMP.hpp) maps them to the reference's
 * print-and-exit behaviour of CUDA_SAFE_CALL (ACMMP.cpp:64-72).
 */
#ifndef ACMMP_C_ABI_H
#define ACMMP_C_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACMMP_ABI_VERSION 1

/* CameraModel, main.h:35-38 */
#define ACMMP_PINHOLE 0
#define ACMMP_SPHERE 11

/* Camera, main.h:40-54 -- identical layout (120 bytes). */
typedef struct acmmp_camera {
    int32_t model;          /* ACMMP_PINHOLE or ACMMP_SPHERE */
    float params[4];        /* SPHERE: f, cx, cy, unused */
    float R[9];             /* world -> camera rotation, row-major */
    float t[3];             /* X_cam = R X_world + t */
    float K[9];             /* PINHOLE intrinsics, row-major */
    int32_t width, height;
    float depth_min, depth_max;
} acmmp_camera;

/* PatchMatchParams, ACMMP.h:32-55 -- identical layout (68 bytes). */
typedef struct acmmp_params {
    int32_t max_iterations;     /* 3; SetGeomConsistencyParams sets 2 (ACMMP.cpp:551) */
    int32_t patch_size;         /* 11 */
    int32_t num_images;         /* reference + sources, 2..33 */
    int32_t max_image_size;     /* 3200 */
    int32_t radius_increment;   /* 2 */
    float sigma_spatial;        /* 5 */
    float sigma_color;          /* 3 */
    int32_t top_k;              /* 4 */
    float baseline;             /* 0.54 (unused by the hot path) */
    float depth_min;            /* cams[0].depth_min * 0.6 (ACMMP.cpp:645) */
    float depth_max;            /* cams[0].depth_max * 1.2 (ACMMP.cpp:646) */
    float disparity_min;        /* unused by the hot path */
    float disparity_max;
    float scaled_cols;          /* hierarchy: coarse map size (ACMMP.cpp:810-811) */
    float scaled_rows;
    uint8_t geom_consistency;
    uint8_t planar_prior;
    uint8_t multi_geometry;
    uint8_t hierarchy;
    uint8_t upsample;
    uint8_t _pad[3];
} acmmp_params;

typedef enum acmmp_status {
    ACMMP_OK = 0,
    ACMMP_ERR_INVALID_ARGUMENT = 1,
    ACMMP_ERR_HIP = 2,
    ACMMP_ERR_OUT_OF_MEMORY = 3,
    ACMMP_ERR_STATE = 4,            /* call order violated (e.g. run before upload) */
    ACMMP_ERR_UNSUPPORTED = 5,      /* e.g. mixed camera models, > 32 source views */
    ACMMP_ERR_NO_DEVICE = 6,
    ACMMP_ERR_COMM = 7            /* RCCL failure */
} acmmp_status;

typedef struct acmmp_ctx acmmp_ctx;
typedef struct acmmp_image_cache acmmp_image_cache;
typedef struct acmmp_comm acmmp_comm;
typedef struct acmmp_fusion acmmp_fusion;
#define ACMMP_COMM_ID_BYTES 128

/* ACMMP::ACMMP() (ACMMP.cpp:99) + cudaSetDevice (main.cpp:77).  `device` is a HIP
 * ordinal; -1 keeps the calling thread's current device. */
acmmp_status acmmp_create(int device, acmmp_ctx **out);
/* ACMMP::~ACMMP() (ACMMP.cpp:101-143): frees every device buffer (no double free). */
void acmmp_destroy(acmmp_ctx *ctx);
const char *acmmp_status_str(acmmp_status s);
/* Message of the last error on this context (empty string if none). */
const char *acmmp_last_error(const acmmp_ctx *ctx);
int acmmp_abi_version(void);

/* Number of visible HIP devices (0 without a GPU); never fails. */
int acmmp_device_count(void);

/* Arithmetic of the NCC's per-sample projection (ComputeBilateralNCC, ACMMP.cu:456-476).
 * ACMMP_MATH_EXACT (default): the fixed IEEE definitions of DESIGN.md §2.3 -- results are
 * bit-identical to the CPU oracle.  ACMMP_MATH_FAST: what the reference's --use_fast_math build
 * (CMakeLists.txt:42) does to the same arithmetic -- hardware rsq/sqrt/rcp (<= 1 ulp), the
 * translation folded into the rotation, the asin/atan2 polynomials without special-argument paths
 * (DESIGN.md §2.4); results within the tolerances of DESIGN.md §2.4, not bit-identical.  Every new
 * context starts exact; callers choose fast explicitly.  No reference counterpart. */
enum { ACMMP_MATH_EXACT = 0, ACMMP_MATH_FAST = 1 };
acmmp_status acmmp_set_math(acmmp_ctx *ctx, int mode);
int acmmp_get_math(const acmmp_ctx *ctx);

/* The params member + Set{GeomConsistency,Hierarchy,PlanarPrior}Params
 * (ACMMP.cpp:548-565).  Copied; may be called again between runs. */
acmmp_status acmmp_set_params(acmmp_ctx *ctx, const acmmp_params *params);

/* Texture part of CudaSpaceInitialization (ACMMP.cpp:685-712): n = num_images
 * float grey images (0..255), images[i] is cams[i].height x cams[i].width,
 * row pitch `pitch_bytes[i]` (NULL -> tightly packed).  cams[0] is the reference. */
acmmp_status acmmp_upload_views(acmmp_ctx *ctx, int n, const float *const *images,
                                const size_t *pitch_bytes, const acmmp_camera *cams);

/* The same from device buffers of this context's GPU (in-memory pipeline: a view's image of one
 * scale is uploaded once and every problem of every pass that reads it copies it HBM to HBM).
 * images[i] are device pointers, otherwise as acmmp_upload_views.  No reference counterpart. */
acmmp_status acmmp_upload_views_device(acmmp_ctx *ctx, int n, const float *const *dev_images,
                                       const size_t *pitch_bytes, const acmmp_camera *cams);

/* Device-side cache of prepared source images (padded fp32 + binary16 copies), shared by the contexts
 * of one GPU.  The reference re-reads, re-converts and re-uploads every image of every problem
 * (InuputInitialization ACMMP.cpp:567-643 + CudaSpaceInitialization :685-712); a pipeline that keys its
 * (view, scale) images prepares each once.  budget_bytes: soft limit (least recently used entries no
 * current problem uses are freed beyond it), 0 = none.  Destroy after every context that used it. */
acmmp_status acmmp_image_cache_create(int device, size_t budget_bytes, acmmp_image_cache **out);
void acmmp_image_cache_destroy(acmmp_image_cache *cache);
/* out = {hits, misses, bytes held, entries, evictions} */
acmmp_status acmmp_image_cache_stats(acmmp_image_cache *cache, unsigned long long out[5]);

/* acmmp_upload_views (device_src = 0) / acmmp_upload_views_device (device_src = 1) with a content key
 * per view: keys[i] != 0 names the exact pixels of images[i] (the caller's promise -- e.g. view id and
 * scale); a view whose key and size are already in `cache` is not copied or converted again.  keys[i]
 * = 0 or cache = NULL: prepared privately, as acmmp_upload_views does.  No reference counterpart. */
acmmp_status acmmp_upload_views_keyed(acmmp_ctx *ctx, acmmp_image_cache *cache, int n, const uint64_t *keys,
                                      const float *const *images, const size_t *pitch_bytes,
                                      const acmmp_camera *cams, int device_src);

/* Geometric-consistency depth textures (ACMMP.cpp:653-678, 726-751): n depth maps,
 * depths[i] is h[i] x w[i] row-major (index 0 = reference, as the reference). */
acmmp_status acmmp_upload_depths(acmmp_ctx *ctx, int n, const float *const *depths,
                                 const int *w, const int *h);

/* The same from device buffers of this context's GPU (in-memory pipeline: the depth maps a geom
 * pass reads stay in HBM instead of the reference's depths*.dmb round trip). */
acmmp_status acmmp_upload_depths_device(acmmp_ctx *ctx, int n, const float *const *dev_depths,
                                        const int *w, const int *h);

/* The last run's depth map (.w of plane_hypotheses, ProcessProblem main.cpp:103-111) copied into a
 * device buffer of P floats on this context's GPU. */
acmmp_status acmmp_export_depth(acmmp_ctx *ctx, float *dev_dst);

/* Reference-view state for geom / hierarchy / planar reuse passes
 * (ACMMP.cpp:772-785, 833-843): planes = P float4 (nx, ny, nz, w) row-major,
 * costs = P floats (may be NULL -> unchanged).  P = cams[0].width*height. */
acmmp_status acmmp_set_state(acmmp_ctx *ctx, const float *planes, const float *costs);

/* The last run's planes (P float4) and costs (P floats) copied into device buffers of this context's GPU
 * (either may be NULL), and acmmp_set_state from such buffers: a geom pass restarts from the previous
 * pass's state without the host round trip of ProcessProblem's .dmb reload (ACMMP.cpp:772-785). */
acmmp_status acmmp_export_state(acmmp_ctx *ctx, float *dev_planes, float *dev_costs);
acmmp_status acmmp_set_state_device(acmmp_ctx *ctx, const float *dev_planes, const float *dev_costs);

/* Hierarchy coarse state scaled_plane_hypotheses (ACMMP.cpp:804-842):
 * sw*sh float4 row-major. */
acmmp_status acmmp_set_scaled_state(acmmp_ctx *ctx, const float *planes, int sw, int sh);

/* CudaPlanarPriorInitialization (ACMMP.cpp:847-867) after the host has expanded
 * labels: prior = P float4 plane params, mask = P labels (0 = no prior). */
acmmp_status acmmp_set_planar_prior(acmmp_ctx *ctx, const float *prior_planes, const uint32_t *masks);

/* ACMMP::RunPatchMatch (ACMMP.cu:1506-1556) minus the final D2H copy:
 * init, max_iterations x (black, red), GetDepthandNormal, black/red filter.
 * `seed` replaces curand_init(clock64(), ...) (ACMMP.cu:684).  Synchronous on
 * return, like the reference.  Results stay resident in HBM until downloaded. */
acmmp_status acmmp_run_patchmatch(acmmp_ctx *ctx, uint64_t seed);

/* Same with the schedule exposed (tests / profiling): n_half_sweeps < 0 means
 * 2*max_iterations; do_post = 0 leaves the raw working state (camera-frame
 * normal, w = plane distance) instead of (world normal, depth). */
acmmp_status acmmp_run_patchmatch_ex(acmmp_ctx *ctx, uint64_t seed, int n_half_sweeps, int do_post);

/* The D2H part of RunPatchMatch (ACMMP.cu:1553-1554) + GetPlaneHypothesis/GetCost
 * (ACMMP.cpp:884-892) in bulk: caller-allocated P float4 / P floats (either may be NULL). */
acmmp_status acmmp_download(acmmp_ctx *ctx, float *planes, float *costs);
/* Extra state readback for tests: selected_views bitmasks and pre_costs (either may be NULL). */
acmmp_status acmmp_download_aux(acmmp_ctx *ctx, uint32_t *selected_views, float *pre_costs);

/* Device-resident outputs (for in-process consumers such as an RCCL depth exchange):
 * returns device pointers to the row-major planes (float4[P]) and costs (float[P]). */
acmmp_status acmmp_device_outputs(acmmp_ctx *ctx, void **planes, void **costs);

/* Wait for all work of this context's device (hipDeviceSynchronize). */
acmmp_status acmmp_synchronize(acmmp_ctx *ctx);

/* Per-stage device time of the last run, measured with HIP events on the stream
 * the kernels run on: [init, propagation (all half-sweeps), post]. */
acmmp_status acmmp_last_timing(const acmmp_ctx *ctx, float ms[3]);

/* Per-kernel device time of the last run's half-sweeps (HIP events around the launches, on the
 * kernels' stream): summed ms and launch count for [k_eval_nb, k_select, k_eval_ref, k_finish]
 * (the stages one CheckerboardPropagation half-sweep is split into).  The k_eval_ref
 * bucket includes its tail launch (k_eval_ref_tail); the neighbour pick (k_pick) runs before the
 * k_eval_nb bucket opens and is in the propagation stage time only.  Only the k_eval_nb bucket is
 * timed unless ACMMP_KERNEL_TIMING=all was set in the environment for the run (each event record
 * idles the GPU a few microseconds); an untimed bucket reports 0 ms over 0 launches. */
acmmp_status acmmp_last_kernel_timing(const acmmp_ctx *ctx, float ms[4], int launches[4]);

/* Work accounting of the last run's k_eval_nb launches: pixels whose NCCs were evaluated, and all
 * pixels processed.  SPHERE pixels whose patch weight sum is below 1e-6 have every cost = 2.0
 * (ACMMP.cu:501-503) and are short-circuited; the roofline counts only evaluated pixels. */
acmmp_status acmmp_last_work(const acmmp_ctx *ctx, unsigned long long *evaluated, unsigned long long *total);

/* Host wall-clock breakdown of the last acmmp_set_planar_prior_from_state / _from_maps call, in ms:
 * [support points (device kernel + copy back; 0 for _from_maps, whose host scan is in the next entry),
 * Delaunay triangulation (host), the rest of the host half (labelled triangles, plane fits, step and trig
 * tables), device half (staging and enqueueing the table upload and the raster and mask kernels on the
 * context's stream -- they complete before its next run; see acmmp_set_planar_prior_from_maps)].
 * No reference counterpart (profiling of main.cpp:113-187's block). */
acmmp_status acmmp_last_planar_timing(const acmmp_ctx *ctx, float ms[4]);

/* Bytes per source texel the NCC fetches read: 2 when every texel of the uploaded views is exactly
 * a binary16 number (8-bit images are) and the engine keeps a binary16 copy of them, 4 for the fp32
 * images, 0 before acmmp_upload_views.  Results are identical either way; the
 * environment variable ACMMP_TEX16=0 at upload time forces 4.  No reference counterpart. */
int acmmp_texel_bytes(const acmmp_ctx *ctx);

/* ---- row-band split of one reference view (SURVEY.md §8e latency mode; no reference counterpart:
 * the reference runs a view on one GPU) -------------------------------------------------------------
 * Several contexts (one per GPU) holding the same uploaded problem each run RunPatchMatch on the image
 * rows [row0, row1) of one view; after every half-sweep each exchanges the updated colour's rows within
 * ACMMP_BAND_HALO of its band with the neighbouring bands.  Each band's output rows are bit-identical to
 * a whole-view acmmp_run_patchmatch with the same seed.  Bands must span >= ACMMP_BAND_HALO rows. */
#define ACMMP_BAND_HALO 23

/* RandomInitialization of the band +- halo (the same per-pixel values every band computes). */
acmmp_status acmmp_band_begin(acmmp_ctx *ctx, uint64_t seed, int row0, int row1);
/* The next half-sweep (black, red, black, ...) on the band's rows; *colour = the colour updated. */
acmmp_status acmmp_band_sweep(acmmp_ctx *ctx, int *colour);
/* Half-sweeps of the band run still to do (0 when none is in progress). */
int acmmp_band_sweeps_left(const acmmp_ctx *ctx);
/* Row ranges [a, b) of the halo exchange after a half-sweep: send to the band above, receive from it,
 * send to the band below, receive from it (empty at the image edges).  A band's "send down" range is
 * the next band's "receive from above" range and vice versa. */
acmmp_status acmmp_band_halo_ranges(const acmmp_ctx *ctx, int ranges[8]);
/* In-process exchange: copy rows [row_a, row_b) of `colour`'s current plane / cost / selected-view
 * state from src to dst (same or peer device; waits for src's stream). */
acmmp_status acmmp_band_copy_rows(acmmp_ctx *dst, acmmp_ctx *src, int colour, int row_a, int row_b);
/* Host transport of the same exchange (ranks without a device-to-device path, e.g. a gloo or MPI run):
 * rows [row_a, row_b) of `colour`'s current state to / from host buffers of (row_b - row_a) * ceil(W / 2)
 * colour-grid pixels -- planes 4 floats, costs 1 float, selected-view masks 1 uint32 each.  get waits for the
 * context's half-sweep; set is complete on return. */
acmmp_status acmmp_band_get_rows(acmmp_ctx *ctx, int colour, int row_a, int row_b, float *planes, float *costs,
                                 uint32_t *selected_views);
acmmp_status acmmp_band_set_rows(acmmp_ctx *ctx, int colour, int row_a, int row_b, const float *planes,
                                 const float *costs, const uint32_t *selected_views);
/* GetDepthandNormal + the two filters on band +- 10 / 5 rows; synchronous.  Rows [row0, row1) of the
 * row-major outputs (acmmp_download / acmmp_device_outputs) are then final. */
acmmp_status acmmp_band_end(acmmp_ctx *ctx, int do_post);

/* ---- device buffers and the multi-GPU communicator (no reference counterpart:
 * the reference is single-GPU and exchanges depth maps through dmb files) ------------------- */

/* Plain device memory on `device` (pipeline depth store); kind: 0 = H2D, 1 = D2H, 2 = D2D. */
acmmp_status acmmp_device_alloc(int device, size_t bytes, void **ptr);
acmmp_status acmmp_device_free(int device, void *ptr);
acmmp_status acmmp_memcpy(int device, void *dst, const void *src, size_t bytes, int kind);

/* 64-bit checksum of `bytes` (a multiple of 4) of device memory on `device`: the sum mod 2^64 over its
 * 32-bit words w_i of splitmix64's finaliser applied to (i << 32) | w_i (position and value both enter).
 * The pipeline's depth exchange compares every rank's checksum of each broadcast map
 * (acmmp/pipeline.py RcclExchange); acmmp.capi.checksum_host is the same function on host arrays. */
acmmp_status acmmp_device_checksum(int device, const void *ptr, size_t bytes, uint64_t *out);

/* Diagnostics for the performance record (bench.py `device`, `clock`); no reference counterpart.
 * acmmp_device_identity: the device's PCI bus id ("dddd:bb:dd.f") and its 16-byte UUID.
 * acmmp_clock_probe: the shader clock the device holds under a VALU-dense load on random operands
 * (MI355X_MICROARCH.md "DVFS give-back"): ~5 ms launches back to back for warm_ms, then one launch whose
 * workgroups read the shader-cycle and 100 MHz counters around their loop.  out = {median GHz over the
 * workgroups, min, max, ms of that launch}.  Synchronous; uses the device's null stream. */
acmmp_status acmmp_device_identity(int device, char *pci_bus_id, int len, uint8_t uuid[16]);
acmmp_status acmmp_clock_probe(int device, float warm_ms, double out[4]);

/* RCCL communicator, one rank per process / GPU.  Rank 0 creates the id and hands the 128 bytes
 * to the other ranks out of band (the Python driver uses the launcher's TCP store). */
acmmp_status acmmp_comm_unique_id(uint8_t id[ACMMP_COMM_ID_BYTES]);
acmmp_status acmmp_comm_create(int device, const uint8_t id[ACMMP_COMM_ID_BYTES], int nranks, int rank,
                               acmmp_comm **out);
void acmmp_comm_destroy(acmmp_comm *comm);

/* Orders every collective queued on comm after this call behind all the work ctx (a context of the
 * same GPU) has queued so far -- e.g. acmmp_export_depth into a buffer about to be broadcast: an event
 * recorded on the engine stream that the communicator's stream waits on, no host wait.  No reference
 * counterpart (the reference hands depth maps over through depths*.dmb files, ACMMP.cpp:653-678). */
acmmp_status acmmp_comm_after(acmmp_comm *comm, acmmp_ctx *ctx);

/* Grouped in-place broadcasts: device buffer bufs[i] (bytes[i]) from rank roots[i] to every rank.
 * Synchronous on return. */
acmmp_status acmmp_comm_broadcast(acmmp_comm *comm, int n, void *const *bufs, const size_t *bytes,
                                  const int *roots);

/* Element-wise max over ranks of n host doubles (timing reductions); synchronous. */
acmmp_status acmmp_comm_allreduce_max(acmmp_comm *comm, double *vals, int n);

/* Halo exchange of a band run over RCCL: after acmmp_band_sweep updated `colour`, grouped ncclSend /
 * ncclRecv of the acmmp_band_halo_ranges rows with rank_up / rank_down (-1 = none), queued on the
 * context's stream (ordered with its kernels, no host wait). */
acmmp_status acmmp_comm_band_exchange(acmmp_comm *comm, acmmp_ctx *ctx, int colour, int rank_up, int rank_down);

/* A whole band run: begin, every half-sweep followed by the RCCL halo exchange, end.  comm may be
 * NULL for a single band covering the view.  Synchronous on return. */
acmmp_status acmmp_run_patchmatch_band(acmmp_ctx *ctx, acmmp_comm *comm, uint64_t seed, int row0, int row1,
                                       int rank_up, int rank_down);

/* ---- GPU depth-map fusion (RunFusionCuda + SimpleFusionKernel, ACMMP.cu:1662-2105) -------------
 * One object per fusion run.  cams[i] is view i's camera already rescaled to its depth map
 * (RescaleImageAndCamera, ACMMP.cpp:213-246).  set_view uploads what the reference puts in textures:
 * the depth map (H x W), world-frame normals (3 floats per pixel, normals.dmb) and the colour image
 * rescaled to the depth size (3 bytes per pixel, OpenCV BGR order).  run fuses reference view `ref`
 * against src_views (indices into the set, -1 = missing, at most 32) and returns the consistent
 * points in pixel order, 9 floats each: x y z nx ny nz c0 c1 c2 (colour slots as the kernel stores them,
 * ACMMP.cu:1706-1708; StoreColorPlyFileBinaryPointCloud writes c2, c1, c0 as red, green, blue).
 * When `cap` is too small *n_points holds the count and ACMMP_ERR_INVALID_ARGUMENT is returned. */
acmmp_status acmmp_fusion_create(int device, int n_views, const acmmp_camera *cams, acmmp_fusion **out);
acmmp_status acmmp_fusion_set_view(acmmp_fusion *f, int view, const float *depth, const float *normals,
                                   const uint8_t *bgr);
acmmp_status acmmp_fusion_run(acmmp_fusion *f, int ref, int n_src, const int *src_views, float *points, int cap,
                              int *n_points);
const char *acmmp_fusion_last_error(const acmmp_fusion *f);
void acmmp_fusion_destroy(acmmp_fusion *f);

/* ---- planar-prior host side (no GPU; ACMMP.cpp:904-1011, main.cpp:113-181) ---------------
 * Host restatements of the reference's planar-prior helpers, so a caller can run ProcessProblem's
 * planar pass without OpenCV.  Delaunay ties / triangle order differ from cv::Subdiv2D
 * (parity unpinned).  Output arrays are caller-allocated; when `cap` is too small
 * the call returns ACMMP_ERR_INVALID_ARGUMENT with the required count in *n_out / *n_tri. */

/* ACMMP::GetSupportPoints (ACMMP.cpp:904-930): per 5x5 tile the min-cost pixel if cost < 0.1;
 * xy = (x, y) pairs in the reference's order (tile columns outer, tile rows inner). */
acmmp_status acmmp_support_points(const float *costs, int W, int H, int *xy, int cap, int *n_out);

/* ACMMP::DelaunayTriangulation (ACMMP.cpp:932-955): triangles as 6 ints (x1 y1 x2 y2 x3 y3). */
acmmp_status acmmp_delaunay(const int *xy, int n, int W, int H, int *tri_xy, int cap, int *n_tri);

/* ACMMP::GetPriorPlaneParams (ACMMP.cpp:957-989): plane (n, w), |n| = 1, w >= 0, through the
 * triangle's three reference-camera points at `depths` (W x H). */
acmmp_status acmmp_prior_plane_params(const acmmp_camera *cam0, const float *depths, int W, int H,
                                      const int tri_xy[6], float plane[4]);

/* ACMMP::GetDepthFromPlaneParam (ACMMP.cpp:991-1011). */
float acmmp_depth_from_plane_param(const acmmp_camera *cam0, const float plane[4], int x, int y);

/* The planar block of ProcessProblem (main.cpp:113-181) + CudaPlanarPriorInitialization's
 * expansion (ACMMP.cpp:851-861): support points, Delaunay, rasterised triangle labels, per-triangle
 * planes, prior-depth range mask -> per-pixel prior planes (float4[P]) and labels (u32[P]) ready for
 * acmmp_set_planar_prior.  depths/costs: the first RunPatchMatch's output. */
acmmp_status acmmp_planar_prior_host(const acmmp_camera *cam0, const float *depths, const float *costs, int W,
                                     int H, float depth_min, float depth_max, float *prior_planes,
                                     uint32_t *masks, int *n_triangles);

/* The same planar block with its per-pixel work on this context's GPU, straight into the context's
 * planar-prior state: support points, Delaunay and the per-triangle planes on the host (depths/costs:
 * the first RunPatchMatch's output, W x H of the uploaded reference view), the triangle
 * rasterisation (main.cpp:153-159), the prior-depth range mask (main.cpp:168-180) and the per-pixel
 * expansion (ACMMP.cpp:855-862) on the device.  Equivalent to acmmp_planar_prior_host followed by
 * acmmp_set_planar_prior, bit for bit (tests/test_gpu_parity.py), without the host raster and the
 * 20 B/pixel upload.  No reference counterpart. */
acmmp_status acmmp_set_planar_prior_from_maps(acmmp_ctx *ctx, const float *depths, const float *costs,
                                              float depth_min, float depth_max, int *n_triangles);
/* The same planar block from the context's own last RunPatchMatch output in HBM (main.cpp:113-181 runs
 * it on the first run's depths and costs): GetSupportPoints (ACMMP.cpp:904-929) on the device, only the
 * support points (and their depths) to the host for the Delaunay triangulation and the per-triangle planes,
 * then the raster / mask / expansion of acmmp_set_planar_prior_from_maps.  Equal to
 * acmmp_set_planar_prior_from_maps on the downloaded maps, bit for bit (tests/test_gpu_planar_state.py);
 * no full-map download.  Both calls return once the raster and mask kernels are enqueued on the context's
 * stream (its next RunPatchMatch runs after them; acmmp_download_planar_prior waits for them). */
acmmp_status acmmp_set_planar_prior_from_state(acmmp_ctx *ctx, float depth_min, float depth_max, int *n_triangles);
/* Test hook: the planar-prior state of the context (P float4 planes, P labels; either may be NULL). */
acmmp_status acmmp_download_planar_prior(acmmp_ctx *ctx, float *prior_planes, uint32_t *masks);

/* RunJBU / JBU::CudaRun (ACMMP.cpp:1071-1122, ACMMP.cu:1558-1649): joint bilateral
 * upsampling of `coarse` (sw x sh) guided by `ref` (W x H).  imagescale as the
 * reference computes it: max(H / sh, W / sw) (integer division). */
acmmp_status acmmp_jbu(acmmp_ctx *ctx, const float *ref, int W, int H, const float *coarse, int sw, int sh,
                       int imagescale, float *out);

/* ---- test hooks: evaluate the device cost functions on arbitrary inputs ---- */
/* costs[k*(num_images-1) + v] = ComputeBilateralNCC (ACMMP.cu:405-516) of plane k at
 * pixel (px[k], py[k]) against source v+1. */
acmmp_status acmmp_debug_ncc(acmmp_ctx *ctx, int n, const int *px, const int *py, const float *planes,
                             float *costs);
/* costs[(k*8 + h)*(num_images-1) + v] = ComputeBilateralNCC (ACMMP.cu:405-516) of plane
 * planes[k*8 + h] at pixel (px[k], py[k]) against source v+1, evaluated by k_eval_nb's own NCC
 * code (the propagation kernel of CheckerboardPropagation, ACMMP.cu:1146-1233): in the fast math
 * mode on SPHERE views whose 6x6 patch spans at most 5 pixels of 2 pi / 2000 rad (patch_size 11,
 * radius_increment 2: from 2000x1000 up; patch_size 21 / increment 4: from 4000x2000 up), with its
 * interpolated sample coordinates and their deferred per-sample fallbacks. */
acmmp_status acmmp_debug_ncc_nb(acmmp_ctx *ctx, int n, const int *px, const int *py, const float *planes,
                                float *costs);
/* costs[(k*5 + h)*(num_images-1) + v]: the same NCC of plane planes[k*5 + h] at pixel (px[k], py[k]) as
 * PlaneHypothesisRefinement (ACMMP.cu:797-936) evaluates its 5 candidates -- k_eval_ref's staging and NCC
 * instance, which in the fast math mode interpolates SPHERE sample coordinates above 4 source views (the
 * size gate of acmmp_debug_ncc_nb); the views whose interpolation falls back are queued as k_eval_ref queues
 * them and recomputed with every sample projected by the per-entry code of k_nb_fix<1, true>, the
 * production path of those fallbacks. */
acmmp_status acmmp_debug_ncc_ref(acmmp_ctx *ctx, int n, const int *px, const int *py, const float *planes,
                                 float *costs);
/* out[k*(num_images-1) + v] = ComputeGeomConsistencyCost (ACMMP.cu:646-671). */
acmmp_status acmmp_debug_geom(acmmp_ctx *ctx, int n, const int *px, const int *py, const float *planes,
                              float *out);

#ifdef __cplusplus
}
#endif
#endif
