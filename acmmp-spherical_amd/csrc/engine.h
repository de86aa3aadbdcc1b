// engine.h -- internal device-side layout of the PatchMatch engine (not part of the ABI).
//
// HBM layout:
//  * source/reference images: one allocation, each view padded by one replicated
//    texel on every side so a bilinear footprint is always two 8-byte row pairs;
//  * reference ray table `dirs`: float4 per pixel of the reference view, padded by
//    the patch radius (PixelToDir, ACMMP.cu:119-134, evaluated once per view
//    instead of per sample);
//  * SPHERE rays are separable: per-row (sin, cos) of latitude and per-column (sin, cos)
//    of longitude (a few KB, cache resident) give PixelToDir's exact bits with two
//    multiplies; the bilateral spatial term per (row, sample) is a small table too, and
//    each lane keeps its pixel's 36 bilateral weights in LDS for the whole launch;
//  * working state colour-split (black = (x+y) even, red = odd), each colour
//    row-major over (H, ceil(W/2)); planes and costs double-buffered per colour so
//    a half-sweep reads the kernel-entry snapshot of its own colour;
//  * persistent state (what the reference keeps in plane_hypotheses_cuda /
//    costs_cuda between runs) row-major.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "acmmp.h"

namespace acmmp {

constexpr int kPinhole = 0;
constexpr int kSphere = 11;
constexpr int kMaxViews = 32;       // cost_vector[32], uint32 view bitmask (ACMMP.cu:522,1153)
constexpr int kNbPix = 32;          // k_eval_nb: pixels per 256-lane block (8 lanes each)
constexpr int kNbFixRegions = 256;  // the queue's regions, one counter each (block % regions)
constexpr int kRefLanes = 5;        // k_eval_ref: refinement candidates (ACMMP.cu:870)
constexpr int kRefPix = 51;         // k_eval_ref: pixels per 256-lane block (255 lanes used)
constexpr int kRefSlots = kRefPix * kRefLanes;  // survivor slots per k_eval_ref block
constexpr unsigned kStatusFixOverflow = 1u;   // KParams::status: k_nb_fix found a region's queue overfull

struct DevCam {
    // The fields the fast-math sample loop reads come first, contiguous and 16-byte aligned, so each
    // view's constants arrive in a few wide scalar loads (s_load_dwordx16 + x4 + x2 per sample and
    // view instead of nine narrow ones; r02 A/B profiles/r02_cam_layout_ab.txt: k_eval_nb -1.3%).
    // The fast projection works in the reference camera's frame: a source point is FR q + Ft for the
    // camera-frame point q = depth * ray of the reference pixel, FR = K R R0^T and Ft = K (R C0 + t)
    // (K = identity for SPHERE; R0, C0: the problem's reference camera, rounded once from doubles).
    float FRxy[6];                  // FR rows 0 and 1 interleaved: FR00 FR10 FR01 FR11 FR02 FR12
    float FRz[3];                   // FR row 2
    float Ft[3];
    float fkx, fky;                 // SPHERE: W / (2 pi), H / pi (fast mode)
    float cx, cy;                   // SPHERE params[1], params[2]
    // row-pair binary16 copy of the padded image (word (X, Y) = (t(X, Y), t(X, Y + 1))), present when
    // every texel of every view is exactly representable (8-bit images are): one 8-byte load per
    // bilinear footprint, same values
    const uint16_t* img16_base;
    int img16_bytes;
    float invW;                     // 1/W             (SPHERE longitude wrap)
    float Wf;
    float Hm1f;                     // H - 1 as float (SPHERE row clamp)
    int Wm1;                        // W - 1 (texel clamp)
    int pitch4;                     // bytes per padded row
    float Hf;                       // H as float (pinhole in-image test)
    int Hm1;                        // H - 1 (texel clamp)
    // the rest
    int model, W, H, img_pitch;     // img_pitch: floats per padded row (W + 2)
    float R[9];
    float t[3];
    float K[9];
    float inv_fx, inv_fy;           // 1/K[0], 1/K[4]  (pinhole world point)
    float C[3];                     // camera centre -(R^T t), computed like ACMMP.cu:592-594
    long long dep_off;              // float offset of the geom depth map (row-major)
    int dep_w, dep_h;
    int img_bytes;                  // bytes of the padded image (buffer descriptor range)
    const float* img_base;          // device address of padded texel (-1,-1) (buffer descriptor base)
};

// Per-pixel state handed from k_select to k_eval_ref / k_finish (80 bytes).
struct PixState {
    float4 plane_now;               // hypothesis entering PlaneHypothesisRefinement
    float4 cur_plane;               // plane_hypotheses[center] as of ACMMP.cu:1299
    uint4 vw;                       // view weights, 4-bit counts packed 8 per word
    float cost_now, depth_now, cur_cost, restricted_cost;
    uint32_t cur_sel, flags;        // flags: 1 = prior restricted, 2 = refinement runs
    float weight_norm;
    uint32_t src;                   // hypothesis ids of plane_now (bits 0-7) and cur_plane (8-15):
                                    // 0-7 neighbour direction, 8 current plane, 9+k candidate k
};

struct KParams {
    int model;                      // kPinhole / kSphere, uniform over all views
    int tex16;                      // 1: NCC fetches read the binary16 images (DevCam::img16_base)
    int fast;                       // 1: fast-math NCC sample projection (acmmp_set_math)
    int W, H, Wh, N, V;             // ref size, colour row width ceil(W/2), images, source views
    int R, inc, nside, S;           // patch radius, radius_increment, offsets per axis, samples
    int interp;                     // fast SPHERE k_eval_nb interpolates sample coordinates
    int homog;                      // fast pinhole staged chunks: homogeneous sample points
    float spread_max;               // interpolation fallback threshold, source pixels (ACMMP_SPREAD_MAX, 256)
    int rows;                       // rows the reference's checkerboard grid covers
    // row ranges (full image by default; a row band in the split latency mode, acmmp_band_*):
    int row_lo, row_hi;             // colour-grid rows the half-sweep kernels update, within [0, rows)
    int init_lo, init_hi;           // rows k_init initialises, within [0, H)
    int merge_lo, merge_hi;         // rows k_merge writes row-major, within [0, H)
    int filt_lo[2], filt_hi[2];     // rows k_filter updates per colour, within [0, rows)
    int dpitch;                     // dir table pitch (W + 2R)
    float depth_min, depth_max, sigma_spatial, sigma_color;
    int top_k;
    int geom, planar, hier, upsample;
    float scaled_cols, scaled_rows;
    int sw, sh;
    uint32_t seed_lo, seed_hi;
    const DevCam* cams;
    const float* dep;
    const float4* dirs;             // PINHOLE ray table, (W+2R) x (H+2R)
    const float2* sph_row;          // SPHERE (sin, cos) latitude, rows -R .. H+R-1
    const float2* sph_col;          // SPHERE (sin, cos) longitude, cols -R .. W+R-1
    const float* spatial;           // [(SPHERE ? H : 1)][S]: -dist / (2 sigma_s^2) (ACMMP.cu:398-403)
    float color_den;                // 2 * sigma_color^2
    float4* planes_rm;              // persistent row-major state
    float* w_rm;                    // planes_rm's .w (depth) as its own array: k_merge -> k_filter's taps (post only)
    float* costs_rm;
    float* pre_rm;
    uint32_t* sel_rm;
    const float4* scaled;           // hierarchy coarse planes (sw x sh)
    const float4* prior;            // planar prior planes (P)
    const uint32_t* mask;           // planar prior labels (P)
    float4* plane_cs[2];            // working state, current buffer per colour
    float* cost_cs[2];
    uint32_t* sel_cs[2];
    uint32_t* rng_cs[2];            // Philox draw counter per pixel
    // half-sweep scratch slab (one colour at a time)
    float* hyp_cost;                // [8][V][Pc] cost vectors of the 8 neighbour hypotheses
    float* cvec[2];                 // per colour [V][Pc]: NCC cost vector of the pixel's current plane
                                    // (NaN = view not evaluated for it yet)
    float* cand_vcost;              // [5][V][Pc] refinement candidates' cost vectors (NaN = not evaluated)
    int* nbpos;                     // [8][Pc] picked neighbour (x | y << 16) or -1
    float4* cand;                   // [5][Pc] refinement candidate planes
    float* cand_dep;                // [5][Pc] their depths (prior term, ACMMP.cu:912)
    float* cand_cost;               // [5][Pc] their aggregated costs
    PixState* pst;                  // [Pc]
    unsigned long long* work;       // [256] k_eval_nb pixels with NCC work (SPHERE patch sum >= 1e-6), per block % 256
    uint32_t nb_views;              // k_eval_nb: the source views this launch evaluates (all, or a chunk of them)
    int nb_chunk;                   // views per k_eval_nb launch (nb_view_chunk)
    int nb_tile;                    // k_eval_nb blocks as 8 x 4 tiles of the colour grid (nb_tile_order)
    int nb_count_work;              // k_eval_nb: this launch adds to `work` (the first launch of a half-sweep)
    long long Pc;                   // H * Wh
    // split refinement: k_eval_ref evaluates views [0, ref_split) of every candidate,
    // drops the ones whose partial aggregate already cannot beat cost_now, and queues the rest
    // (ci * 8 + candidate) for k_eval_ref_tail, which adds views [ref_split, V).  0 = no split.
    int ref_split;
    uint32_t* surv;                 // queued candidates: kRefSlots (255) slots per k_eval_ref block
    unsigned* surv_count;           // [k_eval_ref blocks] slots used (zeroed before each k_eval_ref)
    unsigned* surv_pre;             // [k_eval_ref blocks + 1] their exclusive prefix (k_tail_scan)
    uint32_t* surv_dense;           // the survivors in block order (k_tail_compact)
    float4* psum;                   // [Pc] (patch sum w, sum w r, sum w r^2, centre texel) for the tail
    // k_eval_nb's deferred interpolation fallbacks (ncc_chunk, k_nb_fix): pixel << 8 | hypothesis << 5 |
    // view; null = none (no interpolation, or ACMMP_SPREAD_MAX off)
    uint32_t* nbfix;                // kNbFixRegions regions of nbfix_cap entries (every entry a launch can queue)
    unsigned* nbfix_count;          // [kNbFixRegions]
    unsigned nbfix_cap;             // entries per region
    // k_eval_ref's interpolated instance (SPHERE V > 4): per queued candidate, its selected views of
    // [0, ref_split) whose interpolation fell back -- k_eval_ref_tail recomputes them and restarts the chain
    uint32_t* cand_rough;           // [5][Pc]
    unsigned* status;               // run status bits (kStatus*), zeroed per run, checked after it
};

// Per-half-sweep output buffers of the colour being updated.
// One view of the fusion set (device pointers): depth (W x H), normals (3 floats per pixel, world
// frame as normals.dmb holds them), colour as the reference's float RGBA texture (4 per pixel, /255).
struct FuseView {
    const float* depth;
    const float* normal;
    const float* rgba;
    int W, H;
};

struct SweepOut {
    float4* plane;
    float* cost;
};

// Host-side launchers (kernels.hip).
hipError_t launch_ray_tables(const KParams& kp, float4* dirs, float2* sph_row, float2* sph_col, hipStream_t s);
hipError_t launch_spatial_table(const KParams& kp, float* spatial, hipStream_t s);
hipError_t launch_init(const KParams& kp, hipStream_t s);
// ev: null, or 5 events recorded around the 4 kernels of the half-sweep (per-kernel timing); all_marks false
// records ev[0] and ev[1] only (the k_eval_nb bucket): each event record in the stream costs ~6 us of idle GPU
hipError_t launch_propagate(const KParams& kp, int colour, int iter, SweepOut out, hipStream_t s,
                            hipEvent_t* ev = nullptr, bool all_marks = true);
hipError_t launch_post(const KParams& kp, int do_post, hipStream_t s);
// Reference Camera -> device camera (derived constants computed as DESIGN.md §2.3 says), capi.cpp.
DevCam make_devcam(const acmmp_camera& cam);
void set_relative_frame(DevCam& d, const acmmp_camera& ref, const acmmp_camera& cam);   // DevCam::FR / Ft
// Current working-state buffers of one colour of a band run (capi.cpp; comm.cpp exchanges their rows).
struct BandBuffers {
    float4* plane;
    float* cost;
    uint32_t* sel;
    int Wh;
    hipStream_t stream;
    int device;
};
acmmp_status band_buffers(acmmp_ctx* c, int colour, BandBuffers* out);
// The context's device and engine stream (every kernel and copy of the context is queued there).
acmmp_status engine_stream(acmmp_ctx* c, int* device, hipStream_t* stream);

// SimpleFusionKernel (ACMMP.cu:1662-1814) for reference view `ref` + compaction in pixel order:
// out_dense/flags are P-sized scratch, block_counts ceil(P/256) ints.
hipError_t launch_fuse(int model, const DevCam* cams, const FuseView* views, int ref, int W, int H, const int* srcs,
                       int n_src, float* out_dense, int* flags, int* block_counts, hipStream_t s);
// block_counts: valid pixels per 256-pixel chunk (written by launch_fuse); block_offsets: their prefix.
hipError_t launch_fuse_compact(int W, int H, const float* out_dense, const int* flags, const int* block_offsets,
                               float* out, hipStream_t s);
hipError_t launch_export_depth(const float4* planes, long long P, float* dst, hipStream_t s);
hipError_t launch_copy(const void* src, void* dst, size_t bytes, hipStream_t s);  // bytes % 4 == 0
hipError_t launch_jbu(const float* ref, int W, int H, const float* coarse, int sw, int sh, int imagescale,
                      float* out, hipStream_t s);
// Diagnostic clock probe (acmmp_clock_probe): per workgroup, shader cycles and 100 MHz ticks around a
// VALU-dense loop of `iters` steps on `rnd` (65536 floats); stamps may be null (warm-up launches).
struct ClockStamp {
    unsigned long long cycles, ticks;
};
hipError_t launch_clock_probe(const float* rnd, int iters, int blocks, ClockStamp* stamps, float* sink, hipStream_t s);
// acmmp_device_checksum: adds the checksum of `bytes` (multiple of 4) at ptr to *out (device, pre-zeroed)
hipError_t launch_checksum(const void* ptr, size_t bytes, unsigned long long* out, hipStream_t s);
// k_eval_nb's source views per launch (kernels.hip, r02 view chunking)
int nb_view_chunk(const KParams& kp);
int nb_tile_order(const KParams& kp);
// k_eval_nb's block count over colour-grid rows [0, rows) of width Wh: 32-pixel row runs, or 8 x 4 tiles
inline long long nb_block_count(long long rows, long long Wh, int tile) {
    return tile ? ((rows + 3) / 4) * ((Wh + 7) / 8) : (rows * Wh + 31) / 32;
}
hipError_t launch_debug(const KParams& kp, int which, int n, const int* px, const int* py, const float4* planes,
                        float* out, hipStream_t s);
// k_eval_nb's NCC instance on n pixels x 8 planes (planes[q * 8 + h]): out[(q * 8 + h) * V + v]
hipError_t launch_debug_nb(const KParams& kp, int n, const int* px, const int* py, const float4* planes, float* out,
                           hipStream_t s);
// k_eval_ref's NCC instance (+ the tail's per-sample fallbacks) on n pixels x 5 planes: out[(q * 5 + h) * V + v]
hipError_t launch_debug_ref(const KParams& kp, int n, const int* px, const int* py, const float4* planes, float* out,
                            hipStream_t s);
// Row-pair binary16 copy of one padded view (W + 2) x (H + 2) (DevCam::img16_base layout); *inexact
// (device int, pre-zeroed) is set when a texel is not exactly representable as a normal binary16
// number or zero.
hipError_t launch_to_f16_pairs(const float* src, int W, int H, uint32_t* dst, int* inexact, hipStream_t s);
hipError_t launch_pad_image(const float* src, size_t pitch_floats, int W, int H, float* dst, int dst_pitch,
                            hipStream_t s);

// Synchronous D2H into pageable caller memory.  Into destination pages that are not resident hipMemcpy
// crawled: 0.32 GB/s for a 800x600 view's planes + costs (30 ms) in heap memory freed and reused, against
// 14-50 GB/s into the same bytes once resident (profiles/r05_d2h_probe.json).  One store per 4 KiB page
// faults them in on the CPU first; the stores write bytes the copy overwrites.  (Heap pages never touched
// before stay slow to fault either way -- the Python binding gives large download arrays hugepage mappings of
// their own, capi.host_empty.)
inline hipError_t d2h(void* dst, const void* src, size_t bytes) {
    if (bytes >= (static_cast<size_t>(256) << 10)) {
        volatile unsigned char* p = static_cast<volatile unsigned char*>(dst);
        for (size_t o = 0; o < bytes; o += 4096) p[o] = 0;
        p[bytes - 1] = 0;
    }
    return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
}

}  // namespace acmmp
