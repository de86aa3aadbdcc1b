// capi.cpp -- implementation of include/acmmp.h (the drop-in boundary).
//
// Owns every device buffer of one reference-view problem, like the reference's ACMMP
// object (ACMMP.h:82-111), and sequences the kernels of ACMMP::RunPatchMatch
// (ACMMP.cu:1506-1556) on one HIP stream.  No OpenCV, no textures: images live in
// plain padded fp32 buffers (engine.h).
#include "../../include/acmmp.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "engine.h"
#include "planar.h"

using namespace acmmp;

static_assert(sizeof(acmmp_camera) == 120, "Camera layout (main.h:40-54)");
static_assert(sizeof(acmmp_params) == 68, "PatchMatchParams layout (ACMMP.h:32-55)");
static_assert(offsetof(acmmp_params, scaled_cols) == 52, "PatchMatchParams layout");
static_assert(offsetof(acmmp_params, geom_consistency) == 60, "PatchMatchParams layout");

// Padded fp32 + row-pair binary16 source images shared by contexts on one GPU, keyed by the caller's
// content key (acmmp_upload_views_keyed): a pipeline prepares each (view, scale) once instead of once
// per problem that reads it.  Entries a context's current problem uses are pinned until its next upload.
struct acmmp_image_cache {
    struct Entry {
        int W = 0, H = 0;
        float* img = nullptr;            // padded (W + 2) x (H + 2) fp32
        uint32_t* img16 = nullptr;       // row-pair binary16 copy, null when some texel is not exact
        bool f16_checked = false;        // the binary16 conversion was attempted (img16 null: inexact)
        size_t bytes = 0;
        int pins = 0;
        uint64_t used = 0;               // LRU clock
    };
    int device = 0;
    size_t budget = 0;                   // soft limit in bytes, 0 = none
    int refs = 1;                        // the creator's + one per context pinning entries
    std::mutex mu;
    std::unordered_map<uint64_t, Entry> map;
    size_t bytes = 0;
    uint64_t clock = 0;
    unsigned long long hits = 0, misses = 0, evictions = 0;
};

struct acmmp_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    acmmp_params params{};
    bool has_params = false;

    int N = 0, W = 0, H = 0, model = -1;
    std::vector<acmmp_camera> cams;
    std::vector<DevCam> dcams;
    DevCam* d_cams = nullptr;
    float* d_img = nullptr;          // padded fp32 images of the views not in an image cache
    uint32_t* d_img16 = nullptr;     // their row-pair binary16 copies
    size_t img_cap = 0, img16_cap = 0;  // texels the two image allocations hold (grow-only)
    char* d_stage = nullptr;         // upload staging for all of a problem's images (grow-only)
    size_t stage_cap = 0;
    int* d_flag = nullptr;           // k_to_f16_pairs' inexact flags, one per view
    size_t flag_cap = 0;
    bool tex16 = false;              // every view of the problem has an exact binary16 copy
    acmmp_image_cache* pin_cache = nullptr;   // entries the current problem pins
    std::vector<uint64_t> pinned;
    std::vector<float*> orphans;     // keyed images another context cached first (freed at the next upload)
    std::vector<uint32_t*> orphans16;
    size_t cams_cap = 0;

    float* d_dep = nullptr;
    bool has_depths = false;

    float4* d_dirs = nullptr;
    int dirs_R = -1;

    float2* d_sph_row = nullptr;
    float2* d_sph_col = nullptr;
    float* d_spatial = nullptr;

    float4* d_planes_rm = nullptr;
    float* d_w_rm = nullptr;                    // the post stage's depth channel (k_merge -> k_filter)
    float* d_costs_rm = nullptr;
    float* d_pre = nullptr;
    uint32_t* d_sel_rm = nullptr;

    float4* d_scaled = nullptr;
    int sw = 0, sh = 0;
    bool has_scaled = false;          // set_scaled_state since the last upload_views

    float4* d_prior = nullptr;
    uint32_t* d_mask = nullptr;
    size_t prior_cap = 0, mask_cap = 0;
    // grow-only capacities of buffers refilled per call (a hipFree waits for the whole device, i.e. for
    // every other context's kernels: reallocating per problem serialised the pipeline's contexts)
    size_t dep_cap = 0, scaled_cap = 0, spatial_cap = 0;
    bool has_prior = false;           // set_planar_prior since the last upload_views
    bool has_result = false;          // planes_rm / costs_rm hold this problem's maps (a run, set_state[_device])
    char* d_pp = nullptr;             // planar-prior triangle tables (acmmp_set_planar_prior_from_maps)
    size_t pp_cap = 0;
    char* h_pp = nullptr;             // their pinned host staging (upload_planar), reused once pp_ev has passed
    size_t h_pp_cap = 0;
    hipEvent_t pp_ev = nullptr;
    bool pp_pending = false;
    int4* d_support = nullptr;        // support-point blocks (acmmp_set_planar_prior_from_state)
    size_t support_cap = 0;

    float4* d_plane_cs[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
    float* d_cost_cs[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
    uint32_t* d_sel_cs[2] = {nullptr, nullptr};
    uint32_t* d_rng_cs[2] = {nullptr, nullptr};
    char* d_scratch = nullptr;
    size_t scratch_bytes = 0;

    float timing[3] = {0.f, 0.f, 0.f};
    float planar_ms[4] = {0.f, 0.f, 0.f, 0.f}; // acmmp_last_planar_timing
    std::vector<hipEvent_t> kev;              // 5 per half-sweep (per-kernel timing)
    float ktiming[4] = {0.f, 0.f, 0.f, 0.f};
    unsigned long long* d_work = nullptr;       // [256] k_eval_nb work counters + [256] the run's status word
    unsigned long long* h_work = nullptr;       // its pinned host copy, enqueued behind the run's last kernel
    unsigned long long work_busy = 0, work_total = 0;
    int klaunch[4] = {0, 0, 0, 0};
    int math = ACMMP_MATH_EXACT;                // acmmp_set_math
    // row-band split (acmmp_band_*): the run in progress
    bool band_active = false;
    KParams band_kp{};
    int band_lo = 0, band_hi = 0, band_sw = 0, band_nsw = 0;
    int band_cur[2] = {0, 0};
    std::string err;
};

namespace {

acmmp_status fail(acmmp_ctx* c, acmmp_status s, const std::string& msg) {
    if (c) c->err = msg;
    return s;
}

#define HIP_TRY(ctx, expr)                                                                         \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            return fail((ctx), e_ == hipErrorOutOfMemory ? ACMMP_ERR_OUT_OF_MEMORY : ACMMP_ERR_HIP, \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                        \
        }                                                                                          \
    } while (0)

template <typename T>
void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

template <typename T>
hipError_t dalloc(T*& p, size_t count) {
    dfree(p);
    return hipMalloc(reinterpret_cast<void**>(&p), sizeof(T) * std::max<size_t>(count, 1));
}

// Grow-only allocation: reallocates only when `count` exceeds the capacity (contents not kept).
template <typename T>
hipError_t dreserve(T*& p, size_t& cap, size_t count) {
    if (p && count <= cap) return hipSuccess;
    cap = 0;
    const hipError_t e = dalloc(p, count);
    if (e == hipSuccess) cap = count;
    return e;
}

// Grow-only with headroom, for buffers whose size follows the problem's scale (the planar-prior tables and
// support blocks): the next power of two of `count`, at least `min_count`, so a pipeline's scales reuse one
// allocation -- a reallocation frees the old buffer, and hipFree waits for the whole device, other contexts'
// kernels included.
template <typename T>
hipError_t dreserve_pow2(T*& p, size_t& cap, size_t count, size_t min_count) {
    if (p && count <= cap) return hipSuccess;
    size_t n = std::max<size_t>(min_count, 1);
    while (n < count) n *= 2;
    return dreserve(p, cap, n);
}

size_t P_of(const acmmp_ctx* c) { return static_cast<size_t>(c->W) * c->H; }
int Wh_of(const acmmp_ctx* c) { return (c->W + 1) / 2; }

// Camera centre exactly as Get3DPointonWorld_cu rounds it (ACMMP.cu:592-594), fused like the kernels.
float neg_dot3(float a0, float a1, float a2, float b0, float b1, float b2) {
    return -std::fmaf(a2, b2, std::fmaf(a1, b1, a0 * b0));
}

}  // namespace

DevCam acmmp::make_devcam(const acmmp_camera& s) {
    DevCam d{};
    d.model = s.model; d.W = s.width; d.H = s.height; d.img_pitch = s.width + 2;
    std::memcpy(d.R, s.R, sizeof d.R);
    std::memcpy(d.t, s.t, sizeof d.t);
    std::memcpy(d.K, s.K, sizeof d.K);
    d.cx = s.params[1]; d.cy = s.params[2];
    d.inv_fx = 1.0f / s.K[0];
    d.inv_fy = 1.0f / s.K[4];
    d.invW = 1.0f / static_cast<float>(s.width);
    d.Wf = static_cast<float>(s.width);
    d.Hf = static_cast<float>(s.height);
    d.C[0] = neg_dot3(s.R[0], s.R[3], s.R[6], s.t[0], s.t[1], s.t[2]);
    d.C[1] = neg_dot3(s.R[1], s.R[4], s.R[7], s.t[0], s.t[1], s.t[2]);
    d.C[2] = neg_dot3(s.R[2], s.R[5], s.R[8], s.t[0], s.t[1], s.t[2]);
    d.dep_w = 1; d.dep_h = 1;
    d.Wm1 = s.width - 1; d.Hm1 = s.height - 1;
    d.Hm1f = static_cast<float>(s.height) - 1.0f;
    d.pitch4 = 4 * (s.width + 2);
    // fast-math constants (float products of the camera's own values)
    d.fkx = static_cast<float>(s.width) * 0.159154936671257019f;
    d.fky = static_cast<float>(s.height) * 0.318309873342514038f;
    set_relative_frame(d, s, s);                      // own frame until the problem's reference is known
    return d;
}

void acmmp::set_relative_frame(DevCam& d, const acmmp_camera& ref, const acmmp_camera& s) {
    double C0[3], M[9], b[3];
    for (int k = 0; k < 3; ++k)                      // reference centre -R0^T t0
        C0[k] = -(double(ref.R[k]) * ref.t[0] + double(ref.R[3 + k]) * ref.t[1] + double(ref.R[6 + k]) * ref.t[2]);
    for (int r = 0; r < 3; ++r) {
        for (int k = 0; k < 3; ++k)                  // R R0^T
            M[3 * r + k] = double(s.R[3 * r]) * ref.R[3 * k] + double(s.R[3 * r + 1]) * ref.R[3 * k + 1] +
                           double(s.R[3 * r + 2]) * ref.R[3 * k + 2];
        b[r] = double(s.R[3 * r]) * C0[0] + double(s.R[3 * r + 1]) * C0[1] + double(s.R[3 * r + 2]) * C0[2] + s.t[r];
    }
    const bool pin = s.model != ACMMP_SPHERE;
    for (int r = 0; r < 3; ++r) {
        for (int k = 0; k < 3; ++k) {
            const double v = pin ? double(s.K[3 * r]) * M[k] + double(s.K[3 * r + 1]) * M[3 + k] + double(s.K[3 * r + 2]) * M[6 + k]
                                 : M[3 * r + k];
            if (r < 2) d.FRxy[2 * k + r] = static_cast<float>(v);   // rows 0, 1 interleaved (packed x, y)
            else d.FRz[k] = static_cast<float>(v);
        }
        const double v = pin ? double(s.K[3 * r]) * b[0] + double(s.K[3 * r + 1]) * b[1] + double(s.K[3 * r + 2]) * b[2] : b[r];
        d.Ft[r] = static_cast<float>(v);
    }
}

extern "C" {

int acmmp_abi_version(void) { return ACMMP_ABI_VERSION; }

int acmmp_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

const char* acmmp_status_str(acmmp_status s) {
    switch (s) {
    case ACMMP_OK: return "ok";
    case ACMMP_ERR_INVALID_ARGUMENT: return "invalid argument";
    case ACMMP_ERR_HIP: return "HIP runtime error";
    case ACMMP_ERR_OUT_OF_MEMORY: return "out of device memory";
    case ACMMP_ERR_STATE: return "call order violated";
    case ACMMP_ERR_UNSUPPORTED: return "unsupported configuration";
    case ACMMP_ERR_NO_DEVICE: return "no HIP device";
    case ACMMP_ERR_COMM: return "RCCL communicator error";
    }
    return "unknown status";
}

const char* acmmp_last_error(const acmmp_ctx* ctx) { return ctx ? ctx->err.c_str() : ""; }

acmmp_status acmmp_create(int device, acmmp_ctx** out) {
    if (!out) return ACMMP_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ACMMP_ERR_NO_DEVICE;
    if (device >= n) return ACMMP_ERR_INVALID_ARGUMENT;
    if (device < 0) {
        if (hipGetDevice(&device) != hipSuccess) return ACMMP_ERR_HIP;
    }
    if (hipSetDevice(device) != hipSuccess) return ACMMP_ERR_HIP;
    acmmp_ctx* c = new acmmp_ctx();
    c->device = device;
    // math stays ACMMP_MATH_EXACT (bit-identical to the oracle) until the caller picks fast explicitly
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return ACMMP_ERR_HIP;
    }
    for (auto& e : c->ev) {
        if (hipEventCreate(&e) != hipSuccess) {
            acmmp_destroy(c);
            return ACMMP_ERR_HIP;
        }
    }
    *out = c;
    return ACMMP_OK;
}

static void unpin_views(acmmp_ctx* c);

void acmmp_destroy(acmmp_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    unpin_views(c);
    dfree(c->d_cams); dfree(c->d_img); dfree(c->d_img16); dfree(c->d_dep); dfree(c->d_dirs);
    dfree(c->d_stage); dfree(c->d_flag);
    dfree(c->d_sph_row); dfree(c->d_sph_col); dfree(c->d_spatial);
    dfree(c->d_planes_rm); dfree(c->d_w_rm); dfree(c->d_costs_rm); dfree(c->d_pre); dfree(c->d_sel_rm);
    dfree(c->d_scaled); dfree(c->d_prior); dfree(c->d_mask); dfree(c->d_pp); dfree(c->d_support); dfree(c->d_scratch); dfree(c->d_work);
    for (int k = 0; k < 2; ++k) {
        for (int b = 0; b < 2; ++b) { dfree(c->d_plane_cs[k][b]); dfree(c->d_cost_cs[k][b]); }
        dfree(c->d_sel_cs[k]); dfree(c->d_rng_cs[k]);
    }
    for (auto& e : c->ev) if (e) (void)hipEventDestroy(e);
    if (c->pp_ev) (void)hipEventDestroy(c->pp_ev);
    if (c->h_pp) (void)hipHostFree(c->h_pp);
    if (c->h_work) (void)hipHostFree(c->h_work);
    for (auto& e : c->kev) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

acmmp_status acmmp_set_math(acmmp_ctx* c, int mode) {
    if (!c) return ACMMP_ERR_INVALID_ARGUMENT;
    if (mode != ACMMP_MATH_EXACT && mode != ACMMP_MATH_FAST) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "unknown math mode");
    c->math = mode;
    return ACMMP_OK;
}

int acmmp_get_math(const acmmp_ctx* c) { return c ? c->math : -1; }

acmmp_status acmmp_set_params(acmmp_ctx* c, const acmmp_params* p) {
    if (!c || !p) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "null argument");
    if (p->num_images < 2 || p->num_images > kMaxViews + 1)
        return fail(c, ACMMP_ERR_UNSUPPORTED, "num_images must be in [2, 33] (32 source views max)");
    if (p->patch_size < 1 || p->radius_increment < 1 || p->top_k < 0 || p->max_iterations < 0)
        return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "invalid patch_size/radius_increment/top_k/max_iterations");
    c->params = *p;
    c->has_params = true;
    return ACMMP_OK;
}


static acmmp_status upload_views_impl(acmmp_ctx* c, int n, const float* const* images, const size_t* pitch_bytes,
                                      const acmmp_camera* cams, bool device_src, acmmp_image_cache* cache,
                                      const uint64_t* keys);

acmmp_status acmmp_upload_views(acmmp_ctx* c, int n, const float* const* images, const size_t* pitch_bytes,
                                const acmmp_camera* cams) {
    return upload_views_impl(c, n, images, pitch_bytes, cams, false, nullptr, nullptr);
}

acmmp_status acmmp_upload_views_device(acmmp_ctx* c, int n, const float* const* dev_images, const size_t* pitch_bytes,
                                       const acmmp_camera* cams) {
    return upload_views_impl(c, n, dev_images, pitch_bytes, cams, true, nullptr, nullptr);
}

acmmp_status acmmp_upload_views_keyed(acmmp_ctx* c, acmmp_image_cache* cache, int n, const uint64_t* keys,
                                      const float* const* images, const size_t* pitch_bytes, const acmmp_camera* cams,
                                      int device_src) {
    if (c && cache && cache->device != c->device)
        return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "image cache belongs to another device");
    return upload_views_impl(c, n, images, pitch_bytes, cams, device_src != 0, cache, keys);
}

acmmp_status acmmp_image_cache_create(int device, size_t budget_bytes, acmmp_image_cache** out) {
    if (!out) return ACMMP_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ACMMP_ERR_NO_DEVICE;
    if (device < 0 || device >= n) return ACMMP_ERR_INVALID_ARGUMENT;
    acmmp_image_cache* k = new acmmp_image_cache();
    k->device = device;
    k->budget = budget_bytes;
    *out = k;
    return ACMMP_OK;
}

}  // extern "C"

// Drop one reference; the last one frees the cache (contexts that still pin entries keep it alive
// until their next upload or their destruction).
static void cache_release(acmmp_image_cache* k) {
    bool last;
    {
        std::lock_guard<std::mutex> lk(k->mu);
        last = --k->refs == 0;
    }
    if (!last) return;
    (void)hipSetDevice(k->device);
    for (auto& kv : k->map) {
        dfree(kv.second.img);
        dfree(kv.second.img16);
    }
    delete k;
}

extern "C" {

void acmmp_image_cache_destroy(acmmp_image_cache* k) {
    if (k) cache_release(k);
}

acmmp_status acmmp_image_cache_stats(acmmp_image_cache* k, unsigned long long out[5]) {
    if (!k || !out) return ACMMP_ERR_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lk(k->mu);
    out[0] = k->hits; out[1] = k->misses; out[2] = k->bytes; out[3] = k->map.size(); out[4] = k->evictions;
    return ACMMP_OK;
}

}  // extern "C"

static void unpin_views(acmmp_ctx* c) {
    for (auto& p : c->orphans) dfree(p);
    for (auto& p : c->orphans16) dfree(p);
    c->orphans.clear();
    c->orphans16.clear();
    if (!c->pin_cache) return;
    {
        std::lock_guard<std::mutex> lk(c->pin_cache->mu);
        for (uint64_t key : c->pinned) {
            auto it = c->pin_cache->map.find(key);
            if (it != c->pin_cache->map.end() && it->second.pins > 0) --it->second.pins;
        }
    }
    c->pinned.clear();
    acmmp_image_cache* k = c->pin_cache;
    c->pin_cache = nullptr;
    cache_release(k);
}

// Least-recently used unpinned entries go first; the budget is soft (pinned entries stay).  Called with
// the cache mutex held: the evicted allocations are handed back in `dead` and freed by the caller after
// it releases the lock (hipFree waits for the device, which would stall every other context's upload).
static void evict_over_budget(acmmp_image_cache* k, std::vector<void*>& dead) {
    if (k->budget == 0) return;
    while (k->bytes > k->budget) {
        auto victim = k->map.end();
        for (auto it = k->map.begin(); it != k->map.end(); ++it)
            if (it->second.pins == 0 && (victim == k->map.end() || it->second.used < victim->second.used)) victim = it;
        if (victim == k->map.end()) return;
        dead.push_back(victim->second.img);
        dead.push_back(victim->second.img16);
        k->bytes -= victim->second.bytes;
        k->map.erase(victim);
        ++k->evictions;
    }
}

// Host images go through one staging buffer; device images are padded straight from their buffers.
// Views found in `cache` (same key and size) reuse its padded and binary16 copies; the others are
// padded, converted and checked here (one flag read and one stream sync per call, for all of them).
static acmmp_status upload_views_impl(acmmp_ctx* c, int n, const float* const* images, const size_t* pitch_bytes,
                                      const acmmp_camera* cams, bool device_src, acmmp_image_cache* cache,
                                      const uint64_t* keys) {
    if (!c || !images || !cams) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "null argument");
    if (n < 2 || n > kMaxViews + 1) return fail(c, ACMMP_ERR_UNSUPPORTED, "need 2..33 images");
    for (int i = 0; i < n; ++i) {
        if (!images[i] || cams[i].width <= 0 || cams[i].height <= 0 || cams[i].width > 32767 || cams[i].height > 32767)
            return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "bad image " + std::to_string(i));
        if (cams[i].model != ACMMP_PINHOLE && cams[i].model != ACMMP_SPHERE)
            return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "unknown camera model");
        if (4LL * (cams[i].width + 2) * (cams[i].height + 2) > 0x7fffffffLL)
            return fail(c, ACMMP_ERR_UNSUPPORTED, "image larger than 2 GiB (32-bit texel offsets)");
        if (cams[i].model != cams[0].model)
            return fail(c, ACMMP_ERR_UNSUPPORTED, "mixed camera models in one problem are not supported");
    }
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));          // the previous problem's kernels read the old images
    unpin_views(c);
    // until this call succeeds the context holds no usable views: a failure below must not leave N > 0
    // with camera entries pointing at images that are now unpinned, reallocated or freed
    c->N = 0;
    c->tex16 = false;
    const bool resized = (c->W != cams[0].width || c->H != cams[0].height);
    // a new problem: the previous problem's prior / scaled state no longer applies (the reference
    // builds a fresh ACMMP object per ProcessProblem, main.cpp:80)
    c->has_prior = false;
    c->has_scaled = false;
    c->has_result = false;
    c->W = cams[0].width;
    c->H = cams[0].height;
    c->model = cams[0].model;
    c->cams.assign(cams, cams + n);
    c->dirs_R = -1;
    // binary16 copies for the NCC fetches when they hold the same values (8-bit images always do): half
    // the bytes per footprint, so twice the views fit a cache level.  ACMMP_TEX16=0 in the
    // environment keeps the fp32 fetches (A/B switch; identical results).
    const char* tex16_env = std::getenv("ACMMP_TEX16");
    const bool want16 = !(tex16_env && tex16_env[0] == '0');

    std::vector<float*> base(n, nullptr);
    std::vector<uint32_t*> base16(n, nullptr);
    std::vector<int> miss;                               // views padded / converted by this call
    std::vector<bool> keyed(n, false);
    if (cache && keys) {
        std::lock_guard<std::mutex> lk(cache->mu);
        ++cache->refs;                                    // released by unpin_views
        for (int i = 0; i < n; ++i) {
            if (!keys[i]) continue;
            auto it = cache->map.find(keys[i]);
            if (it != cache->map.end() && it->second.W == cams[i].width && it->second.H == cams[i].height &&
                (it->second.f16_checked || !want16)) {
                base[i] = it->second.img;
                base16[i] = want16 ? it->second.img16 : nullptr;
                ++it->second.pins;
                it->second.used = ++cache->clock;
                c->pinned.push_back(keys[i]);
                ++cache->hits;
            } else {
                keyed[i] = it == cache->map.end() || it->second.pins == 0;   // (re)insert this key
                ++cache->misses;
            }
        }
        c->pin_cache = cache;
    }
    std::vector<bool> is_miss(n, false);
    for (int i = 0; i < n; ++i) if (!base[i]) { miss.push_back(i); is_miss[i] = true; }

    // private (unkeyed) views share the context's grow-only allocation; keyed misses get their own
    std::vector<long long> off(n, 0);
    long long total = 0;
    for (int i : miss) {
        if (keyed[i]) continue;
        off[i] = total;                                  // base = padded texel (-1,-1)
        total += static_cast<long long>(cams[i].width + 2) * (cams[i].height + 2);
        total = (total + 63) & ~63LL;
    }
    if (total > 0) {
        HIP_TRY(c, dreserve(c->d_img, c->img_cap, static_cast<size_t>(total)));
        if (want16) HIP_TRY(c, dreserve(c->d_img16, c->img16_cap, static_cast<size_t>(total)));
    }
    std::vector<float*> own(n, nullptr);
    std::vector<uint32_t*> own16(n, nullptr);
    // keyed misses that did not end up in the cache -- all of them when a step below fails -- stay with
    // this context until its next upload (unpin_views frees them)
    struct OwnGuard {
        acmmp_ctx* c;
        std::vector<float*>& own;
        std::vector<uint32_t*>& own16;
        ~OwnGuard() {
            for (float* p : own) if (p) c->orphans.push_back(p);
            for (uint32_t* p : own16) if (p) c->orphans16.push_back(p);
        }
    } own_guard{c, own, own16};
    for (int i : miss) {
        if (keyed[i]) {
            const size_t texels = static_cast<size_t>(cams[i].width + 2) * (cams[i].height + 2);
            HIP_TRY(c, dalloc(own[i], texels));
            if (want16) HIP_TRY(c, dalloc(own16[i], texels));
            base[i] = own[i];
            base16[i] = own16[i];
        } else {
            base[i] = c->d_img + off[i];
            base16[i] = want16 ? c->d_img16 + off[i] : nullptr;
        }
    }
    if (!miss.empty()) {
        std::vector<size_t> soff(n + 1, 0);
        for (int i = 0; i < n; ++i) {
            const size_t rowb = sizeof(float) * cams[i].width;
            const size_t pb = pitch_bytes ? pitch_bytes[i] : rowb;
            soff[i + 1] = soff[i] + (is_miss[i] ? ((pb * (cams[i].height - 1) + rowb + 255) & ~static_cast<size_t>(255)) : 0);
        }
        if (!device_src) HIP_TRY(c, dreserve(c->d_stage, c->stage_cap, soff[n]));
        if (want16) {
            HIP_TRY(c, dreserve(c->d_flag, c->flag_cap, static_cast<size_t>(n)));
            HIP_TRY(c, hipMemsetAsync(c->d_flag, 0, sizeof(int) * n, c->stream));
        }
        for (int i : miss) {
            const size_t rowb = sizeof(float) * cams[i].width;
            const size_t pb = pitch_bytes ? pitch_bytes[i] : rowb;
            const size_t bytes = pb * (cams[i].height - 1) + rowb;
            const float* src = images[i];
            if (!device_src) {
                float* staging = reinterpret_cast<float*>(c->d_stage + soff[i]);
                HIP_TRY(c, hipMemcpyAsync(staging, images[i], bytes, hipMemcpyHostToDevice, c->stream));
                src = staging;
            }
            HIP_TRY(c, launch_pad_image(src, pb / sizeof(float), cams[i].width, cams[i].height, base[i],
                                        cams[i].width + 2, c->stream));
            if (want16)
                HIP_TRY(c, launch_to_f16_pairs(base[i], cams[i].width, cams[i].height, base16[i], c->d_flag + i,
                                               c->stream));
        }
        std::vector<int> inexact(n, 0);
        if (want16) HIP_TRY(c, hipMemcpyAsync(inexact.data(), c->d_flag, sizeof(int) * n, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));      // staging, padding and flags done before returning
        for (int i : miss) {
            if (inexact[i]) {
                if (keyed[i]) { dfree(own16[i]); own16[i] = nullptr; }
                base16[i] = nullptr;
            }
        }
        if (cache && keys) {
            std::vector<void*> dead;
            {
                std::lock_guard<std::mutex> lk(cache->mu);
                for (int i : miss) {
                    if (!keyed[i]) continue;
                    auto it = cache->map.find(keys[i]);
                    if (it != cache->map.end()) {
                        if (it->second.pins > 0) {              // another context inserted it meanwhile: use ours privately
                            keyed[i] = false;
                            continue;
                        }
                        dead.push_back(it->second.img);
                        dead.push_back(it->second.img16);
                        cache->bytes -= it->second.bytes;
                        cache->map.erase(it);
                    }
                    acmmp_image_cache::Entry e;
                    e.W = cams[i].width; e.H = cams[i].height;
                    e.img = own[i]; e.img16 = own16[i];
                    e.f16_checked = want16;
                    e.bytes = sizeof(float) * static_cast<size_t>(e.W + 2) * (e.H + 2) * (own16[i] ? 2 : 1);
                    e.pins = 1;
                    e.used = ++cache->clock;
                    cache->bytes += e.bytes;
                    cache->map.emplace(keys[i], e);
                    c->pinned.push_back(keys[i]);
                    own[i] = nullptr; own16[i] = nullptr;      // owned by the cache now
            }
            evict_over_budget(cache, dead);
            }
            for (void* p : dead) dfree(p);
        }
    }
    c->tex16 = want16;
    for (int i = 0; i < n; ++i) c->tex16 = c->tex16 && base16[i] != nullptr;

    c->dcams.assign(n, DevCam{});
    for (int i = 0; i < n; ++i) {
        const acmmp_camera& s = cams[i];
        DevCam& d = c->dcams[i];
        d = make_devcam(s);
        d.img_base = base[i];
        d.img_bytes = static_cast<int>(4LL * (s.width + 2) * (s.height + 2));
        d.img16_base = c->tex16 ? reinterpret_cast<const uint16_t*>(base16[i]) : nullptr;
        d.img16_bytes = static_cast<int>(4LL * (s.width + 2) * (s.height + 2));
        d.dep_off = 0; d.dep_w = 1; d.dep_h = 1;
        set_relative_frame(d, cams[0], s);
    }
    HIP_TRY(c, dreserve(c->d_cams, c->cams_cap, static_cast<size_t>(n)));
    HIP_TRY(c, hipMemcpyAsync(c->d_cams, c->dcams.data(), sizeof(DevCam) * n, hipMemcpyHostToDevice, c->stream));
    c->has_depths = false;

    if (resized || !c->d_planes_rm) {
        const size_t P = P_of(c);
        const size_t Pc = static_cast<size_t>(c->H) * Wh_of(c);
        HIP_TRY(c, dalloc(c->d_planes_rm, P));
        HIP_TRY(c, dalloc(c->d_w_rm, P));
        HIP_TRY(c, dalloc(c->d_costs_rm, P));
        HIP_TRY(c, dalloc(c->d_pre, P));
        HIP_TRY(c, dalloc(c->d_sel_rm, P));
        HIP_TRY(c, hipMemsetAsync(c->d_planes_rm, 0, sizeof(float4) * P, c->stream));
        HIP_TRY(c, hipMemsetAsync(c->d_costs_rm, 0, sizeof(float) * P, c->stream));
        HIP_TRY(c, hipMemsetAsync(c->d_sel_rm, 0, sizeof(uint32_t) * P, c->stream));
        for (int k = 0; k < 2; ++k) {
            for (int b = 0; b < 2; ++b) {
                HIP_TRY(c, dalloc(c->d_plane_cs[k][b], Pc));
                HIP_TRY(c, dalloc(c->d_cost_cs[k][b], Pc));
            }
            HIP_TRY(c, dalloc(c->d_sel_cs[k], Pc));
            HIP_TRY(c, dalloc(c->d_rng_cs[k], Pc));
        }
        dfree(c->d_prior); dfree(c->d_mask);
        c->prior_cap = c->mask_cap = 0;
        dfree(c->d_scratch);
        c->scratch_bytes = 0;
    }
    // pre_costs are written only by the upsample branch (ACMMP.cu:776) and otherwise read as zero
    // (DESIGN.md §2.2): zero them for every problem so a context reused across problems never leaks
    // another view's costs into k_finish's hierarchy gate
    HIP_TRY(c, hipMemsetAsync(c->d_pre, 0, sizeof(float) * P_of(c), c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->N = n;
    return ACMMP_OK;
}

static acmmp_status upload_depths(acmmp_ctx* c, int n, const float* const* depths, const int* w, const int* h,
                                  hipMemcpyKind kind) {
    if (!c || !depths || !w || !h) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "null argument");
    if (c->N == 0) return fail(c, ACMMP_ERR_STATE, "upload_views first");
    if (n < c->N) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "need one depth map per image");
    HIP_TRY(c, hipSetDevice(c->device));
    size_t total = 0;
    std::vector<size_t> off(c->N);
    for (int i = 0; i < c->N; ++i) {
        if (!depths[i] || w[i] <= 0 || h[i] <= 0) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "bad depth map");
        off[i] = total;
        total += static_cast<size_t>(w[i]) * h[i];
    }
    HIP_TRY(c, dreserve(c->d_dep, c->dep_cap, total));
    for (int i = 0; i < c->N; ++i) {
        // device sources through the copy kernel (compute queue, HBM rate), host ones through the DMA engine
        if (kind == hipMemcpyDeviceToDevice)
            HIP_TRY(c, launch_copy(depths[i], c->d_dep + off[i], sizeof(float) * w[i] * h[i], c->stream));
        else
            HIP_TRY(c, hipMemcpyAsync(c->d_dep + off[i], depths[i], sizeof(float) * w[i] * h[i], kind, c->stream));
        c->dcams[i].dep_off = static_cast<long long>(off[i]);
        c->dcams[i].dep_w = w[i];
        c->dcams[i].dep_h = h[i];
    }
    HIP_TRY(c, hipMemcpyAsync(c->d_cams, c->dcams.data(), sizeof(DevCam) * c->N, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));             // the sources may be reused once this returns
    c->has_depths = true;
    return ACMMP_OK;
}

extern "C" {

acmmp_status acmmp_upload_depths(acmmp_ctx* c, int n, const float* const* depths, const int* w, const int* h) {
    return upload_depths(c, n, depths, w, h, hipMemcpyHostToDevice);
}

acmmp_status acmmp_upload_depths_device(acmmp_ctx* c, int n, const float* const* depths, const int* w, const int* h) {
    return upload_depths(c, n, depths, w, h, hipMemcpyDeviceToDevice);
}

acmmp_status acmmp_export_depth(acmmp_ctx* c, float* dev_dst) {
    if (!c || !dev_dst) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "null argument");
    if (!c->d_planes_rm) return fail(c, ACMMP_ERR_STATE, "no result yet");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, launch_export_depth(c->d_planes_rm, static_cast<long long>(P_of(c)), dev_dst, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return ACMMP_OK;
}

acmmp_status acmmp_set_state(acmmp_ctx* c, const float* planes, const float* costs) {
    if (!c) return ACMMP_ERR_INVALID_ARGUMENT;
    if (c->N == 0) return fail(c, ACMMP_ERR_STATE, "upload_views first");
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t P = P_of(c);
    if (planes)
        HIP_TRY(c, hipMemcpyAsync(c->d_planes_rm, planes, sizeof(float4) * P, hipMemcpyHostToDevice, c->stream));
    if (costs) HIP_TRY(c, hipMemcpyAsync(c->d_costs_rm, costs, sizeof(float) * P, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (planes && costs) c->has_result = true;
    return ACMMP_OK;
}

acmmp_status acmmp_export_state(acmmp_ctx* c, float* dev_planes, float* dev_costs) {
    if (!c || (!dev_planes && !dev_costs)) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "null argument");
    if (!c->d_planes_rm) return fail(c, ACMMP_ERR_STATE, "no result yet");
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t P = P_of(c);
    if (dev_planes)
        HIP_TRY(c, launch_copy(c->d_planes_rm, dev_planes, sizeof(float4) * P, c->stream));
    if (dev_costs)
        HIP_TRY(c, launch_copy(c->d_costs_rm, dev_costs, sizeof(float) * P, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));           // another context may read the buffers next
    return ACMMP_OK;
}

acmmp_status acmmp_set_state_device(acmmp_ctx* c, const float* dev_planes, const float* dev_costs) {
    if (!c) return ACMMP_ERR_INVALID_ARGUMENT;
    if (c->N == 0) return fail(c, ACMMP_ERR_STATE, "upload_views first");
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t P = P_of(c);
    if (dev_planes)
        HIP_TRY(c, launch_copy(dev_planes, c->d_planes_rm, sizeof(float4) * P, c->stream));
    if (dev_costs)
        HIP_TRY(c, launch_copy(dev_costs, c->d_costs_rm, sizeof(float) * P, c->stream));
    if (dev_planes && dev_costs) c->has_result = true;
    // stream-ordered before this context's next kernels; the caller keeps the buffers until its run
    return ACMMP_OK;
}

acmmp_status acmmp_set_scaled_state(acmmp_ctx* c, const float* planes, int sw, int sh) {
    if (!c || !planes || sw <= 0 || sh <= 0) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "bad scaled state");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, dreserve(c->d_scaled, c->scaled_cap, static_cast<size_t>(sw) * sh));
    HIP_TRY(c, hipMemcpyAsync(c->d_scaled, planes, sizeof(float4) * sw * sh, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->sw = sw;
    c->sh = sh;
    c->has_scaled = true;
    return ACMMP_OK;
}

acmmp_status acmmp_set_planar_prior(acmmp_ctx* c, const float* prior, const uint32_t* masks) {
    if (!c || !prior || !masks) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "null argument");
    if (c->N == 0) return fail(c, ACMMP_ERR_STATE, "upload_views first");
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t P = P_of(c);
    HIP_TRY(c, dreserve(c->d_prior, c->prior_cap, P));
    HIP_TRY(c, dreserve(c->d_mask, c->mask_cap, P));
    HIP_TRY(c, hipMemcpyAsync(c->d_prior, prior, sizeof(float4) * P, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->d_mask, masks, sizeof(uint32_t) * P, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->has_prior = true;
    return ACMMP_OK;
}

// The device half of the planar block for host-computed triangles: one upload of the tables, the raster
// and the prior-depth mask / expansion kernels, into the context's planar-prior state.
using planar_clock = std::chrono::steady_clock;
static float ms_since(planar_clock::time_point t0) {
    return std::chrono::duration<float, std::milli>(planar_clock::now() - t0).count();
}

static acmmp_status upload_planar(acmmp_ctx* c, const PlanarTriangles& pt, float depth_min, float depth_max,
                                  int* n_triangles) {
    const auto t0 = planar_clock::now();
    const acmmp_camera& cam = c->cams[0];
    const int W = c->W, H = c->H;
    const size_t P = P_of(c);
    const int m = static_cast<int>(pt.step.size());
    // one upload: first[] (8 B aligned) | plane (float4) | tri | step | row/col trig
    auto up = [](size_t b) { return (b + 255) & ~static_cast<size_t>(255); };
    const size_t o_first = 0, n_first = sizeof(long long) * (m + 1);
    const size_t o_plane = up(o_first + n_first), n_plane = sizeof(float) * pt.plane.size();
    const size_t o_tri = up(o_plane + n_plane), n_tri = sizeof(int) * pt.tri.size();
    const size_t o_step = up(o_tri + n_tri), n_step = sizeof(float) * pt.step.size();
    const size_t o_row = up(o_step + n_step), n_row = sizeof(float2) * pt.row_trig.size();
    const size_t o_col = up(o_row + n_row), n_col = sizeof(float2) * pt.col_trig.size();
    const size_t bytes = up(o_col + n_col);
    // the tables go through a pinned staging buffer of the context, so the copy and the two kernels are only
    // enqueued here: the next run_patchmatch on this stream follows them, acmmp_download_planar_prior waits for
    // them, and the next call waits (pp_ev) before it rewrites the staging.  (Waiting here for the kernels put
    // this call behind other contexts' RunPatchMatch kernels in the pipeline's overlapped planar passes: 83 of
    // the stage's 206 ms at the bench scene, against 17 ms run alone -- profiles/r06_e2e_planar.json.)
    if (c->pp_pending) {
        HIP_TRY(c, hipEventSynchronize(c->pp_ev));
        c->pp_pending = false;
    }
    if (!c->pp_ev) HIP_TRY(c, hipEventCreateWithFlags(&c->pp_ev, hipEventDisableTiming));
    if (bytes > c->h_pp_cap) {                               // (the same headroom as d_pp: hipHostFree syncs too)
        if (c->h_pp) HIP_TRY(c, hipHostFree(c->h_pp));
        c->h_pp = nullptr;
        c->h_pp_cap = 0;
        size_t n = static_cast<size_t>(16) << 20;
        while (n < bytes) n *= 2;
        HIP_TRY(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_pp), n, hipHostMallocDefault));
        c->h_pp_cap = n;
    }
    char* host = c->h_pp;
    std::memcpy(host + o_first, pt.first.data(), n_first);
    if (n_plane) std::memcpy(host + o_plane, pt.plane.data(), n_plane);
    if (n_tri) std::memcpy(host + o_tri, pt.tri.data(), n_tri);
    if (n_step) std::memcpy(host + o_step, pt.step.data(), n_step);
    if (n_row) std::memcpy(host + o_row, pt.row_trig.data(), n_row);
    if (n_col) std::memcpy(host + o_col, pt.col_trig.data(), n_col);
    HIP_TRY(c, dreserve_pow2(c->d_pp, c->pp_cap, bytes, static_cast<size_t>(16) << 20));
    HIP_TRY(c, dreserve(c->d_prior, c->prior_cap, P));
    HIP_TRY(c, dreserve(c->d_mask, c->mask_cap, P));
    HIP_TRY(c, hipMemcpyAsync(c->d_pp, host, bytes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->d_mask, 0, sizeof(uint32_t) * P, c->stream));
    PlanarDev pd;
    pd.first = reinterpret_cast<const long long*>(c->d_pp + o_first);
    pd.plane = reinterpret_cast<const float4*>(c->d_pp + o_plane);
    pd.tri = reinterpret_cast<const int*>(c->d_pp + o_tri);
    pd.step = reinterpret_cast<const float*>(c->d_pp + o_step);
    pd.row_trig = reinterpret_cast<const float2*>(c->d_pp + o_row);
    pd.col_trig = reinterpret_cast<const float2*>(c->d_pp + o_col);
    pd.n_tri = m;
    pd.n_steps = pt.first[m];
    pd.W = W; pd.H = H; pd.model = cam.model;
    pd.K0 = cam.K[0]; pd.K2 = cam.K[2]; pd.K4 = cam.K[4]; pd.K5 = cam.K[5];
    pd.depth_min = depth_min; pd.depth_max = depth_max;
    HIP_TRY(c, launch_planar_raster(pd, c->d_mask, c->stream));
    HIP_TRY(c, launch_planar_mask(pd, c->d_mask, c->d_prior, c->stream));
    HIP_TRY(c, hipEventRecord(c->pp_ev, c->stream));
    c->pp_pending = true;
    c->planar_ms[3] = ms_since(t0);
    c->has_prior = true;
    if (n_triangles) *n_triangles = m;
    return ACMMP_OK;
}

acmmp_status acmmp_set_planar_prior_from_maps(acmmp_ctx* c, const float* depths, const float* costs, float depth_min,
                                              float depth_max, int* n_triangles) {
    if (!c || !depths || !costs) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "null argument");
    if (c->N == 0) return fail(c, ACMMP_ERR_STATE, "upload_views first");
    HIP_TRY(c, hipSetDevice(c->device));
    const auto t0 = planar_clock::now();
    PlanarTriangles pt;
    const acmmp_status st = planar_triangles(c->cams[0], depths, costs, c->W, c->H, &pt);
    if (st != ACMMP_OK) return fail(c, st, "planar_triangles");
    c->planar_ms[0] = 0.f;                                  // the support-point scan is inside planar_triangles
    c->planar_ms[1] = pt.delaunay_ms;
    c->planar_ms[2] = ms_since(t0) - pt.delaunay_ms;
    return upload_planar(c, pt, depth_min, depth_max, n_triangles);
}

acmmp_status acmmp_set_planar_prior_from_state(acmmp_ctx* c, float depth_min, float depth_max, int* n_triangles) {
    if (!c) return ACMMP_ERR_INVALID_ARGUMENT;
    if (c->N == 0) return fail(c, ACMMP_ERR_STATE, "upload_views and run_patchmatch first");
    // the maps must be this problem's: a run (or set_state of both maps) since the last upload_views
    if (!c->has_result) return fail(c, ACMMP_ERR_STATE, "no depth / cost maps since the last upload_views");
    HIP_TRY(c, hipSetDevice(c->device));
    const int W = c->W, H = c->H;
    const size_t nb = static_cast<size_t>((W + 4) / 5) * ((H + 4) / 5);
    const auto t0 = planar_clock::now();
    HIP_TRY(c, dreserve_pow2(c->d_support, c->support_cap, nb, static_cast<size_t>(1) << 17));
    HIP_TRY(c, launch_support_points(c->d_costs_rm, c->d_planes_rm, W, H, c->d_support, c->stream));
    std::vector<int4> blocks(nb);
    HIP_TRY(c, hipMemcpyAsync(blocks.data(), c->d_support, sizeof(int4) * nb, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    std::vector<int> xy;
    std::vector<float> depth_at;
    for (const int4& b : blocks) {                          // the reference's order: strip-major
        if (!b.x) continue;
        xy.push_back(b.y);
        xy.push_back(b.z);
        float d;
        std::memcpy(&d, &b.w, sizeof d);
        depth_at.push_back(d);
    }
    c->planar_ms[0] = ms_since(t0);
    const auto t1 = planar_clock::now();
    PlanarTriangles pt;
    const acmmp_status st = planar_triangles_pts(c->cams[0], xy, depth_at, W, H, &pt);
    if (st != ACMMP_OK) return fail(c, st, "planar_triangles");
    c->planar_ms[1] = pt.delaunay_ms;
    c->planar_ms[2] = ms_since(t1) - pt.delaunay_ms;
    return upload_planar(c, pt, depth_min, depth_max, n_triangles);
}

acmmp_status acmmp_download_planar_prior(acmmp_ctx* c, float* prior, uint32_t* masks) {
    if (!c) return ACMMP_ERR_INVALID_ARGUMENT;
    if (!c->has_prior) return fail(c, ACMMP_ERR_STATE, "no planar prior set since the last upload_views");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));           // the raster / mask kernels upload_planar enqueued
    const size_t P = P_of(c);
    if (prior) HIP_TRY(c, d2h(prior, c->d_prior, sizeof(float4) * P));
    if (masks) HIP_TRY(c, d2h(masks, c->d_mask, sizeof(uint32_t) * P));
    return ACMMP_OK;
}

// pixels of one colour inside the checkerboard grid (the half-sweep's work items)
static unsigned long long colour_pixels(const acmmp_ctx* c, const KParams& kp, int colour) {
    unsigned long long n = 0;
    for (int y = kp.row_lo; y < kp.row_hi; ++y) {
        const int first = (y + colour) & 1;                  // black = (x + y) even
        n += first < c->W ? static_cast<unsigned long long>((c->W - first + 1) / 2) : 0ull;
    }
    return n;
}

// Split point of the refinement evaluation: half the views up to 4 views, one 4-view NCC
// chunk above (r03 sweep, profiles/r03_ref_split_sweep.txt / r03_ref_split_v20.txt: at V = 10, 15 and 20
// S = 4 beats 6 / 8 / 12 by 1-4%); 0 (no split) for one view, for colour grids too large for the 32-bit
// queue entries, or with ACMMP_REF_SPLIT=0 in the environment (A/B switch).
// Read at every run (one getenv per RunPatchMatch), so tests can switch it within one process.
// interp_ref: the refinement's first part interpolates SPHERE sample coordinates (fast mode, V > 4, views
// of the interpolation's size), which makes its views cheaper than the tail's per-sample ones: S = 8 there
// from V = 9 up (C3 V = 15: 88.9 -> 90.4 Mpix-it/s against S = 4; S = 10 / 12 lose, and the exact mode
// loses 5% at S = 8, profiles/r04_split_ab.txt, r04_split2_ab.txt)
static int ref_split_point(int V, size_t Pc, bool interp_ref) {
    const char* e_on = std::getenv("ACMMP_REF_SPLIT");
    const char* e_at = std::getenv("ACMMP_REF_SPLIT_AT");  // ACMMP_REF_SPLIT_AT=S: fixed split (A/B)
    const int enabled = e_on ? std::atoi(e_on) : 1;
    const int at = e_at ? std::atoi(e_at) : 0;
    if (!enabled || V < 2 || Pc >= (static_cast<size_t>(1) << 29)) return 0;
    if (at > 0) return at < V ? at : 0;
    if (interp_ref && V > 8) return 8;
    return V <= 4 ? V / 2 : 4;
}

static acmmp_status build_kparams(acmmp_ctx* c, KParams& kp, uint64_t seed) {
    const acmmp_params& p = c->params;
    if (!c->has_params) return fail(c, ACMMP_ERR_STATE, "set_params first");
    if (c->N == 0) return fail(c, ACMMP_ERR_STATE, "upload_views first");
    if (p.num_images != c->N) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "params.num_images != uploaded images");
    if (p.geom_consistency && !c->has_depths) return fail(c, ACMMP_ERR_STATE, "geom_consistency needs upload_depths");
    if (p.planar_prior && !c->has_prior) return fail(c, ACMMP_ERR_STATE, "planar_prior needs set_planar_prior");
    if (!p.geom_consistency && p.hierarchy && !p.planar_prior && !c->has_scaled)
        return fail(c, ACMMP_ERR_STATE, "hierarchy needs set_scaled_state");
    if (p.upsample && !p.planar_prior && p.hierarchy &&
        (c->sw != static_cast<int>(p.scaled_cols) || c->sh != static_cast<int>(p.scaled_rows)))
        return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "scaled_cols/rows != scaled state size");
    if (p.hierarchy && !p.upsample && !p.geom_consistency && !p.planar_prior && (c->sw != c->W || c->sh != c->H))
        return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "hierarchy reuse needs a full-size scaled state");
    const int R = p.patch_size / 2;
    if (R > 64) return fail(c, ACMMP_ERR_UNSUPPORTED, "patch radius > 64");
    int nside = 0;
    for (int i = -R; i <= R; i += p.radius_increment) ++nside;
    kp = KParams{};
    kp.model = c->model;
    kp.W = c->W; kp.H = c->H; kp.Wh = Wh_of(c); kp.N = c->N; kp.V = c->N - 1;
    kp.R = R; kp.inc = p.radius_increment; kp.nside = nside; kp.S = nside * nside;
    // interpolated SPHERE sample coordinates in the fast k_eval_nb: 6x6 patches whose
    // radius spans at most 5 pixels of 2 pi / 2000 rad (patch_size 11, radius_increment 2 from 2000x1000
    // up) -- a wider patch angle makes the interpolation's NCC error exceed 1e-4 in the tail near source
    // poles, where the 256-pixel corner-spread fallback no longer catches it (1600x800: 3.7e-3 at a spread
    // of 65 px; scripts/interp_feasibility.py, tests/test_interp_design.py).  patch_size 21 / increment 4
    // also gives 6x6 samples but spans twice the angle: it projects every sample below 4000x2000.
    kp.interp = c->model == kSphere && nside == 6 && 2000LL * R <= 5LL * c->W && 1000LL * R <= 5LL * c->H;
    // ACMMP_INTERP=0 projects every sample in the fast mode too (the per-sample fast arithmetic the
    // interpolation is gated against, tests/test_gpu_fastmath.py T2); read per run
    if (const char* e = std::getenv("ACMMP_INTERP")) kp.interp = kp.interp && std::atoi(e) != 0;
    // fast pinhole: each sample's source point from the per-view homogeneous affine form (ncc_chunk);
    // ACMMP_PIN_HOMOG=0 projects it through depth and point per sample instead (A/B, tests)
    kp.homog = 1;
    if (const char* e = std::getenv("ACMMP_PIN_HOMOG")) kp.homog = std::atoi(e) != 0;
    // the interpolation's corner-spread fallback threshold (ncc_chunk); ACMMP_SPREAD_MAX overrides it (tests
    // force fallbacks with a small one, A/B without any with a huge one)
    kp.spread_max = 256.0f;
    if (const char* e = std::getenv("ACMMP_SPREAD_MAX")) kp.spread_max = std::strtof(e, nullptr);
    kp.rows = std::min(c->H, 32 * (((c->H / 2) + 15) / 16));
    kp.row_lo = 0; kp.row_hi = kp.rows;
    kp.init_lo = 0; kp.init_hi = c->H;
    kp.merge_lo = 0; kp.merge_hi = c->H;
    for (int k = 0; k < 2; ++k) { kp.filt_lo[k] = 0; kp.filt_hi[k] = kp.rows; }
    kp.dpitch = c->W + 2 * R;
    kp.depth_min = p.depth_min; kp.depth_max = p.depth_max;
    kp.sigma_spatial = p.sigma_spatial; kp.sigma_color = p.sigma_color;
    kp.top_k = p.top_k;
    kp.geom = p.geom_consistency; kp.planar = p.planar_prior; kp.hier = p.hierarchy; kp.upsample = p.upsample;
    kp.scaled_cols = p.scaled_cols; kp.scaled_rows = p.scaled_rows;
    kp.sw = c->sw; kp.sh = c->sh;
    kp.seed_lo = static_cast<uint32_t>(seed);
    kp.seed_hi = static_cast<uint32_t>(seed >> 32);
    kp.Pc = static_cast<long long>(c->H) * kp.Wh;
    const size_t Pc = static_cast<size_t>(kp.Pc);

    if (kp.S > 64) return fail(c, ACMMP_ERR_UNSUPPORTED, "more than 64 patch samples (patch_size / radius_increment)");
    kp.cams = c->d_cams;
    if (c->dirs_R != R) {
        if (c->model == kSphere) {
            dfree(c->d_dirs);
            HIP_TRY(c, dalloc(c->d_sph_row, static_cast<size_t>(c->H + 2 * R)));
            HIP_TRY(c, dalloc(c->d_sph_col, static_cast<size_t>(c->W + 2 * R)));
        } else {
            HIP_TRY(c, dalloc(c->d_dirs, static_cast<size_t>(c->W + 2 * R) * (c->H + 2 * R)));
        }
        HIP_TRY(c, launch_ray_tables(kp, c->d_dirs, c->d_sph_row, c->d_sph_col, c->stream));
        c->dirs_R = R;
    }
    kp.color_den = 2.0f * p.sigma_color * p.sigma_color;
    HIP_TRY(c, dreserve(c->d_spatial, c->spatial_cap, static_cast<size_t>(c->model == kSphere ? c->H : 1) * kp.S));
    HIP_TRY(c, launch_spatial_table(kp, c->d_spatial, c->stream));
    // queue of k_eval_nb's deferred interpolation fallbacks (pixel << 8 | hypothesis << 5 | view: colour
    // grids below 2^24 pixels), fast SPHERE with interpolated coordinates only: per region (blocks b with
    // b % kNbFixRegions equal) room for every entry its blocks can queue, kNbPix x 8 hypotheses x the
    // launch's views each -- so none is ever dropped (metric 193 MB, C3 656 MB)
    kp.nb_chunk = nb_view_chunk(kp);
    kp.nb_tile = nb_tile_order(kp);
    // the queue's key holds the colour-grid pixel in 24 bits: a larger grid (views of 8192x4096 and up) has no
    // queue, and then k_eval_nb does not interpolate (ncc_chunk interpolates only with somewhere to put its
    // fallbacks).  ACMMP_NBFIX_MAX_PC lowers the limit (a test forces that branch at a small size).
    size_t fix_max_pc = static_cast<size_t>(1) << 24;
    if (const char* e = std::getenv("ACMMP_NBFIX_MAX_PC")) fix_max_pc = std::min<size_t>(fix_max_pc, std::strtoull(e, nullptr, 10));
    const bool fixq = c->model == kSphere && c->math == ACMMP_MATH_FAST && c->tex16 && kp.interp && Pc < fix_max_pc;
    if (!fixq && c->model == kSphere && c->math == ACMMP_MATH_FAST && c->tex16 && kp.interp && Pc >= fix_max_pc) kp.interp = 0;
    const size_t nb_blocks = static_cast<size_t>(nb_block_count(kp.rows, kp.Wh, kp.nb_tile));
    // the refinement's interpolated instance (fast SPHERE, V > 4) queues its survivors' fallback views of
    // [0, ref_split) into the same regions after k_eval_nb's queue is drained: a region's k_eval_ref blocks x
    // kRefSlots survivors x ref_split views.  The room is the larger of the two producers' worst cases (the
    // split can exceed the view chunk: ACMMP_REF_SPLIT_AT / ACMMP_NB_VIEW_CHUNK)
    const int ref_split = ref_split_point(kp.V, Pc, kp.model == kSphere && c->math == ACMMP_MATH_FAST && c->tex16 &&
                                                        kp.interp && kp.V > 4);
    const size_t ref_blocks = (static_cast<size_t>(kp.rows) * kp.Wh + kRefPix - 1) / kRefPix;
    const size_t fix_cap = !fixq ? 0 : std::max(
        (nb_blocks + kNbFixRegions - 1) / kNbFixRegions * kNbPix * 8 * static_cast<size_t>(kp.nb_chunk),
        (ref_blocks + kNbFixRegions - 1) / kNbFixRegions * kRefSlots * static_cast<size_t>(std::max(ref_split, 0)));
    // half-sweep scratch slab: carve the pieces of engine.h's KParams out of one allocation
    size_t off[18];
    {
        const size_t VP = static_cast<size_t>(kp.V) * Pc;
        const size_t sizes[17] = {sizeof(float) * 8 * VP, sizeof(int) * 8 * Pc,
                                  sizeof(float4) * 5 * Pc, sizeof(float) * 5 * Pc, sizeof(float) * 5 * Pc,
                                  sizeof(PixState) * Pc, sizeof(float) * VP, sizeof(float) * VP,
                                  sizeof(float) * 5 * VP, sizeof(uint32_t) * (5 * Pc + 256),
                                  sizeof(unsigned) * (Pc / 51 + 2),
                                  sizeof(float4) * Pc, sizeof(uint32_t) * kNbFixRegions * fix_cap,
                                  sizeof(unsigned) * kNbFixRegions,
                                  sizeof(unsigned) * (Pc / 51 + 3), sizeof(uint32_t) * (5 * Pc + 256),
                                  sizeof(uint32_t) * 5 * Pc};
        off[0] = 0;
        for (int k = 0; k < 17; ++k) off[k + 1] = (off[k] + sizes[k] + 255) & ~static_cast<size_t>(255);
    }
    if (c->scratch_bytes < off[17]) {
        HIP_TRY(c, dalloc(c->d_scratch, off[17]));
        c->scratch_bytes = off[17];
    }
    kp.cams = c->d_cams;
    kp.tex16 = c->tex16;
    kp.fast = c->math == ACMMP_MATH_FAST;
    kp.dep = c->d_dep;
    kp.dirs = c->d_dirs;
    kp.sph_row = c->d_sph_row;
    kp.sph_col = c->d_sph_col;
    kp.spatial = c->d_spatial;
    kp.planes_rm = c->d_planes_rm; kp.w_rm = c->d_w_rm; kp.costs_rm = c->d_costs_rm; kp.pre_rm = c->d_pre; kp.sel_rm = c->d_sel_rm;
    kp.scaled = c->d_scaled; kp.prior = c->d_prior; kp.mask = c->d_mask;
    for (int k = 0; k < 2; ++k) {
        kp.plane_cs[k] = c->d_plane_cs[k][0];
        kp.cost_cs[k] = c->d_cost_cs[k][0];
        kp.sel_cs[k] = c->d_sel_cs[k];
        kp.rng_cs[k] = c->d_rng_cs[k];
    }
    kp.hyp_cost = reinterpret_cast<float*>(c->d_scratch + off[0]);
    kp.nbpos = reinterpret_cast<int*>(c->d_scratch + off[1]);
    kp.cand = reinterpret_cast<float4*>(c->d_scratch + off[2]);
    kp.cand_dep = reinterpret_cast<float*>(c->d_scratch + off[3]);
    kp.cand_cost = reinterpret_cast<float*>(c->d_scratch + off[4]);
    kp.pst = reinterpret_cast<PixState*>(c->d_scratch + off[5]);
    kp.cvec[0] = reinterpret_cast<float*>(c->d_scratch + off[6]);
    kp.cvec[1] = reinterpret_cast<float*>(c->d_scratch + off[7]);
    kp.cand_vcost = reinterpret_cast<float*>(c->d_scratch + off[8]);
    kp.surv = reinterpret_cast<uint32_t*>(c->d_scratch + off[9]);
    kp.surv_count = reinterpret_cast<unsigned*>(c->d_scratch + off[10]);
    kp.psum = reinterpret_cast<float4*>(c->d_scratch + off[11]);
    kp.nbfix = fixq ? reinterpret_cast<uint32_t*>(c->d_scratch + off[12]) : nullptr;
    kp.nbfix_count = reinterpret_cast<unsigned*>(c->d_scratch + off[13]);
    kp.surv_pre = reinterpret_cast<unsigned*>(c->d_scratch + off[14]);
    kp.surv_dense = reinterpret_cast<uint32_t*>(c->d_scratch + off[15]);
    kp.cand_rough = reinterpret_cast<uint32_t*>(c->d_scratch + off[16]);
    kp.nbfix_cap = static_cast<unsigned>(fix_cap);
    kp.ref_split = ref_split;
    if (!c->d_work) HIP_TRY(c, dalloc(c->d_work, 257));
    kp.work = c->d_work;
    kp.status = reinterpret_cast<unsigned*>(c->d_work + 256);
    kp.nb_views = kp.V >= 32 ? 0xFFFFFFFFu : ((1u << kp.V) - 1u);
    kp.nb_count_work = 1;
    return ACMMP_OK;
}

acmmp_status acmmp_run_patchmatch_ex(acmmp_ctx* c, uint64_t seed, int n_half_sweeps, int do_post) {
    if (!c) return ACMMP_ERR_INVALID_ARGUMENT;
    HIP_TRY(c, hipSetDevice(c->device));
    KParams kp;
    acmmp_status st = build_kparams(c, kp, seed);
    if (st != ACMMP_OK) return st;
    if (n_half_sweeps < 0) n_half_sweeps = 2 * c->params.max_iterations;
    const size_t Pc = static_cast<size_t>(kp.Pc);
    hipStream_t s = c->stream;
    HIP_TRY(c, hipMemsetAsync(c->d_work, 0, sizeof(unsigned long long) * 257, s));
    HIP_TRY(c, hipEventRecord(c->ev[0], s));
    HIP_TRY(c, launch_init(kp, s));
    // rows outside the reference's checkerboard grid are never rewritten: keep both buffers equal
    int cur[2] = {0, 0};
    for (int k = 0; k < 2; ++k) {
        HIP_TRY(c, hipMemcpyAsync(c->d_plane_cs[k][1], c->d_plane_cs[k][0], sizeof(float4) * Pc,
                                  hipMemcpyDeviceToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(c->d_cost_cs[k][1], c->d_cost_cs[k][0], sizeof(float) * Pc,
                                  hipMemcpyDeviceToDevice, s));
    }
    while (c->kev.size() < static_cast<size_t>(5 * n_half_sweeps)) {
        hipEvent_t e = nullptr;
        HIP_TRY(c, hipEventCreate(&e));
        c->kev.push_back(e);
    }
    // per-kernel events: the k_eval_nb bucket always (the bench's roofline prices it); the other three buckets with
    // ACMMP_KERNEL_TIMING=all in the environment (read per run) -- an event record between two kernels leaves the
    // GPU idle ~6 us, 3 x 6 per half-sweep (0.45% of the metric's RunPatchMatch, profiles/r06_ab9_events_ab.txt)
    const char* e_kt = std::getenv("ACMMP_KERNEL_TIMING");
    const bool time_all = e_kt && std::strcmp(e_kt, "all") == 0;
    HIP_TRY(c, hipEventRecord(c->ev[1], s));
    for (int sw = 0; sw < n_half_sweeps; ++sw) {
        const int colour = sw & 1, iter = sw / 2;
        SweepOut out{c->d_plane_cs[colour][cur[colour] ^ 1], c->d_cost_cs[colour][cur[colour] ^ 1]};
        HIP_TRY(c, launch_propagate(kp, colour, iter, out, s, &c->kev[5 * sw], time_all));
        cur[colour] ^= 1;
        kp.plane_cs[colour] = c->d_plane_cs[colour][cur[colour]];
        kp.cost_cs[colour] = c->d_cost_cs[colour][cur[colour]];
    }
    HIP_TRY(c, hipEventRecord(c->ev[2], s));
    HIP_TRY(c, launch_post(kp, do_post, s));
    HIP_TRY(c, hipEventRecord(c->ev[3], s));
    // the work counters and status word come back in the same wait as the kernels (a blocking copy after the
    // synchronize cost a second host round trip, ~40 us of idle GPU per run)
    if (!c->h_work) HIP_TRY(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_work), sizeof(unsigned long long) * 257,
                                             hipHostMallocDefault));
    HIP_TRY(c, hipMemcpyAsync(c->h_work, c->d_work, sizeof(unsigned long long) * 257, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    // keep buffer 0 current for the next run
    for (int k = 0; k < 2; ++k) {
        if (cur[k]) {
            std::swap(c->d_plane_cs[k][0], c->d_plane_cs[k][1]);
            std::swap(c->d_cost_cs[k][0], c->d_cost_cs[k][1]);
        }
    }
    for (int i = 0; i < 3; ++i) HIP_TRY(c, hipEventElapsedTime(&c->timing[i], c->ev[i], c->ev[i + 1]));
    {
        const unsigned long long* w = c->h_work;
        if (w[256]) return fail(c, ACMMP_ERR_HIP, "run status " + std::to_string(w[256]) + ": an interpolation fallback queue overflowed");
        c->has_result = true;
        c->work_busy = 0;
        for (int k = 0; k < 256; ++k) c->work_busy += w[k];
        c->work_total = 0;
        for (int sw = 0; sw < n_half_sweeps; ++sw) c->work_total += colour_pixels(c, kp, sw & 1);
    }
    for (int k = 0; k < 4; ++k) { c->ktiming[k] = 0.f; c->klaunch[k] = k == 0 || time_all ? n_half_sweeps : 0; }
    for (int sw = 0; sw < n_half_sweeps; ++sw)
        for (int k = 0; k < (time_all ? 4 : 1); ++k) {
            float ms = 0.f;
            HIP_TRY(c, hipEventElapsedTime(&ms, c->kev[5 * sw + k], c->kev[5 * sw + k + 1]));
            c->ktiming[k] += ms;
        }
    return ACMMP_OK;
}

acmmp_status acmmp_run_patchmatch(acmmp_ctx* c, uint64_t seed) { return acmmp_run_patchmatch_ex(c, seed, -1, 1); }

// ------------------------------------------------------------------ row-band split
//
// One reference view over several contexts (GPUs), each updating the image rows [lo, hi) of the
// checkerboard grid.  A pixel's update reads other pixels' plane / cost / selected views at most
// ACMMP_BAND_HALO rows away (the far neighbour scan reaches 3 + 2 * 10 rows, ACMMP.cu:971-979), so after
// each half-sweep a context receives the updated colour's rows [lo - 23, lo) and [hi, hi + 23) from its
// neighbours; everything else a band reads is per pixel (init, RNG, images, priors) and is computed
// locally on band +- halo.  The post stage needs the other colour within 5 rows for the median filter,
// whose black pass feeds the red one: merge covers band +- 10 rows and the black filter band +- 5.  The
// band's rows then equal the whole-view run's bit for bit (tests/test_gpu_band.py).

}  // extern "C"

namespace {

void band_ranges(const KParams& kp, int lo, int hi, int& sup_a, int& sup_b, int& rup_a, int& rup_b, int& sdn_a,
                 int& sdn_b, int& rdn_a, int& rdn_b) {
    const int h = ACMMP_BAND_HALO, rows = kp.rows;
    sup_a = std::min(lo, rows); sup_b = std::min(std::min(lo + h, hi), rows);        // to the band above
    rup_a = std::min(std::max(0, lo - h), rows); rup_b = std::min(lo, rows);         // from it
    sdn_a = std::min(std::max(lo, hi - h), rows); sdn_b = std::min(hi, rows);        // to the band below
    rdn_a = std::min(hi, rows); rdn_b = std::min(hi + h, rows);                      // from it
    if (lo == 0) sup_a = sup_b = rup_a = rup_b = 0;
    if (hi >= kp.H) sdn_a = sdn_b = rdn_a = rdn_b = 0;
}

}  // namespace

acmmp_status acmmp::engine_stream(acmmp_ctx* c, int* device, hipStream_t* stream) {
    if (!c || !device || !stream) return ACMMP_ERR_INVALID_ARGUMENT;
    *device = c->device;
    *stream = c->stream;
    return ACMMP_OK;
}

acmmp_status acmmp::band_buffers(acmmp_ctx* c, int colour, BandBuffers* b) {
    if (!c || !b || colour < 0 || colour > 1) return ACMMP_ERR_INVALID_ARGUMENT;
    if (!c->band_active) return fail(c, ACMMP_ERR_STATE, "no band run in progress");
    b->plane = c->d_plane_cs[colour][c->band_cur[colour]];
    b->cost = c->d_cost_cs[colour][c->band_cur[colour]];
    b->sel = c->d_sel_cs[colour];
    b->Wh = c->band_kp.Wh;
    b->stream = c->stream;
    b->device = c->device;
    return ACMMP_OK;
}

extern "C" {

acmmp_status acmmp_band_begin(acmmp_ctx* c, uint64_t seed, int row0, int row1) {
    if (!c) return ACMMP_ERR_INVALID_ARGUMENT;
    if (c->N == 0) return fail(c, ACMMP_ERR_STATE, "upload_views first");
    if (row0 < 0 || row1 > c->H || row0 >= row1) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "band rows outside the image");
    if (!(row0 == 0 && row1 == c->H) && row1 - row0 < ACMMP_BAND_HALO)
        return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "a band must span at least ACMMP_BAND_HALO rows");
    HIP_TRY(c, hipSetDevice(c->device));
    KParams& kp = c->band_kp;
    acmmp_status st = build_kparams(c, kp, seed);
    if (st != ACMMP_OK) return st;
    const int h = ACMMP_BAND_HALO, rows = kp.rows, H = c->H;
    kp.row_lo = std::min(row0, rows); kp.row_hi = std::min(row1, rows);
    kp.init_lo = std::max(0, row0 - h); kp.init_hi = std::min(H, row1 + h);
    kp.merge_lo = std::max(0, row0 - 10); kp.merge_hi = std::min(H, row1 + 10);
    kp.filt_lo[0] = std::min(std::max(0, row0 - 5), rows); kp.filt_hi[0] = std::min(row1 + 5, rows);
    kp.filt_lo[1] = kp.row_lo; kp.filt_hi[1] = kp.row_hi;
    const size_t Pc = static_cast<size_t>(kp.Pc);
    hipStream_t s = c->stream;
    HIP_TRY(c, hipMemsetAsync(c->d_work, 0, sizeof(unsigned long long) * 257, s));
    HIP_TRY(c, hipEventRecord(c->ev[0], s));
    HIP_TRY(c, launch_init(kp, s));
    for (int k = 0; k < 2; ++k) {
        HIP_TRY(c, hipMemcpyAsync(c->d_plane_cs[k][1], c->d_plane_cs[k][0], sizeof(float4) * Pc, hipMemcpyDeviceToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(c->d_cost_cs[k][1], c->d_cost_cs[k][0], sizeof(float) * Pc, hipMemcpyDeviceToDevice, s));
    }
    HIP_TRY(c, hipEventRecord(c->ev[1], s));
    c->band_lo = row0; c->band_hi = row1;
    c->band_sw = 0; c->band_nsw = 2 * c->params.max_iterations;
    c->band_cur[0] = c->band_cur[1] = 0;
    c->band_active = true;
    return ACMMP_OK;
}

acmmp_status acmmp_band_sweep(acmmp_ctx* c, int* colour_out) {
    if (!c) return ACMMP_ERR_INVALID_ARGUMENT;
    if (!c->band_active) return fail(c, ACMMP_ERR_STATE, "band_begin first");
    if (c->band_sw >= c->band_nsw) return fail(c, ACMMP_ERR_STATE, "every half-sweep of the run is done");
    HIP_TRY(c, hipSetDevice(c->device));
    KParams& kp = c->band_kp;
    const int sw = c->band_sw, colour = sw & 1, iter = sw / 2;
    int* cur = c->band_cur;
    SweepOut out{c->d_plane_cs[colour][cur[colour] ^ 1], c->d_cost_cs[colour][cur[colour] ^ 1]};
    HIP_TRY(c, launch_propagate(kp, colour, iter, out, c->stream, nullptr));
    cur[colour] ^= 1;
    kp.plane_cs[colour] = c->d_plane_cs[colour][cur[colour]];
    kp.cost_cs[colour] = c->d_cost_cs[colour][cur[colour]];
    ++c->band_sw;
    if (colour_out) *colour_out = colour;
    return ACMMP_OK;
}

int acmmp_band_sweeps_left(const acmmp_ctx* c) { return c && c->band_active ? c->band_nsw - c->band_sw : 0; }

acmmp_status acmmp_band_halo_ranges(const acmmp_ctx* c, int ranges[8]) {
    if (!c || !ranges) return ACMMP_ERR_INVALID_ARGUMENT;
    if (!c->band_active) return ACMMP_ERR_STATE;
    band_ranges(c->band_kp, c->band_lo, c->band_hi, ranges[0], ranges[1], ranges[2], ranges[3], ranges[4], ranges[5],
                ranges[6], ranges[7]);
    return ACMMP_OK;
}

acmmp_status acmmp_band_copy_rows(acmmp_ctx* dst, acmmp_ctx* src, int colour, int row_a, int row_b) {
    if (!dst || !src || dst == src) return ACMMP_ERR_INVALID_ARGUMENT;
    BandBuffers d{}, s{};
    acmmp_status st = band_buffers(dst, colour, &d);
    if (st == ACMMP_OK) st = band_buffers(src, colour, &s);
    if (st != ACMMP_OK) return st;
    if (d.Wh != s.Wh || dst->H != src->H || row_a < 0 || row_b > dst->H || row_a > row_b)
        return fail(dst, ACMMP_ERR_INVALID_ARGUMENT, "band contexts differ in size or rows out of range");
    if (row_a == row_b) return ACMMP_OK;
    // the source's half-sweep must be complete before its rows are read
    HIP_TRY(src, hipSetDevice(src->device));
    HIP_TRY(src, hipStreamSynchronize(src->stream));
    HIP_TRY(dst, hipSetDevice(dst->device));
    const size_t off = static_cast<size_t>(row_a) * d.Wh, n = static_cast<size_t>(row_b - row_a) * d.Wh;
    HIP_TRY(dst, hipMemcpyAsync(d.plane + off, s.plane + off, sizeof(float4) * n, hipMemcpyDeviceToDevice, dst->stream));
    HIP_TRY(dst, hipMemcpyAsync(d.cost + off, s.cost + off, sizeof(float) * n, hipMemcpyDeviceToDevice, dst->stream));
    HIP_TRY(dst, hipMemcpyAsync(d.sel + off, s.sel + off, sizeof(uint32_t) * n, hipMemcpyDeviceToDevice, dst->stream));
    return ACMMP_OK;
}

acmmp_status acmmp_band_get_rows(acmmp_ctx* c, int colour, int row_a, int row_b, float* planes, float* costs,
                                 uint32_t* sel) {
    if (!c || !planes || !costs || !sel) return ACMMP_ERR_INVALID_ARGUMENT;
    BandBuffers b{};
    const acmmp_status st = band_buffers(c, colour, &b);
    if (st != ACMMP_OK) return st;
    if (row_a < 0 || row_b > c->H || row_a > row_b) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "rows out of range");
    if (row_a == row_b) return ACMMP_OK;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));            // the half-sweep that wrote them is complete
    const size_t off = static_cast<size_t>(row_a) * b.Wh, n = static_cast<size_t>(row_b - row_a) * b.Wh;
    HIP_TRY(c, d2h(planes, b.plane + off, sizeof(float4) * n));
    HIP_TRY(c, d2h(costs, b.cost + off, sizeof(float) * n));
    HIP_TRY(c, d2h(sel, b.sel + off, sizeof(uint32_t) * n));
    return ACMMP_OK;
}

acmmp_status acmmp_band_set_rows(acmmp_ctx* c, int colour, int row_a, int row_b, const float* planes, const float* costs,
                                 const uint32_t* sel) {
    if (!c || !planes || !costs || !sel) return ACMMP_ERR_INVALID_ARGUMENT;
    BandBuffers b{};
    const acmmp_status st = band_buffers(c, colour, &b);
    if (st != ACMMP_OK) return st;
    if (row_a < 0 || row_b > c->H || row_a > row_b) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "rows out of range");
    if (row_a == row_b) return ACMMP_OK;
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t off = static_cast<size_t>(row_a) * b.Wh, n = static_cast<size_t>(row_b - row_a) * b.Wh;
    HIP_TRY(c, hipMemcpyAsync(b.plane + off, planes, sizeof(float4) * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(b.cost + off, costs, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(b.sel + off, sel, sizeof(uint32_t) * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));            // the caller's (pageable) buffers may go next
    return ACMMP_OK;
}

acmmp_status acmmp_band_end(acmmp_ctx* c, int do_post) {
    if (!c) return ACMMP_ERR_INVALID_ARGUMENT;
    if (!c->band_active) return fail(c, ACMMP_ERR_STATE, "band_begin first");
    HIP_TRY(c, hipSetDevice(c->device));
    KParams& kp = c->band_kp;
    hipStream_t s = c->stream;
    HIP_TRY(c, hipEventRecord(c->ev[2], s));
    HIP_TRY(c, launch_post(kp, do_post, s));
    HIP_TRY(c, hipEventRecord(c->ev[3], s));
    HIP_TRY(c, hipStreamSynchronize(s));
    for (int k = 0; k < 2; ++k) {
        if (c->band_cur[k]) {
            std::swap(c->d_plane_cs[k][0], c->d_plane_cs[k][1]);
            std::swap(c->d_cost_cs[k][0], c->d_cost_cs[k][1]);
        }
    }
    for (int i = 0; i < 3; ++i) HIP_TRY(c, hipEventElapsedTime(&c->timing[i], c->ev[i], c->ev[i + 1]));
    c->band_active = false;
    unsigned long long status = 0;
    HIP_TRY(c, hipMemcpy(&status, c->d_work + 256, sizeof status, hipMemcpyDeviceToHost));
    if (status) return fail(c, ACMMP_ERR_HIP, "band run status " + std::to_string(status) + ": an interpolation fallback queue overflowed");
    c->has_result = true;
    return ACMMP_OK;
}

acmmp_status acmmp_download(acmmp_ctx* c, float* planes, float* costs) {
    if (!c) return ACMMP_ERR_INVALID_ARGUMENT;
    if (c->N == 0) return fail(c, ACMMP_ERR_STATE, "nothing to download");
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t P = P_of(c);
    if (planes) HIP_TRY(c, d2h(planes, c->d_planes_rm, sizeof(float4) * P));
    if (costs) HIP_TRY(c, d2h(costs, c->d_costs_rm, sizeof(float) * P));
    return ACMMP_OK;
}

acmmp_status acmmp_download_aux(acmmp_ctx* c, uint32_t* sel, float* pre) {
    if (!c) return ACMMP_ERR_INVALID_ARGUMENT;
    if (c->N == 0) return fail(c, ACMMP_ERR_STATE, "nothing to download");
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t P = P_of(c);
    if (sel) HIP_TRY(c, d2h(sel, c->d_sel_rm, sizeof(uint32_t) * P));
    if (pre) HIP_TRY(c, d2h(pre, c->d_pre, sizeof(float) * P));
    return ACMMP_OK;
}

acmmp_status acmmp_device_outputs(acmmp_ctx* c, void** planes, void** costs) {
    if (!c) return ACMMP_ERR_INVALID_ARGUMENT;
    if (planes) *planes = c->d_planes_rm;
    if (costs) *costs = c->d_costs_rm;
    return ACMMP_OK;
}

acmmp_status acmmp_synchronize(acmmp_ctx* c) {
    if (!c) return ACMMP_ERR_INVALID_ARGUMENT;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipDeviceSynchronize());
    return ACMMP_OK;
}

acmmp_status acmmp_last_timing(const acmmp_ctx* c, float ms[3]) {
    if (!c || !ms) return ACMMP_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < 3; ++i) ms[i] = c->timing[i];
    return ACMMP_OK;
}

acmmp_status acmmp_last_planar_timing(const acmmp_ctx* c, float ms[4]) {
    if (!c || !ms) return ACMMP_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < 4; ++i) ms[i] = c->planar_ms[i];
    return ACMMP_OK;
}

acmmp_status acmmp_last_work(const acmmp_ctx* c, unsigned long long* evaluated, unsigned long long* total) {
    if (!c || !evaluated || !total) return ACMMP_ERR_INVALID_ARGUMENT;
    *evaluated = c->work_busy;
    *total = c->work_total;
    return ACMMP_OK;
}

int acmmp_texel_bytes(const acmmp_ctx* c) {
    if (!c || c->N == 0) return 0;
    return c->tex16 ? 2 : 4;
}

acmmp_status acmmp_last_kernel_timing(const acmmp_ctx* c, float ms[4], int launches[4]) {
    if (!c || !ms || !launches) return ACMMP_ERR_INVALID_ARGUMENT;
    for (int k = 0; k < 4; ++k) { ms[k] = c->ktiming[k]; launches[k] = c->klaunch[k]; }
    return ACMMP_OK;
}

acmmp_status acmmp_jbu(acmmp_ctx* c, const float* ref, int W, int H, const float* coarse, int sw, int sh,
                       int imagescale, float* out) {
    if (!c || !ref || !coarse || !out || W <= 0 || H <= 0 || sw <= 0 || sh <= 0 || imagescale < 0)
        return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "bad JBU arguments");
    HIP_TRY(c, hipSetDevice(c->device));
    float *d_ref = nullptr, *d_coarse = nullptr, *d_out = nullptr;
    const size_t P = static_cast<size_t>(W) * H, p = static_cast<size_t>(sw) * sh;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&d_ref), sizeof(float) * P);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d_coarse), sizeof(float) * p);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d_out), sizeof(float) * P);
    if (e == hipSuccess) e = hipMemcpy(d_ref, ref, sizeof(float) * P, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_coarse, coarse, sizeof(float) * p, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_jbu(d_ref, W, H, d_coarse, sw, sh, imagescale, d_out, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = d2h(out, d_out, sizeof(float) * P);
    dfree(d_ref); dfree(d_coarse); dfree(d_out);
    if (e != hipSuccess) return fail(c, ACMMP_ERR_HIP, std::string("jbu: ") + hipGetErrorString(e));
    return ACMMP_OK;
}

// which: 0 = NCC (per-sample projection), 1 = geom cost, 2 = k_eval_nb's NCC on n pixels x 8 planes,
// 3 = the refinement's NCC (k_eval_ref + the tail's fallbacks) on n pixels x 5 planes
static acmmp_status debug_eval(acmmp_ctx* c, int which, int n, const int* px, const int* py, const float* planes,
                               float* out) {
    if (!c || !px || !py || !planes || !out || n <= 0) return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "bad debug args");
    HIP_TRY(c, hipSetDevice(c->device));
    KParams kp;
    acmmp_status st = build_kparams(c, kp, 0);
    if (st != ACMMP_OK) return st;
    for (int q = 0; q < n; ++q)
        if (px[q] < 0 || py[q] < 0 || px[q] >= c->W || py[q] >= c->H)
            return fail(c, ACMMP_ERR_INVALID_ARGUMENT, "query pixel outside the reference image");
    if (which == 1 && !c->has_depths) return fail(c, ACMMP_ERR_STATE, "geom cost needs upload_depths");
    int *dx = nullptr, *dy = nullptr;
    float4* dp = nullptr;
    float* dout = nullptr;
    const int per = which == 2 ? 8 : (which == 3 ? 5 : 1);   // planes per query pixel
    const size_t nout = static_cast<size_t>(n) * per * kp.V;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&dx), sizeof(int) * n);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&dy), sizeof(int) * n);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&dp), sizeof(float4) * n * per);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&dout), sizeof(float) * nout);
    if (e == hipSuccess) e = hipMemcpy(dx, px, sizeof(int) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dy, py, sizeof(int) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dp, planes, sizeof(float4) * n * per, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = which == 2 ? launch_debug_nb(kp, n, dx, dy, dp, dout, c->stream)
          : which == 3 ? launch_debug_ref(kp, n, dx, dy, dp, dout, c->stream)
                       : launch_debug(kp, which, n, dx, dy, dp, dout, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = d2h(out, dout, sizeof(float) * nout);
    dfree(dx); dfree(dy); dfree(dp); dfree(dout);
    if (e != hipSuccess) return fail(c, ACMMP_ERR_HIP, std::string("debug: ") + hipGetErrorString(e));
    return ACMMP_OK;
}

acmmp_status acmmp_debug_ncc(acmmp_ctx* c, int n, const int* px, const int* py, const float* planes, float* costs) {
    return debug_eval(c, 0, n, px, py, planes, costs);
}
acmmp_status acmmp_debug_geom(acmmp_ctx* c, int n, const int* px, const int* py, const float* planes, float* out) {
    return debug_eval(c, 1, n, px, py, planes, out);
}
acmmp_status acmmp_debug_ncc_nb(acmmp_ctx* c, int n, const int* px, const int* py, const float* planes, float* costs) {
    return debug_eval(c, 2, n, px, py, planes, costs);
}
acmmp_status acmmp_debug_ncc_ref(acmmp_ctx* c, int n, const int* px, const int* py, const float* planes, float* costs) {
    return debug_eval(c, 3, n, px, py, planes, costs);
}

}  // extern "C"
