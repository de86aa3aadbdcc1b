// fusion.cpp -- host object of the GPU depth-map fusion.
//
// Replaces RunFusionCuda's device half (ACMMP.cu:1817-2105): one upload per view of what the
// reference puts into textures (depth, normals, the colour image as float RGBA / 255), then per
// reference view SimpleFusionKernel (`k_fuse`) and an in-order compaction of the valid pixels -- the
// order RunFusionCuda's host loop collects them in (ACMMP.cu:2064-2071).  Everything stays in HBM; only
// the fused points come back.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "acmmp.h"
#include "engine.h"

using namespace acmmp;

struct acmmp_fusion {
    int device = 0, model = 0, n = 0;
    hipStream_t stream = nullptr;
    std::vector<DevCam> cams;
    std::vector<FuseView> views;                 // device pointers
    DevCam* d_cams = nullptr;
    FuseView* d_views = nullptr;
    int* d_srcs = nullptr;
    float* d_dense = nullptr;
    int* d_flags = nullptr;
    int* d_counts = nullptr;
    int* d_offsets = nullptr;
    float* d_out = nullptr;
    size_t cap_P = 0, cap_out = 0;
    std::string err;
};

namespace {

acmmp_status ffail(acmmp_fusion* f, acmmp_status s, const std::string& m) {
    if (f) f->err = m;
    return s;
}

#define F_HIP(f, expr)                                                                          \
    do {                                                                                        \
        const hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                                   \
            return ffail((f), e_ == hipErrorOutOfMemory ? ACMMP_ERR_OUT_OF_MEMORY : ACMMP_ERR_HIP, \
                         std::string(#expr) + ": " + hipGetErrorString(e_));                     \
    } while (0)

template <typename T>
hipError_t fre(T*& p) {
    hipError_t e = hipSuccess;
    if (p) e = hipFree(const_cast<void*>(static_cast<const void*>(p)));
    p = nullptr;
    return e;
}

template <typename T>
hipError_t alloc(T*& p, size_t count) {
    (void)fre(p);
    return hipMalloc(reinterpret_cast<void**>(&p), sizeof(T) * (count ? count : 1));
}

}  // namespace

extern "C" {

acmmp_status acmmp_fusion_create(int device, int n_views, const acmmp_camera* cams, acmmp_fusion** out) {
    if (!out || !cams || n_views < 1) return ACMMP_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) return ACMMP_ERR_NO_DEVICE;
    if (device < 0 || device >= nd) return ACMMP_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < n_views; ++i) {
        if (cams[i].model != ACMMP_PINHOLE && cams[i].model != ACMMP_SPHERE) return ACMMP_ERR_INVALID_ARGUMENT;
        if (cams[i].model != cams[0].model) return ACMMP_ERR_UNSUPPORTED;
        if (cams[i].width <= 0 || cams[i].height <= 0) return ACMMP_ERR_INVALID_ARGUMENT;
    }
    if (hipSetDevice(device) != hipSuccess) return ACMMP_ERR_HIP;
    acmmp_fusion* f = new acmmp_fusion();
    f->device = device;
    f->model = cams[0].model;
    f->n = n_views;
    f->cams.resize(n_views);
    for (int i = 0; i < n_views; ++i) f->cams[i] = make_devcam(cams[i]);
    f->views.assign(n_views, FuseView{nullptr, nullptr, nullptr, 0, 0});
    acmmp_status s = ACMMP_OK;
    if (hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking) != hipSuccess ||
        alloc(f->d_cams, n_views) != hipSuccess || alloc(f->d_views, n_views) != hipSuccess ||
        alloc(f->d_srcs, 32) != hipSuccess ||
        hipMemcpy(f->d_cams, f->cams.data(), sizeof(DevCam) * n_views, hipMemcpyHostToDevice) != hipSuccess)
        s = ACMMP_ERR_HIP;
    if (s != ACMMP_OK) { acmmp_fusion_destroy(f); return s; }
    *out = f;
    return ACMMP_OK;
}

void acmmp_fusion_destroy(acmmp_fusion* f) {
    if (!f) return;
    (void)hipSetDevice(f->device);
    if (f->stream) (void)hipStreamSynchronize(f->stream);
    for (FuseView& v : f->views) { (void)fre(v.depth); (void)fre(v.normal); (void)fre(v.rgba); }
    (void)fre(f->d_cams); (void)fre(f->d_views); (void)fre(f->d_srcs); (void)fre(f->d_dense);
    (void)fre(f->d_flags); (void)fre(f->d_counts); (void)fre(f->d_offsets); (void)fre(f->d_out);
    if (f->stream) (void)hipStreamDestroy(f->stream);
    delete f;
}

const char* acmmp_fusion_last_error(const acmmp_fusion* f) { return f ? f->err.c_str() : ""; }

acmmp_status acmmp_fusion_set_view(acmmp_fusion* f, int view, const float* depth, const float* normals,
                                   const uint8_t* bgr) {
    if (!f || !depth || !normals || !bgr) return ffail(f, ACMMP_ERR_INVALID_ARGUMENT, "null argument");
    if (view < 0 || view >= f->n) return ffail(f, ACMMP_ERR_INVALID_ARGUMENT, "view index out of range");
    F_HIP(f, hipSetDevice(f->device));
    const int W = f->cams[view].W, H = f->cams[view].H;
    const size_t P = static_cast<size_t>(W) * H;
    // the reference's colour texture: cvtColor(BGR2RGBA) + convertTo(CV_32FC4, 1/255) (ACMMP.cu:1950-1953)
    std::vector<float> rgba(4 * P);
    const float s = static_cast<float>(1.0 / 255.0);
    for (size_t i = 0; i < P; ++i) {
        rgba[4 * i + 0] = static_cast<float>(bgr[3 * i + 2]) * s;
        rgba[4 * i + 1] = static_cast<float>(bgr[3 * i + 1]) * s;
        rgba[4 * i + 2] = static_cast<float>(bgr[3 * i + 0]) * s;
        rgba[4 * i + 3] = 255.0f * s;
    }
    FuseView& v = f->views[view];
    float* d = nullptr;
    float* nrm = nullptr;
    float* col = nullptr;
    (void)fre(v.depth); (void)fre(v.normal); (void)fre(v.rgba);
    F_HIP(f, alloc(d, P));
    F_HIP(f, alloc(nrm, 3 * P));
    F_HIP(f, alloc(col, 4 * P));
    v = FuseView{d, nrm, col, W, H};
    F_HIP(f, hipMemcpy(d, depth, sizeof(float) * P, hipMemcpyHostToDevice));
    F_HIP(f, hipMemcpy(nrm, normals, sizeof(float) * 3 * P, hipMemcpyHostToDevice));
    F_HIP(f, hipMemcpy(col, rgba.data(), sizeof(float) * 4 * P, hipMemcpyHostToDevice));
    F_HIP(f, hipMemcpy(f->d_views + view, &v, sizeof(FuseView), hipMemcpyHostToDevice));
    return ACMMP_OK;
}

acmmp_status acmmp_fusion_run(acmmp_fusion* f, int ref, int n_src, const int* src_views, float* points, int cap,
                              int* n_points) {
    if (!f || !n_points || n_src < 0 || n_src > 32 || (n_src > 0 && !src_views) || cap < 0 || (cap > 0 && !points))
        return ffail(f, ACMMP_ERR_INVALID_ARGUMENT, "bad argument");
    if (ref < 0 || ref >= f->n) return ffail(f, ACMMP_ERR_INVALID_ARGUMENT, "reference index out of range");
    for (int j = 0; j < n_src; ++j)
        if (src_views[j] >= f->n) return ffail(f, ACMMP_ERR_INVALID_ARGUMENT, "source index out of range");
    std::vector<int> used(1, ref);
    for (int j = 0; j < n_src; ++j) if (src_views[j] >= 0) used.push_back(src_views[j]);
    for (int v : used)
        if (!f->views[v].depth) return ffail(f, ACMMP_ERR_STATE, "set_view first for every view used");
    F_HIP(f, hipSetDevice(f->device));
    const int W = f->cams[ref].W, H = f->cams[ref].H;
    const size_t P = static_cast<size_t>(W) * H;
    const size_t nblk = (P + 255) / 256;
    if (f->cap_P < P) {
        F_HIP(f, alloc(f->d_dense, 9 * P));
        F_HIP(f, alloc(f->d_flags, P));
        F_HIP(f, alloc(f->d_counts, nblk));
        F_HIP(f, alloc(f->d_offsets, nblk));
        f->cap_P = P;
    }
    hipStream_t s = f->stream;
    if (n_src > 0) F_HIP(f, hipMemcpyAsync(f->d_srcs, src_views, sizeof(int) * n_src, hipMemcpyHostToDevice, s));
    F_HIP(f, launch_fuse(f->model, f->d_cams, f->d_views, ref, W, H, f->d_srcs, n_src, f->d_dense, f->d_flags,
                         f->d_counts, s));
    std::vector<int> counts(nblk);
    F_HIP(f, hipMemcpyAsync(counts.data(), f->d_counts, sizeof(int) * nblk, hipMemcpyDeviceToHost, s));
    F_HIP(f, hipStreamSynchronize(s));
    long long total = 0;
    for (size_t b = 0; b < nblk; ++b) { const int c = counts[b]; counts[b] = static_cast<int>(total); total += c; }
    *n_points = static_cast<int>(total);
    if (total > cap) return ffail(f, ACMMP_ERR_INVALID_ARGUMENT, "points capacity too small");
    if (total == 0) return ACMMP_OK;
    if (f->cap_out < static_cast<size_t>(total)) {
        F_HIP(f, alloc(f->d_out, 9 * static_cast<size_t>(total)));
        f->cap_out = static_cast<size_t>(total);
    }
    F_HIP(f, hipMemcpyAsync(f->d_offsets, counts.data(), sizeof(int) * nblk, hipMemcpyHostToDevice, s));
    F_HIP(f, launch_fuse_compact(W, H, f->d_dense, f->d_flags, f->d_offsets, f->d_out, s));
    F_HIP(f, hipMemcpyAsync(points, f->d_out, sizeof(float) * 9 * total, hipMemcpyDeviceToHost, s));
    F_HIP(f, hipStreamSynchronize(s));
    return ACMMP_OK;
}

}  // extern "C"
