// ACMMP.hpp -- C++ mirror of the reference's ACMMP class (ACMMP.h:57-111) over the C ABI.
//
// Header-only, OpenCV-free.  Method names, call order and argument meaning follow the
// reference so ProcessProblem (main.cpp:73-210) ports line for line.
// Images are passed already decoded (float grey, 0..255) instead of read from JPEG.
// Errors keep the reference's CUDA_SAFE_CALL behaviour (ACMMP.cpp:64-72): print and exit.
#pragma once

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/acmmp.h"

namespace acmmp_host {

using Camera = acmmp_camera;                 // main.h:40-54
using PatchMatchParams = acmmp_params;       // ACMMP.h:32-55

struct Float4 { float x, y, z, w; };         // the reference's float4 plane hypothesis
struct Point { int x, y; };                  // cv::Point
struct Triangle { Point pt1, pt2, pt3; };    // main.h:66-69

// In-class defaults of PatchMatchParams (ACMMP.h:33-54).
inline PatchMatchParams DefaultParams() {
    PatchMatchParams p;
    std::memset(&p, 0, sizeof p);
    p.max_iterations = 3; p.patch_size = 11; p.num_images = 5; p.max_image_size = 3200;
    p.radius_increment = 2; p.sigma_spatial = 5.0f; p.sigma_color = 3.0f; p.top_k = 4;
    p.baseline = 0.54f; p.depth_min = 0.0f; p.depth_max = 1.0f; p.disparity_min = 0.0f; p.disparity_max = 1.0f;
    return p;
}

inline void SafeCall(acmmp_status s, const acmmp_ctx* ctx, const char* file, int line) {
    if (s != ACMMP_OK) {
        std::printf("%s in %s at line %i (%s)\n", acmmp_status_str(s), file, line, ctx ? acmmp_last_error(ctx) : "");
        std::exit(EXIT_FAILURE);
    }
}
#define ACMMP_SAFE_CALL(expr) ::acmmp_host::SafeCall((expr), ctx_, __FILE__, __LINE__)

struct Image {                               // one decoded grey view
    int width = 0, height = 0;
    std::vector<float> data;                 // row-major, width * height
};

class ACMMP {
public:
    explicit ACMMP(int device = 0) : params_(DefaultParams()) { ACMMP_SAFE_CALL(acmmp_create(device, &ctx_)); }
    ~ACMMP() { acmmp_destroy(ctx_); }
    ACMMP(const ACMMP&) = delete;
    ACMMP& operator=(const ACMMP&) = delete;

    // ACMMP.cpp:548-565
    void SetGeomConsistencyParams(bool multi_geometry = false) {
        params_.geom_consistency = 1;
        params_.max_iterations = 2;
        if (multi_geometry) params_.multi_geometry = 1;
    }
    void SetHierarchyParams() { params_.hierarchy = 1; }
    void SetPlanarPriorParams() { params_.planar_prior = 1; }

    // InuputInitialization (ACMMP.cpp:567-679) after decoding/rescaling: images[0] is the reference,
    // cameras already scaled to the image sizes.  depths (geom) are the previous pass's maps.
    void InuputInitialization(const std::vector<Image>& images, const std::vector<Camera>& cameras,
                              const std::vector<Image>* depths = nullptr) {
        images_ = images;
        cameras_ = cameras;
        params_.depth_min = cameras_[0].depth_min * 0.6f;                 // ACMMP.cpp:645-646
        params_.depth_max = cameras_[0].depth_max * 1.2f;
        params_.num_images = static_cast<int>(images_.size());
        params_.disparity_min = cameras_[0].K[0] * params_.baseline / params_.depth_max;
        params_.disparity_max = cameras_[0].K[0] * params_.baseline / params_.depth_min;
        if (depths) depths_ = *depths;
    }

    // CudaSpaceInitialization (ACMMP.cpp:681-845): upload views (+ geom depths / reloaded state).
    // `state` = (normal, depth) planes and costs of the previous pass for geom / hierarchy reuse;
    // `scaled` = coarse (normal, cost or depth) planes for hierarchy (ACMMP.cpp:816-831).
    void CudaSpaceInitialization(const std::vector<Float4>* state = nullptr, const std::vector<float>* costs = nullptr,
                                 const std::vector<Float4>* scaled = nullptr, int scaled_w = 0, int scaled_h = 0) {
        std::vector<const float*> ptrs;
        for (auto& im : images_) ptrs.push_back(im.data.data());
        ACMMP_SAFE_CALL(acmmp_set_params(ctx_, &params_));
        ACMMP_SAFE_CALL(acmmp_upload_views(ctx_, static_cast<int>(images_.size()), ptrs.data(), nullptr,
                                           cameras_.data()));
        if (params_.geom_consistency) {
            std::vector<const float*> dp;
            std::vector<int> w, h;
            for (auto& d : depths_) { dp.push_back(d.data.data()); w.push_back(d.width); h.push_back(d.height); }
            ACMMP_SAFE_CALL(acmmp_upload_depths(ctx_, static_cast<int>(dp.size()), dp.data(), w.data(), h.data()));
        }
        if (state || costs)
            ACMMP_SAFE_CALL(acmmp_set_state(ctx_, state ? &(*state)[0].x : nullptr, costs ? costs->data() : nullptr));
        if (scaled) {
            if (scaled_w != images_[0].width || scaled_h != images_[0].height) {
                params_.upsample = 1;
                params_.scaled_cols = static_cast<float>(scaled_w);
                params_.scaled_rows = static_cast<float>(scaled_h);
            } else {
                params_.upsample = 0;
            }
            ACMMP_SAFE_CALL(acmmp_set_params(ctx_, &params_));
            ACMMP_SAFE_CALL(acmmp_set_scaled_state(ctx_, &(*scaled)[0].x, scaled_w, scaled_h));
        }
    }

    // CudaPlanarPriorInitialization (ACMMP.cpp:847-867): PlaneParams indexed by mask label - 1.
    void CudaPlanarPriorInitialization(const std::vector<Float4>& plane_params, const std::vector<float>& masks) {
        const size_t P = static_cast<size_t>(GetReferenceImageWidth()) * GetReferenceImageHeight();
        std::vector<Float4> prior(P, Float4{0, 0, 0, 0});
        std::vector<uint32_t> m(P, 0);
        for (size_t i = 0; i < P; ++i) {
            m[i] = static_cast<uint32_t>(masks[i]);
            if (masks[i] > 0) prior[i] = plane_params[static_cast<size_t>(masks[i]) - 1];
        }
        ACMMP_SAFE_CALL(acmmp_set_params(ctx_, &params_));
        ACMMP_SAFE_CALL(acmmp_set_planar_prior(ctx_, &prior[0].x, m.data()));
    }

    // RunPatchMatch (ACMMP.cu:1506-1556): runs and copies the result back like the reference.
    // The reference seeds its generators from clock64() (ACMMP.cu:684); here the seed is explicit.
    void RunPatchMatch(uint64_t seed = 1234) {
        ACMMP_SAFE_CALL(acmmp_set_params(ctx_, &params_));
        ACMMP_SAFE_CALL(acmmp_run_patchmatch(ctx_, seed));
        const size_t P = static_cast<size_t>(GetReferenceImageWidth()) * GetReferenceImageHeight();
        planes_.resize(P);
        costs_.resize(P);
        ACMMP_SAFE_CALL(acmmp_download(ctx_, &planes_[0].x, costs_.data()));
    }

    // Planar-prior host helpers (ACMMP.cpp:904-1011) over the C ABI's host functions.
    void GetSupportPoints(std::vector<Point>& support2DPoints) const {
        int n = 0;
        acmmp_support_points(costs_.data(), GetReferenceImageWidth(), GetReferenceImageHeight(), nullptr, 0, &n);
        std::vector<int> xy(2 * static_cast<size_t>(n));
        acmmp_support_points(costs_.data(), GetReferenceImageWidth(), GetReferenceImageHeight(), xy.data(), n, &n);
        support2DPoints.resize(n);
        for (int i = 0; i < n; ++i) support2DPoints[i] = Point{xy[2 * i], xy[2 * i + 1]};
    }
    std::vector<Triangle> DelaunayTriangulation(int width, int height, const std::vector<Point>& points) const {
        std::vector<int> xy;
        for (const Point& p : points) { xy.push_back(p.x); xy.push_back(p.y); }
        int m = 0;
        const int n = static_cast<int>(points.size());
        acmmp_delaunay(xy.data(), n, width, height, nullptr, 0, &m);
        std::vector<int> t(6 * static_cast<size_t>(m));
        acmmp_delaunay(xy.data(), n, width, height, t.data(), m, &m);
        std::vector<Triangle> out(m);
        for (int k = 0; k < m; ++k)
            out[k] = Triangle{{t[6 * k], t[6 * k + 1]}, {t[6 * k + 2], t[6 * k + 3]}, {t[6 * k + 4], t[6 * k + 5]}};
        return out;
    }
    Float4 GetPriorPlaneParams(const Triangle& tri, const std::vector<float>& depths) const {
        const int t[6] = {tri.pt1.x, tri.pt1.y, tri.pt2.x, tri.pt2.y, tri.pt3.x, tri.pt3.y};
        Float4 n4{0, 0, 0, 0};
        acmmp_prior_plane_params(&cameras_[0], depths.data(), GetReferenceImageWidth(), GetReferenceImageHeight(), t,
                                 &n4.x);
        return n4;
    }
    float GetDepthFromPlaneParam(const Float4& plane, int x, int y) const {
        return acmmp_depth_from_plane_param(&cameras_[0], &plane.x, x, y);
    }

    int GetReferenceImageWidth() const { return cameras_[0].width; }
    int GetReferenceImageHeight() const { return cameras_[0].height; }
    const Image& GetReferenceImage() const { return images_[0]; }
    Float4 GetPlaneHypothesis(int index) const { return planes_[index]; }
    float GetCost(int index) const { return costs_[index]; }
    float GetMinDepth() const { return params_.depth_min; }
    float GetMaxDepth() const { return params_.depth_max; }
    const PatchMatchParams& params() const { return params_; }

private:
    acmmp_ctx* ctx_ = nullptr;
    PatchMatchParams params_;
    std::vector<Image> images_, depths_;
    std::vector<Camera> cameras_;
    std::vector<Float4> planes_;
    std::vector<float> costs_;
};

#undef ACMMP_SAFE_CALL

}  // namespace acmmp_host
