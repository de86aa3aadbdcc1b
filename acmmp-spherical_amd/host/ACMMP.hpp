// ACMMP.hpp -- C++ mirror of the reference's ACMMP class (ACMMP.h:57-111) over the C ABI.
//
// OpenCV-free.  Method names, call order and argument meaning follow the reference, so
// ProcessProblem (main.cpp:73-210) ports line for line -- acmmp_main.cpp is that port.  Two input
// paths:
//   * the reference's: InuputInitialization(dense_folder, problems, idx) reads images/%08d.jpg
//     (jpeg.hpp), cams/%08d_cam.txt (ReadCamera) and, for geom passes, the depths*.dmb of the
//     previous pass; CudaSpaceInitialization(dense_folder, problem) reloads normals/costs/depths
//     .dmb for geom and hierarchy passes (ACMMP.cpp:567-845);
//   * in memory: InuputInitialization(images, cameras[, depths]) with decoded views and
//     CudaSpaceInitialization(state, costs, scaled, ...) with the reloaded state.
// Errors keep the reference's CUDA_SAFE_CALL behaviour (ACMMP.cpp:64-72): print and exit.
// Link: formats.cpp + jpeg.cpp (host) and libacmmp.so (the engine).
#pragma once

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/acmmp.h"
#include "formats.hpp"

namespace acmmp_host {

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

class ACMMP {
public:
    // ACMMP::ACMMP (ACMMP.cpp:99) + cudaSetDevice (main.cpp:77): owns a context on `device`.
    explicit ACMMP(int device = 0) : params_(DefaultParams()), own_(true) {
        ACMMP_SAFE_CALL(acmmp_create(device, &ctx_));
    }
    // Borrow a context (device memory kept across problems; results identical -- every upload
    // resets the per-problem state, see include/acmmp.h).
    explicit ACMMP(acmmp_ctx* shared) : ctx_(shared), params_(DefaultParams()), own_(false) {}
    ~ACMMP() { if (own_) acmmp_destroy(ctx_); }
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

    // ---- the reference's dense-folder path ------------------------------------------------

    // InuputInitialization (ACMMP.cpp:567-679): grey images + cameras of the problem, rescaled to
    // cur_image_size (a source view to ITS problem's size, indexing problems by image id as the
    // reference does, :609); geom passes also read the previous pass's depth maps.
    void InuputInitialization(const std::string& dense_folder, const std::vector<Problem>& problems, int idx) {
        images_.clear();
        cameras_.clear();
        const Problem& problem = problems[idx];
        std::vector<int> ids{problem.ref_image_id};
        ids.insert(ids.end(), problem.src_image_ids.begin(), problem.src_image_ids.end());
        for (int id : ids) {
            Image im = ReadGrayImage(ImagePath(dense_folder, id));
            Camera cam = ReadCamera(CameraPath(dense_folder, id));
            cam.height = im.height;
            cam.width = im.width;
            images_.push_back(std::move(im));
            cameras_.push_back(cam);
        }
        int max_image_size = problems[idx].cur_image_size;
        for (size_t i = 0; i < images_.size(); ++i) {
            if (i > 0) max_image_size = problems[problem.src_image_ids[i - 1]].cur_image_size;
            if (images_[i].width <= max_image_size && images_[i].height <= max_image_size) continue;
            int new_rows, new_cols;
            ScaledDims(images_[i].height, images_[i].width, max_image_size, &new_rows, &new_cols);
            const float scale_x = new_cols / static_cast<float>(images_[i].width);
            const float scale_y = new_rows / static_cast<float>(images_[i].height);
            images_[i] = ResizeLinear(images_[i], new_cols, new_rows);
            if (cameras_[i].model == ACMMP_SPHERE) {
                cameras_[i].params[1] *= scale_x;
                cameras_[i].params[2] *= scale_y;
            } else {
                cameras_[i].K[0] *= scale_x; cameras_[i].K[2] *= scale_x;
                cameras_[i].K[4] *= scale_y; cameras_[i].K[5] *= scale_y;
            }
            cameras_[i].height = new_rows;
            cameras_[i].width = new_cols;
        }
        SetDepthRange();
        if (params_.geom_consistency) {
            depths_.clear();
            const std::string suffix = params_.multi_geometry ? "/depths_geom.dmb" : "/depths.dmb";
            for (int id : ids) {
                FloatMap d;
                readDepthDmb(ResultFolder(dense_folder, id) + suffix, &d);
                depths_.push_back(std::move(d));
            }
        }
    }

    // CudaSpaceInitialization (ACMMP.cpp:681-845): upload; geom passes restart from the stored
    // (normals, depth) planes and costs, hierarchy passes from the coarse scale's normals with
    // the costs (upsample) or depths as .w and the JBU depth as the start depth.
    void CudaSpaceInitialization(const std::string& dense_folder, const Problem& problem) {
        const std::string folder = ResultFolder(dense_folder, problem.ref_image_id);
        if (params_.geom_consistency) {
            FloatMap depth, normal, cost;
            readDepthDmb(folder + (params_.multi_geometry ? "/depths_geom.dmb" : "/depths.dmb"), &depth);
            readNormalDmb(folder + "/normals.dmb", &normal);
            readDepthDmb(folder + "/costs.dmb", &cost);
            const size_t P = static_cast<size_t>(depth.width) * depth.height;
            std::vector<Float4> planes(P);
            for (size_t c = 0; c < P; ++c)
                planes[c] = Float4{normal.data[3 * c], normal.data[3 * c + 1], normal.data[3 * c + 2], depth.data[c]};
            CudaSpaceInitialization(&planes, &cost.data);
        } else if (params_.hierarchy) {
            FloatMap depth, normal, cost;
            readDepthDmb(folder + "/depths.dmb", &depth);
            readNormalDmb(folder + "/normals.dmb", &normal);
            readDepthDmb(folder + "/costs.dmb", &cost);
            const int sw = normal.width, sh = normal.height;
            const bool upsample = sw != images_[0].width || sh != images_[0].height;
            std::vector<Float4> scaled(static_cast<size_t>(sw) * sh);
            for (size_t c = 0; c < scaled.size(); ++c)
                scaled[c] = Float4{normal.data[3 * c], normal.data[3 * c + 1], normal.data[3 * c + 2],
                                   upsample ? cost.data[c] : depth.data[c]};
            // start depth = the JBU map; .xyz is uninitialised in the reference (ACMMP.cpp:833-840),
            // zero here; a depth map of another size (JBU skipped) reads as zeros
            const int W = images_[0].width, H = images_[0].height;
            std::vector<Float4> state(static_cast<size_t>(W) * H, Float4{0, 0, 0, 0});
            if (depth.width == W && depth.height == H)
                for (size_t c = 0; c < state.size(); ++c) state[c].w = depth.data[c];
            CudaSpaceInitialization(&state, nullptr, &scaled, sw, sh);
        } else {
            CudaSpaceInitialization();
        }
    }

    // ---- in-memory path -------------------------------------------------------------------

    // InuputInitialization after decoding/rescaling: images[0] is the reference, cameras already
    // scaled to the image sizes; depths (geom) are the previous pass's maps.
    void InuputInitialization(const std::vector<Image>& images, const std::vector<Camera>& cameras,
                              const std::vector<Image>* depths = nullptr) {
        images_ = images;
        cameras_ = cameras;
        SetDepthRange();
        if (depths) {
            depths_.clear();
            for (const Image& d : *depths) depths_.push_back(FloatMap{d.width, d.height, 1, d.data});
        }
    }

    // `state` = (normal, depth) planes and costs of the previous pass for geom / hierarchy reuse;
    // `scaled` = coarse (normal, cost or depth) planes for hierarchy (ACMMP.cpp:816-831).
    void CudaSpaceInitialization(const std::vector<Float4>* state = nullptr, const std::vector<float>* costs = nullptr,
                                 const std::vector<Float4>* scaled = nullptr, int scaled_w = 0, int scaled_h = 0) {
        if (scaled) {
            if (scaled_w != images_[0].width || scaled_h != images_[0].height) {
                params_.upsample = 1;
                params_.scaled_cols = static_cast<float>(scaled_w);
                params_.scaled_rows = static_cast<float>(scaled_h);
            } else {
                params_.upsample = 0;
            }
        }
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
        if (scaled) ACMMP_SAFE_CALL(acmmp_set_scaled_state(ctx_, &(*scaled)[0].x, scaled_w, scaled_h));
        if (state || costs)
            ACMMP_SAFE_CALL(acmmp_set_state(ctx_, state ? &(*state)[0].x : nullptr, costs ? costs->data() : nullptr));
    }

    // CudaPlanarPriorInitialization (ACMMP.cpp:847-867): PlaneParams indexed by mask label - 1.
    void CudaPlanarPriorInitialization(const std::vector<Float4>& plane_params, const std::vector<uint32_t>& masks) {
        const size_t P = static_cast<size_t>(GetReferenceImageWidth()) * GetReferenceImageHeight();
        std::vector<Float4> prior(P, Float4{0, 0, 0, 0});
        for (size_t i = 0; i < P; ++i)
            if (masks[i] > 0) prior[i] = plane_params[masks[i] - 1];
        ACMMP_SAFE_CALL(acmmp_set_params(ctx_, &params_));
        ACMMP_SAFE_CALL(acmmp_set_planar_prior(ctx_, &prior[0].x, masks.data()));
    }
    void CudaPlanarPriorInitialization(const std::vector<Float4>& plane_params, const std::vector<float>& masks) {
        std::vector<uint32_t> m(masks.size());
        for (size_t i = 0; i < m.size(); ++i) m[i] = static_cast<uint32_t>(masks[i]);
        CudaPlanarPriorInitialization(plane_params, m);
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
    acmmp_ctx* context() const { return ctx_; }

private:
    void SetDepthRange() {                                            // ACMMP.cpp:645-651
        params_.depth_min = cameras_[0].depth_min * 0.6f;
        params_.depth_max = cameras_[0].depth_max * 1.2f;
        params_.num_images = static_cast<int>(images_.size());
        params_.disparity_min = cameras_[0].K[0] * params_.baseline / params_.depth_max;
        params_.disparity_max = cameras_[0].K[0] * params_.baseline / params_.depth_min;
    }

    acmmp_ctx* ctx_ = nullptr;
    PatchMatchParams params_;
    bool own_ = true;
    std::vector<Image> images_;
    std::vector<FloatMap> depths_;
    std::vector<Camera> cameras_;
    std::vector<Float4> planes_;
    std::vector<float> costs_;
};

// RunJBU (ACMMP.cpp:1071-1122) on `ctx`: upsamples src_depthmap guided by scaled_image_float and
// writes ACMMP/2333_<id>/depths.dmb; returns without writing when Imagescale == 1 (:1077-1080).
inline void RunJBU(acmmp_ctx* ctx_, const Image& scaled_image_float, const FloatMap& src_depthmap,
                   const std::string& dense_folder, const Problem& problem) {
    const int rows = scaled_image_float.height, cols = scaled_image_float.width;
    const int Imagescale = std::max(rows / src_depthmap.height, cols / src_depthmap.width);
    if (Imagescale == 1) {
        std::cout << "Image.rows = Depthmap.rows" << std::endl;
        return;
    }
    FloatMap out;
    out.width = cols;
    out.height = rows;
    out.data.resize(static_cast<size_t>(rows) * cols);
    ACMMP_SAFE_CALL(acmmp_jbu(ctx_, scaled_image_float.data.data(), cols, rows, src_depthmap.data.data(),
                              src_depthmap.width, src_depthmap.height, Imagescale, out.data.data()));
    writeDepthDmb(ResultFolder(dense_folder, problem.ref_image_id) + "/depths.dmb", out);
}

#undef ACMMP_SAFE_CALL

}  // namespace acmmp_host
