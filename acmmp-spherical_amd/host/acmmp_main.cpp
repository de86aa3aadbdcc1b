// acmmp_main.cpp -- the reference's ACMMP executable (main.cpp) in C++ over the C ABI: same
// dense-folder layout, same schedule, same outputs (ACMMP/2333_%08d/{depths,depths_geom,normals,
// costs}.dmb, ACMMP/ACMM_model_cuda_5.ply), no OpenCV and no CUDA.
//
//   ACMMP dense_folder [--seed S] [--math exact|fast] [--device D] [--no-fusion] [--geom-iterations N]
//                      [--size-bound B]
//
//   GenerateSampleList / ComputeMultiScaleSettings  main.cpp:4-71  (formats.cpp)
//   ProcessProblem                                  main.cpp:73-210
//   JointBilateralUpsampling                        main.cpp:212-238
//   main's multi-scale schedule                     main.cpp:392-482
//   RunFusionCuda                                   ACMMP.cu:1817-2105 (acmmp_fusion_* of the ABI)
//
// Differences from the reference, all deliberate: the seed of every RunPatchMatch is explicit
// (the reference uses clock64(), ACMMP.cu:684) -- seed + 7919 * pass + 31 * ref_image_id (+1 for
// the planar run), the scheme of acmmp/pipeline.py, so both drivers produce the same files; one
// engine context serves every problem (the reference constructs an ACMMP per problem); the
// triangulation.png debug image (main.cpp:117-137) is not written.
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "ACMMP.hpp"

using namespace acmmp_host;

namespace {

struct Options {
    std::string dense_folder;
    uint64_t seed = 1234;
    int device = 0;
    int math = -1;              // -1: the engine's default (exact); --math fast to opt in
    bool fusion = true;
    int geom_iterations = 2;
    int size_bound = 1000;      // main.cpp:38 (the coarsest scale's bound); tests use small scenes
};

void ProcessProblem(acmmp_ctx* ctx, const std::string& dense_folder, const std::vector<Problem>& problems, int idx,
                    bool geom_consistency, bool planar_prior, bool hierarchy, bool multi_geometrty, uint64_t run_seed) {
    const Problem problem = problems[idx];
    std::cout << "Processing image " << std::setw(8) << std::setfill('0') << problem.ref_image_id << "..." << std::endl;
    const std::string result_folder = ResultFolder(dense_folder, problem.ref_image_id);
    mkdir(result_folder.c_str(), 0777);

    ACMMP acmmp(ctx);
    if (geom_consistency) acmmp.SetGeomConsistencyParams(multi_geometrty);
    if (hierarchy) acmmp.SetHierarchyParams();
    acmmp.InuputInitialization(dense_folder, problems, idx);
    acmmp.CudaSpaceInitialization(dense_folder, problem);
    acmmp.RunPatchMatch(run_seed);

    const int width = acmmp.GetReferenceImageWidth();
    const int height = acmmp.GetReferenceImageHeight();
    const size_t P = static_cast<size_t>(width) * height;
    FloatMap depths{width, height, 1, std::vector<float>(P)};
    FloatMap normals{width, height, 3, std::vector<float>(3 * P)};
    FloatMap costs{width, height, 1, std::vector<float>(P)};
    auto collect = [&]() {                                         // main.cpp:103-111, 188-196
        for (size_t c = 0; c < P; ++c) {
            const Float4 ph = acmmp.GetPlaneHypothesis(static_cast<int>(c));
            depths.data[c] = ph.w;
            normals.data[3 * c] = ph.x; normals.data[3 * c + 1] = ph.y; normals.data[3 * c + 2] = ph.z;
            costs.data[c] = acmmp.GetCost(static_cast<int>(c));
        }
    };
    collect();

    if (planar_prior) {                                            // main.cpp:113-197
        std::cout << "Run Planar Prior Assisted PatchMatch MVS ..." << std::endl;
        acmmp.SetPlanarPriorParams();
        std::vector<Point> support2DPoints;
        acmmp.GetSupportPoints(support2DPoints);
        const std::vector<Triangle> triangles = acmmp.DelaunayTriangulation(width, height, support2DPoints);
        auto contains = [&](const Point& p) { return p.x >= 0 && p.x < width && p.y >= 0 && p.y < height; };

        std::vector<uint32_t> mask_tri(P, 0u);                     // float labels in the reference, exact < 2^24
        std::vector<Float4> planeParams_tri;
        uint32_t label = 0;
        for (const Triangle& triangle : triangles) {
            if (!(contains(triangle.pt1) && contains(triangle.pt2) && contains(triangle.pt3))) continue;
            // main.cpp:146-159: sample the triangle with barycentric steps of 1 / longest edge
            const float L01 = static_cast<float>(std::sqrt(std::pow(triangle.pt1.x - triangle.pt2.x, 2) + std::pow(triangle.pt1.y - triangle.pt2.y, 2)));
            const float L02 = static_cast<float>(std::sqrt(std::pow(triangle.pt1.x - triangle.pt3.x, 2) + std::pow(triangle.pt1.y - triangle.pt3.y, 2)));
            const float L12 = static_cast<float>(std::sqrt(std::pow(triangle.pt2.x - triangle.pt3.x, 2) + std::pow(triangle.pt2.y - triangle.pt3.y, 2)));
            const float max_edge_length = std::max(L01, std::max(L02, L12));
            const float step = static_cast<float>(1.0 / max_edge_length);
            for (float p = 0; p < 1.0; p += step) {
                for (float q = 0; q < 1.0 - p; q += step) {
                    const int x = static_cast<int>(static_cast<double>(p * triangle.pt1.x + q * triangle.pt2.x) +
                                                   (1.0 - p - q) * triangle.pt3.x);
                    const int y = static_cast<int>(static_cast<double>(p * triangle.pt1.y + q * triangle.pt2.y) +
                                                   (1.0 - p - q) * triangle.pt3.y);
                    mask_tri[static_cast<size_t>(y) * width + x] = label + 1;
                }
            }
            planeParams_tri.push_back(acmmp.GetPriorPlaneParams(triangle, depths.data));
            label++;
        }
        for (int i = 0; i < width; ++i) {                          // main.cpp:168-181
            for (int j = 0; j < height; ++j) {
                uint32_t& m = mask_tri[static_cast<size_t>(j) * width + i];
                if (m > 0) {
                    const float d = acmmp.GetDepthFromPlaneParam(planeParams_tri[m - 1], i, j);
                    if (!(d <= acmmp.GetMaxDepth() && d >= acmmp.GetMinDepth())) m = 0;
                }
            }
        }
        acmmp.CudaPlanarPriorInitialization(planeParams_tri, mask_tri);
        acmmp.RunPatchMatch(run_seed + 1);
        collect();
    }

    const std::string suffix = geom_consistency ? "/depths_geom.dmb" : "/depths.dmb";
    writeDepthDmb(result_folder + suffix, depths);
    writeNormalDmb(result_folder + "/normals.dmb", normals);
    writeDepthDmb(result_folder + "/costs.dmb", costs);
    std::cout << "Processing image " << std::setw(8) << std::setfill('0') << problem.ref_image_id << " done!" << std::endl;
}

void JointBilateralUpsampling(acmmp_ctx* ctx, const std::string& dense_folder, const Problem& problem, int acmmp_size) {
    const std::string result_folder = ResultFolder(dense_folder, problem.ref_image_id);
    FloatMap ref_depth;
    readDepthDmb(result_folder + "/depths_geom.dmb", &ref_depth);
    const Image image_float = ReadGrayImage(ImagePath(dense_folder, problem.ref_image_id));
    int new_rows, new_cols;                                        // main.cpp:227-231 (no <= early-out)
    ScaledDims(image_float.height, image_float.width, acmmp_size, &new_rows, &new_cols);
    const Image scaled_image_float = (new_cols == image_float.width && new_rows == image_float.height)
                                         ? image_float : ResizeLinear(image_float, new_cols, new_rows);
    std::cout << "Run JBU for image " << problem.ref_image_id << ".jpg" << std::endl;
    mkdir(result_folder.c_str(), 0777);
    RunJBU(ctx, scaled_image_float, ref_depth, dense_folder, problem);
}

// RunFusionCuda (ACMMP.cu:1817-2105): load every view's final maps and colour image rescaled to
// its depth size, fuse each reference view against its (at most 32) sources, write the PLY.
void RunFusionCuda(int device, const std::string& dense_folder, const std::vector<Problem>& problems,
                   bool geom_consistency) {
    const size_t N = problems.size();
    std::cout << "[CUDA Fusion] Starting simple fusion with " << N << " images..." << std::endl;
    std::vector<Camera> cams;
    std::vector<FloatMap> deps, normals;
    std::vector<ColorImage> imgs;
    std::vector<Problem> valid_problems;
    std::map<int, int> id_to_index;
    for (size_t i = 0; i < N; ++i) {
        const int id = problems[i].ref_image_id;
        Camera cam = ReadCamera(CameraPath(dense_folder, id));
        FloatMap depth, normal;
        const std::string folder = ResultFolder(dense_folder, id);
        if (readDepthDmb(folder + (geom_consistency ? "/depths_geom.dmb" : "/depths.dmb"), &depth) != 0) {
            std::cerr << "Warning: Could not load depth for image " << id << std::endl;
            continue;
        }
        if (readNormalDmb(folder + "/normals.dmb", &normal) != 0) {
            std::cerr << "Warning: Could not load normals for image " << id << std::endl;
            continue;
        }
        const ColorImage img = ReadColorImage(ImagePath(dense_folder, id));
        if (img.data.empty()) {
            std::cerr << "Warning: Could not load image " << id << std::endl;
            continue;
        }
        ColorImage scaled;
        RescaleImageAndCamera(img, &scaled, depth, &cam);
        id_to_index[id] = static_cast<int>(cams.size());
        cams.push_back(cam);
        deps.push_back(std::move(depth));
        normals.push_back(std::move(normal));
        imgs.push_back(std::move(scaled));
        valid_problems.push_back(problems[i]);
    }
    const size_t num_valid = cams.size();
    std::cout << "[CUDA Fusion] Successfully loaded " << num_valid << "/" << N << " images" << std::endl;
    if (num_valid == 0) {
        std::cerr << "Error: No valid images to process!" << std::endl;
        return;
    }
    acmmp_fusion* fu = nullptr;
    const acmmp_ctx* ctx_ = nullptr;
    auto check = [&](acmmp_status s, int line) {
        if (s != ACMMP_OK) {
            std::printf("%s in %s at line %i (%s)\n", acmmp_status_str(s), __FILE__, line, fu ? acmmp_fusion_last_error(fu) : "");
            std::exit(EXIT_FAILURE);
        }
    };
    (void)ctx_;
    check(acmmp_fusion_create(device, static_cast<int>(num_valid), cams.data(), &fu), __LINE__);
    for (size_t i = 0; i < num_valid; ++i)
        check(acmmp_fusion_set_view(fu, static_cast<int>(i), deps[i].data.data(), normals[i].data.data(), imgs[i].data.data()),
              __LINE__);
    std::vector<PointList> all_points;
    for (size_t i = 0; i < num_valid; ++i) {
        const int n_src = std::min(static_cast<int>(valid_problems[i].src_image_ids.size()), 32);
        std::vector<int> src(n_src);
        for (int j = 0; j < n_src; ++j) {
            const auto it = id_to_index.find(valid_problems[i].src_image_ids[j]);
            src[j] = it != id_to_index.end() ? it->second : -1;
        }
        const int cap = cams[i].width * cams[i].height;
        std::vector<float> pts(9 * static_cast<size_t>(cap));
        int n = 0;
        check(acmmp_fusion_run(fu, static_cast<int>(i), n_src, src.data(), pts.data(), cap, &n), __LINE__);
        for (int k = 0; k < n; ++k) {
            PointList p;
            std::memcpy(&p, &pts[9 * static_cast<size_t>(k)], sizeof p);
            all_points.push_back(p);
        }
        std::cout << "  -> Generated " << n << " points" << std::endl;
    }
    acmmp_fusion_destroy(fu);
    const std::string output_path = dense_folder + "/ACMMP/ACMM_model_cuda_5.ply";
    StoreColorPlyFileBinaryPointCloud(output_path, all_points);
    std::cout << "[CUDA Fusion] Complete! Wrote " << all_points.size() << " points to " << output_path << std::endl;
}

bool ParseArgs(int argc, char** argv, Options* o) {
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char* { return i + 1 < argc ? argv[++i] : nullptr; };
        if (a == "--seed") { const char* v = next(); if (!v) return false; o->seed = std::stoull(v); }
        else if (a == "--device") { const char* v = next(); if (!v) return false; o->device = std::stoi(v); }
        else if (a == "--geom-iterations") { const char* v = next(); if (!v) return false; o->geom_iterations = std::stoi(v); }
        else if (a == "--size-bound") { const char* v = next(); if (!v) return false; o->size_bound = std::stoi(v); }
        else if (a == "--math") {
            const char* v = next();
            if (!v) return false;
            const std::string m = v;
            if (m == "exact") o->math = ACMMP_MATH_EXACT;
            else if (m == "fast") o->math = ACMMP_MATH_FAST;
            else return false;
        }
        else if (a == "--no-fusion") o->fusion = false;
        else if (!a.empty() && a[0] == '-') return false;
        else if (o->dense_folder.empty()) o->dense_folder = a;
        else return false;
    }
    return !o->dense_folder.empty();
}

}  // namespace

int main(int argc, char** argv) {
    Options opt;
    if (!ParseArgs(argc, argv, &opt)) {
        std::cout << "USAGE: ACMMP dense_folder [--seed S] [--math exact|fast] [--device D] [--no-fusion] "
                     "[--geom-iterations N] [--size-bound B]" << std::endl;
        return -1;
    }
    const auto t0 = std::chrono::steady_clock::now();
    const std::string dense_folder = opt.dense_folder;
    std::vector<Problem> problems;
    GenerateSampleList(dense_folder, problems);
    const std::string output_folder = dense_folder + "/ACMMP";
    mkdir(output_folder.c_str(), 0777);
    const size_t num_images = problems.size();
    std::cout << "There are " << num_images << " problems needed to be processed!" << std::endl;
    int max_num_downscale = ComputeMultiScaleSettings(dense_folder, problems, opt.size_bound);

    acmmp_ctx* ctx = nullptr;
    {
        const acmmp_status s = acmmp_create(opt.device, &ctx);
        if (s != ACMMP_OK) {
            std::printf("%s in %s at line %i (%s)\n", acmmp_status_str(s), __FILE__, __LINE__,
                        ctx ? acmmp_last_error(ctx) : "no HIP device / context");
            return EXIT_FAILURE;
        }
    }
    if (opt.math >= 0 && acmmp_set_math(ctx, opt.math) != ACMMP_OK) {
        std::printf("acmmp_set_math failed\n");
        return EXIT_FAILURE;
    }
    {
        const int m = acmmp_get_math(ctx);
        std::cout << "Engine math: " << (m == ACMMP_MATH_FAST ? "fast (--use_fast_math arithmetic, tolerance parity)"
                                                               : "exact (bit-identical to the CPU oracle)") << std::endl;
    }

    int flag = 0, pass = 0;
    const int geom_iterations = opt.geom_iterations;
    bool geom_consistency = false, planar_prior = false, hierarchy = false, multi_geometry = false;
    auto seed_of = [&](int i) { return opt.seed + 7919ull * pass + 31ull * problems[i].ref_image_id; };
    while (max_num_downscale >= 0) {                               // main.cpp:417-476
        std::cout << "Scale: " << max_num_downscale << std::endl;
        for (size_t i = 0; i < num_images; ++i) {
            if (problems[i].num_downscale >= 0) {
                problems[i].cur_image_size = static_cast<int>(problems[i].max_image_size / std::pow(2, problems[i].num_downscale));
                problems[i].num_downscale--;
            }
        }
        if (flag == 0) {
            flag = 1;
            geom_consistency = false;
            planar_prior = true;
            for (size_t i = 0; i < num_images; ++i)
                ProcessProblem(ctx, dense_folder, problems, static_cast<int>(i), geom_consistency, planar_prior, hierarchy,
                               false, seed_of(static_cast<int>(i)));
            pass++;
        } else {
            for (size_t i = 0; i < num_images; ++i)
                JointBilateralUpsampling(ctx, dense_folder, problems[i], problems[i].cur_image_size);
            hierarchy = true;
            geom_consistency = false;
            planar_prior = true;
            for (size_t i = 0; i < num_images; ++i)
                ProcessProblem(ctx, dense_folder, problems, static_cast<int>(i), geom_consistency, planar_prior, hierarchy,
                               false, seed_of(static_cast<int>(i)));
            pass++;
            hierarchy = false;
        }
        geom_consistency = true;
        planar_prior = false;
        for (int geom_iter = 0; geom_iter < geom_iterations; ++geom_iter) {
            multi_geometry = geom_iter != 0;
            for (size_t i = 0; i < num_images; ++i)
                ProcessProblem(ctx, dense_folder, problems, static_cast<int>(i), geom_consistency, planar_prior, hierarchy,
                               multi_geometry, seed_of(static_cast<int>(i)));
            pass++;
        }
        max_num_downscale--;
    }
    acmmp_destroy(ctx);

    geom_consistency = true;
    if (opt.fusion) RunFusionCuda(opt.device, dense_folder, problems, geom_consistency);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("{\"driver\": \"c++\", \"views\": %zu, \"passes\": %d, \"seconds\": %.3f}\n", num_images, pass, s);
    return 0;
}
