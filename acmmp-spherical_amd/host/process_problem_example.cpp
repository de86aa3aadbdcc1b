// process_problem_example.cpp -- the first RunPatchMatch of ProcessProblem (main.cpp:83-111)
// ported onto the C++ facade.  Build: see INTEGRATION.md.  Synthetic fronto-parallel inputs.
#include <cmath>
#include <cstdio>

#include "ACMMP.hpp"

int main() {
    using namespace acmmp_host;
    const int W = 160, H = 120;
    std::vector<Image> images(2);
    std::vector<Camera> cams(2);
    for (int v = 0; v < 2; ++v) {
        images[v].width = W; images[v].height = H; images[v].data.resize(W * H);
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x)
                images[v].data[y * W + x] = std::round(127.5f + 60.f * std::sin(0.37f * (x + 8 * v)) * std::cos(0.29f * y));
        Camera& c = cams[v];
        std::memset(&c, 0, sizeof c);
        c.model = ACMMP_PINHOLE;
        c.K[0] = c.K[4] = 128.f; c.K[2] = W / 2.f; c.K[5] = H / 2.f; c.K[8] = 1.f;
        c.R[0] = c.R[4] = c.R[8] = 1.f;
        c.t[0] = -0.5f * v;
        c.width = W; c.height = H; c.depth_min = 3.f; c.depth_max = 8.f;
    }
    ACMMP acmmp;                                           // main.cpp:83
    acmmp.InuputInitialization(images, cams);             // main.cpp:91
    acmmp.CudaSpaceInitialization();                      // main.cpp:93
    acmmp.RunPatchMatch(1234);                            // main.cpp:94
    const int width = acmmp.GetReferenceImageWidth(), height = acmmp.GetReferenceImageHeight();
    double mean_depth = 0.0;
    for (int i = 0; i < width * height; ++i) mean_depth += acmmp.GetPlaneHypothesis(i).w;  // main.cpp:103-111
    std::printf("mean depth %.4f over %dx%d\n", mean_depth / (width * height), width, height);

    // planar pass (main.cpp:113-187): support points, Delaunay, per-triangle planes, second run
    std::vector<float> depths(width * height);
    for (int i = 0; i < width * height; ++i) depths[i] = acmmp.GetPlaneHypothesis(i).w;
    acmmp.SetPlanarPriorParams();
    std::vector<Point> support;
    acmmp.GetSupportPoints(support);
    const std::vector<Triangle> triangles = acmmp.DelaunayTriangulation(width, height, support);
    std::vector<float> mask_tri(width * height, 0.0f);
    std::vector<Float4> planes;
    for (const Triangle& t : triangles) {
        planes.push_back(acmmp.GetPriorPlaneParams(t, depths));
        const int cx = (t.pt1.x + t.pt2.x + t.pt3.x) / 3, cy = (t.pt1.y + t.pt2.y + t.pt3.y) / 3;
        mask_tri[cy * width + cx] = static_cast<float>(planes.size());   // centroid label only (example)
    }
    acmmp.CudaPlanarPriorInitialization(planes, mask_tri);
    acmmp.RunPatchMatch();
    std::printf("planar pass: %zu support points, %zu triangles\n", support.size(), triangles.size());
    return 0;
}
