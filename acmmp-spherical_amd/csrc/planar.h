// planar.h -- internal split of the planar-prior block of ProcessProblem (main.cpp:113-181) between
// the host (planar_prior.cpp: support points, Delaunay, per-triangle planes and sampling steps) and
// the device (kernels.hip: triangle rasterisation, prior-depth range mask, per-pixel expansion).
// Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "acmmp.h"

namespace acmmp {

// The triangles ProcessProblem labels (all three vertices inside the image), in label order
// (label = index + 1), with what the rasteriser needs per triangle.
struct PlanarTriangles {
    std::vector<int> tri;          // 6 ints per triangle: x1 y1 x2 y2 x3 y3
    std::vector<float> plane;      // 4 per triangle: GetPriorPlaneParams (ACMMP.cpp:957-989)
    std::vector<float> step;       // 1 / longest edge (main.cpp:146-151), float
    std::vector<long long> first;  // exclusive prefix of the p-steps per triangle (size n + 1)
    std::vector<float2> row_trig;  // SPHERE: (sin, cos) of each row's latitude, host libm (H)
    std::vector<float2> col_trig;  // SPHERE: (sin, cos) of each column's longitude (W)
    float delaunay_ms = 0.f;       // host wall time of the triangulation (acmmp_last_planar_timing)
};

// Host half: support points of `costs`, Delaunay, labelled triangles, their planes through `depths`.
acmmp_status planar_triangles(const acmmp_camera& cam, const float* depths, const float* costs, int W, int H,
                              PlanarTriangles* out);
// The same from support points found elsewhere (xy: 2 ints per point in the reference's order) and the
// depth at each point.
acmmp_status planar_triangles_pts(const acmmp_camera& cam, const std::vector<int>& xy,
                                  const std::vector<float>& depth_at, int W, int H, PlanarTriangles* out);

// Device half (kernels.hip).  mask: P uint32 zeroed by the caller; prior: P float4.
struct PlanarDev {
    const int* tri;
    const float* step;
    const long long* first;
    const float4* plane;
    const float2* row_trig;
    const float2* col_trig;
    int n_tri;
    long long n_steps;            // first[n_tri]
    int W, H, model;
    float K0, K2, K4, K5;         // PINHOLE intrinsics (GetDepthFromPlaneParam, ACMMP.cpp:1008-1009)
    float depth_min, depth_max;
};
hipError_t launch_planar_raster(const PlanarDev& pd, uint32_t* mask, hipStream_t s);
hipError_t launch_planar_mask(const PlanarDev& pd, uint32_t* mask, float4* prior, hipStream_t s);
// GetSupportPoints on device maps (costs, planes' .w = depth, row-major W x H): ((W + 4) / 5) * ((H + 4) / 5)
// int4 (kept, x, y, depth bits), strip-major.
hipError_t launch_support_points(const float* costs, const float4* planes, int W, int H, int4* out, hipStream_t s);

}  // namespace acmmp
