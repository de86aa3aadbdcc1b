// formats.hpp -- the reference's host-side formats and helpers in C++ without OpenCV
// (SURVEY.md §8f row 2), for the C++ drop-in driver (acmmp_main.cpp) and the ACMMP facade.
//
//   ReadCamera                       ACMMP.cpp:146-209   (SPHERE / PINHOLE, reader quirks kept)
//   readDepthDmb / writeDepthDmb     ACMMP.cpp:363-420
//   readNormalDmb / writeNormalDmb   ACMMP.cpp:422-479
//   StoreColorPlyFileBinaryPointCloud ACMMP.cpp:481-534
//   GenerateSampleList               main.cpp:4-33
//   ComputeMultiScaleSettings        main.cpp:35-71
//   RescaleImageAndCamera            ACMMP.cpp:213-246
//   cv::resize(INTER_LINEAR)         float and 8-bit, as restated in acmmp/pipeline.py
//                                    (resize_linear / resize_linear_u8; cv parity unpinned)
//   cv::imread                       jpeg.hpp (libjpeg-turbo's decoder, pinned against it)
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/acmmp.h"

namespace acmmp_host {

using Camera = acmmp_camera;                 // main.h:40-54

struct Image {                               // one grey view, float 0..255 (cv::Mat_<float>)
    int width = 0, height = 0;
    std::vector<float> data;                 // row-major, width * height
};

struct ColorImage {                          // cv::Mat_<cv::Vec3b>, BGR
    int width = 0, height = 0;
    std::vector<uint8_t> data;               // row-major, width * height * 3
};

struct FloatMap {                            // cv::Mat_<float> (nb = 1) or cv::Mat_<cv::Vec3f> (nb = 3)
    int width = 0, height = 0, channels = 1;
    std::vector<float> data;
    bool empty() const { return data.empty(); }
};

struct Problem {                             // main.h:58-64
    int ref_image_id = 0;
    std::vector<int> src_image_ids;
    int max_image_size = 3200;
    int num_downscale = 0;
    int cur_image_size = 3200;
};

struct PointList {                           // main.h:71-75: coord, normal, colour (9 floats)
    float coord[3], normal[3], color[3];
};

Camera ReadCamera(const std::string& cam_path);
int readDepthDmb(const std::string& path, FloatMap* depth);          // 0 ok, -1 as the reference
int writeDepthDmb(const std::string& path, const FloatMap& depth);
int readNormalDmb(const std::string& path, FloatMap* normal);
int writeNormalDmb(const std::string& path, const FloatMap& normal);
void StoreColorPlyFileBinaryPointCloud(const std::string& path, const std::vector<PointList>& pc);

void GenerateSampleList(const std::string& dense_folder, std::vector<Problem>& problems);
int ComputeMultiScaleSettings(const std::string& dense_folder, std::vector<Problem>& problems, int size_bound = 1000);

// cv::imread(path, IMREAD_GRAYSCALE) + convertTo(CV_32F) / cv::imread(path, IMREAD_COLOR).
// Empty image (width 0) when the file is missing or unsupported, as cv::imread.
Image ReadGrayImage(const std::string& path);
ColorImage ReadColorImage(const std::string& path);
std::string ImagePath(const std::string& dense_folder, int id);      // images/%08d.jpg
std::string CameraPath(const std::string& dense_folder, int id);     // cams/%08d_cam.txt
std::string ResultFolder(const std::string& dense_folder, int id);   // ACMMP/2333_%08d

// std::round(x * factor) sizes of InuputInitialization / JointBilateralUpsampling
// (ACMMP.cpp:616-621, main.cpp:227-231): factor = min(size / cols, size / rows) in float.
void ScaledDims(int rows, int cols, int max_image_size, int* new_rows, int* new_cols);
Image ResizeLinear(const Image& src, int new_cols, int new_rows);
ColorImage ResizeLinearU8(const ColorImage& src, int new_cols, int new_rows);
void RescaleImageAndCamera(const ColorImage& src, ColorImage* dst, const FloatMap& depth, Camera* camera);

}  // namespace acmmp_host
