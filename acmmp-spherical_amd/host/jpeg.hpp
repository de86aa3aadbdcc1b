// jpeg.hpp -- baseline JPEG decoder for the C++ host driver (the reference's
// cv::imread, ACMMP.cpp:578 IMREAD_GRAYSCALE and ACMMP.cu:1846 IMREAD_COLOR).
//
// OpenCV decodes JPEG with libjpeg-turbo; this restates the parts of its decoder that decide the
// output bits, so the C++ driver reads the same pixels the reference does without OpenCV:
//   * baseline sequential Huffman (SOF0/SOF1, 8-bit), interleaved and non-interleaved scans,
//     restart intervals;
//   * the accurate integer inverse DCT (jidctint.c, JDCT_ISLOW -- libjpeg-turbo's default, whose
//     SIMD versions are bitwise identical to the C one) with its post-IDCT range limit;
//   * grey output (JCS_GRAYSCALE): the luma plane as decoded (no colour conversion);
//   * colour output: "fancy" triangle-filter chroma upsampling (jdsample.c h2v1/h2v2/h1v2, edge
//     rows and columns replicated as jdmainct.c does) and the fixed-point YCbCr->RGB tables of
//     jdcolor.c, returned in OpenCV's BGR order.
// Progressive, arithmetic-coded, 12-bit, lossless and CMYK/YCCK files are refused with a message.
// Pinned bit for bit against libjpeg-turbo as bundled with PIL (tests/test_host_driver.py).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace acmmp_host {

struct JpegImage {
    int width = 0, height = 0, channels = 0;   // channels: 1 (grey) or 3 (BGR)
    std::vector<uint8_t> pixels;               // row-major, width * height * channels
};

// Decode `path`; want_color = false -> IMREAD_GRAYSCALE, true -> IMREAD_COLOR (BGR).  Returns false
// (and sets *error) on an unreadable or unsupported file -- cv::imread returns an empty Mat there.
bool DecodeJpegFile(const std::string& path, bool want_color, JpegImage* out, std::string* error);
bool DecodeJpegMemory(const uint8_t* data, size_t size, bool want_color, JpegImage* out, std::string* error);

}  // namespace acmmp_host
