// host_capi.cpp -- C entry points of the host-side helpers (libacmmp_host.so) so the Python tests
// can pin them: the JPEG decoder against libjpeg-turbo (PIL), the resizers and ReadCamera against
// acmmp/pipeline.py and acmmp/io.py.  Test surface only; the driver links the C++ directly.
#include <cstring>
#include <string>

#include "formats.hpp"
#include "jpeg.hpp"

using namespace acmmp_host;

extern "C" {

// Decodes `path` (want_color 0: grey, 1: BGR) into `out` (cap bytes).  Returns 0 on success, 1 when
// cap is too small (w/h/c set), -1 on a decode error (message copied to err, err_cap bytes).
int acmmp_host_decode_jpeg(const char* path, int want_color, unsigned char* out, long long cap, int* w, int* h, int* c,
                           char* err, int err_cap) {
    JpegImage im;
    std::string e;
    if (!DecodeJpegFile(path, want_color != 0, &im, &e)) {
        if (err && err_cap > 0) {
            std::strncpy(err, e.c_str(), static_cast<size_t>(err_cap) - 1);
            err[err_cap - 1] = 0;
        }
        return -1;
    }
    *w = im.width;
    *h = im.height;
    *c = im.channels;
    if (static_cast<long long>(im.pixels.size()) > cap) return 1;
    std::memcpy(out, im.pixels.data(), im.pixels.size());
    return 0;
}

void acmmp_host_resize_linear(const float* src, int w, int h, float* dst, int nw, int nh) {
    Image in;
    in.width = w;
    in.height = h;
    in.data.assign(src, src + static_cast<size_t>(w) * h);
    const Image out = ResizeLinear(in, nw, nh);
    std::memcpy(dst, out.data.data(), out.data.size() * sizeof(float));
}

void acmmp_host_resize_linear_u8(const unsigned char* src, int w, int h, unsigned char* dst, int nw, int nh) {
    ColorImage in;
    in.width = w;
    in.height = h;
    in.data.assign(src, src + static_cast<size_t>(w) * h * 3);
    const ColorImage out = ResizeLinearU8(in, nw, nh);
    std::memcpy(dst, out.data.data(), out.data.size());
}

void acmmp_host_scaled_dims(int rows, int cols, int size, int* new_rows, int* new_cols) {
    ScaledDims(rows, cols, size, new_rows, new_cols);
}

int acmmp_host_read_camera(const char* path, acmmp_camera* cam) {
    *cam = ReadCamera(path);
    return 0;
}

}  // extern "C"
