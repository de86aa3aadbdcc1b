// formats.cpp -- see formats.hpp.  Compiled with -ffp-contract=off: every float expression below
// rounds where the reference's (and acmmp/pipeline.py's) does.
#include "formats.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>

#include "jpeg.hpp"

namespace acmmp_host {

Camera ReadCamera(const std::string& cam_path) {
    Camera camera;
    std::memset(&camera, 0, sizeof camera);   // the reference leaves unread fields uninitialised
    std::ifstream file(cam_path);
    if (!file.is_open()) {
        std::cerr << "Error: Could not open camera file: " << cam_path << std::endl;
        return camera;
    }
    std::string token;
    file >> token;                                               // "extrinsic"
    for (int i = 0; i < 3; ++i) file >> camera.R[3 * i + 0] >> camera.R[3 * i + 1] >> camera.R[3 * i + 2] >> camera.t[i];
    float dummy;
    for (int i = 0; i < 4; ++i) file >> dummy;                   // 0 0 0 1
    file >> token;                                               // "intrinsic"
    file >> token;
    if (token == "SPHERE") {                                     // ACMMP.cpp:172-193
        camera.model = ACMMP_SPHERE;
        file >> camera.params[0] >> camera.params[1] >> camera.params[2];
        float depth_min, depth_interval, depth_max;
        int n_planes;
        file >> depth_min >> depth_interval >> n_planes >> depth_max;
        camera.depth_min = depth_min;
        camera.depth_max = depth_max;
    } else {                                                     // ACMMP.cpp:194-206
        camera.model = ACMMP_PINHOLE;
        camera.K[0] = std::stof(token);
        for (int k = 1; k < 9; ++k) file >> camera.K[k];
        float d1, d2;
        file >> camera.depth_min >> camera.depth_max >> d1 >> d2;   // 2nd token -> depth_max (quirk kept)
    }
    return camera;
}

static int read_dmb(const std::string& path, FloatMap* m, int want_nb) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) {
        std::cout << "Error opening file " << path << std::endl;
        return -1;
    }
    int32_t hdr[4] = {-1, 0, 0, 0};
    const size_t got = std::fread(hdr, sizeof(int32_t), 4, f);
    if (got != 4 || hdr[0] != 1) {
        std::fclose(f);
        return -1;
    }
    m->height = hdr[1];
    m->width = hdr[2];
    m->channels = want_nb;                                       // cv::Mat type of the caller
    const size_t n = static_cast<size_t>(hdr[1]) * hdr[2] * hdr[3];
    m->data.assign(static_cast<size_t>(hdr[1]) * hdr[2] * want_nb, 0.0f);
    const size_t take = std::min(n, m->data.size());
    const size_t rd = std::fread(m->data.data(), sizeof(float), take, f);
    (void)rd;                                                    // short file: zeros remain, as cv::Mat::zeros
    std::fclose(f);
    return 0;
}

static int write_dmb(const std::string& path, const FloatMap& m, int nb) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) {
        std::cout << "Error opening file " << path << std::endl;
        return -1;
    }
    const int32_t hdr[4] = {1, m.height, m.width, nb};
    std::fwrite(hdr, sizeof(int32_t), 4, f);
    std::fwrite(m.data.data(), sizeof(float), static_cast<size_t>(m.width) * m.height * nb, f);
    std::fclose(f);
    return 0;
}

int readDepthDmb(const std::string& path, FloatMap* depth) { return read_dmb(path, depth, 1); }
int writeDepthDmb(const std::string& path, const FloatMap& depth) { return write_dmb(path, depth, 1); }
int readNormalDmb(const std::string& path, FloatMap* normal) { return read_dmb(path, normal, 3); }
int writeNormalDmb(const std::string& path, const FloatMap& normal) { return write_dmb(path, normal, 3); }

void StoreColorPlyFileBinaryPointCloud(const std::string& path, const std::vector<PointList>& pc) {
    std::cout << "store 3D points to ply file" << std::endl;
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) {
        std::cout << "Error opening file " << path << std::endl;
        return;
    }
    std::fprintf(f, "ply\nformat binary_little_endian 1.0\nelement vertex %d\n", static_cast<int>(pc.size()));
    std::fprintf(f, "property float x\nproperty float y\nproperty float z\n");
    std::fprintf(f, "property float nx\nproperty float ny\nproperty float nz\n");
    std::fprintf(f, "property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n");
    std::vector<uint8_t> rec(27 * pc.size());
    for (size_t i = 0; i < pc.size(); ++i) {
        const PointList& p = pc[i];
        float X[3] = {p.coord[0], p.coord[1], p.coord[2]};
        auto to_char = [](float v) -> uint8_t {                  // (char)(int)v; non-finite -> 0 here
            if (!std::isfinite(v) || v >= 2147483648.0f || v < -2147483648.0f) return 0;
            return static_cast<uint8_t>(static_cast<int>(v) & 0xFF);
        };
        const uint8_t rgb[3] = {to_char(p.color[2]), to_char(p.color[1]), to_char(p.color[0])};
        if (!(X[0] < FLT_MAX && X[0] > -FLT_MAX) || !(X[1] < FLT_MAX && X[1] > -FLT_MAX) ||
            !(X[2] < FLT_MAX && X[2] >= -FLT_MAX))
            X[0] = X[1] = X[2] = 0.0f;
        uint8_t* r = &rec[27 * i];
        std::memcpy(r, X, 12);
        std::memcpy(r + 12, p.normal, 12);
        std::memcpy(r + 24, rgb, 3);
    }
    std::fwrite(rec.data(), 1, rec.size(), f);
    std::fclose(f);
}

void GenerateSampleList(const std::string& dense_folder, std::vector<Problem>& problems) {
    problems.clear();
    std::ifstream file(dense_folder + "/pair.txt");
    int num_images = 0;
    file >> num_images;
    for (int i = 0; i < num_images; ++i) {
        Problem problem;
        file >> problem.ref_image_id;
        int num_src = 0;
        file >> num_src;
        for (int j = 0; j < num_src; ++j) {
            int id;
            float score;
            file >> id >> score;
            if (score <= 0.0f) continue;
            problem.src_image_ids.push_back(id);
        }
        problems.push_back(problem);
    }
}

std::string ImagePath(const std::string& dense_folder, int id) {
    std::stringstream s;
    s << dense_folder << "/images/" << std::setw(8) << std::setfill('0') << id << ".jpg";
    return s.str();
}
std::string CameraPath(const std::string& dense_folder, int id) {
    std::stringstream s;
    s << dense_folder << "/cams/" << std::setw(8) << std::setfill('0') << id << "_cam.txt";
    return s.str();
}
std::string ResultFolder(const std::string& dense_folder, int id) {
    std::stringstream s;
    s << dense_folder << "/ACMMP" << "/2333_" << std::setw(8) << std::setfill('0') << id;
    return s.str();
}

Image ReadGrayImage(const std::string& path) {
    Image im;
    JpegImage j;
    std::string err;
    if (!DecodeJpegFile(path, false, &j, &err)) {
        std::cerr << "imread " << path << ": " << err << std::endl;
        return im;
    }
    im.width = j.width;
    im.height = j.height;
    im.data.assign(j.pixels.begin(), j.pixels.end());            // convertTo(CV_32F)
    return im;
}

ColorImage ReadColorImage(const std::string& path) {
    ColorImage im;
    JpegImage j;
    std::string err;
    if (!DecodeJpegFile(path, true, &j, &err)) {
        std::cerr << "imread " << path << ": " << err << std::endl;
        return im;
    }
    im.width = j.width;
    im.height = j.height;
    im.data = std::move(j.pixels);
    return im;
}

int ComputeMultiScaleSettings(const std::string& dense_folder, std::vector<Problem>& problems, int size_bound) {
    int max_num_downscale = -1;
    const int max_image_size = 3200;                             // PatchMatchParams default (ACMMP.h:36)
    for (Problem& p : problems) {
        const Image im = ReadGrayImage(ImagePath(dense_folder, p.ref_image_id));
        int max_size = std::max(im.height, im.width);
        if (max_size > max_image_size) max_size = max_image_size;
        p.max_image_size = max_size;
        int k = 0;
        while (max_size > size_bound) {
            max_size /= 2;
            k++;
        }
        if (k > max_num_downscale) max_num_downscale = k;
        p.num_downscale = k;
    }
    return max_num_downscale;
}

void ScaledDims(int rows, int cols, int max_image_size, int* new_rows, int* new_cols) {
    const float fx = static_cast<float>(max_image_size) / cols;
    const float fy = static_cast<float>(max_image_size) / rows;
    const float factor = std::min(fx, fy);
    *new_cols = static_cast<int>(std::round(cols * factor));
    *new_rows = static_cast<int>(std::round(rows * factor));
}

namespace {
struct Taps {
    std::vector<int> s0, s1;
    std::vector<float> a0, a1;
};
// source taps of INTER_LINEAR: fx = (d + 0.5) * scale - 0.5 (double, then float), clamped at the borders
Taps linear_taps(int dsize, int ssize) {
    Taps t;
    t.s0.resize(dsize); t.s1.resize(dsize); t.a0.resize(dsize); t.a1.resize(dsize);
    const double scale = static_cast<double>(ssize) / dsize;
    for (int d = 0; d < dsize; ++d) {
        float f = static_cast<float>((d + 0.5) * scale - 0.5);
        long long s = static_cast<long long>(std::floor(f));
        f = f - static_cast<float>(s);
        if (s < 0) { f = 0.0f; s = 0; }
        if (s >= ssize - 1) { f = 0.0f; s = ssize - 1; }
        t.s0[d] = static_cast<int>(s);
        t.s1[d] = static_cast<int>(std::min<long long>(s + 1, ssize - 1));
        t.a0[d] = 1.0f - f;
        t.a1[d] = f;
    }
    return t;
}
}  // namespace

Image ResizeLinear(const Image& src, int new_cols, int new_rows) {
    const Taps tx = linear_taps(new_cols, src.width), ty = linear_taps(new_rows, src.height);
    std::vector<float> h(static_cast<size_t>(src.height) * new_cols);
    for (int y = 0; y < src.height; ++y) {
        const float* s = &src.data[static_cast<size_t>(y) * src.width];
        float* o = &h[static_cast<size_t>(y) * new_cols];
        for (int x = 0; x < new_cols; ++x) {
            const float p0 = s[tx.s0[x]] * tx.a0[x];
            const float p1 = s[tx.s1[x]] * tx.a1[x];
            o[x] = p0 + p1;
        }
    }
    Image out;
    out.width = new_cols;
    out.height = new_rows;
    out.data.resize(static_cast<size_t>(new_rows) * new_cols);
    for (int y = 0; y < new_rows; ++y) {
        const float* r0 = &h[static_cast<size_t>(ty.s0[y]) * new_cols];
        const float* r1 = &h[static_cast<size_t>(ty.s1[y]) * new_cols];
        float* o = &out.data[static_cast<size_t>(y) * new_cols];
        for (int x = 0; x < new_cols; ++x) {
            const float p0 = r0[x] * ty.a0[y];
            const float p1 = r1[x] * ty.a1[y];
            o[x] = p0 + p1;
        }
    }
    return out;
}

ColorImage ResizeLinearU8(const ColorImage& src, int new_cols, int new_rows) {
    // fixed point: 11-bit coefficients, horizontal sums kept as ints, (b0*S0 + b1*S1 + 2^21) >> 22
    const Taps tx = linear_taps(new_cols, src.width), ty = linear_taps(new_rows, src.height);
    auto q = [](float a) { return static_cast<long long>(std::nearbyint(a * 2048.0f)); };
    std::vector<long long> h(static_cast<size_t>(src.height) * new_cols * 3);
    for (int y = 0; y < src.height; ++y)
        for (int x = 0; x < new_cols; ++x)
            for (int c = 0; c < 3; ++c)
                h[(static_cast<size_t>(y) * new_cols + x) * 3 + c] =
                    src.data[(static_cast<size_t>(y) * src.width + tx.s0[x]) * 3 + c] * q(tx.a0[x]) +
                    src.data[(static_cast<size_t>(y) * src.width + tx.s1[x]) * 3 + c] * q(tx.a1[x]);
    ColorImage out;
    out.width = new_cols;
    out.height = new_rows;
    out.data.resize(static_cast<size_t>(new_rows) * new_cols * 3);
    for (int y = 0; y < new_rows; ++y)
        for (int x = 0; x < new_cols; ++x)
            for (int c = 0; c < 3; ++c) {
                const long long v = h[(static_cast<size_t>(ty.s0[y]) * new_cols + x) * 3 + c] * q(ty.a0[y]) +
                                    h[(static_cast<size_t>(ty.s1[y]) * new_cols + x) * 3 + c] * q(ty.a1[y]);
                const long long r = (v + (1LL << 21)) >> 22;
                out.data[(static_cast<size_t>(y) * new_cols + x) * 3 + c] = static_cast<uint8_t>(std::min(255LL, std::max(0LL, r)));
            }
    return out;
}

void RescaleImageAndCamera(const ColorImage& src, ColorImage* dst, const FloatMap& depth, Camera* camera) {
    const int cols = depth.width, rows = depth.height;
    camera->width = cols;
    camera->height = rows;
    if (cols == src.width && rows == src.height) {
        *dst = src;
        return;
    }
    const float scale_x = cols / static_cast<float>(src.width);
    const float scale_y = rows / static_cast<float>(src.height);
    *dst = ResizeLinearU8(src, cols, rows);
    if (camera->model == ACMMP_SPHERE) {
        camera->params[1] *= scale_x;
        camera->params[2] *= scale_y;
    } else {
        camera->K[0] *= scale_x; camera->K[2] *= scale_x;
        camera->K[4] *= scale_y; camera->K[5] *= scale_y;
    }
}

}  // namespace acmmp_host
