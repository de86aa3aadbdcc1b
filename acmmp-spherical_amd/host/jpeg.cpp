// jpeg.cpp -- see jpeg.hpp.  Restated from the JPEG standard (ITU T.81) and the published
// algorithms of libjpeg-turbo's decoder (jidctint.c, jdsample.c, jdcolor.c, jdmainct.c), written for
// this driver so that it decodes bit-identically to the library OpenCV's imread uses.  Credit: the
// integer IDCT `idct_islow` follows the Independent JPEG Group's jpeg_idct_islow (jidctint.c, as kept
// in libjpeg-turbo) step for step -- its LL&M factorisation, CONST_BITS/PASS1_BITS scaling, the
// tmp0..3 / z1..z5 intermediates and the zero-AC column shortcut -- because bit parity with that
// library requires the same rounding points (IJG licence: this notice acknowledges the IJG's work).
#include "jpeg.hpp"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>

namespace acmmp_host {
namespace {

// zig-zag index -> natural (row-major) index
const int kNatural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};  // overrun guard, as libjpeg's table

struct Huffman {
    bool present = false;
    int maxcode[18];          // largest code of each length, -1 if none
    int valptr[17];           // index of the first value of each length
    int mincode[17];
    uint8_t vals[256];
    // 8-bit lookahead: (length << 8) | value, 0 = longer code
    uint16_t look[256];
};

struct Component {
    int id = 0, h = 1, v = 1, tq = 0;
    int td = 0, ta = 0;       // Huffman tables of the current scan
    int dw = 0, dh = 0;       // downsampled width / height (jdinput.c: ceil(W * h / hmax))
    int stride = 0, rows = 0; // plane size (whole MCUs)
    int dc_pred = 0;
    std::vector<uint8_t> plane;
};

class Decoder {
public:
    Decoder(const uint8_t* d, size_t n) : d_(d), n_(n) {}

    bool decode(bool want_color, JpegImage* out, std::string* err) {
        if (!parse(err)) return false;
        return emit(want_color, out, err);
    }

private:
    const uint8_t* d_;
    size_t n_, pos_ = 0;
    uint16_t qt_[4][64] = {};  // natural order
    bool qt_set_[4] = {};
    Huffman dc_[4], ac_[4];
    Component comp_[4];
    int ncomp_ = 0, W_ = 0, H_ = 0, hmax_ = 1, vmax_ = 1, mcux_ = 0, mcuy_ = 0;
    int restart_ = 0;
    bool frame_ = false, jfif_ = false, adobe_ = false;
    int adobe_transform_ = -1;
    std::string msg_;
    // bit reader
    uint32_t buf_ = 0;
    int cnt_ = 0;
    bool marker_hit_ = false;

    bool fail(std::string* err, const std::string& m) {
        if (err) *err = m;
        return false;
    }
    int byte() { return pos_ < n_ ? d_[pos_++] : -1; }
    int u16() {
        const int a = byte(), b = byte();
        return (a < 0 || b < 0) ? -1 : (a << 8 | b);
    }

    bool parse(std::string* err) {
        if (n_ < 4 || d_[0] != 0xFF || d_[1] != 0xD8) return fail(err, "not a JPEG file (no SOI)");
        pos_ = 2;
        for (;;) {
            int c = byte();
            while (c >= 0 && c != 0xFF) c = byte();           // skip garbage between markers
            while (c == 0xFF) c = byte();                      // fill bytes
            if (c < 0) return fail(err, "premature end of file");
            const int m = c;
            if (m == 0xD9) return frame_ ? true : fail(err, "no image");   // EOI
            if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;          // parameterless
            const int len = u16();
            if (len < 2 || pos_ + len - 2 > n_) return fail(err, "bad marker length");
            const size_t seg = pos_, end = pos_ + len - 2;
            switch (m) {
                case 0xC0: case 0xC1:
                    if (!sof(seg, end, err)) return false;
                    break;
                case 0xC2: case 0xC6: case 0xCA: case 0xCE:
                    return fail(err, "progressive JPEG is not supported");
                case 0xC3: case 0xC5: case 0xC7: case 0xC9: case 0xCB: case 0xCD: case 0xCF:
                    return fail(err, "lossless / hierarchical / arithmetic JPEG is not supported");
                case 0xC4:
                    if (!dht(seg, end, err)) return false;
                    break;
                case 0xDB:
                    if (!dqt(seg, end, err)) return false;
                    break;
                case 0xDD:
                    if (end - seg < 2) return fail(err, "bad DRI");
                    restart_ = (d_[seg] << 8) | d_[seg + 1];
                    break;
                case 0xE0:
                    if (end - seg >= 5 && !std::memcmp(d_ + seg, "JFIF\0", 5)) jfif_ = true;
                    break;
                case 0xEE:
                    if (end - seg >= 12 && !std::memcmp(d_ + seg, "Adobe", 5)) {
                        adobe_ = true;
                        adobe_transform_ = d_[seg + 11];
                    }
                    break;
                case 0xDA:
                    pos_ = end;
                    if (!sos(seg, end, err)) return false;
                    continue;                                  // sos() leaves pos_ at the next marker
                default:
                    break;                                     // APPn, COM, ...
            }
            pos_ = end;
        }
    }

    bool sof(size_t p, size_t end, std::string* err) {
        if (frame_) return fail(err, "multiple frames");
        if (end - p < 6) return fail(err, "bad SOF");
        if (d_[p] != 8) return fail(err, "only 8-bit JPEG is supported");
        H_ = (d_[p + 1] << 8) | d_[p + 2];
        W_ = (d_[p + 3] << 8) | d_[p + 4];
        ncomp_ = d_[p + 5];
        if (W_ <= 0 || H_ <= 0) return fail(err, "bad image size");
        if (ncomp_ != 1 && ncomp_ != 3) return fail(err, "only 1- and 3-component JPEG is supported");
        if (end - p < static_cast<size_t>(6 + 3 * ncomp_)) return fail(err, "bad SOF");
        hmax_ = vmax_ = 1;
        for (int i = 0; i < ncomp_; ++i) {
            Component& c = comp_[i];
            c.id = d_[p + 6 + 3 * i];
            c.h = d_[p + 7 + 3 * i] >> 4;
            c.v = d_[p + 7 + 3 * i] & 15;
            c.tq = d_[p + 8 + 3 * i] & 3;
            if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4) return fail(err, "bad sampling factors");
            hmax_ = std::max(hmax_, c.h);
            vmax_ = std::max(vmax_, c.v);
        }
        for (int i = 0; i < ncomp_; ++i)       // upsample() needs integral ratios (libjpeg rejects the rest)
            if (hmax_ % comp_[i].h || vmax_ % comp_[i].v) return fail(err, "unsupported sampling factors");
        mcux_ = (W_ + 8 * hmax_ - 1) / (8 * hmax_);
        mcuy_ = (H_ + 8 * vmax_ - 1) / (8 * vmax_);
        for (int i = 0; i < ncomp_; ++i) {
            Component& c = comp_[i];
            c.dw = static_cast<int>((static_cast<long>(W_) * c.h + hmax_ - 1) / hmax_);
            c.dh = static_cast<int>((static_cast<long>(H_) * c.v + vmax_ - 1) / vmax_);
            c.stride = mcux_ * c.h * 8;
            c.rows = mcuy_ * c.v * 8;
            c.plane.assign(static_cast<size_t>(c.stride) * c.rows, 0);
        }
        frame_ = true;
        return true;
    }

    bool dqt(size_t p, size_t end, std::string* err) {
        while (p < end) {
            const int pq = d_[p] >> 4, tq = d_[p] & 3;
            ++p;
            if (p + (pq ? 128 : 64) > end) return fail(err, "bad DQT");
            for (int k = 0; k < 64; ++k) {
                int v;
                if (pq) { v = (d_[p] << 8) | d_[p + 1]; p += 2; }
                else { v = d_[p]; p += 1; }
                qt_[tq][kNatural[k]] = static_cast<uint16_t>(v);
            }
            qt_set_[tq] = true;
        }
        return true;
    }

    bool dht(size_t p, size_t end, std::string* err) {
        while (p < end) {
            const int tc = d_[p] >> 4, th = d_[p] & 3;
            ++p;
            if (p + 16 > end) return fail(err, "bad DHT");
            int counts[17] = {0}, total = 0;
            for (int l = 1; l <= 16; ++l) { counts[l] = d_[p + l - 1]; total += counts[l]; }
            p += 16;
            if (total > 256 || p + total > end) return fail(err, "bad DHT");
            Huffman& hf = tc ? ac_[th] : dc_[th];
            std::memcpy(hf.vals, d_ + p, total);
            p += total;
            // canonical codes (T.81 Annex C)
            int code = 0, k = 0, lastl = 0;
            for (int l = 1; l <= 16; ++l) if (counts[l]) lastl = l;
            std::memset(hf.look, 0, sizeof hf.look);
            for (int l = 1; l <= 16; ++l) {
                hf.valptr[l] = k;
                hf.mincode[l] = code;
                // every code of length l must fit in l bits and not be all ones (libjpeg's
                // JERR_BAD_HUFF_TABLE test, applied up to the longest length in use); an
                // oversubscribed table would index look[] past its end below
                if (l <= lastl && code + counts[l] >= (1 << l)) return fail(err, "bad DHT");
                for (int i = 0; i < counts[l]; ++i, ++k, ++code)
                    if (l <= 8)
                        for (int fill = 0; fill < (1 << (8 - l)); ++fill)
                            hf.look[(code << (8 - l)) | fill] = static_cast<uint16_t>((l << 8) | hf.vals[k]);
                hf.maxcode[l] = counts[l] ? code - 1 : -1;
                code <<= 1;
            }
            hf.maxcode[17] = 0x7FFFFFFF;
            hf.present = true;
        }
        return true;
    }

    // ---- entropy-coded segment
    void fill(int need) {
        while (cnt_ < need) {
            int b = 0;
            if (!marker_hit_ && pos_ < n_) {
                b = d_[pos_];
                if (b == 0xFF) {
                    const int nx = pos_ + 1 < n_ ? d_[pos_ + 1] : -1;
                    if (nx == 0x00) pos_ += 2;
                    else { marker_hit_ = true; b = 0; }      // a marker: feed zeros (libjpeg does)
                } else {
                    ++pos_;
                }
            }
            buf_ |= static_cast<uint32_t>(b) << (24 - cnt_);
            cnt_ += 8;
        }
    }
    int bits(int n) {
        if (n == 0) return 0;
        fill(n);
        const int v = static_cast<int>(buf_ >> (32 - n));
        buf_ <<= n;
        cnt_ -= n;
        return v;
    }
    int decode(const Huffman& hf) {
        fill(16);
        const uint16_t e = hf.look[buf_ >> 24];
        if (e) {
            const int l = e >> 8;
            buf_ <<= l;
            cnt_ -= l;
            return e & 0xFF;
        }
        int l = 9;
        int code = static_cast<int>(buf_ >> (32 - l));
        while (l <= 16 && code > hf.maxcode[l]) { ++l; code = static_cast<int>(buf_ >> (32 - l)); }
        if (l > 16) { buf_ <<= 16; cnt_ -= 16; return 0; }     // corrupt data: libjpeg warns, yields 0
        buf_ <<= l;
        cnt_ -= l;
        return hf.vals[hf.valptr[l] + code - hf.mincode[l]];
    }
    static int extend(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }

    void restart_sync() {
        buf_ = 0; cnt_ = 0;
        // skip to the RSTn marker and past it
        while (pos_ + 1 < n_ && !(d_[pos_] == 0xFF && d_[pos_ + 1] >= 0xD0 && d_[pos_ + 1] <= 0xD7)) {
            if (d_[pos_] == 0xFF && d_[pos_ + 1] != 0x00 && d_[pos_ + 1] != 0xFF) break;   // another marker
            ++pos_;
        }
        if (pos_ + 1 < n_ && d_[pos_] == 0xFF && d_[pos_ + 1] >= 0xD0 && d_[pos_ + 1] <= 0xD7) pos_ += 2;
        marker_hit_ = false;
    }

    bool sos(size_t p, size_t end, std::string* err) {
        if (!frame_) return fail(err, "SOS before SOF");
        const int ns = d_[p];
        if (ns < 1 || ns > 4 || end - p < static_cast<size_t>(1 + 2 * ns + 3)) return fail(err, "bad SOS");
        int sc[4];
        for (int i = 0; i < ns; ++i) {
            const int cid = d_[p + 1 + 2 * i], t = d_[p + 2 + 2 * i];
            int ci = -1;
            for (int k = 0; k < ncomp_; ++k) if (comp_[k].id == cid) ci = k;
            if (ci < 0) return fail(err, "bad component in SOS");
            comp_[ci].td = t >> 4;
            comp_[ci].ta = t & 15;
            if (comp_[ci].td > 3 || comp_[ci].ta > 3 || !dc_[comp_[ci].td].present || !ac_[comp_[ci].ta].present)
                return fail(err, "missing Huffman table");
            if (!qt_set_[comp_[ci].tq]) return fail(err, "missing quantisation table");
            comp_[ci].dc_pred = 0;
            sc[i] = ci;
        }
        buf_ = 0; cnt_ = 0; marker_hit_ = false;
        int16_t coef[64];
        int todo = restart_;
        auto block = [&](Component& c, int bx, int by) {
            std::memset(coef, 0, sizeof coef);
            const int t = decode(dc_[c.td]);
            const int diff = t ? extend(bits(t), t) : 0;
            c.dc_pred += diff;
            coef[0] = static_cast<int16_t>(c.dc_pred);
            for (int k = 1; k < 64;) {
                const int rs = decode(ac_[c.ta]);
                const int r = rs >> 4, s = rs & 15;
                if (s) {
                    k += r;
                    const int v = extend(bits(s), s);
                    coef[kNatural[std::min(k, 63 + 16)]] = static_cast<int16_t>(v);
                    ++k;
                } else {
                    if (r != 15) break;
                    k += 16;
                }
            }
            idct_islow(coef, qt_[c.tq], &c.plane[static_cast<size_t>(by) * 8 * c.stride + bx * 8], c.stride);
        };
        auto restart_check = [&]() {
            if (!restart_) return;
            if (todo == 0) {
                restart_sync();
                for (int i = 0; i < ns; ++i) comp_[sc[i]].dc_pred = 0;
                todo = restart_;
            }
            --todo;
        };
        if (ns == 1) {                                 // non-interleaved: the component's own block grid
            Component& c = comp_[sc[0]];
            const int bw = (c.dw + 7) / 8, bh = (c.dh + 7) / 8;
            for (int by = 0; by < bh; ++by)
                for (int bx = 0; bx < bw; ++bx) {
                    restart_check();
                    block(c, bx, by);
                }
        } else {
            for (int my = 0; my < mcuy_; ++my)
                for (int mx = 0; mx < mcux_; ++mx) {
                    restart_check();
                    for (int i = 0; i < ns; ++i) {
                        Component& c = comp_[sc[i]];
                        for (int v = 0; v < c.v; ++v)
                            for (int h = 0; h < c.h; ++h) block(c, mx * c.h + h, my * c.v + v);
                    }
                }
        }
        // leave pos_ at the next marker
        while (pos_ + 1 < n_ && !(d_[pos_] == 0xFF && d_[pos_ + 1] != 0x00 && !(d_[pos_ + 1] >= 0xD0 && d_[pos_ + 1] <= 0xD7)))
            ++pos_;
        return true;
    }

    // ---- jidctint.c: accurate integer IDCT (CONST_BITS 13, PASS1_BITS 2) with the post-IDCT range limit
    static uint8_t range_limit_idct(long long x) {
        int v = static_cast<int>(x & 1023);
        if (v >= 512) v -= 1024;
        v += 128;
        return static_cast<uint8_t>(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
    static void idct_islow(const int16_t* in, const uint16_t* q, uint8_t* out, int stride) {
        typedef long long L;
        const L F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
                F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
        const int CB = 13, P1 = 2;
        int ws[64];
        auto descale = [](L x, int n) { return (x + (L(1) << (n - 1))) >> n; };
        for (int c = 0; c < 8; ++c) {                    // pass 1: columns
            const int16_t* ip = in + c;
            const uint16_t* qp = q + c;
            if (!ip[8] && !ip[16] && !ip[24] && !ip[32] && !ip[40] && !ip[48] && !ip[56]) {
                const int dc = static_cast<int>(L(ip[0]) * qp[0] * (1 << P1));
                for (int r = 0; r < 8; ++r) ws[r * 8 + c] = dc;
                continue;
            }
            L z2 = L(ip[16]) * qp[16], z3 = L(ip[48]) * qp[48];
            L z1 = (z2 + z3) * F0541;
            L tmp2 = z1 + z3 * -F1847, tmp3 = z1 + z2 * F0765;
            z2 = L(ip[0]) * qp[0];
            z3 = L(ip[32]) * qp[32];
            L tmp0 = (z2 + z3) * (L(1) << CB), tmp1 = (z2 - z3) * (L(1) << CB);
            const L t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
            tmp0 = L(ip[56]) * qp[56]; tmp1 = L(ip[40]) * qp[40]; tmp2 = L(ip[24]) * qp[24]; tmp3 = L(ip[8]) * qp[8];
            z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
            L z4 = tmp1 + tmp3;
            const L z5 = (z3 + z4) * F1175;
            tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
            z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
            z3 += z5; z4 += z5;
            tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
            ws[0 * 8 + c] = static_cast<int>(descale(t10 + tmp3, CB - P1));
            ws[7 * 8 + c] = static_cast<int>(descale(t10 - tmp3, CB - P1));
            ws[1 * 8 + c] = static_cast<int>(descale(t11 + tmp2, CB - P1));
            ws[6 * 8 + c] = static_cast<int>(descale(t11 - tmp2, CB - P1));
            ws[2 * 8 + c] = static_cast<int>(descale(t12 + tmp1, CB - P1));
            ws[5 * 8 + c] = static_cast<int>(descale(t12 - tmp1, CB - P1));
            ws[3 * 8 + c] = static_cast<int>(descale(t13 + tmp0, CB - P1));
            ws[4 * 8 + c] = static_cast<int>(descale(t13 - tmp0, CB - P1));
        }
        for (int r = 0; r < 8; ++r) {                    // pass 2: rows
            const int* w = ws + r * 8;
            uint8_t* o = out + static_cast<size_t>(r) * stride;
            if (!w[1] && !w[2] && !w[3] && !w[4] && !w[5] && !w[6] && !w[7]) {
                const uint8_t dc = range_limit_idct(descale(w[0], P1 + 3));
                for (int k = 0; k < 8; ++k) o[k] = dc;
                continue;
            }
            L z2 = w[2], z3 = w[6];
            L z1 = (z2 + z3) * F0541;
            L tmp2 = z1 + z3 * -F1847, tmp3 = z1 + z2 * F0765;
            L tmp0 = (L(w[0]) + w[4]) * (L(1) << CB), tmp1 = (L(w[0]) - w[4]) * (L(1) << CB);
            const L t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
            tmp0 = w[7]; tmp1 = w[5]; tmp2 = w[3]; tmp3 = w[1];
            z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
            L z4 = tmp1 + tmp3;
            const L z5 = (z3 + z4) * F1175;
            tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
            z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
            z3 += z5; z4 += z5;
            tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
            const int S = CB + P1 + 3;
            o[0] = range_limit_idct(descale(t10 + tmp3, S));
            o[7] = range_limit_idct(descale(t10 - tmp3, S));
            o[1] = range_limit_idct(descale(t11 + tmp2, S));
            o[6] = range_limit_idct(descale(t11 - tmp2, S));
            o[2] = range_limit_idct(descale(t12 + tmp1, S));
            o[5] = range_limit_idct(descale(t12 - tmp1, S));
            o[3] = range_limit_idct(descale(t13 + tmp0, S));
            o[4] = range_limit_idct(descale(t13 - tmp0, S));
        }
    }

    // ---- jdsample.c: upsample component c to the full (hmax, vmax) grid; rows/cols past the
    // downsampled size replicate the last real one (jdmainct.c's context pointers)
    std::vector<uint8_t> upsample(const Component& c, int* out_stride) const {
        const int ow = c.dw * (hmax_ / c.h), oh = c.dh * (vmax_ / c.v);
        std::vector<uint8_t> o(static_cast<size_t>(ow) * oh);
        *out_stride = ow;
        auto in = [&](int y, int x) -> int {
            y = std::max(0, std::min(y, c.dh - 1));
            return c.plane[static_cast<size_t>(y) * c.stride + x];
        };
        const int fh = hmax_ / c.h, fv = vmax_ / c.v;
        if (fh == 1 && fv == 1) {
            for (int y = 0; y < oh; ++y) std::memcpy(&o[static_cast<size_t>(y) * ow], &c.plane[static_cast<size_t>(y) * c.stride], ow);
        } else if (fh == 2 && fv == 1 && c.dw > 2) {                 // h2v1_fancy_upsample
            for (int y = 0; y < oh; ++y) {
                uint8_t* op = &o[static_cast<size_t>(y) * ow];
                const int n = c.dw;
                op[0] = static_cast<uint8_t>(in(y, 0));
                op[1] = static_cast<uint8_t>((in(y, 0) * 3 + in(y, 1) + 2) >> 2);
                for (int x = 1; x < n - 1; ++x) {
                    const int v3 = in(y, x) * 3;
                    op[2 * x] = static_cast<uint8_t>((v3 + in(y, x - 1) + 1) >> 2);
                    op[2 * x + 1] = static_cast<uint8_t>((v3 + in(y, x + 1) + 2) >> 2);
                }
                op[2 * n - 2] = static_cast<uint8_t>((in(y, n - 1) * 3 + in(y, n - 2) + 1) >> 2);
                op[2 * n - 1] = static_cast<uint8_t>(in(y, n - 1));
            }
        } else if (fh == 1 && fv == 2) {                             // h1v2_fancy_upsample
            for (int y = 0; y < oh; ++y) {
                const int iy = y >> 1, far = (y & 1) ? iy + 1 : iy - 1, bias = (y & 1) ? 2 : 1;
                uint8_t* op = &o[static_cast<size_t>(y) * ow];
                for (int x = 0; x < ow; ++x) op[x] = static_cast<uint8_t>((in(iy, x) * 3 + in(far, x) + bias) >> 2);
            }
        } else if (fh == 2 && fv == 2 && c.dw > 2) {                 // h2v2_fancy_upsample
            std::vector<int> cs(c.dw);
            for (int y = 0; y < oh; ++y) {
                const int iy = y >> 1, far = (y & 1) ? iy + 1 : iy - 1;
                for (int x = 0; x < c.dw; ++x) cs[x] = in(iy, x) * 3 + in(far, x);
                uint8_t* op = &o[static_cast<size_t>(y) * ow];
                const int n = c.dw;
                op[0] = static_cast<uint8_t>((cs[0] * 4 + 8) >> 4);
                op[1] = static_cast<uint8_t>((cs[0] * 3 + cs[1] + 7) >> 4);
                for (int x = 1; x < n - 1; ++x) {
                    op[2 * x] = static_cast<uint8_t>((cs[x] * 3 + cs[x - 1] + 8) >> 4);
                    op[2 * x + 1] = static_cast<uint8_t>((cs[x] * 3 + cs[x + 1] + 7) >> 4);
                }
                op[2 * n - 2] = static_cast<uint8_t>((cs[n - 1] * 3 + cs[n - 2] + 8) >> 4);
                op[2 * n - 1] = static_cast<uint8_t>((cs[n - 1] * 4 + 7) >> 4);
            }
        } else {                                                     // int_upsample / h2v1 / h2v2: replicate
            for (int y = 0; y < oh; ++y)
                for (int x = 0; x < ow; ++x) o[static_cast<size_t>(y) * ow + x] = static_cast<uint8_t>(in(y / fv, x / fh));
        }
        return o;
    }

    bool emit(bool want_color, JpegImage* out, std::string* err) {
        out->width = W_;
        out->height = H_;
        out->channels = want_color ? 3 : 1;
        out->pixels.assign(static_cast<size_t>(W_) * H_ * out->channels, 0);
        // colour space (jdapimin.c default_decompress_parms)
        bool rgb = false;
        if (ncomp_ == 3) {
            if (jfif_) rgb = false;
            else if (adobe_) rgb = adobe_transform_ == 0;
            else rgb = comp_[0].id == 'R' && comp_[1].id == 'G' && comp_[2].id == 'B';
        }
        if (ncomp_ == 1 || !want_color) {
            int st0;
            const std::vector<uint8_t> y = upsample(comp_[0], &st0);
            if (ncomp_ == 3 && rgb) {                                // rgb_gray_convert (jdcolor.c)
                int s1, s2;
                const std::vector<uint8_t> g = upsample(comp_[1], &s1), b = upsample(comp_[2], &s2);
                const long long FR = 19595, FG = 38470, FB = 7471, HALF = 1LL << 15;   // FIX(0.299/0.587/0.114)
                for (int r = 0; r < H_; ++r)
                    for (int x = 0; x < W_; ++x) {
                        const long long v = FR * y[static_cast<size_t>(r) * st0 + x] + FG * g[static_cast<size_t>(r) * s1 + x] +
                                            FB * b[static_cast<size_t>(r) * s2 + x] + HALF;
                        const uint8_t gy = static_cast<uint8_t>(v >> 16);
                        for (int k = 0; k < out->channels; ++k) out->pixels[(static_cast<size_t>(r) * W_ + x) * out->channels + k] = gy;
                    }
                return true;
            }
            for (int r = 0; r < H_; ++r)
                for (int x = 0; x < W_; ++x) {
                    const uint8_t v = y[static_cast<size_t>(r) * st0 + x];
                    for (int k = 0; k < out->channels; ++k) out->pixels[(static_cast<size_t>(r) * W_ + x) * out->channels + k] = v;
                }
            return true;
        }
        int s0, s1, s2;
        const std::vector<uint8_t> c0 = upsample(comp_[0], &s0), c1 = upsample(comp_[1], &s1), c2 = upsample(comp_[2], &s2);
        if (rgb) {
            for (int r = 0; r < H_; ++r)
                for (int x = 0; x < W_; ++x) {
                    uint8_t* o = &out->pixels[(static_cast<size_t>(r) * W_ + x) * 3];
                    o[2] = c0[static_cast<size_t>(r) * s0 + x];
                    o[1] = c1[static_cast<size_t>(r) * s1 + x];
                    o[0] = c2[static_cast<size_t>(r) * s2 + x];
                }
            return true;
        }
        // ycc_rgb_convert with jdcolor.c's tables (SCALEBITS 16)
        int crr[256], cbb[256];
        long long crg[256], cbg[256];
        const long long HALF = 1LL << 15;
        auto FIX = [](double v) { return static_cast<long long>(v * 65536.0 + 0.5); };
        for (int i = 0; i < 256; ++i) {
            const long long x = i - 128;
            crr[i] = static_cast<int>((FIX(1.40200) * x + HALF) >> 16);
            cbb[i] = static_cast<int>((FIX(1.77200) * x + HALF) >> 16);
            crg[i] = -FIX(0.71414) * x;
            cbg[i] = -FIX(0.34414) * x + HALF;
        }
        auto clamp = [](int v) { return static_cast<uint8_t>(v < 0 ? 0 : (v > 255 ? 255 : v)); };
        for (int r = 0; r < H_; ++r)
            for (int x = 0; x < W_; ++x) {
                const int y = c0[static_cast<size_t>(r) * s0 + x], cb = c1[static_cast<size_t>(r) * s1 + x],
                          cr = c2[static_cast<size_t>(r) * s2 + x];
                uint8_t* o = &out->pixels[(static_cast<size_t>(r) * W_ + x) * 3];
                o[2] = clamp(y + crr[cr]);
                o[1] = clamp(y + static_cast<int>((cbg[cb] + crg[cr]) >> 16));
                o[0] = clamp(y + cbb[cb]);
            }
        (void)err;
        return true;
    }
};

}  // namespace

bool DecodeJpegMemory(const uint8_t* data, size_t size, bool want_color, JpegImage* out, std::string* error) {
    Decoder d(data, size);
    return d.decode(want_color, out, error);
}

bool DecodeJpegFile(const std::string& path, bool want_color, JpegImage* out, std::string* error) {
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        if (error) *error = "cannot open " + path;
        return false;
    }
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    return DecodeJpegMemory(buf.data(), buf.size(), want_color, out, error);
}

}  // namespace acmmp_host
