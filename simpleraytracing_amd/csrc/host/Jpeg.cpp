// Jpeg.cpp -- Image::saveJPEGFile without libjpeg (this image has no libjpeg
// headers): a baseline sequential JPEG encoder written from the JPEG standard
// (ITU-T T.81), configured as the reference configures libjpeg in
// src/Image.cxx:85-144:
//   * RGB input, 3 components, from applyLUT (the fixed LUT: three equal
//     channels, include/Image.inl:189-216 without its [i] / [i*3] bug);
//   * jpeg_set_defaults: YCbCr (JFIF APP0), Y sampled 2x2 and Cb/Cr 1x1
//     (4:2:0), the standard (Annex K) quantisation and Huffman tables;
//   * jpeg_set_quality(100, TRUE): every quantiser 1 (libjpeg's scale factor
//     200 - 2 * 100 = 0 clamps each table entry to 1);
//   * JDCT_FLOAT: a floating-point forward DCT.
// The entropy-coded stream is what a baseline decoder reads; byte parity with
// libjpeg's output is not claimed ("parity unpinned": no libjpeg here to
// compare with).  tests/test_scenes.py decodes the file with PIL.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "Image.h"

namespace {

// Annex K.3 standard Huffman tables (jpeg_set_defaults' std_huff_tables):
// BITS (codes of each length 1..16) then HUFFVAL.
const uint8_t kDcLumBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t kDcLumVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kDcChrBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t kDcChrVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kAcLumBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const uint8_t kAcLumVal[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71,
    0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72,
    0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37,
    0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59,
    0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const uint8_t kAcChrBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const uint8_t kAcChrVal[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22,
    0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1,
    0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36,
    0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58,
    0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a,
    0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba,
    0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

// Zig-zag scan: kZigzag[k] = natural (row-major) index of the k-th coefficient.
const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Annex C: code lengths from BITS, codes assigned in order of length.
struct HuffTable {
    uint16_t code[256] = {};
    uint8_t size[256] = {};
    HuffTable(const uint8_t* bits, const uint8_t* vals)
    {
        uint16_t c = 0;
        int k = 0;
        for (int len = 1; len <= 16; ++len) {
            for (int i = 0; i < bits[len - 1]; ++i, ++k) {
                code[vals[k]] = c++;
                size[vals[k]] = (uint8_t)len;
            }
            c <<= 1;
        }
    }
};

class BitWriter {
public:
    explicit BitWriter(std::vector<uint8_t>& out) : m_out(out) {}
    void put(uint32_t bits, int n)
    {
        for (int i = n - 1; i >= 0; --i) {
            m_acc = (uint8_t)((m_acc << 1) | ((bits >> i) & 1u));
            if (++m_n == 8) emit();
        }
    }
    void flush()                       // pad the last byte with 1 bits (F.1.2.3)
    {
        while (m_n) put(1u, 1);
    }

private:
    void emit()
    {
        m_out.push_back(m_acc);
        if (m_acc == 0xFF) m_out.push_back(0x00);   // byte stuffing
        m_acc = 0;
        m_n = 0;
    }
    std::vector<uint8_t>& m_out;
    uint8_t m_acc = 0;
    int m_n = 0;
};

// Magnitude category and its additional bits (F.1.2.1).
inline void encode_value(BitWriter& bw, const HuffTable& t, int symbol_high, int v)
{
    int a = v < 0 ? -v : v, s = 0;
    while (a) {
        ++s;
        a >>= 1;
    }
    const int sym = (symbol_high << 4) | s;
    bw.put(t.code[sym], t.size[sym]);
    if (s) bw.put((uint32_t)(v < 0 ? v + (1 << s) - 1 : v), s);
}

// Forward DCT-II of an 8x8 block of level-shifted samples (JDCT_FLOAT's
// transform; here evaluated directly in double) and quantisation by 1.
void fdct_quantise(const float in[64], int out[64])
{
    static double c[8][8];
    static bool init = false;
    if (!init) {
        for (int u = 0; u < 8; ++u)
            for (int x = 0; x < 8; ++x)
                c[u][x] = (u == 0 ? std::sqrt(0.125) : 0.5) * std::cos((2 * x + 1) * u * M_PI / 16.0);
        init = true;
    }
    double tmp[64];
    for (int y = 0; y < 8; ++y)
        for (int u = 0; u < 8; ++u) {
            double s = 0.0;
            for (int x = 0; x < 8; ++x) s += c[u][x] * in[y * 8 + x];
            tmp[y * 8 + u] = s;
        }
    for (int v = 0; v < 8; ++v)
        for (int u = 0; u < 8; ++u) {
            double s = 0.0;
            for (int y = 0; y < 8; ++y) s += c[v][y] * tmp[y * 8 + u];
            out[v * 8 + u] = (int)std::lround(s);   // quantiser 1 (quality 100)
        }
}

void put16(std::vector<uint8_t>& o, unsigned v)
{
    o.push_back((uint8_t)(v >> 8));
    o.push_back((uint8_t)v);
}

void put_dht(std::vector<uint8_t>& o, int cls_id, const uint8_t* bits, const uint8_t* vals)
{
    int n = 0;
    for (int i = 0; i < 16; ++i) n += bits[i];
    o.push_back(0xFF);
    o.push_back(0xC4);
    put16(o, (unsigned)(2 + 1 + 16 + n));
    o.push_back((uint8_t)cls_id);
    o.insert(o.end(), bits, bits + 16);
    o.insert(o.end(), vals, vals + n);
}

}  // namespace

// Baseline JPEG of applyLUT(vmin, vmax) (src/Image.cxx:85-144, see above).
void Image::saveJPEGFile(const std::string& file_name, float vmin, float vmax) const
{
    if (!m_width || !m_height || m_width > 65535 || m_height > 65535)
        throw std::runtime_error("saveJPEGFile: a baseline JPEG holds 1..65535 pixels a side: " + file_name);
    const std::vector<unsigned char> rgb = applyLUT(vmin, vmax);
    const unsigned W = m_width, H = m_height;
    // JFIF's YCbCr (libjpeg's jccolor.c coefficients), full resolution
    std::vector<float> Y((size_t)W * H), Cb((size_t)W * H), Cr((size_t)W * H);
    for (size_t i = 0; i < (size_t)W * H; ++i) {
        const float r = rgb[3 * i], g = rgb[3 * i + 1], b = rgb[3 * i + 2];
        Y[i] = 0.299f * r + 0.587f * g + 0.114f * b;
        Cb[i] = -0.168736f * r - 0.331264f * g + 0.5f * b + 128.0f;
        Cr[i] = 0.5f * r - 0.418688f * g - 0.081312f * b + 128.0f;
    }
    // samples past the right / bottom edge repeat the last column / row
    auto at = [&](const std::vector<float>& p, unsigned x, unsigned y) {
        return p[(size_t)std::min(y, H - 1) * W + std::min(x, W - 1)];
    };

    std::vector<uint8_t> o;
    o.reserve((size_t)W * H / 2 + 1024);
    o.insert(o.end(), {0xFF, 0xD8});                                      // SOI
    o.insert(o.end(), {0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0x00,   // APP0 JFIF 1.01, no density
                       0x01, 0x01, 0x00, 0x00, 0x01, 0x00, 0x01, 0x00, 0x00});
    for (int t = 0; t < 2; ++t) {                                         // DQT: all ones (quality 100)
        o.insert(o.end(), {0xFF, 0xDB});
        put16(o, 67);
        o.push_back((uint8_t)t);
        for (int k = 0; k < 64; ++k) o.push_back(1);
    }
    o.insert(o.end(), {0xFF, 0xC0});                                      // SOF0 baseline
    put16(o, 17);
    o.push_back(8);
    put16(o, H);
    put16(o, W);
    o.push_back(3);
    o.insert(o.end(), {1, 0x22, 0, 2, 0x11, 1, 3, 0x11, 1});              // Y 2x2 q0, Cb/Cr 1x1 q1
    put_dht(o, 0x00, kDcLumBits, kDcLumVal);
    put_dht(o, 0x10, kAcLumBits, kAcLumVal);
    put_dht(o, 0x01, kDcChrBits, kDcChrVal);
    put_dht(o, 0x11, kAcChrBits, kAcChrVal);
    o.insert(o.end(), {0xFF, 0xDA, 0x00, 0x0C, 3, 1, 0x00, 2, 0x11, 3, 0x11, 0x00, 0x3F, 0x00});   // SOS

    static const HuffTable dc_lum(kDcLumBits, kDcLumVal), ac_lum(kAcLumBits, kAcLumVal);
    static const HuffTable dc_chr(kDcChrBits, kDcChrVal), ac_chr(kAcChrBits, kAcChrVal);
    BitWriter bw(o);
    int pred[3] = {0, 0, 0};
    auto block = [&](const float in[64], int comp) {
        int q[64];
        fdct_quantise(in, q);
        const HuffTable& dc = comp ? dc_chr : dc_lum;
        const HuffTable& ac = comp ? ac_chr : ac_lum;
        encode_value(bw, dc, 0, q[0] - pred[comp]);
        pred[comp] = q[0];
        int run = 0;
        for (int k = 1; k < 64; ++k) {
            const int v = q[kZigzag[k]];
            if (!v) {
                ++run;
                continue;
            }
            while (run > 15) {                                            // ZRL
                bw.put(ac.code[0xF0], ac.size[0xF0]);
                run -= 16;
            }
            encode_value(bw, ac, run, v);
            run = 0;
        }
        if (run) bw.put(ac.code[0x00], ac.size[0x00]);                     // EOB
    };
    float blk[64];
    for (unsigned my = 0; my < (H + 15) / 16; ++my)
        for (unsigned mx = 0; mx < (W + 15) / 16; ++mx) {
            for (unsigned b = 0; b < 4; ++b) {                            // four 8x8 Y blocks
                const unsigned x0 = mx * 16 + (b & 1) * 8, y0 = my * 16 + (b >> 1) * 8;
                for (unsigned y = 0; y < 8; ++y)
                    for (unsigned x = 0; x < 8; ++x) blk[y * 8 + x] = at(Y, x0 + x, y0 + y) - 128.0f;
                block(blk, 0);
            }
            for (int c = 1; c <= 2; ++c) {                                // Cb, Cr: 2x2 averages
                const std::vector<float>& p = c == 1 ? Cb : Cr;
                for (unsigned y = 0; y < 8; ++y)
                    for (unsigned x = 0; x < 8; ++x) {
                        const unsigned sx = mx * 16 + 2 * x, sy = my * 16 + 2 * y;
                        blk[y * 8 + x] = 0.25f * (at(p, sx, sy) + at(p, sx + 1, sy) + at(p, sx, sy + 1) +
                                                  at(p, sx + 1, sy + 1)) - 128.0f;
                    }
                block(blk, c);
            }
        }
    bw.flush();
    o.insert(o.end(), {0xFF, 0xD9});                                      // EOI

    std::FILE* f = std::fopen(file_name.c_str(), "wb");
    if (!f) throw std::runtime_error("Cannot create the file " + file_name);
    const bool ok = std::fwrite(o.data(), 1, o.size(), f) == o.size();
    std::fclose(f);
    if (!ok) throw std::runtime_error("Cannot write the file " + file_name);
}
