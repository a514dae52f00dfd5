// Image.cpp -- see Image.h.
#include "Image.h"

#include "xrt_host.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace {
[[noreturn]] void out_of_range_error(const char* fn, unsigned col, unsigned row, unsigned w, unsigned h)
{
    std::stringstream msg;
    msg << "pixel (" << col << ", " << row << ") outside " << w << "x" << h << " image, in Function "
        << fn;
    throw std::out_of_range(msg.str());
}
}  // namespace

unsigned char lutValue(float v, float vmin, float vmax)
{
    if (v < vmin) return 0;
    if (v > vmax) return 255;
    if (v != v) return 0;
    return (unsigned char)std::round(255.0 * (v - vmin) / (vmax - vmin));
}

Image::Image() = default;

Image::Image(unsigned int width, unsigned int height, float value) { setSize(width, height, value); }

Image::Image(const Image& other) : m_width(other.m_width), m_height(other.m_height)
{
    if (m_width && m_height && other.m_data) {
        m_data = new float[(size_t)m_width * m_height];
        std::memcpy(m_data, other.m_data, sizeof(float) * m_width * m_height);
    }
}

Image::~Image() { destroy(); }

Image& Image::operator=(const Image& other)
{
    if (this == &other) return *this;
    destroy();
    if (other.m_width && other.m_height && other.m_data) {
        setSize(other.m_width, other.m_height);
        std::memcpy(m_data, other.m_data, sizeof(float) * m_width * m_height);
    }
    m_width = other.m_width;
    m_height = other.m_height;
    return *this;
}

void Image::destroy()
{
    delete[] m_data;
    m_data = nullptr;
    m_width = 0;
    m_height = 0;
}

void Image::setSize(unsigned int width, unsigned int height, float value)
{
    if (width == m_width && height == m_height && (m_data || !width || !height)) return;
    destroy();
    m_width = width;
    m_height = height;
    if (width && height) {
        size_t n = (size_t)width * height;
        m_data = new float[n];
        for (size_t i = 0; i < n; ++i) m_data[i] = value;
    }
}

void Image::getSize(unsigned int& width, unsigned int& height) const
{
    width = m_width;
    height = m_height;
}

void Image::setPixel(unsigned int col, unsigned int row, float value)
{
    if (col >= m_width || row >= m_height) out_of_range_error("setPixel", col, row, m_width, m_height);
    m_data[(size_t)row * m_width + col] = value;
}

void Image::getPixel(unsigned int col, unsigned int row, float& value) const
{
    if (col >= m_width || row >= m_height) out_of_range_error("getPixel", col, row, m_width, m_height);
    value = m_data[(size_t)row * m_width + col];
}

// Text layout of src/Image.cxx:225-234: operator<<(float) (6 significant
// digits, %g style), '\t' between columns, '\n' between rows, no trailing
// newline.  snprintf("%.6g") is what libstdc++'s default float formatting uses.
void Image::saveTextFile(const std::string& file_name) const
{
    std::FILE* f = std::fopen(file_name.c_str(), "wb");
    if (!f) throw std::runtime_error("Cannot create the file " + file_name);
    std::vector<char> line;
    char buf[32];
    for (unsigned row = 0; row < m_height; ++row) {
        line.clear();
        for (unsigned col = 0; col < m_width; ++col) {
            int n = std::snprintf(buf, sizeof buf, "%.6g", (double)m_data[(size_t)row * m_width + col]);
            line.insert(line.end(), buf, buf + n);
            if (col + 1 < m_width) line.push_back('\t');
        }
        if (row + 1 < m_height) line.push_back('\n');
        if (!line.empty() && std::fwrite(line.data(), 1, line.size(), f) != line.size()) {
            std::fclose(f);
            throw std::runtime_error("Cannot write the file " + file_name);
        }
    }
    std::fclose(f);
}

std::vector<unsigned char> Image::applyLUT(float vmin, float vmax) const
{
    std::vector<unsigned char> rgb(3 * (size_t)m_width * m_height);
    for (size_t i = 0; i < (size_t)m_width * m_height; ++i) {
        unsigned char v = lutValue(m_data[i], vmin, vmax);
        rgb[3 * i] = rgb[3 * i + 1] = rgb[3 * i + 2] = v;
    }
    return rgb;
}

void Image::saveTGAFile(const std::string& file_name, float vmin, float vmax) const
{
    std::FILE* f = std::fopen(file_name.c_str(), "wb");
    if (!f) throw std::runtime_error("Cannot create the file " + file_name);
    unsigned char header[18] = {0};
    header[2] = 2;   // uncompressed true colour
    header[12] = m_width & 0xFF;
    header[13] = (m_width >> 8) & 0xFF;
    header[14] = m_height & 0xFF;
    header[15] = (m_height >> 8) & 0xFF;
    header[16] = 24;
    std::fwrite(header, 1, sizeof header, f);
    std::vector<unsigned char> rgb = applyLUT(vmin, vmax);
    // bottom-up rows, BGR order
    std::vector<unsigned char> row_buf(3 * (size_t)m_width);
    for (unsigned r = 0; r < m_height; ++r) {
        const unsigned char* src = &rgb[3 * (size_t)m_width * (m_height - 1 - r)];
        for (unsigned c = 0; c < m_width; ++c) {
            row_buf[3 * c + 0] = src[3 * c + 2];
            row_buf[3 * c + 1] = src[3 * c + 1];
            row_buf[3 * c + 2] = src[3 * c + 0];
        }
        std::fwrite(row_buf.data(), 1, row_buf.size(), f);
    }
    std::fclose(f);
}

void Image::savePGMFile(const std::string& file_name, float vmin, float vmax) const
{
    std::FILE* f = std::fopen(file_name.c_str(), "wb");
    if (!f) throw std::runtime_error("Cannot create the file " + file_name);
    std::fprintf(f, "P5\n%u %u\n255\n", m_width, m_height);
    std::vector<unsigned char> g((size_t)m_width * m_height);
    for (size_t i = 0; i < g.size(); ++i) g[i] = lutValue(m_data[i], vmin, vmax);
    std::fwrite(g.data(), 1, g.size(), f);
    std::fclose(f);
}

// C entry point of the image writers (include/xrt_host.h).
extern "C" int xrt_host_save_image(const float* pixels, uint32_t width, uint32_t height, const char* path,
                                   int format, float vmin, float vmax)
{
    if (!path || (!pixels && width && height)) return XRT_ERR_ARGUMENT;
    try {
        Image image(width, height);
        if (width && height) std::memcpy(image.getData(), pixels, sizeof(float) * (size_t)width * height);
        switch (format) {
        case XRT_IMAGE_TEXT: image.saveTextFile(path); break;
        case XRT_IMAGE_TGA: image.saveTGAFile(path, vmin, vmax); break;
        case XRT_IMAGE_PGM: image.savePGMFile(path, vmin, vmax); break;
        case XRT_IMAGE_JPEG: image.saveJPEGFile(path, vmin, vmax); break;
        default: return XRT_ERR_ARGUMENT;
        }
    } catch (const std::exception&) {
        return XRT_ERR_IO;
    }
    return XRT_OK;
}
