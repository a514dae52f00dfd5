// Image.h -- single-channel float image of the drop-in host API.
//
// Interface of the reference's Image (include/Image.h:35-215): a row-major
// float buffer (index row * width + col, include/Image.inl:147), bounds-
// checked setPixel/getPixel that throw std::out_of_range, and saveTextFile
// writing what the reference writes (src/Image.cxx:210-235).  applyLUT is the
// reference's intended 8-bit mapping with its indexing bug fixed
// (include/Image.inl:189-216 reads [i*3] and writes [i]); saveTGAFile writes
// that LUT as an uncompressed 24-bit TGA (src/Image.cxx:148-206) and
// saveJPEGFile as a baseline JPEG, quality 100 (src/Image.cxx:85-144; host/Jpeg.cpp,
// an encoder of its own: this image has no libjpeg headers).
#pragma once

#include <string>
#include <vector>

class Image {
public:
    Image();
    Image(const Image& other);
    Image(unsigned int width, unsigned int height, float value = 0);
    ~Image();
    Image& operator=(const Image& other);

    void destroy();

    void saveTextFile(const std::string& file_name) const;
    void saveTGAFile(const std::string& file_name, float vmin = 0.0, float vmax = 1.0) const;
    void saveJPEGFile(const std::string& file_name, float vmin = 0.0, float vmax = 1.0) const;
    // Binary 8-bit greyscale PGM of applyLUT's first channel.
    void savePGMFile(const std::string& file_name, float vmin = 0.0, float vmax = 1.0) const;

    void getSize(unsigned int& width, unsigned int& height) const;
    unsigned int getWidth() const { return m_width; }
    unsigned int getHeight() const { return m_height; }
    float* getData() const { return m_data; }

    void setPixel(unsigned int col, unsigned int row, float value);
    void getPixel(unsigned int col, unsigned int row, float& value) const;

    // RGB triplets (three equal channels), 3 * width * height bytes.
    std::vector<unsigned char> applyLUT(float vmin, float vmax) const;

protected:
    void setSize(unsigned int width, unsigned int height, float value = 0);

    float* m_data = nullptr;
    unsigned int m_width = 0;
    unsigned int m_height = 0;
};

// The per-pixel LUT value: v < vmin -> 0, v > vmax -> 255, otherwise
// round(255 * (v - vmin) / (vmax - vmin)) with (v - vmin) in float and the rest
// in double (include/Image.inl:195-211).  NaN maps to 0.
unsigned char lutValue(float v, float vmin, float vmax);
