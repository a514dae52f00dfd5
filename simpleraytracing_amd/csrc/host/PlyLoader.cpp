// PlyLoader.cpp -- see PlyLoader.h.
#include "PlyLoader.h"

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace {

enum class Scalar { I8, U8, I16, U16, I32, U32, F32, F64 };

struct Property {
    std::string name;
    Scalar type = Scalar::F32;
    bool is_list = false;
    Scalar count_type = Scalar::U8;
};

struct Element {
    std::string name;
    uint64_t count = 0;
    std::vector<Property> props;
};

Scalar parse_scalar(const std::string& s)
{
    if (s == "char" || s == "int8") return Scalar::I8;
    if (s == "uchar" || s == "uint8") return Scalar::U8;
    if (s == "short" || s == "int16") return Scalar::I16;
    if (s == "ushort" || s == "uint16") return Scalar::U16;
    if (s == "int" || s == "int32") return Scalar::I32;
    if (s == "uint" || s == "uint32") return Scalar::U32;
    if (s == "float" || s == "float32") return Scalar::F32;
    if (s == "double" || s == "float64") return Scalar::F64;
    throw std::runtime_error("PLY: unknown property type '" + s + "'");
}

size_t scalar_size(Scalar t)
{
    switch (t) {
    case Scalar::I8: case Scalar::U8: return 1;
    case Scalar::I16: case Scalar::U16: return 2;
    case Scalar::I32: case Scalar::U32: case Scalar::F32: return 4;
    case Scalar::F64: return 8;
    }
    return 0;
}

class Reader {
public:
    Reader(const std::vector<char>& buf, size_t pos, int format)
        : m_buf(buf), m_pos(pos), m_format(format) {}

    // Reads one value; integers come back exactly, floats as double.
    double read(Scalar t)
    {
        if (m_format == 0) return read_ascii();
        size_t n = scalar_size(t);
        if (m_pos + n > m_buf.size()) throw std::runtime_error("PLY: unexpected end of file");
        unsigned char b[8];
        std::memcpy(b, m_buf.data() + m_pos, n);
        m_pos += n;
        if (m_format == 2) std::reverse(b, b + n);   // big endian
        switch (t) {
        case Scalar::I8: return (double)(int8_t)b[0];
        case Scalar::U8: return (double)b[0];
        case Scalar::I16: { int16_t v; std::memcpy(&v, b, 2); return v; }
        case Scalar::U16: { uint16_t v; std::memcpy(&v, b, 2); return v; }
        case Scalar::I32: { int32_t v; std::memcpy(&v, b, 4); return v; }
        case Scalar::U32: { uint32_t v; std::memcpy(&v, b, 4); return v; }
        case Scalar::F32: { float v; std::memcpy(&v, b, 4); return v; }
        case Scalar::F64: { double v; std::memcpy(&v, b, 8); return v; }
        }
        return 0.0;
    }

    // float values are returned through float so the vertex keeps its f32 bits
    float read_float(Scalar t)
    {
        if (m_format != 0 && t == Scalar::F32) {
            if (m_pos + 4 > m_buf.size()) throw std::runtime_error("PLY: unexpected end of file");
            unsigned char b[4];
            std::memcpy(b, m_buf.data() + m_pos, 4);
            m_pos += 4;
            if (m_format == 2) std::reverse(b, b + 4);
            float v;
            std::memcpy(&v, b, 4);
            return v;
        }
        return (float)read(t);
    }

private:
    double read_ascii()
    {
        while (m_pos < m_buf.size() && std::isspace((unsigned char)m_buf[m_pos])) ++m_pos;
        if (m_pos >= m_buf.size()) throw std::runtime_error("PLY: unexpected end of file");
        const char* start = m_buf.data() + m_pos;
        char* end = nullptr;
        double v = std::strtod(start, &end);
        if (end == start) throw std::runtime_error("PLY: malformed ascii value");
        m_pos += (size_t)(end - start);
        return v;
    }

    const std::vector<char>& m_buf;
    size_t m_pos;
    int m_format;   // 0 ascii, 1 little endian, 2 big endian
};

}  // namespace

PlyMesh loadPly(const std::string& file_name)
{
    std::ifstream in(file_name, std::ios::binary);
    if (!in) throw std::runtime_error("Cannot open the file " + file_name);
    // the whole file in one read (a byte-at-a-time istreambuf_iterator copy
    // was most of a 434-KB mesh's load time)
    in.seekg(0, std::ios::end);
    const std::streamoff size = in.tellg();
    in.seekg(0, std::ios::beg);
    std::vector<char> buf(size > 0 ? (size_t)size : 0u);
    if (size > 0 && !in.read(buf.data(), size)) throw std::runtime_error("Cannot read the file " + file_name);

    size_t pos = 0;
    auto next_line = [&](std::string& line) {
        size_t eol = pos;
        while (eol < buf.size() && buf[eol] != '\n') ++eol;
        if (eol >= buf.size()) throw std::runtime_error("PLY: truncated header in " + file_name);
        line.assign(buf.data() + pos, eol - pos);
        if (!line.empty() && line.back() == '\r') line.pop_back();
        pos = eol + 1;
    };

    std::string line;
    next_line(line);
    if (line != "ply") throw std::runtime_error("Not a PLY file: " + file_name);
    int format = -1;
    std::vector<Element> elements;
    for (;;) {
        next_line(line);
        std::istringstream ss(line);
        std::string kw;
        ss >> kw;
        if (kw == "format") {
            std::string f;
            ss >> f;
            if (f == "ascii") format = 0;
            else if (f == "binary_little_endian") format = 1;
            else if (f == "binary_big_endian") format = 2;
            else throw std::runtime_error("PLY: unknown format " + f);
        } else if (kw == "element") {
            Element e;
            ss >> e.name >> e.count;
            elements.push_back(e);
        } else if (kw == "property") {
            if (elements.empty()) throw std::runtime_error("PLY: property before element");
            Property p;
            std::string t;
            ss >> t;
            if (t == "list") {
                std::string ct, it;
                ss >> ct >> it >> p.name;
                p.is_list = true;
                p.count_type = parse_scalar(ct);
                p.type = parse_scalar(it);
            } else {
                p.type = parse_scalar(t);
                ss >> p.name;
            }
            elements.back().props.push_back(p);
        } else if (kw == "end_header") {
            break;
        }
    }
    if (format < 0) throw std::runtime_error("PLY: missing format line in " + file_name);

    PlyMesh mesh;
    Reader rd(buf, pos, format);
    uint64_t num_vertices = 0;
    for (const Element& e : elements) {
        const bool is_vertex = e.name == "vertex";
        const bool is_face = e.name == "face";
        int ix = -1, iy = -1, iz = -1;
        for (size_t k = 0; k < e.props.size(); ++k) {
            if (e.props[k].name == "x") ix = (int)k;
            if (e.props[k].name == "y") iy = (int)k;
            if (e.props[k].name == "z") iz = (int)k;
        }
        if (is_vertex) {
            if (ix < 0 || iy < 0 || iz < 0) throw std::runtime_error("PLY: vertex without x/y/z");
            num_vertices = e.count;
            mesh.vertices.resize(3 * e.count);
        }
        std::vector<uint64_t> poly;
        for (uint64_t r = 0; r < e.count; ++r) {
            for (size_t k = 0; k < e.props.size(); ++k) {
                const Property& p = e.props[k];
                if (!p.is_list) {
                    if (is_vertex && ((int)k == ix || (int)k == iy || (int)k == iz)) {
                        float v = rd.read_float(p.type);
                        mesh.vertices[3 * r + ((int)k == ix ? 0 : (int)k == iy ? 1 : 2)] = v;
                    } else {
                        rd.read(p.type);
                    }
                    continue;
                }
                uint64_t n = (uint64_t)rd.read(p.count_type);
                poly.resize(n);
                for (uint64_t q = 0; q < n; ++q) poly[q] = (uint64_t)rd.read(p.type);
                if (!is_face || (p.name != "vertex_indices" && p.name != "vertex_index")) continue;
                for (uint64_t q = 1; q + 1 < n; ++q) {
                    for (uint64_t id : {poly[0], poly[q], poly[q + 1]}) {
                        if (id >= num_vertices)
                            throw std::runtime_error("PLY: face index out of range in " + file_name);
                        mesh.indices.push_back((unsigned int)id);
                    }
                }
            }
        }
    }
    return mesh;
}
