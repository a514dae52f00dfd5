// TriangleMesh.cpp -- see TriangleMesh.h.
#include "TriangleMesh.h"

#include <algorithm>
#include <limits>
#include <stdexcept>

namespace {
inline Vec3 vertex_at(const std::vector<float>& v, size_t i)
{
    return Vec3(v.at(3 * i + 0), v.at(3 * i + 1), v.at(3 * i + 2));
}
}  // namespace

void TriangleMesh::setGeometry(const std::vector<float>& v)
{
    if (v.size() % 9 != 0) throw std::length_error("buffer size error");
    m_triangles.clear();
    m_triangles.reserve(v.size() / 9);
    for (size_t i = 0; i < v.size() / 9; ++i)
        m_triangles.emplace_back(vertex_at(v, 3 * i), vertex_at(v, 3 * i + 1), vertex_at(v, 3 * i + 2));
    computeBoundingBox();
}

void TriangleMesh::setGeometry(const std::vector<float>& v, const std::vector<unsigned int>& idx)
{
    if (v.size() % 3 != 0 || idx.size() % 3 != 0) throw std::length_error("buffer size error");
    m_triangles.clear();
    m_triangles.reserve(idx.size() / 3);
    for (size_t f = 0; f < idx.size(); f += 3)
        m_triangles.emplace_back(vertex_at(v, idx[f]), vertex_at(v, idx[f + 1]), vertex_at(v, idx[f + 2]));
    computeBoundingBox();
}

void TriangleMesh::setGeometry(const std::vector<float>& v, const std::vector<float>& tc)
{
    setGeometry(v);
    if (tc.size() != v.size()) throw std::length_error("buffer size error");
    for (size_t i = 0; i < m_triangles.size(); ++i)
        m_triangles[i].setTextCoords(vertex_at(tc, 3 * i), vertex_at(tc, 3 * i + 1), vertex_at(tc, 3 * i + 2));
}

void TriangleMesh::setGeometry(const std::vector<float>& v, const std::vector<unsigned int>& idx,
                               const std::vector<float>& tc)
{
    setGeometry(v, idx);
    if (tc.size() != v.size()) throw std::length_error("buffer size error");
    for (size_t f = 0, i = 0; f < idx.size(); f += 3, ++i)
        m_triangles[i].setTextCoords(vertex_at(tc, idx[f]), vertex_at(tc, idx[f + 1]), vertex_at(tc, idx[f + 2]));
}

void TriangleMesh::setGeometry(const std::vector<Triangle>& triangles)
{
    m_triangles = triangles;
    computeBoundingBox();
}

// Running min/max over p1, p2, p3 of each triangle with std::min/std::max,
// the order of src/TriangleMesh.cxx:200-227.
void TriangleMesh::computeBoundingBox()
{
    const float inf = std::numeric_limits<float>::infinity();
    m_lower = Vec3(inf, inf, inf);
    m_upper = Vec3(-inf, -inf, -inf);
    for (const Triangle& t : m_triangles) {
        for (const Vec3* p : {&t.getP1(), &t.getP2(), &t.getP3()}) {
            for (unsigned k = 0; k < 3; ++k) {
                m_lower[k] = std::min(m_lower[k], (*p)[k]);
                m_upper[k] = std::max(m_upper[k], (*p)[k]);
            }
        }
    }
}

std::vector<float> TriangleMesh::flatten() const
{
    std::vector<float> out;
    out.reserve(9 * m_triangles.size());
    for (const Triangle& t : m_triangles)
        for (const Vec3* p : {&t.getP1(), &t.getP2(), &t.getP3()})
            for (unsigned k = 0; k < 3; ++k) out.push_back((*p)[k]);
    return out;
}
