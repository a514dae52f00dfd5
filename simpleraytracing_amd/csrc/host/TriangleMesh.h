// TriangleMesh.h -- triangle mesh of the drop-in host API.
//
// Interface of the reference's TriangleMesh (include/TriangleMesh.h:106-169)
// for geometry: triangle soups or indexed vertex sets (optionally with texture
// coordinates), the triangle accessors, the bounding box
// (src/TriangleMesh.cxx:192-228) and intersectBBox, which the reference
// stubs to `true` (include/TriangleMesh.inl:232-235) and so does this.
// Materials and textures belong to the Phong renderer, which is out of scope.
#pragma once

#include <cstddef>
#include <vector>

#include "Ray.h"
#include "Triangle.h"
#include "Vec3.h"

class TriangleMesh {
public:
    TriangleMesh() = default;
    explicit TriangleMesh(const std::vector<float>& vertices) { setGeometry(vertices); }
    TriangleMesh(const std::vector<float>& vertices, const std::vector<unsigned int>& indices)
    {
        setGeometry(vertices, indices);
    }
    TriangleMesh(const std::vector<float>& vertices, const std::vector<float>& texcoords)
    {
        setGeometry(vertices, texcoords);
    }
    TriangleMesh(const std::vector<float>& vertices, const std::vector<unsigned int>& indices,
                 const std::vector<float>& texcoords)
    {
        setGeometry(vertices, indices, texcoords);
    }
    explicit TriangleMesh(const std::vector<Triangle>& triangles) { setGeometry(triangles); }

    // 9 floats per triangle (throws std::length_error otherwise, as the reference)
    void setGeometry(const std::vector<float>& vertices);
    // xyz per vertex + 3 indices per triangle
    void setGeometry(const std::vector<float>& vertices, const std::vector<unsigned int>& indices);
    void setGeometry(const std::vector<float>& vertices, const std::vector<float>& texcoords);
    void setGeometry(const std::vector<float>& vertices, const std::vector<unsigned int>& indices,
                     const std::vector<float>& texcoords);
    void setGeometry(const std::vector<Triangle>& triangles);

    size_t getNumberOfTriangles() const { return m_triangles.size(); }
    const Triangle& getTriangle(unsigned int i) const { return m_triangles[i]; }

    const Vec3& getLowerBBoxCorner() const { return m_lower; }
    const Vec3& getUpperBBoxCorner() const { return m_upper; }

    bool intersectBBox(const Ray&) const { return true; }

    // p1, p2, p3 of every triangle, 9 f32 each: the ABI's mesh layout.
    std::vector<float> flatten() const;

private:
    void computeBoundingBox();

    std::vector<Triangle> m_triangles;
    Vec3 m_lower, m_upper;
};
