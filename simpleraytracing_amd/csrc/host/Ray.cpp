// Ray.cpp -- Ray::intersect (see Ray.h): src/Ray.cxx:72-124 restated over the
// drop-in Vec3 (host/Vec3.h keeps the reference's f32 operation order; the host
// library is built without FMA contraction).  A single-pair utility of the
// drop-in class -- the render path is renderLoop's kernel, which computes the
// same test (xrt_device.h mt_intersect; both checked against the oracle KATs).
#include "Ray.h"

#include <cmath>
#include <stdexcept>

#include "xrt_host.h"

bool Ray::intersect(const Triangle& triangle, float& t) const
{
    const Vec3 edge1 = triangle.getP2() - triangle.getP1();          // Ray.cxx:86
    const Vec3 edge2 = triangle.getP3() - triangle.getP1();          // :87
    const Vec3 pvec = m_direction.crossProduct(edge2);               // :90
    const float det = edge1.dotProduct(pvec);                        // :93
    if (std::fpclassify(det) == FP_ZERO) return false;               // :94
    const float inv_det = (float)(1.0 / (double)det);                // :99
    const Vec3 tvec = m_origin - triangle.getP1();                   // :102
    const float u = tvec.dotProduct(pvec) * inv_det;                 // :105
    if (u < 0.0f || u > 1.0f) return false;                          // :106
    const Vec3 qvec = tvec.crossProduct(edge1);                      // :112
    const float v = m_direction.dotProduct(qvec) * inv_det;          // :115
    if (v < 0.0f || u + v > 1.0f) return false;                      // :116
    t = edge2.dotProduct(qvec) * inv_det;                            // :122
    return true;
}

void intersectBatch(const std::vector<Ray>& rays, const std::vector<Triangle>& triangles,
                    std::vector<unsigned char>& hits, std::vector<float>& ts)
{
    if (rays.size() != triangles.size()) throw std::length_error("intersectBatch: size mismatch");
    hits.assign(rays.size(), 0);
    ts.assign(rays.size(), 0.0f);
    for (size_t i = 0; i < rays.size(); ++i) {
        float t = 0.0f;
        if (rays[i].intersect(triangles[i], t)) {
            hits[i] = 1;
            ts[i] = t;
        }
    }
}

extern "C" void xrt_host_intersect_batch(const float* rays, const float* triangles, uint64_t n, uint8_t* hit,
                                         float* t)
{
    for (uint64_t i = 0; i < n; ++i) {
        const float* r = rays + 6 * i;
        const float* p = triangles + 9 * i;
        const Ray ray(Vec3(r[0], r[1], r[2]), Vec3(r[3], r[4], r[5]));
        const Triangle tri(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]), Vec3(p[6], p[7], p[8]));
        float ti = 0.0f;
        hit[i] = ray.intersect(tri, ti) ? 1 : 0;
        t[i] = hit[i] ? ti : 0.0f;
    }
}
