// Ray.h -- ray of the drop-in host API (include/Ray.h:84-107).
//
// The constructor normalises the direction unless its length is zero, as
// include/Ray.inl:74-85 does.  Ray::intersect is src/Ray.cxx:72-124 on the
// host (the drop-in class's single-pair utility); renderLoop's kernel is the
// bulk path.
#pragma once

#include <vector>

#include "Triangle.h"
#include "Vec3.h"

class Ray {
public:
    Ray(const Vec3& origin, const Vec3& direction) : m_origin(origin)
    {
        float len = direction.getLength();
        if (std::fpclassify(len) != FP_ZERO) m_direction = direction / len;
    }

    const Vec3& getOrigin() const { return m_origin; }
    const Vec3& getDirection() const { return m_direction; }
    void setOrigin(const Vec3& p) { m_origin = p; }
    void setDirection(const Vec3& d) { m_direction = d / d.getLength(); }
    Vec3 getPointAt(float t) const { return m_origin + m_direction * t; }

    // src/Ray.cxx:72-124.
    bool intersect(const Triangle& triangle, float& t) const;

private:
    Vec3 m_origin;
    Vec3 m_direction;
};

// Batched form: hits[i] / ts[i] for (rays[i], triangles[i]).
void intersectBatch(const std::vector<Ray>& rays, const std::vector<Triangle>& triangles,
                    std::vector<unsigned char>& hits, std::vector<float>& ts);
