// Triangle.h -- triangle of the drop-in host API.
//
// Interface of the reference's Triangle (include/Triangle.h:92-136): three
// vertices, an optional texture coordinate per vertex, and a unit normal
// computed from (p2 - p1) x (p3 - p1) (include/Triangle.inl:170-178).  The
// render path only consumes p1, p2, p3 (flattened to a soup for the ABI).
#pragma once

#include <cmath>
#include <ostream>

#include "Vec3.h"

class Triangle {
public:
    Triangle(const Vec3& a, const Vec3& b, const Vec3& c, const Vec3& ta = Vec3(),
             const Vec3& tb = Vec3(), const Vec3& tc = Vec3())
        : m_p1(a), m_p2(b), m_p3(c), m_tex1(ta), m_tex2(tb), m_tex3(tc)
    {
        computeNormal();
    }

    const Vec3& getP1() const { return m_p1; }
    const Vec3& getP2() const { return m_p2; }
    const Vec3& getP3() const { return m_p3; }
    const Vec3& getNormal() const { return m_normal; }
    const Vec3& getTextCoord1() const { return m_tex1; }
    const Vec3& getTextCoord2() const { return m_tex2; }
    const Vec3& getTextCoord3() const { return m_tex3; }

    void setVertices(const Vec3& a, const Vec3& b, const Vec3& c)
    {
        m_p1 = a;
        m_p2 = b;
        m_p3 = c;
        computeNormal();
    }
    void setTextCoords(const Vec3& a, const Vec3& b, const Vec3& c)
    {
        m_tex1 = a;
        m_tex2 = b;
        m_tex3 = c;
    }

    // Half the cross-product magnitude: f32 components, squared and summed in
    // double, as include/Triangle.inl:206-214 (pow(float, 2) promotes) does.
    float getArea() const
    {
        Vec3 ab = m_p2 - m_p1, ac = m_p3 - m_p1;
        float cx = ab[1] * ac[2] - ab[2] * ac[1];
        float cy = ab[2] * ac[0] - ab[0] * ac[2];
        float cz = ab[0] * ac[1] - ab[1] * ac[0];
        double s = (double)cx * cx + (double)cy * cy + (double)cz * cz;
        return (float)(0.5 * std::sqrt(s));
    }

private:
    void computeNormal()
    {
        m_normal = (m_p2 - m_p1).crossProduct(m_p3 - m_p1);
        m_normal.normalise();
    }

    Vec3 m_p1, m_p2, m_p3;
    Vec3 m_normal;
    Vec3 m_tex1, m_tex2, m_tex3;
};

inline std::ostream& operator<<(std::ostream& os, const Triangle& t)
{
    os << "facet normal " << t.getNormal() << "\nouter loop\n";
    os << "    vertex " << t.getP1() << "\n    vertex " << t.getP2() << "\n    vertex " << t.getP3() << "\n";
    return os << "endloop\nendfacet";
}
