// Vec3.h -- 3-component float vector of the drop-in host API.
//
// Same interface and, crucially, the same rounding as the reference's Vec3
// (include/Vec3.h:138-201, include/Vec3.inl): components are f32; scaling by a
// float is an f32 multiply, scaling by a double is done in double and narrowed
// (Vec3.inl:229-241); dot products sum left to right (:313-317); normalise
// divides by a correctly rounded sqrtf length (:461-476).  Host code only;
// the kernels restate these operations in kernels/xrt_device.h.
#pragma once

#include <cmath>
#include <ostream>
#include <stdexcept>

class Vec3 {
public:
    Vec3(float x = 0.0, float y = 0.0, float z = 0.0) : m_v{x, y, z} {}
    Vec3(const Vec3& o) = default;
    Vec3& operator=(const Vec3& o) = default;

    Vec3 operator-() const { return Vec3(-m_v[0], -m_v[1], -m_v[2]); }
    Vec3 operator+(const Vec3& o) const { return Vec3(m_v[0] + o.m_v[0], m_v[1] + o.m_v[1], m_v[2] + o.m_v[2]); }
    Vec3 operator-(const Vec3& o) const { return Vec3(m_v[0] - o.m_v[0], m_v[1] - o.m_v[1], m_v[2] - o.m_v[2]); }
    Vec3& operator+=(const Vec3& o) { return *this = *this + o; }
    Vec3& operator-=(const Vec3& o) { return *this = *this - o; }

    Vec3 operator*(float s) const { return Vec3(m_v[0] * s, m_v[1] * s, m_v[2] * s); }
    Vec3 operator/(float s) const { return Vec3(m_v[0] / s, m_v[1] / s, m_v[2] / s); }
    // double scalars: evaluated in double, narrowed per component
    Vec3 operator*(double s) const { return Vec3(float(m_v[0] * s), float(m_v[1] * s), float(m_v[2] * s)); }
    Vec3 operator/(double s) const { return Vec3(float(m_v[0] / s), float(m_v[1] / s), float(m_v[2] / s)); }
    Vec3& operator*=(float s) { return *this = *this * s; }
    Vec3& operator/=(float s) { return *this = *this / s; }
    Vec3& operator*=(double s) { return *this = *this * s; }
    Vec3& operator/=(double s) { return *this = *this / s; }

    // component-wise product
    Vec3 operator*(const Vec3& o) const { return Vec3(m_v[0] * o.m_v[0], m_v[1] * o.m_v[1], m_v[2] * o.m_v[2]); }
    Vec3& operator*=(const Vec3& o) { return *this = *this * o; }

    float dotProduct(const Vec3& o) const { return m_v[0] * o.m_v[0] + m_v[1] * o.m_v[1] + m_v[2] * o.m_v[2]; }
    Vec3 crossProduct(const Vec3& o) const
    {
        return Vec3(m_v[1] * o.m_v[2] - m_v[2] * o.m_v[1],
                    m_v[2] * o.m_v[0] - m_v[0] * o.m_v[2],
                    m_v[0] * o.m_v[1] - m_v[1] * o.m_v[0]);
    }

    float& operator[](unsigned int i)
    {
        if (i > 2) throw std::out_of_range("Valid range is [0, 2]");
        return m_v[i];
    }
    const float& operator[](unsigned int i) const
    {
        if (i > 2) throw std::out_of_range("Valid range is [0, 2]");
        return m_v[i];
    }

    float getX() const { return m_v[0]; }
    float getY() const { return m_v[1]; }
    float getZ() const { return m_v[2]; }
    float getR() const { return m_v[0]; }
    float getG() const { return m_v[1]; }
    float getB() const { return m_v[2]; }
    void setX(float v) { m_v[0] = v; }
    void setY(float v) { m_v[1] = v; }
    void setZ(float v) { m_v[2] = v; }
    void setR(float v) { m_v[0] = v; }
    void setG(float v) { m_v[1] = v; }
    void setB(float v) { m_v[2] = v; }

    float getLength() const { return std::sqrt(dotProduct(*this)); }
    void normalise()
    {
        float len = getLength();
        m_v[0] /= len;
        m_v[1] /= len;
        m_v[2] /= len;
    }
    void normalize() { normalise(); }

private:
    float m_v[3];
};

inline Vec3 operator*(float s, const Vec3& v) { return v * s; }
inline Vec3 operator*(double s, const Vec3& v) { return v * s; }
inline Vec3 normalise(const Vec3& v)
{
    Vec3 r(v);
    r.normalise();
    return r;
}
inline Vec3 normalize(const Vec3& v) { return normalise(v); }
inline float dot(const Vec3& a, const Vec3& b) { return a.dotProduct(b); }
inline Vec3 reflect(const Vec3& I, const Vec3& N) { return I - 2.0 * N.dotProduct(I) * N; }
inline std::ostream& operator<<(std::ostream& os, const Vec3& v)
{
    return os << v.getX() << " " << v.getY() << " " << v.getZ();
}
