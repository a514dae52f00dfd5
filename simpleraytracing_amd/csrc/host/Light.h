// Light.h -- the reference's Light (include/Light.h:80-110): colour, direction
// and position of a light source.  RayTracerInfo carries one (main.cxx:117),
// set by initialiseRayTracing (main.cxx:598-601); only the Phong renderer,
// which is out of scope, shades with it -- the X-ray path never reads it.
#pragma once

#include "Vec3.h"

class Light {
public:
    Light() = default;
    Light(const Vec3& colour, const Vec3& direction, const Vec3& position)
        : m_colour(colour), m_direction(direction), m_position(position)
    {
    }

    void setColour(const Vec3& c) { m_colour = c; }
    void setDirection(const Vec3& d) { m_direction = d; }
    void setPosition(const Vec3& p) { m_position = p; }

    Vec3& getColour() { return m_colour; }
    const Vec3& getColour() const { return m_colour; }
    Vec3& getDirection() { return m_direction; }
    const Vec3& getDirection() const { return m_direction; }
    Vec3& getPosition() { return m_position; }
    const Vec3& getPosition() const { return m_position; }

private:
    Vec3 m_colour, m_direction, m_position;
};
