// Material.h -- the reference's Material (include/Material.h:86-123): the
// Phong parameters of a mesh.  Declared so code written against the
// reference's headers (applyShading's prototype, main.cxx:133-137) compiles;
// the X-ray path never reads a material.
#pragma once

#include "Vec3.h"

class Material {
public:
    Material() = default;
    Material(const Vec3& ambient, const Vec3& diffuse, const Vec3& specular, float shininess)
        : m_ambient(ambient), m_diffuse(diffuse), m_specular(specular), m_shininess(shininess)
    {
    }

    void setAmbient(const Vec3& v) { m_ambient = v; }
    void setDiffuse(const Vec3& v) { m_diffuse = v; }
    void setSpecular(const Vec3& v) { m_specular = v; }
    void setShininess(float s) { m_shininess = s; }

    Vec3& getAmbient() { return m_ambient; }
    const Vec3& getAmbient() const { return m_ambient; }
    Vec3& getDiffuse() { return m_diffuse; }
    const Vec3& getDiffuse() const { return m_diffuse; }
    Vec3& getSpecular() { return m_specular; }
    const Vec3& getSpecular() const { return m_specular; }
    float& getShininess() { return m_shininess; }
    float getShininess() const { return m_shininess; }

private:
    Vec3 m_ambient, m_diffuse, m_specular;
    float m_shininess = 0.0f;
};
