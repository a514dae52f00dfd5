// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/libxrt_ref.so).
//
// Drives the reference's own, unmodified classes -- Vec3 (include/Vec3.inl),
// Ray (include/Ray.inl + src/Ray.cxx), Triangle (include/Triangle.inl +
// src/Triangle.cxx) and TriangleMesh (include/TriangleMesh.inl +
// src/TriangleMesh.cxx) -- compiled from /root/reference by oracle/Makefile.
// No reference source is copied and no header is stubbed: src/main.cxx itself
// needs Assimp and libjpeg headers this image lacks, so it is NOT built; the
// per-pixel loop below is this repo's restatement of renderLoop
// (src/main.cxx:649-742) written against the reference's classes, so that the
// arithmetic that matters (ray set-up, Ray ctor, Ray::intersect, Vec3 rounding)
// is the reference's own compiled code.
//
// Used only to pin oracle/xrt_oracle.c (tests/test_oracle.py) and, optionally,
// as bench.py's "reference" CPU baseline.  Never shipped to the product path.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "Ray.h"
#include "Triangle.h"
#include "TriangleMesh.h"
#include "Vec3.h"

extern "C" {

// Ray::intersect known-answer entry: rays[6i] = origin, direction (the Ray
// ctor re-normalises the direction, include/Ray.inl:74-85, exactly as in the
// reference call path); tris[9i] = p1, p2, p3.
void ref_intersect_batch(const float* rays, const float* tris, uint64_t n,
                         uint8_t* hit, float* t_out)
{
    for (uint64_t i = 0; i < n; ++i) {
        const float* r = rays + 6 * i;
        const float* p = tris + 9 * i;
        Ray ray(Vec3(r[0], r[1], r[2]), Vec3(r[3], r[4], r[5]));
        Triangle tri(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]), Vec3(p[6], p[7], p[8]));
        float t = 0.0f;
        bool h = ray.intersect(tri, t);
        hit[i] = h ? 1 : 0;
        t_out[i] = h ? t : 0.0f;
    }
}

// Bounding box through TriangleMesh::setGeometry(vertices, indices)
// (src/TriangleMesh.cxx:104-131) and computeBoundingBox (:192-228).
void ref_mesh_bbox(const float* tris, uint64_t ntris, float lower[3], float upper[3])
{
    std::vector<float> v(tris, tris + 9 * ntris);
    std::vector<unsigned int> idx(3 * ntris);
    for (uint64_t i = 0; i < 3 * ntris; ++i) idx[i] = (unsigned int)i;
    TriangleMesh mesh(v, idx);
    for (int k = 0; k < 3; ++k) {
        lower[k] = mesh.getLowerBBoxCorner()[k];
        upper[k] = mesh.getUpperBBoxCorner()[k];
    }
}

// Camera restated over the reference's Vec3 (initialiseRayTracing,
// src/main.cxx:575-604, and the renderLoop prologue :637-641).
// cam[0..2] origin, [3..5] detector, [6..8] up, [9..11] right, [12] spacing.
void ref_camera(const float lower_in[3], const float upper_in[3], uint32_t width,
                uint32_t height, float cam[13])
{
    Vec3 lower(lower_in[0], lower_in[1], lower_in[2]);
    Vec3 upper(upper_in[0], upper_in[1], upper_in[2]);
    Vec3 range = upper - lower;
    Vec3 centre = lower + range / 2.0;
    float diagonal = range.getLength();
    Vec3 up(0.0, 0.0, -1.0);
    Vec3 origin(centre - Vec3(diagonal * 1, 0, 0));
    Vec3 detector(centre + Vec3(diagonal * 0.6, 0, 0));
    Vec3 direction(detector - origin);
    direction.normalize();
    direction.normalise();
    Vec3 right(direction.crossProduct(up));
    float res1 = range[2] / width;
    float res2 = range[1] / height;
    float spacing = 2 * std::max(res1, res2);
    for (int k = 0; k < 3; ++k) {
        cam[k] = origin[k];
        cam[3 + k] = detector[k];
        cam[6 + k] = up[k];
        cam[9 + k] = right[k];
    }
    cam[12] = spacing;
}

// One pixel of renderLoop (src/main.cxx:652-742) through the reference
// classes; returns true for an odd hit count ("Only one intersect", :710).
static bool ref_pixel(const TriangleMesh& mesh, const float cam[13], uint32_t width, uint32_t height,
                      uint32_t row, uint32_t col, std::vector<float>& hits, float& photon, float& lval)
{
    const Vec3 origin(cam[0], cam[1], cam[2]);
    const Vec3 detector(cam[3], cam[4], cam[5]);
    const Vec3 up(cam[6], cam[7], cam[8]);
    const Vec3 right(cam[9], cam[10], cam[11]);
    const float spacing = cam[12];
    float v_off = spacing * (0.5 + row - height / 2.0);
    float u_off = spacing * (0.5 + col - width / 2.0);
    Vec3 dir = detector + up * v_off + right * u_off - origin;
    dir.normalise();
    Ray ray(origin, dir);

    hits.clear();
    for (unsigned int k = 0; k < mesh.getNumberOfTriangles(); ++k) {
        float t;
        if (ray.intersect(mesh.getTriangle(k), t) && t > 0.0000001) hits.push_back(t);
    }
    float path = 0;
    bool odd = false;
    lval = std::numeric_limits<float>::infinity();
    if (!hits.empty()) {
        if (hits.size() % 2 == 0) {
            std::sort(hits.begin(), hits.end());
            for (size_t i = 0; i < hits.size(); i += 2) path += hits[i + 1] - hits[i];
        } else {
            odd = true;
        }
        lval = path;
    }
    path = path * 0.1;
    photon = 80.000f * std::exp(-(0.3971f * path));
    return odd;
}

static TriangleMesh* make_mesh(const float* tris, uint64_t ntris)
{
    std::vector<float> v(tris, tris + 9 * ntris);
    std::vector<unsigned int> idx(3 * ntris);
    for (uint64_t i = 0; i < 3 * ntris; ++i) idx[i] = (unsigned int)i;
    return new TriangleMesh(v, idx);
}

// One image row range through the reference classes.  Outputs are
// strip-relative; odd-count rays are counted and returned.
int64_t ref_render_rows(const float* tris, uint64_t ntris, const float cam[13],
                        uint32_t width, uint32_t height, uint32_t row_begin,
                        uint32_t row_end, float* image, float* lbuffer)
{
    TriangleMesh* mesh = make_mesh(tris, ntris);
    int64_t odd = 0;
    std::vector<float> hits;
    for (uint32_t row = row_begin; row < row_end; ++row) {
        for (uint32_t col = 0; col < width; ++col) {
            float photon, lval;
            odd += ref_pixel(*mesh, cam, width, height, row, col, hits, photon, lval) ? 1 : 0;
            size_t o = (size_t)(row - row_begin) * width + col;
            if (image) image[o] = photon;
            if (lbuffer) lbuffer[o] = lval;
        }
    }
    delete mesh;
    return odd;
}

// A TriangleMesh built once and shared, read-only, by several threads
// (bench.py's "reference" CPU baseline renders spans of rows on every host
// thread over one mesh, as main-pthreads-redo.cxx's threads share theirs).
void* ref_mesh_create(const float* tris, uint64_t ntris) { return make_mesh(tris, ntris); }

void ref_mesh_destroy(void* mesh) { delete static_cast<TriangleMesh*>(mesh); }

// Pixels [col_begin, col_end) of one row over a shared mesh; outputs indexed
// from col_begin.  Returns the odd-count rays.
int64_t ref_render_span(const void* mesh, const float cam[13], uint32_t width, uint32_t height, uint32_t row,
                        uint32_t col_begin, uint32_t col_end, float* image, float* lbuffer)
{
    const TriangleMesh& m = *static_cast<const TriangleMesh*>(mesh);
    int64_t odd = 0;
    std::vector<float> hits;
    for (uint32_t col = col_begin; col < col_end; ++col) {
        float photon, lval;
        odd += ref_pixel(m, cam, width, height, row, col, hits, photon, lval) ? 1 : 0;
        if (image) image[col - col_begin] = photon;
        if (lbuffer) lbuffer[col - col_begin] = lval;
    }
    return odd;
}

// Triangle::getNormal of the reference's Triangle (include/Triangle.inl:170-178).
void ref_triangle_normals(const float* tris, uint64_t n, float* normals)
{
    for (uint64_t i = 0; i < n; ++i) {
        const float* p = tris + 9 * i;
        Triangle tri(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]), Vec3(p[6], p[7], p[8]));
        for (int k = 0; k < 3; ++k) normals[3 * i + k] = tri.getNormal()[k];
    }
}

// The signed L-buffer of src/main-pthreads-lbuffer.cxx:750-811 restated over
// the reference's classes (the fork itself needs glm and Assimp): a scene of
// meshes (soups one after another, mesh_ntris[m] triangles each), rows
// [row_begin, row_end); lbuffer = the fork's L_buffer values.  Returns the
// number of pixels flagged -1.
int64_t ref_render_signed_rows(const float* tris, const uint64_t* mesh_ntris, uint32_t nmeshes,
                               const float cam[13], uint32_t width, uint32_t height, uint32_t row_begin,
                               uint32_t row_end, float* lbuffer)
{
    std::vector<TriangleMesh> meshes(nmeshes);    // built in place (no TriangleMesh copies)
    uint64_t first = 0;
    for (uint32_t m = 0; m < nmeshes; ++m) {
        std::vector<float> v(tris + 9 * first, tris + 9 * (first + mesh_ntris[m]));
        std::vector<unsigned int> idx(3 * mesh_ntris[m]);
        for (uint64_t i = 0; i < idx.size(); ++i) idx[i] = (unsigned int)i;
        meshes[m].setGeometry(v, idx);
        first += mesh_ntris[m];
    }
    const Vec3 origin(cam[0], cam[1], cam[2]);
    const Vec3 detector(cam[3], cam[4], cam[5]);
    const Vec3 up(cam[6], cam[7], cam[8]);
    const Vec3 right(cam[9], cam[10], cam[11]);
    const float spacing = cam[12];
    int64_t flagged = 0;
    for (uint32_t row = row_begin; row < row_end; ++row) {
        for (uint32_t col = 0; col < width; ++col) {
            float v_off = spacing * (0.5 + row - height / 2.0);
            float u_off = spacing * (0.5 + col - width / 2.0);
            Vec3 direction = detector + up * v_off + right * u_off - origin;
            direction.normalise();
            Ray ray(origin, direction);
            float L = 80.000f;
            for (size_t m = 0; m < meshes.size(); ++m) {
                if (L == -1) break;
                float distance = 0.0f;
                int sign_sum = 0;
                for (unsigned int k = 0; k < meshes[m].getNumberOfTriangles(); ++k) {
                    const Triangle& triangle = meshes[m].getTriangle(k);
                    float t;
                    bool intersect = ray.intersect(triangle, t);
                    if (intersect && m == 0 && t > 0.0000001) {
                        float dp = direction.dotProduct(triangle.getNormal());
                        int sign = (0.0f < dp) - (dp < 0.0f);
                        distance += (sign * t);
                        sign_sum += sign;
                    }
                }
                float mu = m == 0 ? 0.1037f : 0.3971f;
                if (sign_sum != 0) L = -1;
                else L = L * std::exp(-(mu * (distance * 0.1)));
            }
            if (L == -1) ++flagged;
            lbuffer[(size_t)(row - row_begin) * width + col] = L;
        }
    }
    return flagged;
}

}  // extern "C"
