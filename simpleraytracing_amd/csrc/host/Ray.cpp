// Ray.cpp -- Ray::intersect through the device (see Ray.h).
#include "Ray.h"

#include <cstdlib>
#include <stdexcept>
#include <string>

#include "xrt.h"
#include "xrt_host.h"

void intersectBatch(const std::vector<Ray>& rays, const std::vector<Triangle>& triangles,
                    std::vector<unsigned char>& hits, std::vector<float>& ts)
{
    if (rays.size() != triangles.size()) throw std::length_error("intersectBatch: size mismatch");
    const size_t n = rays.size();
    std::vector<float> r(6 * n), t(9 * n);
    for (size_t i = 0; i < n; ++i) {
        for (unsigned k = 0; k < 3; ++k) {
            r[6 * i + k] = rays[i].getOrigin()[k];
            r[6 * i + 3 + k] = rays[i].getDirection()[k];
            t[9 * i + k] = triangles[i].getP1()[k];
            t[9 * i + 3 + k] = triangles[i].getP2()[k];
            t[9 * i + 6 + k] = triangles[i].getP3()[k];
        }
    }
    hits.assign(n, 0);
    ts.assign(n, 0.0f);
    const char* d = std::getenv("XRT_DEVICE");
    xrt_context* ctx = xrt_host_device_context(d ? std::atoi(d) : 0);
    if (xrt_probe_intersect(ctx, r.data(), t.data(), n, hits.data(), ts.data()) != XRT_OK)
        throw std::runtime_error(std::string("Ray::intersect: ") + xrt_last_error(ctx));
}

bool Ray::intersect(const Triangle& triangle, float& t) const
{
    std::vector<unsigned char> hits;
    std::vector<float> ts;
    intersectBatch(std::vector<Ray>{*this}, std::vector<Triangle>{triangle}, hits, ts);
    if (hits[0]) t = ts[0];
    return hits[0] != 0;
}
