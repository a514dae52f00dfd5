"""Known-answer (ray, triangle) pairs for Ray::intersect (src/Ray.cxx:72-124).

Seeded random pairs plus crafted edge cases:
rays through vertices and edges, u + v = 1, det = +-0, t near 1e-7, tiny and
denormal determinants, degenerate triangles, a zero direction, huge
coordinates.  Shared by the CPU oracle tests (against the reference's own
compiled Ray.cxx) and the GPU probe test (against the oracle); kept apart from
test_oracle.py so the GPU tests do not map the reference build.
"""
import numpy as np


def kat_vectors(seed=20250302, n=65536):
    rng = np.random.default_rng(seed)
    rays = np.zeros((n, 6), np.float32)
    tris = np.zeros((n, 9), np.float32)
    # random triangles near the origin of a random ray aimed at them
    tris[:] = rng.normal(0, 1, (n, 9)).astype(np.float32)
    rays[:, :3] = rng.normal(0, 5, (n, 3)).astype(np.float32)
    centre = tris.reshape(n, 3, 3).mean(axis=1)
    jitter = rng.normal(0, 0.7, (n, 3)).astype(np.float32)
    rays[:, 3:] = (centre + jitter - rays[:, :3]).astype(np.float32)
    k = 0
    # crafted: axis-aligned unit triangle, rays through vertices / edges / u+v = 1
    base = np.array([0, 0, 0, 1, 0, 0, 0, 1, 0], np.float32)
    for (u, v) in [(0, 0), (1, 0), (0, 1), (0.5, 0.5), (0.25, 0.75), (0, 0.5), (0.5, 0),
                   (1e-8, 1e-8), (-1e-8, 0.5), (0.5, -1e-8), (0.5000001, 0.5), (0.3, 0.7000001)]:
        tris[k] = base
        rays[k] = [u, v, 5, 0, 0, -1]
        k += 1
    # ray in the triangle's plane (det = +-0)
    tris[k] = base; rays[k] = [-1, 0.25, 0, 1, 0, 0]; k += 1
    tris[k] = base; rays[k] = [0.2, 0.2, 0, 0, 0, 1]; k += 1   # origin on the triangle (t = 0)
    tris[k] = base; rays[k] = [0.2, 0.2, 1e-7, 0, 0, -1]; k += 1  # t ~ 1e-7
    tris[k] = base; rays[k] = [0.2, 0.2, 1.1e-7, 0, 0, -1]; k += 1
    tris[k] = base; rays[k] = [0.2, 0.2, -5, 0, 0, -1]; k += 1   # behind the origin
    # tiny / denormal determinants
    tiny = np.array([0, 0, 0, 1e-20, 0, 0, 0, 1e-20, 0], np.float32)
    tris[k] = tiny; rays[k] = [1e-21, 1e-21, 1, 0, 0, -1]; k += 1
    tris[k] = tiny * np.float32(1e-5); rays[k] = [1e-27, 1e-27, 1, 0, 0, -1]; k += 1
    # degenerate triangles
    tris[k] = [0, 0, 0, 1, 1, 1, 2, 2, 2]; rays[k] = [0.5, 0.5, 5, 0, 0, -1]; k += 1
    tris[k] = [1, 1, 1, 1, 1, 1, 1, 1, 1]; rays[k] = [1, 1, 5, 0, 0, -1]; k += 1
    # zero direction
    tris[k] = base; rays[k] = [0.2, 0.2, 1, 0, 0, 0]; k += 1
    # huge coordinates
    tris[k] = base * np.float32(1e18); rays[k] = [1e17, 1e17, 1e19, 0, 0, -1]; k += 1
    return rays, tris
