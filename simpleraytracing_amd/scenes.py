"""Synthetic scenes for the benchmark configurations (BASELINE.json configs).

``tiled_mesh`` builds the "1M-triangle synthetic mesh (tiled dragon)" of
SURVEY.md 8(d): n x n copies of a mesh translated in (y, z) -- the plane
facing the detector -- by (j * 1.05 * range_y, k * 1.05 * range_z) for
j, k in -(n//2) .. n//2, offsets added in float32, copies appended
copy-major (j outer, k inner).  For dragon.ply and n = 7 that is
22,866 * 49 = 1,120,434 triangles; tiling across the detector keeps the hit
count per ray at the single dragon's (<= 12), as tiling along the ray would not.
Deterministic: no randomness.

``orbit_camera`` turns a camera about its up axis through a centre: a
projection sweep (bench.py --orbit, the moving-camera parity test).
"""
from __future__ import annotations

import ctypes

import numpy as np


def tiled_mesh(tris: np.ndarray, n: int = 7) -> np.ndarray:
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    v = tris.reshape(-1, 3)
    lo = v.min(axis=0)
    hi = v.max(axis=0)
    rng = (hi - lo).astype(np.float32)
    dy = np.float32(1.05) * rng[1]
    dz = np.float32(1.05) * rng[2]
    half = n // 2
    out = []
    for j in range(-half, n - half):
        for k in range(-half, n - half):
            off = np.array([0.0, np.float32(j) * dy, np.float32(k) * dz], np.float32)
            out.append((tris.reshape(-1, 3, 3) + off[None, None, :]).astype(np.float32).reshape(-1, 9))
    return np.ascontiguousarray(np.concatenate(out), np.float32)


def orbit_camera(cam, centre, deg):
    """cam turned deg degrees about its up axis through centre (Rodrigues in
    f64, stored as float32): origin, detector and the right axis turn; up,
    spacing and size stay."""
    out = type(cam)()
    ctypes.pointer(out)[0] = cam
    up = np.array(cam.up[:], np.float64)
    k = up / np.linalg.norm(up)
    th = np.radians(deg)
    c, s = np.cos(th), np.sin(th)

    def rot(v):
        return v * c + np.cross(k, v) * s + k * np.dot(k, v) * (1.0 - c)

    for name, is_point in (("origin", True), ("detector", True), ("right", False)):
        v = np.array(getattr(cam, name)[:], np.float64)
        r = rot(v - centre) + centre if is_point else rot(v)
        getattr(out, name)[:] = [float(np.float32(x)) for x in r]
    return out
