"""Host-side scene helpers (no GPU): the projection-sweep camera of
bench.py --orbit and the moving-camera parity test."""
import numpy as np

import simpleraytracing_amd as xrt
from simpleraytracing_amd.scenes import orbit_camera
from conftest import DRAGON


def _vec(cam, name):
    return np.array(getattr(cam, name)[:], np.float64)


def test_orbit_camera_turns_about_up_through_centre():
    tris = xrt.load_ply(DRAGON)
    cam = xrt.camera_for_mesh(tris, 256, 192)
    lo, hi = xrt.mesh_bbox(tris)
    centre = 0.5 * (np.asarray(lo, np.float64) + np.asarray(hi, np.float64))
    same = orbit_camera(cam, centre, 0.0)
    for name in ("origin", "detector", "up", "right"):
        assert np.array_equal(_vec(same, name), _vec(cam, name))
    assert (same.width, same.height, same.pixel_spacing) == (cam.width, cam.height, cam.pixel_spacing)
    k = _vec(cam, "up") / np.linalg.norm(_vec(cam, "up"))
    for deg in (1.0, 37.5, 90.0, 180.0):
        turned = orbit_camera(cam, centre, deg)
        assert np.array_equal(_vec(turned, "up"), _vec(cam, "up"))
        for name in ("origin", "detector"):
            a, b = _vec(cam, name) - centre, _vec(turned, name) - centre
            # distance to the centre and height along up are kept; the angle is deg
            assert np.isclose(np.linalg.norm(a), np.linalg.norm(b), rtol=1e-6)
            assert np.isclose(a @ k, b @ k, rtol=1e-6, atol=1e-3)
            pa, pb = a - (a @ k) * k, b - (b @ k) * k
            ang = np.degrees(np.arctan2(np.cross(pa, pb) @ k, pa @ pb)) % 360.0
            assert np.isclose(ang, deg, atol=1e-3)
        assert np.isclose(np.linalg.norm(_vec(turned, "right")), np.linalg.norm(_vec(cam, "right")), rtol=1e-6)
    full = orbit_camera(cam, centre, 360.0)
    for name in ("origin", "detector", "right"):
        assert np.allclose(_vec(full, name), _vec(cam, name), atol=1e-3)
