"""CPU: the oracle is pinned against the reference's own golden output and the
reference's own compiled Ray::intersect (oracle/_ref)."""
import os

import numpy as np
import pytest

from oracle import oracle
from conftest import DRAGON, GOLDEN, bits

REF = oracle.ref_lib()
needs_ref = pytest.mark.skipif(REF is None, reason="oracle/_ref not built (needs /root/reference)")


def test_dragon_facts(dragon):
    # 11,429 vertices, 22,866 triangles, 1 mesh
    assert dragon.shape == (22866, 9)
    lo, hi = oracle.bbox(dragon)
    assert np.all(lo < hi)


def test_golden_128_text_byte_exact(dragon):
    """out/dragon-128x128-serial.txt (the reference's own golden) reproduced byte for byte."""
    cam = oracle.camera_for_mesh(dragon, 128, 128)
    img, lb, u8, nh, odd = oracle.render_rows(dragon, cam, 128, 128)
    got = oracle.text_bytes(img, 128, 128)
    want = open(os.path.join(GOLDEN, "dragon-128x128-serial.txt"), "rb").read()
    assert got == want
    # hit-count histogram at 128^2 (misses are exactly 80)
    assert np.count_nonzero(nh == 0) == 11050
    assert np.all(img[nh == 0] == np.float32(80.0))
    assert np.all(np.isinf(lb[nh == 0]))
    assert odd == 0


@needs_ref
def test_camera_matches_reference_classes(dragon):
    lo, hi = oracle.bbox(dragon)
    lo2 = np.zeros(3, np.float32)
    hi2 = np.zeros(3, np.float32)
    REF.ref_mesh_bbox(oracle._fp(np.ascontiguousarray(dragon)), len(dragon), oracle._fp(lo2), oracle._fp(hi2))
    assert np.array_equal(bits(lo), bits(lo2)) and np.array_equal(bits(hi), bits(hi2))
    for (w, h) in [(128, 128), (2048, 2048), (4096, 4096), (640, 480), (1, 1)]:
        c1 = oracle.camera(lo, hi, w, h)
        c2 = np.zeros(13, np.float32)
        REF.ref_camera(oracle._fp(lo), oracle._fp(hi), w, h, oracle._fp(c2))
        assert np.array_equal(bits(c1), bits(c2)), (w, h)


def kat_vectors(seed=20250302, n=65536):
    """Seeded random + crafted (ray, triangle) pairs."""
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


@needs_ref
def test_intersect_kat_vs_reference():
    rays, tris = kat_vectors()
    h1, t1 = oracle.intersect_batch(rays, tris)
    h2, t2 = oracle.ref_intersect_batch(rays, tris)
    assert np.array_equal(h1, h2)
    assert np.array_equal(bits(t1), bits(t2))
    assert 0.05 < h1.mean() < 0.95


@needs_ref
def test_render_rows_vs_reference_classes(dragon):
    """Oracle renderLoop vs the same loop over the reference's compiled classes."""
    W = H = 48
    cam = oracle.camera_for_mesh(dragon, W, H)
    img, lb, u8, nh, odd = oracle.render_rows(dragon, cam, W, H, 10, 30)
    R = REF
    img2 = np.zeros_like(img)
    lb2 = np.zeros_like(lb)
    odd2 = R.ref_render_rows(oracle._fp(np.ascontiguousarray(dragon)), len(dragon), oracle._fp(cam), W, H, 10, 30,
                             oracle._fp(img2), oracle._fp(lb2))
    assert odd == odd2
    assert np.array_equal(bits(img), bits(img2))
    assert np.array_equal(bits(lb), bits(lb2))


def test_lut_formula():
    assert oracle.lut_u8(80.0) == 255
    assert oracle.lut_u8(0.0) == 0
    assert oracle.lut_u8(-1.0) == 0
    assert oracle.lut_u8(81.0) == 255
    assert oracle.lut_u8(40.0) == 128          # 127.5 rounds half away from zero
    assert oracle.lut_u8(float("nan")) == 0


def test_row_list_matches_rows(dragon):
    W = H = 64
    cam = oracle.camera_for_mesh(dragon, W, H)
    full = oracle.render_rows(dragon, cam, W, H)
    rows = [0, 7, 31, 32, 63]
    part = oracle.render_row_list(dragon, cam, W, H, rows)
    for i, r in enumerate(rows):
        assert np.array_equal(bits(part[0][i * W:(i + 1) * W]), bits(full[0][r * W:(r + 1) * W]))
