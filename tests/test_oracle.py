"""CPU: the oracle is pinned against the reference's own golden output and the
reference's own compiled Ray::intersect (oracle/_ref)."""
import os

import numpy as np
import pytest

from oracle import oracle
from conftest import DRAGON, GOLDEN, bits
from kat import kat_vectors
from scene_kit import corner_soup, second_mesh_for, striped_sheets, synthetic_soup


@pytest.fixture(scope="module")
def REF():
    """The reference's own compiled classes (oracle/_ref), mapped only by the
    CPU tests that use them; skipped where it has not been built."""
    r = oracle.ref_lib()
    if r is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    return r


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


def test_camera_matches_reference_classes(REF, dragon):
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


def test_intersect_kat_vs_reference(REF):
    rays, tris = kat_vectors()
    h1, t1 = oracle.intersect_batch(rays, tris)
    h2, t2 = oracle.ref_intersect_batch(rays, tris)
    assert np.array_equal(h1, h2)
    assert np.array_equal(bits(t1), bits(t2))
    assert 0.05 < h1.mean() < 0.95


def test_render_rows_vs_reference_classes(REF, dragon):
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


def test_reference_spans_threaded_vs_oracle(REF, dragon):
    """bench.py's "reference" CPU baseline: spans of rows over one shared mesh
    of the reference's classes on several threads equal the oracle's rows."""
    W, H = 64, 56
    cam = oracle.camera_for_mesh(dragon, W, H)
    rows = [0, 7, 21, 28, 40, 55]
    img, lb, u8, nh, odd = oracle.render_row_list(dragon, cam, W, H, np.array(rows, np.uint32))
    r_img, r_lb, r_odd = oracle.ref_render_spans(dragon, cam, W, H, rows, 0, W, threads=4)
    assert np.array_equal(bits(r_img.ravel()), bits(img)) and np.array_equal(bits(r_lb.ravel()), bits(lb))
    assert r_odd == odd
    assert np.array_equal(oracle.lut_u8_array(r_img.ravel()), u8)
    s_img, s_lb, _ = oracle.ref_render_spans(dragon, cam, W, H, rows, 17, 45, threads=3)
    assert np.array_equal(bits(s_img), bits(r_img[:, 17:45])) and np.array_equal(bits(s_lb), bits(r_lb[:, 17:45]))


def test_lut_array_equals_scalar_formula():
    rng = np.random.default_rng(5)
    v = np.concatenate([rng.uniform(-3.0, 90.0, 20000).astype(np.float32),
                        np.array([np.nan, np.inf, -np.inf, 0.0, -0.0, 80.0, 0.15686275, 40.0], np.float32)])
    assert np.array_equal(oracle.lut_u8_array(v), np.array([oracle.lut_u8(x) for x in v], np.uint8))


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


# --------------------------------------------------------------------------- the L-buffer fork
def test_triangle_normals_vs_reference_classes(REF, dragon):
    soup = np.concatenate([dragon, synthetic_soup(n=600)])
    got = oracle.triangle_normals(soup)
    want = oracle.ref_triangle_normals(soup)
    same = (bits(got) == bits(want)) | (np.isnan(got) & np.isnan(want))
    assert same.all()


def _signed_scenes(dragon):
    sheets = striped_sheets()
    return {
        "dragon+box": ([dragon, second_mesh_for(dragon)], 40, 36),
        "sheets": ([sheets], 48, 40),
        "corner": ([corner_soup()], 33, 31),
        "soup+dragon": ([synthetic_soup(seed=7, n=400), dragon[:2000]], 30, 26),
    }


@pytest.mark.parametrize("name", ["dragon+box", "sheets", "corner", "soup+dragon"])
def test_signed_lbuffer_vs_reference_classes(REF, dragon, name):
    """The signed L-buffer (main-pthreads-lbuffer.cxx:750-811) restated in C
    equals its restatement over the reference's own compiled classes, bit for
    bit (the fork itself needs glm and Assimp: parity of the fork's own build
    is unpinned)."""
    meshes, W, H = _signed_scenes(dragon)[name]
    cam = oracle.camera_for_scene(meshes, W, H)
    lb, nh, flagged = oracle.render_signed_rows(meshes, cam, W, H)
    lbr, flr = oracle.ref_render_signed_rows(meshes, cam, W, H)
    assert np.array_equal(bits(lb), bits(lbr))
    assert flagged == flr
    if name == "sheets":
        assert flagged > 50


def _hole_fill_py(L, W, H):
    """main-pthreads-lbuffer.cxx:327-404 in Python, unsigned 32-bit index arithmetic."""
    size = W * H
    out = L.copy()
    for pixel in range(size):
        row, col = divmod(pixel, W)
        if L[row * W + col] != -1:
            continue
        vals = []
        for d in range(4):
            value = np.float32(0)
            for i in range(1, 5):
                idx = [row * W + col + i, (row - i) * W + col, row * W + col - i, (row + i) * W + col][d]
                idx &= 0xFFFFFFFF
                if idx >= size:
                    break
                if L[idx] != -1:
                    value = L[idx]
                    break
            if value != 0:
                vals.append(value)
        s = np.float32(0)
        for v in vals:
            s = np.float32(s + v)
        with np.errstate(invalid="ignore", divide="ignore"):
            out[pixel] = np.float32(s) / np.float32(len(vals))
    return out


@pytest.mark.parametrize("W,H,seed", [(1, 1, 0), (7, 5, 1), (9, 9, 2), (16, 3, 3), (3, 16, 4)])
def test_hole_fill_vs_python_restatement(W, H, seed):
    rng = np.random.default_rng(seed)
    L = rng.uniform(1, 80, W * H).astype(np.float32)
    L[rng.random(W * H) < 0.45] = -1
    L[rng.random(W * H) < 0.05] = 0
    L[rng.random(W * H) < 0.03] = np.inf
    L[rng.random(W * H) < 0.03] = np.float32(np.nan)
    got = oracle.hole_fill(L, W, H)
    want = _hole_fill_py(L, W, H)
    assert np.array_equal(np.isnan(got), np.isnan(want))
    ok = ~np.isnan(want)
    assert np.array_equal(bits(got[ok]), bits(want[ok]))
    assert np.all(got != -1)


def test_scene_bbox_is_getbbox_of_mesh_boxes(REF, dragon):
    meshes = [dragon, second_mesh_for(dragon), synthetic_soup(n=50)]
    lo, hi = oracle.scene_bbox(meshes)
    los, his = [], []
    for m in meshes:
        l = np.zeros(3, np.float32)
        h = np.zeros(3, np.float32)
        REF.ref_mesh_bbox(oracle._fp(np.ascontiguousarray(m)), len(m), oracle._fp(l), oracle._fp(h))
        los.append(l)
        his.append(h)
    assert np.array_equal(lo, np.min(los, axis=0)) and np.array_equal(hi, np.max(his, axis=0))
    assert not np.array_equal(oracle.camera_for_scene(meshes, 64, 64), oracle.camera_for_mesh(dragon, 64, 64))


# --- fixtures generated from the reference's own classes (tools/gen_golden.py) ---

def _golden(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)


def test_fixture_kat_intersect():
    """tests/golden/kat_intersect.npz: the 64 K pairs of tests/kat.py through the
    reference's own Ray::intersect (generated here from oracle/_ref); the
    oracle reproduces every hit flag and distance bit for bit."""
    import hashlib
    g = _golden("kat_intersect")
    rays, tris = kat_vectors()
    assert hashlib.sha256(rays.tobytes() + tris.tobytes()).hexdigest() == str(g["inputs_sha256"])
    hit, t = oracle.intersect_batch(rays, tris)
    assert np.array_equal(hit, g["hit"]) and np.array_equal(bits(t), bits(g["t"]))


@pytest.mark.parametrize("name", ["planes_dragon_128", "planes_dragon_256", "rows_dragon_1024"])
def test_fixture_rows_oracle(dragon, name):
    """The oracle against the committed frames / strip-boundary rows rendered by
    the reference's own classes (tests/golden/<name>.npz): camera, image,
    L-buffer bit for bit (u8, hit counts and odd rays were the oracle's at
    generation and are pinned by the same run)."""
    g = _golden(name)
    W, H = int(g["width"]), int(g["height"])
    cam = oracle.camera_for_mesh(dragon, W, H)
    assert np.array_equal(bits(cam), bits(g["camera"]))
    img, lb, u8, nh, odd = oracle.render_row_list(dragon, cam, W, H, g["rows"])
    assert np.array_equal(bits(img), bits(g["image"].reshape(-1)))
    assert np.array_equal(bits(lb), bits(g["lbuffer"].reshape(-1)))
    assert np.array_equal(u8, g["u8"].reshape(-1)) and np.array_equal(nh, g["nhits"].reshape(-1))
    assert odd == int(g["odd"])
