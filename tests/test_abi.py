"""CPU: the C-ABI libraries load, export every declared symbol, and their
host-side arithmetic (bbox, camera, PLY ingestion, expf restatement) is
bit-identical to the oracle.  No compute call touches a GPU here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import simpleraytracing_amd as xrt
from simpleraytracing_amd import _abi
from oracle import oracle
from conftest import DRAGON, ROOT, bits


def declared_functions(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = text.split("#ifdef __cplusplus\n}")[0]        # C part only
    return sorted(set(re.findall(r"\b(xrt_\w+)\s*\(", text)) - {"xrt_status"})


@pytest.mark.parametrize("header", ["xrt.h", "xrt_debug.h"])
def test_libxrt_exports_every_declared_symbol(header):
    """The drop-in surface (xrt.h) and the test/diagnostic hooks (xrt_debug.h)."""
    lib = _abi.load()
    names = declared_functions(header)
    assert len(names) >= (18 if header == "xrt.h" else 10)
    for n in names:
        assert hasattr(lib, n), n
        assert n in _abi.XRT_SYMBOLS, f"{n} declared in {header} but not bound in _abi.py"


def test_product_header_has_no_test_hooks():
    """Probes, test hooks and diagnostics live in xrt_debug.h, not in the drop-in header."""
    names = declared_functions("xrt.h")
    hooks = [n for n in names if n.startswith(("xrt_probe_", "xrt_debug_", "xrt_host_"))
             or n in ("xrt_set_hit_capacity", "xrt_set_bin_capacity", "xrt_set_fill_plan")]
    assert not hooks, hooks


def test_libxrt_host_exports_every_declared_symbol():
    host = _abi.load_host()
    for n in declared_functions("xrt_host.h"):
        assert hasattr(host, n), n


def test_abi_version():
    assert _abi.load().xrt_abi_version() == 5


def test_create_without_gpu_fails_cleanly():
    if xrt.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(xrt.XrtError) as e:
        xrt.Context(0)
    assert e.value.code == _abi.XRT_ERR_DEVICE


def test_load_ply_matches_oracle(dragon):
    soup = xrt.load_ply(DRAGON)
    assert soup.shape == dragon.shape
    assert np.array_equal(bits(soup), bits(dragon))


def test_load_ply_errors(tmp_path):
    with pytest.raises(xrt.XrtError) as e:
        xrt.load_ply(str(tmp_path / "missing.ply"))
    assert e.value.code == _abi.XRT_ERR_IO
    bad = tmp_path / "bad.ply"
    bad.write_bytes(b"ply\nformat binary_little_endian 1.0\nelement vertex 3\nproperty float x\nend_header\n")
    with pytest.raises(xrt.XrtError):
        xrt.load_ply(str(bad))


def test_ascii_ply_and_quads(tmp_path):
    p = tmp_path / "quad.ply"
    p.write_text("ply\nformat ascii 1.0\nelement vertex 4\nproperty float x\nproperty float y\n"
                 "property float z\nelement face 1\nproperty list uchar int vertex_indices\nend_header\n"
                 "0 0 0\n1 0 0\n1 1 0\n0 1 0\n4 0 1 2 3\n")
    soup = xrt.load_ply(str(p))
    ref = oracle.load_ply(str(p))
    assert soup.shape == (2, 9)
    assert np.array_equal(soup, ref)


def test_bbox_and_camera_match_oracle(dragon):
    lo, hi = xrt.mesh_bbox(dragon)
    lo2, hi2 = oracle.bbox(dragon)
    assert np.array_equal(bits(lo), bits(lo2)) and np.array_equal(bits(hi), bits(hi2))
    for (w, h) in [(128, 128), (2048, 2048), (4096, 4096), (8192, 8192), (640, 480), (3, 1000)]:
        cam = xrt.camera_from_bbox(lo, hi, w, h)
        c13 = oracle.camera(lo, hi, w, h)
        got = np.array(list(cam.origin) + list(cam.detector) + list(cam.up) + list(cam.right) +
                       [cam.pixel_spacing], np.float32)
        assert np.array_equal(bits(got), bits(c13)), (w, h)
        assert (cam.width, cam.height) == (w, h)


def test_dragon_2048_camera_values(dragon):
    # dragon 2048^2 camera
    cam = xrt.camera_for_mesh(dragon, 2048, 2048)
    assert np.float32(cam.pixel_spacing) == np.float32(0.151470721)
    assert np.allclose(list(cam.origin), [-220.841003, -671.790405, 298.21048])
    assert np.allclose(list(cam.detector), [115.792053, -671.790405, 298.21048])
    assert list(cam.right)[1] == 1.0


def test_host_expf_restatement_matches_libm():
    """The device expf source (host-compiled) vs glibc expf: all floats in
    [-0.5, 0] and a stride over [-104, 89] plus specials."""
    lib = _abi.load()
    ui = np.arange(0x80000000, 0xBF000001, 3, dtype=np.uint64).astype(np.uint32)   # -0 .. -0.5
    x = np.concatenate([
        ui.view(np.float32),
        np.arange(0xBF000000, 0xC2D00000, 97, dtype=np.uint64).astype(np.uint32).view(np.float32),
        np.arange(0x00000000, 0x42B20000, 997, dtype=np.uint64).astype(np.uint32).view(np.float32),
        np.array([np.inf, -np.inf, np.nan, 88.0, 88.8, -103.9, -104.0, -1e-45, 1e-45, 0.0, -0.0],
                 np.float32)])
    got = np.empty_like(x)
    lib.xrt_host_expf_batch(x.ctypes.data_as(_abi._fp), got.ctypes.data_as(_abi._fp), x.size)
    want = oracle.expf(x)
    same = (bits(got) == bits(want)) | (np.isnan(got) & np.isnan(want))
    assert same.all(), x[~same][:10]


def _mt_inputs(n, seed):
    """(det, a, b, tnum) near every decision boundary of Ray::intersect:
    u, v, u + v at 0 and 1 within a few ulps, t near 1e-7, det from denormal
    to huge, signs flipped, zeros, infinities and NaNs."""
    rng = np.random.default_rng(seed)
    f32 = np.float32
    det = (rng.choice([-1, 1], n) * 2.0 ** rng.uniform(-149, 127, n)).astype(f32)
    det[rng.random(n) < 0.02] = f32(0.0)
    det[rng.random(n) < 0.01] = f32(-0.0)
    u = rng.choice([0.0, 1.0, 0.5, 1e-7, -1e-7, 0.999999, 1.000001], n) + rng.normal(0, 1e-7, n)
    v = rng.choice([0.0, 0.5, 1e-7, -1e-7], n) + rng.normal(0, 1e-7, n)
    v = np.where(rng.random(n) < 0.5, 1.0 - u + rng.normal(0, 1e-7, n), v)
    t = rng.choice([1e-7, 1.0, -1.0, 0.0, 1e-30, 1e30], n) * (1 + rng.normal(0, 1e-6, n))
    a = (det.astype(np.float64) * u).astype(f32)
    b = (det.astype(np.float64) * v).astype(f32)
    tn = (det.astype(np.float64) * t).astype(f32)
    # a few ulps around each numerator
    for arr in (a, b, tn):
        arr.view(np.int32)[:] += rng.integers(-4, 5, n).astype(np.int32) * (arr != 0)
    specials = np.array([np.inf, -np.inf, np.nan, 0.0, -0.0, 1e-45, -1e-45, 3.4e38], f32)
    for arr in (det, a, b, tn):
        m = rng.random(n) < 0.003
        arr[m] = rng.choice(specials, int(m.sum()))
    return det, a, b, tn


def test_host_pre_reject_never_drops_a_hit():
    """The culled render's division-free reject (mt_may_hit, host-compiled from
    the device source) may only reject inputs that Ray::intersect rejects."""
    lib = _abi.load()
    u8p = ctypes.POINTER(ctypes.c_uint8)
    for seed in range(4):
        det, a, b, tn = _mt_inputs(1 << 20, seed)
        may = np.empty(det.size, np.uint8)
        hit = np.empty(det.size, np.uint8)
        t = np.empty(det.size, np.float32)
        lib.xrt_host_mt_check(det.ctypes.data_as(_abi._fp), a.ctypes.data_as(_abi._fp),
                              b.ctypes.data_as(_abi._fp), tn.ctypes.data_as(_abi._fp), det.size,
                              may.ctypes.data_as(u8p), hit.ctypes.data_as(u8p), t.ctypes.data_as(_abi._fp))
        bad = (hit == 1) & (may == 0)
        assert not bad.any(), list(zip(det[bad][:5], a[bad][:5], b[bad][:5], tn[bad][:5]))
        assert hit.sum() > 1000 and (may == 0).sum() > det.size // 4     # both sides exercised


def cli_exe():
    """xrt_main, or its sanitizer build under tools/san_check.sh ($XRT_MAIN)."""
    return os.environ.get("XRT_MAIN") or os.path.join(ROOT, "simpleraytracing_amd", "lib", "xrt_main")


def test_cli_help_and_bad_option():
    exe = cli_exe()
    r = subprocess.run([exe, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "--size" in r.stderr
    r = subprocess.run([exe, "--bogus"], capture_output=True, text=True)
    assert r.returncode == 1 and "Usage" in r.stderr


def test_cli_without_gpu_reports_error(tmp_path):
    if xrt.device_count() > 0:
        pytest.skip("a GPU is present")
    exe = cli_exe()
    r = subprocess.run([exe, "-s", "8", "8", "-i", DRAGON, "-f", "x.txt"], capture_output=True,
                       text=True, cwd=tmp_path)
    assert r.returncode == 1 and r.stderr.startswith("ERROR:")


def test_fp_identities_exhaustive(tmp_path):
    """The f32 identities the device code uses (inv_det_of, accept_t, lut_u8),
    checked on every f32 input by tools/check_fp_identities.c."""
    src = os.path.join(ROOT, "tools", "check_fp_identities.c")
    exe = str(tmp_path / "cfi")
    subprocess.run(["gcc", "-O2", "-o", exe, src, "-lm"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr


def test_host_ray_intersect_kat_matches_oracle():
    """The drop-in Ray::intersect (host C++, src/Ray.cxx:72-124 over host/Vec3.h)
    on the KAT pairs: bit-equal to the oracle (itself pinned to the reference's
    compiled Ray.cxx in test_oracle.py)."""
    from kat import kat_vectors
    rays, tris = kat_vectors()
    host = _abi.load_host()
    n = len(rays)
    hit = np.zeros(n, np.uint8)
    t = np.zeros(n, np.float32)
    host.xrt_host_intersect_batch(rays.ctypes.data_as(_abi._fp), tris.ctypes.data_as(_abi._fp), n,
                                  hit.ctypes.data_as(_abi._u8p), t.ctypes.data_as(_abi._fp))
    h2, t2 = oracle.intersect_batch(rays, tris)
    assert np.array_equal(hit, h2)
    assert np.array_equal(bits(t), bits(t2))


# --------------------------------------------------------------------------- the L-buffer fork, scenes
def test_host_exp_restatement_matches_libm():
    """The device glibc exp source (host-compiled) vs libm exp: the exponents
    the signed model forms from a stride over every f32 distance, random
    doubles over the whole range, specials.  (tools/check_exp.cpp covers all
    2^32 distances: 0 mismatches.)"""
    lib = _abi.load()
    d = np.arange(0, 1 << 32, 4099, dtype=np.uint64).astype(np.uint32).view(np.float32)
    with np.errstate(invalid="ignore"):
        x1 = -(np.float64(np.float32(0.1037)) * (d.astype(np.float64) * 0.1))
    rng = np.random.default_rng(1)
    x2 = rng.uniform(-746, 710, 200000)
    x3 = np.array([0.0, -0.0, 1e-300, -1e-300, 5e-324, 709.78, 709.79, -708.4, -745.13, -745.2, 1024, -1024,
                   np.inf, -np.inf, np.nan, 512.0, -512.0], np.float64)
    x = np.ascontiguousarray(np.concatenate([x1, x2, x3]))
    got = np.empty_like(x)
    lib.xrt_host_exp_batch(x.ctypes.data_as(_abi._dp), got.ctypes.data_as(_abi._dp), x.size)
    want = oracle.exp(x)
    same = (got.view(np.uint64) == want.view(np.uint64)) | (np.isnan(got) & np.isnan(want))
    assert same.all(), x[~same][:8]


def test_host_signed_lbuffer_update():
    """(float)(80 * exp(-(mu * (d * 0.1)))) as the fork evaluates it, -1 for a
    non-zero sign sum, and x86's NaN for a NaN distance (0x7FC00000)."""
    lib = _abi.load()
    rng = np.random.default_rng(2)
    d = np.concatenate([rng.uniform(-50, 400, 100000), [0.0, -0.0, np.inf, -np.inf, 1e30, -1e30]]).astype(np.float32)
    d = np.concatenate([d, np.array([0xFFC00000], np.uint32).view(np.float32)])
    ss = np.zeros(d.size, np.int32)
    ss[::97] = rng.choice([-2, -1, 1, 3], ss[::97].size)
    mu = np.float32(0.1037)
    got = np.empty_like(d)
    lib.xrt_host_signed_lbuffer_batch(d.ctypes.data_as(_abi._fp), ss.ctypes.data_as(_abi._i32p), mu,
                                      got.ctypes.data_as(_abi._fp), d.size)
    with np.errstate(over="ignore", invalid="ignore"):
        want = (np.float64(80.0) * oracle.exp(-(np.float64(mu) * (d.astype(np.float64) * 0.1)))).astype(np.float32)
    want[np.isnan(d)] = np.array([0x7FC00000], np.uint32).view(np.float32)[0]
    want[ss != 0] = -1
    assert np.array_equal(bits(got), bits(want))


def test_obj_scene_loading(tmp_path):
    p = tmp_path / "scene.obj"
    p.write_text("# two objects\nmtllib x.mtl\nv 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvt 0 0\nvn 0 0 1\n"
                 "o first\nusemtl a\nf 1/1/1 2/1/1 3/1/1 4/1/1\n"
                 "o empty\n"
                 "g second\nv 5 5 5\nv 6 5 5\nv 5 6 7\nf -3 -2 -1\nf 1//1 3//1 5//1\nl 1 2\n")
    meshes = xrt.load_meshes(str(p))
    assert [len(m) for m in meshes] == [2, 2]
    assert np.array_equal(meshes[0], np.array([[0, 0, 0, 1, 0, 0, 1, 1, 0], [0, 0, 0, 1, 1, 0, 0, 1, 0]], np.float32))
    assert np.array_equal(meshes[1][0], np.array([5, 5, 5, 6, 5, 5, 5, 6, 7], np.float32))
    assert np.array_equal(meshes[1][1], np.array([0, 0, 0, 1, 1, 0, 5, 5, 5], np.float32))
    lo, hi = xrt.scene_bbox(meshes)
    lo2, hi2 = oracle.scene_bbox(meshes)
    assert np.array_equal(lo, lo2) and np.array_equal(hi, hi2)
    assert list(lo) == [0, 0, 0] and list(hi) == [6, 6, 7]
    ply = xrt.load_meshes(DRAGON)
    assert len(ply) == 1 and ply[0].shape == (22866, 9)
    bad = tmp_path / "bad.obj"
    bad.write_text("v 0 0 0\nf 1 2 3\n")
    with pytest.raises(xrt.XrtError):
        xrt.load_meshes(str(bad))


def test_scene_camera_differs_from_mesh0_camera(dragon):
    from scene_kit import second_mesh_for
    meshes = [dragon, second_mesh_for(dragon)]
    cam = xrt.camera_for_scene(meshes, 256, 256)
    c13 = oracle.camera_for_scene(meshes, 256, 256)
    got = np.array(list(cam.origin) + list(cam.detector) + list(cam.up) + list(cam.right) + [cam.pixel_spacing],
                   np.float32)
    assert np.array_equal(bits(got), bits(c13))
    assert not np.array_equal(c13, oracle.camera_for_mesh(dragon, 256, 256))


@pytest.mark.parametrize("W,H", [(128, 128), (131, 77), (1, 1), (17, 300)])
def test_jpeg_writer(tmp_path, W, H):
    """Image::saveJPEGFile (src/Image.cxx:85-144) through xrt_host_save_image:
    a baseline JPEG (SOF0, 3 components, 4:2:0, quality 100) of the LUT over
    [0, 80] that PIL decodes to the u8 plane within JPEG quality-100 error
    (every channel within 2 levels of it, mean error below 0.5).  Byte parity
    with libjpeg is unpinned (no libjpeg here).  The 128x128 image is the
    reference's golden render (out/dragon-128x128-serial.txt)."""
    PIL = pytest.importorskip("PIL.Image")
    if (W, H) == (128, 128):
        text = open(os.path.join(ROOT, "tests", "golden", "dragon-128x128-serial.txt")).read()
        img = np.array([[float(v) for v in row.split("\t")] for row in text.split("\n")], np.float32)
    else:
        yy, xx = np.mgrid[0:H, 0:W]
        img = (40.0 + 39.0 * np.sin(xx / 5.0) * np.cos(yy / 7.0)).astype(np.float32)
        img[::13, ::11] = 80.0                             # isolated bright pixels: sharp edges
    flat = np.ascontiguousarray(img.reshape(-1))
    lut = np.array([oracle.lut_u8(v) for v in flat], np.uint8).reshape(H, W)
    path = tmp_path / "i.jpg"
    host = _abi.load_host()
    rc = host.xrt_host_save_image(flat.ctypes.data_as(_abi._fp), W, H, str(path).encode(), _abi.XRT_IMAGE_JPEG,
                                  0.0, 80.0)
    assert rc == _abi.XRT_OK
    data = path.read_bytes()
    assert data[:2] == b"\xff\xd8" and data[-2:] == b"\xff\xd9" and b"JFIF\x00" in data[:20]
    with PIL.open(path) as im:
        assert im.format == "JPEG" and im.mode == "RGB" and im.size == (W, H)
        px = np.asarray(im, dtype=np.int16)
    err = np.abs(px - lut[:, :, None].astype(np.int16))
    assert err.max() <= 2 and err.mean() < 0.5, (err.max(), err.mean())


def test_image_writers(tmp_path):
    """Image::saveTextFile / saveTGAFile / savePGMFile through xrt_host_save_image:
    the text as the oracle writes it (src/Image.cxx:210-235), the TGA's 18-byte
    header and bottom-up rows (src/Image.cxx:148-206) and the PGM carrying the
    LUT over [0, 80] (applyLUT's intended mapping, include/Image.inl:189-216);
    the JPEG writer is test_jpeg_writer's."""
    H, W = 5, 7
    rng = np.random.default_rng(3)
    img = rng.uniform(-10, 90, (H, W)).astype(np.float32)
    img[0, 0], img[1, 2], img[4, 6] = np.nan, 0.0, 80.0
    flat = np.ascontiguousarray(img.reshape(-1))
    host = _abi.load_host()
    lut = np.array([oracle.lut_u8(v) for v in flat], np.uint8).reshape(H, W)

    def save(name, fmt):
        path = tmp_path / name
        rc = host.xrt_host_save_image(flat.ctypes.data_as(_abi._fp), W, H, str(path).encode(), fmt, 0.0, 80.0)
        return rc, path

    rc, path = save("i.txt", _abi.XRT_IMAGE_TEXT)
    assert rc == _abi.XRT_OK and path.read_bytes() == oracle.text_bytes(flat, W, H)
    rc, path = save("i.tga", _abi.XRT_IMAGE_TGA)
    data = path.read_bytes()
    assert rc == _abi.XRT_OK and len(data) == 18 + 3 * W * H
    assert data[:18] == bytes([0, 0, 2] + [0] * 9 + [W & 255, W >> 8, H & 255, H >> 8, 24, 0])
    px = np.frombuffer(data[18:], np.uint8).reshape(H, W, 3)
    assert np.array_equal(px, np.repeat(lut[::-1, :, None], 3, axis=2))
    rc, path = save("i.pgm", _abi.XRT_IMAGE_PGM)
    data = path.read_bytes()
    head = f"P5\n{W} {H}\n255\n".encode()
    assert rc == _abi.XRT_OK and data[:len(head)] == head
    assert np.array_equal(np.frombuffer(data[len(head):], np.uint8).reshape(H, W), lut)
    assert save("no/such/dir.tga", _abi.XRT_IMAGE_TGA)[0] == _abi.XRT_ERR_IO
    assert save("x", 9)[0] == _abi.XRT_ERR_ARGUMENT


def test_direction_grid_bisection_equals_scan():
    """The cull's direction grid per camera: the
    library's bisection along an axis (x is monotone in the pixel index) equals
    the scan of every row or column it replaced, on orbit cameras of the dragon
    and on random cameras with axis-aligned up / right vectors (the scanned
    branches), 1..8192 pixels a side (host code: no device)."""
    import numpy as np
    import simpleraytracing_amd as xrt
    from simpleraytracing_amd.scenes import orbit_camera
    lib = _abi.load()
    grids = (ctypes.c_int * 2)()
    tris = xrt.load_ply(DRAGON)
    lo, hi = xrt.mesh_bbox(tris)
    centre = 0.5 * (np.asarray(lo, np.float64) + np.asarray(hi, np.float64))
    cams = []
    for size in (7, 1024, 2048, 8192):
        base = xrt.camera_for_mesh(tris, size, size)
        cams += [orbit_camera(base, centre, d) for d in (0.0, 0.25, 1.0, 37.0, 90.0, 180.0)]
    rng = np.random.default_rng(20250302)
    for _ in range(300):
        c = xrt.Camera()
        c.width, c.height = (int(v) for v in rng.integers(1, 8193, 2))
        for name in ("origin", "detector", "up", "right"):
            v = rng.normal(0.0, float(rng.choice([1e-3, 1.0, 100.0])), 3).astype(np.float32)
            if name in ("up", "right"):
                v[rng.integers(0, 3)] = 0.0                  # the scanned branches
                if rng.random() < 0.3:
                    v[rng.integers(0, 3)] = 0.0
            getattr(c, name)[:] = [float(x) for x in v]
        c.pixel_spacing = float(np.float32(rng.choice([1e-4, 0.01, 0.3, -0.05])))
        cams.append(c)
    for c in cams:
        assert lib.xrt_debug_direction_grid(ctypes.byref(c), grids) == 0
        assert grids[0] == grids[1], (list(c.origin), list(c.detector), list(c.up), list(c.right),
                                      c.pixel_spacing, c.width, c.height, grids[0], grids[1])
