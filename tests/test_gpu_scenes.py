"""GPU parity for multi-mesh scenes (main.cxx:427-510, :538-563, :687) and the
L-buffer fork's signed multi-material model (main-pthreads-lbuffer.cxx:733-813,
hole fill :327-404): the HIP path through the C ABI vs the CPU oracle, bit for
bit.  The signed model's oracle is pinned against a restatement over the
reference's own classes (tests/test_oracle.py); the fork itself does not build
here (glm, Assimp), so its parity is "unpinned" by a fork-built fixture."""
import os
import subprocess

import numpy as np
import pytest

import simpleraytracing_amd as xrt
from simpleraytracing_amd import _abi
from oracle import oracle
from conftest import DRAGON, ROOT, bits
from scene_kit import box, corner_soup, plane_stack, second_mesh_for, striped_sheets, synthetic_soup

pytestmark = pytest.mark.gpu
KERNELS = [xrt.XRT_KERNEL_BRUTE, xrt.XRT_KERNEL_TILED, xrt.XRT_KERNEL_BINNED]
SIGNED_KERNELS = [xrt.XRT_KERNEL_BRUTE, xrt.XRT_KERNEL_BINNED]
EXE = os.path.join(ROOT, "simpleraytracing_amd", "lib", "xrt_main")


def cam13(cam):
    return np.array(list(cam.origin) + list(cam.detector) + list(cam.up) + list(cam.right) +
                    [cam.pixel_spacing], np.float32)


def lut(img):
    return np.array([oracle.lut_u8(v) for v in img], np.uint8)


@pytest.fixture
def signed(ctx):
    """ctx in the signed model (mesh-0 mu 0.1037f, fork :800), restored afterwards."""
    ctx.set_model(xrt.XRT_MODEL_SIGNED, 0.1037)
    try:
        yield ctx
    finally:
        ctx.set_model(xrt.XRT_MODEL_ATTENUATION, 0.0)
        ctx.set_hit_capacity(0)
        ctx.set_kernel(xrt.XRT_KERNEL_AUTO)


# --------------------------------------------------------------------------- multi-mesh scenes
@pytest.mark.parametrize("kernel", KERNELS)
def test_two_mesh_scene(ctx, dragon, kernel):
    """Camera from the box of both meshes, hits from mesh 0 only."""
    meshes = [dragon, second_mesh_for(dragon)]
    W, H = 160, 128
    cam = xrt.camera_for_scene(meshes, W, H)
    assert not np.array_equal(cam13(cam), cam13(xrt.camera_for_mesh(dragon, W, H)))   # mesh 1 moves the camera
    ctx.set_kernel(kernel)
    ctx.upload_mesh(meshes[0])
    img, lb, u8, st = ctx.render_rows(cam)
    rimg, rlb, ru8, rnh, rodd = oracle.render_scene_rows(meshes, cam13(cam), W, H)
    assert np.array_equal(bits(img), bits(rimg)) and np.array_equal(bits(lb), bits(rlb))
    assert np.array_equal(u8, ru8) and st.odd_rays == rodd and st.hits == int(rnh.sum())
    # mesh 1 is in view: counting its hits would change the image
    merged = oracle.render_rows(np.concatenate(meshes), cam13(cam), W, H)
    assert not np.array_equal(bits(merged[0]), bits(rimg))


def _write_obj(path, soup):
    with open(path, "w") as f:
        for t in soup:
            for k in range(3):
                f.write("v %r %r %r\n" % tuple(float(x) for x in t[3 * k:3 * k + 3]))
        for i in range(len(soup)):
            f.write(f"f {3 * i + 1} {3 * i + 2} {3 * i + 3}\n")


def test_cli_scene_of_two_files(tmp_path, dragon):
    """xrt_main -i dragon.ply -i box.obj: the text image of the two-mesh scene."""
    second = second_mesh_for(dragon)
    _write_obj(tmp_path / "box.obj", second)
    (tmp_path / "out").mkdir()
    r = subprocess.run([EXE, "-s", "96", "80", "-i", DRAGON, "-i", str(tmp_path / "box.obj"), "-f", "s.txt"],
                       capture_output=True, text=True, cwd=tmp_path, timeout=300)
    assert r.returncode == 0, r.stderr
    meshes = [dragon, xrt.load_meshes(str(tmp_path / "box.obj"))[0]]
    assert np.array_equal(meshes[1], second)
    ref = oracle.render_scene_rows(meshes, oracle.camera_for_scene(meshes, 96, 80), 96, 80)
    assert (tmp_path / "out" / "s.txt").read_bytes() == oracle.text_bytes(ref[0], 96, 80)


# --------------------------------------------------------------------------- the signed model
def test_probe_signed_lbuffer_update(ctx):
    """Device glibc exp restatement: the signed L update for a stride over all
    f32 distances equals the host build's (itself equal to libm's, CPU suite)."""
    d = np.arange(0, 1 << 32, 257, dtype=np.uint64).astype(np.uint32).view(np.float32)
    got = ctx.probe_math(_abi.XRT_PROBE_SIGNED_L, d)
    want = np.empty_like(d)
    _abi.load().xrt_host_signed_lbuffer_batch(d.ctypes.data_as(_abi._fp), None, np.float32(0.1037),
                                              want.ctypes.data_as(_abi._fp), d.size)
    assert np.array_equal(bits(got), bits(want))


def test_probe_prep_normals(signed, dragon):
    """k_prep's unit normals (Triangle::computeNormal) in the records' pad words."""
    soup = np.concatenate([dragon, synthetic_soup(n=600)])
    signed.upload_mesh(soup)
    rec, _ = signed.probe_prep(xrt.camera_for_mesh(soup, 64, 64), len(soup))
    got = np.ascontiguousarray(rec.reshape(-1, 16)[:, 13:16])
    want = oracle.triangle_normals(soup)
    same = (bits(got) == bits(want)) | (np.isnan(got) & np.isnan(want))
    assert same.all()


def _signed_case(name, dragon):
    if name == "dragon+box":
        return [dragon, second_mesh_for(dragon)], 128, 112
    if name == "sheets":
        return [striped_sheets()], 96, 80
    if name == "corner":
        return [corner_soup()], 33, 31
    return [synthetic_soup(seed=9, n=2000)], 80, 72


@pytest.mark.parametrize("kernel", SIGNED_KERNELS)
@pytest.mark.parametrize("name", ["dragon+box", "sheets", "corner", "soup"])
def test_signed_scene_matches_oracle(signed, dragon, kernel, name):
    meshes, W, H = _signed_case(name, dragon)
    cam = xrt.camera_for_scene(meshes, W, H)
    signed.set_kernel(kernel)
    signed.upload_mesh(meshes[0])
    img, lb, u8, st = signed.render_signed(cam)
    rlb, rnh, flagged = oracle.render_signed_rows(meshes, cam13(cam), W, H)
    assert np.array_equal(bits(lb), bits(rlb)), np.nonzero(bits(lb) != bits(rlb))[0][:8]
    rimg = oracle.hole_fill(rlb, W, H)
    assert np.array_equal(bits(img), bits(rimg))
    assert np.array_equal(u8, lut(rimg))
    assert st.odd_rays == flagged and st.hits == int(rnh.sum()) and st.hit_rays == int(np.count_nonzero(rnh))
    if name in ("sheets", "soup"):
        assert flagged > 20


@pytest.mark.parametrize("kernel", SIGNED_KERNELS)
@pytest.mark.parametrize("cap", [1, 2, 5])
def test_signed_overflow_path_exact(signed, dragon, kernel, cap):
    """Rays with more hits than the list: the wave's triangle-order re-scan."""
    meshes = [striped_sheets(seed=4)]
    W, H = 64, 56
    cam = xrt.camera_for_scene(meshes, W, H)
    signed.set_kernel(kernel)
    signed.set_hit_capacity(cap)
    signed.upload_mesh(meshes[0])
    _, lb, _, st = signed.render_signed(cam)
    rlb, rnh, _ = oracle.render_signed_rows(meshes, cam13(cam), W, H)
    assert st.overflow_rays > 0
    assert np.array_equal(bits(lb), bits(rlb))


@pytest.mark.parametrize("kernel", SIGNED_KERNELS)
@pytest.mark.parametrize("planes,size", [(40, 24), (128, 16), (150, 16)])
def test_signed_deep_stack_overflow(signed, kernel, planes, size):
    """Rays through 40..150 alternately wound planes (signs cancel, so the rays
    are not flagged and their sums need the overflow path): the fix-up over the
    tile's survivors (<= 256) and over all candidates past that."""
    meshes = [plane_stack(planes, alternate=True)]
    cam = xrt.camera_for_scene(meshes, size, size)
    signed.set_kernel(kernel)
    signed.upload_mesh(meshes[0])
    _, lb, _, st = signed.render_signed(cam)
    rlb, rnh, flagged = oracle.render_signed_rows(meshes, cam13(cam), size, size)
    assert int(rnh.max()) > 12 and st.overflow_rays > 0 and flagged < size * size
    assert np.array_equal(bits(lb), bits(rlb)), np.nonzero(bits(lb) != bits(rlb))[0][:8]


def test_signed_strips_assemble(signed, dragon):
    meshes, W, H = _signed_case("dragon+box", dragon)
    cam = xrt.camera_for_scene(meshes, W, H)
    signed.set_kernel(xrt.XRT_KERNEL_BINNED)
    signed.upload_mesh(meshes[0])
    _, full, _, _ = signed.render_signed(cam)
    parts = [signed.render_rows(cam, r0, r1, image=False, u8=False)[1] for r0, r1 in [(0, 37), (37, 40), (40, H)]]
    assert np.array_equal(bits(np.concatenate(parts)), bits(full))
    with pytest.raises(xrt.XrtError):          # the signed model's image is the hole fill's
        signed.render_rows(cam, 0, H)


def test_signed_dragon_512(signed, dragon):
    """dragon.ply at 512^2: 3 flagged rays (the odd rays of the main path), filled."""
    W = H = 512
    cam = xrt.camera_for_mesh(dragon, W, H)
    signed.set_kernel(xrt.XRT_KERNEL_BINNED)
    signed.upload_mesh(dragon)
    img, lb, u8, st = signed.render_signed(cam)
    rlb, rnh, flagged = oracle.render_signed_rows([dragon], cam13(cam), W, H)
    assert flagged == 3 and st.odd_rays == 3
    assert np.array_equal(bits(lb), bits(rlb))
    assert np.array_equal(bits(img), bits(oracle.hole_fill(rlb, W, H)))


@pytest.mark.parametrize("W,H", [(1, 1), (7, 5), (64, 48), (1000, 3), (3, 700)])
def test_hole_fill_device(ctx, W, H):
    rng = np.random.default_rng(W * 31 + H)
    L = rng.uniform(1, 80, W * H).astype(np.float32)
    L[rng.random(W * H) < 0.4] = -1
    L[rng.random(W * H) < 0.05] = 0
    L[rng.random(W * H) < 0.02] = np.inf
    L[rng.random(W * H) < 0.02] = np.array([0x7FC00000], np.uint32).view(np.float32)[0]
    img, u8 = ctx.hole_fill(L, W, H)
    want = oracle.hole_fill(L, W, H)
    assert np.array_equal(bits(img), bits(want))
    assert np.array_equal(u8, lut(want))


def test_cli_signed_text(tmp_path, dragon):
    """xrt_main --signed: the fork's output (filled image) as the reference's text."""
    second = second_mesh_for(dragon)
    _write_obj(tmp_path / "box.obj", second)
    (tmp_path / "out").mkdir()
    r = subprocess.run([EXE, "--signed", "-s", "64", "64", "-i", DRAGON, "-i", str(tmp_path / "box.obj"),
                        "-f", "l.txt", "--lbuffer", str(tmp_path / "l.f32")],
                       capture_output=True, text=True, cwd=tmp_path, timeout=300)
    assert r.returncode == 0, r.stderr
    meshes = [dragon, second]
    rlb, _, _ = oracle.render_signed_rows(meshes, oracle.camera_for_scene(meshes, 64, 64), 64, 64)
    assert np.array_equal(bits(np.fromfile(tmp_path / "l.f32", np.float32)), bits(rlb))
    assert (tmp_path / "out" / "l.txt").read_bytes() == oracle.text_bytes(oracle.hole_fill(rlb, 64, 64), 64, 64)


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_signed_strips(signed, dragon, devices):
    """The signed model over row strips: L-buffer strips gathered to device 0,
    which fills the holes of the assembled frame -- equal to one device's
    render and to the oracle (flagged pixels near strip boundaries included)."""
    meshes = [striped_sheets(seed=6)]
    W, H = 96, 83
    cam = xrt.camera_for_scene(meshes, W, H)
    signed.set_kernel(xrt.XRT_KERNEL_BINNED)
    signed.upload_mesh(meshes[0])
    ref = signed.render_signed(cam)
    with xrt.MultiContext(devices) as m:
        m.set_kernel(xrt.XRT_KERNEL_BINNED)
        m.upload_mesh(meshes[0])
        m.set_model(xrt.XRT_MODEL_SIGNED, 0.1037)
        for _ in range(3):                              # the strip buffers rotate
            img, lb, u8, st = m.render(cam)
            assert np.array_equal(bits(lb), bits(ref[1])) and np.array_equal(bits(img), bits(ref[0]))
            assert np.array_equal(u8, ref[2]) and st.odd_rays == ref[3].odd_rays
        m.set_model(xrt.XRT_MODEL_ATTENUATION, 0.0)      # back to the attenuation model: unchanged
        att = m.render(cam)
    rlb, _, _ = oracle.render_signed_rows(meshes, cam13(cam), W, H)
    assert np.array_equal(bits(lb), bits(rlb))
    signed.set_model(xrt.XRT_MODEL_ATTENUATION, 0.0)
    one = signed.render_rows(cam)
    assert np.array_equal(bits(att[0]), bits(one[0])) and np.array_equal(bits(att[1]), bits(one[1]))


def test_cli_signed_two_gpus_rehearsal(tmp_path, dragon):
    """xrt_main --signed -g 2 (XRT_MULTI_DEVICES=0,0): the same text as one GPU."""
    (tmp_path / "out").mkdir()
    env = dict(os.environ, XRT_MULTI_DEVICES="0,0")
    for name, extra in (("one.txt", []), ("two.txt", ["-g", "2"])):
        r = subprocess.run([EXE, "--signed", "-s", "80", "72", "-i", DRAGON, "-f", name] + extra,
                           capture_output=True, text=True, cwd=tmp_path, timeout=300, env=env)
        assert r.returncode == 0, r.stderr
    assert (tmp_path / "out" / "one.txt").read_bytes() == (tmp_path / "out" / "two.txt").read_bytes()


def test_exit_with_live_contexts():
    """A process that leaves a context and a multi context alive (renders
    done, frames streamed through the pinned ring and copy threads, nothing
    destroyed) exits with status 0: libxrt holds no static object with a
    destructor, so the finalizers the process's exit runs in an order libxrt
    does not control never tear anything of it down (round 5 saw one SIGSEGV in
    __cxa_finalize at a child's exit).  XRT_SEGV_TRACE=1 names the library of a
    fatal signal, should one come."""
    env = dict(os.environ, XRT_SEGV_TRACE="1")
    r = subprocess.run([os.sys.executable, os.path.join(ROOT, "tests", "_exit_job.py")], capture_output=True,
                       text=True, timeout=110, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-1000:], r.stderr[-3000:])
    assert "exit job: ok" in r.stdout
