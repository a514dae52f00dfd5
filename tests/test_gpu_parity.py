"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle, the
reference's golden text and size-independent properties.  Bit-exact on the
f32 image, the f32 L-buffer and the 8-bit image (the north star's bar is
bit-exact u8 and 1e-5 relative on the L-buffer; these tests demand 0 ULP)."""
import os
import subprocess
import time

import numpy as np
import pytest

import simpleraytracing_amd as xrt
from simpleraytracing_amd import _abi
from simpleraytracing_amd.scenes import orbit_camera, tiled_mesh
from oracle import oracle
from conftest import DRAGON, GOLDEN, ROOT, bits
from kat import kat_vectors
from scene_kit import corner_soup, plane_stack, synthetic_soup

pytestmark = pytest.mark.gpu
KERNELS = [xrt.XRT_KERNEL_BRUTE, xrt.XRT_KERNEL_TILED, xrt.XRT_KERNEL_BINNED]
KNAME = {xrt.XRT_KERNEL_BRUTE: "brute", xrt.XRT_KERNEL_TILED: "tiled", xrt.XRT_KERNEL_BINNED: "binned"}


def cam13(cam):
    return np.array(list(cam.origin) + list(cam.detector) + list(cam.up) + list(cam.right) +
                    [cam.pixel_spacing], np.float32)


def render(ctx, tris, W, H, kernel, r0=0, r1=None, cam=None):
    ctx.set_kernel(kernel)
    ctx.upload_mesh(tris)
    cam = cam or xrt.camera_for_mesh(tris, W, H)
    return ctx.render_rows(cam, r0, r1)


def assert_same(gpu, ref, what=""):
    img, lb, u8, st = gpu
    rimg, rlb, ru8, rnh, rodd = ref
    assert np.array_equal(bits(img), bits(rimg)), f"{what}: image differs at {np.nonzero(bits(img) != bits(rimg))[0][:8]}"
    assert np.array_equal(bits(lb), bits(rlb)), f"{what}: L-buffer differs"
    assert np.array_equal(u8, ru8), f"{what}: u8 differs"
    assert st.odd_rays == rodd
    assert st.hit_rays == int(np.count_nonzero(rnh))
    assert st.hits == int(rnh.sum())
    assert st.max_hits == (int(rnh.max()) if rnh.size else 0)


# --------------------------------------------------------------------------- probes
def test_probe_expf_matches_libm(ctx):
    # every float in [-0.25, 0] plus strides over [-16, -0.25] and the full range
    parts = [np.arange(0x80000000, 0xBE800001, 1, dtype=np.uint64),
             np.arange(0xBE800000, 0xC1800000, 5, dtype=np.uint64),
             np.arange(0xC1800000, 0xFF800001, 4099, dtype=np.uint64),
             np.arange(0x00000000, 0x7F800001, 4099, dtype=np.uint64)]
    for p in parts:
        for c in range(0, p.size, 1 << 26):
            x = p[c:c + (1 << 26)].astype(np.uint32).view(np.float32)
            got = ctx.probe_math(_abi.XRT_PROBE_EXPF, x)
            want = oracle.expf(x)
            same = (bits(got) == bits(want)) | (np.isnan(got) & np.isnan(want))
            assert same.all(), x[~same][:8]


def special_floats():
    rng = np.random.default_rng(7)
    r = rng.integers(0, 2**32, 1 << 22, dtype=np.uint64).astype(np.uint32).view(np.float32)
    den = rng.integers(1, 0x800000, 1 << 16, dtype=np.uint64).astype(np.uint32).view(np.float32)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, 2.0, 3.0, 1e-45, 1.17549435e-38,
                   3.4028235e38, 0.5, 1e-38], np.float32)
    return np.concatenate([r, den, -den, sp])


def test_probe_sqrt_correctly_rounded(ctx):
    x = np.abs(special_floats())
    got = ctx.probe_math(_abi.XRT_PROBE_SQRTF, x)
    want = np.sqrt(x)
    same = (bits(got) == bits(want)) | (np.isnan(got) & np.isnan(want))
    assert same.all(), x[~same][:8]


def test_probe_reciprocal_matches_double_division(ctx):
    # the device's 1.0f / det against Ray.cxx:99's (float)(1.0 / (double)det)
    # (identical for every f32: tools/check_fp_identities.c); specials plus a
    # stride-61 sweep of all 2^32 bit patterns
    sweep = np.arange(0, 1 << 32, 61, dtype=np.uint64).astype(np.uint32).view(np.float32)
    for x in (special_floats(), sweep):
        for c in range(0, x.size, 1 << 25):
            xc = x[c:c + (1 << 25)]
            got = ctx.probe_math(_abi.XRT_PROBE_RCP, xc)
            with np.errstate(divide="ignore", over="ignore"):
                want = (1.0 / xc.astype(np.float64)).astype(np.float32)
            same = (bits(got) == bits(want)) | (np.isnan(got) & np.isnan(want))
            assert same.all(), xc[~same][:8]


@pytest.mark.parametrize("op", [_abi.XRT_PROBE_RCP, _abi.XRT_PROBE_RCP_FAST])
def test_probe_reciprocal_every_exponent(ctx, op):
    # every biased exponent x 2^16 mantissas (both signs), incl. the ends of
    # the short sequence's range (2^-126 and 2^126) and the mantissa extremes
    rng = np.random.default_rng(20250302)
    man = np.concatenate([np.arange(64, dtype=np.uint32), (1 << 23) - 1 - np.arange(64, dtype=np.uint32),
                          rng.integers(0, 1 << 23, (1 << 16) - 128, dtype=np.uint32)])
    exps = np.arange(256, dtype=np.uint32)
    x = ((exps[:, None] << 23) | man[None, :]).ravel()
    x = np.concatenate([x, x | np.uint32(0x80000000)]).view(np.float32)
    got = ctx.probe_math(op, x)
    with np.errstate(divide="ignore", over="ignore"):
        want = (np.float32(1.0) / x).astype(np.float32)
    same = (bits(got) == bits(want)) | (np.isnan(got) & np.isnan(want))
    assert same.all(), x[~same][:8]


def test_probe_fast_reciprocal_sweep(ctx):
    # the culled tests' reciprocal on the stride-61 sweep of all 2^32 patterns
    sweep = np.arange(0, 1 << 32, 61, dtype=np.uint64).astype(np.uint32).view(np.float32)
    for x in (special_floats(), sweep):
        for c in range(0, x.size, 1 << 25):
            xc = x[c:c + (1 << 25)]
            got = ctx.probe_math(_abi.XRT_PROBE_RCP_FAST, xc)
            with np.errstate(divide="ignore", over="ignore"):
                want = (np.float32(1.0) / xc).astype(np.float32)
            same = (bits(got) == bits(want)) | (np.isnan(got) & np.isnan(want))
            assert same.all(), xc[~same][:8]


def test_probe_lut_sweep(ctx):
    # every 13th f32 in [0, 80] against Image.inl:195-211's formula in f64
    # (round half away from zero == floor(x + 0.5) here, exactly)
    v = np.arange(0, 0x42A00001, 13, dtype=np.uint64).astype(np.uint32).view(np.float32)
    for c in range(0, v.size, 1 << 24):
        vc = v[c:c + (1 << 24)]
        got = ctx.probe_math(_abi.XRT_PROBE_LUT_U8, vc)
        want = np.floor(255.0 * vc.astype(np.float64) / 80.0 + 0.5).astype(np.float32)
        assert np.array_equal(got, want), vc[got != want][:8]


def test_probe_lut(ctx):
    v = np.concatenate([np.linspace(-1, 81, 200001, dtype=np.float32),
                        np.arange(0, 256, dtype=np.float32) * np.float32(80.0 / 255.0),
                        (np.arange(0, 255, dtype=np.float64) + 0.5).astype(np.float32) * np.float32(80.0 / 255.0)])
    got = ctx.probe_math(_abi.XRT_PROBE_LUT_U8, v)
    want = np.array([oracle.lut_u8(float(a)) for a in v], np.float32)
    assert np.array_equal(got, want)


def test_probe_intersect_kat(ctx):
    rays, tris = kat_vectors()
    h1, t1 = ctx.probe_intersect(rays, tris)
    h2, t2 = oracle.intersect_batch(rays, tris)
    assert np.array_equal(h1, h2)
    assert np.array_equal(bits(t1), bits(t2))


# --------------------------------------------------------------------------- renders
@pytest.mark.parametrize("kernel", KERNELS)
def test_golden_128(ctx, dragon, kernel):
    """The reference's own golden, out/dragon-128x128-serial.txt, byte for byte."""
    img, lb, u8, st = render(ctx, dragon, 128, 128, kernel)
    want = open(os.path.join(GOLDEN, "dragon-128x128-serial.txt"), "rb").read()
    assert oracle.text_bytes(img, 128, 128) == want
    cam = oracle.camera_for_mesh(dragon, 128, 128)
    assert_same((img, lb, u8, st), oracle.render_rows(dragon, cam, 128, 128), KNAME[kernel])
    assert st.rays == 128 * 128 and st.kernel == kernel


@pytest.mark.parametrize("kernel", KERNELS)
def test_full_256(ctx, dragon, kernel):
    got = render(ctx, dragon, 256, 256, kernel)
    cam = oracle.camera_for_mesh(dragon, 256, 256)
    assert_same(got, oracle.render_rows(dragon, cam, 256, 256), KNAME[kernel])


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("W,H,r0,r1", [(1, 1, 0, 1), (7, 13, 0, 13), (33, 17, 0, 17), (100, 3, 0, 3),
                                        (3, 100, 0, 100), (65, 65, 5, 50), (64, 64, 63, 64),
                                        (97, 41, 40, 41), (50, 50, 20, 20)])
def test_ragged_sizes_and_strips(ctx, dragon, kernel, W, H, r0, r1):
    got = render(ctx, dragon, W, H, kernel, r0, r1)
    cam = oracle.camera_for_mesh(dragon, W, H)
    assert_same(got, oracle.render_rows(dragon, cam, W, H, r0, r1), f"{KNAME[kernel]} {W}x{H}")


@pytest.mark.parametrize("kernel", KERNELS)
def test_strips_assemble_to_full_image(ctx, dragon, kernel):
    W = H = 160
    full = render(ctx, dragon, W, H, kernel)
    for n in (2, 3, 8):
        rows_per, rem = divmod(H, n)
        parts, start = [], 0
        for g in range(n):
            end = start + rows_per + (1 if g < rem else 0)
            parts.append(render(ctx, dragon, W, H, kernel, start, end)[0])
            start = end
        assert np.array_equal(bits(np.concatenate(parts)), bits(full[0]))


def test_binned_list_overflow_falls_back_exactly(ctx, dragon):
    """Region lists capped at 16 entries: every region with more candidates
    takes the whole-mesh path (3x3 regions at 96x96, each holds far more)."""
    cam = oracle.camera_for_mesh(dragon, 96, 96)
    ref = oracle.render_rows(dragon, cam, 96, 96)
    ctx.set_bin_capacity(16)
    try:
        got = render(ctx, dragon, 96, 96, xrt.XRT_KERNEL_BINNED)
    finally:
        ctx.set_bin_capacity(0)
    assert got[3].candidates >= len(dragon)         # at least one region is the whole mesh
    assert_same(got, ref, "binned overflow")
    again = render(ctx, dragon, 96, 96, xrt.XRT_KERNEL_BINNED)
    assert again[3].candidates < 9 * len(dragon)
    assert_same(again, ref, "binned")


@pytest.mark.parametrize("kernel", KERNELS)
def test_overflow_path_exact(ctx, dragon, kernel):
    """Hit lists capped at 1 and 2 entries: the exact overflow kernel takes over."""
    cam = oracle.camera_for_mesh(dragon, 96, 96)
    ref = oracle.render_rows(dragon, cam, 96, 96)
    for cap in (1, 2):
        ctx.set_hit_capacity(cap)
        try:
            got = render(ctx, dragon, 96, 96, kernel)
        finally:
            ctx.set_hit_capacity(0)
        assert got[3].overflow_rays == int(np.count_nonzero(ref[3] > cap))
        assert_same(got, ref, f"{KNAME[kernel]} cap={cap}")


MAX_HITS = 12  # the register hit list (XRT_MAX_HITS); rays past it take the exact fix-up


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("planes,size", [(40, 48), (128, 24), (129, 24), (300, 16), (2100, 8)])
def test_deep_stack_overflow(ctx, kernel, planes, size):
    """Rays with 40..4200 hits: the wave-wide overflow fix-up must equal the
    oracle's std::sort + pair sum -- over the tile's survivors (up to 256: 128
    planes fill all four slots on the diagonal tiles, where both triangles of a
    square survive), and over all candidates past that (129 planes on the
    diagonal, 300, 2100; register lists bitonic-sorted across the wave up to 8
    hits a lane, streamed beyond)."""
    if kernel == xrt.XRT_KERNEL_BRUTE and planes > 100:
        pytest.skip("brute force is covered by the 40-plane case")
    soup = plane_stack(planes)
    cam = oracle.camera_for_mesh(soup, size, size)
    ref = oracle.render_rows(soup, cam, size, size)
    got = render(ctx, soup, size, size, kernel)
    assert int(ref[3].max()) > MAX_HITS
    assert got[3].overflow_rays == int(np.count_nonzero(ref[3] > MAX_HITS))
    assert_same(got, ref, f"{KNAME[kernel]} {planes} planes")


@pytest.mark.parametrize("kernel", KERNELS)
def test_empty_mesh(ctx, dragon, kernel):
    cam = xrt.camera_for_mesh(dragon, 40, 30)
    ctx.set_kernel(kernel)
    ctx.upload_mesh(np.zeros((0, 9), np.float32))
    img, lb, u8, st = ctx.render_rows(cam)
    assert np.all(img == np.float32(80.0)) and np.all(np.isinf(lb)) and np.all(u8 == 255)
    assert st.hits == 0


@pytest.mark.parametrize("kernel", KERNELS)
def test_synthetic_soup_with_degenerates(ctx, kernel):
    soup = synthetic_soup()
    got = render(ctx, soup, 80, 72, kernel)
    cam = oracle.camera_for_mesh(soup, 80, 72)
    ref = oracle.render_rows(soup, cam, 80, 72)
    assert ref[4] > 0      # odd rays occur (open soup)
    assert_same(got, ref, KNAME[kernel])


@pytest.mark.parametrize("kernel", KERNELS)
def test_custom_camera_triangles_around_source(ctx, kernel):
    """Camera inside the scene: triangles behind, through and around the source."""
    soup = synthetic_soup(seed=5, n=1500)
    lo, hi = oracle.bbox(soup[:200])     # camera fitted to a sub-box: source lies inside the soup
    cam = xrt.camera_from_bbox(lo, hi, 64, 48)
    ctx.set_kernel(kernel)
    ctx.upload_mesh(soup)
    got = ctx.render_rows(cam)
    ref = oracle.render_rows(soup, cam13(cam), 64, 48)
    assert_same(got, ref, KNAME[kernel])


@pytest.mark.parametrize("kernel", KERNELS)
def test_infinite_hit_corner(ctx, kernel):
    """The cull's former non-conservative corner (DESIGN.md "Tile cull", step 0):
    t = +inf hits, inf - inf = NaN path lengths (x86's default NaN bits) --
    every kernel equal to the oracle bit for bit."""
    soup = corner_soup()
    W, H = 33, 31
    cam = oracle.camera_for_mesh(soup, W, H)
    ref = oracle.render_rows(soup, cam, W, H)
    assert np.isnan(ref[1]).sum() > 0 and ref[3].reshape(H, W)[:, W // 2].max() > 2
    got = render(ctx, soup, W, H, kernel)
    assert_same(got, ref, f"{KNAME[kernel]} corner")


def strip_boundary_rows(H, n=8):
    """SURVEY.md 8(c)'s fixture rows: 0, H/n*k - 1, H/n*k, H/2, H - 1."""
    rows = {0, H // 2, H - 1}
    for k in range(1, n):
        rows |= {H // n * k - 1, H // n * k}
    return sorted(rows)


def test_dragon_1024_full_frame(ctx, dragon):
    """BASELINE configs[1] (dragon 1024^2, one GPU): binned == brute over the whole
    frame, strip-boundary rows vs the oracle, SURVEY facts as properties."""
    W = H = 1024
    a = render(ctx, dragon, W, H, xrt.XRT_KERNEL_BINNED)
    b = render(ctx, dragon, W, H, xrt.XRT_KERNEL_BRUTE)
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(bits(x), bits(y))
    assert (a[3].hit_rays, a[3].odd_rays, a[3].max_hits) == (b[3].hit_rays, b[3].odd_rays, b[3].max_hits)
    rows = strip_boundary_rows(H)
    cam = oracle.camera_for_mesh(dragon, W, H)
    ref = oracle.render_row_list(dragon, cam, W, H, rows)
    for plane, want in zip(a[:3], ref[:3]):
        assert np.array_equal(bits(plane.reshape(H, W)[rows].ravel()), bits(want))
    miss = np.isinf(a[1])
    assert np.all(a[0][miss] == np.float32(80.0)) and np.all(a[2][miss] == 255)
    assert np.all(a[1][~miss] >= 0) and np.all(a[0] <= np.float32(80.0)) and np.all(a[0] > 0)


def test_tiled_mesh_8192_strip_rows(ctx, dragon):
    """BASELINE configs[4] at full size: the 1,120,434-triangle tiled dragon at
    8192^2.  The binned frame, rendered whole and as the 8 row strips of the
    8-GPU split (rows_per = H/8), is bit-equal on every strip-boundary row to
    the literal brute-force kernel, and to the CPU oracle on sampled columns."""
    t0 = time.time()
    big = tiled_mesh(dragon, 7)
    W = H = 8192
    ctx.set_kernel(xrt.XRT_KERNEL_BINNED)
    ctx.upload_mesh(big)
    cam = xrt.camera_for_mesh(big, W, H)
    full = ctx.render_rows(cam, lbuffer=True, u8=True)
    # oblique rays at the frame's edges cross two neighbouring copies: more
    # hits than the register list holds, resolved by the exact in-wave fix-up
    assert full[3].max_hits > 12 and full[3].overflow_rays > 0
    rows = strip_boundary_rows(H)
    for g in range(8):                                   # the 8 strips of the 8-GPU split
        r0, r1 = g * H // 8, (g + 1) * H // 8
        part = ctx.render_rows(cam, r0, r1)
        for plane, whole in zip(part[:3], full[:3]):
            assert np.array_equal(bits(plane), bits(whole[r0 * W:r1 * W])), (r0, r1)
        del part
    print(f"8192: binned frame and its 8 strips equal ({time.time() - t0:.1f} s)", flush=True)
    ctx.set_kernel(xrt.XRT_KERNEL_BRUTE)
    for r in rows:
        one = ctx.render_rows(cam, r, r + 1)
        for plane, whole in zip(one[:3], full[:3]):
            assert np.array_equal(bits(plane), bits(whole[r * W:(r + 1) * W])), r
    print(f"8192: brute rows equal ({time.time() - t0:.1f} s)", flush=True)
    cam13 = oracle.camera_for_mesh(big, W, H)
    for c0, c1 in [(0, 64), (W // 2 - 128, W // 2 + 128), (W - 64, W)]:   # both edges and the centre
        img, lb, u8, _, _ = oracle.render_row_list_span(big, cam13, W, H, rows, c0, c1, threads=16)
        sl = np.concatenate([np.arange(r * W + c0, r * W + c1) for r in rows])
        assert np.array_equal(bits(img), bits(full[0][sl])), c0
        assert np.array_equal(bits(lb), bits(full[1][sl])), c0
        assert np.array_equal(u8, full[2][sl]), c0
        print(f"8192: oracle columns [{c0}, {c1}) equal ({time.time() - t0:.1f} s)", flush=True)


def test_all_kernels_equal_2048(ctx, dragon):
    """Full 2048^2 frame: the three kernels bit-identical; sampled rows vs the
    oracle; SURVEY.md's dragon facts (hit rays, odd rays, max hits)."""
    W = H = 2048
    a = render(ctx, dragon, W, H, xrt.XRT_KERNEL_BINNED)
    for k in (xrt.XRT_KERNEL_TILED, xrt.XRT_KERNEL_BRUTE):
        b = render(ctx, dragon, W, H, k)
        for x, y in zip(a[:3], b[:3]):
            assert np.array_equal(bits(x), bits(y)), KNAME[k]
    st = a[3]
    assert (st.hit_rays, st.odd_rays, st.max_hits) == (1365802, 24, 12)
    # the cull is effective: ~75k region-list entries and ~3 exact tests per ray
    assert st.candidates < 200000 and st.tile_tests * 64 < 5 * W * H, (st.candidates, st.tile_tests)
    rows = [0, 255, 256, 511, 512, 1023, 1024, 1535, 1536, 1792, 2047]
    cam = oracle.camera_for_mesh(dragon, W, H)
    ref = oracle.render_row_list(dragon, cam, W, H, rows)
    img = a[0].reshape(H, W)[rows].ravel()
    lb = a[1].reshape(H, W)[rows].ravel()
    u8 = a[2].reshape(H, W)[rows].ravel()
    assert np.array_equal(bits(img), bits(ref[0]))
    assert np.array_equal(bits(lb), bits(ref[1]))
    assert np.array_equal(u8, ref[2])
    # size-independent properties over the whole frame
    miss = np.isinf(a[1])
    assert np.all(a[0][miss] == np.float32(80.0)) and np.all(a[2][miss] == 255)
    assert np.all(a[1][~miss] >= 0) and np.all(a[0] <= np.float32(80.0)) and np.all(a[0] > 0)


STAT_FIELDS = ("rays", "hit_rays", "odd_rays", "overflow_rays", "hits", "max_hits", "tile_tests", "candidates")


def _stats(st):
    return tuple(getattr(st, f) for f in STAT_FIELDS)


@pytest.mark.parametrize("W,H,r0,r1", [(2048, 2048, 0, None), (1024, 1024, 0, None), (1000, 700, 0, None),
                                       (333, 517, 100, 400), (4096, 4096, 1536, 2048)])
def test_fill_plan_changes_nothing(ctx, dragon, W, H, r0, r1):
    """The fill plan (regions the sizing frame counted empty rendered as one
    miss-filling workgroup each, DESIGN.md "Fill plan") leaves every bit and
    every statistic of the frame as the plan-free render has them: the
    geometry's first frame (sized on the device, its empty regions one fill
    workgroup each too), the host-sized frame and a later frame of the
    geometry."""
    ctx.set_fill_plan(0)
    try:
        off = render(ctx, dragon, W, H, xrt.XRT_KERNEL_BINNED, r0, r1)
        off = ctx.render_rows(xrt.camera_for_mesh(dragon, W, H), r0, r1)
        assert ctx.fill_regions() == 0
    finally:
        ctx.set_fill_plan(1)
    cam = xrt.camera_for_mesh(dragon, W, H)
    for frame in range(3):          # the first frame, the sizing frame, a frame reusing the plan
        on = render(ctx, dragon, W, H, xrt.XRT_KERNEL_BINNED, r0, r1) if frame == 0 else ctx.render_rows(cam, r0, r1)
        n_fill = ctx.fill_regions()
        rows = (r1 or H) - r0
        regions = -(-W // 32) * -(-rows // 32)
        if frame == 0:
            assert n_fill == 0 and ctx.first_frames()["device_sized"] > 0, (frame, n_fill)
        else:
            assert 0 < n_fill < regions, (frame, n_fill, regions)
        for x, y in zip(on[:3], off[:3]):
            assert np.array_equal(bits(x), bits(y)), frame
        assert _stats(on[3]) == _stats(off[3]), frame


@pytest.mark.parametrize("W,H,r0,r1,degs", [
    (512, 512, 0, None, [0, 1, 2, 3, 3.5, 10, 10, 10, 45, 46, 90, 91, 0]),
    (1000, 700, 0, None, [0, 0.5, 1, 1.5, 30, 30.5, 30.5, 30.5, 180, 181]),
    (1024, 1024, 256, 700, [0, 1, 2, 20, 21, 22, 22, 22]),
])
def test_moving_camera_reuses_lists_exactly(dragon, W, H, r0, r1, degs):
    """A projection sweep: each frame a new camera over the same region grid, so
    the context renders over the lists sized for an earlier camera (no
    synchronous re-sizing, no fill plan), k_prep flags a list that overflows
    (that region renders from the whole mesh, the next frame re-sizes), and a
    camera that stays put for two frames more is sized for itself again (fill
    plan back).  Every frame is bit-identical, image, L-buffer, u8 and hit
    statistics, to a fresh context's brute-force render of that camera; the
    geometry counters show which path each frame took."""
    lo, hi = xrt.mesh_bbox(dragon)
    centre = 0.5 * (np.asarray(lo, np.float64) + np.asarray(hi, np.float64))
    base = xrt.camera_for_mesh(dragon, W, H)
    seq = xrt.Context(0)
    seq.set_kernel(xrt.XRT_KERNEL_BINNED)
    seq.upload_mesh(dragon)
    fills, paths = [], []
    for i, d in enumerate(degs):
        cam = orbit_camera(base, centre, d)
        before = seq.geometry_counters()
        got = seq.render_rows(cam, r0, r1)
        after = seq.geometry_counters()
        paths.append({k: after[k] - before[k] for k in after})
        fills.append(seq.fill_regions())
        with xrt.Context(0) as fresh:
            fresh.set_kernel(xrt.XRT_KERNEL_BRUTE)
            fresh.upload_mesh(dragon)
            ref = fresh.render_rows(cam, r0, r1)
        for x, y in zip(got[:3], ref[:3]):
            assert np.array_equal(bits(x), bits(y)), (i, d)
        for f in ("rays", "hit_rays", "odd_rays", "max_hits"):
            assert getattr(got[3], f) == getattr(ref[3], f), (i, d, f)
    total = seq.geometry_counters()
    seq.close()
    # the first frame sized on the device (no host plan); later cameras over its
    # grid take the moving camera's path
    assert paths[0]["sizings"] == 0 and fills[0] == 0, (paths[0], fills[0])
    assert total["reused"] > 0 and total["sizings"] < len(degs), total
    # reused frames run without a fill plan; the third frame in a row on one
    # camera is sized for it (a fill plan again)
    for i, p in enumerate(paths):
        if p["reused"]:
            assert fills[i] == 0 and p["sizings"] == 0, (i, p, fills[i])
    still = max(i for i in range(2, len(degs)) if degs[i] == degs[i - 1] == degs[i - 2])
    assert paths[still]["sizings"] == 1 and fills[still] > 0, (paths[still], fills[still])


@pytest.mark.parametrize("device_fill", ["1", "0"])
def test_moving_camera_pool_overflow_exact(dragon, monkeypatch, device_fill):
    """A moving camera's device-sized lists with a pool far too small
    (XRT_MOTION_POOL=300 entries): the lists that do not fit get what is left,
    their regions render from the whole mesh (exact), k_prep's flags report
    the overflows when the set is next used; every frame, through device planes
    on two streams, equals a brute-force render of its camera -- over the
    device fill plan (empty regions one fill workgroup each) and without it."""
    import torch
    monkeypatch.setenv("XRT_MOTION_POOL", "300")
    monkeypatch.setenv("XRT_DEVICE_FILL", device_fill)
    W, H = 512, 384
    lo, hi = xrt.mesh_bbox(dragon)
    centre = 0.5 * (np.asarray(lo, np.float64) + np.asarray(hi, np.float64))
    base = xrt.camera_for_mesh(dragon, W, H)
    cams = [orbit_camera(base, centre, 2.0 * k) for k in range(10)]
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    with xrt.Context(0) as brute:
        brute.set_kernel(xrt.XRT_KERNEL_BRUTE)
        brute.upload_mesh(dragon)
        refs = [brute.render_rows(c) for c in cams]
    with xrt.Context(0) as c:
        c.set_kernel(xrt.XRT_KERNEL_BINNED)
        c.upload_mesh(dragon)
        outs = [(torch.empty(W * H, device=dev), torch.empty(W * H, device=dev),
                 torch.empty(W * H, dtype=torch.uint8, device=dev)) for _ in cams]
        for k, cam in enumerate(cams):
            c.render_rows_device(cam, 0, H, *(t.data_ptr() for t in outs[k]), streams[k % 2].cuda_stream)
        torch.cuda.synchronize(dev)
        for k in range(len(cams)):
            for x, y in zip(outs[k], refs[k][:3]):
                assert np.array_equal(bits(x.cpu().numpy()), bits(y)), k
        for cam in cams[:4]:                                   # the sets come round: flags read
            c.render_rows(cam)
        g = c.geometry_counters()
    assert g["reused"] >= 9 and g["overflows"] > 0, g


def _box_masks_case(name, dragon):
    if name == "dragon-strip":
        return dragon, 1000, 777, 13, 700
    if name == "soup":
        return synthetic_soup(seed=3, n=3000), 300, 200, 0, None
    if name == "corner":
        return corner_soup(), 33, 31, 0, None
    return tiled_mesh(dragon, 3), 1024, 1024, 0, None


@pytest.mark.parametrize("model", ["attenuation", "signed"])
@pytest.mark.parametrize("name", ["dragon-strip", "soup", "corner", "tiled3-1024"])
def test_box_masks_exact(dragon, monkeypatch, name, model):
    """Box tile masks (BinBuffers::box_masks) forced on (XRT_BOX_MASKS=2) and
    off (0): a tile outside its region's mask stores its misses without reading
    the list.  Both frames -- image, L-buffer, u8, statistics -- are
    bit-identical to a brute-force render, in both models, over a row strip
    starting off the tile grid (row 13), odd frame sizes and a mesh of 206 K
    triangles."""
    tris, W, H, r0, r1 = _box_masks_case(name, dragon)
    cam = xrt.camera_for_mesh(tris, W, H)
    outs = {}
    for mode in ("2", "0", "brute"):
        monkeypatch.setenv("XRT_BOX_MASKS", "0" if mode == "brute" else mode)
        with xrt.Context(0) as c:
            if model == "signed":
                c.set_model(xrt.XRT_MODEL_SIGNED, 0.1037)
            c.set_kernel(xrt.XRT_KERNEL_BRUTE if mode == "brute" else xrt.XRT_KERNEL_BINNED)
            c.upload_mesh(tris)
            # the sizing frame, then a steady one (the signed model: whole frames)
            outs[mode] = [c.render_signed(cam) if model == "signed" else c.render_rows(cam, r0, r1) for _ in range(2)]
    for mode in ("2", "0"):
        for k in range(2):
            got, ref = outs[mode][k], outs["brute"][0]
            for x, y in zip(got[:3], ref[:3]):
                assert np.array_equal(bits(x), bits(y)), (mode, k)
            for f in ("rays", "hits", "hit_rays", "odd_rays", "max_hits"):
                assert getattr(got[3], f) == getattr(ref[3], f), (mode, k, f)


@pytest.mark.parametrize("case", ["dragon-strip", "planes-recount", "soup"])
def test_first_frame_device_sized_exact(dragon, case):
    """A geometry's first host-buffer frame is sized on the device (the count
    pass, one read-back of its pair total, k_size_lists / k_scatter_pairs, the
    device fill plan): equal to brute force bit for bit, statistics included --
    a strip starting off the region grid; planes each covering every region, so
    the first pool (6 pairs a triangle, at least 65,536) is too small and the
    pass counts again; a random soup.  The same camera again is sized on the host, a new
    one takes the moving path, every frame exact."""
    from scene_kit import plane_stack
    if case == "dragon-strip":
        tris, W, H, r0, r1 = dragon, 1000, 777, 13, 700
    elif case == "planes-recount":
        tris, W, H, r0, r1 = plane_stack(20, spacing=0.05), 2048, 2048, 0, None
    else:
        tris, W, H, r0, r1 = synthetic_soup(seed=5, n=4000), 400, 300, 0, None
    cam = xrt.camera_for_mesh(tris, W, H)
    if case == "planes-recount":
        cam.pixel_spacing *= 0.25          # the squares fill the frame: ~2,000 regions a triangle
    lo, hi = xrt.mesh_bbox(tris)
    centre = 0.5 * (np.asarray(lo, np.float64) + np.asarray(hi, np.float64))
    cams = [cam, cam, orbit_camera(cam, centre, 3.0)]
    with xrt.Context(0) as brute:
        brute.set_kernel(xrt.XRT_KERNEL_BRUTE)
        brute.upload_mesh(tris)
        refs = [brute.render_rows(c, r0, r1) for c in cams]
    with xrt.Context(0) as c:
        c.set_kernel(xrt.XRT_KERNEL_BINNED)
        c.upload_mesh(tris)
        paths = []
        for k, cm in enumerate(cams):
            g0, f0 = c.geometry_counters(), c.first_frames()
            got = c.render_rows(cm, r0, r1)
            g1, f1 = c.geometry_counters(), c.first_frames()
            if k == 0:
                ff = f1
            paths.append((f1["device_sized"] - f0["device_sized"], f1["recounted"] - f0["recounted"],
                          g1["sizings"] - g0["sizings"], g1["reused"] - g0["reused"]))
            for x, y in zip(got[:3], refs[k][:3]):
                assert np.array_equal(bits(x), bits(y)), (case, k)
            for f in ("rays", "hits", "hit_rays", "odd_rays", "max_hits"):
                assert getattr(got[3], f) == getattr(refs[k][3], f), (case, k, f)
    assert paths[0][0] == 1 and paths[0][2] == 0, paths       # device-sized, no host sizing
    assert paths[1][2] == 1 and paths[1][0] == 0, paths       # the same camera: sized on the host
    assert paths[2][3] == 1, paths                            # a new camera: the moving path
    if case == "planes-recount":
        assert paths[0][1] == 1, (paths, ff)


def test_contexts_share_device_streams_exact(dragon):
    """Contexts of one device share its prep and host streams (acquire_streams):
    two contexts interleaving frames in flight on two caller streams -- one
    camera still, the other moving -- then the first destroyed while the second
    keeps rendering and a third joins: every frame equals brute force."""
    import torch
    W, H = 512, 384
    lo, hi = xrt.mesh_bbox(dragon)
    centre = 0.5 * (np.asarray(lo, np.float64) + np.asarray(hi, np.float64))
    base = xrt.camera_for_mesh(dragon, W, H)
    cams = [orbit_camera(base, centre, 1.5 * k) for k in range(6)]
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    with xrt.Context(0) as brute:
        brute.set_kernel(xrt.XRT_KERNEL_BRUTE)
        brute.upload_mesh(dragon)
        ref_still = brute.render_rows(base)
        refs = [brute.render_rows(c) for c in cams]

    def make():
        c = xrt.Context(0)
        c.set_kernel(xrt.XRT_KERNEL_BINNED)
        c.upload_mesh(dragon)
        return c

    def planes():
        return (torch.empty(W * H, device=dev), torch.empty(W * H, device=dev),
                torch.empty(W * H, dtype=torch.uint8, device=dev))

    def check(out, ref, what):
        for x, y in zip(out, ref[:3]):
            assert np.array_equal(bits(x.cpu().numpy()), bits(y)), what

    a, b = make(), make()
    outs_a = [planes() for _ in cams]
    outs_b = [planes() for _ in cams]
    for k, cam in enumerate(cams):
        a.render_rows_device(base, 0, H, *(t.data_ptr() for t in outs_a[k]), streams[k % 2].cuda_stream)
        b.render_rows_device(cam, 0, H, *(t.data_ptr() for t in outs_b[k]), streams[(k + 1) % 2].cuda_stream)
    torch.cuda.synchronize(dev)
    for k in range(len(cams)):
        check(outs_a[k], ref_still, ("a", k))
        check(outs_b[k], refs[k], ("b", k))
    a.close()                                   # b keeps the device's streams
    c = make()
    for k, cam in enumerate(cams):
        b.render_rows_device(cam, 0, H, *(t.data_ptr() for t in outs_b[k]), streams[k % 2].cuda_stream)
        c.render_rows_device(base, 0, H, *(t.data_ptr() for t in outs_a[k]), streams[(k + 1) % 2].cuda_stream)
    torch.cuda.synchronize(dev)
    for k in range(len(cams)):
        check(outs_b[k], refs[k], ("b after a closed", k))
        check(outs_a[k], ref_still, ("c", k))
    for k in (0, 3):                            # host-buffer calls on the shared host stream
        got_b, got_c = b.render_rows(cams[k]), c.render_rows(base)
        for x, y in zip(got_b[:3], refs[k][:3]):
            assert np.array_equal(bits(x), bits(y)), ("b host", k)
        for x, y in zip(got_c[:3], ref_still[:3]):
            assert np.array_equal(bits(x), bits(y)), ("c host", k)
    b.close()
    c.close()


def test_box_masks_moving_camera_exact(dragon, monkeypatch):
    """Box tile masks forced on in a moving camera's device-sized frames (the
    count pass ORs the masks; the default leaves them off there): every frame of
    a sweep, through device planes on two streams, equals brute force."""
    import torch
    monkeypatch.setenv("XRT_BOX_MASKS", "2")
    W, H = 640, 480
    lo, hi = xrt.mesh_bbox(dragon)
    centre = 0.5 * (np.asarray(lo, np.float64) + np.asarray(hi, np.float64))
    base = xrt.camera_for_mesh(dragon, W, H)
    cams = [orbit_camera(base, centre, 0.75 * k) for k in range(8)]
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    with xrt.Context(0) as brute:
        brute.set_kernel(xrt.XRT_KERNEL_BRUTE)
        brute.upload_mesh(dragon)
        refs = [brute.render_rows(c) for c in cams]
    with xrt.Context(0) as c:
        c.set_kernel(xrt.XRT_KERNEL_BINNED)
        c.upload_mesh(dragon)
        outs = [(torch.empty(W * H, device=dev), torch.empty(W * H, device=dev),
                 torch.empty(W * H, dtype=torch.uint8, device=dev)) for _ in cams]
        for k, cam in enumerate(cams):
            c.render_rows_device(cam, 0, H, *(t.data_ptr() for t in outs[k]), streams[k % 2].cuda_stream)
        torch.cuda.synchronize(dev)
        for k in range(len(cams)):
            for x, y in zip(outs[k], refs[k][:3]):
                assert np.array_equal(bits(x.cpu().numpy()), bits(y)), k
        g = c.geometry_counters()
    assert g["reused"] >= 6, g


@pytest.mark.parametrize("devices", [[0, 0]])
def test_multi_strips_orbit_exact(dragon, devices):
    """xrt_render_rows_multi under a moving camera: its contexts size
    every camera for itself; each gathered frame of a sweep equals a fresh
    single-device brute-force render bit for bit."""
    W, H = 1000, 777
    lo, hi = xrt.mesh_bbox(dragon)
    centre = 0.5 * (np.asarray(lo, np.float64) + np.asarray(hi, np.float64))
    base = xrt.camera_for_mesh(dragon, W, H)
    with xrt.MultiContext(devices) as multi:
        multi.set_kernel(xrt.XRT_KERNEL_BINNED)
        multi.upload_mesh(dragon)
        for d in (0, 0.5, 1.0, 30, 30, 31):
            cam = orbit_camera(base, centre, d)
            got = multi.render(cam)
            with xrt.Context(0) as fresh:
                fresh.set_kernel(xrt.XRT_KERNEL_BRUTE)
                fresh.upload_mesh(dragon)
                ref = fresh.render_rows(cam)
            for x, y in zip(got[:3], ref[:3]):
                assert np.array_equal(bits(x), bits(y)), d


def test_global_list_and_fill_plan(ctx, dragon):
    """The global list (footprints reaching more than 4,096 regions) against the
    fill plan: dragon 4096^2 has edge-on slivers whose boxes span the frame but
    whose loosened triangles reach few regions -- binned, not global, so regions
    stay empty and the plan fills them; a genuinely big triangle goes global,
    no region is empty and no plan is used.  Binned == brute on the latter."""
    render(ctx, dragon, 4096, 4096, xrt.XRT_KERNEL_BINNED, 0, 64)       # (the first frame: device-sized)
    st = ctx.render_rows(xrt.camera_for_mesh(dragon, 4096, 4096), 0, 64)[3]
    assert st.global_triangles == 0 and ctx.fill_regions() > 0
    W = H = 2112                                           # 66 x 66 = 4,356 regions
    cam = xrt.camera_for_mesh(dragon, W, H)
    o, d = np.array(cam.origin, np.float64), np.array(cam.detector, np.float64)
    up, right = np.array(cam.up, np.float64), np.array(cam.right, np.float64)
    c = o + 0.95 * (d - o)                                 # a triangle across the whole view, behind the dragon
    span = 4.0 * cam.pixel_spacing * W
    big = np.array([np.concatenate([c - span * up - span * right, c - span * up + 2 * span * right,
                                    c + 2 * span * up - span * right])], np.float32)
    scene = np.ascontiguousarray(np.concatenate([dragon, big]))
    a = render(ctx, scene, W, H, xrt.XRT_KERNEL_BINNED, cam=cam)
    assert a[3].global_triangles >= 1 and ctx.fill_regions() == 0
    assert a[3].hit_rays == W * H                          # every ray meets the big triangle
    b = render(ctx, scene, W, H, xrt.XRT_KERNEL_BRUTE, cam=cam)
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(bits(x), bits(y))
    assert (a[3].hit_rays, a[3].odd_rays, a[3].max_hits) == (b[3].hit_rays, b[3].odd_rays, b[3].max_hits)


def test_fill_plan_rejected_when_k_prep_bins_into_it(ctx, dragon):
    """Test hook 2 plans every region as empty.  k_prep then bins pairs into
    planned-empty regions and flags it, and the host launches that frame with
    every region rendered as tiles (no region is filled) -- exact against the
    oracle and the plan-free render."""
    W, H = 160, 96
    cam = oracle.camera_for_mesh(dragon, W, H)
    ref = oracle.render_rows(dragon, cam, W, H)
    ctx.set_fill_plan(2)
    try:
        got = render(ctx, dragon, W, H, xrt.XRT_KERNEL_BINNED)
        assert ctx.fill_regions() == 0
        assert_same(got, ref, "rejected plan")
        big = render(ctx, dragon, 1024, 1024, xrt.XRT_KERNEL_BINNED)
        assert ctx.fill_regions() == 0
    finally:
        ctx.set_fill_plan(1)
    plain = render(ctx, dragon, 1024, 1024, xrt.XRT_KERNEL_BINNED)
    for x, y in zip(big[:3], plain[:3]):
        assert np.array_equal(bits(x), bits(y))
    assert _stats(big[3]) == _stats(plain[3])


@pytest.mark.parametrize("kernel", [xrt.XRT_KERNEL_TILED, xrt.XRT_KERNEL_BINNED])
def test_culled_4096_rows_vs_oracle(ctx, dragon, kernel):
    W = H = 4096
    img, lb, u8, st = render(ctx, dragon, W, H, kernel)
    rows = [0, 511, 512, 2048, 3584, 4095]
    cam = oracle.camera_for_mesh(dragon, W, H)
    ref = oracle.render_row_list(dragon, cam, W, H, rows)
    assert np.array_equal(bits(img.reshape(H, W)[rows].ravel()), bits(ref[0]))
    assert np.array_equal(bits(lb.reshape(H, W)[rows].ravel()), bits(ref[1]))
    assert np.array_equal(u8.reshape(H, W)[rows].ravel(), ref[2])


def test_binned_equals_brute_full_4096(ctx, dragon):
    """The whole 4096^2 frame (BASELINE configs[3]'s): the binned render equals the
    literal brute-force render bit for bit on every pixel and statistic (about a
    quarter second of brute force)."""
    W = H = 4096
    a = render(ctx, dragon, W, H, xrt.XRT_KERNEL_BINNED)
    b = render(ctx, dragon, W, H, xrt.XRT_KERNEL_BRUTE)
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(bits(x), bits(y))
    for f in ("rays", "hit_rays", "odd_rays", "hits", "max_hits", "overflow_rays"):
        assert getattr(a[3], f) == getattr(b[3], f), f


def _setters():
    """Every setter that starts a new settings generation (frames prepared ahead
    become stale), with a value that changes nothing in the attenuation render's
    output and one that restores the default: (name, apply, restore)."""
    return [
        ("kernel", lambda c: c.set_kernel(xrt.XRT_KERNEL_TILED), lambda c: c.set_kernel(xrt.XRT_KERNEL_BINNED)),
        ("hit_capacity", lambda c: c.set_hit_capacity(2), lambda c: c.set_hit_capacity(0)),
        ("bin_capacity", lambda c: c.set_bin_capacity(16), lambda c: c.set_bin_capacity(0)),
        ("fill_plan", lambda c: c.set_fill_plan(0), lambda c: c.set_fill_plan(1)),
        ("model", lambda c: c.set_model(xrt.XRT_MODEL_ATTENUATION, 0.5),
         lambda c: c.set_model(xrt.XRT_MODEL_ATTENUATION, 0.1037)),
    ]


@pytest.mark.parametrize("name", [s[0] for s in _setters()])
def test_setter_toggles_keep_frames_exact(dragon, name):
    """the binning of a geometry is trusted across frames (its
    k_prep check is armed on the first frame over a plan only), so a setting
    changed and restored between frames of ONE geometry must not leave a stale
    plan or list behind: every frame -- before, under and after the setting,
    device-pointer frames prepared ahead included -- equals a fresh brute-force
    render bit for bit."""
    import torch
    apply, restore = [(a, r) for n, a, r in _setters() if n == name][0]
    W, H = 640, 512
    cam = xrt.camera_for_mesh(dragon, W, H)
    with xrt.Context(0) as fresh:
        fresh.set_kernel(xrt.XRT_KERNEL_BRUTE)
        fresh.upload_mesh(dragon)
        ref = fresh.render_rows(cam)
    dev = torch.device("cuda", 0)
    planes = [torch.empty(W * H, dtype=torch.float32, device=dev), torch.empty(W * H, dtype=torch.float32, device=dev),
              torch.empty(W * H, dtype=torch.uint8, device=dev)]
    with xrt.Context(0) as c:
        c.set_kernel(xrt.XRT_KERNEL_BINNED)
        c.upload_mesh(dragon)
        for phase in ("before", "applied", "restored"):
            if phase == "applied":
                apply(c)
            elif phase == "restored":
                restore(c)
            for i in range(4):
                if i % 2:
                    got = c.render_rows(cam)[:3]
                else:
                    for _ in range(3):           # repeated geometry: frames prepared ahead
                        c.render_rows_device(cam, 0, H, *(t.data_ptr() for t in planes), 0)
                    torch.cuda.synchronize(dev)
                    got = [t.cpu().numpy() for t in planes]
                for x, y in zip(got, ref[:3]):
                    assert np.array_equal(bits(x), bits(y)), (name, phase, i)


def test_two_timed_regions_keep_their_spans(ctx, dragon):
    """a timed region's frames keep their timing records in device
    chunks of 64 frames; a second region on the same context reuses the first
    region's chunks.  Each region's mean span (xrt_timing_end) agrees with its
    own HIP-event samples and with the last frame's span read afterwards, so no
    region sums another's (or unwritten) records."""
    import torch
    W = H = 1024
    cam = xrt.camera_for_mesh(dragon, W, H)
    ctx.set_kernel(xrt.XRT_KERNEL_BINNED)
    ctx.upload_mesh(dragon)
    dev = torch.device("cuda", 0)
    planes = [torch.empty(W * H, dtype=torch.float32, device=dev), torch.empty(W * H, dtype=torch.float32, device=dev),
              torch.empty(W * H, dtype=torch.uint8, device=dev)]
    means = []
    for region in range(3):
        n = 150 if region < 2 else 20
        ctx.timing_begin()
        for _ in range(n):
            ctx.render_rows_device(cam, 0, H, *(t.data_ptr() for t in planes), 0)
        ms, launches = ctx.timing_end()
        ev_ms, ev_launches = ctx.timing_events()
        assert launches == n and ev_launches == -(-n // 16)
        mean, ev_mean = ms / launches, ev_ms / ev_launches
        # spans are the kernels' own execution; events add a launch and a write-back
        assert 0.3 * ev_mean < mean < 1.2 * ev_mean, (region, mean, ev_mean)
        last = ctx.read_stats().kernel_ms                 # the region's last frame, read after it
        assert 0.3 * mean < last < 3.0 * mean, (region, last, mean)
        means.append(mean)
    assert max(means[:2]) < 1.5 * min(means[:2]), means


@pytest.mark.parametrize("split_min,W,H,r0,r1,cap", [(1, 2048, 2048, 0, None, 0), (1, 1000, 700, 100, 650, 0),
                                                    (1, 512, 512, 0, None, 2), (1, 512, 512, 0, None, 5),
                                                    (64, 1024, 1024, 0, None, 0), (0, 1024, 1024, 0, None, 0)])
def test_split_tiles_exact(dragon, monkeypatch, split_min, W, H, r0, r1, cap):
    """Split tiles (DESIGN.md "Split tiles"): the plan's heaviest regions render
    each tile with two waves that test alternate survivors, and half 0 merges
    half 1's sorted hit list into its own.  XRT_SPLIT_MIN=1 splits every
    non-empty region; with the hit list capped at 2 or 5 entries the merged
    counts pass the cap and take the exact fix-up.  Every frame (the sizing
    frame and a later one) equals the brute-force render bit for bit, with the
    same statistics."""
    monkeypatch.setenv("XRT_SPLIT_MIN", str(split_min))
    cam = xrt.camera_for_mesh(dragon, W, H)
    with xrt.Context(0) as b:
        b.set_kernel(xrt.XRT_KERNEL_BRUTE)
        b.upload_mesh(dragon)
        if cap:
            b.set_hit_capacity(cap)
        ref = b.render_rows(cam, r0, r1)
    with xrt.Context(0) as c:
        c.set_kernel(xrt.XRT_KERNEL_BINNED)
        c.upload_mesh(dragon)
        if cap:
            c.set_hit_capacity(cap)
        for frame in range(2):
            got = c.render_rows(cam, r0, r1)
            for x, y in zip(got[:3], ref[:3]):
                assert np.array_equal(bits(x), bits(y)), (split_min, frame)
            for f in ("rays", "hit_rays", "odd_rays", "hits", "max_hits", "overflow_rays"):
                assert getattr(got[3], f) == getattr(ref[3], f), (split_min, frame, f)
    if cap:
        assert ref[3].overflow_rays > 0


def test_tiled_mesh_1m_parity(ctx, dragon):
    """1,120,434-triangle tiled dragon: tiled == brute at 256^2, rows vs oracle."""
    big = tiled_mesh(dragon, 7)
    assert big.shape == (1120434, 9)
    W = H = 256
    a = render(ctx, big, W, H, xrt.XRT_KERNEL_BINNED)
    for k in (xrt.XRT_KERNEL_TILED, xrt.XRT_KERNEL_BRUTE):
        b = render(ctx, big, W, H, k)
        for x, y in zip(a[:3], b[:3]):
            assert np.array_equal(bits(x), bits(y)), KNAME[k]
    rows = [37, 128]
    cam = oracle.camera_for_mesh(big, W, H)
    ref = oracle.render_row_list(big, cam, W, H, rows)
    assert np.array_equal(bits(a[0].reshape(H, W)[rows].ravel()), bits(ref[0]))
    assert a[3].max_hits <= 16


def test_device_buffers_and_timing(ctx, dragon):
    """xrt_render_rows_device on torch-allocated device memory and a torch stream."""
    import torch
    W = H = 192
    cam = xrt.camera_for_mesh(dragon, W, H)
    ctx.set_kernel(xrt.XRT_KERNEL_TILED)
    ctx.upload_mesh(dragon)
    dev = torch.device("cuda", ctx.device)
    img = torch.empty(W * H, dtype=torch.float32, device=dev)
    lb = torch.empty(W * H, dtype=torch.float32, device=dev)
    u8 = torch.empty(W * H, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)
    ctx.timing_begin()
    with torch.cuda.stream(stream):
        for _ in range(8):
            ctx.render_rows_device(cam, 0, H, img.data_ptr(), lb.data_ptr(), u8.data_ptr(),
                                   stream.cuda_stream)
    ms, launches = ctx.timing_end()
    st = ctx.read_stats()
    assert launches == 8 and ms > 0            # every frame's in-kernel span
    ev_ms, ev_launches = ctx.timing_events()
    assert ev_launches == 1 and ev_ms > 0      # HIP events on every 16th dispatch
    ref = ctx.render_rows(cam)
    assert np.array_equal(bits(img.cpu().numpy()), bits(ref[0]))
    assert np.array_equal(u8.cpu().numpy(), ref[2])
    assert st.rays == W * H


@pytest.mark.parametrize("W,H,r0,r1,kernel", [(512, 512, 0, 512, xrt.XRT_KERNEL_BINNED),
                                               (1000, 777, 100, 700, xrt.XRT_KERNEL_BINNED),
                                               (192, 192, 0, 192, xrt.XRT_KERNEL_TILED)])
def test_prepared_ahead_frames_exact(dragon, W, H, r0, r1, kernel):
    """Prepare-ahead (DESIGN.md "Pipelining"): device-pointer frames that repeat
    their geometry are rendered from preparations enqueued during earlier calls;
    a change of camera, of a setting (hit capacity, miss code) or a host-buffer
    call in between drops them.  Every frame of the sequence -- each into its
    own planes, no host sync until the end -- is bit-identical to a fresh
    brute-force render of its camera, and the pipeline counters show frames
    taken from ahead, dropped preparations and renders launched with no wait."""
    import torch
    lo, hi = xrt.mesh_bbox(dragon)
    centre = 0.5 * (np.asarray(lo, np.float64) + np.asarray(hi, np.float64))
    base = xrt.camera_for_mesh(dragon, W, H)
    cams = {"A": base, "B": orbit_camera(base, centre, 40.0)}
    refs = {}
    for name, cam in cams.items():
        with xrt.Context(0) as fresh:
            fresh.set_kernel(xrt.XRT_KERNEL_BRUTE)
            fresh.upload_mesh(dragon)
            refs[name] = fresh.render_rows(cam, r0, r1)
    seq = "AAAAAA" + "BBBBB" + "h" + "BBBB" + "x" + "BBBB" + "AAAAAAAA"
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    n = (r1 - r0) * W
    outs = []
    with xrt.Context(0) as ctx:
        ctx.set_kernel(kernel)
        ctx.upload_mesh(dragon)
        with torch.cuda.stream(stream):
            for step in seq:
                if step == "h":                       # a setting change between device frames
                    ctx.set_hit_capacity(5)
                    continue
                if step == "x":                       # a host-buffer render in between
                    got = ctx.render_rows(cams["B"], r0, r1)
                    assert np.array_equal(bits(got[1]), bits(refs["B"][1]))
                    continue
                planes = (torch.empty(n, dtype=torch.float32, device=dev),
                          torch.empty(n, dtype=torch.float32, device=dev),
                          torch.empty(n, dtype=torch.uint8, device=dev))
                ctx.render_rows_device(cams[step], r0, r1, planes[0].data_ptr(), planes[1].data_ptr(),
                                       planes[2].data_ptr(), stream.cuda_stream)
                outs.append((step, planes))
        stream.synchronize()
        pc = ctx.pipeline_counters()
        st = ctx.read_stats()
    for i, (step, planes) in enumerate(outs):
        ref = refs[step]
        for x, y in zip(planes, ref[:3]):
            assert np.array_equal(bits(x.cpu().numpy()), bits(y)), (i, step)
    assert st.hit_rays == refs["A"][3].hit_rays and st.odd_rays == refs["A"][3].odd_rays
    assert pc["ahead_used"] >= 8 and pc["ahead_dropped"] >= 4, pc
    # whether a frame's preparation is complete at its launch is a race with the
    # host; at 192^2 (TILED) the host can outrun every one of them
    assert pc["no_wait"] > 0 or kernel == xrt.XRT_KERNEL_TILED, pc


@pytest.mark.parametrize("n_streams", [2, 3])
def test_frames_in_flight_on_streams_exact(dragon, n_streams):
    """Frames in flight (bench.py --inflight): frame k renders on stream
    k % n_streams into its own planes, so renders of consecutive frames overlap
    on the device, over steady runs (prepared ahead) and camera changes; every
    frame is bit-identical to a brute-force render of its camera."""
    import torch
    W = H = 512
    lo, hi = xrt.mesh_bbox(dragon)
    centre = 0.5 * (np.asarray(lo, np.float64) + np.asarray(hi, np.float64))
    base = xrt.camera_for_mesh(dragon, W, H)
    cams = {"A": base, "B": orbit_camera(base, centre, 25.0)}
    refs = {}
    for name, cam in cams.items():
        with xrt.Context(0) as fresh:
            fresh.set_kernel(xrt.XRT_KERNEL_BRUTE)
            fresh.upload_mesh(dragon)
            refs[name] = fresh.render_rows(cam)
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(device=dev) for _ in range(n_streams)]
    seq = "A" * 12 + "B" * 9 + "A" * 7
    outs = [(name, (torch.full((W * H,), -1.0, device=dev), torch.full((W * H,), -1.0, device=dev),
                    torch.zeros(W * H, dtype=torch.uint8, device=dev))) for name in seq]
    with xrt.Context(0) as ctx:
        ctx.set_kernel(xrt.XRT_KERNEL_BINNED)
        ctx.upload_mesh(dragon)
        torch.cuda.synchronize(dev)               # the planes' fills, before other streams write them
        for k, (name, planes) in enumerate(outs):  # no host sync between frames
            ctx.render_rows_device(cams[name], 0, H, *(t.data_ptr() for t in planes),
                                   streams[k % n_streams].cuda_stream)
        torch.cuda.synchronize(dev)
        pc = ctx.pipeline_counters()
    for k, (name, planes) in enumerate(outs):
        for x, y in zip(planes, refs[name][:3]):
            assert np.array_equal(bits(x.cpu().numpy()), bits(y)), (k, name)
    assert pc["ahead_used"] >= 10, pc


def test_pipelined_frames_without_sync(ctx, dragon):
    """Many frames enqueued back to back on one stream with no host sync --
    different cameras, image sizes, strips, kernels and output buffers, so the
    two alternating buffer sets and the prep stream are exercised under
    overlap -- each equal to its own synchronous render."""
    import torch
    dev = torch.device("cuda", ctx.device)
    stream = torch.cuda.Stream(device=dev)
    ctx.upload_mesh(dragon)
    jobs = [(256, 256, 0, 256, xrt.XRT_KERNEL_BINNED), (200, 120, 0, 120, xrt.XRT_KERNEL_BINNED),
            (256, 256, 64, 200, xrt.XRT_KERNEL_BINNED), (160, 160, 0, 160, xrt.XRT_KERNEL_TILED),
            (300, 300, 0, 300, xrt.XRT_KERNEL_BINNED), (256, 256, 0, 256, xrt.XRT_KERNEL_AUTO),
            (96, 320, 10, 300, xrt.XRT_KERNEL_BINNED), (256, 256, 0, 256, xrt.XRT_KERNEL_BINNED)] * 2
    cams = {}
    for W, H, *_ in jobs:                  # first frame of each geometry sizes its lists (sync)
        cams[(W, H)] = xrt.camera_for_mesh(dragon, W, H)
    refs = []
    for W, H, r0, r1, k in jobs:
        ctx.set_kernel(k)
        refs.append(ctx.render_rows(cams[(W, H)], r0, r1))
    outs = []
    with torch.cuda.stream(stream):
        for W, H, r0, r1, k in jobs:
            n = (r1 - r0) * W
            bufs = (torch.full((n,), -1.0, device=dev), torch.full((n,), -1.0, device=dev),
                    torch.zeros(n, dtype=torch.uint8, device=dev))
            ctx.set_kernel(k)
            ctx.render_rows_device(cams[(W, H)], r0, r1, bufs[0].data_ptr(), bufs[1].data_ptr(),
                                   bufs[2].data_ptr(), stream.cuda_stream)
            outs.append(bufs)
    stream.synchronize()
    for (img, lb, u8), ref, job in zip(outs, refs, jobs):
        assert np.array_equal(bits(img.cpu().numpy()), bits(ref[0])), job
        assert np.array_equal(bits(lb.cpu().numpy()), bits(ref[1])), job
        assert np.array_equal(u8.cpu().numpy(), ref[2]), job


def test_cli_golden_text(tmp_path):
    """xrt_main (the reference's CLI over the GPU path) writes the golden text."""
    exe = os.path.join(ROOT, "simpleraytracing_amd", "lib", "xrt_main")
    (tmp_path / "out").mkdir()
    for kernel in ("brute", "tiled", "binned"):
        r = subprocess.run([exe, "-s", "128", "128", "-i", DRAGON, "-f", f"d-{kernel}.txt", "-k", kernel],
                           capture_output=True, text=True, cwd=tmp_path, timeout=300)
        assert r.returncode == 0, r.stderr
        got = (tmp_path / "out" / f"d-{kernel}.txt").read_bytes()
        assert got == open(os.path.join(GOLDEN, "dragon-128x128-serial.txt"), "rb").read()


def test_cli_odd_ray_messages(tmp_path):
    """The reference prints one line per odd-count ray (main.cxx:710): 24 at 2048^2."""
    exe = os.path.join(ROOT, "simpleraytracing_amd", "lib", "xrt_main")
    (tmp_path / "out").mkdir()
    r = subprocess.run([exe, "-s", "2048", "2048", "-i", DRAGON, "-f", "d.txt"], capture_output=True,
                       text=True, cwd=tmp_path, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("Only one intersect on this ray") == 24


@pytest.mark.parametrize("W,rows", [(256, list(range(256))), (2048, [0, 700, 1024, 1025, 1400, 2047])])
def test_footprints_contain_every_hit(ctx, dragon, W, rows):
    """Direct check of the tile cull's conservativeness: every (pixel, triangle)
    pair the reference's Ray::intersect reports (t > 1e-7) lies inside that
    triangle's footprint box and satisfies its three relaxed edge functions."""
    H = W
    cam = xrt.camera_for_mesh(dragon, W, H)
    ctx.upload_mesh(dragon)
    _, fp = ctx.probe_prep(cam, len(dragon))
    px, tri = oracle.hit_pairs(dragon, cam13(cam), W, H, rows)
    assert len(px) > 0
    row = np.asarray(rows, np.float32)[px // W]
    col = (px % W).astype(np.float32)
    f = fp[tri]
    assert np.all((f[:, 0] <= col) & (col <= f[:, 1]) & (f[:, 2] <= row) & (row <= f[:, 3]))
    for k in range(3):
        a, b, c = f[:, 4 + 4 * k], f[:, 5 + 4 * k], f[:, 6 + 4 * k]
        assert np.all(a * col + b * row + c >= 0), k
    # the footprints are tight: median box no wider than the triangle's projection + 2 px
    w = fp[:, 1] - fp[:, 0]
    assert np.median(w[np.isfinite(w)]) < W / 16


@pytest.mark.parametrize("devices,W,H", [([0], 160, 131), ([0, 0], 160, 131), ([0, 0, 0], 160, 131),
                                          ([0, 0], 1000, 777), ([0, 0, 0], 1000, 777)])
def test_multi_strips_equal_single_frame(dragon, devices, W, H):
    """xrt_render_rows_multi: row strips (rows_per = H/n, remainder first) on the
    listed devices, gathered into device 0's frame as packed regions (the strips'
    fill plans leave their empty regions behind; 1000 x 777 has many) -- bit-equal
    to one device's frame and to the oracle.  One GPU here: a device listed twice
    runs the strip, packing and double-buffer logic with the device-copy gather
    (the RCCL gather needs distinct devices; the 8-GPU node runs it)."""
    # 131 = 3 * 43 + 2: uneven strips
    cam = xrt.camera_for_mesh(dragon, W, H)
    with xrt.Context(0) as one:
        one.set_kernel(xrt.XRT_KERNEL_BINNED)
        one.upload_mesh(dragon)
        ref = one.render_rows(cam)
    with xrt.MultiContext(devices) as m:
        m.set_kernel(xrt.XRT_KERNEL_BINNED)
        m.upload_mesh(dragon)
        for _ in range(3):                              # the strip buffers rotate
            got = m.render(cam)
            for x, y in zip(got[:3], ref[:3]):
                assert np.array_equal(bits(x), bits(y))
            assert got[3].odd_rays == ref[3].odd_rays and got[3].hit_rays == ref[3].hit_rays
    if W * H <= 160 * 131:
        o = oracle.render_rows(dragon, oracle.camera_for_mesh(dragon, W, H), W, H)
        assert np.array_equal(bits(got[0]), bits(o[0]))


@pytest.mark.parametrize("devices,W,H", [([0, 0], 160, 131), ([0, 0, 0], 1000, 777)])
def test_multi_rccl_gather_one_rank(dragon, devices, W, H):
    """The RCCL gather itself on one GPU: XRT_GATHER_RCCL over one device listed
    n times builds a one-rank communicator (ncclCommInitAll) and moves every
    strip with the grouped ncclSend / ncclRecv of the distinct-device gather
    (the rank sends to itself).  Packed regions at 1000 x 777; bit-equal to one
    device's frame, frames in rotation, then back to the copy gather."""
    cam = xrt.camera_for_mesh(dragon, W, H)
    with xrt.Context(0) as one:
        one.set_kernel(xrt.XRT_KERNEL_BINNED)
        one.upload_mesh(dragon)
        ref = one.render_rows(cam)
    with xrt.MultiContext(devices) as m:
        m.set_kernel(xrt.XRT_KERNEL_BINNED)
        m.upload_mesh(dragon)
        for mode in (xrt.XRT_GATHER_RCCL, xrt.XRT_GATHER_COPY, xrt.XRT_GATHER_RCCL):
            m.set_gather(mode)
            for _ in range(3):                          # the strip buffers rotate
                got = m.render(cam)
                for x, y in zip(got[:3], ref[:3]):
                    assert np.array_equal(bits(x), bits(y))


def test_multi_hit_transit_empty_strips(dragon):
    """xrt_render_rows_multi over 8 equal strips with the camera zoomed out, so
    the top strips' regions are all filled by their plans (no tile of theirs
    travels): the hit frames equal one device's frame bit for bit."""
    W = H = 1024
    cam = xrt.camera_for_mesh(dragon, W, H)
    cam.pixel_spacing *= 3.0
    with xrt.Context(0) as one:
        one.set_kernel(xrt.XRT_KERNEL_BINNED)
        one.upload_mesh(dragon)
        ref = one.render_rows(cam)
    with xrt.MultiContext([0] * 8) as m:
        m.set_kernel(xrt.XRT_KERNEL_BINNED)
        m.upload_mesh(dragon)
        m.set_gather(xrt.XRT_GATHER_RCCL)
        m.set_split(xrt.XRT_SPLIT_EQUAL)
        for _ in range(3):                                     # packed, then hits
            got = m.render(cam)
            for x, y in zip(got[:3], ref[:3]):
                assert np.array_equal(bits(x), bits(y))
        st = m.transit_stats()
        assert st["frames_packed"] == 1 and st["frames_hits"] == 2 and st["bad"] == 0, st


@pytest.mark.parametrize("gather", ["rccl", "copy"])
def test_multi_hit_transit(dragon, gather):
    """xrt_render_rows_multi's hit transit (XRT_TRANSIT_HITS, the default): a
    new geometry's frame travels packed, its repeats in the hit layout (the
    senders' plans made once); in an alternation of two cameras the planned
    one travels as hits, the other packed; XRT_TRANSIT_PACKED keeps the
    blocks.  Every frame bit-equal to one device's frame; the hit frames move
    fewer bytes; no mask disagrees."""
    W, H, n = 1024, 1024, 4
    cams = [xrt.camera_for_mesh(dragon, W, H), xrt.camera_from_bbox(*oracle.bbox(dragon[:5000]), W, H)]
    with xrt.Context(0) as one:
        one.set_kernel(xrt.XRT_KERNEL_BINNED)
        one.upload_mesh(dragon)
        refs = [one.render_rows(c) for c in cams]
    with xrt.MultiContext([0] * n) as m:
        m.set_kernel(xrt.XRT_KERNEL_BINNED)
        m.upload_mesh(dragon)
        m.set_gather(xrt.XRT_GATHER_RCCL if gather == "rccl" else xrt.XRT_GATHER_COPY)
        m.set_split(xrt.XRT_SPLIT_EQUAL)

        def check(k):
            got = m.render(cams[k])
            for x, y in zip(got[:3], refs[k][:3]):
                assert np.array_equal(bits(x), bits(y))

        check(0)
        packed_bytes = m.transit_stats()["last_bytes"]
        for _ in range(3):
            check(0)
        st = m.transit_stats()
        assert st["frames_packed"] == 1 and st["frames_hits"] == 3 and st["bad"] == 0, st
        assert 0 < st["last_bytes"] < 0.75 * packed_bytes, (st, packed_bytes)
        for k in (1, 0, 1, 0):                                 # camera 0 keeps its plan
            check(k)
        st = m.transit_stats()
        assert st["frames_packed"] == 3 and st["frames_hits"] == 5, st
        check(0)
        assert m.transit_stats()["frames_hits"] == 6
        m.set_transit(xrt.XRT_TRANSIT_PACKED)
        for _ in range(2):
            check(0)
        st = m.transit_stats()
        assert st["frames_hits"] == 6 and st["frames_packed"] == 5 and st["bad"] == 0, st
        assert st["last_bytes"] == packed_bytes


@pytest.mark.parametrize("W,H,n,link", [(4096, 4096, 8, 0.0), (1000, 777, 3, 3.0e4), (512, 512, 4, 1.0e3)])
def test_multi_balanced_split_rccl_one_rank(dragon, W, H, n, link):
    """xrt_render_rows_multi with the balanced split (the default): one GPU listed
    n times, gathered through a one-rank RCCL communicator -- 4096^2 in 8
    strips is BASELINE configs[3]'s split.  The first frame splits equally
    (the reference's rule; no model yet, no extra render, no link probe) and
    models the split from its strips' own records; the next frame plans the
    balanced split from them.  The strips are band-aligned, cover the frame,
    device 0's run may sit anywhere; every frame is bit-equal to one device's
    frame; the equal split still gives the reference's strips."""
    from simpleraytracing_amd.strips import strip_bounds
    cam = xrt.camera_for_mesh(dragon, W, H)
    equal = [strip_bounds(H, n, g) for g in range(n)]
    with xrt.Context(0) as one:
        one.set_kernel(xrt.XRT_KERNEL_BINNED)
        one.upload_mesh(dragon)
        ref = one.render_rows(cam)
    with xrt.MultiContext([0] * n) as m:
        m.set_kernel(xrt.XRT_KERNEL_BINNED)
        m.upload_mesh(dragon)
        m.set_gather(xrt.XRT_GATHER_RCCL)
        m.set_split(xrt.XRT_SPLIT_BALANCED, link)
        bounds, info = m.plan(cam)
        assert bounds == equal and info["predicted_step_us"] == 0.0       # no model before a frame
        got = m.render(cam)
        for x, y in zip(got[:3], ref[:3]):
            assert np.array_equal(bits(x), bits(y))
        st = m.plan_stats()
        assert st["plans"] == 0 and st["link_probes"] == 0 and st["models"] == 0 and st["equal_no_model"] >= 1, st
        bounds, info = m.plan(cam)
        assert len(bounds) == n and all(e > b for b, e in bounds)
        spans = sorted(bounds)
        assert spans[0][0] == 0 and spans[-1][1] == H and all(b % 32 == 0 for b, _ in spans)
        assert all(spans[i][1] == spans[i + 1][0] for i in range(n - 1))
        assert [b for b, _ in bounds[1:]] == sorted(b for b, _ in bounds[1:])     # senders in frame order
        assert info["frame_span_us"] > 0 and info["predicted_step_us"] > 0
        assert info["link_bytes_per_us"] == link if link else info["link_bytes_per_us"] > 0
        assert m.plan(cam)[0] == bounds                        # planned once per camera
        for _ in range(3):                                     # the strip buffers rotate
            got = m.render(cam)
            for x, y in zip(got[:3], ref[:3]):
                assert np.array_equal(bits(x), bits(y))
            assert got[3].hit_rays == ref[3].hit_rays and got[3].odd_rays == ref[3].odd_rays
        st = m.plan_stats()
        assert st["plans"] == 1 and st["models"] == 1 and st["link_probes"] == (0 if link else 1), st
        m.set_split(xrt.XRT_SPLIT_EQUAL)
        assert m.plan(cam)[0] == equal
        got = m.render(cam)
        for x, y in zip(got[:3], ref[:3]):
            assert np.array_equal(bits(x), bits(y))


def test_multi_orbit_balanced_rccl_one_rank(dragon):
    """An 8-frame orbit (1 degree a frame) through xrt_render_rows_multi on one
    device listed 8 times with RCCL, balanced split: the first frame splits
    equally, every later frame plans from an earlier frame's strip records
    (no whole-frame model render: no extra renders at all), the link is probed
    once, and every frame equals one device's render of its camera."""
    from simpleraytracing_amd.scenes import orbit_camera
    W = H = 1024
    cam0 = xrt.camera_for_mesh(dragon, W, H)
    lo, hi = xrt.mesh_bbox(dragon)
    centre = 0.5 * (np.asarray(lo, np.float64) + np.asarray(hi, np.float64))
    cams = [orbit_camera(cam0, centre, k * 1.0) for k in range(8)]
    with xrt.Context(0) as one:
        one.set_kernel(xrt.XRT_KERNEL_BINNED)
        one.upload_mesh(dragon)
        refs = [one.render_rows(c) for c in cams]
    with xrt.MultiContext([0] * 8) as m:
        m.set_kernel(xrt.XRT_KERNEL_BINNED)
        m.upload_mesh(dragon)
        m.set_gather(xrt.XRT_GATHER_RCCL)
        for k, c in enumerate(cams):
            got = m.render(c)
            for x, y in zip(got[:3], refs[k][:3]):
                assert np.array_equal(bits(x), bits(y)), k
        st = m.plan_stats()
    # (frame k's model is taken by frame k + 1's plan: the last one is still pending)
    assert st["equal_no_model"] == 1 and st["plans"] == 7 and st["link_probes"] == 1 and st["models"] == 7, st


def test_multi_hit_mismatch_reported_and_replanned(dragon):
    """A received hit mask that disagrees with its sender's plan (test hook: the
    plan's expected count of one tile off by one) fails that frame's call with
    XRT_ERR_DEVICE and drops the hit plans; the next frames travel packed,
    then plan again, each bit-equal to one device's frame."""
    W, H, n = 1024, 1024, 4
    cam = xrt.camera_for_mesh(dragon, W, H)
    with xrt.Context(0) as one:
        one.set_kernel(xrt.XRT_KERNEL_BINNED)
        one.upload_mesh(dragon)
        ref = one.render_rows(cam)
    with xrt.MultiContext([0] * n) as m:
        m.set_kernel(xrt.XRT_KERNEL_BINNED)
        m.upload_mesh(dragon)
        m.set_gather(xrt.XRT_GATHER_RCCL)
        m.set_split(xrt.XRT_SPLIT_EQUAL)
        for _ in range(3):                                     # packed, then hits
            m.render(cam)
        assert m.transit_stats()["frames_hits"] == 2
        m.corrupt_hit_plan()
        with pytest.raises(xrt.XrtError) as e:
            m.render(cam)
        assert e.value.code == 2 and "hit mask" in str(e.value)
        before = m.transit_stats()
        for _ in range(3):                                     # packed (plans dropped), then hits again
            got = m.render(cam)
            for x, y in zip(got[:3], ref[:3]):
                assert np.array_equal(bits(x), bits(y))
        st = m.transit_stats()
        assert st["frames_packed"] == before["frames_packed"] + 1 and st["frames_hits"] == before["frames_hits"] + 2
        assert st["bad"] == 0, st


def test_fresh_context_after_two_stream_loop(dragon):
    """Round 4 saw a fresh context's first host-buffer render wait 13.6-22.7 ms
    (in its layout upload's synchronisations) right after a frames-in-flight
    loop on two streams.  Here, run once, the same sequence: 400 frames of
    2048^2 alternating two streams and two plane sets, then a new context's first
    xrt_render_rows (list sizing included) -- enqueued within 3 ms, its
    synchronisations short, and its planes equal to the loop's frames."""
    import torch
    W = H = 2048
    dev = torch.device("cuda", 0)
    cam = xrt.camera_for_mesh(dragon, W, H)
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    sets = [(torch.empty(W * H, device=dev), torch.empty(W * H, device=dev),
             torch.empty(W * H, dtype=torch.uint8, device=dev)) for _ in streams]
    with xrt.Context(0) as c:
        c.upload_mesh(dragon)
        for k in range(400):
            img, lb, u8 = sets[k % 2]
            c.render_rows_device(cam, 0, H, img.data_ptr(), lb.data_ptr(), u8.data_ptr(), streams[k % 2].cuda_stream)
        torch.cuda.synchronize(dev)
        with xrt.Context(0) as fresh:
            fresh.upload_mesh(dragon)
            got = fresh.render_rows(cam)
            hc = fresh.host_call_ms()
            again = fresh.render_rows(cam)
    print("first host-buffer call after the loop:", hc)
    assert hc["enqueue"] <= 3.0, hc
    assert hc["of_which_device_sync"] <= 1.0, hc
    for planes in sets:
        for x, y in zip(planes, got[:3]):
            assert np.array_equal(bits(x.cpu().numpy()), bits(y))
    for x, y in zip(again[:3], got[:3]):
        assert np.array_equal(bits(x), bits(y))


def test_host_buffer_d2h_pieces_exact(dragon):
    """The pinned-ring D2H of the host-buffer entry points (1-MB pieces, 32 ring
    slots, copy threads): frames whose planes span many ring rounds (1024 x
    1531, 3000 x 2000) and a strip that is not a multiple of a piece arrive
    exactly -- equal to the device planes of the same frame copied by torch."""
    import torch
    dev = torch.device("cuda", 0)
    with xrt.Context(0) as c:
        c.upload_mesh(dragon)
        for W, H, r0, r1 in [(1024, 1531, 0, 1531), (3000, 2000, 0, 2000), (777, 555, 13, 500)]:
            cam = xrt.camera_for_mesh(dragon, W, H)
            n = (r1 - r0) * W
            planes = (torch.empty(n, device=dev), torch.empty(n, device=dev), torch.empty(n, dtype=torch.uint8,
                                                                                           device=dev))
            c.render_rows_device(cam, r0, r1, *(p.data_ptr() for p in planes), 0)
            torch.cuda.synchronize(dev)
            got = c.render_rows(cam, r0, r1)
            for x, y in zip(planes, got[:3]):
                assert np.array_equal(bits(x.cpu().numpy()), bits(y)), (W, H)
            assert c.host_call_ms()["d2h_mb"] == pytest.approx(9 * n / 1e6)


@pytest.mark.parametrize("W,H,r0,r1", [(2048, 2048, 0, 2048), (1000, 777, 0, 777), (4096, 4096, 1024, 2080),
                                       (333, 517, 100, 400)])
def test_tile_plan_frames_exact(dragon, W, H, r0, r1):
    """The tile plan (opt-in; SlotDesc::live from one render's records): later frames of
    the same geometry store the misses of the tiles that had no survivor
    without reading their region's list -- every such frame bit-equal to a
    brute-force render; a camera change re-plans, and the old plan is not used."""
    cams = [xrt.camera_for_mesh(dragon, W, H), xrt.camera_from_bbox(*oracle.bbox(dragon[:7000]), W, H)]
    with xrt.Context(0) as brute:
        brute.set_kernel(xrt.XRT_KERNEL_BRUTE)
        brute.upload_mesh(dragon)
        refs = [brute.render_rows(c, r0, r1) for c in cams]
    with xrt.Context(0) as c:
        c.set_kernel(xrt.XRT_KERNEL_BINNED)
        c.upload_mesh(dragon)
        c.set_tile_plan(True)                  # opt-in (off by default)
        for k in range(8):
            ci = (k // 4) % 2
            got = c.render_rows(cams[ci], r0, r1)
            for x, y in zip(got[:3], refs[ci][:3]):
                assert np.array_equal(bits(x), bits(y)), (k, ci)
        counters = c.tile_plan_counters()
    # (the first frame of camera 0 is sized on the device, the second on the
    # host: its plan serves frames 2 and 3; camera 1's frames 4 and 5 take the
    # moving path, frame 6 is sized, frame 7 uses its plan)
    assert counters["plans"] == 2 and counters["frames"] >= 3, counters


def test_split_tiles_with_packed_transit_exact(dragon, monkeypatch):
    """Split tiles (XRT_SPLIT_MIN=1: every non-empty region) rendered straight
    into the packed transit layout of a strip (xrt_set_transit_layout) and
    unpacked: equal to the strip's direct render (round-4 advice: the split
    halves' merge was pinned only for row-major planes)."""
    import torch
    monkeypatch.setenv("XRT_SPLIT_MIN", "1")
    W, H, r0, r1 = 1024, 1024, 256, 768
    cam = xrt.camera_for_mesh(dragon, W, H)
    rows = r1 - r0
    dev = torch.device("cuda", 0)
    with xrt.Context(0) as c:
        c.set_kernel(xrt.XRT_KERNEL_BINNED)
        c.upload_mesh(dragon)
        ref = c.render_rows(cam, r0, r1)
        stream = torch.cuda.current_stream(dev)
        c.set_miss_code(xrt._abi.XRT_MISS_TRANSIT)
        lb = torch.zeros(W * rows, device=dev)
        c.render_rows_device(cam, r0, r1, 0, lb.data_ptr(), 0, stream.cuda_stream)
        rmap, n_packed = c.plan_region_map(W, rows)
        packed = torch.full((max(n_packed, 1) * 1024,), -3.0, device=dev)
        c.set_transit_layout(packed.numel())
        for _ in range(3):                            # the sizing frame's plan, then steady frames
            c.render_rows_device(cam, r0, r1, 0, packed.data_ptr(), 0, stream.cuda_stream)
        c.set_transit_layout(0)
        c.set_miss_code(0)
        d_map = torch.from_numpy(rmap.view(np.int32)).to(dev)
        out = [torch.zeros(W * rows, device=dev), torch.zeros(W * rows, device=dev),
               torch.zeros(W * rows, dtype=torch.uint8, device=dev)]
        c.unpack_regions_device(W, rows, d_map.data_ptr(), packed.data_ptr(), out[0].data_ptr(), out[1].data_ptr(),
                                out[2].data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
    assert n_packed < len(rmap)
    assert np.array_equal(bits(out[1].cpu().numpy()), bits(ref[0]))
    assert np.array_equal(bits(out[0].cpu().numpy()), bits(ref[1]))
    assert np.array_equal(out[2].cpu().numpy(), ref[2])


def test_timing_region_before_any_frame_and_twice(dragon):
    """xrt_timing_begin on a fresh context (no frame yet to size the record
    space from) keeps every frame of a region of 2048^2 frames; a second begin
    while a region is open ends it first."""
    import torch
    W = H = 2048
    cam = xrt.camera_for_mesh(dragon, W, H)
    dev = torch.device("cuda", 0)
    planes = [torch.empty(W * H, device=dev), torch.empty(W * H, device=dev),
              torch.empty(W * H, dtype=torch.uint8, device=dev)]
    with xrt.Context(0) as c:
        c.upload_mesh(dragon)
        c.timing_begin()
        for _ in range(40):
            c.render_rows_device(cam, 0, H, *(p.data_ptr() for p in planes), 0)
        ms, n = c.timing_end()
        assert n == 40 and ms > 0
        c.timing_begin()
        for _ in range(3):
            c.render_rows_device(cam, 0, H, *(p.data_ptr() for p in planes), 0)
        c.timing_begin()                              # the open region ends, a new one starts
        for _ in range(5):
            c.render_rows_device(cam, 0, H, *(p.data_ptr() for p in planes), 0)
        ms2, n2 = c.timing_end()
        assert n2 == 5 and ms2 > 0
        assert c.read_stats().kernel_ms > 0


def test_multi_device_pipelined(dragon):
    """xrt_render_rows_multi_device: frames enqueued back to back into torch
    device planes (the next frame's strips render while the last one's gather is
    in flight), each equal to the single-device frame."""
    import torch
    W = H = 256
    dev = torch.device("cuda", 0)
    cams = [xrt.camera_for_mesh(dragon, W, H), xrt.camera_from_bbox(*oracle.bbox(dragon[:5000]), W, H)]
    with xrt.Context(0) as one:
        one.upload_mesh(dragon)
        refs = [one.render_rows(c) for c in cams]
    stream = torch.cuda.Stream(device=dev)
    with xrt.MultiContext([0, 0]) as m:
        m.upload_mesh(dragon)
        outs = []
        with torch.cuda.stream(stream):
            for k in range(6):
                planes = (torch.empty(W * H, device=dev), torch.empty(W * H, device=dev),
                          torch.empty(W * H, dtype=torch.uint8, device=dev))
                m.render_device(cams[k % 2], planes[0].data_ptr(), planes[1].data_ptr(), planes[2].data_ptr(),
                                stream.cuda_stream)
                outs.append(planes)
        stream.synchronize()
        m.read_stats()
    for k, planes in enumerate(outs):
        for x, y in zip(planes, refs[k % 2][:3]):
            assert np.array_equal(bits(x.cpu().numpy()), bits(y)), k


@pytest.mark.parametrize("soup", ["dragon", "corner"])
def test_transit_expand_equals_direct_render(ctx, dragon, soup):
    """An L-buffer strip rendered with misses coded XRT_MISS_TRANSIT, expanded by
    xrt_expand_rows_device, equals the direct render's three planes -- also for
    the t = +inf hits of the corner soup, whose L is +inf like a miss's but whose
    image is 0, not 80."""
    import torch
    tris = dragon if soup == "dragon" else corner_soup()
    W, H = (192, 160) if soup == "dragon" else (33, 31)
    cam = xrt.camera_for_mesh(tris, W, H)
    ctx.upload_mesh(tris)
    ctx.set_kernel(xrt.XRT_KERNEL_BINNED)
    ref = ctx.render_rows(cam)
    dev = torch.device("cuda", ctx.device)
    lb = torch.full((W * H,), -1.0, device=dev)
    img = torch.zeros(W * H, device=dev)
    u8 = torch.zeros(W * H, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    ctx.set_miss_code(xrt._abi.XRT_MISS_TRANSIT)
    try:
        ctx.render_rows_device(cam, 0, H, 0, lb.data_ptr(), 0, stream.cuda_stream)
        coded = lb.cpu().numpy().copy()
        ctx.expand_rows_device(W * H, lb.data_ptr(), img.data_ptr(), u8.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
    finally:
        ctx.set_miss_code(0)
    n_coded = int(np.count_nonzero(coded.view(np.uint32) == xrt._abi.XRT_MISS_TRANSIT))
    assert n_coded == W * H - ref[3].hit_rays                       # every miss, and only misses
    assert np.array_equal(bits(img.cpu().numpy()), bits(ref[0]))
    assert np.array_equal(bits(lb.cpu().numpy()), bits(ref[1]))
    assert np.array_equal(u8.cpu().numpy(), ref[2])


@pytest.mark.parametrize("W,H,r0,r1", [(1000, 700, 0, 700), (2048, 2048, 1024, 2048), (333, 517, 100, 400)])
def test_packed_transit_equals_direct_render(ctx, dragon, W, H, r0, r1):
    """A transit L-buffer strip packed by its fill plan (only the regions the
    plan did not fill travel) and unpacked into the three planes equals the
    direct render of the strip; the packed size is the unfilled regions'."""
    import torch
    cam = xrt.camera_for_mesh(dragon, W, H)
    ctx.upload_mesh(dragon)
    ctx.set_kernel(xrt.XRT_KERNEL_BINNED)
    ref = ctx.render_rows(cam, r0, r1)
    rows = r1 - r0
    dev = torch.device("cuda", ctx.device)
    stream = torch.cuda.current_stream(dev)
    lb = torch.full((W * rows,), -1.0, device=dev)
    ctx.set_miss_code(xrt._abi.XRT_MISS_TRANSIT)
    try:
        ctx.render_rows_device(cam, r0, r1, 0, lb.data_ptr(), 0, stream.cuda_stream)
        rmap, n_packed = ctx.plan_region_map(W, rows)
        n_fill = ctx.fill_regions()
    finally:
        ctx.set_miss_code(0)
    assert 0 < n_fill and n_packed == len(rmap) - n_fill
    assert np.count_nonzero(rmap == 0xFFFFFFFF) == n_fill
    assert sorted(rmap[rmap != 0xFFFFFFFF].tolist()) == list(range(n_packed))
    d_map = torch.from_numpy(rmap.view(np.int32)).to(dev)
    packed = torch.zeros(n_packed * 1024, device=dev)
    ctx.pack_regions_device(W, rows, d_map.data_ptr(), lb.data_ptr(), packed.data_ptr(), stream.cuda_stream)
    out = [torch.full((W * rows,), -2.0, device=dev), torch.zeros(W * rows, device=dev),
           torch.zeros(W * rows, dtype=torch.uint8, device=dev)]
    ctx.unpack_regions_device(W, rows, d_map.data_ptr(), packed.data_ptr(), out[0].data_ptr(), out[1].data_ptr(),
                              out[2].data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    assert np.array_equal(bits(out[1].cpu().numpy()), bits(ref[0]))
    assert np.array_equal(bits(out[0].cpu().numpy()), bits(ref[1]))
    assert np.array_equal(out[2].cpu().numpy(), ref[2])
    # the same blocks written by the render itself (xrt_set_transit_layout)
    direct = torch.full((n_packed * 1024,), -3.0, device=dev)
    ctx.set_miss_code(xrt._abi.XRT_MISS_TRANSIT)
    ctx.set_transit_layout(direct.numel())
    try:
        ctx.render_rows_device(cam, r0, r1, 0, direct.data_ptr(), 0, stream.cuda_stream)
        assert ctx.fill_regions() == n_fill
        with pytest.raises(RuntimeError):          # image / u8 planes have no packed layout
            ctx.render_rows_device(cam, r0, r1, out[1].data_ptr(), direct.data_ptr(), 0, stream.cuda_stream)
    finally:
        ctx.set_transit_layout(0)
        ctx.set_miss_code(0)
    out2 = [torch.full((W * rows,), -2.0, device=dev), torch.zeros(W * rows, device=dev),
            torch.zeros(W * rows, dtype=torch.uint8, device=dev)]
    ctx.unpack_regions_device(W, rows, d_map.data_ptr(), direct.data_ptr(), out2[0].data_ptr(), out2[1].data_ptr(),
                              out2[2].data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    for x, y in zip(out2, out):
        assert np.array_equal(x.cpu().numpy().view(np.uint8), y.cpu().numpy().view(np.uint8))


def _hit_strip(c, cam, W, r0, r1, dev, stream, frames=3):
    """One context's strip [r0, r1) in the hit layout: the geometry's first
    frame (row-major), its region map and hit plan, then `frames` frames
    rendered straight into the message.  Returns (map, tile hits, message)."""
    import torch
    rows = r1 - r0
    lb = torch.zeros(W * rows, device=dev)
    c.render_rows_device(cam, r0, r1, 0, lb.data_ptr(), 0, stream.cuda_stream)
    rmap, n_packed = c.plan_region_map(W, rows)
    hits, words = c.plan_hit_layout()
    assert len(hits) == 16 * n_packed and words == 2 * len(hits) + int(hits.sum())
    msg = torch.full((words + 64,), -5.0, device=dev)
    c.set_transit_hits(msg.numel())
    try:
        for _ in range(frames):                        # the tile plan comes in after the first
            c.render_rows_device(cam, r0, r1, 0, msg.data_ptr(), 0, stream.cuda_stream)
    finally:
        c.set_transit_hits(0)
    torch.cuda.synchronize(dev)
    return rmap, hits, msg[:words]


@pytest.mark.parametrize("W,H,cuts", [(1000, 700, [0, 700]), (2048, 2048, [0, 900, 2048]), (1024, 1024, [0, 32, 1024]),
                                      (333, 517, [0, 100, 400, 517]), (4096, 4096, [0, 1536, 2560, 4096])])
def test_hit_transit_equals_direct_render(dragon, W, H, cuts):
    """Strips rendered straight into the hit layout (xrt_set_transit_hits: a
    64-bit hit mask per tile of the fill plan, then the hit rays' L values),
    gathered into one buffer and unpacked by one xrt_unpack_hits_device launch,
    equal the single-device frame's three planes bit for bit; the message is
    2 words per planned tile plus one per hit ray; no mask disagrees with its
    plan."""
    _hit_transit_frame(dragon, W, H, cuts, xrt.camera_for_mesh(dragon, W, H))


def test_hit_transit_empty_strips(dragon):
    """A strip whose every region the fill plan fills (the camera zoomed out,
    the top rows clear of the mesh): no tile of it travels -- a plan of 0
    tiles, the minimum message -- and the gathered frame still equals the
    single-device frame bit for bit."""
    W = H = 1024
    cam = xrt.camera_for_mesh(dragon, W, H)
    cam.pixel_spacing *= 3.0
    plans = _hit_transit_frame(dragon, W, H, [0, 160, 864, 1024], cam)
    assert len(plans[0]) == 0 and len(plans[1]) > 0     # (the mesh reaches the bottom strip)


def _hit_transit_frame(dragon, W, H, cuts, cam):
    """test_hit_transit_equals_direct_render's body; returns the strips' plans."""
    import torch
    from simpleraytracing_amd.strips import hit_descriptors
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    spans = list(zip(cuts[:-1], cuts[1:]))
    maps, plans, msgs = [], [], []
    for r0, r1 in spans:
        with xrt.Context(0) as c:
            c.set_kernel(xrt.XRT_KERNEL_BINNED)
            c.upload_mesh(dragon)
            rmap, hits, msg = _hit_strip(c, cam, W, r0, r1, dev, stream)
            st = c.read_stats()
        assert int(hits.sum()) == st.hit_rays          # every hit ray of the strip travels, once
        maps.append(rmap)
        plans.append(hits)
        msgs.append(msg)
    desc, tdesc, bases, words, total = hit_descriptors(W, spans, maps, plans)
    assert words == [max(m.numel(), 4) for m in msgs]
    rbuf = torch.zeros(total, dtype=torch.float32, device=dev)
    for b, m in zip(bases, msgs):
        rbuf[b:b + m.numel()] = m
    d_desc = torch.from_numpy(desc.reshape(-1).view(np.int32)).to(dev)
    d_tdesc = torch.from_numpy(tdesc.reshape(-1).view(np.int32)).to(dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    out = [torch.full((W * H,), -2.0, device=dev), torch.full((W * H,), -2.0, device=dev),
           torch.zeros(W * H, dtype=torch.uint8, device=dev)]
    with xrt.Context(0) as c:
        c.unpack_hits_device(W, len(desc), d_desc.data_ptr(), d_tdesc.data_ptr(), rbuf.data_ptr(), out[0].data_ptr(),
                             out[1].data_ptr(), out[2].data_ptr(), bad.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        assert int(bad.item()) == 0
        c.upload_mesh(dragon)
        c.set_kernel(xrt.XRT_KERNEL_BINNED)
        ref = c.render_rows(cam)
    assert np.array_equal(bits(out[1].cpu().numpy()), bits(ref[0]))
    assert np.array_equal(bits(out[0].cpu().numpy()), bits(ref[1]))
    assert np.array_equal(out[2].cpu().numpy(), ref[2])
    return plans


def test_hit_transit_split_tiles_exact(dragon, monkeypatch):
    """The hit layout with split tiles (XRT_SPLIT_MIN=1: every non-empty
    region's tiles by two waves; half 0 stores the tile's mask and hits):
    strips gathered and unpacked equal the single-device frame bit for bit."""
    monkeypatch.setenv("XRT_SPLIT_MIN", "1")
    _hit_transit_frame(dragon, 1024, 1024, [0, 256, 768, 1024], xrt.camera_for_mesh(dragon, 1024, 1024))


def test_hit_transit_guards(dragon):
    """The hit layout's guards: a message whose mask disagrees with the plan
    sets the unpack's flag; a frame of another geometry (or with no plan) is
    not rendered (XRT_ERR_OVERFLOW); image / u8 planes have no hit layout; the
    plan needs a binned frame over a fill plan just before."""
    import torch
    from simpleraytracing_amd.strips import hit_descriptors
    W, H, r0, r1 = 1024, 1024, 256, 768
    cam = xrt.camera_for_mesh(dragon, W, H)
    cam2 = xrt.camera_from_bbox(*oracle.bbox(dragon[:5000]), W, H)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    with xrt.Context(0) as c:
        c.set_kernel(xrt.XRT_KERNEL_BINNED)
        c.upload_mesh(dragon)
        with pytest.raises(RuntimeError):             # no frame yet
            c.plan_hit_layout()
        rmap, hits, msg = _hit_strip(c, cam, W, r0, r1, dev, stream, frames=1)
        big = torch.zeros(msg.numel() + 64, device=dev)
        c.set_transit_hits(big.numel())
        try:
            with pytest.raises(RuntimeError):         # another camera: not this plan's geometry
                c.render_rows_device(cam2, r0, r1, 0, big.data_ptr(), 0, stream.cuda_stream)
            img = torch.zeros(W * (r1 - r0), device=dev)
            with pytest.raises(RuntimeError):
                c.render_rows_device(cam, r0, r1, img.data_ptr(), big.data_ptr(), 0, stream.cuda_stream)
        finally:
            c.set_transit_hits(0)
        c.set_transit_hits(msg.numel())               # no room for a tile's overrun
        try:
            with pytest.raises(RuntimeError):
                c.render_rows_device(cam, r0, r1, 0, big.data_ptr(), 0, stream.cuda_stream)
        finally:
            c.set_transit_hits(0)
        torch.cuda.synchronize(dev)
    desc, tdesc, bases, words, total = hit_descriptors(W, [(r0, r1)], [rmap], [hits])
    d_desc = torch.from_numpy(desc.reshape(-1).view(np.int32)).to(dev)
    d_tdesc = torch.from_numpy(tdesc.reshape(-1).view(np.int32)).to(dev)
    out = torch.zeros(W * H, device=dev)
    i = int(np.flatnonzero(hits)[0])                  # a tile with hits: drop one from its mask
    bad_msg = msg.clone()
    m = bad_msg[2 * i:2 * i + 2].view(torch.int32).cpu().numpy().view(np.uint32).copy()
    lo = int(m[0]) | (int(m[1]) << 32)
    lo &= lo - 1
    bad_msg[2 * i:2 * i + 2] = torch.from_numpy(np.array([lo & 0xFFFFFFFF, lo >> 32], np.uint32).view(np.float32))
    for src, expect in ((msg, 0), (bad_msg, 1)):
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        with xrt.Context(0) as c:
            c.unpack_hits_device(W, len(desc), d_desc.data_ptr(), d_tdesc.data_ptr(), src.data_ptr(),
                                 out.data_ptr(), 0, 0, bad.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize(dev)
        assert int(bad.item()) == expect


@pytest.mark.parametrize("transit,ranks,share,size", [("packed", 2, "auto", 512), ("dense", 2, "auto", 512),
                                                       ("packed", 3, "equal", 512), ("dense", 3, "0.5", 512),
                                                       ("packed", 3, "balanced", 512), ("dense", 2, "balanced", 512),
                                                       ("packed", 4, "balanced", 512),
                                                       ("hits", 2, "auto", 512), ("hits", 3, "balanced", 512),
                                                       ("hits", 4, "equal", 1024),
                                                       ("packed", 8, "balanced", 4096), ("hits", 8, "balanced", 4096)])
def test_bench_strips_two_ranks_one_gpu(tmp_path, transit, ranks, share, size):
    """bench.py's N > 1 path (row strips, transit L-buffers sent to rank 0 --
    packed by region or dense --, expanded there) with 2-8 ranks on the one GPU
    (gloo, host-staged): the gathered frame is bit-equal to rank 0's
    single-device render.  The 8-rank cases are BASELINE configs[3]'s real split
    (4096^2, 8 strips, balanced; packed, and hits -- the default), and they also run the bench's
    capi_multi leg: the C ABI's xrt_render_rows_multi_device over device 0
    listed 8 times (one-rank RCCL), bit-equal as well."""
    import json
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    port = 29500 + (os.getpid() % 1000) + {"dense": 7, "hits": 3}.get(transit, 0) + 13 * ranks + (size == 4096)
    capi = ranks == 8
    cmd = ["python", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", str(ranks), "--dist-backend", "gloo", "--same-device", "--size", str(size), str(size),
           "--steps", "4", "--warmup", "1", "--transit", transit, "--kernel", "binned", "--root-share", share,
           "--loaded-ms", "0", "--capi-multi", "auto" if capi else "off"]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=280, cwd=ROOT)
    if r.returncode != 0:
        print(r.stderr[-6000:])
    assert r.returncode == 0
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["config"]["mode"] == "strips" and d["n_gpus"] == ranks
    assert d["gather_check"]["bit_exact_vs_single_device_frame"] is True
    g = d["gather_check"]
    rows = g["strip_rows"]
    assert sum(rows) == size and len(rows) == ranks
    if capi:
        c = d["capi_multi"]
        assert "error" not in c, c
        assert c["bit_exact_vs_single_device_frame"] is True and c["devices"] == [0] * 8
        assert sum(c["strip_rows"]) == size and c["plan"]["predicted_step_us"] > 0
    else:
        assert "capi_multi" not in d
    if share == "equal":
        assert max(rows) - min(rows) <= 1
    elif share == "balanced":                     # band-aligned strips, the root's anywhere in the frame
        spans = sorted(map(tuple, g["strips"]))
        assert spans[0][0] == 0 and spans[-1][1] == size and all(s0 % 32 == 0 for s0, _ in spans)
        assert all(spans[i][1] == spans[i + 1][0] for i in range(ranks - 1))
        assert g["split"]["link_bytes_per_us"] > 0 and g["split"]["predicted_step_us"] > 0
    else:
        assert rows[0] > size // ranks
    if transit in ("packed", "hits"):
        assert g["bytes_gathered_per_step"] < g["dense_bytes_per_step"]
    else:
        assert g["bytes_gathered_per_step"] == g["dense_bytes_per_step"]


def test_render_frames_batch_equals_single_calls(dragon):
    """xrt_render_frames_device: 7, 5 and 12 frames of one geometry, each run in ONE
    call, alternating two plane sets on two streams (each frame prepared and
    rendered in full) --
    every set's last frame bit-equal to a single xrt_render_rows; the
    host-buffer xrt_render_frames likewise, with its per-frame device time."""
    import torch
    dev = torch.device("cuda", 0)
    for W, H, r0, r1 in [(1024, 1024, 0, 1024), (640, 480, 100, 380)]:
        cam = xrt.camera_for_mesh(dragon, W, H)
        n = (r1 - r0) * W
        streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        sets = [(torch.full((n,), -1.0, device=dev), torch.full((n,), -1.0, device=dev),
                 torch.zeros(n, dtype=torch.uint8, device=dev), s) for s in streams]
        with xrt.Context(0) as c:
            c.upload_mesh(dragon)
            ref = c.render_rows(cam, r0, r1)
            # 7, 5, then 12 frames (each call's sets start where the last one's ended)
            for nf in (7, 5, 12):
                c.render_frames_device(cam, r0, r1, nf, [(a.data_ptr(), b.data_ptr(), u.data_ptr(), s.cuda_stream)
                                                         for a, b, u, s in sets])
            torch.cuda.synchronize(dev)
            for a, b, u, _ in sets:
                for x, y in zip((a, b, u), ref[:3]):
                    assert np.array_equal(bits(x.cpu().numpy()), bits(y)), (W, H)
            img, lb, u8, st, ms = c.render_frames(cam, 5, r0, r1)
        for x, y in zip((img, lb, u8), ref[:3]):
            assert np.array_equal(bits(x), bits(y))
        assert st.hit_rays == ref[3].hit_rays and ms > 0


def test_cli_rows_and_batch(tmp_path):
    """xrt_main --rows A:B writes only the strip's text rows; --batch N renders the
    frame N times back to back (xrt_render_frames) and writes the last -- the
    golden text's rows either way."""
    exe = os.path.join(ROOT, "simpleraytracing_amd", "lib", "xrt_main")
    (tmp_path / "out").mkdir()
    golden = open(os.path.join(GOLDEN, "dragon-128x128-serial.txt"), "rb").read().split(b"\n")
    for extra, name, want in [(["--rows", "32:96"], "r.txt", b"\n".join(golden[32:96])),
                              (["--batch", "3", "--time"], "b.txt", b"\n".join(golden)),
                              (["--rows", "0:17", "--batch", "2"], "rb.txt", b"\n".join(golden[0:17]))]:
        r = subprocess.run([exe, "-s", "128", "128", "-i", DRAGON, "-f", name, *extra], capture_output=True,
                           text=True, cwd=tmp_path, timeout=300)
        assert r.returncode == 0, r.stderr
        assert (tmp_path / "out" / name).read_bytes() == want, extra
        if "--time" in extra:
            assert "device time per frame" in r.stdout
    r = subprocess.run([exe, "-s", "128", "128", "-i", DRAGON, "--rows", "90:40"], capture_output=True, text=True,
                       cwd=tmp_path, timeout=60)
    assert r.returncode == 1 and "ERROR" in r.stderr


def test_cli_multi_gpu_golden_text(tmp_path):
    """xrt_main -g 2 (renderLoopMultiGPU over xrt_render_rows_multi): strips on a
    device listed twice (one GPU here), the golden text byte for byte."""
    exe = os.path.join(ROOT, "simpleraytracing_amd", "lib", "xrt_main")
    (tmp_path / "out").mkdir()
    env = dict(os.environ, XRT_MULTI_DEVICES="0,0")
    r = subprocess.run([exe, "-s", "128", "128", "-i", DRAGON, "-f", "d.txt", "-g", "2"], capture_output=True,
                       text=True, cwd=tmp_path, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    got = (tmp_path / "out" / "d.txt").read_bytes()
    assert got == open(os.path.join(GOLDEN, "dragon-128x128-serial.txt"), "rb").read()


FIXTURES = ["planes_dragon_128", "planes_dragon_256", "rows_dragon_1024", "rows_dragon_2048", "rows_dragon_4096",
            "rows_dragon_8192", "rows_tiled7_8192"]


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_rows_device(dragon, name):
    """The device against the committed fixtures the reference's own classes
    rendered (tools/gen_golden.py): every 8-GPU strip boundary row
    (k*H/8 - 1, k*H/8), row 0, H/2 and H - 1 of dragon.ply at 1024^2..8192^2 and
    of the 1.12 M-triangle tiled dragon at 8192^2, and whole 128^2 / 256^2
    frames -- from a whole-frame BINNED render (device planes, the rows
    gathered on the device) and from each row as a one-row strip, image,
    L-buffer and u8 bit for bit, hit rays per row.  Nothing is recomputed on
    this box: its libm is on neither side."""
    import hashlib

    import torch
    from simpleraytracing_amd.scenes import tiled_mesh
    g = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    W, H = int(g["width"]), int(g["height"])
    tris = tiled_mesh(dragon, 7) if "tiled7" in name else dragon
    assert hashlib.sha256(np.ascontiguousarray(tris, np.float32).tobytes()).hexdigest() == str(g["mesh_sha256"])
    cam = xrt.camera_for_mesh(tris, W, H)
    cam13 = np.array(list(cam.origin) + list(cam.detector) + list(cam.up) + list(cam.right) + [cam.pixel_spacing],
                     np.float32)
    assert np.array_equal(bits(cam13), bits(g["camera"]))
    rows = g["rows"].astype(np.int64)
    dev = torch.device("cuda", 0)
    with xrt.Context(0) as c:
        c.set_kernel(xrt.XRT_KERNEL_BINNED)
        c.upload_mesh(tris)
        planes = (torch.empty(W * H, device=dev), torch.empty(W * H, device=dev),
                  torch.empty(W * H, dtype=torch.uint8, device=dev))
        c.render_rows_device(cam, 0, H, *(p.data_ptr() for p in planes), 0)
        torch.cuda.synchronize(dev)
        idx = torch.from_numpy(rows).to(dev)
        got = [p.view(H, W).index_select(0, idx).cpu().numpy() for p in planes]
        assert np.array_equal(bits(got[0]), bits(g["image"])), "image"
        assert np.array_equal(bits(got[1]), bits(g["lbuffer"])), "lbuffer"
        assert np.array_equal(got[2], g["u8"]), "u8"
        del planes
        for i, r in enumerate(rows[:: max(1, len(rows) // 17)]):       # one-row strips
            k = int(np.nonzero(rows == r)[0][0])
            img, lb, u8, st = c.render_rows(cam, int(r), int(r) + 1)
            assert np.array_equal(bits(img), bits(g["image"][k])) and np.array_equal(bits(lb), bits(g["lbuffer"][k]))
            assert np.array_equal(u8, g["u8"][k]) and st.hit_rays == int((g["nhits"][k] > 0).sum()), int(r)
