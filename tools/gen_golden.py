"""Golden fixtures for the large BASELINE configs, generated
HERE, where the reference's sources are: every pixel comes from the
reference's own compiled classes (oracle/_ref: src/Ray.cxx, Triangle.cxx,
TriangleMesh.cxx unmodified, driven by renderLoop's per-pixel loop,
main.cxx:649-742) and is cross-checked bit for bit against the C restatement
(oracle/xrt_oracle.c) before it is written.  The GPU tests then compare the
device against these files, so the GPU box's own libm (expf) is not on both
sides of the check.

  tests/golden/rows_<mesh>_<W>.npz  full-width rows {0, k*H/8 - 1, k*H/8 (k = 1..7),
                                    H/2, H - 1} -- every 8-GPU strip boundary -- of
                                    dragon.ply at 1024^2, 2048^2, 4096^2, 8192^2 and of
                                    the 1.12 M-triangle tiled dragon (scenes.tiled_mesh,
                                    7x7; the mesh is regenerated, its SHA-256 stored) at
                                    8192^2: rows, camera (13 f32), image f32, L-buffer f32,
                                    u8, hit counts i32, odd-ray count
  tests/golden/planes_dragon_{128,256}.npz   every pixel of the frame, same fields
  tests/golden/kat_intersect.npz             the 64 K (ray, triangle) pairs of
                                    tests/kat.py through the reference's Ray::intersect
                                    (hit flags, distances; the inputs' SHA-256)

  python tools/gen_golden.py [--threads N] [--only NAME ...]
"""
import argparse
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def boundary_rows(H):
    rows = {0, H // 2, H - 1}
    for k in range(1, 8):
        rows |= {k * H // 8 - 1, k * H // 8}
    return np.array(sorted(rows), np.uint32)


def rows_fixture(name, tris, W, H, rows, threads):
    from oracle import oracle
    cam = oracle.camera_for_mesh(tris, W, H)
    t0 = time.time()
    img_r, lb_r, odd_r = oracle.ref_render_spans(tris, cam, W, H, rows, threads=threads)
    t1 = time.time()
    img, lb, u8, nh, odd = oracle.render_row_list(tris, cam, W, H, rows, threads=threads)
    t2 = time.time()
    img, lb, u8, nh = (a.reshape(len(rows), W) for a in (img, lb, u8, nh))
    if not (np.array_equal(img.view(np.uint32), img_r.view(np.uint32)) and
            np.array_equal(lb.view(np.uint32), lb_r.view(np.uint32)) and odd == odd_r):
        raise SystemExit(f"{name}: the reference's classes and the oracle differ")
    sha = hashlib.sha256(np.ascontiguousarray(tris, np.float32).tobytes()).hexdigest()
    np.savez_compressed(os.path.join(GOLDEN, f"{name}.npz"), rows=rows, camera=cam, image=img_r, lbuffer=lb_r,
                        u8=u8, nhits=nh, odd=np.int64(odd_r), width=np.int64(W), height=np.int64(H),
                        triangles=np.int64(len(tris)), mesh_sha256=np.array(sha))
    print(f"{name}: {len(rows)} rows x {W}, reference {t1 - t0:.1f} s, oracle {t2 - t1:.1f} s, "
          f"hit pixels {(nh > 0).sum()}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--only", nargs="*", default=None)
    args = ap.parse_args()
    from oracle import oracle
    from simpleraytracing_amd.scenes import tiled_mesh
    import kat
    dragon = oracle.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
    want = (lambda n: args.only is None or n in args.only)
    for S in (128, 256):
        name = f"planes_dragon_{S}"
        if want(name):
            rows_fixture(name, dragon, S, S, np.arange(S, dtype=np.uint32), args.threads)
    if want("kat_intersect"):
        rays, tris = kat.kat_vectors()
        hit, t = oracle.ref_intersect_batch(rays, tris)
        hit_o, t_o = oracle.intersect_batch(rays, tris)
        if not (np.array_equal(hit, hit_o) and np.array_equal(t.view(np.uint32), t_o.view(np.uint32))):
            raise SystemExit("kat: the reference's Ray::intersect and the oracle differ")
        # the inputs are tests/kat.py's (regenerated there from its seed): their hash, not their bytes
        sha = hashlib.sha256(rays.tobytes() + tris.tobytes()).hexdigest()
        np.savez_compressed(os.path.join(GOLDEN, "kat_intersect.npz"), inputs_sha256=np.array(sha), hit=hit, t=t)
        print(f"kat_intersect: {len(rays)} pairs, {int(hit.sum())} hits", flush=True)
    for S in (1024, 2048, 4096, 8192):
        name = f"rows_dragon_{S}"
        if want(name):
            rows_fixture(name, dragon, S, S, boundary_rows(S), args.threads)
    name = "rows_tiled7_8192"
    if want(name):
        rows_fixture(name, tiled_mesh(dragon, 7), 8192, 8192, boundary_rows(8192), args.threads)


if __name__ == "__main__":
    main()
