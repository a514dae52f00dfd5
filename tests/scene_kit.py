"""Test scenes (synthetic, seeded): shared by the CPU and GPU suites."""
import numpy as np


def box(lo, hi):
    """A closed axis-aligned box of 12 triangles, normals pointing out."""
    (x0, y0, z0), (x1, y1, z1) = lo, hi
    v = np.array([[x0, y0, z0], [x1, y0, z0], [x1, y1, z0], [x0, y1, z0],
                  [x0, y0, z1], [x1, y0, z1], [x1, y1, z1], [x0, y1, z1]], np.float32)
    faces = [(0, 2, 1), (0, 3, 2), (4, 5, 6), (4, 6, 7), (0, 1, 5), (0, 5, 4),
             (2, 3, 7), (2, 7, 6), (1, 2, 6), (1, 6, 5), (0, 4, 7), (0, 7, 3)]
    return np.array([np.concatenate([v[a], v[b], v[c]]) for a, b, c in faces], np.float32)


def second_mesh_for(dragon):
    """A box beside the dragon along +y (and a little above in z): it widens the
    scene's bounding box, so it moves the camera, and it lies in the view."""
    lo = dragon.reshape(-1, 3).min(0)
    hi = dragon.reshape(-1, 3).max(0)
    r = hi - lo
    return box(lo + np.float32(0.6) * r * np.array([0.2, 1.0, 0.1], np.float32),
               hi + np.float32(0.35) * r * np.array([-0.2, 1.0, 0.25], np.float32))


def synthetic_soup(seed=11, n=3000):
    """Random open triangles with collinear, duplicate and zero-edge members."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(-50, 50, (n, 1, 3))
    t = (c + rng.normal(0, 6, (n, 3, 3))).astype(np.float32)
    soup = t.reshape(n, 9)
    k = n // 10
    soup[:k, 6:9] = (soup[:k, 0:3] + 2 * (soup[:k, 3:6] - soup[:k, 0:3])).astype(np.float32)  # collinear
    soup[k:2 * k] = soup[2 * k:3 * k]                                                    # duplicates (ties)
    soup[3 * k:3 * k + 20, 3:6] = soup[3 * k:3 * k + 20, 0:3]                             # zero-length edge
    return np.ascontiguousarray(soup)


def corner_soup():
    """Triangles with 1e-20 edges one unit in front of the source, on the image's
    centre column (odd W: the ray direction's y component is exactly 0 there):
    det is a nonzero denormal, 1/det overflows to inf, a = u * det is exactly
    0, so Ray.cxx:99-122 computes u = 0 * inf = NaN (passes both u tests),
    v = +inf, u + v = NaN (passes) and t = +inf > 1e-7: the reference records
    a hit at infinity for rays nowhere near the triangle.  The frame triangles
    fix a bbox symmetric about y = 0 and z = 0 (the source's y and z)."""
    tris = [[40, -10, -10, 40, 10, -10, 40, 10, 10], [60, -10, -10, 60, 10, 10, 60, -10, 10]]
    for x0, sz in [(45, 1), (47, -1), (50, 1), (52, -1), (55, 1)]:
        tris.append([x0, 0, 0, x0, 1e-20, 0, x0, 0, sz * 1e-20])
        tris.append([x0, 0, 0, x0, 0, sz * 1e-20, x0, 1e-20, 0])
    return np.array(tris, np.float32)


def striped_sheets(seed=3, n=40):
    """Open quads (two triangles each) in front of a closed box: rays through a
    quad see an odd number of surfaces, so the signed model flags them; the
    stripes are 1 to 12 pixels wide at 96 x 80, so the hole fill finds
    neighbours in some directions, in none for the widest."""
    rng = np.random.default_rng(seed)
    out = [box(np.array([50, -30, -25], np.float32), np.array([70, 30, 25], np.float32))]
    for _ in range(n):
        y0 = rng.uniform(-30, 28)
        w = rng.uniform(0.2, 4.0)
        z0, z1 = sorted(rng.uniform(-25, 25, 2))
        x = rng.uniform(42, 48)
        q = np.array([[x, y0, z0, x, y0 + w, z0, x, y0 + w, z1], [x, y0, z0, x, y0 + w, z1, x, y0, z1]], np.float32)
        out.append(q if rng.random() < 0.5 else q[:, [0, 1, 2, 6, 7, 8, 3, 4, 5]])   # both windings
    return np.ascontiguousarray(np.concatenate(out))


def plane_stack(n, spacing=0.01, alternate=False):
    """n parallel unit squares (2 triangles each) facing the detector: every ray
    through the square hits each plane (twice on the shared diagonal).  With
    alternate, every second square is wound the other way (its normal flips),
    so the signed model's signs cancel over each pair of planes."""
    x = (np.arange(n, dtype=np.float32) * np.float32(spacing)).astype(np.float32)
    a = np.stack([x, np.zeros(n, np.float32), np.zeros(n, np.float32)], 1)
    b = np.stack([x, np.ones(n, np.float32), np.zeros(n, np.float32)], 1)
    c = np.stack([x, np.ones(n, np.float32), np.ones(n, np.float32)], 1)
    d = np.stack([x, np.zeros(n, np.float32), np.ones(n, np.float32)], 1)
    t1 = np.concatenate([a, b, c], 1)
    t2 = np.concatenate([a, c, d], 1)
    if alternate:
        odd = np.arange(n) % 2 == 1
        t1[odd] = np.concatenate([a, c, b], 1)[odd]
        t2[odd] = np.concatenate([a, d, c], 1)[odd]
    return np.ascontiguousarray(np.stack([t1, t2], 1).reshape(2 * n, 9), dtype=np.float32)
