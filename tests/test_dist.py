"""CPU, world_size 2 (gloo): the multi-rank path of bench.py -- row-strip
partition, packed strip buffers and the gather to rank 0 -- assembles exactly
the single-rank frame.  The strip renderer here is the CPU oracle standing in
for the GPU (tests may use the oracle; the product never does)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from simpleraytracing_amd.strips import assemble, packed_size, strip_bounds, views
from conftest import DRAGON, ROOT


def test_weighted_bounds_cover_image():
    """Root-weighted strips (bench.py --root-share): contiguous, covering, rank 0
    first with at least its equal share, the others within one row of each other."""
    from simpleraytracing_amd.strips import root_share, weighted_bounds
    for H in (1, 7, 100, 131, 4096):
        for n in (1, 2, 3, 4, 8):
            if n > H:
                continue
            for share in (root_share(n), 0.0, 0.5, 0.99):
                spans = [weighted_bounds(H, n, r, share) for r in range(n)]
                assert spans[0][0] == 0 and spans[-1][1] == H
                assert all(spans[r][1] == spans[r + 1][0] for r in range(n - 1))
                assert all(e > b for b, e in spans)
                assert spans[0][1] >= -(-H // n)
                rest = [e - b for b, e in spans[1:]]
                assert not rest or max(rest) - min(rest) <= 1
    assert root_share(1) == 1.0 and abs(root_share(2) - 2.5 / 3.5) < 1e-12
    assert abs(root_share(8) - 2.5 / 9.5) < 1e-12 and root_share(8, rho=0.01) == 1.0 / 8


def test_unpack_descriptors_cover_strips():
    """The root's block descriptors (one unpack launch for every sender's packed
    regions): every pixel of every strip covered once, packed blocks numbered
    back to back per strip, filled regions marked empty."""
    from simpleraytracing_amd.strips import EMPTY, unpack_descriptors
    W = 100
    spans = [(10, 77), (77, 131)]
    rng = np.random.default_rng(3)
    maps = []
    for b, e in spans:
        n = 4 * -(-(e - b) // 32)
        m = np.full(n, EMPTY, np.uint32)
        keep = np.sort(rng.choice(n, n // 2, replace=False))
        m[keep] = rng.permutation(len(keep))
        maps.append(m)
    desc, bases, total = unpack_descriptors(W, spans, maps)
    assert bases == [0, 6] and total == 6 + 4
    cover = np.zeros((131, W), np.int32)
    for r0, rows, c0, blk in desc:
        assert 1 <= rows <= 32
        cover[r0:r0 + rows, c0:c0 + 32] += 1
    assert np.all(cover[10:131] == 1) and not cover[:10].any()
    blocks = desc[desc[:, 3] != EMPTY, 3]
    assert sorted(blocks.tolist()) == list(range(total))


def test_strip_bounds_cover_image():
    for H in (1, 7, 128, 2048, 4097):
        for n in (1, 2, 3, 4, 8):
            if n > H:
                continue
            spans = [strip_bounds(H, n, r) for r in range(n)]
            assert spans[0][0] == 0 and spans[-1][1] == H
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, out_path):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    from oracle import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tris = oracle.load_ply(DRAGON)
    cam = oracle.camera_for_mesh(tris, W, H)
    b, e = strip_bounds(H, world, rank)
    n_max = packed_size(W, H, world) // 9
    buf = torch.zeros(9 * n_max, dtype=torch.uint8)
    img, lb, u8 = views(buf.numpy(), n_max)
    s_img, s_lb, s_u8, _, _ = oracle.render_rows(tris, cam, W, H, b, e, threads=2)
    img[: s_img.size] = s_img
    lb[: s_lb.size] = s_lb
    u8[: s_u8.size] = s_u8
    gathered = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gathered, dst=0)
    if rank == 0:
        full = assemble([g.numpy() for g in gathered], W, H)
        np.savez(out_path, img=full[0], lb=full[1], u8=full[2])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H", [(2, 40, 33), (3, 24, 20)])
def test_gloo_gather_assembles_full_frame(tmp_path, world, W, H):
    from oracle import oracle
    out = str(tmp_path / "frame.npz")
    mp.spawn(_worker, args=(world, _free_port(), W, H, out), nprocs=world, join=True)
    got = np.load(out)
    tris = oracle.load_ply(DRAGON)
    ref = oracle.render_rows(tris, oracle.camera_for_mesh(tris, W, H), W, H)
    assert np.array_equal(got["img"].view(np.uint32), ref[0].view(np.uint32))
    assert np.array_equal(got["lb"].view(np.uint32), ref[1].view(np.uint32))
    assert np.array_equal(got["u8"], ref[2])
