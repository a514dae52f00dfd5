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


def test_hit_descriptors_round_trip():
    """The hit layout's descriptors (xrt_unpack_hits_device): strips encoded as
    a sender's render writes them (per planned tile a 64-bit hit mask, then
    the hit values in bit order) and decoded through desc / tdesc exactly as
    k_unpack_hits reads them give back every hit of every strip, and misses
    elsewhere; messages start at 16-B aligned words; a strip with no planned
    tile sends the minimum message."""
    from simpleraytracing_amd.strips import EMPTY, hit_descriptors
    W = 100
    spans = [(10, 77), (77, 131), (131, 140)]
    rng = np.random.default_rng(5)
    rx = -(-W // 32)
    maps, plans, msgs, truth = [], [], [], np.full((140, W), np.nan, np.float32)
    for b, e in spans:
        ry = -(-(e - b) // 32)
        n = rx * ry
        m = np.full(n, EMPTY, np.uint32)
        # the last strip: every region filled by its plan (no tile travels)
        keep = np.sort(rng.choice(n, 0 if b == 131 else max(n // 2, 1), replace=False))
        m[keep] = rng.permutation(len(keep))
        n_slots = len(keep)
        masks = np.zeros(16 * n_slots, np.uint64)
        vals = [[] for _ in range(16 * n_slots)]
        for r in keep:
            s_ = int(m[r])
            y0, x0 = b + 32 * (r // rx), 32 * (r % rx)
            for t in range(16):
                for lane in range(64):
                    row, col = y0 + 8 * (t // 4) + lane // 8, x0 + 8 * (t % 4) + lane % 8
                    if row < e and col < W and rng.random() < 0.4:
                        v = np.float32(rng.random() * 10)
                        masks[16 * s_ + t] |= np.uint64(1 << lane)
                        vals[16 * s_ + t].append(v)
                        truth[row, col] = v
        hits = np.array([len(v) for v in vals], np.uint32)
        msg = np.concatenate([masks.view(np.uint32)] + [np.array(v, np.float32).view(np.uint32) for v in vals])
        maps.append(m)
        plans.append(hits)
        msgs.append(msg.astype(np.uint32))
    desc, tdesc, bases, words, total = hit_descriptors(W, spans, maps, plans)
    assert all(b % 4 == 0 for b in bases) and words == [max(len(x), 4) for x in msgs]
    buf = np.zeros(total, np.uint32)
    for b0, x in zip(bases, msgs):
        buf[b0:b0 + len(x)] = x
    out = np.full((140, W), -1.0, np.float32)
    for r0, rows, c0, first in desc:
        for r in range(rows):
            for c in range(32):
                if c0 + c >= W:
                    continue
                v = np.nan
                if first != EMPTY:
                    mw, hw, cnt, _ = tdesc[first + (r // 8) * 4 + c // 8]
                    mask = int(buf[mw]) | (int(buf[mw + 1]) << 32)
                    bit = (r % 8) * 8 + c % 8
                    assert bin(mask).count("1") == cnt
                    if (mask >> bit) & 1:
                        v = buf[hw + bin(mask & ((1 << bit) - 1)).count("1")].view(np.float32)
                out[r0 + r, c0 + c] = v
    assert np.array_equal(out[10:140], truth[10:140], equal_nan=True)


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


def _brute_best_step(cost, byts, n, link, unpack):
    """The smallest step over every layout balanced_bounds may choose: one
    contiguous root run, the bands above and below it cut into n - 1 non-empty
    contiguous sender strips."""
    import itertools
    nb = len(cost)

    def c(i, j):
        return sum(cost[i:j])

    def s(i, j):
        return max(c(i, j), sum(byts[i:j]) / link)
    best = float("inf")
    for a in range(nb):
        for b in range(a + 1, nb + 1):
            outside = [(0, a), (b, nb)]
            for k_above in range(0, n):
                k_below = n - 1 - k_above
                if k_above > a or k_below > nb - b or (k_above == 0) != (a == 0) or (k_below == 0) != (b == nb):
                    continue
                for cuts_a in itertools.combinations(range(1, a), max(k_above - 1, 0)):
                    ea = [0, *cuts_a, a] if k_above else []
                    for cuts_b in itertools.combinations(range(b + 1, nb), max(k_below - 1, 0)):
                        eb = [b, *cuts_b, nb] if k_below else []
                        parts = [(ea[i], ea[i + 1]) for i in range(len(ea) - 1)] + \
                                [(eb[i], eb[i + 1]) for i in range(len(eb) - 1)]
                        step = max([c(a, b) + unpack] + [s(i, j) for i, j in parts])
                        best = min(best, step)
            del outside
    return best


def test_balanced_bounds_optimal_small():
    """strips.balanced_bounds (bench.py --root-share balanced): contiguous strips
    covering the frame, every rank non-empty, and a step within 0.1 % of the best
    layout of its family, found by brute force on small random band costs."""
    from simpleraytracing_amd.strips import balanced_bounds, gather_step_us
    rng = np.random.default_rng(7)
    for trial in range(40):
        nb = int(rng.integers(3, 9))
        n = int(rng.integers(1, min(nb, 4) + 1))
        cost = rng.uniform(0.1, 10.0, nb)
        byts = rng.uniform(0.0, 2e5, nb) * (rng.uniform(size=nb) > 0.3)
        link = float(rng.uniform(5e3, 8e4))
        H = 32 * nb - int(rng.integers(0, 31))
        b = balanced_bounds(cost, byts, n, link, H, unpack_us=1.0)
        assert len(b) == n
        cover = sorted(b)
        assert cover[0][0] == 0 and cover[-1][1] == H
        assert all(cover[i][1] == cover[i + 1][0] for i in range(n - 1)) and all(e > s for s, e in b)
        assert all(s0 % 32 == 0 for s0, _ in b)
        if n == 1:
            continue
        got = gather_step_us(b, cost, byts, link, unpack_us=1.0)
        best = _brute_best_step(list(cost), list(byts), n, link, 1.0)
        assert got <= best * 1.001 + 1e-9, (trial, got, best, b)


def _balanced_bounds_py(band_cost, band_bytes, n: int, link_bytes_per_us: float, height: int,
                    band_rows: int = 32, unpack_us: float = 5.0):
    """Pure-Python restatement of the balanced split (the round-4 bench implementation), a
    cross-check of the C one (xrt_balanced_bounds) that both multi-GPU paths now share."""
    cost = [float(c) for c in band_cost]
    byts = [float(b) for b in band_bytes]
    nb = len(cost)
    if nb != len(byts) or nb == 0:
        raise ValueError("band_cost and band_bytes must have one entry per band")
    if n <= 1:
        return [(0, height)]
    if nb < n:
        raise ValueError("fewer bands than ranks")
    link = max(float(link_bytes_per_us), 1e-9)
    pre_c = [0.0]
    pre_b = [0.0]
    for c, b in zip(cost, byts):
        pre_c.append(pre_c[-1] + c)
        pre_b.append(pre_b[-1] + b)

    def sender_cost(i, j):            # bands [i, j) on one sender
        return max(pre_c[j] - pre_c[i], (pre_b[j] - pre_b[i]) / link)

    def pieces(i, j, step):           # fewest senders covering [i, j) within step (greedy); None: impossible
        k, a = 0, i
        while a < j:
            b = a + 1
            if sender_cost(a, b) > step:
                return None
            while b < j and sender_cost(a, b + 1) <= step:
                b += 1
            k, a = k + 1, b
        return k

    def plan(step):                   # (a, b): the root's run of bands, or None
        for a in range(nb):
            # the longest run from a within the step that leaves a band for every sender
            b = None
            for e in range(nb, a, -1):
                if a + (nb - e) >= n - 1 and pre_c[e] - pre_c[a] + unpack_us <= step:
                    b = e
                    break
            if b is None:
                continue
            ka, kb = pieces(0, a, step), pieces(b, nb, step)
            if ka is not None and kb is not None and ka + kb <= n - 1:
                return a, b           # the senders left over split pieces (never raises the step)
        return None

    lo, hi = 0.0, pre_c[nb] + unpack_us + pre_b[nb] / link
    root = plan(hi)
    for _ in range(60):
        mid = 0.5 * (lo + hi)
        r = plan(mid)
        if r is None:
            lo = mid
        else:
            hi, root = mid, r
    a, b = root
    # senders: greedy pieces within the step found, then split until n - 1 pieces
    step = hi

    def split(i, j):
        out, s0 = [], i
        while s0 < j:
            e = s0 + 1
            while e < j and sender_cost(s0, e + 1) <= step:
                e += 1
            out.append([s0, e])
            s0 = e
        return out
    above, below = split(0, a), split(b, nb)
    while len(above) + len(below) < n - 1:
        cand = [(sender_cost(x, y), k, side) for side, lst in ((0, above), (1, below))
                for k, (x, y) in enumerate(lst) if y - x >= 2]
        if not cand:
            raise ValueError("cannot give every rank a band")
        _, k, side = max(cand)
        lst = above if side == 0 else below
        x, y = lst[k]
        m = (x + y) // 2
        lst[k:k + 1] = [[x, m], [m, y]]
    rows = lambda band: min(band * band_rows, height)                        # noqa: E731
    return [(rows(a), rows(b))] + [(rows(x), rows(y)) for x, y in above + below]


def test_balanced_bounds_c_equals_python_restatement():
    """The C split (xrt_balanced_bounds, used by xrt_render_rows_multi and, through
    strips.balanced_bounds, by bench.py) gives the same strips as the pure-Python
    restatement, on random band models of 4-300 bands and 2-8 ranks."""
    from simpleraytracing_amd.strips import balanced_bounds
    rng = np.random.default_rng(11)
    for trial in range(60):
        nb = int(rng.integers(4, 300))
        n = int(rng.integers(2, min(nb, 8) + 1))
        cost = rng.uniform(0.0, 10.0, nb) * (rng.uniform(size=nb) > 0.2)
        byts = rng.uniform(0.0, 3e5, nb) * (rng.uniform(size=nb) > 0.3)
        link = float(rng.uniform(1e3, 2e5))
        H = 32 * nb - int(rng.integers(0, 31))
        want = _balanced_bounds_py(cost, byts, n, link, H, unpack_us=5.0)
        got = balanced_bounds(cost, byts, n, link, H, unpack_us=5.0)
        assert [tuple(x) for x in got] == [tuple(x) for x in want], (trial, got, want)


def _link_worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rate = bench.measure_link(dist, torch, world, rank, None, False, nbytes=1 << 16, reps=2)
    rates = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(rates, torch.tensor([rate], dtype=torch.float64))
    if rank == 0:
        np.save(out_path, np.array([float(r.item()) for r in rates]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("corrupt", [False, True])
def test_wrong_gathered_strip_fails_every_rank(corrupt):
    """bench.py's end of a strips run (bench.planes_equal + bench.gather_verdict)
    under torch.distributed.run, gloo, 2 ranks: an exact gather exits 0; one
    flipped L-buffer bit in rank 1's strip makes EVERY rank exit with
    bench.EXIT_GATHER_MISMATCH, so the launcher reports the job failed."""
    import subprocess
    import sys
    import bench
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "_gather_job.py")] + (["--corrupt"] if corrupt else [])
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    out = r.stdout + r.stderr
    if not corrupt:
        assert r.returncode == 0, out
        assert "rank 0 exit 0" in out and "rank 1 exit 0" in out
    else:
        assert r.returncode != 0, out
        code = bench.EXIT_GATHER_MISMATCH
        assert f"rank 0 exit {code}" in out and f"rank 1 exit {code}" in out, out
        assert "not bit-exact" in out


def test_frames_in_flight_rule():
    """bench.frames_in_flight: two frames in flight up to 2048^2 in frames mode,
    one above it and in strips mode; an explicit count wins, but strips mode
    takes only 1 and no count below 1 is accepted."""
    import bench
    assert bench.frames_in_flight(None, False, 2048, 2048) == 2
    assert bench.frames_in_flight(None, False, 1024, 1024) == 2
    assert bench.frames_in_flight(None, False, 4096, 4096) == 1
    assert bench.frames_in_flight(None, False, 8192, 8192) == 1
    assert bench.frames_in_flight(None, True, 2048, 2048) == 1
    assert bench.frames_in_flight(3, False, 4096, 4096) == 3
    assert bench.frames_in_flight(1, True, 4096, 4096) == 1
    with pytest.raises(SystemExit):
        bench.frames_in_flight(2, True, 4096, 4096)
    with pytest.raises(SystemExit):
        bench.frames_in_flight(0, False, 2048, 2048)


def test_bench_exits_nonzero_on_rank_exception():
    """bench.run(): an exception in main() leaves through os._exit(1) after its
    traceback (no hang in a collective or RCCL teardown)."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import bench\n"
            "def boom():\n    raise RuntimeError('rank failure')\n"
            "bench.main = boom\nbench.run()\nprint('not reached')\n") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1
    assert "rank failure" in r.stderr and "not reached" not in r.stdout


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_link_rate_agreed(tmp_path, world):
    """bench.measure_link under gloo: every sender sends to rank 0 at once, rank 0
    times it and every rank ends with the same positive rate (the balanced
    split is computed from it on rank 0 and broadcast)."""
    out = str(tmp_path / "rates.npy")
    mp.spawn(_link_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    rates = np.load(out)
    assert rates.shape == (world,) and rates[0] > 0 and np.all(rates == rates[0])
