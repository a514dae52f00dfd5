"""Row-strip partition and the packed strip layout gathered across ranks.

Partition: contiguous row strips, rows_per = H // n with the remainder going to
the first strips -- the rule of the reference's row-range pthreads renderer
(src/main-pthreads-rows.cxx:311-334) and of its pixel-range twin
(src/main-pthreads-redo.cxx:627-658).  Assembly: each rank renders its strip
into one packed byte buffer [image f32 | L-buffer f32 | u8] of the largest
strip's size, and one gather to rank 0 (RCCL over xGMI on GPUs, gloo in the CPU
tests) replaces the reference's MPI point-to-point root gather
(src/main-mpi.cxx:855-881).
"""
from __future__ import annotations

import numpy as np


def strip_bounds(height: int, n: int, rank: int):
    """[begin, end) image rows of strip `rank` of `n`."""
    if not 0 <= rank < n:
        raise ValueError("rank out of range")
    rows_per, rem = divmod(height, n)
    begin = rank * rows_per + min(rank, rem)
    end = begin + rows_per + (1 if rank < rem else 0)
    return begin, end


def root_share(n: int, rho: float = 2.5) -> float:
    """Fraction of the rows the gather's root renders itself.  Its rows need no
    transfer, the others' do: with rho = (transfer time / render time) per row of
    a sender's strip, the steps balance when the root takes rho / (rho + n - 1)
    (never less than 1/n).  rho = 2.5: a packed 4096-px row (~7.4 KB) over one
    xGMI link against ~27 ns of render per row (DESIGN.md "Multi-GPU")."""
    if n <= 1:
        return 1.0
    return max(1.0 / n, rho / (rho + n - 1))


def weighted_bounds(height: int, n: int, rank: int, share0: float):
    """[begin, end) rows of rank `rank`: rank 0 renders the first
    round(share0 * height) rows (at least its equal share, at most all but one
    row per other rank), the others split the rest as strip_bounds does."""
    if not 0 <= rank < n:
        raise ValueError("rank out of range")
    if n == 1:
        return 0, height
    r0 = int(round(share0 * height))
    r0 = min(max(r0, -(-height // n)), height - (n - 1))
    if rank == 0:
        return 0, r0
    b, e = strip_bounds(height - r0, n - 1, rank - 1)
    return r0 + b, r0 + e


def balanced_bounds(band_cost, band_bytes, n: int, link_bytes_per_us: float, height: int,
                    band_rows: int = 32, unpack_us: float = 5.0):
    """Row strips for a gather-bound frame: every rank's rows, [begin, end),
    from per-band costs (band = `band_rows` image rows, the region height, so
    each strip's region grid is the frame's): band_cost[b] = render time of
    band b (us), band_bytes[b] = the bytes its packed strip sends to rank 0.

    The root's own rows need no transfer, a sender's cost it max(render,
    bytes / link) on its own link, and frame k's gather overlaps frame k+1's
    render, so the step is the largest of: the root's render (+ the unpack),
    each sender's render and each sender's transfer.  The root takes ONE
    contiguous run of bands anywhere in the frame (the dense middle of the
    object, whose bytes would cost the most on a link); the senders split the
    bands above and below it into contiguous strips, in frame order (ranks 1..
    above, then below).  Every rank keeps at least one band.

    One implementation for both multi-GPU paths: this calls the C ABI's
    xrt_balanced_bounds, the split xrt_render_rows_multi plans with
    (simpleraytracing_amd/csrc/xrt_multi.inc, balanced_split)."""
    import ctypes

    from . import _abi
    cost = np.ascontiguousarray(band_cost, np.float64).reshape(-1)
    byts = np.ascontiguousarray(band_bytes, np.float64).reshape(-1)
    if cost.size != byts.size or cost.size == 0:
        raise ValueError("band_cost and band_bytes must have one entry per band")
    if n <= 1:
        return [(0, height)]
    if cost.size < n:
        raise ValueError("fewer bands than ranks")
    out = (ctypes.c_uint32 * (2 * n))()
    step = ctypes.c_double()
    dp = ctypes.POINTER(ctypes.c_double)
    rc = _abi.load().xrt_balanced_bounds(cost.ctypes.data_as(dp), byts.ctypes.data_as(dp), cost.size, n,
                                         float(link_bytes_per_us), height, band_rows, float(unpack_us), out,
                                         ctypes.byref(step))
    if rc != _abi.XRT_OK:
        raise ValueError(f"xrt_balanced_bounds failed ({rc})")
    return [(int(out[2 * g]), int(out[2 * g + 1])) for g in range(n)]


def gather_step_us(bounds, band_cost, band_bytes, link_bytes_per_us: float, band_rows: int = 32,
                   unpack_us: float = 5.0) -> float:
    """The step bounds imply under balanced_bounds' model (us)."""
    def band(r):
        return -(-r // band_rows)
    cost = [sum(band_cost[band(b0):band(e0)]) for b0, e0 in bounds]
    byts = [sum(band_bytes[band(b0):band(e0)]) for b0, e0 in bounds]
    return max([cost[0] + unpack_us] + [max(c, b / link_bytes_per_us) for c, b in zip(cost[1:], byts[1:])])


EMPTY = 0xFFFFFFFF


def unpack_descriptors(width: int, spans, maps):
    """Descriptors of xrt_unpack_blocks_device for the packed strips of `spans`
    ([begin, end) rows) with region maps `maps` (xrt_plan_region_map, one per
    strip): one (first row, rows, first column, block) per 32x32 region, the
    strips' packed blocks back to back in one buffer (at least one per strip:
    a strip with no unfilled region still sends one).  Returns (desc as an
    (n, 4) uint32 array, first block of each strip, total blocks)."""
    rows_out, bases, base = [], [], 0
    rx = -(-width // 32)
    for (b, e), m in zip(spans, maps):
        m = np.asarray(m, np.uint32)
        ry = -(-(e - b) // 32)
        if m.size != rx * ry:
            raise ValueError("region map does not match the strip")
        r = np.arange(m.size, dtype=np.uint64)
        y, x = r // rx, r % rx
        d = np.empty((m.size, 4), np.uint32)
        d[:, 0] = b + 32 * y
        d[:, 1] = np.minimum(32, (e - b) - 32 * y)
        d[:, 2] = 32 * x
        d[:, 3] = np.where(m == EMPTY, EMPTY, m.astype(np.uint64) + base).astype(np.uint32)
        rows_out.append(d)
        bases.append(base)
        base += max(int(np.count_nonzero(m != EMPTY)), 1)     # a strip with none still sends one block
    desc = np.concatenate(rows_out) if rows_out else np.zeros((0, 4), np.uint32)
    return desc, bases, base


def hit_descriptors(width: int, spans, maps, tile_hits):
    """Descriptors of xrt_unpack_hits_device for the hit-layout messages of
    `spans` ([begin, end) rows) with region maps `maps` (xrt_plan_region_map)
    and hit plans `tile_hits` (xrt_plan_hit_layout: the hit count of tile
    16 s + t of tile slot s), the strips' messages back to back in one buffer,
    each at a 16-B aligned word (a strip with no tile still sends 4 words).
    Returns (desc (n, 4) uint32 -- first row, rows, first column, index of the
    region's first tile descriptor or EMPTY --, tdesc (m, 4) uint32 -- mask
    word, first hit word, hit count, 0 per tile --, each strip's first word,
    each strip's message words, total words)."""
    rx = -(-width // 32)
    descs, tdescs, bases, words = [], [], [], []
    base, tbase = 0, 0
    for (b, e), m, h in zip(spans, maps, tile_hits):
        m = np.asarray(m, np.uint32)
        h = np.asarray(h, np.uint64)
        ry = -(-(e - b) // 32)
        if m.size != rx * ry:
            raise ValueError("region map does not match the strip")
        n_tiles = h.size
        if n_tiles != 16 * int(np.count_nonzero(m != EMPTY)):
            raise ValueError("hit plan does not match the region map")
        r = np.arange(m.size, dtype=np.uint64)
        y, x = r // rx, r % rx
        d = np.empty((m.size, 4), np.uint32)
        d[:, 0] = b + 32 * y
        d[:, 1] = np.minimum(32, (e - b) - 32 * y)
        d[:, 2] = 32 * x
        d[:, 3] = np.where(m == EMPTY, EMPTY, 16 * m.astype(np.uint64) + tbase).astype(np.uint32)
        off = np.concatenate([[0], np.cumsum(h)[:-1]]).astype(np.uint64) if n_tiles else np.zeros(0, np.uint64)
        t = np.zeros((n_tiles, 4), np.uint32)
        t[:, 0] = base + 2 * np.arange(n_tiles, dtype=np.uint64)
        t[:, 1] = base + 2 * n_tiles + off
        t[:, 2] = h
        descs.append(d)
        tdescs.append(t)
        bases.append(base)
        w = max(2 * n_tiles + int(h.sum()), 4)
        words.append(w)
        base += -(-w // 4) * 4
        tbase += n_tiles
    desc = np.concatenate(descs) if descs else np.zeros((0, 4), np.uint32)
    tdesc = np.concatenate(tdescs) if tdescs else np.zeros((0, 4), np.uint32)
    if tdesc.size == 0:
        tdesc = np.zeros((1, 4), np.uint32)
    return desc, tdesc, bases, words, base


def max_strip_pixels(width: int, height: int, n: int) -> int:
    b, e = strip_bounds(height, n, 0)
    return (e - b) * width


def packed_size(width: int, height: int, n: int) -> int:
    return 9 * max_strip_pixels(width, height, n)


def views(buf, n_max: int):
    """(image f32, lbuffer f32, u8) views into a packed strip buffer (torch or numpy)."""
    if hasattr(buf, "view") and not isinstance(buf, np.ndarray):   # torch tensor
        import torch
        return (buf[: 4 * n_max].view(torch.float32), buf[4 * n_max: 8 * n_max].view(torch.float32),
                buf[8 * n_max: 9 * n_max])
    return (buf[: 4 * n_max].view(np.float32), buf[4 * n_max: 8 * n_max].view(np.float32),
            buf[8 * n_max: 9 * n_max])


def assemble(gathered, width: int, height: int):
    """Concatenates gathered packed strips (numpy uint8 arrays, rank order) into
    full-frame (image, lbuffer, u8)."""
    n = len(gathered)
    n_max = max_strip_pixels(width, height, n)
    img = np.empty(width * height, np.float32)
    lb = np.empty(width * height, np.float32)
    u8 = np.empty(width * height, np.uint8)
    for r, buf in enumerate(gathered):
        b, e = strip_bounds(height, n, r)
        cnt = (e - b) * width
        i, l, u = views(np.asarray(buf), n_max)
        img[b * width: e * width] = i[:cnt]
        lb[b * width: e * width] = l[:cnt]
        u8[b * width: e * width] = u[:cnt]
    return img, lb, u8
