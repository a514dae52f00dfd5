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
