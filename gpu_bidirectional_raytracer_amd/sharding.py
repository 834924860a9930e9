"""Pixel-band sharding of one frame over the GPUs of a node, and the frame assembly.

The reference is single-GPU (smallpt_cpu.c:422).  Here every rank renders the rows whose band
(y // band_rows) is congruent to its rank modulo the world size -- the same rule the path kernel
applies (bdpt_set_shard) -- and leaves every other pixel at zero.  The only exchange is the
assembly of the frame: a sum-reduce (torch.distributed, "nccl" = RCCL over xGMI on MI355X, "gloo"
on CPU) of the float radiance and the counters to one rank, which is exact because each pixel is
non-zero on exactly one rank (x + 0 == x).
"""
from __future__ import annotations

from typing import List


def band_owner(y: int, world: int, band_rows: int) -> int:
    return (y // band_rows) % world


def owned_rows(height: int, rank: int, world: int, band_rows: int) -> List[int]:
    return [y for y in range(height) if band_owner(y, world, band_rows) == rank]


def owned_row_ranges(height: int, rank: int, world: int, band_rows: int):
    """[(y0, y1), ...] half-open bands of `rank`."""
    return [(y0, min(height, y0 + band_rows)) for y0 in range(0, height, band_rows)
            if band_owner(y0, world, band_rows) == rank]


def owned_pixels(width: int, height: int, rank: int, world: int, band_rows: int) -> int:
    return width * sum(y1 - y0 for y0, y1 in owned_row_ranges(height, rank, world, band_rows))


class _DeviceArray:
    """__cuda_array_interface__ view of a device pointer owned by libbdpt (no copy)."""

    def __init__(self, ptr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False),
                                         "version": 3}


def device_tensors(renderer, device):
    """torch tensors aliasing the renderer's colors (float32, W*H*3) and counter (int32, W*H)."""
    import torch

    col_ptr, cnt_ptr, _ = renderer.device_buffers()
    n = renderer.width * renderer.height
    t_col = torch.as_tensor(_DeviceArray(col_ptr, 3 * n, "<f4"), device=device)
    t_cnt = torch.as_tensor(_DeviceArray(cnt_ptr, n, "<i4"), device=device)
    return t_col, t_cnt


def reduce_frame(t_col, t_cnt, dst: int = 0) -> None:
    """Sum-reduce the zero-padded per-rank frames to `dst` (exact: disjoint pixel support).
    RCCL ("nccl") reduces the device buffers in place; a gloo group (CPU tests, multi-rank
    rehearsals on one GPU) stages them through host memory."""
    import torch.distributed as dist

    for t in (t_col, t_cnt):
        if t.is_cuda and dist.get_backend() == "gloo":
            h = t.cpu()
            dist.reduce(h, dst=dst, op=dist.ReduceOp.SUM)
            if dist.get_rank() == dst:
                t.copy_(h)
        else:
            dist.reduce(t, dst=dst, op=dist.ReduceOp.SUM)
