"""Pixel-band sharding of one frame over the GPUs of a node, and the frame assembly.

The reference is single-GPU (smallpt_cpu.c:422).  Here every rank renders the rows whose band
(y // band_rows) is congruent to its rank modulo the world size -- the same rule the path kernel
applies (bdpt_set_shard) -- and leaves every other pixel at zero.  The only exchange is the
assembly of the frame on one rank (torch.distributed: "nccl" = RCCL over xGMI on MI355X, "gloo"
on CPU), in one of two exact forms:
* gather_frame: every rank packs its own rows (radiance and counter, 16 B per pixel) and the
  destination receives each peer's 1/N of the frame over that peer's link and copies it into
  place -- (N-1)/N of one frame into the destination, point to point;
* reduce_frame: a sum-reduce of the zero-padded frames (each pixel is non-zero on exactly one
  rank, and x + 0 == x) -- a ring moves about twice the frame over every link.
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


def gather_frame(t_col, t_cnt, width: int, height: int, band_rows: int, dst: int = 0,
                 nshards: int | None = None) -> None:
    """Assemble the frame on `dst` from every rank's own rows (exact: copies).  t_col (float32,
    W*H*3) and t_cnt (int32, W*H) are this rank's zero-padded frame; rank r owns the bands of
    shard r of `nshards` (default: the world size; weak64's fixed bands: 8); on `dst` the peers'
    rows are written into them.  One gather of a packed [rows][W*4] int32 buffer per rank (radiance bits
    and counter side by side, padded to the largest rank's row count); a gloo group with device
    tensors (multi-rank rehearsals on one GPU) stages it through host memory."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(), dist.get_world_size()
    rows = [owned_rows(height, r, nshards or world, band_rows) for r in range(world)]
    m = max(len(x) for x in rows)
    col2 = t_col.view(height, 3 * width)
    cnt2 = t_cnt.view(height, width)
    dev = t_col.device
    idx = torch.tensor(rows[rank], dtype=torch.long, device=dev)
    pack = torch.zeros((m, 4 * width), dtype=torch.int32, device=dev)
    if len(rows[rank]):
        pack[:len(rows[rank]), :3 * width] = col2.index_select(0, idx).view(torch.int32)
        pack[:len(rows[rank]), 3 * width:] = cnt2.index_select(0, idx)
    stage = t_col.is_cuda and dist.get_backend() == "gloo"
    send = pack.cpu() if stage else pack
    got = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, got, dst=dst)
    if rank != dst:
        return
    for r in range(world):
        if r == dst or not rows[r]:
            continue                                         # dst's own rows are in place
        g = got[r].to(dev) if stage else got[r]
        ri = torch.tensor(rows[r], dtype=torch.long, device=dev)
        col2.index_copy_(0, ri, g[:len(rows[r]), :3 * width].contiguous().view(torch.float32))
        cnt2.index_copy_(0, ri, g[:len(rows[r]), 3 * width:].contiguous())
