"""Multi-GPU path on CPU: world_size-2 gloo runs of the band sharding + frame assembly (sum-reduce
or gather of owned rows, gpu_bidirectional_raytracer_amd.sharding).  Each rank renders its own bands through the PRODUCT:
a C-ABI context on the host-CPU backend (bdpt_create(..., BDPT_DEVICE_CPU)) with bdpt_set_shard,
the same band rule the GPU kernel applies; every rank checks its ownership (rendered bands at the
full count, zeros elsewhere) and rank 0 compares the reduced frame with the oracle's full frame bit
for bit (4-row bands on cornell_glass, and bench.py's 8-row bands on cornell)."""
import os
import socket

import numpy as np
import pytest

from gpu_bidirectional_raytracer_amd import sharding as shd


def test_band_partition_covers_every_row_once():
    for H, world, band in [(1081, 2, 16), (1081, 8, 16), (513, 4, 64), (7, 3, 1), (5, 8, 16)]:
        seen = np.zeros(H, int)
        for r in range(world):
            for y in shd.owned_rows(H, r, world, band):
                seen[y] += 1
            assert shd.owned_pixels(3, H, r, world, band) == 3 * len(shd.owned_rows(H, r, world, band))
        assert (seen == 1).all()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, band, scene, assembly="reduce"):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BDPT_CPU_THREADS="2")
    import torch
    import torch.distributed as dist
    import gpu_bidirectional_raytracer_amd as g
    import oracle
    from gpu_bidirectional_raytracer_amd import sharding as shd

    dist.init_process_group("gloo", rank=rank, world_size=world)
    scn = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets", "scenes",
                       scene + ".scn")
    W, H = 29, 37
    cam, sp = g.read_scene(scn)
    g.update_camera(cam, W, H)
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(4)
    with g.Renderer(sp, W, H, cam, device=-1) as r:          # the product, host-CPU backend
        r.set_shard(rank, world, band)
        r.light_pass(0)
        r.path_passes(sid, vlp)
        col, cnt = r.read_radiance()
    owned = (np.arange(H) // band) % world == rank
    local_ok = (cnt[owned] == len(sid)).all() and (cnt[~owned] == 0).all() and (col[~owned] == 0).all()
    t_col = torch.from_numpy(col.reshape(-1).copy())
    t_cnt = torch.from_numpy(cnt.reshape(-1).astype(np.int32))
    if assembly == "gather":
        shd.gather_frame(t_col, t_cnt, W, H, band, dst=0)
    else:
        shd.reduce_frame(t_col, t_cnt, dst=0)
    flags = torch.tensor([int(local_ok)])
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    if rank == 0:
        rnd = oracle.mt607(0)
        lp = oracle.light_pass(sp, rnd, 0)
        full, fcnt, _ = oracle.path_passes(sp, rnd, cam, W, H, lp, sid, vlp, nthreads=1)
        ok = bool(flags.item()) and np.array_equal(t_col.numpy().reshape(H, W, 3).view(np.uint32),
                                                  full.view(np.uint32)) and \
            np.array_equal(t_cnt.numpy().reshape(H, W), fcnt.astype(np.int32))
        open(os.path.join(out_dir, "result"), "w").write("ok" if ok else "mismatch")
    dist.destroy_process_group()


@pytest.mark.parametrize("band,scene,assembly", [(4, "cornell_glass", "reduce"), (8, "cornell", "reduce"),
                                                 (8, "cornell", "gather"), (3, "caustic", "gather")])
def test_gloo_world2_frame_assembly(tmp_path, band, scene, assembly):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), band, scene, assembly), nprocs=2, join=True)
    assert (tmp_path / "result").read_text() == "ok"


def _gather_worker(rank, world, port, out_dir, W, H, band, nshards):
    """gather_frame on synthetic frames: rank r's shard-r rows hold distinct bit patterns (NaN
    payloads and -0 included, so the assembly must copy bits, not add), other rows 0."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from gpu_bidirectional_raytracer_amd import sharding as shd

    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(7)
    bits = rng.integers(0, 2**32, size=(world, H, W * 3), dtype=np.uint64).astype(np.uint32)
    cnts = rng.integers(0, 30000, size=(world, H, W), dtype=np.int64).astype(np.int32)
    owner = (np.arange(H) // band) % (nshards or world)
    col = np.zeros((H, W * 3), np.uint32)
    cnt = np.zeros((H, W), np.int32)
    col[owner == rank] = bits[rank][owner == rank]
    cnt[owner == rank] = cnts[rank][owner == rank]
    t_col = torch.from_numpy(col.view(np.float32).reshape(-1).copy())
    t_cnt = torch.from_numpy(cnt.reshape(-1).copy())
    shd.gather_frame(t_col, t_cnt, W, H, band, dst=0, nshards=nshards)
    if rank == 0:
        want_col = np.zeros_like(col)
        want_cnt = np.zeros_like(cnt)
        for r in range(world):
            want_col[owner == r] = bits[r][owner == r]
            want_cnt[owner == r] = cnts[r][owner == r]
        ok = np.array_equal(t_col.numpy().view(np.uint32).reshape(H, W * 3), want_col) and \
            np.array_equal(t_cnt.numpy().reshape(H, W), want_cnt)
        open(os.path.join(out_dir, "result"), "w").write("ok" if ok else "mismatch")
    dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,band,nshards", [(2, 13, 37, 8, None), (3, 5, 29, 4, None),
                                                    (2, 7, 41, 5, 8), (4, 3, 9, 1, None)])
def test_gloo_gather_frame_bits(tmp_path, world, W, H, band, nshards):
    """Every rank's rows land on rank 0 bit for bit, for uneven row counts per rank (padding),
    ranks without rows, and fixed bands with fewer ranks than shards (weak64's rule)."""
    pytest.importorskip("torch")
    import torch.multiprocessing as mp
    mp.spawn(_gather_worker, args=(world, _free_port(), str(tmp_path), W, H, band, nshards),
             nprocs=world, join=True)
    assert (tmp_path / "result").read_text() == "ok"
