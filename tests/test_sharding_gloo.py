"""Multi-GPU path on CPU: world_size-2 gloo runs of the band sharding + sum-reduce frame assembly
(gpu_bidirectional_raytracer_amd.sharding).  Each rank renders its own bands through the PRODUCT:
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


def _worker(rank, world, port, out_dir, band, scene):
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


@pytest.mark.parametrize("band,scene", [(4, "cornell_glass"), (8, "cornell")])
def test_gloo_world2_frame_assembly(tmp_path, band, scene):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), band, scene), nprocs=2, join=True)
    assert (tmp_path / "result").read_text() == "ok"
