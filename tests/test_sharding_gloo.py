"""Multi-GPU path on CPU: world_size-2 gloo run of the band sharding + sum-reduce frame assembly
(gpu_bidirectional_raytracer_amd.sharding), with the oracle rendering each rank's bands."""
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


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import oracle
    from golden.make_golden import read_scene_py  # noqa: E402
    from gpu_bidirectional_raytracer_amd import sharding as shd

    dist.init_process_group("gloo", rank=rank, world_size=world)
    scn = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets", "scenes",
                       "cornell_glass.scn")
    orig, target, sp = read_scene_py(scn)
    W, H, band = 29, 37, 4
    cam = oracle.update_camera(orig, target, W, H)
    rnd = oracle.mt607(0)
    lp = oracle.light_pass(sp, rnd, 0)
    sid, vlp = [5, 77777, 123456, 4242424], [1, 1, 2, 2]
    col = np.zeros((H, W, 3), np.float32)
    cnt = np.zeros((H, W), np.uint32)
    for y0, y1 in shd.owned_row_ranges(H, rank, world, band):
        col, cnt, _ = oracle.path_passes(sp, rnd, cam, W, H, lp, sid, vlp, colors=col, counter=cnt,
                                         rows=(y0, y1), nthreads=1)
    t_col = torch.from_numpy(col.reshape(-1).copy())
    t_cnt = torch.from_numpy(cnt.reshape(-1).astype(np.int32))
    shd.reduce_frame(t_col, t_cnt, dst=0)
    if rank == 0:
        full, fcnt, _ = oracle.path_passes(sp, rnd, cam, W, H, lp, sid, vlp, nthreads=1)
        ok = np.array_equal(t_col.numpy().reshape(H, W, 3), full) and \
            np.array_equal(t_cnt.numpy().reshape(H, W), fcnt.astype(np.int32))
        open(os.path.join(out_dir, "result"), "w").write("ok" if ok else "mismatch")
    dist.destroy_process_group()


def test_gloo_world2_frame_assembly(tmp_path):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert (tmp_path / "result").read_text() == "ok"
