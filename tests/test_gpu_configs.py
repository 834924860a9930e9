"""BASELINE.json configs at their full sizes (internal = CLI + 1), on one GPU.

configs[1] cornell 513x513, 256 spp      -> whole frame bit-exact vs the oracle
configs[2] cornell_glass 1921x1081, 1024 spp -> counters, pixel = toInt(colors), oracle rows
configs[3] caustic 1921x1081, 4096 spp on 8 pixel-band shards -> shard sum == one-context
           frame bit for bit (the RCCL reduce is a sum of disjoint frames), oracle rows
configs[4] synthetic64 4097x4097 -> one 4097x512 band (what one of 8 GPUs renders) at the
           full 8192 spp (vlp_index wraps inside the run): ownership, counters, oracle spans
"""
import os

import numpy as np
import pytest

import gpu_bidirectional_raytracer_amd as g
import oracle
from conftest import SCENES

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rnd0():
    return oracle.mt607(0)


def _setup(name, W, H, gpu):
    cam, sp = g.read_scene(os.path.join(SCENES, name + ".scn"))
    g.update_camera(cam, W, H)
    r = g.Renderer(sp, W, H, cam, device=gpu)
    r.light_pass(0)
    return r, cam, sp


def _schedule(n):
    s = g.PassScheduler()
    s.light()
    return s.next(n)


def _same(a, b, what):
    if a.dtype.kind == "f":
        a, b = a.view(np.uint32), b.view(np.uint32)
    bad = np.argwhere(a != b)
    assert bad.size == 0, f"{what}: {len(bad)} mismatches, first at {bad[:3].tolist()}"


def _pixels_are_toint(r, col):
    thr = np.zeros(256, np.float32)
    g._lib.lib.bdpt_gamma_thresholds(g._lib.ctypes.c_void_p(thr.ctypes.data))
    k = np.searchsorted(thr, col.reshape(-1), side="right").reshape(col.shape) - 1
    _same(r.read_pixels()[..., :3], k.astype(np.uint8), "pixels vs toInt(colors)")


def test_config1_cornell_513_256spp_full_frame(gpu, rnd0):
    W, H, spp = 513, 513, 256
    r, cam, sp = _setup("cornell", W, H, gpu)
    sid, vlp = _schedule(spp)
    r.path_passes(sid, vlp)
    col, cnt = r.read_radiance()
    lp = oracle.light_pass(sp, rnd0, 0)
    ocol, ocnt, opix = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)
    _same(cnt, ocnt, "counter")
    _same(col, ocol, "colors")
    _same(r.read_pixels(), opix, "pixels")
    r.close()


def test_config2_cornell_glass_1080p_1024spp(gpu, rnd0):
    W, H, spp = 1921, 1081, 1024
    r, cam, sp = _setup("cornell_glass", W, H, gpu)
    sid, vlp = _schedule(spp)
    r.path_passes(sid, vlp)
    col, cnt = r.read_radiance()
    assert (cnt == spp).all() and np.isfinite(col).all() and (col >= 0).all()
    _pixels_are_toint(r, col)
    lp = oracle.light_pass(sp, rnd0, 0)
    for y in (0, 523, 1080):
        ocol, _, _ = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp, rows=(y, y + 1))
        _same(col[y], ocol[y], f"row {y}")
    r.close()


def test_config3_caustic_1080p_4096spp_8_shards(gpu, rnd0):
    W, H, spp, N = 1921, 1081, 4096, 8
    sid, vlp = _schedule(spp)
    full, cam, sp = _setup("caustic", W, H, gpu)
    full.path_passes(sid, vlp)
    fc, fn = full.read_radiance()
    full.close()
    acc_c, acc_n = np.zeros_like(fc), np.zeros_like(fn)
    for rank in range(N):
        r, _, _ = _setup("caustic", W, H, gpu)
        r.set_shard(rank, N, 8)
        r.path_passes(sid, vlp)
        assert r.last_streams > 1                        # a 1/8 band uses pass streams
        c, n = r.read_radiance()
        owned = (np.arange(H) // 8) % N == rank
        assert (n[owned] == spp).all() and (n[~owned] == 0).all() and (c[~owned] == 0).all()
        acc_c += c
        acc_n += n
        r.close()
    _same(acc_c, fc, "shard sum colors")
    _same(acc_n, fn, "shard sum counters")
    lp = oracle.light_pass(sp, rnd0, 0)
    for y in (0, 700):
        ocol, _, _ = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp, rows=(y, y + 1))
        _same(fc[y], ocol[y], f"row {y}")


def test_config4_synthetic64_4097_band_8192spp(gpu, rnd0):
    """configs[4] as one GPU of the 8-GPU weak-scaling run renders it (bench.py --workload weak64):
    the 64-sphere synthetic scene at 4097x4097, one 4097x512 band (rank 3 of 8 fixed bands), the
    full 8192 spp -- so vlp_index wraps past LIGHT_POINTS inside the run (pass 8190, SURVEY
    Appendix A.3).  Counters and ownership over the frame, oracle spot checks on 4 pixel spans
    at the full spp."""
    W, H, spp, N, rank, band = 4097, 4097, 8192, 8, 3, 512
    r, cam, sp = _setup("synthetic64", W, H, gpu)
    assert len(sp) == 64
    r.set_shard(rank, N, band)
    sid, vlp = _schedule(spp)
    assert vlp[8189] == 4095 and vlp[8190] == 0
    r.path_passes(sid, vlp)
    col, cnt = r.read_radiance()
    owned = (np.arange(H) // band) % N == rank
    assert (cnt[owned] == spp).all() and (cnt[~owned] == 0).all()
    assert np.isfinite(col).all() and (col[~owned] == 0).all()
    _pixels_are_toint(r, col)
    lp = oracle.light_pass(sp, rnd0, 0)
    y0 = rank * band
    for y, x in ((y0, 0), (y0 + 200, 2000), (y0 + 377, 4000), (y0 + band - 1, 1500)):
        p0 = y * W + x
        p1 = min(p0 + 96, (y + 1) * W)
        ocol, ocnt, _ = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp, span=(p0, p1))
        _same(col.reshape(-1, 3)[p0:p1], ocol.reshape(-1, 3)[p0:p1], f"pixels {p0}..{p1}")
        _same(cnt.reshape(-1)[p0:p1], ocnt.reshape(-1)[p0:p1], f"counters {p0}..{p1}")
    r.close()
