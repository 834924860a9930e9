"""Pass streams with pixel pools (bdpt_kernels.hip BDPT_POOL; forced here with BDPT_POOL=R, the
auto stream mode measures them): a wave renders one pass and restarts lanes on new pixels of
it, claimed in chunks of R x 64 from the pass's eight counters (BDPT_POOL_GRID=G: G x 64 pixels
per wave and pass).  Every pixel must still get exactly its passes, in pass order through the
fold, so the frame is the oracle's bit for bit -- whole frames, two calls (the counters carry
over), chunks larger than the frame, more waves than chunks (waves that find their pass
drained), and shards whose bands are whole tile rows (the grid enumerates only them) or not
(pixels of other shards inside a chunk are passed over)."""
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


def _oracle(name, W, H, sid, vlp, rnd0):
    cam, sp = g.read_scene(os.path.join(SCENES, name + ".scn"))
    g.update_camera(cam, W, H)
    lp = oracle.light_pass(sp, rnd0, 0)
    return oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)


def _render(name, W, H, sid, vlp, split, shard=None):
    cam, sp = g.read_scene(os.path.join(SCENES, name + ".scn"))
    g.update_camera(cam, W, H)
    with g.Renderer(sp, W, H, cam, device=0) as r:
        if shard:
            r.set_shard(*shard)
        r.set_streams(len(sid))
        r.light_pass(0)
        r.path_passes(sid[:split], vlp[:split])
        r.path_passes(sid[split:], vlp[split:])
        assert r.last_streams > 1 and r.last_specialized, r.specialize_status
        assert "pixel_pools" in r.last_features, r.last_features
        col, cnt = r.read_radiance()
        px = r.read_pixels()
    return col, cnt, px


@pytest.mark.parametrize("pool,grid", [(1, 16), (4, 16), (16, 16), (4, 1), (2, 64)])
@pytest.mark.parametrize("name", ["cornell", "caustic", "cornell_glass", "synthetic64"])
def test_pool_matches_oracle(gpu, rnd0, name, pool, grid, monkeypatch):
    monkeypatch.setenv("BDPT_POOL", str(pool))
    monkeypatch.setenv("BDPT_POOL_GRID", str(grid))
    W, H, npass = 47, 35, 16
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(npass)
    col, cnt, px = _render(name, W, H, sid, vlp, 6)
    ocol, ocnt, opx = _oracle(name, W, H, sid, vlp, rnd0)
    assert np.array_equal(cnt, ocnt)
    assert np.array_equal(col.view(np.uint32), ocol.view(np.uint32)), \
        f"{name} pool {pool} grid {grid}: {int((col != ocol).sum())} values differ"
    assert np.array_equal(px, opx)


@pytest.mark.parametrize("band", [8, 5])
def test_pool_shard_matches_oracle(gpu, rnd0, band, monkeypatch):
    monkeypatch.setenv("BDPT_POOL", "4")
    W, H, npass, N, rank = 83, 61, 12, 3, 1
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(npass)
    col, cnt, px = _render("cornell", W, H, sid, vlp, 5, shard=(rank, N, band))
    ocol, ocnt, opx = _oracle("cornell", W, H, sid, vlp, rnd0)
    owned = (np.arange(H) // band) % N == rank
    assert (cnt[owned] == npass).all() and (cnt[~owned] == 0).all() and (col[~owned] == 0).all()
    assert np.array_equal(col[owned].view(np.uint32), ocol[owned].view(np.uint32))


@pytest.mark.parametrize("name", ["caustic", "cornell"])
def test_pool_long_call_sparse_fold(gpu, rnd0, name, monkeypatch):
    """One call of 200 passes = two pooled launches of 100 (all four mask words of a pixel, and a
    fold tail of 100 mod 16 passes); caustic's samples are mostly +0 (sparse radiance)."""
    monkeypatch.setenv("BDPT_POOL", "4")
    W, H, npass = 31, 17, 200
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(npass)
    cam, sp = g.read_scene(os.path.join(SCENES, name + ".scn"))
    g.update_camera(cam, W, H)
    with g.Renderer(sp, W, H, cam, device=0) as r:
        r.set_streams(128)
        r.light_pass(0)
        r.path_passes(sid, vlp)
        assert "pixel_pools" in r.last_features, r.last_features
        col, cnt = r.read_radiance()
    ocol, ocnt, _ = _oracle(name, W, H, sid, vlp, rnd0)
    assert np.array_equal(cnt, ocnt)
    assert np.array_equal(col.view(np.uint32), ocol.view(np.uint32))


def test_pool_counter_cap(gpu, rnd0, monkeypatch):
    """Pooled launches across the 30000-pass counter cap: passes past it are neither rendered nor
    folded (their mask bits stay clear and the fold stops at the cap)."""
    monkeypatch.setenv("BDPT_POOL", "4")
    W, H = 5, 3
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(30004)
    cam, sp = g.read_scene(os.path.join(SCENES, "caustic.scn"))
    g.update_camera(cam, W, H)
    with g.Renderer(sp, W, H, cam, device=0) as r:
        r.set_streams(128)
        r.light_pass(0)
        r.path_passes(sid[:29950], vlp[:29950])
        r.path_passes(sid[29950:], vlp[29950:])               # the cap falls inside this call
        assert "pixel_pools" in r.last_features, r.last_features
        col, cnt = r.read_radiance()
    assert (cnt == 30000).all()
    ocol, ocnt, _ = _oracle("caustic", W, H, sid, vlp, rnd0)
    assert np.array_equal(col.view(np.uint32), ocol.view(np.uint32))


def test_pool_overlapped_launches_then_write_lightpaths(gpu, rnd0, monkeypatch):
    """bdpt_write_lightpaths right after overlapped pooled launches (they run on the pool streams,
    which the context's stream follows only through the last fold): the copy must wait for them,
    so the first call's passes see the old VLPs and the next call's the new ones."""
    monkeypatch.setenv("BDPT_POOL", "16")
    W, H, n1, n2 = 161, 97, 256, 32
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(n1 + n2)
    cam, sp = g.read_scene(os.path.join(SCENES, "cornell.scn"))
    g.update_camera(cam, W, H)
    with g.Renderer(sp, W, H, cam, device=0) as r:
        r.set_streams(128)
        r.light_pass(0)
        lp1 = r.read_lightpaths()
        lp2 = lp1.copy()
        lp2["rad"] *= np.float32(0.5)
        r.path_passes(sid[:n1], vlp[:n1], sync=False)    # two launches of 128, left running
        r.write_lightpaths(lp2)
        r.path_passes(sid[n1:], vlp[n1:])
        assert "pixel_pools" in r.last_features, r.last_features
        col, cnt = r.read_radiance()
    olp = oracle.light_pass(sp, rnd0, 0)
    assert olp.tobytes() == lp1.tobytes()
    ocol, ocnt, _ = oracle.path_passes(sp, rnd0, cam, W, H, olp, sid[:n1], vlp[:n1])
    ocol, ocnt, _ = oracle.path_passes(sp, rnd0, cam, W, H, lp2, sid[n1:], vlp[n1:], colors=ocol, counter=ocnt)
    assert np.array_equal(cnt, ocnt)
    assert np.array_equal(col.view(np.uint32), ocol.view(np.uint32))
