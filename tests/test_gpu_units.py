"""Pass streams with the ordered fold inside the kernel (bdpt_kernels.hip BDPT_UNITS; forced here
with BDPT_UNITS=P): a workgroup renders one unit = (32x8 tile, range of P passes), one lane per
pixel, the passes of the range in order with the running mean in registers; the units of a tile
run in range order (per-wave-tile flags, agent-scope coherent loads / stores), so there is no
radiance buffer and no fold kernel.  Every pixel must get exactly its passes in pass order: the
frame is the oracle's bit for bit -- whole frames, two calls (the counters carry over), ranges of
1 pass to the whole launch, frames whose edges are packed into full waves (65 = 2 x 32 + 1,
49 = 6 x 8 + 1), frames of a few hundred workgroups per range (the handover is exercised), and
shards whose bands are whole tile rows (the grid enumerates only them) or not."""
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


def _oracle(name, W, H, sid, vlp, rnd0, rows=None):
    cam, sp = g.read_scene(os.path.join(SCENES, name + ".scn"))
    g.update_camera(cam, W, H)
    lp = oracle.light_pass(sp, rnd0, 0)
    return oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp, rows=rows)


def _render(name, W, H, sid, vlp, split, shard=None, streams=None):
    cam, sp = g.read_scene(os.path.join(SCENES, name + ".scn"))
    g.update_camera(cam, W, H)
    with g.Renderer(sp, W, H, cam, device=0) as r:
        if shard:
            r.set_shard(*shard)
        r.set_streams(streams or len(sid))
        r.light_pass(0)
        r.path_passes(sid[:split], vlp[:split])
        r.path_passes(sid[split:], vlp[split:])
        assert r.last_streams > 1 and r.last_specialized, r.specialize_status
        assert "unit_fold" in r.last_features, r.last_features
        col, cnt = r.read_radiance()
        px = r.read_pixels()
    return col, cnt, px


def _same(got, want, what):
    col, cnt, px = got
    ocol, ocnt, opx = want
    assert np.array_equal(cnt, ocnt), what
    assert np.array_equal(col.view(np.uint32), ocol.view(np.uint32)), \
        f"{what}: {int((col != ocol).sum())} values differ"
    assert np.array_equal(px, opx), what


@pytest.mark.parametrize("P", [1, 3, 16])
@pytest.mark.parametrize("name", ["cornell", "caustic", "cornell_glass", "synthetic64"])
def test_units_match_oracle(gpu, rnd0, name, P, monkeypatch):
    monkeypatch.setenv("BDPT_UNITS", str(P))
    W, H, npass = 47, 35, 16
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(npass)
    _same(_render(name, W, H, sid, vlp, 6), _oracle(name, W, H, sid, vlp, rnd0), f"{name} P={P}")


@pytest.mark.parametrize("W,H", [(65, 49), (33, 9)])
def test_units_packed_edges(gpu, rnd0, W, H, monkeypatch):
    monkeypatch.setenv("BDPT_UNITS", "2")
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(10)
    _same(_render("cornell", W, H, sid, vlp, 4), _oracle("cornell", W, H, sid, vlp, rnd0), f"{W}x{H}")


def test_units_many_workgroups(gpu, rnd0, monkeypatch):
    """321 x 241 = 11 x 31 tile workgroups per range, 24 passes in ranges of 4 (6 ranges, two
    calls): many units of a tile follow each other; checked on every 6th row against the oracle."""
    monkeypatch.setenv("BDPT_UNITS", "4")
    W, H = 321, 241
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(24)
    col, cnt, px = _render("caustic", W, H, sid, vlp, 8, streams=12)
    assert (cnt == 24).all()
    rows = list(range(0, H, 6))
    for y in rows[:12]:
        ocol, ocnt, opx = _oracle("caustic", W, H, sid, vlp, rnd0, rows=(y, y + 1))
        assert np.array_equal(col[y].view(np.uint32), ocol[y].view(np.uint32)), f"row {y}"
        assert np.array_equal(px[y], opx[y]), f"row {y}"


@pytest.mark.parametrize("band", [8, 5])
def test_units_shard_matches_oracle(gpu, rnd0, band, monkeypatch):
    monkeypatch.setenv("BDPT_UNITS", "3")
    W, H, npass, N, rank = 83, 61, 12, 3, 1
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(npass)
    col, cnt, px = _render("cornell", W, H, sid, vlp, 5, shard=(rank, N, band))
    ocol, ocnt, opx = _oracle("cornell", W, H, sid, vlp, rnd0)
    owned = (np.arange(H) // band) % N == rank
    assert (cnt[owned] == npass).all() and (cnt[~owned] == 0).all() and (col[~owned] == 0).all()
    assert np.array_equal(col[owned].view(np.uint32), ocol[owned].view(np.uint32))
