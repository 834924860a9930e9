"""The fused S = 1 kernel's variants against the oracle, bit for bit: grouped path regeneration
(BDPT_REGEN_K, default 48 lanes; 1 = restart at once, 64 = whole-wave lockstep) and paired segment
loads (BDPT_RNG_PAIR, which the auto stream mode switches off where it measures slower).
Each variant is a scene-specialised build selected through BDPT_JIT_FLAGS (its own JIT cache
entry); the pass order of every pixel, and so its running mean, must be unchanged."""
import os

import numpy as np
import pytest

import gpu_bidirectional_raytracer_amd as g
import oracle
from conftest import SCENES

pytestmark = pytest.mark.gpu

VARIANTS = ["", "-DBDPT_RNG_PAIR=0", "-DBDPT_REGEN_K=1", "-DBDPT_REGEN_K=64"]


@pytest.fixture(scope="module")
def rnd0():
    return oracle.mt607(0)


@pytest.mark.parametrize("flags", VARIANTS)
@pytest.mark.parametrize("name", ["caustic", "open", "cornell_glass", "hall_of_mirrors"])
def test_fused_variant_matches_oracle(gpu, rnd0, name, flags, monkeypatch):
    if flags:
        monkeypatch.setenv("BDPT_JIT_FLAGS", flags)
    else:
        monkeypatch.delenv("BDPT_JIT_FLAGS", raising=False)
    W, H, npass = 47, 35, 24
    cam, sp = g.read_scene(os.path.join(SCENES, name + ".scn"))
    g.update_camera(cam, W, H)
    r = g.Renderer(sp, W, H, cam, device=gpu)
    r.light_pass(0)
    r.set_streams(1)
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(npass)
    r.path_passes(sid[:10], vlp[:10])                     # two calls: the counters carry over
    r.path_passes(sid[10:], vlp[10:])
    assert r.last_streams == 1 and r.last_specialized
    col, cnt = r.read_radiance()
    px = r.read_pixels()
    r.close()
    lp = oracle.light_pass(sp, rnd0, 0)
    ocol, ocnt, opx = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)
    assert np.array_equal(cnt, ocnt)
    assert np.array_equal(col.view(np.uint32), ocol.view(np.uint32)), \
        f"{name} [{flags}]: {int((col != ocol).sum())} values differ"
    assert np.array_equal(px, opx)
