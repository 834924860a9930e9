"""The host-CPU backend (bdpt_create(..., BDPT_DEVICE_CPU), csrc/bdpt_cpu.cpp) on the seeded
random scenes of test_gpu_fuzz.py against the oracle, bit for bit: the same geometries, materials,
emitter counts and cameras, on the CPU (runs without a GPU)."""
import numpy as np
import pytest

import gpu_bidirectional_raytracer_amd as g
import oracle
from test_gpu_fuzz import NPASS, SEEDS, random_scene

W, H = 23, 17


@pytest.fixture(scope="module")
def rnd0():
    return oracle.mt607(0)


@pytest.mark.parametrize("seed", range(SEEDS))
def test_cpu_backend_random_scene(rnd0, seed):
    cam, sp = random_scene(1000 + seed)
    g.update_camera(cam, W, H)
    r = g.Renderer(sp, W, H, cam, device=-1)                # BDPT_DEVICE_CPU
    r.light_pass(0)
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(NPASS)
    r.path_passes(sid, vlp)
    col, cnt = r.read_radiance()
    px = r.read_pixels()
    r.close()
    lp = oracle.light_pass(sp, rnd0, 0)
    ocol, ocnt, opx = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)
    assert np.array_equal(cnt, ocnt)
    assert np.array_equal(col.view(np.uint32), ocol.view(np.uint32)), f"seed {seed}"
    assert np.array_equal(px, opx)


@pytest.mark.parametrize("seed", range(max(6, SEEDS // 8)))
def test_cpu_backend_random_large_scene(rnd0, seed):
    from test_gpu_fuzz import random_large_scene
    cam, sp = random_large_scene(2000 + seed)
    g.update_camera(cam, W, H)
    r = g.Renderer(sp, W, H, cam, device=-1)                # BDPT_DEVICE_CPU
    r.light_pass(0)
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(3)
    r.path_passes(sid, vlp)
    col, cnt = r.read_radiance()
    r.close()
    lp = oracle.light_pass(sp, rnd0, 0)
    ocol, ocnt, _ = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)
    assert np.array_equal(cnt, ocnt)
    assert np.array_equal(col.view(np.uint32), ocol.view(np.uint32)), f"seed {seed}"
