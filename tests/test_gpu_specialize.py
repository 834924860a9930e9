"""Scene-specialised path kernels (run-time compiled with the sphere geometry folded in,
bdpt_host.cpp jit_path_kernel) give bit-identical frames to the precompiled kernels, with and
without pass streams, on every scene kind the specialisation covers (1..64 spheres, one or
several emitters, refractive / specular / diffuse)."""
import os

import numpy as np
import pytest

import gpu_bidirectional_raytracer_amd as g
import oracle
from conftest import SCENES

pytestmark = pytest.mark.gpu


def render(name, W, H, npass, specialize, streams, gpu):
    cam, sp = g.read_scene(os.path.join(SCENES, name + ".scn"))
    g.update_camera(cam, W, H)
    with g.Renderer(sp, W, H, cam, device=gpu) as r:
        r.set_specialize(specialize)
        r.set_streams(streams)
        r.light_pass(0)
        s = g.PassScheduler()
        s.light()
        sid, vlp = s.next(npass)
        r.path_passes(sid, vlp)
        col, cnt = r.read_radiance()
        px = r.read_pixels()
        used, why = r.last_specialized, r.specialize_status
    return col, cnt, px, used, why


@pytest.mark.parametrize("name", ["cornell", "cornell_glass", "caustic", "cornell_2luci", "simple",
                                  "cornell_multi", "hall_of_mirrors", "open", "synthetic64"])
@pytest.mark.parametrize("streams", [0, 1])
def test_specialised_equals_precompiled(gpu, name, streams):
    W, H, npass = 97, 61, 6
    ref = render(name, W, H, npass, False, streams, gpu)
    got = render(name, W, H, npass, True, streams, gpu)
    assert not ref[3]
    assert got[3], f"specialised kernel not used: {got[4]}"
    for a, b, what in zip(got[:3], ref[:3], ("colors", "counter", "pixels")):
        assert np.array_equal(a, b), f"{name} streams={streams}: {what} differ"


def test_specialised_matches_oracle(gpu):
    name, W, H, npass = "cornell", 65, 49, 8
    col, cnt, px, used, why = render(name, W, H, npass, True, 0, gpu)
    assert used, why
    cam, sp = g.read_scene(os.path.join(SCENES, name + ".scn"))
    g.update_camera(cam, W, H)
    rnd = oracle.mt607(0)
    lp = oracle.light_pass(sp, rnd, 0)
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(npass)
    ocol, ocnt, opx = oracle.path_passes(sp, rnd, cam, W, H, lp, sid, vlp)
    assert np.array_equal(col, ocol) and np.array_equal(cnt, ocnt) and np.array_equal(px, opx)


def test_specialisation_follows_scene_edits(gpu):
    """set_scene (ReInitScene) with moved spheres compiles a new kernel for the new geometry."""
    W, H, npass = 49, 37, 4
    cam, sp = g.read_scene(os.path.join(SCENES, "cornell.scn"))
    g.update_camera(cam, W, H)
    moved = sp.copy()
    moved[6]["p"][0] += 3.0
    out = []
    for spec in (True, False):
        with g.Renderer(sp, W, H, cam, device=gpu) as r:
            r.set_specialize(spec)
            r.light_pass(0)
            s = g.PassScheduler()
            s.light()
            sid, vlp = s.next(2 * npass)
            r.path_passes(sid[:npass], vlp[:npass])
            r.set_scene(moved)
            r.reset_accum()
            r.light_pass(0)
            r.path_passes(sid[npass:], vlp[npass:])
            out.append(r.read_radiance()[0])
    assert np.array_equal(out[0], out[1])
