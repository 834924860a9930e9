"""Checkpoint / resume of the accumulation (bdpt_write_radiance,
bdpt_save_checkpoint / bdpt_load_checkpoint): a render stopped, saved, restored into a fresh
context and continued equals the uninterrupted render bit for bit -- through the Python mirror,
the C host `smallpt`, and a multi-device context."""
import filecmp
import os
import subprocess

import numpy as np
import pytest

import gpu_bidirectional_raytracer_amd as g
from conftest import REPO, SCENES

pytestmark = pytest.mark.gpu
SMALLPT = os.path.join(REPO, "gpu_bidirectional_raytracer_amd", "smallpt")


def frame(r):
    col, cnt = r.read_radiance()
    return col, cnt, r.read_pixels()


def same(a, b, what):
    for x, y, w in zip(a, b, ("colors", "counter", "pixels")):
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), f"{what}: {w}"


@pytest.mark.parametrize("kw", [{}, {"devices": [0, 0]}])
def test_resume_equals_uninterrupted(gpu, tmp_path, kw):
    W, H = 121, 89
    cam, sp = g.read_scene(os.path.join(SCENES, "cornell_glass.scn"))
    g.update_camera(cam, W, H)
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(14)
    with g.Renderer(sp, W, H, cam, device=gpu) as r:
        r.light_pass(0)
        r.path_passes(sid, vlp)
        ref = frame(r)
    ck = str(tmp_path / "run.ckpt")
    with g.Renderer(sp, W, H, cam, **(kw or {"device": gpu})) as r:
        r.light_pass(0)
        r.path_passes(sid[:5], vlp[:5])
        r.save_checkpoint(ck, b"state!")
    with g.Renderer(sp, W, H, cam, **(kw or {"device": gpu})) as r:
        r.light_pass(0)
        assert r.load_checkpoint(ck, 6) == b"state!"
        r.path_passes(sid[5:], vlp[5:])
        same(frame(r), ref, "resumed")


def test_write_radiance_round_trip_and_errors(gpu, tmp_path):
    W, H = 33, 17
    cam, sp = g.read_scene(os.path.join(SCENES, "cornell.scn"))
    g.update_camera(cam, W, H)
    rng = np.random.default_rng(3)
    col = rng.random((H, W, 3), dtype=np.float32)
    cnt = rng.integers(0, 29999, (H, W)).astype(np.uint32)
    with g.Renderer(sp, W, H, cam, device=gpu) as r:
        r.write_radiance(col, cnt)
        c2, n2 = r.read_radiance()
        assert np.array_equal(c2, col) and np.array_equal(n2, cnt)
        ck = str(tmp_path / "a.ckpt")
        r.save_checkpoint(ck)
    with g.Renderer(sp, W + 1, H, cam, device=gpu) as r:             # other frame size
        with pytest.raises(g.BdptError):
            r.load_checkpoint(ck)
    bad = tmp_path / "bad.ckpt"
    bad.write_bytes(b"not a checkpoint at all")
    with g.Renderer(sp, W, H, cam, device=gpu) as r:
        with pytest.raises(g.BdptError):
            r.load_checkpoint(str(bad))
        with pytest.raises(g.BdptError):
            r.load_checkpoint(ck, 4)                                  # host-state size differs


def test_smallpt_mirror_checkpoint_keeps_the_schedule(gpu, tmp_path):
    """SmallPT.SaveCheckpoint carries the pass schedule (rand state, flag, vlp_index) too."""
    scn = os.path.join(SCENES, "cornell.scn")
    a = g.SmallPT(48, 36, scn)
    a.IdleFunc()
    a.UpdateRendering(9)
    ref = frame(a.renderer)
    b = g.SmallPT(48, 36, scn)
    b.IdleFunc()
    b.UpdateRendering(3)
    ck = str(tmp_path / "m.ckpt")
    b.SaveCheckpoint(ck)
    b.FreeBuffers()
    c = g.SmallPT(48, 36, scn)
    c.IdleFunc()
    c.LoadCheckpoint(ck)
    assert c.current_sample == 4
    c.UpdateRendering(6)
    same(frame(c.renderer), ref, "mirror resume")
    for x in (a, c):
        x.FreeBuffers()


def test_smallpt_host_resume(gpu, tmp_path):
    scn = os.path.join(SCENES, "caustic.scn")
    full, part = tmp_path / "full.ppm", tmp_path / "part.ppm"
    ck = tmp_path / "h.ckpt"
    base = [SMALLPT, "57", "41", scn, "--batch", "3"]
    subprocess.check_call(base + ["--spp", "12", "--out", str(full)], cwd=REPO, timeout=120)
    subprocess.check_call(base + ["--spp", "5", "--checkpoint", str(ck)], cwd=REPO, timeout=120)
    r = subprocess.run(base + ["--spp", "7", "--resume", str(ck), "--out", str(part)], cwd=REPO,
                       timeout=120, capture_output=True, text=True)
    assert r.returncode == 0 and "Resumed at pass 5" in r.stderr, r.stderr
    assert filecmp.cmp(full, part, shallow=False)


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_mirror_resume_after_keys(gpu, tmp_path, devices):
    """A checkpoint taken after camera / sphere keys restores the edited camera, scene, MT table
    and VLPs (bdpt_ckpt.c): the resumed session equals the uninterrupted one bit for bit (one
    device, and a two-shard multi-device context)."""
    scn = os.path.join(SCENES, "cornell_glass.scn")

    def start():
        s = g.SmallPT(40, 30, scn, device=gpu)
        if devices is not None:                          # swap in a multi-device context
            s.renderer.close()
            s.renderer = g.Renderer(s.spheres, s.width, s.height, s.camera, s.dat_path, devices=devices)
        return s

    def head(s):
        s.IdleFunc()
        s.UpdateRendering(2)
        for k in "s+8":
            s.KeyFunc(k)
            s.UpdateRendering(3)

    def tail(s):
        s.UpdateRendering(4)
        s.KeyFunc("a")
        s.UpdateRendering(2)
        return frame(s.renderer)

    a = start()
    head(a)
    ref = tail(a)
    a.FreeBuffers()
    b = start()
    head(b)
    ck = str(tmp_path / "keys.ckpt")
    b.SaveCheckpoint(ck)
    b.FreeBuffers()
    c = start()
    c.IdleFunc()
    c.LoadCheckpoint(ck)
    same(tail(c), ref, "resume after keys")
    c.FreeBuffers()
