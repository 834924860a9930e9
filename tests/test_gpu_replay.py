"""SURVEY 8(f)1 -- headless camera-control and scene-edit replay, bit-exact against the oracle's
restatement of the reference's host loop (oracle/replay.py: IdleFunc, UpdateRendering[2],
ReInit, ReInitScene, KeyFunc, SpecialFunc).  Product side: the SmallPT mirror (Python over the
C-ABI) and the C host program `smallpt --keys`."""
import os
import subprocess

import numpy as np
import pytest

import gpu_bidirectional_raytracer_amd as g
import oracle
from conftest import REPO, SCENES
from oracle.replay import Session

pytestmark = pytest.mark.gpu

DAT = os.path.join(REPO, "assets", "data", "MersenneTwister.dat")
# KeyFunc / SpecialFunc events; every kind of key the reference handles
SCRIPT = ["w", "left", "+", "4", "up", " ", "a", "page_up", "-", "9", "s", "r", "right", "d",
          "f", "down", "page_down", "3", "6", "8", "2", "x", " "]


def _session(scene, cw, ch, rows=None):
    cam, sp = g.read_scene(os.path.join(SCENES, scene + ".scn"))
    o = np.array([cam.orig.x, cam.orig.y, cam.orig.z], np.float32)
    t = np.array([cam.target.x, cam.target.y, cam.target.z], np.float32)
    return Session(sp, o, t, cw + 1, ch + 1, rows=rows)


def _same(a, b, what):
    assert a.shape == b.shape, what
    if a.dtype.kind == "f":
        a, b = a.view(np.uint32), b.view(np.uint32)
    bad = np.argwhere(a != b)
    assert bad.size == 0, f"{what}: {len(bad)} mismatches, first at {bad[:3].tolist()}"


@pytest.mark.parametrize("scene", ["cornell", "cornell_glass"])
def test_key_replay_mirror_matches_oracle(gpu, scene):
    cw, ch = 20, 14
    spt = g.SmallPT(cw, ch, os.path.join(SCENES, scene + ".scn"), device=gpu)
    ora = _session(scene, cw, ch)
    for _ in range(3):
        spt.IdleFunc()
        ora.IdleFunc()
    for step, k in enumerate(SCRIPT):
        if len(k) > 1:
            spt.SpecialFunc(k)
            ora.SpecialFunc(k)
        else:
            spt.KeyFunc(k)
            ora.KeyFunc(k)
        for _ in range(2):
            spt.IdleFunc()
            ora.IdleFunc()
        col, cnt = spt.colors()
        tag = f"{scene} step {step} key {k!r}"
        _same(cnt, ora.counter, tag + " counter")
        _same(col, ora.colors, tag + " colors")
        _same(spt.pixels(), ora.pixels, tag + " pixels")
        assert spt.flag == ora.flag and spt.current_sample == ora.current_sample, tag
    spt.FreeBuffers()


def _read_ppm(path):
    toks = open(path).read().split()
    assert toks[0] == "P3" and toks[3] == "255"
    w, h = int(toks[1]), int(toks[2])
    v = np.array(toks[4:], np.int64).reshape(h, w, 3)
    return v[::-1]                                       # file rows are bottom-up


def test_smallpt_host_keys_match_oracle(gpu, tmp_path):
    """`smallpt 24 18 cornell.scn --spp 3 --keys ...`: light pass, 3 passes, then per key the
    handler and 3 more passes; the PPM equals the oracle session's toInt pixels."""
    keys = "wL+4U aPdQ-9R3"
    names = {"U": "up", "D": "down", "L": "left", "R": "right", "P": "page_up", "Q": "page_down"}
    out = tmp_path / "k.ppm"
    exe = os.path.join(REPO, "gpu_bidirectional_raytracer_amd", "smallpt")
    subprocess.check_call([exe, "24", "18", os.path.join(SCENES, "cornell.scn"), "--spp", "3",
                           "--batch", "2", "--keys", keys, "--out", str(out), "--dat", DAT],
                          cwd=tmp_path, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    ora = _session("cornell", 24, 18)
    for _ in range(3):
        ora.IdleFunc()
    for k in keys:
        if k in names:
            ora.SpecialFunc(names[k])
        else:
            ora.KeyFunc(k)
        for _ in range(3):
            ora.IdleFunc()
    _same(_read_ppm(out), ora.pixels[..., :3].astype(np.int64), "smallpt --keys PPM")


def test_smallpt_save_key_and_p6(gpu, tmp_path):
    """'p' saves with the reference's name pattern (P3, the pixels at that moment); --p6 writes
    the same image as binary P6 (two deterministic runs of one configuration)."""
    exe = os.path.join(REPO, "gpu_bidirectional_raytracer_amd", "smallpt")
    base = [exe, "16", "12", os.path.join(SCENES, "caustic.scn"), "--spp", "2", "--dat", DAT]
    quiet = dict(cwd=tmp_path, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    subprocess.check_call(base + ["--keys", "p", "--out", str(tmp_path / "after.ppm")], **quiet)
    saved = [f for f in os.listdir(tmp_path) if f.startswith("max1_secondi")]
    assert len(saved) == 1 and saved[0].endswith("_exe2.ppm"), saved
    subprocess.check_call(base + ["--out", str(tmp_path / "a.ppm")], **quiet)
    subprocess.check_call(base + ["--out", str(tmp_path / "b.ppm"), "--p6"], **quiet)
    p3 = _read_ppm(tmp_path / "a.ppm")
    assert np.array_equal(_read_ppm(tmp_path / saved[0]), p3)   # 'p' saw 2 passes too
    raw = (tmp_path / "b.ppm").read_bytes()
    head = b"P6\n17 13\n255\n"
    assert raw.startswith(head)
    p6 = np.frombuffer(raw[len(head):], np.uint8).reshape(13, 17, 3)[::-1]
    assert np.array_equal(p3, p6.astype(np.int64))
