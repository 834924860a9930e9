"""Host-side replay parity: the product's camera/sphere key handling and
UpdateCamera (csrc/bdpt_util.c) against the oracle's restatement of display_func.c, bit for bit.
No GPU needed."""
import os
import random

import numpy as np

import gpu_bidirectional_raytracer_amd as g
import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(REPO, "assets", "scenes")
ASCII = list("adwsrf ") + ["x", "p", "h"]
SPECIAL = list(oracle.GLUT_SPECIAL)


def _vec(v):
    return np.array([v.x, v.y, v.z], np.float32)


def _same_camera(pc, oc, what):
    for f in ("orig", "target", "dir", "x", "y"):
        a, b = _vec(getattr(pc, f)), oc[f][0]
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (what, f, a, b)


def test_update_camera_all_scenes():
    for name in sorted(os.listdir(SCENES)):
        if not name.endswith(".scn"):
            continue
        for W, H in ((641, 481), (1921, 1081), (4097, 4097), (33, 25)):
            cam, _ = g.read_scene(os.path.join(SCENES, name))
            g.update_camera(cam, W, H)
            oc = oracle.update_camera(_vec(cam.orig), _vec(cam.target), W, H)
            _same_camera(cam, oc, (name, W, H))


def test_key_sequences_match_oracle():
    rng = random.Random(7)
    for scene in ("cornell.scn", "caustic.scn", "complex.scn"):
        cam, _ = g.read_scene(os.path.join(SCENES, scene))
        W, H = 641, 481
        g.update_camera(cam, W, H)
        oc = oracle.update_camera(_vec(cam.orig), _vec(cam.target), W, H)
        for step in range(300):
            if rng.random() < 0.5:
                k = rng.choice(ASCII)
                moved = g.camera_key(cam, k)
                omoved = oracle.key_camera(oc, k)
            else:
                k = rng.choice(SPECIAL)
                moved = g.camera_key(cam, k)
                omoved = oracle.special_key(oc, k)
            assert moved == omoved, (scene, step, k)
            _same_camera(cam, oc, (scene, step, k, "key"))
            if moved:                                    # ReInit -> UpdateCamera
                g.update_camera(cam, W, H)
                oc2 = oracle.update_camera(oc["orig"][0], oc["target"][0], W, H)
                oc[...] = oc2
                _same_camera(cam, oc, (scene, step, k, "UpdateCamera"))


def test_host_vnorm_is_c_double_sqrt():
    """display_func.c is C: vnorm's sqrt is the double libm sqrt, rounded once to float."""
    cam, _ = g.read_scene(os.path.join(SCENES, "cornell.scn"))
    g.update_camera(cam, 1921, 1081)
    d = _vec(cam.target) - _vec(cam.orig)
    dd = np.float32(d[0] * d[0] + d[1] * d[1]) + np.float32(d[2] * d[2])
    lc = np.float32(1.0 / np.sqrt(np.float64(dd)))
    np.testing.assert_array_equal(_vec(cam.dir), lc * d)


def test_save_ppm_matches_oracle(tmp_path):
    from oracle.replay import ppm_name, save_ppm_text
    rng = np.random.default_rng(3)
    for h, w in ((1, 1), (7, 5), (25, 33)):
        px = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
        g.save_ppm(str(tmp_path / "a.ppm"), px)
        assert (tmp_path / "a.ppm").read_text() == save_ppm_text(px)
        g.save_ppm(str(tmp_path / "b.ppm"), px, binary=True)
        raw = (tmp_path / "b.ppm").read_bytes()
        head = b"P6\n%d %d\n255\n" % (w, h)
        assert raw[:len(head)] == head
        assert raw[len(head):] == px[::-1, :, :3].tobytes()
    for t, n in ((0.0, 0), (1.23456, 17), (999.9996, 1024), (12345.678, 8192)):
        assert g.ppm_name(t, n) == ppm_name(t, n)


def test_oracle_rand_matches_libc():
    """oracle.replay.GlibcRand restates glibc rand(): same sequence as libc.so.6 for several
    seeds (including 0, which glibc maps to 1, and seeds above 2^31)."""
    import ctypes
    from oracle.replay import GlibcRand
    libc = ctypes.CDLL("libc.so.6")
    for seed in (1, 0, 7, 12345, 2**31 + 5, 2**32 - 1):
        libc.srand(ctypes.c_uint(seed))
        want = [libc.rand() for _ in range(2000)]
        r = GlibcRand(seed)
        assert [r.rand() for _ in range(2000)] == want, seed
    libc.srand(1)
