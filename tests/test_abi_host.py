"""C-ABI library (libbdpt.so) on the CPU: exports, ABI layouts and the host-side drop-in pieces
(scene loader, UpdateCamera, key moves, SavePPM, glibc rand, pass state machine, toInt table).
No compute kernels run here."""
import ctypes
import math
import os
import re

import numpy as np
import pytest

import gpu_bidirectional_raytracer_amd as g
from gpu_bidirectional_raytracer_amd import _lib
import oracle
from conftest import REPO, SCENES
from make_golden import read_scene_py

HEADER = os.path.join(REPO, "include", "bdpt.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(bdpt_[a-z0-9_]+)\s*\(", src))
    return names


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 30
    so = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in sorted(names) if not hasattr(so, n)]
    assert not missing, missing
    assert names == set(_lib.EXPORTED), names ^ set(_lib.EXPORTED)


def test_feature_bits_match_header():
    """The Python names of the kernel-feature bits (Renderer.last_features) are the header's
    BDPT_FEAT_* values, one for one."""
    src = open(HEADER).read()
    bits = {int(v): n for n, v in re.findall(r"#define\s+BDPT_FEAT_([A-Z_]+)\s+(\d+)", src)}
    assert sorted(bits) == sorted(_lib.FEATURES), (bits, _lib.FEATURES)
    assert bits[64] == "POOLS" and _lib.FEATURES[64] == "pixel_pools"


def test_struct_layouts_match_reference_headers():
    assert ctypes.sizeof(g.Vec) == 12          # vec.h:4-6
    assert ctypes.sizeof(_lib.Sphere) == 44    # geom.h:23-27 (enum as int)
    assert ctypes.sizeof(_lib.LightPath) == 36  # geom.h:29-33
    assert ctypes.sizeof(_lib.Camera) == 60    # camera.h:7-12
    assert _lib.Sphere.refl.offset == 40 and _lib.Sphere.c.offset == 28


@pytest.mark.parametrize("name", sorted(f[:-4] for f in os.listdir(SCENES) if f.endswith(".scn")))
def test_read_scene_matches_text(name):
    cam, sp = g.read_scene(os.path.join(SCENES, name + ".scn"))
    orig, target, ref = read_scene_py(os.path.join(SCENES, name + ".scn"))
    assert list(cam.orig) == list(orig) and list(cam.target) == list(target)
    assert len(sp) == len(ref)
    assert sp.tobytes() == ref.astype(sp.dtype).tobytes()


def test_read_scene_errors(tmp_path):
    with pytest.raises(g.BdptError):
        g.read_scene(str(tmp_path / "missing.scn"))
    bad = tmp_path / "bad.scn"
    bad.write_text("camera 1 2 3  4 5 6\nsize 1\nsphere 1  0 0 0  0 0 0  1 1 1  7\n")
    with pytest.raises(g.BdptError):
        g.read_scene(str(bad))


@pytest.mark.parametrize("name,w,h", [("cornell", 1921, 1081), ("caustic", 513, 513),
                                      ("simple", 257, 257), ("cornell_glass", 4097, 4097),
                                      ("gantz", 641, 481)])
def test_update_camera_bit_exact(name, w, h):
    cam, _ = g.read_scene(os.path.join(SCENES, name + ".scn"))
    g.update_camera(cam, w, h)
    ref = oracle.update_camera(list(cam.orig), list(cam.target), w, h)
    got = oracle.camera_array(cam)
    assert got.tobytes() == ref.tobytes()


def test_default_scene_is_scene_h_cornell():
    cam, sp = g.default_scene()
    assert len(sp) == 9
    assert list(cam.orig) == [50.0, 44.0, 176.0]
    assert sp[8]["e"].tolist() == [12.0, 12.0, 12.0] and sp[8]["refl"] == g.REFR
    assert sp[0]["rad"] == np.float32(1e4) and sp[0]["p"][0] == np.float32(1e4 + 1)


def test_glibc_rand_matches_libc():
    libc = ctypes.CDLL("libc.so.6")
    for seed in (1, 7, 12345):
        libc.srand(seed)
        ref = [libc.rand() for _ in range(700)]
        assert g.glibc_rand(700, seed).tolist() == ref


def test_pass_state_machine():
    """flag/vlp_index: 1,1,2,2,3,3,... after the first light pass (smallpt_cpu.c:292-293)."""
    s = g.PassScheduler()
    assert s.flag == 1 and s.vlp_index == 1
    s.light()
    sid, vlp = s.next(8)
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(1)
    assert sid.tolist() == [libc.rand() % g.RAND_N for _ in range(8)]
    assert vlp.tolist() == [1, 1, 2, 2, 3, 3, 4, 4]
    # an odd pass count then a light pass (ReInit with even reinit_counter) restarts the pair
    sid, vlp = s.next(1)
    assert vlp.tolist() == [5] and s.flag == 3
    s.light()
    assert s.next(3)[1].tolist() == [5, 5, 6]


def test_pass_state_vlp_wraps_at_light_points():
    s = g.PassScheduler()
    s.light()
    _, vlp = s.next(8200)
    assert vlp.max() == 4095 and vlp[8189] == 4095 and vlp[8190] == 0   # raw index 4096 -> 0


def test_gamma_thresholds_equal_toint():
    thr = np.zeros(256, np.float32)
    _lib.lib.bdpt_gamma_thresholds(ctypes.c_void_p(thr.ctypes.data))
    assert np.isneginf(thr[0]) and np.all(np.diff(thr[1:]) > 0)
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.random(20000, dtype=np.float32), rng.random(2000, dtype=np.float32) * 3 - 1,
                         thr[1:], np.nextafter(thr[1:], np.float32(-1)), np.float32([0, 1, -0.0, 2, 1e-30])])
    for x in xs:
        k = int(np.searchsorted(thr, x, side="right") - 1)
        assert k == oracle.to_int(float(x)), (x, k)


def test_camera_keys():
    cam, _ = g.read_scene(os.path.join(SCENES, "cornell.scn"))
    g.update_camera(cam, 641, 481)
    o = np.array(list(cam.orig), np.float32)
    d = np.array(list(cam.dir), np.float32)
    assert g.camera_key(cam, "w")
    np.testing.assert_array_equal(np.array(list(cam.orig), np.float32), o + np.float32(10) * d)
    assert not g.camera_key(cam, "z")
    t = np.array(list(cam.target), np.float32) - np.array(list(cam.orig), np.float32)
    g.camera_key(cam, "left")
    a = -2.0 * math.pi / 180.0
    tx = np.float32(float(t[0]) * math.cos(a) - float(t[2]) * math.sin(a))
    tz = np.float32(float(tx) * math.sin(a) + float(t[2]) * math.cos(a))   # reuses new x (A.9)
    got = np.array(list(cam.target), np.float32) - np.array(list(cam.orig), np.float32)
    assert abs(float(got[0]) - float(tx)) < 1e-4 and abs(float(got[2]) - float(tz)) < 1e-4


def test_sphere_keys():
    _, sp = g.read_scene(os.path.join(SCENES, "cornell.scn"))
    p = sp[6]["p"].copy()
    assert g.sphere_key(sp, 6, "4") and sp[6]["p"][0] == p[0] - 5
    assert g.sphere_key(sp, 6, "9") and sp[6]["p"][1] == p[1] + 5
    assert not g.sphere_key(sp, 6, "x")


def test_save_ppm_format(tmp_path):
    rgba = np.zeros((2, 3, 4), np.uint8)
    rgba[0, :, 0] = [1, 2, 3]       # row 0 = bottom row in the file (written last)
    rgba[1, :, 1] = [4, 5, 6]
    path = tmp_path / "x.ppm"
    g.save_ppm(str(path), rgba)
    txt = path.read_text()
    assert txt == "P3\n3 2\n255\n0 4 0 0 5 0 0 6 0 1 0 0 2 0 0 3 0 0 "


def test_create_fails_cleanly_without_gpu():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    cam, sp = g.read_scene(os.path.join(SCENES, "simple.scn"))
    with pytest.raises(g.BdptError) as e:
        g.Renderer(sp, 17, 9, cam)
    assert e.value.code in (_lib.BDPT_EHIP, _lib.BDPT_EIO)
    with pytest.raises(g.BdptError):
        g.Renderer(sp, 17, 9, cam, dat_path="/nonexistent.dat")


def test_create_multi_argument_errors():
    cam, sp = g.read_scene(os.path.join(SCENES, "simple.scn"))
    arr = g.spheres_to_array(sp)
    h = ctypes.c_void_p()
    ptr = ctypes.cast(ctypes.c_void_p(arr.ctypes.data), ctypes.POINTER(_lib.Sphere))
    devs = np.zeros(2, np.int32)
    rc = _lib.lib.bdpt_create_multi(ctypes.byref(h), ptr, len(arr), 17, 9, _lib.DEFAULT_DAT.encode(),
                                    ctypes.c_void_p(devs.ctypes.data), 0)
    assert rc == _lib.BDPT_EINVAL and not h.value
    rc = _lib.lib.bdpt_create_multi(ctypes.byref(h), ptr, len(arr), 17, 9, _lib.DEFAULT_DAT.encode(), None, 2)
    assert rc == _lib.BDPT_EINVAL and b"device list" in _lib.lib.bdpt_create_error()
    assert _lib.lib.bdpt_reduce_backend(None) == b"null context"
    assert _lib.lib.bdpt_num_devices(None) == _lib.BDPT_EINVAL


def test_create_multi_fails_cleanly_without_gpu():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    cam, sp = g.read_scene(os.path.join(SCENES, "simple.scn"))
    with pytest.raises(g.BdptError) as e:
        g.Renderer(sp, 17, 9, cam, devices=[0, 1])
    assert e.value.code == _lib.BDPT_EHIP


def test_reduce_bracket_closes_the_group_on_every_error():
    """assemble()'s RCCL group bracket (bdpt_host.cpp reduce_bracket), driven by fake calls with a
    failing hipSetDevice or ncclReduce injected at every position: the group is always closed
    (one ncclGroupEnd per ncclGroupStart), issuing stops at the failure, and the failure is
    reported -- so the context stays usable for the next reduce."""
    hook = _lib.lib.bdpt__test_reduce_bracket
    hook.restype, hook.argtypes = ctypes.c_int, [ctypes.c_int] * 3 + [ctypes.POINTER(ctypes.c_int)] * 3
    for ndev in (1, 2, 8):
        for fail_dev in range(-1, ndev):
            for fail_red in range(-1, 2 * ndev):
                op, nred, herr = ctypes.c_int(9), ctypes.c_int(-1), ctypes.c_int(-1)
                r = hook(ndev, fail_dev, fail_red, ctypes.byref(op), ctypes.byref(nred), ctypes.byref(herr))
                assert op.value == 0, (ndev, fail_dev, fail_red)
                dev_first = fail_dev >= 0 and (fail_red < 0 or fail_red >= 2 * fail_dev)
                if dev_first:
                    assert herr.value != 0 and r == 0 and nred.value == 2 * fail_dev
                elif fail_red >= 0:
                    assert r != 0 and herr.value == 0 and nred.value == fail_red + 1
                else:
                    assert r == 0 and herr.value == 0 and nred.value == 2 * ndev


def test_rccl_version_and_reduce_info():
    v = _lib.lib.bdpt_rccl_version()
    if v == _lib.BDPT_ESTATE:
        pytest.skip("librccl not loadable here")
    assert v >= 20000, v                       # major.minor.patch as m*10000 + n*100 + p
    buf = ctypes.create_string_buffer(64)
    assert _lib.lib.bdpt_reduce_info(None, buf, 64) == _lib.BDPT_EINVAL
