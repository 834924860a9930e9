"""ORACLE -- test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

ctypes wrapper of oracle/liboracle.so, the plain-C CPU restatement of the reference render path
(see oracle/bdpt_oracle.c for the file:line citations and the floating-point contract).
The product never imports this package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
LIB_PATH = os.path.join(_HERE, "liboracle.so")
RAND_N = 4096 * 1876
LIGHT_POINTS = 4096

SPHERE_DTYPE = np.dtype([("rad", "<f4"), ("p", "<f4", 3), ("e", "<f4", 3), ("c", "<f4", 3),
                         ("refl", "<i4")])
LIGHTPATH_DTYPE = np.dtype([("hp", "<f4", 3), ("rad", "<f4", 3), ("nl", "<f4", 3)])
CAMERA_DTYPE = np.dtype([("orig", "<f4", 3), ("target", "<f4", 3), ("dir", "<f4", 3),
                         ("x", "<f4", 3), ("y", "<f4", 3)])
STAT_NAMES = ("samples", "segments", "closest", "shadow", "sphere_tests", "diffuse", "rng_reads", "refr")


def _load():
    if not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "oracle/liboracle.so"], cwd=_REPO)
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    lib.oracle_mt607.argtypes = [P, ctypes.c_uint32, P]
    lib.oracle_mt607.restype = None
    lib.oracle_light_pass.argtypes = [P, ctypes.c_uint, P, ctypes.c_int, P]
    lib.oracle_light_pass.restype = None
    lib.oracle_path_passes.argtypes = [P, ctypes.c_uint, P, P, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_int, P, P, P,
                                       ctypes.c_int, P]
    lib.oracle_path_passes.restype = None
    lib.oracle_path_span.argtypes = [P, ctypes.c_uint, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_long,
                                     ctypes.c_long, P, P, P, ctypes.c_int, P, P, P, ctypes.c_int, P]
    lib.oracle_path_span.restype = None
    lib.oracle_update_camera.argtypes = [P, ctypes.c_int, ctypes.c_int]
    lib.oracle_update_camera.restype = None
    lib.oracle_key_camera.argtypes = [P, ctypes.c_int]
    lib.oracle_key_camera.restype = ctypes.c_int
    lib.oracle_special_key.argtypes = [P, ctypes.c_int]
    lib.oracle_special_key.restype = ctypes.c_int
    lib.oracle_to_int.argtypes = [ctypes.c_float]
    lib.oracle_to_int.restype = ctypes.c_int
    lib.oracle_fnv1a64.argtypes = [P, ctypes.c_uint64]
    lib.oracle_fnv1a64.restype = ctypes.c_uint64
    lib.oracle_fnv1_64.argtypes = [P, ctypes.c_uint64]
    lib.oracle_fnv1_64.restype = ctypes.c_uint64
    return lib


lib = _load()


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def load_mt_params(path: str = os.path.join(_REPO, "assets", "data", "MersenneTwister.dat")) -> np.ndarray:
    """loadMTGPU (MersenneTwister_kernel.cu:23-36): 4096 records of 4 uint32."""
    p = np.fromfile(path, dtype="<u4")
    assert p.size == 4 * 4096, p.size
    return p


def mt607(seed: int, params: np.ndarray | None = None) -> np.ndarray:
    params = load_mt_params() if params is None else np.ascontiguousarray(params, "<u4")
    out = np.empty(RAND_N, np.float32)
    lib.oracle_mt607(_p(params), seed, _p(out))
    return out


def fnv1a64(a: np.ndarray) -> int:
    a = np.ascontiguousarray(a)
    return int(lib.oracle_fnv1a64(_p(a), a.nbytes))


def fnv1_64(a) -> int:
    """FNV-1 (multiply before xor) 64 over the bytes of a (numpy array or bytes)."""
    a = np.frombuffer(a, np.uint8) if isinstance(a, (bytes, bytearray)) else np.ascontiguousarray(a)
    return int(lib.oracle_fnv1_64(_p(a), a.nbytes))


def light_pass(spheres: np.ndarray, rnd: np.ndarray, current_sample: int = 0,
               lp: np.ndarray | None = None) -> np.ndarray:
    sp = np.ascontiguousarray(spheres.astype(SPHERE_DTYPE, copy=False))
    lp = np.zeros(LIGHT_POINTS, LIGHTPATH_DTYPE) if lp is None else lp.copy()
    lib.oracle_light_pass(_p(sp), len(sp), _p(rnd), current_sample, _p(lp))
    return lp


def camera_array(cam) -> np.ndarray:
    """ctypes Camera (or CAMERA_DTYPE array) -> 1-element CAMERA_DTYPE array."""
    if isinstance(cam, np.ndarray):
        return np.ascontiguousarray(cam.astype(CAMERA_DTYPE, copy=False).reshape(1))
    a = np.zeros(1, CAMERA_DTYPE)
    ctypes.memmove(a.ctypes.data, ctypes.addressof(cam), CAMERA_DTYPE.itemsize)
    return a


def update_camera(orig, target, width: int, height: int) -> np.ndarray:
    c = np.zeros(1, CAMERA_DTYPE)
    c["orig"] = orig
    c["target"] = target
    lib.oracle_update_camera(_p(c), width, height)
    return c


GLUT_SPECIAL = {"left": 100, "up": 101, "right": 102, "down": 103, "page_up": 104, "page_down": 105}


def key_camera(cam: np.ndarray, key: str) -> bool:
    """KeyFunc camera keys (display_func.c:276-336) on a CAMERA_DTYPE array, in place.
    True when the reference calls ReInit(1) for the key."""
    assert cam.dtype == CAMERA_DTYPE and cam.flags.c_contiguous
    return bool(lib.oracle_key_camera(_p(cam), ord(key)))


def special_key(cam: np.ndarray, key: str) -> bool:
    """SpecialFunc (display_func.c:384-433): key in GLUT_SPECIAL."""
    assert cam.dtype == CAMERA_DTYPE and cam.flags.c_contiguous
    return bool(lib.oracle_special_key(_p(cam), GLUT_SPECIAL[key]))


def path_passes(spheres, rnd, cam, width, height, lp, sid, vlp, colors=None, counter=None,
                pixels=None, rows=None, nthreads: int = 0, stats: bool = False, span=None):
    """npass x RadiancePathTracingKernel over rows [y0, y1) (or the row-major pixel range
    span = (p0, p1)) -> (colors, counter, pixels[, stats])."""
    sp = np.ascontiguousarray(spheres.astype(SPHERE_DTYPE, copy=False))
    cam = camera_array(cam)
    sid = np.ascontiguousarray(sid, np.uint32)
    vlp = np.ascontiguousarray(vlp, np.int32)
    colors = np.zeros((height, width, 3), np.float32) if colors is None else colors.copy()
    counter = np.zeros((height, width), np.uint32) if counter is None else counter.copy()
    pixels = np.zeros((height, width, 4), np.uint8) if pixels is None else pixels.copy()
    y0, y1 = (0, height) if rows is None else rows
    st = np.zeros(8, np.uint64)
    p0, p1 = (y0 * width, y1 * width) if span is None else span
    lib.oracle_path_span(_p(sp), len(sp), _p(rnd), _p(cam), width, height, p0, p1, _p(lp),
                         _p(sid), _p(vlp), len(sid), _p(colors), _p(counter), _p(pixels),
                         nthreads, _p(st) if stats else None)
    if stats:
        return colors, counter, pixels, dict(zip(STAT_NAMES, (int(v) for v in st)))
    return colors, counter, pixels


def to_int(x: float) -> int:
    return int(lib.oracle_to_int(x))
