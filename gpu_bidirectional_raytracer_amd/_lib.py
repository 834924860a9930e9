"""ctypes binding of the C-ABI in include/bdpt.h (libbdpt.so, built in-tree by `make`).

The product path has no fallback: if the HIP library is missing this module raises on import.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BDPT_LIB") or os.path.join(_HERE, "libbdpt.so")   # BDPT_LIB: A/B builds
REPO_ROOT = os.path.dirname(_HERE)
DEFAULT_DAT = os.path.join(REPO_ROOT, "assets", "data", "MersenneTwister.dat")
SCENE_DIR = os.path.join(REPO_ROOT, "assets", "scenes")

RAND_N = 4096 * 1876
LIGHT_POINTS = 4096
COUNTER_CAP = 30000

BDPT_OK, BDPT_EINVAL, BDPT_EIO, BDPT_EHIP, BDPT_ENOMEM, BDPT_ESTATE = 0, -1, -2, -3, -4, -5
DIFF, SPEC, REFR, LITE = 0, 1, 2, 3
KEY_UP, KEY_DOWN, KEY_LEFT, KEY_RIGHT, KEY_PAGE_UP, KEY_PAGE_DOWN = range(0x101, 0x107)
CHOICES = {1: "decided", 2: "fused", 4: "paired", 8: "quarter", 16: "pools", 32: "units"}   # BDPT_CHOICE_*
FEATURES = {1: "specialized", 2: "det_skip", 4: "zero_exit", 8: "last_skip", 16: "bvh", 32: "pass_streams",
            64: "pixel_pools", 128: "unit_fold", 256: "sincos_planes"}


class Vec(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float)]

    def __iter__(self):
        return iter((self.x, self.y, self.z))

    def __repr__(self):
        return f"Vec({self.x!r}, {self.y!r}, {self.z!r})"


class Sphere(ctypes.Structure):
    _fields_ = [("rad", ctypes.c_float), ("p", Vec), ("e", Vec), ("c", Vec), ("refl", ctypes.c_int)]


class LightPath(ctypes.Structure):
    _fields_ = [("hp", Vec), ("rad", Vec), ("nl", Vec)]


class Camera(ctypes.Structure):
    _fields_ = [("orig", Vec), ("target", Vec), ("dir", Vec), ("x", Vec), ("y", Vec)]


class RandState(ctypes.Structure):
    _fields_ = [("state", ctypes.c_int * 31), ("f", ctypes.c_int), ("r", ctypes.c_int)]


class PassState(ctypes.Structure):
    _fields_ = [("rng", RandState), ("flag", ctypes.c_int), ("vlp_index", ctypes.c_int)]


assert ctypes.sizeof(Vec) == 12 and ctypes.sizeof(Sphere) == 44
assert ctypes.sizeof(LightPath) == 36 and ctypes.sizeof(Camera) == 60

# every symbol include/bdpt.h declares: (name, restype, argtypes)
_P = ctypes.c_void_p
_SIGS = [
    ("bdpt_create", ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(Sphere), ctypes.c_uint,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    ("bdpt_create_multi", ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(Sphere), ctypes.c_uint,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_char_p, _P, ctypes.c_int]),
    ("bdpt_num_devices", ctypes.c_int, [_P]),
    ("bdpt_reduce_backend", ctypes.c_char_p, [_P]),
    ("bdpt_reduce_info", ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_int]),
    ("bdpt_rccl_version", ctypes.c_int, []),
    ("bdpt_reduce_frame", ctypes.c_int, [_P]),
    ("bdpt_destroy", None, [_P]),
    ("bdpt_last_error", ctypes.c_char_p, [_P]),
    ("bdpt_create_error", ctypes.c_char_p, []),
    ("bdpt_set_scene", ctypes.c_int, [_P, ctypes.POINTER(Sphere), ctypes.c_uint]),
    ("bdpt_set_camera", ctypes.c_int, [_P, ctypes.POINTER(Camera)]),
    ("bdpt_reset_accum", ctypes.c_int, [_P]),
    ("bdpt_set_shard", ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    ("bdpt_set_streams", ctypes.c_int, [_P, ctypes.c_int]),
    ("bdpt_last_streams", ctypes.c_int, [_P]),
    ("bdpt_stream_choice", ctypes.c_int, [_P]),
    ("bdpt_set_stream_choice", ctypes.c_int, [_P, ctypes.c_int]),
    ("bdpt_device_mode", ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    ("bdpt_set_specialize", ctypes.c_int, [_P, ctypes.c_int]),
    ("bdpt_last_specialized", ctypes.c_int, [_P]),
    ("bdpt_specialize_status", ctypes.c_char_p, [_P]),
    ("bdpt_set_traversal", ctypes.c_int, [_P, ctypes.c_int]),
    ("bdpt_kernel_timing", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]),
    ("bdpt_device_timing", ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                          ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong)]),
    ("bdpt_scene_has_bvh", ctypes.c_int, [_P]),
    ("bdpt_last_traversal", ctypes.c_int, [_P]),
    ("bdpt_last_kernel_features", ctypes.c_int, [_P]),
    ("bdpt_zero_exit_safe", ctypes.c_int, [ctypes.POINTER(Sphere), ctypes.c_uint]),
    ("bdpt_light_pass", ctypes.c_int, [_P, ctypes.c_int]),
    ("bdpt_generate_rand", ctypes.c_int, [_P, ctypes.c_uint]),
    ("bdpt_path_passes", ctypes.c_int, [_P, _P, _P, ctypes.c_int]),
    ("bdpt_synchronize", ctypes.c_int, [_P]),
    ("bdpt_last_path_ms", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_float)]),
    ("bdpt_path_timing", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]),
    ("bdpt_read_radiance", ctypes.c_int, [_P, _P, _P]),
    ("bdpt_read_pixels", ctypes.c_int, [_P, _P]),
    ("bdpt_read_rand", ctypes.c_int, [_P, _P]),
    ("bdpt_read_lightpaths", ctypes.c_int, [_P, _P]),
    ("bdpt_write_lightpaths", ctypes.c_int, [_P, _P]),
    ("bdpt_rand_seed", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint)]),
    ("bdpt_get_camera", ctypes.c_int, [_P, ctypes.POINTER(Camera)]),
    ("bdpt_frame_size", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    ("bdpt_get_scene", ctypes.c_int, [_P, ctypes.POINTER(Sphere), ctypes.c_uint]),
    ("bdpt_device_buffers", ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_P)]),
    ("bdpt_update_pixels", ctypes.c_int, [_P]),
    ("bdpt_gl_register_pbo", ctypes.c_int, [_P, ctypes.c_uint]),
    ("bdpt_gl_publish", ctypes.c_int, [_P]),
    ("bdpt_gl_unregister", ctypes.c_int, [_P]),
    ("bdpt_write_radiance", ctypes.c_int, [_P, _P, _P]),
    ("bdpt_save_checkpoint", ctypes.c_int, [_P, ctypes.c_char_p, _P, ctypes.c_uint]),
    ("bdpt_load_checkpoint", ctypes.c_int, [_P, ctypes.c_char_p, _P, ctypes.c_uint]),
    ("bdpt_read_scene", ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(Camera),
                                        ctypes.POINTER(ctypes.POINTER(Sphere)), ctypes.POINTER(ctypes.c_uint)]),
    ("bdpt_free_scene", None, [ctypes.POINTER(Sphere)]),
    ("bdpt_default_scene", ctypes.c_uint, [ctypes.POINTER(Camera), ctypes.POINTER(Sphere)]),
    ("bdpt_update_camera", None, [ctypes.POINTER(Camera), ctypes.c_int, ctypes.c_int]),
    ("bdpt_camera_key", ctypes.c_int, [ctypes.POINTER(Camera), ctypes.c_int]),
    ("bdpt_sphere_key", ctypes.c_int, [ctypes.POINTER(Sphere), ctypes.c_uint, ctypes.c_int, ctypes.c_int]),
    ("bdpt_save_ppm", ctypes.c_int, [ctypes.c_char_p, _P, ctypes.c_int, ctypes.c_int]),
    ("bdpt_save_ppm_binary", ctypes.c_int, [ctypes.c_char_p, _P, ctypes.c_int, ctypes.c_int]),
    ("bdpt_ppm_name", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_float, ctypes.c_int]),
    ("bdpt_gamma_thresholds", None, [_P]),
    ("bdpt_srand", None, [ctypes.POINTER(RandState), ctypes.c_uint]),
    ("bdpt_rand", ctypes.c_int, [ctypes.POINTER(RandState)]),
    ("bdpt_pass_state_init", None, [ctypes.POINTER(PassState)]),
    ("bdpt_pass_state_light", None, [ctypes.POINTER(PassState)]),
    ("bdpt_pass_state_next", None, [ctypes.POINTER(PassState), ctypes.POINTER(ctypes.c_uint),
                                     ctypes.POINTER(ctypes.c_int)]),
    ("bdpt_pass_schedule", None, [ctypes.POINTER(PassState), ctypes.c_int, _P, _P]),
]
EXPORTED = [s[0] for s in _SIGS]


def _single_hip_runtime():
    """Exactly one HIP runtime per process.  torch bundles its own libamdhip64/libhsa-runtime64
    (same SONAME libamdhip64.so.7 as /opt/rocm's).  If libbdpt.so loaded the system runtime first,
    a later `import torch` would map a second HSA runtime that cannot open the device.  Loading
    torch first makes libbdpt.so bind to torch's runtime, so device pointers can be shared with
    torch.distributed (RCCL) in the same process.  Without torch the system runtime is used."""
    if os.environ.get("BDPT_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def _load():
    _single_hip_runtime()
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is not built: run `make` (or __graft_entry__.build()) first; "
                          "there is no CPU fallback for the render path")
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in _SIGS:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


class BdptError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"bdpt error {code}: {msg}")
        self.code = code
