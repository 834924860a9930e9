"""MI355X-native bidirectional path tracer: the render path of sim186/gpu_bidirectional_raytracer
(per-pixel eye path with NEE + VLP connection, MT607 random table, light pass) as hand-written
HIP kernels for gfx950 behind a C-ABI (include/bdpt.h, libbdpt.so).

This package is the host-side mirror of the reference's operator interface (src/smallpt_cpu.c,
src/display_func.c): `SmallPT` keeps the reference's names (AllocateBuffers, UpdateRendering,
UpdateRendering2, ReInit, ReInitScene, SavePPM, KeyFunc, SpecialFunc) and argument meaning;
`Renderer` is a thin object over one C-ABI context.  No torch types anywhere: torch is only
used by bench.py for torch.distributed plumbing.
"""
from __future__ import annotations

import ctypes
import os
import struct
from typing import Optional, Sequence, Tuple

import numpy as np

from ._lib import (BDPT_OK, CHOICES, COUNTER_CAP, DEFAULT_DAT, DIFF, FEATURES, KEY_DOWN, KEY_LEFT, KEY_PAGE_DOWN,
                   KEY_PAGE_UP, KEY_RIGHT, KEY_UP, LIGHT_POINTS, LITE, RAND_N, REFR, SCENE_DIR, SPEC,
                   BdptError, Camera, LightPath, PassState, RandState, Sphere, Vec, lib)

__all__ = [
    "Vec", "Sphere", "Camera", "LightPath", "Renderer", "SmallPT", "PassScheduler", "read_scene",
    "default_scene", "update_camera", "camera_key", "sphere_key", "save_ppm", "ppm_name", "glibc_rand",
    "spheres_to_array", "RAND_N", "LIGHT_POINTS", "COUNTER_CAP", "DIFF", "SPEC", "REFR", "LITE",
    "SCENE_DIR", "DEFAULT_DAT", "BdptError",
]

SPHERE_DTYPE = np.dtype([("rad", "<f4"), ("p", "<f4", 3), ("e", "<f4", 3), ("c", "<f4", 3),
                         ("refl", "<i4")])
assert SPHERE_DTYPE.itemsize == ctypes.sizeof(Sphere)
LIGHTPATH_DTYPE = np.dtype([("hp", "<f4", 3), ("rad", "<f4", 3), ("nl", "<f4", 3)])


def _ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def spheres_to_array(spheres) -> np.ndarray:
    """ctypes Sphere array / list of Sphere / structured array -> contiguous SPHERE_DTYPE array."""
    if isinstance(spheres, np.ndarray):
        return np.ascontiguousarray(spheres.astype(SPHERE_DTYPE, copy=False))
    n = len(spheres)
    arr = np.zeros(n, SPHERE_DTYPE)
    if n:
        buf = (Sphere * n)(*spheres)
        ctypes.memmove(arr.ctypes.data, buf, ctypes.sizeof(buf))
    return arr


def _sphere_ptr(arr: np.ndarray):
    return ctypes.cast(ctypes.c_void_p(arr.ctypes.data), ctypes.POINTER(Sphere))


# ---- host utilities (display_func.c / smallpt_cpu.c) ----------------------------------------

def read_scene(path: str) -> Tuple[Camera, np.ndarray]:
    """ReadScene (display_func.c:112-175): returns (camera with orig/target set, spheres)."""
    cam = Camera()
    sp = ctypes.POINTER(Sphere)()
    n = ctypes.c_uint(0)
    rc = lib.bdpt_read_scene(os.fsencode(path), ctypes.byref(cam), ctypes.byref(sp), ctypes.byref(n))
    if rc != BDPT_OK:
        raise BdptError(rc, f"cannot read scene {path}")
    arr = np.zeros(n.value, SPHERE_DTYPE)
    if n.value:
        ctypes.memmove(arr.ctypes.data, sp, n.value * ctypes.sizeof(Sphere))
    lib.bdpt_free_scene(sp)
    return cam, arr


def default_scene() -> Tuple[Camera, np.ndarray]:
    """CornellSpheres (scene.h:7-18) + the no-argument camera (smallpt_cpu.c:404-405)."""
    cam = Camera()
    buf = (Sphere * 9)()
    n = lib.bdpt_default_scene(ctypes.byref(cam), buf)
    arr = np.zeros(n, SPHERE_DTYPE)
    ctypes.memmove(arr.ctypes.data, buf, ctypes.sizeof(buf))
    return cam, arr


def update_camera(cam: Camera, width: int, height: int) -> Camera:
    """UpdateCamera (display_func.c:177-190); width/height are the internal (+1) sizes."""
    lib.bdpt_update_camera(ctypes.byref(cam), int(width), int(height))
    return cam


_KEYS = {"up": KEY_UP, "down": KEY_DOWN, "left": KEY_LEFT, "right": KEY_RIGHT,
         "page_up": KEY_PAGE_UP, "page_down": KEY_PAGE_DOWN}


def camera_key(cam: Camera, key) -> bool:
    """KeyFunc/SpecialFunc camera moves; returns True when the key moved the camera."""
    code = _KEYS[key] if isinstance(key, str) and len(key) > 1 else (ord(key) if isinstance(key, str) else int(key))
    return bool(lib.bdpt_camera_key(ctypes.byref(cam), code))


def sphere_key(spheres: np.ndarray, current: int, key: str) -> bool:
    """KeyFunc sphere edits ('4','6','8','2','9','3'), in place; True when a sphere moved."""
    assert spheres.dtype == SPHERE_DTYPE and spheres.flags.c_contiguous
    return bool(lib.bdpt_sphere_key(_sphere_ptr(spheres), len(spheres), int(current), ord(key)))


def save_ppm(path: str, rgba: np.ndarray, binary: bool = False) -> None:
    """SavePPM (smallpt_cpu.c:239-262): ASCII P3, rows bottom-up; binary=True writes P6."""
    rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
    h, w = rgba.shape[:2]
    fn = lib.bdpt_save_ppm_binary if binary else lib.bdpt_save_ppm
    rc = fn(os.fsencode(path), _ptr(rgba), w, h)
    if rc != BDPT_OK:
        raise BdptError(rc, f"cannot write {path}")


def ppm_name(total_time: float, current_sample: int) -> str:
    """SavePPM's file name (smallpt_cpu.c:245): max1_secondi<total_time %.3f>_exe<sample>.ppm."""
    buf = ctypes.create_string_buffer(128)
    lib.bdpt_ppm_name(buf, len(buf), float(total_time), int(current_sample))
    return buf.value.decode()


def glibc_rand(n: int, seed: int = 1) -> np.ndarray:
    """n values of glibc rand() after srand(seed) (the library's own implementation)."""
    st = RandState()
    lib.bdpt_srand(ctypes.byref(st), seed)
    return np.array([lib.bdpt_rand(ctypes.byref(st)) for _ in range(n)], dtype=np.int64)


class PassScheduler:
    """sid = rand() % RAND_N and the flag/vlp_index state machine of smallpt_cpu.c:270,292-293."""

    def __init__(self):
        self.state = PassState()
        lib.bdpt_pass_state_init(ctypes.byref(self.state))

    def light(self) -> None:
        lib.bdpt_pass_state_light(ctypes.byref(self.state))

    def next(self, npass: int) -> Tuple[np.ndarray, np.ndarray]:
        sid = np.empty(npass, np.uint32)
        vlp = np.empty(npass, np.int32)
        if npass:
            lib.bdpt_pass_schedule(ctypes.byref(self.state), npass, _ptr(sid), _ptr(vlp))
        return sid, vlp

    @property
    def flag(self) -> int:
        return self.state.flag

    @property
    def vlp_index(self) -> int:
        return self.state.vlp_index


# ---- one render context on one GPU -----------------------------------------------------------

class Renderer:
    """One C-ABI context (bdpt_create): device buffers, MT table, VLPs and the accumulation."""

    def __init__(self, spheres, width: int, height: int, camera: Optional[Camera] = None,
                 dat_path: str = DEFAULT_DAT, device: int = 0, devices: Optional[Sequence[int]] = None):
        """devices=[d0, d1, ...]: one multi-device context (bdpt_create_multi): pixel bands over
        the devices, frame assembled on d0 (RCCL when the devices are distinct)."""
        self.width, self.height = int(width), int(height)
        self.spheres = spheres_to_array(spheres)
        h = ctypes.c_void_p()
        if devices is not None:
            devs = np.ascontiguousarray(devices, dtype=np.int32)
            rc = lib.bdpt_create_multi(ctypes.byref(h), _sphere_ptr(self.spheres), len(self.spheres),
                                       self.width, self.height, os.fsencode(dat_path), _ptr(devs), len(devs))
        else:
            rc = lib.bdpt_create(ctypes.byref(h), _sphere_ptr(self.spheres), len(self.spheres),
                                 self.width, self.height, os.fsencode(dat_path), int(device))
        if rc != BDPT_OK:
            raise BdptError(rc, lib.bdpt_create_error().decode())
        self._h = h
        if camera is not None:
            self.set_camera(camera)

    # -- lifecycle
    def close(self) -> None:
        if getattr(self, "_h", None):
            lib.bdpt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _chk(self, rc: int) -> None:
        if rc != BDPT_OK:
            raise BdptError(rc, lib.bdpt_last_error(self._h).decode())

    # -- state
    def set_camera(self, cam: Camera) -> None:
        self.camera = cam
        self._chk(lib.bdpt_set_camera(self._h, ctypes.byref(cam)))

    def set_scene(self, spheres) -> None:
        self.spheres = spheres_to_array(spheres)
        self._chk(lib.bdpt_set_scene(self._h, _sphere_ptr(self.spheres), len(self.spheres)))

    def reset_accum(self) -> None:
        self._chk(lib.bdpt_reset_accum(self._h))

    def set_shard(self, shard: int, nshards: int, band_rows: int = 8) -> None:
        self._chk(lib.bdpt_set_shard(self._h, shard, nshards, band_rows))

    def set_streams(self, streams: int) -> None:
        """Pass streams per pixel (0 = auto: measured choice, -1 = one pass per lane, 1 = fused); results are bit-identical for every value."""
        self._chk(lib.bdpt_set_streams(self._h, streams))

    @property
    def last_streams(self) -> int:
        return int(lib.bdpt_last_streams(self._h))

    @property
    def stream_choice(self) -> int:
        """BDPT_CHOICE_* bits of the auto stream mode's decision (0 while measuring / not auto)."""
        return int(lib.bdpt_stream_choice(self._h))

    def set_stream_choice(self, choice: int) -> None:
        """Apply a decision of the auto stream mode (e.g. rank 0's) without measuring."""
        self._chk(lib.bdpt_set_stream_choice(self._h, int(choice)))

    def device_mode(self, k: int = 0) -> dict:
        """Device k's last kernel: {streams, features, choice} (bdpt_device_mode)."""
        st, ft, ch = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._chk(lib.bdpt_device_mode(self._h, k, ctypes.byref(st), ctypes.byref(ft), ctypes.byref(ch)))
        return {"streams": st.value, "features": [n for b, n in sorted(FEATURES.items()) if ft.value & b],
                "choice": [n for b, n in sorted(CHOICES.items()) if ch.value & b]}

    def set_specialize(self, on: bool) -> None:
        """Scene-specialised kernels (run-time compiled, <= 64 spheres); results are bit-identical."""
        self._chk(lib.bdpt_set_specialize(self._h, int(bool(on))))

    @property
    def last_specialized(self) -> bool:
        return bool(lib.bdpt_last_specialized(self._h))

    @property
    def specialize_status(self) -> str:
        """Why the last path pass did not run a specialised kernel ('' if it did or was not asked)."""
        return lib.bdpt_specialize_status(self._h).decode()

    def set_traversal(self, mode: str) -> None:
        """'auto' (BVH when the scene has one), 'brute' (every sphere) or 'bvh'."""
        self._chk(lib.bdpt_set_traversal(self._h, {"auto": 0, "brute": 1, "bvh": 2}[mode]))

    @property
    def has_bvh(self) -> bool:
        return bool(lib.bdpt_scene_has_bvh(self._h))

    @property
    def last_traversal(self) -> str:
        return {1: "brute", 2: "bvh"}[int(lib.bdpt_last_traversal(self._h))]

    @property
    def last_features(self) -> list:
        """What the last path-pass kernel compiled in (include/bdpt.h BDPT_FEAT_*), by name."""
        bits = int(lib.bdpt_last_kernel_features(self._h))
        return [name for bit, name in sorted(FEATURES.items()) if bits & bit]

    @property
    def num_devices(self) -> int:
        return int(lib.bdpt_num_devices(self._h))

    @property
    def reduce_backend(self) -> str:
        """'rccl' / 'peer' for a multi-device context, 'none' for a one-device context."""
        return lib.bdpt_reduce_backend(self._h).decode()

    @property
    def reduce_info(self) -> str:
        """The frame reduce in words (bdpt_reduce_info): RCCL version, ranks and devices, or why not RCCL."""
        buf = ctypes.create_string_buffer(512)
        n = lib.bdpt_reduce_info(self._h, buf, len(buf))
        if n < 0:
            self._chk(n)
        return buf.value.decode()

    def reduce_frame(self) -> None:
        self._chk(lib.bdpt_reduce_frame(self._h))

    # -- work
    def generate_rand(self, seed: int) -> None:
        self._chk(lib.bdpt_generate_rand(self._h, seed))

    def light_pass(self, current_sample: int = 0) -> None:
        self._chk(lib.bdpt_light_pass(self._h, current_sample))

    def path_passes(self, sid: Sequence[int], vlp: Sequence[int], sync: bool = True) -> None:
        sid = np.ascontiguousarray(sid, dtype=np.uint32)
        vlp = np.ascontiguousarray(vlp, dtype=np.int32)
        assert sid.shape == vlp.shape and sid.ndim == 1
        self._chk(lib.bdpt_path_passes(self._h, _ptr(sid), _ptr(vlp), len(sid)))
        if sync:
            self.synchronize()

    def synchronize(self) -> None:
        self._chk(lib.bdpt_synchronize(self._h))

    def last_path_ms(self) -> float:
        ms = ctypes.c_float()
        self._chk(lib.bdpt_last_path_ms(self._h, ctypes.byref(ms)))
        return ms.value

    def path_timing(self, reset: bool = False) -> Tuple[float, int]:
        """(device ms, kernel launches) of the path passes since the last reset."""
        ms, n = ctypes.c_double(), ctypes.c_longlong()
        self._chk(lib.bdpt_path_timing(self._h, ctypes.byref(ms), ctypes.byref(n), int(reset)))
        return ms.value, n.value

    def kernel_timing(self, reset: bool = False) -> Tuple[float, int]:
        """(ms inside the path kernels alone, launches) since the last reset."""
        ms, n = ctypes.c_double(), ctypes.c_longlong()
        self._chk(lib.bdpt_kernel_timing(self._h, ctypes.byref(ms), ctypes.byref(n), int(reset)))
        return ms.value, n.value

    def device_timing(self) -> list:
        """Per device of the context (devices[0] first): {device, kernel_ms, path_ms, launches,
        owned_pixels} since the last timing reset (bdpt_device_timing; no reset)."""
        out = []
        for k in range(self.num_devices):
            d, km, pm = ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
            n, own = ctypes.c_longlong(), ctypes.c_longlong()
            self._chk(lib.bdpt_device_timing(self._h, k, ctypes.byref(d), ctypes.byref(km), ctypes.byref(pm),
                                             ctypes.byref(n), ctypes.byref(own)))
            out.append({"device": d.value, "kernel_ms": km.value, "path_ms": pm.value,
                        "launches": n.value, "owned_pixels": own.value})
        return out

    def update_pixels(self) -> None:
        self._chk(lib.bdpt_update_pixels(self._h))

    # -- read-back
    def read_radiance(self) -> Tuple[np.ndarray, np.ndarray]:
        col = np.empty((self.height, self.width, 3), np.float32)
        cnt = np.empty((self.height, self.width), np.uint32)
        self._chk(lib.bdpt_read_radiance(self._h, _ptr(col), _ptr(cnt)))
        return col, cnt

    def write_radiance(self, colors: np.ndarray, counter: np.ndarray) -> None:
        """Upload an accumulation state (the counterpart of read_radiance); pixels follow."""
        col = np.ascontiguousarray(colors, np.float32).reshape(self.height, self.width, 3)
        cnt = np.ascontiguousarray(counter, np.uint32).reshape(self.height, self.width)
        self._chk(lib.bdpt_write_radiance(self._h, _ptr(col), _ptr(cnt)))

    def save_checkpoint(self, path: str, host_state: bytes = b"") -> None:
        buf = ctypes.create_string_buffer(host_state, len(host_state)) if host_state else None
        self._chk(lib.bdpt_save_checkpoint(self._h, os.fsencode(path), buf, len(host_state)))

    def load_checkpoint(self, path: str, host_bytes: int = 0) -> bytes:
        """Restore the render state saved with the frame -- scene, camera, MT table (by its seed),
        VLPs -- and the accumulation (bdpt_load_checkpoint); self.spheres and self.camera follow
        the restored values.  Returns the caller state saved with it (host_bytes long)."""
        buf = ctypes.create_string_buffer(host_bytes) if host_bytes else None
        self._chk(lib.bdpt_load_checkpoint(self._h, os.fsencode(path), buf, host_bytes))
        self.spheres = self.get_scene()
        cam = self.get_camera()
        if cam is not None:
            self.camera = cam
        return buf.raw if buf is not None else b""

    def read_pixels(self) -> np.ndarray:
        px = np.empty((self.height, self.width, 4), np.uint8)
        self._chk(lib.bdpt_read_pixels(self._h, _ptr(px)))
        return px

    def read_rand(self) -> np.ndarray:
        t = np.empty(RAND_N, np.float32)
        self._chk(lib.bdpt_read_rand(self._h, _ptr(t)))
        return t

    def read_lightpaths(self) -> np.ndarray:
        lp = np.empty(LIGHT_POINTS, LIGHTPATH_DTYPE)
        self._chk(lib.bdpt_read_lightpaths(self._h, _ptr(lp)))
        return lp

    def write_lightpaths(self, lp: np.ndarray) -> None:
        lp = np.ascontiguousarray(lp, LIGHTPATH_DTYPE)
        assert lp.shape == (LIGHT_POINTS,)
        self._chk(lib.bdpt_write_lightpaths(self._h, _ptr(lp)))

    def rand_seed(self) -> Optional[int]:
        """Seed of the current MT607 table (None before the first light pass)."""
        s = ctypes.c_uint()
        return int(s.value) if lib.bdpt_rand_seed(self._h, ctypes.byref(s)) == BDPT_OK else None

    def get_camera(self) -> Optional[Camera]:
        cam = Camera()
        return cam if lib.bdpt_get_camera(self._h, ctypes.byref(cam)) == BDPT_OK else None

    def get_scene(self) -> np.ndarray:
        n = lib.bdpt_get_scene(self._h, None, 0)
        if n < 0:
            raise BdptError(n, lib.bdpt_last_error(self._h).decode())
        arr = np.zeros(n, SPHERE_DTYPE)
        if n:
            lib.bdpt_get_scene(self._h, _sphere_ptr(arr), n)
        return arr

    def device_buffers(self) -> Tuple[int, int, int]:
        c, n, p = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        self._chk(lib.bdpt_device_buffers(self._h, ctypes.byref(c), ctypes.byref(n), ctypes.byref(p)))
        return c.value, n.value, p.value

    # -- optional display: HIP-GL interop of the caller's pixel-unpack buffer
    def gl_register_pbo(self, pbo: int) -> None:
        """cudaGLRegisterBufferObject (smallpt_cpu.c:122): needs a current OpenGL context."""
        self._chk(lib.bdpt_gl_register_pbo(self._h, int(pbo)))

    def gl_publish(self) -> None:
        """IdleFunc's map / render / unmap (display_func.c:199-215): the frame's pixels into the PBO."""
        self._chk(lib.bdpt_gl_publish(self._h))

    def gl_unregister(self) -> None:
        self._chk(lib.bdpt_gl_unregister(self._h))


# ---- the reference's operator interface (smallpt_cpu.c / display_func.c) --------------------

class SmallPT:
    """Mirror of smallpt_cpu.c's module state and functions, headless.

    SmallPT(w, h, scene) behaves like `smallptCPU <w> <h> <scene>`: sizes get +1
    (smallpt_cpu.c:409-410), UpdateCamera, AllocateBuffers.  IdleFunc() is one frame of the GLUT
    idle loop (display_func.c:192-217); KeyFunc/SpecialFunc replay the keyboard handlers.
    """

    def __init__(self, width: Optional[int] = None, height: Optional[int] = None,
                 scene: Optional[str] = None, device: int = 0, dat_path: str = DEFAULT_DAT):
        if scene is not None:
            self.camera, self.spheres = read_scene(scene)
            self.width, self.height = int(width), int(height)
        else:
            self.camera, self.spheres = default_scene()
            self.width, self.height = 640, 480
        self.height += 1
        self.width += 1
        update_camera(self.camera, self.width, self.height)
        self.device, self.dat_path = device, dat_path
        self.current_sample = 0
        self.reinit_counter = 0
        self.current_sphere = 0
        self.total_time = 0.0
        self.sched = PassScheduler()
        self.renderer: Optional[Renderer] = None
        self.AllocateBuffers()

    @property
    def flag(self) -> int:
        return self.sched.flag

    def AllocateBuffers(self) -> None:                       # smallpt_cpu.c:153
        if self.renderer is None:
            self.renderer = Renderer(self.spheres, self.width, self.height, self.camera,
                                     self.dat_path, self.device)
        else:                                                 # buffers persist (Appendix A.6)
            self.renderer.reset_accum()
            self.renderer.set_scene(self.spheres)

    def FreeBuffers(self) -> None:                           # smallpt_cpu.c:98
        if self.renderer is not None:
            self.renderer.close()
            self.renderer = None

    def UpdateRendering2(self) -> None:                      # smallpt_cpu.c:300-362
        self.renderer.light_pass(self.current_sample)
        self.sched.light()

    def UpdateRendering(self, npass: int = 1) -> float:      # smallpt_cpu.c:265-297 (x npass)
        import time
        sid, vlp = self.sched.next(npass)
        t0 = time.perf_counter()
        self.renderer.path_passes(sid, vlp)
        dt = time.perf_counter() - t0
        self.current_sample += npass
        # static float total_time; total_time += (float)elapsed (smallpt_cpu.c:35,283)
        self.total_time = float(np.float32(np.float32(self.total_time) + np.float32(dt)))
        return self.width * self.height * npass / dt if dt > 0 else float("inf")

    def IdleFunc(self, npass: int = 1) -> None:              # display_func.c:192-217
        if self.flag == 1:
            self.UpdateRendering2()
        if self.flag > 1:
            self.UpdateRendering(npass)

    def ReInit(self, realloc: bool = True) -> None:          # smallpt_cpu.c:373-387
        if realloc:
            self.AllocateBuffers()
        self.reinit_counter += 1
        update_camera(self.camera, self.width, self.height)
        self.renderer.set_camera(self.camera)
        self.current_sample = 0
        if self.reinit_counter % 2 == 0:
            self.UpdateRendering2()
        self.UpdateRendering(1)

    def ReInitScene(self) -> None:                           # smallpt_cpu.c:365-371
        self.current_sample = 0
        self.sched.state.flag = 1
        self.AllocateBuffers()
        self.UpdateRendering2()

    def KeyFunc(self, key: str) -> None:                     # display_func.c:278-382
        if key in "+-":
            n = len(self.spheres)
            self.current_sphere = (self.current_sphere + (1 if key == "+" else n - 1)) % n
            self.ReInitScene()
        elif key in "468293":
            if sphere_key(self.spheres, self.current_sphere, key):
                self.ReInitScene()
        elif camera_key(self.camera, key):
            self.ReInit(True)

    def SpecialFunc(self, key: str) -> None:                 # display_func.c:384-437
        if camera_key(self.camera, key):
            self.ReInit(True)

    def colors(self) -> Tuple[np.ndarray, np.ndarray]:
        return self.renderer.read_radiance()

    def pixels(self) -> np.ndarray:
        return self.renderer.read_pixels()

    _STATE = struct.Struct("<35i3if")          # bdpt_pass_state (31 + f, r, flag, vlp) + 3 ints + float

    def SaveCheckpoint(self, path: str) -> None:
        """Accumulation + pass schedule + host counters (no reference counterpart)."""
        st = self.sched.state
        words = list(st.rng.state) + [st.rng.f, st.rng.r, st.flag, st.vlp_index]
        blob = self._STATE.pack(*words, self.current_sample, self.reinit_counter, self.current_sphere,
                                self.total_time)
        self.renderer.save_checkpoint(path, blob)

    def LoadCheckpoint(self, path: str) -> None:
        """Restore what SaveCheckpoint wrote; rendering continues bit for bit.  The checkpoint
        carries the render state too (camera, spheres, MT table seed, VLPs -- keys may have
        edited them before the save): the context restores it, and the mirror takes over the
        camera and spheres, so later keys continue from the saved state."""
        v = self._STATE.unpack(self.renderer.load_checkpoint(path, self._STATE.size))
        cam = self.renderer.get_camera()
        if cam is not None:
            self.camera = cam
        self.spheres = self.renderer.get_scene()
        self.renderer.spheres = self.spheres
        st = self.sched.state
        for k in range(31):
            st.rng.state[k] = v[k]
        st.rng.f, st.rng.r, st.flag, st.vlp_index = v[31:35]
        self.current_sample, self.reinit_counter, self.current_sphere = v[35:38]
        self.total_time = v[38]

    def SavePPM(self, path: Optional[str] = None, binary: bool = False) -> str:   # smallpt_cpu.c:239-262
        if path is None:
            path = ppm_name(self.total_time, self.current_sample)
        save_ppm(path, self.pixels(), binary)
        return path
