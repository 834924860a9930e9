"""ORACLE -- test infrastructure only.  Restatement of the reference's host control flow:
the GLUT idle loop and key handlers driving the render path, on top of the CPU restatement.

    IdleFunc        display_func.c:192-217  (flag == 1 -> light pass; flag > 1 -> path pass)
    UpdateRendering smallpt_cpu.c:265-297   (sid = rand() % RAND_N; flag / vlp_index machine)
    UpdateRendering2 smallpt_cpu.c:300-362  (MT table seeded current_sample*5 + light pass; flag=2)
    ReInitScene     smallpt_cpu.c:365-371   (current_sample=0, flag=1, realloc, light pass)
    ReInit          smallpt_cpu.c:373-387   (realloc, reinit_counter++, UpdateCamera,
                                             light pass on even counts, one path pass)
    KeyFunc         display_func.c:276-382, SpecialFunc display_func.c:384-437

Buffers follow the documented fixes: AllocateBuffers zeroes the counter
(smallpt_cpu.c:204) and the colors follow from `counter == 0` assigning; the MT table and
dev_lp persist across a re-allocation (Appendix A.6) instead of being left uninitialised.
`rand()` is glibc's, seeded 1 as by default: GlibcRand restates glibc's random_r TYPE_3 with
private state (pinned against libc.so.6's rand() in tests/test_replay_host.py).  Calling
libc's rand() itself would share the process-global state with every library in the process
(an in-process compiler draws from it, shifting the sequence under the test).
"""
from __future__ import annotations

import numpy as np

from . import (RAND_N, SPHERE_DTYPE, key_camera, light_pass, mt607, path_passes,
               special_key, update_camera)

MAX_ITER = 3          # smallpt_cpu.c: flag cycles 2 -> 3 -> (vlp_index += MAX_VLP; 1 -> 2)
MAX_VLP = 1


class GlibcRand:
    """glibc rand()/srand() (stdlib/random_r.c, TYPE_3: x**31 + x**3 + 1, 310 discarded
    outputs after seeding), with the state owned by this object."""

    def __init__(self, seed: int = 1):
        self.srand(seed)

    def srand(self, seed: int) -> None:
        seed = seed & 0xFFFFFFFF or 1
        r = [seed if seed < 2**31 else seed - 2**32]
        word = r[0]
        for _ in range(1, 31):                       # 16807 * word % (2^31 - 1), Schrage's method
            hi = abs(word) // 127773 * (1 if word >= 0 else -1)       # C division truncates
            lo = word - hi * 127773
            word = 16807 * lo - 2836 * hi
            if word < 0:
                word += 2147483647
            r.append(word)
        self._r = [x & 0xFFFFFFFF for x in r]
        self._f, self._b = 3, 0
        for _ in range(310):
            self.rand()

    def rand(self) -> int:
        val = (self._r[self._f] + self._r[self._b]) & 0xFFFFFFFF
        self._r[self._f] = val
        self._f += 1
        if self._f >= 31:
            self._f = 0
            self._b += 1
        else:
            self._b += 1
            if self._b >= 31:
                self._b = 0
        return val >> 1


class Session:
    """One reference process: globals of smallpt_cpu.c / display_func.c as attributes."""

    def __init__(self, spheres: np.ndarray, orig, target, width: int, height: int,
                 rows: tuple[int, int] | None = None):
        self._rand = GlibcRand(1)
        self.spheres = np.ascontiguousarray(spheres.astype(SPHERE_DTYPE, copy=True))
        self.width, self.height = width, height          # internal (+1 applied by caller)
        self.camera = update_camera(orig, target, width, height)
        self.rows = rows
        self.current_sample = 0
        self.reinit_counter = 0
        self.current_sphere = 0
        self.flag = 1
        self.vlp_index = MAX_VLP
        self.rnd = None
        self.lp = None
        self.colors = np.zeros((height, width, 3), np.float32)
        self.counter = np.zeros((height, width), np.uint32)
        self.pixels = np.zeros((height, width, 4), np.uint8)

    # AllocateBuffers smallpt_cpu.c:153-237 (the spheres are re-uploaded; counter := 0)
    def AllocateBuffers(self):
        self.counter[...] = 0

    def UpdateRendering2(self):
        self.rnd = mt607(self.current_sample * 5)
        self.lp = light_pass(self.spheres, self.rnd, self.current_sample)
        self.flag = 2

    def UpdateRendering(self):
        sid = self._rand.rand() % RAND_N
        vlp = self.vlp_index % 4096                      # Appendix A.3 wrap
        self.colors, self.counter, self.pixels = path_passes(
            self.spheres, self.rnd, self.camera, self.width, self.height, self.lp,
            np.array([sid], np.uint32), np.array([vlp], np.int32),
            self.colors, self.counter, self.pixels, rows=self.rows)
        self.current_sample += 1
        if self.flag == MAX_ITER:
            self.vlp_index += MAX_VLP
            self.flag = 1
        if self.flag < MAX_ITER:
            self.flag += 1

    def IdleFunc(self):
        if self.flag == 1:
            self.UpdateRendering2()
        if self.flag > 1:
            self.UpdateRendering()

    def ReInitScene(self):
        self.current_sample = 0
        self.flag = 1
        self.AllocateBuffers()
        self.UpdateRendering2()

    def ReInit(self, realloc: int = 1):
        if realloc:
            self.AllocateBuffers()
        self.reinit_counter += 1
        c = update_camera(self.camera["orig"][0], self.camera["target"][0], self.width, self.height)
        self.camera = c
        self.current_sample = 0
        if self.reinit_counter % 2 == 0:
            self.UpdateRendering2()
        self.UpdateRendering()

    def KeyFunc(self, key: str):
        n = len(self.spheres)
        if key == "+":
            self.current_sphere = (self.current_sphere + 1) % n
            self.ReInitScene()
        elif key == "-":
            self.current_sphere = (self.current_sphere + (n - 1)) % n
            self.ReInitScene()
        elif key in "468293" and len(key) == 1:          # display_func.c:347-370
            p = self.spheres[self.current_sphere]["p"]
            axis, sign = {"4": (0, -1), "6": (0, 1), "8": (2, -1), "2": (2, 1),
                          "9": (1, 1), "3": (1, -1)}[key]
            p[axis] = np.float32(p[axis] + np.float32(sign) * (np.float32(0.5) * np.float32(10.0)))
            self.ReInitScene()
        elif key_camera(self.camera, key):
            self.ReInit(1)

    def SpecialFunc(self, key: str):
        if special_key(self.camera, key):
            self.ReInit(1)


def save_ppm_text(pixels: np.ndarray) -> str:
    """SavePPM file body (smallpt_cpu.c:247-258): "P3\\n%d %d\\n%d\\n", then rows from y = H-1
    down to 0, "%d %d %d " per pixel (R, G, B of the uchar4)."""
    h, w = pixels.shape[:2]
    parts = ["P3\n%d %d\n%d\n" % (w, h, 255)]
    for y in range(h - 1, -1, -1):
        parts.append("".join("%d %d %d " % (int(p[0]), int(p[1]), int(p[2])) for p in pixels[y]))
    return "".join(parts)


def ppm_name(total_time: float, current_sample: int) -> str:
    """smallpt_cpu.c:245 sprintf(name, "max%d_secondi%.3f_exe%d.ppm", MAX_VLP, total_time, ...)
    with the float total_time promoted to double by the varargs call."""
    return "max%d_secondi%.3f_exe%d.ppm" % (MAX_VLP, float(np.float32(total_time)), current_sample)
