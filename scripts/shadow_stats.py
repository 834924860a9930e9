"""Shadow-round statistics of the path kernel (instrumentation build: make variant NAME=stats
EXTRA_HIPFLAGS=-DBDPT_STATS; run with BDPT_LIB=variants/stats/libbdpt.so): rays per shadow step,
rounds per step, queue-round lane utilisation, alive lanes per wave segment."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: F401,E402  (one HIP runtime: torch's)

import gpu_bidirectional_raytracer_amd as g  # noqa: E402
from gpu_bidirectional_raytracer_amd import _lib  # noqa: E402

for scene in (sys.argv[1:] or ["cornell"]):
    W, H = 1921, 1081
    cam, sp = g.read_scene(os.path.join(REPO, "assets", "scenes", scene + ".scn"))
    g.update_camera(cam, W, H)
    out = (ctypes.c_ulonglong * 8)()
    with g.Renderer(sp, W, H, cam, device=0) as r:
        r.light_pass(0)
        sched = g.PassScheduler()
        sched.light()
        sid, vlp = sched.next(32)
        r.synchronize()
        _lib.lib.bdpt_debug_stats(out, 1)
        r.path_passes(sid, vlp)
        r.synchronize()
        _lib.lib.bdpt_debug_stats(out, 1)
    st = np.array(list(out), dtype=np.float64)
    print(f"{scene}: shadow steps {st[0]:.0f}, rays/step {st[2]/st[0]:.2f}, rounds/step {st[1]/st[0]:.3f}, "
          f"round lane utilisation {st[2]/(64*st[1]):.3f}, diffuse lanes/step {st[3]/st[0]:.2f}, "
          f"wave segments {st[4]:.0f}, alive lanes/segment {st[5]/st[4]:.2f}, shadow steps/segment {st[0]/st[4]:.3f}")
