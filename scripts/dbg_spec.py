"""Debug: SmallPT key replay with and without scene-specialised kernels, compared step by step."""
import os, sys, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import gpu_bidirectional_raytracer_amd as g
S = "assets/scenes/cornell.scn"
SCRIPT = ["w", "left", "+", "4", "up", " ", "a", "page_up", "-", "9"]
runs = []
for spec in (True, False):
    spt = g.SmallPT(20, 14, S, device=0)
    spt.renderer.set_specialize(spec)
    for _ in range(3):
        spt.IdleFunc()
    out = []
    for k in SCRIPT:
        (spt.SpecialFunc if len(k) > 1 else spt.KeyFunc)(k)
        for _ in range(2):
            spt.IdleFunc()
        col, cnt = spt.colors()
        out.append((col.copy(), cnt.copy(), spt.renderer.last_specialized, spt.renderer.specialize_status,
                    spt.spheres.copy()))
    runs.append(out)
for i, k in enumerate(SCRIPT):
    a, b = runs[0][i], runs[1][i]
    print(i, repr(k), "spec", a[2], repr(a[3]), "col mismatch", int((a[0] != b[0]).sum()),
          "cnt mismatch", int((a[1] != b[1]).sum()))
# direct: moved sphere, one pass per call (non-stream kernel)
cam, sp = g.read_scene(S)
W, H = 21, 15
g.update_camera(cam, W, H)
sp[1]["p"][0] -= 5.0
res = []
for spec in (True, False):
    with g.Renderer(sp, W, H, cam, device=0) as r:
        r.set_specialize(spec)
        r.light_pass(0)
        s = g.PassScheduler(); s.light()
        for _ in range(3):
            sid, vlp = s.next(1)
            r.path_passes(sid, vlp)
        res.append((r.read_radiance()[0], r.last_specialized, r.last_streams))
print("direct npass=1 moved: spec", res[0][1], "streams", res[0][2], "mismatch", int((res[0][0] != res[1][0]).sum()))
