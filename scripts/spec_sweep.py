"""Per-scene A/B of scene-specialised vs precompiled path kernels in one process (same box):
1921x1081, 32 passes per launch, path-kernel device time from the library's HIP events.

    python scripts/spec_sweep.py [scene ...] > gpurun_out/spec_sweep.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import gpu_bidirectional_raytracer_amd as g  # noqa: E402

SCENES = os.path.join(os.path.dirname(g.__file__), "..", "assets", "scenes")
W, H, NPASS, LAUNCHES = 1921, 1081, 32, int(os.environ.get("SWEEP_LAUNCHES", "4"))


def run(name, spec, waves=None):
    cam, sp = g.read_scene(os.path.join(SCENES, name + ".scn"))
    g.update_camera(cam, W, H)
    with g.Renderer(sp, W, H, cam, device=0) as r:
        r.set_specialize(spec)
        r.light_pass(0)
        s = g.PassScheduler()
        s.light()
        sid, vlp = s.next(NPASS)
        r.path_passes(sid, vlp)                                 # warm-up (and compile)
        r.kernel_timing(reset=True)
        for _ in range(LAUNCHES):
            sid, vlp = s.next(NPASS)
            r.path_passes(sid, vlp, sync=False)
        r.synchronize()
        ms, n = r.kernel_timing(reset=True)
        return ms / n, r.last_specialized, r.specialize_status, r.last_traversal


def main():
    names = sys.argv[1:] or sorted(f[:-4] for f in os.listdir(SCENES) if f.endswith(".scn"))
    for name in names:
        base = run(name, False)
        spec = run(name, True)
        rec = {"scene": name, "ms_precompiled": round(base[0], 4), "ms_specialised": round(spec[0], 4),
               "speedup": round(base[0] / spec[0], 4), "specialised": spec[1], "status": spec[2],
               "traversal": base[3],
               "msamples_s_specialised": round(W * H * NPASS / spec[0] / 1e3, 1)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
