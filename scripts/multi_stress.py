"""Repeated one-GPU multi-device contexts (bdpt_create_multi([0]): in-process RCCL communicator of
one) in one process, to reproduce an intermittent abort inside bdpt_create_multi seen twice in the
full GPU suite (round 6, sessions s1 and s5).  Run with NCCL_DEBUG=WARN so RCCL's reason is printed.

    NCCL_DEBUG=WARN python scripts/multi_stress.py [--n 40]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import gpu_bidirectional_raytracer_amd as g  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=40)
    args = ap.parse_args()
    cam, sp = g.read_scene(os.path.join(REPO, "assets", "scenes", "cornell.scn"))
    g.update_camera(cam, 65, 49)
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(8)
    t0 = time.time()
    for k in range(args.n):
        with g.Renderer(sp, 65, 49, cam, devices=[0]) as r:
            r.light_pass(0)
            r.path_passes(sid, vlp)
            r.read_radiance()
            info = r.reduce_info
        with g.Renderer(sp, 65, 49, cam, device=0) as r:     # a plain context in between
            r.light_pass(0)
            r.path_passes(sid, vlp)
        print(f"{k} ok {time.time() - t0:.1f}s {info}", flush=True)


if __name__ == "__main__":
    main()
