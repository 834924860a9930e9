"""Wall time per step of back-to-back path-pass calls on one GPU, for one forced stream mode.

    python scripts/probe_step.py --scene cornell --passes 128 --streams 64 [--reps 5]

Prints one JSON line (ms per step, path / kernel ms, Msamples/s).  Used for A/B probes whose
variants are selected through the environment (BDPT_JIT_FLAGS, BDPT_POOL, ablation switches):
unlike bench.py it does not check the frame, so ablations that change results can be timed.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))

import gpu_bidirectional_raytracer_amd as g  # noqa: E402
from shard_probe import WARM, run  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--width", type=int, default=1921)
    ap.add_argument("--height", type=int, default=1081)
    ap.add_argument("--passes", type=int, default=128)
    ap.add_argument("--streams", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    W, H = args.width, args.height
    cam, sp = g.read_scene(os.path.join(REPO, "assets", "scenes", args.scene + ".scn"))
    g.update_camera(cam, W, H)
    sched = g.PassScheduler()
    sched.light()
    sid, vlp = sched.next(args.passes * (args.reps + WARM))
    wall, ms, kms, S = run(sp, cam, W, H, sid, vlp, 0, 1, 8, args.streams, args.reps)
    print(json.dumps({"tag": args.tag, "scene": args.scene, "streams_req": args.streams, "streams": S,
                      "ms_per_step": round(wall, 4), "path_ms": round(ms, 4), "kernel_ms": round(kms, 4),
                      "Msamples_s": round(W * H * args.passes / wall / 1e3, 1),
                      "env": {k: v for k, v in os.environ.items() if k.startswith("BDPT_")}}), flush=True)


if __name__ == "__main__":
    main()
