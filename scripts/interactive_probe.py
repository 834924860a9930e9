"""Per-call cost of the drop-in's interactive pattern (the reference's IdleFunc: one
UpdateRendering = one pass per call, then read the pixels for display) vs fused passes.

    python scripts/interactive_probe.py [--width 640 --height 480 --calls 200]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import gpu_bidirectional_raytracer_amd as g  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--scene", default="cornell")
    args = ap.parse_args()
    W, H = args.width + 1, args.height + 1
    cam, sp = g.read_scene(os.path.join(REPO, "assets", "scenes", args.scene + ".scn"))
    g.update_camera(cam, W, H)
    r = g.Renderer(sp, W, H, cam, device=0)
    r.light_pass(0)
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(4 * args.calls + 20)
    for k in range(10):                                    # warm-up
        r.path_passes(sid[k:k + 1], vlp[k:k + 1])
    # the multi-pass call below resolves (compiles) the pass-stream kernel and runs the auto mode's
    # measured calls: do that untimed, then reset the mode so one-pass calls stay fused
    for k in range(7):
        b = 10 + 3 * args.calls + k * (args.calls // 7)
        r.path_passes(sid[b:b + args.calls // 7], vlp[b:b + args.calls // 7])
    out = {"W": W, "H": H, "calls": args.calls}
    for mode in ("pass", "pass+pixels"):
        base = 10 if mode == "pass" else 10 + args.calls
        t0 = time.perf_counter()
        for k in range(args.calls):
            r.path_passes(sid[base + k:base + k + 1], vlp[base + k:base + k + 1])
            if mode == "pass+pixels":
                r.read_pixels()
        dt = time.perf_counter() - t0
        out[mode + "_us_per_call"] = round(dt / args.calls * 1e6, 1)
    base = 10 + 2 * args.calls
    r.path_timing(reset=True)
    t0 = time.perf_counter()
    r.path_passes(sid[base:base + args.calls], vlp[base:base + args.calls])
    dt = time.perf_counter() - t0
    kms, _ = r.kernel_timing()
    out["fused_us_per_pass"] = round(dt / args.calls * 1e6, 1)
    out["kernel_us_per_pass"] = round(kms * 1e3 / args.calls, 1)
    r.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
