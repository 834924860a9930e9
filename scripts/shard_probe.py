"""Single-GPU rehearsal of the multi-GPU step (bench.py --gpus N).

For each N, the first and last rank's share of an N-way band shard (1/N of the rows; N x passes
for weak scaling, the same passes with --strong) is rendered on one GPU with auto pass streams
(after the auto mode's ten measured calls) and with the S values asked for, and its device time
is compared with the N = 1 step: efficiency = t(N=1) / t(rank share), over N for --strong, with t
the wall time of back-to-back asynchronous calls between two synchronisations (as bench.py times its steps:
a pass-stream call's fold overlaps the next call's path kernel); the device ms of the calls
(path_ms, which ends with each call's fold) and of the path kernels alone (kernel_ms) are printed
beside it.  The RCCL reduce is not included (it runs once per frame, not per step).

    python scripts/shard_probe.py [--scene cornell] [--passes 16] [--reps 3]
    python scripts/shard_probe.py --scene caustic --passes 128 --strong --streams 1,32
    python scripts/shard_probe.py --workload weak64 [--passes 128] [--reps 3]

--workload weak64 rehearses BASELINE configs[4] (bench.py `weak64`): synthetic64 at 4097x4097 cut
into 8 FIXED bands of 512 rows, GPU r of 8 renders band r at the bench's passes per step.  Every band
is timed as rank r of 8 on this one GPU; the one-GPU bench times band 0, and an 8-GPU step lasts as
long as the slowest band, so the predicted weak-scaling efficiency is T1 / T8 = t(band 0) / max_r
t(band r) (before the frame reduce).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import gpu_bidirectional_raytracer_amd as g  # noqa: E402
from gpu_bidirectional_raytracer_amd import sharding as shd  # noqa: E402


WARM = 11


def run(sp, cam, W, H, sid, vlp, shard, nshards, band, streams, reps):
    r = g.Renderer(sp, W, H, cam, device=0)
    r.set_shard(shard, nshards, band)
    r.set_streams(streams)
    r.light_pass(0)
    n = len(sid) // (reps + WARM)
    for k in range(WARM):                               # warm-up (the auto mode measures 10 calls)
        r.path_passes(sid[k * n:(k + 1) * n], vlp[k * n:(k + 1) * n], sync=False)
    r.synchronize()
    r.path_timing(reset=True)
    r.kernel_timing(reset=True)
    t0 = time.perf_counter()
    for k in range(WARM, WARM + reps):
        r.path_passes(sid[k * n:(k + 1) * n], vlp[k * n:(k + 1) * n], sync=False)
    r.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    ms, launches = r.path_timing()
    kms, _ = r.kernel_timing()
    S = r.last_streams
    r.close()
    return wall / reps, ms / reps, kms / reps, S


def weak64(args):
    """Per-band cost of configs[4]'s eight fixed 512-row bands (see the module docstring)."""
    W, H, band, nb = 4097, 4097, 512, 8
    cam, sp = g.read_scene(os.path.join(REPO, "assets", "scenes", "synthetic64.scn"))
    g.update_camera(cam, W, H)
    sched = g.PassScheduler()
    sched.light()
    sid, vlp = sched.next(args.passes * (args.reps + WARM))
    rows = []
    for r in range(nb):
        wall, ms, kms, S = run(sp, cam, W, H, sid, vlp, r, nb, band, 0, args.reps)
        rr = shd.owned_row_ranges(H, r, nb, band)               # band 0 also owns row 4096
        px = shd.owned_pixels(W, H, r, nb, band)
        rec = {"band": r, "rows": [list(x) for x in rr], "streams": S, "ms_per_step": round(wall, 3),
               "path_ms": round(ms, 3), "kernel_ms": round(kms, 3),
               "Msamples_s": round(px * args.passes / wall / 1e3, 1)}
        rows.append(rec)
        print(json.dumps(rec), flush=True)
    t1, t8 = rows[0]["ms_per_step"], max(x["ms_per_step"] for x in rows)
    slow = max(rows, key=lambda x: x["ms_per_step"])["band"]
    print(json.dumps({"workload": "weak64", "passes_per_step": args.passes, "t1_band0_ms": t1,
                      "t8_slowest_band_ms": t8, "slowest_band": slow,
                      "predicted_weak_efficiency_T1_over_T8": round(t1 / t8, 4),
                      "mean_band_ms": round(sum(x["ms_per_step"] for x in rows) / nb, 3),
                      "note": "one GPU times each band as rank r of 8; the RCCL frame reduce is not included"}),
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default=None, choices=["weak64"],
                    help="weak64: time configs[4]'s eight fixed bands one after another")
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--passes", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--streams", default="", help="S values to try besides auto, e.g. 1,2,8")
    ap.add_argument("--strong", action="store_true", help="same passes for every N (strong scaling)")
    args = ap.parse_args()
    if args.workload == "weak64":
        if args.passes == 16:                           # the bench's passes per step for weak64
            args.passes = 128
        return weak64(args)
    W, H = 1921, 1081
    cam, sp = g.read_scene(os.path.join(REPO, "assets", "scenes", args.scene + ".scn"))
    g.update_camera(cam, W, H)
    sched = g.PassScheduler()
    sched.light()
    t1 = None
    for N in [int(x) for x in args.ns.split(",")]:
        per = args.passes * (1 if args.strong else N)
        sid, vlp = sched.next(per * (args.reps + WARM))
        extra = [int(x) for x in args.streams.split(",") if x] if args.streams else ([] if N == 1 else [1])
        for streams in [0] + extra:
            worst = wpath = wkern = 0.0
            for shard in sorted({0, N - 1}):
                wall, ms, kms, S = run(sp, cam, W, H, sid, vlp, shard, N, args.band_rows, streams, args.reps)
                worst, wpath, wkern = max(worst, wall), max(wpath, ms), max(wkern, kms)
            if N == 1 and streams == 0:
                t1 = worst
            eff = t1 / worst / (N if args.strong else 1) if t1 else None
            print(json.dumps({"N": N, "streams_req": streams, "streams": S, "ms_per_step": round(worst, 3),
                              "path_ms": round(wpath, 3), "kernel_ms": round(wkern, 3),
                              "efficiency": round(eff, 4) if eff else None,
                              "whole_job_Msamples_s": round(W * H * per / worst / 1e3, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
