#!/usr/bin/env python3
"""bench.py -- path-pass throughput (Msamples/s) of the MI355X path tracer at 1080p cornell.scn.

One "step" = `--passes` x N fused path passes (RadiancePathTracingKernel, device.cu:544) over this
rank's pixel bands of the 1921x1081 frame (CLI 1920x1080 + the reference's +1).  Weak scaling:
each rank owns 1/N of the pixels (16-row bands interleaved over ranks) and renders N x passes per
step, so the per-GPU work is constant and the job renders N x the spp of the same frame.  The
timed region ends with the RCCL (torch.distributed "nccl") sum-reduce of the radiance frame to
rank 0, which assembles the image (pixels outside a rank's bands are zero, so the sum is exact).

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement" for every field).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Msamples/sec (rays·bounces/s) at 1080p cornell.scn, 1/2/4/8 GPU"

# Per-sample work of the workload, measured once by the CPU restatement over the full 1921x1081
# cornell frame (tests/test_work_model.py keeps these honest; DESIGN.md "Roofline").
WORK = {
    "cornell": {"sphere_tests": 129.4711, "segments": 6.8441, "diffuse": 6.1386, "refr": 0.4528, "rng_reads": 27.0071},
    "cornell_glass": {"sphere_tests": 92.9047, "segments": 6.8374, "diffuse": 4.2323, "refr": 1.02, "rng_reads": 19.9494},
    "caustic": {"sphere_tests": 5.1332, "segments": 1.5151, "diffuse": 0.4516, "refr": 0.0638, "rng_reads": 3.8704},
    "simple": {"sphere_tests": 8.7195, "segments": 1.5033, "diffuse": 0.5039, "refr": 0.0, "rng_reads": 4.0156},
    "synthetic64": {"sphere_tests": 609.1571, "segments": 6.9145, "diffuse": 5.6567, "refr": 0.908, "rng_reads": 25.5348},
    # large scenes: counted on every 36th row (the full frame takes the oracle a minute)
    "complex": {"sphere_tests": 1527.9675, "segments": 1.6307, "diffuse": 0.6397, "refr": 0.0, "rng_reads": 4.5589,
                "_rows_step": 36},
    "mod_cornell": {"sphere_tests": 11602.571, "segments": 6.8993, "diffuse": 6.7583, "refr": 0.1145,
                    "rng_reads": 29.1478, "_rows_step": 36},
}
# FLOP model per primitive (DESIGN.md "Roofline"): sphere test 18, segment shading 28,
# diffuse vertex (NEE to one light + VLP + new direction) 153, refraction 40, camera ray +
# running mean 59.
FLOP = {"sphere_tests": 18, "segments": 28, "diffuse": 153, "refr": 40, "per_sample": 59}
ACCUM_BYTES_PER_PIXEL = 36       # colors 12R+12W, counter 4R+4W, pixels 4W per launch
HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3         # vector fp32 spec (FMA = 2 FLOP)
FP32_NOFMA_TFLOPS = 78.6         # 256 CU x 128 lanes x 2.4 GHz, one mul/add per lane-cycle


def flop_per_sample(w):
    return (FLOP["sphere_tests"] * w["sphere_tests"] + FLOP["segments"] * w["segments"]
            + FLOP["diffuse"] * w["diffuse"] + FLOP["refr"] * w["refr"] + FLOP["per_sample"])


def cpu_baseline(sp, cam, W, H, sid, vlp, seconds):
    """The oracle (CPU restatement) on this host's cores: a bounded sample of the same frame."""
    import numpy as np
    import oracle

    threads = min(16, os.cpu_count() or 1)
    rnd = oracle.mt607(0)
    lp = oracle.light_pass(sp, rnd, 0)
    t = time.perf_counter()
    oracle.path_passes(sp, rnd, cam, W, H, lp, sid[:1], vlp[:1], nthreads=threads)
    t_pass = time.perf_counter() - t
    npass = max(1, min(len(sid), int(round(seconds / max(t_pass, 1e-3)))))
    t = time.perf_counter()
    oracle.path_passes(sp, rnd, cam, W, H, lp, sid[:npass], vlp[:npass], nthreads=threads)
    dt = time.perf_counter() - t
    # one core: every 4th 16-row band, one pass
    t1, n1 = 0.0, 0
    for y0 in range(0, H, 64):
        y1 = min(H, y0 + 16)
        t = time.perf_counter()
        oracle.path_passes(sp, rnd, cam, W, H, lp, sid[:1], vlp[:1], rows=(y0, y1), nthreads=1)
        t1 += time.perf_counter() - t
        n1 += (y1 - y0) * W
    return {"value": W * H * npass / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ CPU restatement, full {W}x{H} cornell frame x {npass} passes "
                      f"(same sids as the GPU), OpenMP {threads} threads; 1-core: every 4th 16-row "
                      f"band x 1 pass",
            "value_1core": n1 / t1 / 1e6, "seconds": round(dt, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--width", type=int, default=1920, help="CLI width (internal = +1)")
    ap.add_argument("--height", type=int, default=1080, help="CLI height (internal = +1)")
    ap.add_argument("--passes", type=int, default=32, help="passes per step per GPU share")
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--traversal", default="auto", choices=["auto", "brute", "bvh"],
                    help="sphere traversal for >16-sphere scenes (results identical)")
    ap.add_argument("--streams", type=int, default=0, help="pass streams per pixel (0 = auto)")
    ap.add_argument("--specialize", type=int, default=1, choices=[0, 1],
                    help="scene-specialised kernels (run-time compiled; results identical)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rehearse", action="store_true",
                    help="multi-rank dry run on fewer GPUs: gloo, ranks share devices (not a measurement)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    import gpu_bidirectional_raytracer_amd as g
    from gpu_bidirectional_raytracer_amd import sharding as shd

    if args.rehearse:
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    W, H = args.width + 1, args.height + 1                   # smallpt_cpu.c:409-410
    cam, sp = g.read_scene(os.path.join(REPO, "assets", "scenes", args.scene + ".scn"))
    g.update_camera(cam, W, H)
    r = g.Renderer(sp, W, H, cam, device=local)
    r.set_shard(rank, world, args.band_rows)
    r.set_traversal(args.traversal)
    r.set_streams(args.streams)
    r.set_specialize(bool(args.specialize))
    r.light_pass(0)                                           # UpdateRendering2
    sched = g.PassScheduler()
    sched.light()
    per_step = args.passes * world
    sid, vlp = sched.next(per_step * (args.warmup + args.steps))

    def step(k):
        a, b = k * per_step, (k + 1) * per_step
        r.path_passes(sid[a:b], vlp[a:b], sync=False)

    def barrier():
        if dist is not None:
            dist.barrier()

    for k in range(args.warmup):
        step(k)
    r.synchronize()
    r.path_timing(reset=True)

    # RCCL reduce target: torch tensors over the library's own device buffers (no copy)
    t_col = t_cnt = None
    if dist is not None:
        t_col, t_cnt = shd.device_tensors(r, f"cuda:{local}")

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        step(k)
    r.synchronize()
    if dist is not None:                                      # assemble the frame on rank 0
        shd.reduce_frame(t_col, t_cnt, dst=0)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([dt], device="cpu" if args.rehearse else f"cuda:{local}", dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    kern_ms, _ = r.kernel_timing()                            # path kernels alone
    dev_ms, launches = r.path_timing()                        # + the pass-stream fold
    samples = W * H * per_step * args.steps                   # every pixel exactly once per pass
    value = samples / dt / 1e6

    if rank == 0:
        if dist is not None:
            r.update_pixels()
            cnt = t_cnt.cpu().numpy()
            assert (cnt == per_step * (args.warmup + args.steps)).all(), "reduced counters wrong"
        own_pixels = shd.owned_pixels(W, H, rank, world, args.band_rows)
        w = WORK.get(args.scene)
        avg_launch_s = kern_ms / 1e3 / max(launches, 1)
        passes_per_launch = per_step * args.steps / max(launches, 1)
        roofline = valu = None
        if w is not None:
            samples_per_launch = own_pixels * passes_per_launch
            if r.last_streams > 1:
                # pass streams: the path kernel reads the counter once and writes 12 B of radiance
                # per sample; the fold kernel (not this launch) does the colors/pixels RMW
                bytes_per_launch = own_pixels * 4 + samples_per_launch * (4 * w["rng_reads"] + 12)
            else:
                bytes_per_launch = own_pixels * ACCUM_BYTES_PER_PIXEL + samples_per_launch * 4 * w["rng_reads"]
            achieved = bytes_per_launch / avg_launch_s / 1e9
            traffic = None
            pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
            if os.path.exists(pmc):
                rec = json.load(open(pmc))
                if rec.get("scene") == args.scene and rec.get("passes_per_launch") == passes_per_launch \
                        and rec.get("pass_streams") in (None, r.last_streams) \
                        and rec.get("specialized", False) == r.last_specialized \
                        and rec.get("width") == W and rec.get("height") == H and world == 1:
                    traffic = rec.get("hbm_bytes_per_launch")
            roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                        "bytes_per_launch": int(bytes_per_launch), "avg_launch_ms": round(avg_launch_s * 1e3, 4),
                        "launches": launches}
            fl = flop_per_sample(w) * samples_per_launch / avg_launch_s / 1e12
            valu = {"achieved": round(fl, 2), "unit": "TFLOP/s", "peak": FP32_PEAK_TFLOPS,
                    "frac": round(fl / FP32_PEAK_TFLOPS, 4), "peak_no_fma": FP32_NOFMA_TFLOPS,
                    "frac_no_fma": round(fl / FP32_NOFMA_TFLOPS, 4),
                    "flop_per_sample": round(flop_per_sample(w), 1),
                    "note": "bound: fp32 VALU (no contraction, correctly rounded div/sqrt); "
                            "FLOP model in DESIGN.md"}
            pv = os.path.join(REPO, "profiles", "pmc_valu.json")
            if os.path.exists(pv) and world == 1:
                rec = json.load(open(pv))
                if rec.get("scene") == args.scene and rec.get("passes_per_launch") == passes_per_launch \
                        and rec.get("pass_streams") == r.last_streams and rec.get("width") == W \
                        and rec.get("specialized", False) == r.last_specialized:
                    valu["busy_pmc"] = rec["valu_busy"]
                    valu["lane_utilisation_pmc"] = rec["valu_lane_utilisation"]
            if r.last_traversal == "bvh":
                valu["note"] = ("reference-equivalent FLOPs: the reference tests every sphere; the BVH "
                                "skips most tests, so this is work avoided, not VALU throughput")
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(sp, cam, W, H, sid, vlp, args.cpu_seconds)
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic: reference cornell.scn + MT607 table (seed 0) + glibc-rand pass offsets",
            "config": {"workload": f"{args.scene}.scn {W}x{H} internal (CLI {args.width}x{args.height}), "
                                   f"<=7-segment eye paths + NEE + 1 VLP per diffuse vertex",
                       "scene": args.scene, "width": W, "height": H, "passes_per_step": per_step,
                       "spp_total": per_step * (args.warmup + args.steps),
                       "parallelism": f"pixel bands x{world} ({args.band_rows}-row, interleaved)",
                       "pass_streams": r.last_streams, "traversal": r.last_traversal,
                       "specialized": r.last_specialized},
            "device_ms_per_step": round(dev_ms / args.steps, 3),
            "roofline": roofline, "valu": valu, "cpu_baseline": cpu,
        }
        if cpu:
            line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        if args.rehearse:
            line["rehearsal"] = "ranks share GPUs over gloo: exercises the multi-rank flow, not a measurement"
        print(json.dumps(line), flush=True)
    r.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
