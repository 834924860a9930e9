#!/usr/bin/env python3
"""bench.py -- path-pass throughput (Msamples/s) of the MI355X path tracer.

One "step" = one batch of fused path passes (RadiancePathTracingKernel, device.cu:544) over this
rank's pixels.  Workloads (`--workload`, BASELINE.json configs):

  cornell1080 (default; the metric's config, configs[1] at 1080p): cornell.scn 1921x1081 internal
      (CLI 1920x1080 + the reference's +1).  Weak scaling: each rank owns 1/N of the pixels
      (8-row bands interleaved over ranks) and renders N x `--passes` passes per step, so the
      per-GPU work is constant and the job renders N x the spp of the same frame.
  caustic8 (configs[3]): caustic.scn 1921x1081, 8-row interleaved bands over N ranks, `--passes`
      passes of the whole frame per step.  Strong scaling (the frame and spp are fixed).
  weak64 (configs[4]): the 64-sphere synthetic scene at 4097x4097, cut into 8 bands of 512 rows;
      rank r renders band r (1 GPU: one 4097x512 band, 8 GPUs: the full frame).  Weak scaling.

With N > 1 the timed region ends with the RCCL (torch.distributed "nccl") sum-reduce of the
radiance frame to rank 0, which assembles the image (pixels outside a rank's bands are zero, so
the sum is exact).  Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement" for the fields).
"""
import argparse
import json
import os
import socket
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Msamples/sec (rays·bounces/s) at 1080p cornell.scn, 1/2/4/8 GPU"

WORKLOADS = {
    "cornell1080": dict(scene="cornell", width=1920, height=1080, passes=32, band_rows=8, fixed_bands=0,
                        scaling="weak", config="configs[1] scene at 1080p (the metric's config)"),
    "caustic8": dict(scene="caustic", width=1920, height=1080, passes=128, band_rows=8, fixed_bands=0,
                     scaling="strong", config="configs[3]: caustic.scn 1920x1080, pixel bands over N GPUs"),
    "weak64": dict(scene="synthetic64", width=4096, height=4096, passes=128, band_rows=512, fixed_bands=8,
                   scaling="weak", config="configs[4]: 64-sphere synthetic 4096x4096, one 4097x512 band per GPU"),
}

# Per-sample work of each scene, measured once by the CPU restatement over the full 1921x1081
# frame (tests/test_work_model.py keeps these honest; DESIGN.md "Roofline").
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
# fp32 VALU: 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz = 78.6 T lane-ops/s; the 157.3 TFLOP/s spec
# counts an FMA as 2 FLOP.  The path is built with -ffp-contract=off (parity), so its adds and
# multiplies issue one per lane-cycle: 78.6 T is its ceiling, 157.3 T the FMA figure.
FP32_NOFMA_TFLOPS = 78.6
FP32_PEAK_TFLOPS = 157.3


def flop_per_sample(w):
    return (FLOP["sphere_tests"] * w["sphere_tests"] + FLOP["segments"] * w["segments"]
            + FLOP["diffuse"] * w["diffuse"] + FLOP["refr"] * w["refr"] + FLOP["per_sample"])


def host_cpus():
    """The CPUs this process may use: affinity mask, capped by a cgroup CPU quota if one is set."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota, "threads": usable, "model": model}


def cpu_baseline(sp, cam, W, H, rows, sid, vlp, seconds):
    """The oracle (CPU restatement) on every CPU this job may use: a bounded sample of the same
    workload (its pixel region `rows`, the same sids), plus a 1-core figure."""
    import oracle

    cpus = host_cpus()
    threads = cpus["threads"]
    rnd = oracle.mt607(0)
    lp = oracle.light_pass(sp, rnd, 0)
    y0, y1 = rows
    cal = (y0, min(y1, y0 + 32))                      # calibration: one pass over 32 rows
    t = time.perf_counter()
    oracle.path_passes(sp, rnd, cam, W, H, lp, sid[:1], vlp[:1], rows=cal, nthreads=threads)
    rate = (cal[1] - cal[0]) * W / max(time.perf_counter() - t, 1e-4)
    target = rate * seconds
    region = (y1 - y0) * W
    if target >= region:
        npass, ry = max(1, min(len(sid), int(target // region))), (y0, y1)
    else:
        npass, ry = 1, (y0, y0 + max(8, int(target // W)))
    t = time.perf_counter()
    oracle.path_passes(sp, rnd, cam, W, H, lp, sid[:npass], vlp[:npass], rows=ry, nthreads=threads)
    dt = time.perf_counter() - t
    value = (ry[1] - ry[0]) * W * npass / dt / 1e6
    # one core: every 4th 8-row band of the region, one pass
    t1, n1 = 0.0, 0
    for b0 in range(y0, y1, 32):
        b1 = min(y1, b0 + 8)
        t = time.perf_counter()
        oracle.path_passes(sp, rnd, cam, W, H, lp, sid[:1], vlp[:1], rows=(b0, b1), nthreads=1)
        t1 += time.perf_counter() - t
        n1 += (b1 - b0) * W
        if t1 > seconds / 3:
            break
    v1 = n1 / t1 / 1e6
    return {"value": round(value, 3), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ CPU restatement (OpenMP, {threads} threads = every CPU this job may use), "
                      f"rows {ry[0]}..{ry[1]} of the {W}x{H} frame x {npass} passes (same sids as the GPU); "
                      f"1-core: every 4th 8-row band x 1 pass",
            "seconds": round(dt, 2), "value_1core": round(v1, 4),
            "nproc": cpus["nproc"], "affinity_cpus": cpus["affinity"], "cgroup_quota_cpus": cpus["cgroup_quota_cpus"],
            "cpu_model": cpus["model"],
            "node_linear_estimate": round(v1 * cpus["nproc"], 2),
            "node_linear_estimate_note": "1-core rate x nproc: an upper bound for the whole host (perfect scaling)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="cornell1080", choices=sorted(WORKLOADS))
    ap.add_argument("--scene", default=None, help="override the workload's scene (same frame layout)")
    ap.add_argument("--width", type=int, default=None, help="CLI width (internal = +1)")
    ap.add_argument("--height", type=int, default=None, help="CLI height (internal = +1)")
    ap.add_argument("--passes", type=int, default=None, help="passes per step (per GPU share for weak scaling)")
    ap.add_argument("--band-rows", type=int, default=None)
    ap.add_argument("--traversal", default="auto", choices=["auto", "brute", "bvh"],
                    help="sphere traversal for >16-sphere scenes (results identical)")
    ap.add_argument("--streams", type=int, default=0, help="pass streams per pixel (0 = auto: measured choice of one pass per lane or the fused kernel; -1 = one pass per lane; 1 = fused)")
    ap.add_argument("--specialize", type=int, default=1, choices=[0, 1],
                    help="scene-specialised kernels (run-time compiled; results identical)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rehearse", action="store_true",
                    help="multi-rank dry run on fewer GPUs: gloo, ranks share devices (not a measurement)")
    args = ap.parse_args()
    wl = dict(WORKLOADS[args.workload])
    for k in ("scene", "width", "height", "passes", "band_rows"):
        if getattr(args, k) is not None:
            wl[k] = getattr(args, k)

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

    W, H = wl["width"] + 1, wl["height"] + 1                 # smallpt_cpu.c:409-410
    band = wl["band_rows"]
    nshards = wl["fixed_bands"] or world                     # weak64: 8 fixed bands, rank r renders band r
    if world > nshards:
        raise SystemExit(f"workload {args.workload} has {nshards} bands: at most {nshards} ranks")
    cam, sp = g.read_scene(os.path.join(REPO, "assets", "scenes", wl["scene"] + ".scn"))
    g.update_camera(cam, W, H)
    r = g.Renderer(sp, W, H, cam, device=local)
    r.set_shard(rank, nshards, band)
    r.set_traversal(args.traversal)
    r.set_streams(args.streams)
    r.set_specialize(bool(args.specialize))
    r.light_pass(0)                                           # UpdateRendering2
    sched = g.PassScheduler()
    sched.light()
    per_step = wl["passes"] * (world if (wl["scaling"] == "weak" and not wl["fixed_bands"]) else 1)
    sid, vlp = sched.next(per_step * (args.warmup + args.steps))
    # samples per step over the whole job: every owned pixel of every rank, once per pass
    job_pixels = sum(shd.owned_pixels(W, H, q, nshards, band) for q in range(world))
    own_pixels = shd.owned_pixels(W, H, rank, nshards, band)

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
    samples = job_pixels * per_step * args.steps
    value = samples / dt / 1e6

    if rank == 0:
        if dist is not None:
            r.update_pixels()
            cnt = t_cnt.cpu().numpy().reshape(H, W)
            owned = (torch.arange(H).numpy() // band) % nshards < world
            assert (cnt[owned] == per_step * (args.warmup + args.steps)).all(), "reduced counters wrong"
        w = WORK.get(wl["scene"])
        avg_launch_s = kern_ms / 1e3 / max(launches, 1)
        passes_per_launch = per_step * args.steps / max(launches, 1)
        roofline = None
        if w is not None:
            samples_per_launch = own_pixels * passes_per_launch
            if r.last_streams > 1:
                # pass streams: the path kernel reads the counter once and writes 12 B of radiance
                # per sample; the fold kernel (not this launch) does the colors/pixels RMW
                bytes_per_launch = own_pixels * 4 + samples_per_launch * (4 * w["rng_reads"] + 12)
            else:
                bytes_per_launch = own_pixels * ACCUM_BYTES_PER_PIXEL + samples_per_launch * 4 * w["rng_reads"]
            gbs = bytes_per_launch / avg_launch_s / 1e9
            fl = flop_per_sample(w) * samples_per_launch / avg_launch_s / 1e12
            traffic = None
            pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
            if os.path.exists(pmc) and world == 1:
                rec = json.load(open(pmc))
                if rec.get("workload", "cornell1080") == args.workload and rec.get("scene") == wl["scene"] \
                        and rec.get("passes_per_launch") == passes_per_launch \
                        and rec.get("pass_streams") in (None, r.last_streams) \
                        and rec.get("specialized", False) == r.last_specialized \
                        and rec.get("width") == W and rec.get("height") == H:
                    traffic = rec.get("hbm_bytes_per_launch")
            roofline = {"bound": "valu", "achieved": round(fl, 3), "peak": FP32_NOFMA_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(fl / FP32_NOFMA_TFLOPS, 4), "traffic": traffic,
                        "peak_fma": FP32_PEAK_TFLOPS, "frac_fma": round(fl / FP32_PEAK_TFLOPS, 4),
                        "flop_per_sample": round(flop_per_sample(w), 1),
                        "samples_per_launch": int(samples_per_launch),
                        "avg_launch_ms": round(avg_launch_s * 1e3, 4), "launches": launches,
                        "hbm": {"achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": round(gbs / HBM_PEAK_GBS, 5), "bytes_per_launch": int(bytes_per_launch)},
                        "note": "fp32 VALU bound: -ffp-contract=off, so one add or mul per lane-cycle (78.6 T/s); "
                                "FLOP model and per-sample bytes in DESIGN.md; traffic = calibrated PMC "
                                "FETCH_SIZE+WRITE_SIZE per launch (profiles/pmc_traffic.json)"}
            pv = os.path.join(REPO, "profiles", "pmc_valu.json")
            if os.path.exists(pv) and world == 1:
                rec = json.load(open(pv))
                if rec.get("scene") == wl["scene"] and rec.get("passes_per_launch") == passes_per_launch \
                        and rec.get("pass_streams") == r.last_streams and rec.get("width") == W \
                        and rec.get("specialized", False) == r.last_specialized:
                    roofline["valu_busy_pmc"] = rec["valu_busy"]
                    roofline["lane_utilisation_pmc"] = rec["valu_lane_utilisation"]
            if r.last_traversal == "bvh":
                roofline["note"] = ("reference-equivalent FLOPs: the reference tests every sphere; the BVH "
                                    "skips most tests, so this is work avoided, not VALU throughput")
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            rows = shd.owned_row_ranges(H, rank, nshards, band)
            region = (rows[0][0], rows[0][1]) if wl["fixed_bands"] else (0, H)
            cpu = cpu_baseline(sp, cam, W, H, region, sid, vlp, args.cpu_seconds)
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": wl["scaling"], "vs_baseline": None, "dtype": "fp32",
            "data": f"synthetic: reference {wl['scene']}.scn + MT607 table (seed 0) + glibc-rand pass offsets",
            "config": {"workload": f"{args.workload}: {wl['scene']}.scn {W}x{H} internal "
                                   f"(CLI {wl['width']}x{wl['height']}), <=7-segment eye paths + NEE + 1 VLP "
                                   f"per diffuse vertex; {wl['config']}",
                       "scene": wl["scene"], "width": W, "height": H, "passes_per_step": per_step,
                       "samples_per_step": job_pixels * per_step,
                       "spp_total": per_step * (args.warmup + args.steps),
                       "parallelism": (f"{nshards} fixed {band}-row bands, rank r renders band r" if wl["fixed_bands"]
                                       else f"pixel bands x{world} ({band}-row, interleaved)"),
                       "pass_streams": r.last_streams, "traversal": r.last_traversal,
                       "specialized": r.last_specialized},
            "device_ms_per_step": round(dev_ms / args.steps, 3),
            "roofline": roofline, "cpu_baseline": cpu,
            "host": {"gpu": torch.cuda.get_device_name(local), "hostname": socket.gethostname()},
        }
        if cpu:
            line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
            line["speedup_vs_cpu_node_linear_estimate"] = round(value / cpu["node_linear_estimate"], 1)
        if args.rehearse:
            line["rehearsal"] = "ranks share GPUs over gloo: exercises the multi-rank flow, not a measurement"
        print(json.dumps(line), flush=True)
    r.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
