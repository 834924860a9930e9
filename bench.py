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
COUNTER_CAP = 30000              # per-pixel pass cap of the path kernel (device.cu:607)

WORKLOADS = {
    "cornell1080": dict(scene="cornell", width=1920, height=1080, passes=128, band_rows=8, fixed_bands=0,
                        scaling="weak", config="configs[1] scene at 1080p (the metric's config)"),
    "caustic8": dict(scene="caustic", width=1920, height=1080, passes=128, band_rows=8, fixed_bands=0,
                     scaling="strong", config="configs[3]: caustic.scn 1920x1080, pixel bands over N GPUs"),
    "weak64": dict(scene="synthetic64", width=4096, height=4096, passes=128, band_rows=512, fixed_bands=8,
                   scaling="weak", config="configs[4]: 64-sphere synthetic 4096x4096, one 4097x512 band per GPU"),
}

# Per-sample work of each scene, measured once by the CPU restatement over the full 1921x1081
# frame (tests/test_work_model.py keeps these honest; DESIGN.md "Roofline").
WORK = {
    "cornell": {"sphere_tests": 129.4711, "segments": 6.8441, "diffuse": 6.1386, "refr": 0.4528, "rng_reads": 27.0071,
                "_nonzero": 0.9884},
    "cornell_glass": {"sphere_tests": 92.9047, "segments": 6.8374, "diffuse": 4.2323, "refr": 1.02, "rng_reads": 19.9494},
    "caustic": {"sphere_tests": 5.1332, "segments": 1.5151, "diffuse": 0.4516, "refr": 0.0638, "rng_reads": 3.8704,
                "_nonzero": 0.2160},
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


def resolve_launch(gpus, env, visible=None, fixed_bands=0, devices=None):
    """How `--gpus N` runs (the driver's contract): under torchrun (WORLD_SIZE set) one rank per
    GPU and WORLD_SIZE must equal N; without it, N = 1 is one context on device 0 and N > 1 one
    in-process multi-device context (bdpt_create_multi: pixel bands over devices 0..N-1, the frame
    assembled by an in-process RCCL reduce).  Returns (mode, world, rank, local); raises
    SystemExit (non-zero) on any mismatch."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    if env.get("WORLD_SIZE") is not None:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but torchrun started WORLD_SIZE={world} ranks; "
                             "launch one rank per GPU (--nproc-per-node N with --gpus N)")
        return "ranks", world, int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0"))
    if devices is not None:                                   # explicit device list (rehearsal)
        if len(devices) != gpus or min(devices) < 0 or (visible is not None and max(devices) >= visible):
            raise SystemExit(f"bench.py: --devices {devices} does not name {gpus} visible GPU(s)")
    elif gpus == 1:
        return "single", 1, 0, 0
    elif visible is not None and gpus > visible:
        raise SystemExit(f"bench.py: --gpus {gpus} but only {visible} GPU(s) are visible")
    if fixed_bands and fixed_bands % gpus:
        raise SystemExit(f"bench.py: this workload has {fixed_bands} fixed bands; --gpus must divide it")
    return "inproc", 1, 0, 0


def is_reduce_fallback(mode, devices, backend, rehearse):
    """True when a multi-GPU frame is assembled by anything but RCCL across distinct GPUs: an
    in-process group on distinct devices whose backend is not "rccl" (RCCL missing or
    ncclCommInitAll failed), or torchrun ranks rehearsing over gloo.  Repeated devices (--devices
    0,0, shards of one GPU) are a rehearsal whose peer copies are expected, not a fallback."""
    if mode == "inproc":
        return len(set(devices)) == len(devices) and len(devices) > 1 and backend != "rccl"
    return bool(mode == "ranks" and rehearse)


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def gpu_identity(device):
    """Which GPU this is: name / arch / CUs / memory from the runtime, and from sysfs (by PCI
    address) its unique id, serial, sclk / mclk levels (current marked), power cap -- so a
    measurement can be placed within the box-to-box spread."""
    import torch
    p = torch.cuda.get_device_properties(device)
    ident = {"name": p.name, "arch": getattr(p, "gcnArchName", None),
             "cus": p.multi_processor_count, "memory_gib": round(p.total_memory / 2 ** 30, 1)}
    dom, bus, dev = (getattr(p, "pci_domain_id", None), getattr(p, "pci_bus_id", None),
                     getattr(p, "pci_device_id", None))
    if bus is not None:
        addr = f"{dom or 0:04x}:{bus:02x}:{dev or 0:02x}.0"
        ident["pci"] = addr
        d = f"/sys/bus/pci/devices/{addr}"
        for key, fn in (("unique_id", "unique_id"), ("serial", "serial_number"), ("product", "product_name"),
                        ("vbios", "vbios_version")):
            v = _read(os.path.join(d, fn))
            if v:
                ident[key] = v
        for key, fn in (("sclk", "pp_dpm_sclk"), ("mclk", "pp_dpm_mclk")):
            v = _read(os.path.join(d, fn))
            if v:
                lines = [l.split(":", 1)[1].strip() for l in v.splitlines() if ":" in l]
                cur = [l.split(":", 1)[1].replace("*", "").strip() for l in v.splitlines() if "*" in l]
                ident[key] = {"levels": lines, "current": cur[0] if cur else None}
        try:
            for hw in sorted(os.listdir(os.path.join(d, "hwmon"))):
                cap = _read(os.path.join(d, "hwmon", hw, "power1_cap"))
                cmax = _read(os.path.join(d, "hwmon", hw, "power1_cap_max"))
                if cap:
                    ident["power_cap_w"] = round(int(cap) / 1e6, 1)
                if cmax:
                    ident["power_cap_max_w"] = round(int(cmax) / 1e6, 1)
        except OSError:
            pass
    return ident


def cpu_topology():
    """{cpu: (package, core)} for every online CPU, from sysfs."""
    topo = {}
    for c in range(os.cpu_count() or 1):
        base = f"/sys/devices/system/cpu/cpu{c}/topology"
        pk, co = _read(os.path.join(base, "physical_package_id")), _read(os.path.join(base, "core_id"))
        if pk is not None and co is not None:
            topo[c] = (int(pk), int(co))
    return topo


def cpu_probe(spec):
    """Child process of cpu_baseline: pin to spec['cpus'], run the oracle with spec['threads']
    threads over a bounded region for about spec['seconds'], print the rate (Msamples/s)."""
    os.sched_setaffinity(0, spec["cpus"])
    import numpy as np
    import oracle
    import gpu_bidirectional_raytracer_amd as g
    W, H = spec["W"], spec["H"]
    cam, sp = g.read_scene(os.path.join(REPO, "assets", "scenes", spec["scene"] + ".scn"))
    g.update_camera(cam, W, H)
    rnd = oracle.mt607(0)
    lp = oracle.light_pass(sp, rnd, 0)
    sid, vlp = np.array(spec["sid"], np.uint32), np.array(spec["vlp"], np.int32)
    y0, th = spec["y0"], spec["threads"]
    oracle.path_passes(sp, rnd, cam, W, H, lp, sid[:1], vlp[:1], rows=(y0, y0 + 2), nthreads=th)   # warm
    rows = spec.get("rows")
    if not rows:                                              # calibrate: rows for ~`seconds`
        t = time.perf_counter()
        oracle.path_passes(sp, rnd, cam, W, H, lp, sid[:1], vlp[:1], rows=(y0, y0 + 8), nthreads=th)
        rate = 8 * W / max(time.perf_counter() - t, 1e-4)
        rows = max(8, min(H - y0, int(rate * spec["seconds"] / W)))
    t = time.perf_counter()
    oracle.path_passes(sp, rnd, cam, W, H, lp, sid[:1], vlp[:1], rows=(y0, y0 + rows), nthreads=th)
    dt = time.perf_counter() - t
    print(json.dumps({"value": rows * W / dt / 1e6, "rows": rows, "seconds": dt}), flush=True)


def smt_yield(scene, W, H, y0, sid, vlp, seconds, usable):
    """Within this job's CPUs: k physical cores with one oracle thread each vs the same k cores
    with both SMT siblings busy (2k threads).  Returns None when the affinity mask holds no core
    with two siblings.  Runs in child processes pinned with sched_setaffinity (OpenMP threads
    inherit the mask)."""
    import subprocess
    topo = cpu_topology()
    try:
        aff = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None
    cores = {}
    for c in aff:
        if c in topo:
            cores.setdefault(topo[c], []).append(c)
    pairs = [sorted(v)[:2] for v in cores.values() if len(v) >= 2]
    k = min(len(pairs), max(1, usable // 2))
    if k < 1:
        return None
    pairs = pairs[:k]
    res, rows = {}, None
    for label, cpus in (("one_thread_per_core", [p[0] for p in pairs]), ("two_threads_per_core", [c for p in pairs for c in p])):
        spec = {"cpus": cpus, "threads": len(cpus), "scene": scene, "W": W, "H": H, "y0": y0, "rows": rows,
                "sid": [int(x) for x in sid[:1]], "vlp": [int(x) for x in vlp[:1]], "seconds": seconds}
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-probe", json.dumps(spec)],
                             capture_output=True, text=True, timeout=600, env=dict(os.environ, OMP_NUM_THREADS=str(len(cpus))))
        lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if out.returncode != 0 or not lines:
            return {"error": (out.stderr or "")[-300:]}
        d = json.loads(lines[-1])
        res[label] = round(d["value"], 4)
        rows = d["rows"]                                      # the same region for both runs
    y = res["two_threads_per_core"] / res["one_thread_per_core"]
    return {"cores_probed": k, "rows": [y0, y0 + rows], "rate_one_thread_per_core": res["one_thread_per_core"],
            "rate_two_threads_per_core": res["two_threads_per_core"], "smt_yield": round(y, 3),
            "node_physical_cores": len(set(topo.values())) or None}


def kernel_kind(features, streams):
    """Which path kernel a run used: "units" (ordered in-kernel fold), "pools" (pass streams with
    pixel pools), "fused" (S = 1) or "streams" (pass streams; then S matters too)."""
    if "unit_fold" in features:
        return "units"
    if "pixel_pools" in features:
        return "pools"
    return "fused" if streams == 1 else "streams"


def pmc_key(workload, kind, streams):
    """Record key of profiles/pmc_*.json: workload@<kind>, plus S<streams> for plain pass streams."""
    return f"{workload}@{kind}" + (f"S{streams}" if kind == "streams" else "")


def _pmc_record(name, workload, scene, W, H, passes_per_launch, streams, specialized, kind=None):
    """The PMC record of profiles/<name> for this exact configuration (one record per workload
    and kernel, keyed pmc_key), or None.  Records without a "kernel" field (round 4 and before)
    are plain pass streams, or the fused kernel at S = 1."""
    path = os.path.join(REPO, "profiles", name)
    if not os.path.exists(path):
        return None
    data = json.load(open(path))
    recs = data.values() if isinstance(data, dict) and "scene" not in data else [data]
    kind = kind or ("fused" if streams == 1 else "streams")
    for rec in recs:
        rkind = rec.get("kernel") or ("fused" if rec.get("pass_streams") == 1 else "streams")
        if rec.get("workload", "cornell1080") == workload and rec.get("scene") == scene \
                and rec.get("width") == W and rec.get("height") == H \
                and float(rec.get("passes_per_launch", -1)) == float(passes_per_launch) \
                and rkind == kind and (kind != "streams" or rec.get("pass_streams") == streams) \
                and bool(rec.get("specialized", False)) == bool(specialized):
            return rec
    return None


def scaling_breakdown(per_dev, steps, dt, render_s, reduce_s, scaling, passes_per_step):
    """Where a multi-GPU step's time goes, from per-device accumulators.

    per_dev: one dict per GPU {kernel_ms, path_ms, launches, owned_pixels, ...} over the `steps`
    timed steps (kernel_ms = the path kernels alone; path_ms = each call's span, which overlaps
    the next call's through the pass-stream fold, so its sum can exceed the wall time).  dt = the
    max-over-ranks wall time of the timed region, render_s = its part before the frame reduce
    (max over ranks), reduce_s = the reduce (max over ranks).  For weak scaling every GPU holds
    the per-GPU work of the one-GPU run, so the mean device's path-kernel time is the estimate of
    what one GPU alone would take: weak_efficiency_vs_1gpu_estimate = that / dt.  Load imbalance
    is the slowest device's path-kernel time over the mean."""
    ps = [max(float(d["kernel_ms"]), 0.0) for d in per_dev]
    mean_p = sum(ps) / max(len(ps), 1)
    max_p = max(ps) if ps else 0.0
    out = {"per_device": [dict(d, kernel_ms_per_step=round(d["kernel_ms"] / steps, 4),
                               path_ms_per_step=round(d["path_ms"] / steps, 4),
                               samples_per_step=int(d["owned_pixels"]) * passes_per_step) for d in per_dev],
           "render_s": round(render_s, 6), "reduce_s": round(reduce_s, 6),
           "reduce_frac": round(reduce_s / dt, 5) if dt > 0 else None,
           "imbalance_max_over_mean": round(max_p / mean_p, 5) if mean_p > 0 else None,
           "host_gap_frac": round(max(render_s - max_p / 1e3, 0.0) / dt, 5) if dt > 0 else None}
    if scaling == "weak" and dt > 0:
        out["weak_efficiency_vs_1gpu_estimate"] = round(mean_p / 1e3 / dt, 4)
        out["weak_efficiency_note"] = ("mean device path-kernel time (one GPU's share = the one-GPU run's "
                                       "work) / the job's wall time; 1 - it = imbalance + reduce + fold and "
                                       "host gaps")
    return out


def rccl_versions(group=None):
    """The RCCL libbdpt binds to (bdpt_rccl_version), torch's (torchrun ranks gather over it) and,
    for an in-process group, bdpt_reduce_info (version, ncclCommCount, devices)."""
    from gpu_bidirectional_raytracer_amd import _lib

    def fmt(v):
        return f"{v // 10000}.{v // 100 % 100}.{v % 100}" if isinstance(v, int) and v > 0 else None
    out = {"libbdpt": fmt(int(_lib.lib.bdpt_rccl_version()))}
    try:
        import torch
        tv = torch.cuda.nccl.version()
        out["torch"] = ".".join(str(x) for x in tv) if isinstance(tv, tuple) else fmt(tv)
    except Exception:                                          # noqa: BLE001 (reporting only)
        out["torch"] = None
    if group is not None:
        out["group"] = group.reduce_info
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this job: under torchrun = WORLD_SIZE (one rank per GPU); without it, "
                         "N > 1 renders on devices 0..N-1 through one in-process multi-device context")
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
    ap.add_argument("--no-smt-probe", action="store_true", help="skip the SMT-yield probe of the CPU baseline")
    ap.add_argument("--rehearse", action="store_true",
                    help="multi-rank dry run on fewer GPUs: gloo, ranks share devices (not a measurement)")
    ap.add_argument("--devices", default=None,
                    help="in-process multi-device run on these devices, e.g. 0,0 (rehearsal of --gpus 2 on one GPU)")
    ap.add_argument("--allow-peer-reduce", action="store_true",
                    help="in-process run on distinct GPUs: time the peer-copy frame reduce if RCCL is unavailable")
    ap.add_argument("--cpu-probe", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.cpu_probe:                                        # child of cpu_baseline: no GPU
        return cpu_probe(json.loads(args.cpu_probe))
    wl = dict(WORKLOADS[args.workload])
    for k in ("scene", "width", "height", "passes", "band_rows"):
        if getattr(args, k) is not None:
            wl[k] = getattr(args, k)

    import torch                                              # device_count() does not initialise HIP
    visible = torch.cuda.device_count()
    dev_list = [int(x) for x in args.devices.split(",")] if args.devices else None
    mode, world, rank, local = resolve_launch(args.gpus, os.environ, visible, wl["fixed_bands"], dev_list)
    if mode == "single" and visible < 1:
        raise SystemExit("bench.py: no GPU visible")
    ndev = args.gpus if mode == "inproc" else 1               # devices of this process

    import gpu_bidirectional_raytracer_amd as g
    from gpu_bidirectional_raytracer_amd import sharding as shd

    if args.rehearse:
        local = local % max(visible, 1)
    if mode == "inproc":
        local = (dev_list or [0])[0]
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
    units = world * ndev                                      # GPUs rendering the job
    nshards = wl["fixed_bands"] or units                      # weak64: 8 fixed bands, GPU r renders band r
    if units > nshards:
        raise SystemExit(f"workload {args.workload} has {nshards} bands: at most {nshards} GPUs")
    cam, sp = g.read_scene(os.path.join(REPO, "assets", "scenes", wl["scene"] + ".scn"))
    g.update_camera(cam, W, H)
    sched = g.PassScheduler()
    sched.light()
    per_step = wl["passes"] * (units if (wl["scaling"] == "weak" and not wl["fixed_bands"]) else 1)
    # the auto stream mode measures its candidates on the first ten calls (bdpt.h
    # bdpt_set_streams): untimed extra steps when --warmup is shorter, so the timed steps run the
    # kernel it settled on
    tune = max(0, 11 - args.warmup) if args.streams == 0 else 0
    # torchrun ranks: one more untimed step after every rank has taken rank 0's choice
    follow = 1 if (args.streams == 0 and world > 1) else 0
    untimed = tune + args.warmup + follow
    sid, vlp = sched.next(per_step * (untimed + args.steps))

    # The CPU baseline (rank 0 at N = 1) runs first, before the GPU is touched: the GPU phase
    # (tuning, warm-up, timed steps) then runs as one block.
    cpu = None
    if world == 1 and ndev == 1 and not args.no_cpu_baseline:
        rows = shd.owned_row_ranges(H, rank, nshards, band)
        region = (rows[0][0], rows[0][1]) if wl["fixed_bands"] else (0, H)
        cpu = cpu_baseline(sp, cam, W, H, region, sid, vlp, args.cpu_seconds)
        if not args.no_smt_probe:
            mid = region[0] + (region[1] - region[0]) // 3
            smt = smt_yield(wl["scene"], W, H, mid, sid, vlp, max(2.0, args.cpu_seconds / 4), cpu["cores"])
            cpu["smt"] = smt
            if smt and smt.get("smt_yield") and smt.get("node_physical_cores"):
                # the verdict's node model: physical cores x 1-core rate x SMT yield
                cpu["node_estimate"] = round(smt["node_physical_cores"] * cpu["value_1core"] * smt["smt_yield"], 2)
                cpu["node_estimate_note"] = ("physical cores of the node x the 1-core rate (value_1core, same "
                                             "frame) x the SMT yield (k cores with both siblings busy / the "
                                             "same k cores with one thread each, same rows); assumes every "
                                             "core keeps the 1-core rate (no memory-bandwidth limit), so it "
                                             "is still an upper estimate of the whole host")
        cpu["order"] = "run before the GPU phase (no GPU work in flight)"

    if mode == "inproc":
        devices = dev_list or list(range(ndev))
        r = g.Renderer(sp, W, H, cam, devices=devices)
        # device k of the group renders shard k of nshards (bdpt_set_shard on a group of ndev
        # devices as shard 0 of nshards / ndev groups)
        r.set_shard(0, nshards // ndev, band)
        # distinct GPUs must assemble the frame over RCCL: a silent peer-copy fallback (e.g. a
        # failed ncclCommInitAll) would time another collective than the one the line names
        if is_reduce_fallback(mode, devices, r.reduce_backend, False) and not args.allow_peer_reduce:
            raise SystemExit(f"bench.py: the {ndev}-GPU frame reduce fell back to '{r.reduce_backend}' "
                             "(RCCL unavailable or ncclCommInitAll failed); --allow-peer-reduce to time it anyway")
    else:
        devices = [local]
        r = g.Renderer(sp, W, H, cam, device=local)
        r.set_shard(rank, nshards, band)
    r.set_traversal(args.traversal)
    r.set_streams(args.streams)
    r.set_specialize(bool(args.specialize))
    r.light_pass(0)                                           # UpdateRendering2
    # samples per step over the whole job: every owned pixel of every GPU, once per pass
    job_pixels = sum(shd.owned_pixels(W, H, q, nshards, band) for q in range(units))
    own_pixels = shd.owned_pixels(W, H, rank, nshards, band)  # this rank's (or device 0's) share

    # The reference renders pass p of a pixel only while its counter is below 30000
    # (device.cu:607): a step that crossed it would skip work.  So the accumulation is reset
    # (bdpt_reset_accum, the reference's ReInit) before a step that would cross it, and every
    # step, timed or not, renders all of its passes (an async counter memset, inside the clock).
    if per_step > COUNTER_CAP:
        raise SystemExit(f"bench.py: {per_step} passes per step exceed the {COUNTER_CAP}-pass counter cap")
    held = [0, 0]                                             # [passes since the last reset, resets]

    def step(k):
        if held[0] + per_step > COUNTER_CAP:
            r.reset_accum()
            held[0] = 0
            held[1] += 1
        a, b = k * per_step, (k + 1) * per_step
        r.path_passes(sid[a:b], vlp[a:b], sync=False)
        held[0] += per_step

    def barrier():
        if dist is not None:
            dist.barrier()

    for k in range(untimed - follow):
        step(k)
    r.synchronize()
    choice_src = None
    if follow:
        # every rank measured the stream-mode candidates on the same calls; rank 0's decision is
        # the job's (the ranks run the same kernels whatever their own timings said)
        ch = [r.stream_choice if rank == 0 else 0]
        dist.broadcast_object_list(ch, src=0)
        if not ch[0]:
            raise SystemExit("bench.py: rank 0's auto stream mode has not decided after the tuning steps")
        r.set_stream_choice(ch[0])
        choice_src = "rank 0 (torch.distributed broadcast, applied with bdpt_set_stream_choice)"
        for k in range(untimed - follow, untimed):
            step(k)
        r.synchronize()
    elif mode == "inproc" and args.streams == 0:
        choice_src = "devices[0] (the group's peers follow its measurement)"
    if mode == "inproc":                                      # RCCL's first-use set-up, untimed
        r.reduce_frame()
    r.path_timing(reset=True)
    r.kernel_timing(reset=True)

    # frame assembly: torch tensors over the library's own device buffers (no copy); rank 0
    # gathers every rank's own rows (sharding.gather_frame: RCCL point to point over xGMI)
    t_col = t_cnt = None
    if dist is not None:
        t_col, t_cnt = shd.device_tensors(r, f"cuda:{local}")
        # one gather of the same sizes on scratch buffers before the clock starts, so the timed
        # one does not pay RCCL's first-use set-up (channels, buffers) for these sizes
        shd.gather_frame(torch.zeros_like(t_col), torch.zeros_like(t_cnt), W, H, band, dst=0, nshards=nshards)
        torch.cuda.synchronize()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(untimed, untimed + args.steps):
        step(k)
    r.synchronize()
    t_render = time.perf_counter()                            # rendering done; the reduce is timed apart
    if dist is not None:                                      # assemble the frame on rank 0
        shd.gather_frame(t_col, t_cnt, W, H, band, dst=0, nshards=nshards)
    elif mode == "inproc":                                    # in-process RCCL reduce to device 0
        r.reduce_frame()
    torch.cuda.synchronize()
    t_reduce = time.perf_counter()
    barrier()
    dt = time.perf_counter() - t0
    render_s, reduce_s = t_render - t0, t_reduce - t_render
    if dist is not None:
        tt = torch.tensor([dt, render_s, reduce_s], device="cpu" if args.rehearse else f"cuda:{local}",
                          dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt, render_s, reduce_s = (float(x) for x in tt.tolist())

    kern_ms, launches = r.kernel_timing()                     # path kernels alone
    dev_ms, _ = r.path_timing()                               # + the pass-stream fold
    per_dev = r.device_timing()                               # each device's own share (no max)
    for k, d in enumerate(per_dev):                           # the kernel each device ran
        d["mode"] = r.device_mode(k)
    samples = job_pixels * per_step * args.steps
    value = samples / dt / 1e6
    ident = gpu_identity(local)
    idents = [ident]
    if dist is not None:
        gathered = [None] * world
        dist.all_gather_object(gathered, ident)
        idents = gathered
        mine = dict(per_dev[0], rank=rank)
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        per_dev = gathered
    elif mode == "inproc":
        idents = [gpu_identity(d) for d in devices]
    scaling = scaling_breakdown(per_dev, args.steps, dt, render_s, reduce_s, wl["scaling"], per_step)
    # one kernel for the whole job: every GPU should have adopted the same choice (a share too small
    # for units runs pass streams; bdpt_host.cpp units_fit) -- say so when they did not
    kinds = {(tuple(d["mode"]["choice"]), "unit_fold" in d["mode"]["features"],
              "pixel_pools" in d["mode"]["features"]) for d in per_dev}
    modes_agree = len(kinds) == 1
    if not modes_agree and rank == 0:
        print(f"bench.py: warning: the GPUs ran different kernels: {sorted(kinds)}", file=sys.stderr)

    spp_total = held[0]                                       # passes since the last reset
    if rank == 0:
        # check the (assembled) frame's counters: every rendered pixel holds every pass since the
        # last reset, the rest none
        if dist is not None:
            r.update_pixels()
            cnt = t_cnt.cpu().numpy().reshape(H, W)
        else:
            cnt = r.read_radiance()[1]
        owned = (torch.arange(H).numpy() // band) % nshards < units
        assert (cnt[owned] == spp_total).all() and (cnt[~owned] == 0).all(), "frame counters wrong"
    if rank == 0:
        w = WORK.get(wl["scene"])
        avg_launch_s = kern_ms / 1e3 / max(launches, 1)
        # overlapped launches (pixel pools: a launch starts while the previous one drains) have
        # event intervals that overlap and add up to more than the wall time: their rate is the
        # timed region's wall time per launch (fold and gaps included, so a lower bound)
        launch_overlap = launches > 0 and kern_ms / 1e3 > 1.02 * dt
        if launch_overlap:
            avg_launch_s = dt / launches
        passes_per_launch = per_step * args.steps / max(launches, 1)
        features = r.last_features
        roofline = None
        if w is not None:
            samples_per_launch = own_pixels * passes_per_launch
            # random-table bytes per sample: 4 B per value the path uses (WORK rng_reads, the
            # oracle's count); kernels with the sin/cos planes load a segment's d_Rand[j..j+3] and
            # two 8-B {sin, cos} pairs instead of d_Rand[j..j+4]: 32 B where 20 were
            rng_bytes = 4 * w["rng_reads"] * (32 / 20 if "sincos_planes" in features else 1)
            if "unit_fold" in features:
                # ordered in-kernel fold: colors + counter read and written once per unit of
                # kUnitPasses (8) passes, pixels once per launch; no radiance buffer
                per_unit = max(1.0, passes_per_launch / 8)          # units of a tile per launch
                bytes_per_launch = own_pixels * (32 * per_unit + 4) + samples_per_launch * rng_bytes
            elif "pixel_pools" in features:
                # pixel pools: the counter and a 16-B pass mask once per pixel; per sample the 12 B
                # of radiance only when it is not +0 (WORK _nonzero: the oracle's fraction)
                nz = w.get("_nonzero", 1.0)
                bytes_per_launch = own_pixels * (4 + 16) + samples_per_launch * (rng_bytes + 12 * nz)
            elif r.last_streams > 1:
                # pass streams: the path kernel reads the counter once and writes 12 B of radiance
                # per sample; the fold kernel (not this launch) does the colors/pixels RMW
                bytes_per_launch = own_pixels * 4 + samples_per_launch * (rng_bytes + 12)
            else:
                bytes_per_launch = own_pixels * ACCUM_BYTES_PER_PIXEL + samples_per_launch * rng_bytes
            gbs = bytes_per_launch / avg_launch_s / 1e9
            fl = flop_per_sample(w) * samples_per_launch / avg_launch_s / 1e12
            single = world == 1 and ndev == 1
            kind = kernel_kind(features, r.last_streams)
            trec = _pmc_record("pmc_traffic.json", args.workload, wl["scene"], W, H, passes_per_launch,
                               r.last_streams, r.last_specialized, kind) if single else None
            skips = [f for f in features if f in ("det_skip", "zero_exit", "last_skip", "bvh")]
            traffic = trec.get("hbm_bytes_per_launch") if trec else None
            roofline = {"bound": "valu", "achieved": round(fl, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(fl / FP32_PEAK_TFLOPS, 4),
                        "frac_spec": round(fl / FP32_PEAK_TFLOPS, 4),
                        "frac_issue_ceiling": round(fl / FP32_NOFMA_TFLOPS, 4),
                        "frac_note": "frac (= frac_spec) is against the 157.3 TFLOP/s fp32 spec (FMA = 2 FLOP); "
                                     "frac_issue_ceiling against the 78.6 T one-op-per-lane-cycle ceiling that "
                                     "applies without FMA contraction",
                        "traffic": traffic,
                        # calibrated counter bytes per launch / the algorithmic bytes of the same launch:
                        # > 1 is re-read / partial-line traffic
                        "traffic_over_model": round(traffic / bytes_per_launch, 3) if traffic else None,
                        "flop_per_sample": round(flop_per_sample(w), 1),
                        "flop_model": "reference-equivalent" if skips else "reference",
                        "kernel_features": features,
                        "samples_per_launch": int(samples_per_launch),
                        "avg_launch_ms": round(avg_launch_s * 1e3, 4), "launches": launches,
                        "launch_overlap": launch_overlap,
                        "hbm": {"achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": round(gbs / HBM_PEAK_GBS, 5), "bytes_per_launch": int(bytes_per_launch)},
                        "note": "fp32 VALU bound: -ffp-contract=off, so one add or mul per lane-cycle (78.6 T/s); "
                                "FLOP model and per-sample bytes in DESIGN.md; traffic = calibrated PMC "
                                "FETCH_SIZE+WRITE_SIZE per launch (profiles/pmc_traffic.json)"}
            if skips:
                roofline["note"] += ("; achieved counts REFERENCE-EQUIVALENT FLOPs: the model prices the "
                                     "reference's every-sphere, every-segment work, and this kernel provably skips "
                                     f"some of it ({', '.join(skips)}: results unchanged), so frac measures "
                                     "work delivered, not VALU efficiency -- see valu_busy_pmc (2 cycles per VALU instruction) and "
                                     "valu_issue_occupancy_pmc (the instruction mix priced at measured gfx950 issue costs, "
                                     "DESIGN.md section 4, Roofline)")
            vrec = _pmc_record("pmc_valu.json", args.workload, wl["scene"], W, H, passes_per_launch,
                               r.last_streams, r.last_specialized, kind) if single else None
            if vrec:
                for k in ("valu_busy", "valu_lane_utilisation", "wait_frac", "issue_stall_frac", "active_frac",
                          "valu_insts_per_wave", "l2_hit_rate", "valu_issue_occupancy"):
                    if k in vrec:
                        roofline[{"valu_busy": "valu_busy_pmc",
                                  "valu_lane_utilisation": "lane_utilisation_pmc"}.get(k, k + "_pmc")] = vrec[k]
        if mode == "ranks":
            reduce_backend = ("gloo gather (torch.distributed, host-staged)" if args.rehearse
                              else "rccl gather of owned rows (torch.distributed nccl)")
        elif mode == "inproc":
            reduce_backend = r.reduce_backend + " (in-process bdpt_create_multi)"
        else:
            reduce_backend = "none"
        reduce_fallback = is_reduce_fallback(mode, devices, r.reduce_backend, args.rehearse)
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "Msamples/s", "n_gpus": units,
            "steps": args.steps, "warmup": args.warmup, "tune_steps": tune, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": wl["scaling"], "vs_baseline": None, "dtype": "fp32",
            "data": f"synthetic: reference {wl['scene']}.scn + MT607 table (seed 0) + glibc-rand pass offsets",
            "config": {"workload": f"{args.workload}: {wl['scene']}.scn {W}x{H} internal "
                                   f"(CLI {wl['width']}x{wl['height']}), <=7-segment eye paths + NEE + 1 VLP "
                                   f"per diffuse vertex; {wl['config']}",
                       "scene": wl["scene"], "width": W, "height": H, "passes_per_step": per_step,
                       "samples_per_step": job_pixels * per_step,
                       "spp_total": spp_total, "accum_resets": held[1],
                       "parallelism": (f"{nshards} fixed {band}-row bands, GPU r renders band r" if wl["fixed_bands"]
                                       else f"pixel bands x{units} ({band}-row, interleaved)"),
                       "launch": {"single": "one process, one GPU", "ranks": f"torchrun: {world} ranks, one GPU each",
                                  "inproc": f"one process, multi-device context over {ndev} GPUs"}[mode],
                       "pass_streams": r.last_streams, "traversal": r.last_traversal,
                       "specialized": r.last_specialized},
            "rccl_ranks": world if mode == "ranks" else (ndev if r.reduce_backend == "rccl" else 0),
            "reduce_backend": reduce_backend,
            "reduce_fallback": reduce_fallback,
            "rccl_version": rccl_versions(r if mode == "inproc" else None),
            "modes_agree": modes_agree,
            "stream_choice_from": choice_src,
            "devices": [{"rank": q, **idents[q]} for q in range(len(idents))] if mode == "ranks"
            else [{"device": d, **idents[i]} for i, d in enumerate(devices)],
            "device_ms_per_step": round(dev_ms / args.steps, 3),
            "scaling_breakdown": scaling,
            "roofline": roofline, "cpu_baseline": cpu,
            "host": {"gpu": ident.get("name"), "hostname": socket.gethostname(), "gpu_pci": ident.get("pci"),
                     "gpu_unique_id": ident.get("unique_id")},
        }
        if cpu:
            line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
            line["speedup_vs_cpu_node_linear_estimate"] = round(value / cpu["node_linear_estimate"], 1)
            if cpu.get("node_estimate"):
                line["speedup_vs_cpu_node_estimate"] = round(value / cpu["node_estimate"], 1)
                line["north_star_100x_at_node_level"] = value / cpu["node_estimate"] >= 100.0
        if args.rehearse:
            line["rehearsal"] = "ranks share GPUs over gloo: exercises the multi-rank flow, not a measurement"
        print(json.dumps(line), flush=True)
    r.close()
    if dist is not None:
        dist.destroy_process_group()

if __name__ == "__main__":
    main()
