"""Write profiles/pmc_traffic.json from a `STEPS="calib pmc"` run (gpurun_out/): FETCH_SIZE and
WRITE_SIZE (KiB, separate --pmc passes) of the path kernel, averaged over its dispatches, and
corrected as MI355X_MICROARCH.md "HBM" prescribes: FETCH_SIZE under-reports wide reads on gfx950
(1/2 for 16-B/lane streams) and other access widths must be calibrated on a known byte count in
the kernel's own access pattern -- scripts/pmc_calib.hip measures the counters on 1 GiB of
16-B streams, 20-B-per-128-B-line gathers (the RNG prefetch), 12-B AoS reads (colors) and 4-B /
12-B stores.  The path kernel's reads are dominated by the gathers, so its FETCH_SIZE is scaled
by line_bytes / FETCH(gather20): HBM bytes at 128-B line granularity, an upper estimate (the
counters include Infinity-Cache hits; the 30.7 MB table lives there)."""
import csv, glob, json, os, sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (record keys: bench.kernel_kind / bench.pmc_key)

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json"
pat = sys.argv[3] if len(sys.argv) > 3 else "pmc*"          # the PMC runs of one workload


def counter(pattern, kernel, name):
    vals = []
    for f in glob.glob(os.path.join(root, pattern, "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]) * 1024)
    return sum(vals) / len(vals) if vals else None, len(vals)


fetch, nd = counter(pat, "path_kernel", "FETCH_SIZE")
write, _ = counter(pat, "path_kernel", "WRITE_SIZE")
known = {}
kb = os.path.join(root, "calib_bytes.jsonl")
if os.path.exists(kb):
    for line in open(kb):
        if line.startswith("{"):
            d = json.loads(line)
            known[d["kernel"]] = d
calib = {}
for k, d in known.items():
    if "read_bytes" in d:
        v, _ = counter("calib_FETCH_SIZE", k, "FETCH_SIZE")
        calib[k] = {"fetch_reported": v, **{x: d[x] for x in d if x != "kernel"}}
    if "write_bytes" in d:
        v, _ = counter("calib_WRITE_SIZE", k, "WRITE_SIZE")
        calib[k] = {"write_reported": v, **{x: d[x] for x in d if x != "kernel"}}
for k, c in calib.items():
    if c.get("fetch_reported"):
        c["read_bytes_per_reported"] = round(c["read_bytes"] / c["fetch_reported"], 4)
        if "line_bytes" in c:
            c["line_bytes_per_reported"] = round(c["line_bytes"] / c["fetch_reported"], 4)
    if c.get("write_reported"):
        c["write_bytes_per_reported"] = round(c["write_bytes"] / c["write_reported"], 4)
if not calib and os.path.exists(out):                      # no calibration run: reuse the recorded one
    prev = json.load(open(out))
    prev = [prev] if "scene" in prev else list(prev.values())
    calib = next((p_["calibration"] for p_ in prev if p_.get("calibration")), {})
fscale = calib.get("gather20", {}).get("line_bytes_per_reported")
wscale = calib.get("store12", {}).get("write_bytes_per_reported")
# the workload of the PMC runs: their own bench.py JSON line
cfg, roof, ppl = {}, {}, 16
for f in sorted(glob.glob(os.path.join(root, pat + ".log"))):
    lines = [l for l in open(f) if l.startswith("{")]
    if lines:
        d = json.loads(lines[-1])
        cfg, roof = d["config"], d.get("roofline") or {}
        nl = roof.get("launches")                         # passes per launch as bench.py measures it
        ppl = cfg.get("passes_per_step", 16) * d["steps"] / nl if nl else cfg.get("passes_per_step", 16)
        break
rec = {"workload": cfg.get("workload", "cornell1080").split(":")[0], "scene": cfg.get("scene", "cornell"), "width": cfg.get("width", 1921), "height": cfg.get("height", 1081),
       "passes_per_launch": float(ppl), "pass_streams": cfg.get("pass_streams"), "specialized": cfg.get("specialized", False),
       "kernel": bench.kernel_kind(roof.get("kernel_features") or [], cfg.get("pass_streams")),
       "fetch_reported_bytes_per_launch": int(fetch), "write_reported_bytes_per_launch": int(write),
       "fetch_scale": fscale, "write_scale": wscale,
       "hbm_bytes_per_launch": int(fetch * (fscale or 1.0) + write * (wscale or 1.0)),
       "dispatches": nd, "calibration": calib,
       "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), x1024, calibrated",
       "method": __doc__}
os.makedirs(os.path.dirname(out), exist_ok=True)
# one record per workload and kernel: {bench.pmc_key: record}
data = json.load(open(out)) if os.path.exists(out) else {}
if "scene" in data:                                       # an older single-record file
    data = {data.get("workload", "cornell1080"): data}
data[bench.pmc_key(rec["workload"], rec["kernel"], rec["pass_streams"])] = rec      # one record per workload and stream count
json.dump(data, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in rec.items() if k not in ("method", "calibration")}))
print(json.dumps(calib))
