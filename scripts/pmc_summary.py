"""Summarise rocprofv3 --pmc CSVs for one kernel: python scripts/pmc_summary.py gpurun_out [kernel]."""
import collections, csv, glob, os, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
kern = sys.argv[2] if len(sys.argv) > 2 else "path_kernel"
vals = collections.defaultdict(list)
pat = sys.argv[3] if len(sys.argv) > 3 else "pmc*"
for f in sorted(glob.glob(os.path.join(root, pat, "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
for k in sorted(m):
    print(f"{k:28s} {m[k]:.4g}")
def g(k): return m.get(k, float("nan"))
print("--- derived (per dispatch)")
print(f"VALU lane utilisation      {g('SQ_THREAD_CYCLES_VALU') / (64 * g('SQ_ACTIVE_INST_VALU')):.3f}")
print(f"wait / issue-stall / active {g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.3f} / "
      f"{g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f} / {g('SQ_ACTIVE_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
cyc = g('GRBM_GUI_ACTIVE') / 8
print(f"kernel cycles (per XCD)     {cyc:.4g}")
print(f"VALU busy (instr*2/(4*256*cyc)) {g('SQ_INSTS_VALU') * 2 / (4 * 256 * cyc):.3f}")
print(f"SALU / VALU instr           {g('SQ_INSTS_SALU') / g('SQ_INSTS_VALU'):.3f}")
print(f"L2 hit rate                 {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.3f}")
print(f"FETCH (MB) / WRITE (MB)     {g('FETCH_SIZE') / 1024:.1f} / {g('WRITE_SIZE') / 1024:.1f}")
# optional: python scripts/pmc_summary.py <root> <kernel> <pattern> <out.json> -- the derived
# figures plus the bench configuration of the PMC runs, read by bench.py into its `valu` object
if len(sys.argv) > 4:
    import json
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench  # noqa: E402  (record keys)
    cfg, ppl, feats = {}, None, []
    for f in sorted(glob.glob(os.path.join(root, pat + ".log"))):
        lines = [l for l in open(f) if l.startswith("{")]
        if lines:
            d = json.loads(lines[-1])
            cfg = d["config"]
            feats = (d.get("roofline") or {}).get("kernel_features") or []
            # passes per launch as the bench measured it (the fused kernel splits a step into
            # launches of at most 64 passes), as bench.py matches it
            nl = (d.get("roofline") or {}).get("launches")
            ppl = cfg.get("passes_per_step") * d["steps"] / nl if nl else cfg.get("passes_per_step")
            break
    rec = {"workload": cfg.get("workload", "cornell1080").split(":")[0],
           "valu_busy": round(g('SQ_INSTS_VALU') * 2 / (4 * 256 * cyc), 4),
           "valu_lane_utilisation": round(g('SQ_THREAD_CYCLES_VALU') / (64 * g('SQ_ACTIVE_INST_VALU')), 4),
           "l2_hit_rate": round(g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')), 4),
           "wait_frac": round(g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'), 4),
           "issue_stall_frac": round(g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'), 4),
           "active_frac": round(g('SQ_ACTIVE_INST_ANY') / g('SQ_WAVE_CYCLES'), 4),
           "valu_insts_per_wave": round(g('SQ_INSTS_VALU') / g('SQ_WAVES'), 1),
           "fetch_reported_kib": g('FETCH_SIZE'), "write_reported_kib": g('WRITE_SIZE'),
           "scene": cfg.get("scene"), "width": cfg.get("width"), "height": cfg.get("height"),
           "passes_per_launch": ppl, "pass_streams": cfg.get("pass_streams"), "specialized": cfg.get("specialized", False),
           "kernel": bench.kernel_kind(feats, cfg.get("pass_streams")),
           "source": "rocprofv3 --pmc SQ_INSTS_VALU / SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU / "
                     "GRBM_GUI_ACTIVE / TCC_HIT_sum / TCC_MISS_sum (separate passes), scripts/pmc_summary.py"}
    # issue-weighted VALU occupancy when the instruction-mix passes ran (scripts/valu_weighted.py)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import valu_weighted
    wv = valu_weighted.weighted(m, valu_weighted.issue_rates())
    if wv:
        rec["valu_issue_occupancy"] = [round(wv[1], 4), round(wv[2], 4)]
    rec = {k: (None if isinstance(v, float) and v != v else v) for k, v in rec.items()}   # NaN -> null
    out = sys.argv[4]
    data = json.load(open(out)) if os.path.exists(out) else {}
    if "scene" in data:                                   # an older single-record file
        data = {data.get("workload", "cornell1080"): data}
    data[bench.pmc_key(rec["workload"], rec["kernel"], rec["pass_streams"])] = rec      # one record per workload and stream count
    json.dump(data, open(out, "w"), indent=1)
