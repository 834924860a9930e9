"""Issue-weighted VALU occupancy of the path kernel from the instruction-mix PMC passes
(scripts/gpu_round.sh PMC_MIX=1, scripts/profile_workloads.sh) and the measured gfx950 issue
costs (profiles/r02_valu_rates.jsonl, 8 waves/SIMD):

    python scripts/valu_weighted.py gpurun_out/mix [kernel] [pattern]

The `valu_busy` figure of scripts/pmc_summary.py charges every VALU instruction 2 cycles, but only
full-rate fp32 / integer ops issue that fast: compares, selects, min/max, add3, mul_lo/hi, fp64,
conversions and any op reading an SGPR take ~3.8 cycles, sqrt/rcp ~7.5.  The counters split the
VALU instructions into classes; the classes that mix full- and half-rate instructions (INT32 and the
remainder: compares, selects, moves, bit ops) are priced at both ends, which bounds the occupancy.
"""
import collections
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def issue_rates(repo=REPO):
    """Measured issue cost (cycles per wave64 instruction per SIMD, 8 waves/SIMD) by class."""
    rates = {}
    for line in open(os.path.join(repo, "profiles", "r02_valu_rates.jsonl")):
        d = json.loads(line)
        if d["waves_per_simd"] == 8:
            rates[d["test"]] = d["cyc_per_wave_instr_per_simd"]
    return {"full": (rates["v_add_f32"] + rates["v_mul_f32"] + rates["v_fma_f32"]) / 3,
            "half": (rates["v_cmp_lt_f32 vcc"] + rates["v_cndmask e64 s[0:1]"] + rates["v_mul_lo_u32"]) / 3,
            "quarter": (rates["v_sqrt_f32"] + rates["v_rcp_f32"]) / 2,
            "f64": rates["v_fma_f64"]}


def weighted(m, r):
    """(classes, lower, upper) issue-weighted VALU occupancy from mean counters m, or None."""
    need = ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE")
    if any(k not in m for k in need):
        return None
    f32 = m["SQ_INSTS_VALU_ADD_F32"] + m["SQ_INSTS_VALU_MUL_F32"] + m["SQ_INSTS_VALU_FMA_F32"]
    trans = m["SQ_INSTS_VALU_TRANS_F32"]
    dp = m["SQ_INSTS_VALU_ADD_F64"] + m["SQ_INSTS_VALU_MUL_F64"] + m["SQ_INSTS_VALU_FMA_F64"]
    i32 = m["SQ_INSTS_VALU_INT32"]
    other_half = m["SQ_INSTS_VALU_INT64"] + m["SQ_INSTS_VALU_CVT"]
    rest = m["SQ_INSTS_VALU"] - (f32 + trans + dp + i32 + other_half)
    simd_cycles = 256 * 4 * m["GRBM_GUI_ACTIVE"] / 8      # 1024 SIMDs x kernel cycles (per XCD)
    fixed = f32 * r["full"] + trans * r["quarter"] + dp * r["f64"] + other_half * r["half"]
    # (both clamped at 1: the costs were measured at 8 waves/SIMD, where an issue slot is contended
    # a little more than at the kernels' 5-6, so a fully busy SIMD can price slightly above 1)
    lo = min(1.0, (fixed + (i32 + rest) * r["full"]) / simd_cycles)
    hi = min(1.0, (fixed + (i32 + rest) * r["half"]) / simd_cycles)
    classes = (("fp32 add/mul/fma (full rate)", f32), ("fp32 sqrt/rcp (quarter)", trans),
               ("fp64 add/mul/fma (half)", dp), ("int32 (full..half)", i32),
               ("int64 + cvt (half)", other_half), ("compares/selects/moves/bits (full..half)", rest))
    return classes, lo, hi


def mean_counters(root, kern="path_kernel", pat="pmc*"):
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, pat, "run_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            if kern in row["Kernel_Name"]:
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mix"
    m = mean_counters(root, *(sys.argv[2:4]))
    r = issue_rates()
    classes, lo, hi = weighted(m, r)
    simd_cycles = 256 * 4 * m["GRBM_GUI_ACTIVE"] / 8
    print(f"VALU instructions per dispatch     {m['SQ_INSTS_VALU']:.4g}")
    for name, v in classes:
        print(f"  {name:42s} {v:.4g}  ({v / m['SQ_INSTS_VALU']:.1%})")
    print(f"issue costs (cycles/wave instr, 8 waves/SIMD): full {r['full']:.2f}, half {r['half']:.2f}, "
          f"quarter {r['quarter']:.2f}, fp64 {r['f64']:.2f}")
    print(f"2-cycle VALU busy (pmc_summary.py)  {m['SQ_INSTS_VALU'] * 2 / simd_cycles:.3f}")
    print(f"issue-weighted VALU occupancy       {lo:.3f} .. {hi:.3f}")
