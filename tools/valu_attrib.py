"""VALU instructions per path by kernel section (DESIGN_LOG §12 "instruction attribution").

    python tools/valu_attrib.py [scene.scn] [--units] [--counts gpurun_out/x.txt] [--pmc-valu V]

Static side: builds the scene-specialised pass-stream kernel offline (tools/jit_codegen_check.py,
plus -gline-tables-only), disassembles it and maps every instruction to a section of
bdpt_path_kernel_t through its line-table entry: the innermost inlined frame that lies in the
kernel body names the section (anchored on the BDPT_TICK markers and a few comments, so line
shifts do not matter), the innermost frame overall says whether a sphere-test instruction belongs
to the discriminant (sphere_det) or the roots (roots_of / key_of / umin*).

Dynamic side: a `bdpt_counts ...` line from a run with -DBDPT_COUNTS=1 and BDPT_PROF=counts
(bdpt_kernels.hip BDPT_CNT sites: wave-level executions of each section).  Each section's static
VALU count times its executions gives an estimate of VALU instructions per path; branches inside a
section that a wave skips make it an upper bound, the sphere tests are split into their det and
roots parts so the wave-uniform skips (counters 10 and 12) are priced exactly.  --pmc-valu compares
the sum with the measured SQ_INSTS_VALU per path.
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import jit_codegen_check as jcc  # noqa: E402

SRC = os.path.join(REPO, "gpu_bidirectional_raytracer_amd", "csrc", "bdpt_kernels.hip")
LLVM = os.path.join(jcc.ROCM, "lib", "llvm", "bin")
# counter slots (bdpt_kernels.hip BDPT_CNT / BDPT_CNTN sites)
C_ITER, C_CAM, C_HIT, C_SHADE, C_BLOCK, C_REFR, C_LIGHT, C_FULL, C_SPLIT, C_STEP, C_CHSKIP, \
    C_END, C_SHSKIP, C_REGEN, C_WAVES, C_PATHS, C_SPLIT_IT, C_NONDIFF, C_DIFFDIR, C_LASTDIFF, \
    C_VLP = range(21)
NCOUNT = 24


def sections():
    """[(name, first line, last line)] of the kernel body, from anchors in the source."""
    lines = open(SRC).read().split("\n")

    def find(pat, start=0):
        for i in range(start, len(lines)):
            if re.search(pat, lines[i]):
                return i + 1
        raise SystemExit(f"anchor not found: {pat}")
    k0 = find(r"^bdpt_path_kernel_t\(|void bdpt_path_kernel_t\(", find(r"template <int N, bool STREAMS>"))
    loop = find(r"while \(__builtin_amdgcn_ballot_w64\(alive \|\| \(kPool", k0)
    cam = find(r"if \(fresh\) \{", loop)
    ch = find(r"// closest hit, scanning", cam)
    t0 = find(r"BDPT_TICK\(0\)", ch)
    blk = find(r"const bool isdiff =", t0)
    last = find(r"if \(depth >= 6u\) \{", blk)
    nxt = find(r"f3 refl = rd;", last)
    sr = find(r"if \(!isdiff\) \{", nxt)
    dirb = find(r"if \(isdiff \|\| refr\) \{", sr)
    fres = find(r"const float aa = nt - nc", dirb)
    fres_end = find(r"rd = reflect \? refl : U;", fres)
    blk_end = find(r"ro = hit;", fres_end)
    t1 = find(r"BDPT_TICK\(1\)", blk_end)
    vlp = find(r"if \(diff && li == 0\) \{", t1)
    vlp_in = find(r"BDPT_CNT\(20,", vlp)
    vlp_end = find(r"// compact this step's shadow rays", vlp_in)
    t2 = find(r"BDPT_TICK\(2\)", vlp_end)
    split = find(r"if \(lg > 0\) \{", t2)
    split_end = find(r"continue;", split)
    t3 = find(r"BDPT_TICK\(3\)", split_end)
    t4 = find(r"BDPT_TICK\(4\)", t3)
    pool = find(r"// lanes whose path ended take the next pixels", t4) - 1      # its `if constexpr (kPool)`
    regen = find(r"// release the parked lanes together", pool) - 1
    t5 = find(r"BDPT_TICK\(5\)", regen)
    end = find(r"^}", t5)
    return [("prologue", k0, loop - 1), ("loop_control", loop, cam - 1), ("camera", cam, ch - 1),
            ("closest_hit", ch, t0), ("shading", t0 + 1, blk - 1), ("block_head", blk, last - 1),
            ("last_segment", last, nxt - 1), ("block_head", nxt, sr - 1), ("spec_refr_head", sr, dirb - 1),
            ("fresnel", fres, fres_end), ("next_direction", dirb, blk_end),
            ("shading", blk_end + 1, t1), ("nee_setup", t1 + 1, vlp_in), ("vlp_setup", vlp_in + 1, vlp_end - 1),
            ("queue_push", vlp_end, t2), ("shadow_split", split, split_end),
            ("shadow_full", t2 + 1, t3), ("shadow_results", t3 + 1, t4), ("path_end", t4 + 1, pool - 1), ("pool_claim", pool, regen - 1),
            ("regen_release", regen, t5), ("epilogue", t5 + 1, end)], (k0, end)


def static_counts(scene, units, keep=None, pool=False):
    secs, (k0, kend) = sections()
    extra = ["-gline-tables-only"] + (["-DBDPT_UNITS=1"] if units else []) + (["-DBDPT_POOL=1"] if pool else [])
    with tempfile.TemporaryDirectory() as tmp:
        wd = keep or tmp
        os.makedirs(wd, exist_ok=True)
        jcc.build(scene, 6, wd, extra)
        dev = os.path.join(wd, "jit_dev.o")
        dis = subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", dev],
                                      text=True)
        insts, infn = [], False
        for line in dis.splitlines():
            m = re.match(r"([0-9a-f]+) <(\S+)>:", line)
            if m:
                infn = "Lb1E" in m.group(2)                      # the pass-stream instance
                continue
            t = line.split()
            if not infn or not t or not re.match(r"[vs]_|global_|buffer_|ds_|flat_", t[0]):
                continue
            ma = re.search(r"//\s*([0-9A-Fa-f]+):", line)
            if ma:
                insts.append((int(ma.group(1), 16), t[0]))
        out = subprocess.run([os.path.join(LLVM, "llvm-symbolizer"), "--inlines", "--obj", dev],
                             input="\n".join(hex(a) for a, _ in insts) + "\n", capture_output=True,
                             text=True, check=True).stdout
    blocks = out.strip().split("\n\n")
    assert len(blocks) == len(insts), (len(blocks), len(insts))

    # the exec-masked fallbacks for out-of-range operands (library sqrt / division; the wave
    # branches over them when no lane needs them): priced apart, not in the estimate
    src = open(SRC).read().split("\n")
    cold = {i + 1 for i, l in enumerate(src)
            if re.search(r"return 1\.f / x;|\*root = sqrtf\(x\);|return 1\.f / \*root;|kq = na / nb;", l)}

    def section(ln):
        for name, a, b in secs:
            if a <= ln <= b:
                return name
        return "other"
    cnt = collections.Counter()
    for (_, op), blk in zip(insts, blocks):
        fr = blk.split("\n")
        frames = [(fr[i], fr[i + 1]) for i in range(0, len(fr) - 1, 2)]
        sec, part = "other", ""
        if any(int(m.group(1)) in cold for _, loc in frames
               for m in [re.search(r"bdpt_kernels\.hip:(\d+)", loc)] if m):
            cnt[("cold", "valu" if op.startswith("v_") else "other")] += 1
            continue
        for fn, loc in frames:
            m = re.search(r"bdpt_kernels\.hip:(\d+)", loc)
            if m and k0 <= int(m.group(1)) <= kend:
                sec = section(int(m.group(1)))
                break
        if sec in ("closest_hit", "shadow_full", "shadow_split"):
            # the helper frames between the instruction and the kernel body (vector helpers
            # such as dot() sit inside them)
            for fn, loc in frames:
                if fn.startswith("sphere_det"):
                    part = ":det"
                    break
                if fn.startswith(("roots_of", "key_of", "umin", "maxt_key", "sphere_roots")):
                    part = ":roots"
                    break
                if fn.startswith("bdpt_path_kernel_t"):
                    break
        cls = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") else
               "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "lds")
        cnt[(sec + part, cls)] += 1
    return cnt


def parse_counts(path):
    for line in open(path):
        m = re.search(r"bdpt_counts\s+(.*)", line)
        if m:
            c = [int(x) for x in re.findall(r"\d+", m.group(1))][:NCOUNT]
            return c + [0] * (NCOUNT - len(c))
    raise SystemExit(f"no bdpt_counts line in {path}")


def attribute(cnt, c, n_spheres, n_small):
    v = lambda k: cnt[(k, "valu")]                                # noqa: E731
    waves, paths = c[C_WAVES], c[C_PATHS]
    # per-sphere parts: the unrolled tests are n_spheres copies of one sequence
    ch_det, ch_roots = v("closest_hit:det") / n_spheres, v("closest_hit:roots") / n_spheres
    sh_det, sh_roots = v("shadow_full:det") / n_spheres, v("shadow_full:roots") / n_spheres
    rows = {
        "prologue + epilogue": (v("prologue") + v("epilogue") + v("other")) * waves,
        "loop control": v("loop_control") * c[C_ITER],
        "camera ray": v("camera") * c[C_CAM],
        "closest hit: det": ch_det * n_spheres * c[C_HIT],
        "closest hit: roots": ch_roots * (n_spheres * c[C_HIT] - c[C_CHSKIP]),
        "closest hit: rest": v("closest_hit") * c[C_HIT],
        "shading (hit point, normal, emitter)": v("shading") * c[C_SHADE],
        "material decode (non-emitter block)": v("block_head") * c[C_BLOCK],
        "last segment (depth 6)": v("last_segment") * c[C_LASTDIFF],
        "specular / refraction set-up": v("spec_refr_head") * c[C_NONDIFF],
        "next direction (cosine / transmitted)": v("next_direction") * c[C_DIFFDIR],
        "Fresnel weights": v("fresnel") * c[C_REFR],
        "NEE set-up (light sample, direction, weight)": v("nee_setup") * c[C_LIGHT],
        "VLP set-up": v("vlp_setup") * c[C_VLP],
        "shadow queue push": v("queue_push") * c[C_LIGHT],
        "shadow split rounds: sphere tests": (v("shadow_split:det") + v("shadow_split:roots")) * c[C_SPLIT_IT],
        "shadow split rounds: rest": v("shadow_split") * c[C_SPLIT],
        "shadow full rounds: det": sh_det * c[C_STEP],
        "shadow full rounds: roots": sh_roots * (c[C_STEP] - c[C_SHSKIP]),
        "shadow full rounds: rest": v("shadow_full") * c[C_FULL],
        "shadow results + contribution": v("shadow_results") * c[C_LIGHT],
        "path end / accumulation / RNG loads": v("path_end") * c[C_ITER],
        "regen release": v("regen_release") * c[C_REGEN],
        "pool claim + next pixel set-up (pools)": v("pool_claim") * c[C_ITER],
    }
    # per path in the PMC's sense: wave instructions per 64 paths (a wave instruction serves 64
    # lanes; scripts/pmc_summary.py valu_insts_per_wave = SQ_INSTS_VALU / SQ_WAVES, over the
    # paths per lane of the launch)
    return {k: x * 64 / paths for k, x in rows.items()}, {
        "waves": waves, "paths": paths, "iterations_per_wave": c[C_ITER] / waves,
        "segments_per_path": c[C_HIT] * 64 / paths if paths else None,
        "closest_hit_small_skips": c[C_CHSKIP] / max(1, n_small * c[C_HIT]),
        "shadow_small_skips_per_step": c[C_SHSKIP] / max(1, c[C_STEP]),
        "full_rounds_per_light_step": c[C_FULL] / max(1, c[C_LIGHT]),
        "split_rounds_per_light_step": c[C_SPLIT] / max(1, c[C_LIGHT]),
        "steps_per_full_round": c[C_STEP] / max(1, c[C_FULL]),
        "static_valu": {k[0]: n for k, n in sorted(cnt.items()) if k[1] == "valu"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scene", nargs="?", default=os.path.join(REPO, "assets", "scenes", "cornell.scn"))
    ap.add_argument("--units", action="store_true", help="the in-kernel fold build (-DBDPT_UNITS=1)")
    ap.add_argument("--pool", action="store_true", help="the pixel-pool build (-DBDPT_POOL=1)")
    ap.add_argument("--counts", help="file holding a bdpt_counts line")
    ap.add_argument("--pmc-valu", type=float, help="measured SQ_INSTS_VALU per wave and path per lane")
    ap.add_argument("--keep")
    args = ap.parse_args()
    cnt = static_counts(args.scene, args.units, args.keep, args.pool)
    if not args.counts:
        print(json.dumps({f"{s}/{c}": n for (s, c), n in sorted(cnt.items())}, indent=1))
        return 0
    sys.path.insert(0, REPO)
    import gpu_bidirectional_raytracer_amd as g
    _, sp = g.read_scene(args.scene)
    n_small = sum(1 for s in sp if float(s["rad"]) < 1e3)        # bdpt_kernels.hip small_sphere
    rows, info = attribute(cnt, parse_counts(args.counts), len(sp), n_small)
    total = sum(rows.values())
    width = max(len(k) for k in rows)
    for k, x in sorted(rows.items(), key=lambda kv: -kv[1]):
        print(f"{k:<{width}}  {x:8.1f}  {x / total:6.1%}")
    print(f"{'total (estimate)':<{width}}  {total:8.1f}")
    if args.pmc_valu:
        print(f"{'measured (PMC)':<{width}}  {args.pmc_valu:8.1f}  estimate / measured {total / args.pmc_valu:.3f}")
    print(json.dumps(info))
    return 0


if __name__ == "__main__":
    sys.exit(main())
