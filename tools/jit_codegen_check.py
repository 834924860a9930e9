"""Offline build of a scene-specialised path kernel (the source hipRTC compiles at run time,
bdpt_host.cpp jit_path_kernel) with hipcc, for inspection: register counts, spills, and a check
that the code writes nothing through the scalar data cache.

    python tools/jit_codegen_check.py [scene.scn] [--waves 6] [--keep DIR]

Prints one JSON line per kernel instance and one summary line; exit status 1 if an instance
spills or a scalar-memory write is found.

The scalar-write check decodes the machine words, not the disassembler's text: every
instruction in the SMEM encoding (first dword bits [31:26] = 0b110000 on gfx9-family targets,
opcode in bits [25:18]) is classified by opcode number.  Loads (0-12), cache invalidates (32, 34)
and the time / probe reads (36-39) are allowed; every other SMEM opcode (stores 16-26,
write-backs 33 and 35, discards 40-41, scalar atomics >= 64) is reported.
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
SMEM_ALLOWED = set(range(0, 13)) | {32, 34, 36, 37, 38, 39}
ENC_WORD = re.compile(r"//\s*[0-9A-Fa-f]+:\s+([0-9A-Fa-f]{8})")


def hexf(v):
    import numpy as np
    return float(np.float32(v)).hex() + "f"


def jit_defines(spheres):
    """The -D options jit_path_kernel passes (same geometry literals: {p, rad*rad} in fp32)."""
    import numpy as np
    parts, emis = [], 0
    for i, s in enumerate(spheres):
        rr = np.float32(s["rad"]) * np.float32(s["rad"])
        parts.append("{" + ",".join(hexf(x) for x in (s["p"][0], s["p"][1], s["p"][2], rr)) + "}")
        if any(float(e) != 0.0 for e in s["e"]):
            emis |= 1 << i
    n = len(spheres)
    n_vac = n - bin(emis).count("1")
    # bdpt_host.cpp jit_path_kernel: the non-emitters' list only where it saves a lane-group iteration
    vac_list = any((1 << k) <= n_vac and -(-n_vac >> k) < -(-n >> k) for k in (1, 2, 3))
    return [f"-DBDPT_JIT_N={n}", f"-DBDPT_JIT_EMIS={emis}ull", "-DBDPT_JIT_GEOM={" + ",".join(parts) + "}",
            f"-DBDPT_JIT_ZERO_SAFE={int(zero_exit_safe(spheres))}"] + ([] if vac_list else ["-DBDPT_VAC_LIST=0"])


def zero_exit_safe(spheres):
    """Python restatement of bdpt_util.c bdpt_zero_exit_safe (the rule that decides
    -DBDPT_JIT_ZERO_SAFE in bdpt_host.cpp jit_path_kernel): some non-emitter is black; all scene
    values finite, every |c| <= 1e3 and every radius > 2^-16 * scene scale; every emitter keeps a
    gap >= max(1, 1e-4 * scale) from every other sphere's surface; and the largest sum a vertex can
    add after a black hit, n_lights * max(e * 4 pi r^2) * 1.1 + 0.5 * max|e| * max(1, max|c|) * g,
    stays below 1e38 (g = the escaped-VLP normal-length factor 1 + 8 * 2^-24 * (|p| + r) / r)."""
    import math
    n = len(spheres)
    if n == 0:
        return False
    scale = cmax = emax = nee = 0.0
    g = 1.0
    black = False
    for o in spheres:
        v = [float(x) for x in (o["rad"], *o["p"], *o["e"], *o["c"])]
        if not all(math.isfinite(x) for x in v):
            return False
        scale = max(scale, math.sqrt(v[1] * v[1] + v[2] * v[2] + v[3] * v[3]) + abs(v[0]))
        cmax = max(cmax, *(abs(x) for x in v[7:10]))
        emits = any(x != 0.0 for x in v[4:7])
        if not emits and all(x == 0.0 for x in v[7:10]):
            black = True
    if not black or not cmax <= 1e3:
        return False
    min_gap, min_rad = max(1.0, 1e-4 * scale), math.ldexp(scale, -16)
    for i, e in enumerate(spheres):
        re = abs(float(e["rad"]))
        if not re > min_rad:
            return False
        ev = [float(x) for x in e["e"]]
        if not any(x != 0.0 for x in ev):
            continue
        em = max(abs(x) for x in ev)
        emax = max(emax, em)
        nee += em * 4.0 * math.pi * re * re
        pn = math.sqrt(sum(float(x) * float(x) for x in e["p"]))
        g = max(g, 1.0 + 8.0 * math.ldexp(pn + re, -24) / re)
        for k, o in enumerate(spheres):
            if k == i:
                continue
            ro = abs(float(o["rad"]))
            d = math.sqrt(sum((float(a) - float(b)) ** 2 for a, b in zip(e["p"], o["p"])))
            if not max(d - re - ro, ro - d - re, re - d - ro) >= min_gap:
                return False
    return nee * 1.1 + 0.5 * emax * max(1.0, cmax) * g < 1e38


def scalar_writes(asm):
    """Instructions of the SMEM encoding whose opcode is not a read (see module docstring)."""
    bad = []
    for line in asm.splitlines():
        m = ENC_WORD.search(line)
        if not m:
            continue
        w = int(m.group(1), 16)
        if (w >> 26) == 0b110000 and ((w >> 18) & 0xFF) not in SMEM_ALLOWED:
            bad.append(line.strip())
    return bad


def build(scene, waves, workdir, extra=()):
    sys.path.insert(0, REPO)
    import gpu_bidirectional_raytracer_amd as g
    _, sp = g.read_scene(scene)
    n = len(sp)
    src = os.path.join(REPO, "gpu_bidirectional_raytracer_amd", "csrc", "bdpt_kernels.hip")
    inst = os.path.join(workdir, "jit_inst.hip")
    with open(inst, "w") as f:
        f.write(f'#include "{src}"\n')
        for st in ("true", "false"):
            f.write(f"template __global__ void bdpt_path_kernel_t<{n}, {st}>(bdpt_path_args);\n")
    co = os.path.join(workdir, "jit.o")
    cmd = [os.path.join(ROCM, "bin", "hipcc"), "--offload-arch=gfx950", "-O3", "-std=c++17",
           "-ffp-contract=off", "-fno-slp-vectorize", "-fno-gpu-flush-denormals-to-zero",
           "-DBDPT_JIT=1", f"-DBDPT_WAVES_PER_SIMD={waves}", *jit_defines(sp),
           *extra, "--cuda-device-only", "-c", "-o", co, inst]
    subprocess.check_call(cmd)
    dev = os.path.join(workdir, "jit_dev.o")
    llvm = os.path.join(ROCM, "lib", "llvm", "bin")
    with open(co, "rb") as f:
        bundled = f.read(24).startswith(b"__CLANG_OFFLOAD_BUNDLE__")
    if bundled:
        subprocess.check_call([os.path.join(llvm, "clang-offload-bundler"), "--unbundle", "--type=o",
                               f"--input={co}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"])
    else:
        dev = co
    asm = subprocess.check_output([os.path.join(llvm, "llvm-objdump"), "-d", dev], text=True)
    notes = subprocess.check_output([os.path.join(llvm, "llvm-readelf"), "--notes", dev], text=True)
    return asm, notes


def kernel_notes(notes):
    kernels, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"\s*\.(name|vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|"
                     r"private_segment_fixed_size):\s+(\S+)", line)
        if not m:
            continue
        if m.group(1) == "name":
            cur = {"name": m.group(2)}
            kernels.append(cur)
        elif cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return kernels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scene", nargs="?", default=os.path.join(REPO, "assets", "scenes", "cornell.scn"))
    ap.add_argument("--waves", type=int, default=6)
    ap.add_argument("--keep", default=None)
    ap.add_argument("--extra", action="append", default=[], help="extra compiler option (experiments)")
    args = ap.parse_args()
    # the host's policy (bdpt_host.cpp jit_path_kernel): a build that spills is rebuilt with one
    # wave per SIMD fewer, down to 5
    final, bad, smem = {}, [], 0
    for waves in range(args.waves, 4, -1):
        with tempfile.TemporaryDirectory() as tmp:
            wd = args.keep or tmp
            os.makedirs(wd, exist_ok=True)
            asm, notes = build(args.scene, waves, wd, args.extra)
        bad += scalar_writes(asm)
        smem += sum(1 for l in asm.splitlines()
                    if (m := ENC_WORD.search(l)) and int(m.group(1), 16) >> 26 == 0b110000)
        for k in kernel_notes(notes):
            if k["name"] not in final or final[k["name"]]["vgpr_spill_count"]:
                # launch bound of the instance: the fused S = 1 kernel is capped at 5
                # (bdpt_kernels.hip BDPT_FUSED_WAVES)
                final[k["name"]] = dict(k, waves=min(waves, 5) if "Lb0E" in k["name"] else waves)
        if not any(k["vgpr_spill_count"] for k in final.values()):
            break
    for k in final.values():
        print(json.dumps(k))
    print(json.dumps({"smem_instructions": smem, "scalar_writes": len(bad), "first": bad[:3]}))
    spills = any(k.get("vgpr_spill_count", 0) for k in final.values())
    return 1 if bad or spills else 0


if __name__ == "__main__":
    sys.exit(main())
