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
    parts, lrec, emis = [], [], 0
    for i, s in enumerate(spheres):
        rr = np.float32(s["rad"]) * np.float32(s["rad"])
        parts.append("{" + ",".join(hexf(x) for x in (s["p"][0], s["p"][1], s["p"][2], rr)) + "}")
        if any(float(e) != 0.0 for e in s["e"]):
            emis |= 1 << i
            r = np.float32(s["rad"])
            area = np.float32(np.float32(np.float32(4.0) * np.float32(np.pi)) * r) * r
            lrec.append("{" + ",".join(hexf(x) for x in (s["p"][0], s["p"][1], s["p"][2], r)) + "}")
            lrec.append("{" + ",".join(hexf(x) for x in (s["e"][0], s["e"][1], s["e"][2], area)) + "}")
    nl = len(lrec) // 2
    if not lrec:
        lrec = ["{0,0,0,0}", "{0,0,0,0}"]
    return [f"-DBDPT_JIT_N={len(spheres)}", f"-DBDPT_JIT_EMIS={emis}ull", "-DBDPT_JIT_GEOM={" + ",".join(parts) + "}",
            f"-DBDPT_JIT_NL={nl}", "-DBDPT_JIT_LREC={" + ",".join(lrec) + "}",
            f"-DBDPT_JIT_ZERO_SAFE={int(zero_exit_safe(spheres))}"]


def zero_exit_safe(spheres):
    """bdpt_host.cpp jit_path_kernel's rule: some non-emitter is black, all scene values are finite
    and colours <= 1e3, every emitter has e * 4 pi r^2 < 1e37 and keeps a gap >= max(1, 1e-4 *
    scene scale) from every other sphere's surface."""
    import math
    vals = [float(v) for o in spheres for v in (o["rad"], *o["p"], *o["e"], *o["c"])]
    if not all(math.isfinite(v) for v in vals) or any(float(v) > 1e3 for o in spheres for v in o["c"]):
        return False
    if not any(not any(float(v) != 0.0 for v in o["e"]) and all(float(v) == 0.0 for v in o["c"])
               for o in spheres):
        return False
    scale = max(math.hypot(*[float(v) for v in o["p"]]) + abs(float(o["rad"])) for o in spheres)
    min_gap = max(1.0, 1e-4 * scale)
    for i, e in enumerate(spheres):
        if not any(float(v) != 0.0 for v in e["e"]):
            continue
        re = float(e["rad"])
        if not max(abs(float(v)) for v in e["e"]) * 4.0 * math.pi * re * re < 1e37:
            return False
        for k, o in enumerate(spheres):
            if k == i:
                continue
            ro = float(o["rad"])
            d = math.dist([float(v) for v in e["p"]], [float(v) for v in o["p"]])
            if not max(d - re - ro, ro - d - re, re - d - ro) >= min_gap:
                return False
    return True


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
        m = re.match(r"\s*\.(name|vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count):\s+(\S+)", line)
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
