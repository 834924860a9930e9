"""Scene-specialised kernels (bdpt_host.cpp jit_path_kernel) on the CPU: the sources embedded in
libbdpt.so are the current csrc/ files, and an offline hipcc build of the specialised source
(tools/jit_codegen_check.py, same options as the run-time compile) succeeds for several scenes
within the 80-VGPR / 6-wave bound, without spilling, and without any write through the scalar
data cache (checked by SMEM opcode on the machine words)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO, SCENES

HIPCC = "/opt/rocm/bin/hipcc"
sys.path.insert(0, os.path.join(REPO, "tools"))


def test_embedded_sources_are_current(tmp_path):
    out = tmp_path / "src.h"
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "embed_jit_sources.py"), str(out)])
    built = os.path.join(REPO, "gpu_bidirectional_raytracer_amd", "csrc", "bdpt_jit_src.h")
    assert os.path.exists(built), "run make"
    assert open(built).read() == out.read_text(), "bdpt_jit_src.h is stale: run make"


def test_scalar_write_decoder():
    """The SMEM opcode classifier on hand-made encodings: loads pass, stores/atomics do not."""
    import jit_codegen_check as jc

    def line(word):
        return f"\tinsn  // 000000001600: {word:08X} 00000000"

    smem = lambda op: (0b110000 << 26) | (op << 18)
    ok = [smem(0), smem(1), smem(8), smem(32), smem(36)]
    bad = [smem(16), smem(18), smem(21), smem(24), smem(33), smem(40), smem(64), smem(128)]
    assert jc.scalar_writes("\n".join(line(w) for w in ok)) == []
    assert len(jc.scalar_writes("\n".join(line(w) for w in bad))) == len(bad)
    assert jc.scalar_writes(line(0xBF800000)) == []          # SOPP, not SMEM


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
@pytest.mark.parametrize("scene", ["cornell", "cornell_glass", "caustic", "cornell_multi", "synthetic64"])
def test_specialised_build_offline(scene):
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "jit_codegen_check.py"),
                        os.path.join(SCENES, scene + ".scn")], capture_output=True, text=True, timeout=300)
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    kernels = [k for k in recs if "name" in k]
    assert len(kernels) == 2, r.stdout + r.stderr
    assert recs[-1]["smem_instructions"] > 0 and recs[-1]["scalar_writes"] == 0, recs[-1]
    for k in kernels:                    # the build the host keeps (6 waves/SIMD, else 5)
        assert k["vgpr_spill_count"] == 0, k
        assert k["vgpr_count"] <= 512 // 8 // k["waves"] * 8, k
    # the default (pass-stream) kernel of the benchmark scenes keeps 6 waves/SIMD
    streams = [k for k in kernels if "Lb1E" in k["name"]]
    if scene in ("cornell", "cornell_glass", "caustic", "synthetic64"):
        assert streams[0]["waves"] == 6, streams
    # no SGPR spills either (a per-lane `break` in the 64-sphere shadow loop once kept a nest of
    # saved exec masks and spilled 86 SGPRs into VGPR lanes; the lane-mask loop has none)
    assert streams[0]["sgpr_spill_count"] == 0, streams
    assert r.returncode == 0, r.stdout + r.stderr


def _c_rule(sp):
    import ctypes
    sys.path.insert(0, REPO)
    import gpu_bidirectional_raytracer_amd as g
    arr = g.spheres_to_array(sp)
    return bool(g._lib.lib.bdpt_zero_exit_safe(ctypes.cast(ctypes.c_void_p(arr.ctypes.data),
                                                           ctypes.POINTER(g.Sphere)), len(arr)))


def test_zero_exit_rule():
    """The black-surface path exit (bdpt_kernels.hip BDPT_ZERO_EXIT) is compiled in only for scenes
    with a black non-emitter whose emitters keep a gap >= 1 from every other surface and whose
    post-black terms are provably finite.  The decision the host makes (bdpt_util.c
    bdpt_zero_exit_safe, called by jit_path_kernel) and its Python restatement
    (tools/jit_codegen_check.py) must agree."""
    import jit_codegen_check as jc
    sys.path.insert(0, REPO)
    import gpu_bidirectional_raytracer_amd as g
    want = {"cornell": True, "cornell_glass": True, "mod_cornell": True,      # black front wall
            "caustic": False, "simple": False, "cornell_multi": False, "open": False}   # nothing black
    for scene, safe in want.items():
        _, sp = g.read_scene(os.path.join(SCENES, scene + ".scn"))
        assert jc.zero_exit_safe(sp) == safe, scene
        assert _c_rule(sp) == safe, scene
    _, base = g.read_scene(os.path.join(SCENES, "cornell.scn"))
    light = int(next(i for i, s in enumerate(base) if any(float(v) != 0 for v in s["e"])))

    def variant(edit):
        sp = base.copy()
        for (idx, field), val in edit.items():
            sp[idx][field] = val
        return sp

    cases = [
        # a light touching a black wall: no exit
        ({(light, "p"): [50.0, 81.6 - 7.5, 81.6]}, False),
        # a small, very hot emitter: e * 4 pi r^2 below 1e37, but its VLPs carry 0.25 e c -> inf
        ({(light, "rad"): 0.5, (light, "e"): [3e36, 3e36, 3e36], (0, "c"): [1e3, 1e3, 1e3]}, False),
        # the same emitter with unit colours: finite
        ({(light, "rad"): 0.5, (light, "e"): [3e36, 3e36, 3e36]}, True),
        # a negative colour beyond 1e3: the throughput before the black hit could overflow
        ({(0, "c"): [-1e30, 0.5, 0.5]}, False),
        ({(0, "c"): [-0.5, 0.5, 0.5]}, True),
        # non-finite values
        ({(0, "c"): [float("nan"), 0.5, 0.5]}, False),
        ({(light, "e"): [float("inf"), 1.0, 1.0]}, False),
        # a degenerate sphere (radius 0)
        ({(1, "rad"): 0.0}, False),
    ]
    for edit, safe in cases:
        sp = variant(edit)
        assert jc.zero_exit_safe(sp) == safe, edit
        assert _c_rule(sp) == safe, edit
    # many emitters whose NEE terms each stay below 1e37 but whose sum would overflow
    many = [base[i].copy() for i in range(len(base)) if i != light]
    hot = base[light].copy()
    for k in range(40):
        h = hot.copy()
        h["rad"] = 1.0
        h["p"] = [12.0 + 2.0 * k, 70.0, 60.0 + (k % 5) * 6.0]
        h["e"] = [7e35, 7e35, 7e35]
        many.append(h)
    many = np.array(many, dtype=base.dtype)
    assert not jc.zero_exit_safe(many) and not _c_rule(many)
    many["e"][len(base) - 1:] = 1.0
    assert jc.zero_exit_safe(many) == _c_rule(many)
    # random scenes around cornell: the two restatements agree on every one
    rng = np.random.default_rng(7)
    for t in range(300):
        sp = base.copy()
        k = rng.integers(0, len(sp))
        which = rng.integers(0, 4)
        if which == 0:
            sp[k]["c"] = rng.choice([0.0, 0.5, -2e3, 999.0, 1e3, 1001.0], size=3)
        elif which == 1:
            sp[k]["e"] = rng.choice([0.0, 1.0, 1e30, 1e36, 1e37], size=3)
        elif which == 2:
            sp[k]["rad"] = rng.choice([0.0, 1e-3, 0.5, 16.5, 1e5])
        else:
            sp[k]["p"] = sp[k]["p"] + rng.normal(0, 20, 3)
        assert jc.zero_exit_safe(sp) == _c_rule(sp), (t, sp[k])


def test_valu_attribution_anchors():
    """tools/valu_attrib.py finds its section anchors in the kernel source, in order, and every
    counter slot it reads has a BDPT_CNT / BDPT_CNTN site (the instrumentation is compiled only
    with -DBDPT_COUNTS, so the production build is untouched)."""
    import re
    import valu_attrib as va
    secs, (k0, kend) = va.sections()
    assert k0 < secs[1][1] and secs[-1][2] <= kend
    for (_, a, b), (_, c, _) in zip(secs, secs[1:]):
        assert a <= b and (c > b or c < a), secs         # ranges do not overlap
    src = open(va.SRC).read()
    sites = {int(m.group(1)) for m in re.finditer(r"BDPT_CNTN?\((\d+),", src)}
    assert sites >= set(range(16)) - {va.C_REFR}, sorted(sites)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
def test_unit_ranges_partition(tmp_path):
    """The units' pass ranges (bdpt_device.h, shared by kernel and launcher) partition every
    launch in order, with the halving tail (tests/native/unit_ranges_check.cpp)."""
    exe = tmp_path / "unit_ranges_check"
    subprocess.check_call([HIPCC, "-O1", "-std=c++17", "-o", str(exe),
                           os.path.join(REPO, "tests", "native", "unit_ranges_check.cpp")])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout
