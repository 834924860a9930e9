"""Scene-specialised kernels (bdpt_host.cpp jit_path_kernel) on the CPU: the sources embedded in
libbdpt.so are the current csrc/ files, and an offline hipcc build of the specialised source
(tools/jit_codegen_check.py, same options as the run-time compile) succeeds for several scenes
without spills beyond a few VGPRs and without scalar-memory stores."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO, SCENES

HIPCC = "/opt/rocm/bin/hipcc"


def test_embedded_sources_are_current(tmp_path):
    out = tmp_path / "src.h"
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "embed_jit_sources.py"), str(out)])
    built = os.path.join(REPO, "gpu_bidirectional_raytracer_amd", "csrc", "bdpt_jit_src.h")
    assert os.path.exists(built), "run make"
    assert open(built).read() == out.read_text(), "bdpt_jit_src.h is stale: run make"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
@pytest.mark.parametrize("scene", ["cornell", "cornell_glass", "caustic", "cornell_multi"])
def test_specialised_build_offline(scene):
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "jit_codegen_check.py"),
                        os.path.join(SCENES, scene + ".scn")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    kernels = [k for k in recs if "name" in k]
    assert len(kernels) == 2 and recs[-1]["scalar_stores"] == 0
    for k in kernels:
        assert k["vgpr_count"] <= 80 and k["vgpr_spill_count"] <= 32, k
