"""The kernel's sqrt core (bdpt_math.h bdpt_sqrt_rn_core) is correctly rounded on x = +0 and
x >= 2^-96, and its fast reciprocal (v_rcp_f32 + one Newton fma, csrc/bdpt_kernels.hip rcp_rn) is
exactly 1.f/x on |x| in [2^-125, 2^125): re-checked on the box that runs the GPU tests, over all
2^32 float inputs (tests/native/hw_exact_check.hip, ~1 s).  Outside that range the kernel takes
the library division, so the product is exact for every input."""
import json
import os
import subprocess

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def test_fast_reciprocal_is_correctly_rounded(gpu):
    exe = os.path.join(REPO, "tests", "native", "hw_exact_check")   # built in-tree by `make`
    assert os.path.exists(exe), "run `make` (or __graft_entry__.build()) first"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    rec = {d["check"]: d for d in (json.loads(l) for l in out.stdout.splitlines() if l.startswith("{"))}
    inrange = [v for k, v in rec.items() if k.startswith("rcp") and "[2^-125, 2^125)" in k]
    assert len(inrange) == 1 and inrange[0]["mismatches"] == 0, rec
    core = [v for k, v in rec.items() if k.startswith("sqrt core")]
    assert len(core) == 1 and core[0]["mismatches"] == 0, rec
