"""The product's fp64 sincos (csrc/bdpt_math.h) agrees with the oracle's glibc-based sinf/cosf
semantics on every input the render path can produce (exhaustive, ~20 s per table on one core)."""
import os
import subprocess

import pytest

from conftest import REPO


@pytest.mark.parametrize("coarse", [0, 1])      # 512-entry table | its even entries (BDPT_SC_COARSE)
def test_sincos_matches_glibc_on_every_reachable_input(tmp_path, coarse):
    exe = tmp_path / "sincos_check"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", f"-DBDPT_SC_COARSE={coarse}", "-o", str(exe),
                           os.path.join(REPO, "tests", "native", "sincos_check.c"), "-lm"])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout
    assert "268435457 inputs, 0 mismatches" in out.stdout, out.stdout
