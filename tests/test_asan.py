"""Sanitizer build ("tests under ASan for the CPU path"): `make asan` builds the C host
(smallpt.c), the host utilities (bdpt_util.c), the CPU backend (bdpt_cpu.cpp) and the oracle with
AddressSanitizer + UBSan (GPU sanitizers are not available on the MI355X pool), and these runs
must finish without a report: a scripted session with every key kind, SavePPM, checkpoint and
resume, and the oracle against the CPU backend on three scenes."""
import os
import subprocess

import pytest

from conftest import REPO, SCENES

ASAN = os.path.join(REPO, "tests", "native", "_asan")
DAT = os.path.join(REPO, "assets", "data", "MersenneTwister.dat")


@pytest.fixture(scope="module")
def built():
    subprocess.check_call(["make", "-s", "-j4", "asan"], cwd=REPO, timeout=600)
    return ASAN


def run(args, cwd):
    env = dict(os.environ, BDPT_CPU_THREADS="4", ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run(args, cwd=cwd, env=env, capture_output=True, text=True, timeout=600)
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    assert "LeakSanitizer" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0, r.stderr[-3000:]
    return r


def test_smallpt_session_under_asan(built, tmp_path):
    exe = os.path.join(built, "smallpt_asan")
    scn = os.path.join(SCENES, "cornell.scn")
    base = [exe, "32", "24", scn, "--device", "-1", "--dat", DAT, "--batch", "2"]
    run(base + ["--spp", "3", "--keys", "wasdrfL+4U 68QP-92R3Dp", "--out", "a.ppm",
                "--checkpoint", "c.ckpt"], tmp_path)
    r = run(base + ["--spp", "2", "--resume", "c.ckpt", "--out", "b.ppm", "--p6"], tmp_path)
    assert "Resumed at pass" in r.stderr
    assert any(f.startswith("max1_secondi") for f in os.listdir(tmp_path))      # the 'p' key
    run([exe, "--device", "-1", "--dat", DAT, "--spp", "1"], tmp_path)            # built-in scene


def test_oracle_and_cpu_backend_under_asan(built):
    scenes = [os.path.join(SCENES, s + ".scn") for s in ("cornell", "caustic", "cornell_2luci")]
    r = run([os.path.join(built, "oracle_asan"), DAT, *scenes], REPO)
    assert r.stdout.count("equal") == 3 and "DIFFERENT" not in r.stdout
