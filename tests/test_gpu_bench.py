"""bench.py end to end on one GPU, on a small frame: the JSON line's contract fields, and the
30000-pass counter cap of the path kernel (device.cu:607) -- a run whose steps would cross it
resets the accumulation before the step that would (so every timed step renders all of its
passes) and the frame's counters hold exactly the passes since that reset."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args):
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO,
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])


def test_bench_crosses_counter_cap():
    # (tuning + 1 warm-up + 240 timed steps) x 128 passes > 30,000: one reset
    d = run_bench("--scene", "simple", "--width", "96", "--height", "64", "--passes", "128",
                  "--steps", "240", "--warmup", "1", "--no-cpu-baseline")
    cfg = d["config"]
    steps = d["tune_steps"] + 1 + 240
    assert 30000 < steps * 128 < 2 * 30000
    assert cfg["accum_resets"] == 1
    assert cfg["spp_total"] == steps * 128 - 30000 // 128 * 128
    assert d["n_gpus"] == 1 and d["steps"] == 240 and d["value"] > 0
    assert cfg["samples_per_step"] == 97 * 65 * 128
    for k in ("metric", "unit", "ms_per_step", "higher_is_better", "scaling", "dtype", "roofline", "cpu_baseline"):
        assert k in d
