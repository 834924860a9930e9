"""bench.py's `--gpus N` contract (the driver runs `python bench.py --gpus 1` and, for the scaling
curve, `torchrun --nproc-per-node N bench.py --gpus N`): the launch resolution on CPU, and a real
`--gpus 2` refusal when the GPUs are not there."""
import os
import subprocess
import sys

import pytest

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_single_process_one_gpu():
    assert bench.resolve_launch(1, {}, visible=1) == ("single", 1, 0, 0)


def test_torchrun_ranks_must_match_gpus():
    env = {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2"}
    assert bench.resolve_launch(4, env, visible=8) == ("ranks", 4, 2, 2)
    with pytest.raises(SystemExit, match="WORLD_SIZE=4"):
        bench.resolve_launch(8, env, visible=8)
    with pytest.raises(SystemExit, match="WORLD_SIZE=1"):
        bench.resolve_launch(2, {"WORLD_SIZE": "1"}, visible=8)


def test_in_process_multi_device():
    assert bench.resolve_launch(8, {}, visible=8) == ("inproc", 1, 0, 0)
    assert bench.resolve_launch(2, {}, visible=1, devices=[0, 0]) == ("inproc", 1, 0, 0)
    with pytest.raises(SystemExit, match="only 1 GPU"):
        bench.resolve_launch(2, {}, visible=1)
    with pytest.raises(SystemExit, match="divide"):
        bench.resolve_launch(3, {}, visible=8, fixed_bands=8)      # weak64's 8 fixed bands
    with pytest.raises(SystemExit, match="--devices"):
        bench.resolve_launch(2, {}, visible=1, devices=[0, 1])
    with pytest.raises(SystemExit):
        bench.resolve_launch(0, {}, visible=8)


def test_gpus_2_without_gpus_refuses_cleanly():
    """No GPU here (and one on the test box): `--gpus 2` must exit non-zero with a message,
    not silently time one GPU."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=600, env=env,
                       cwd=REPO)
    if r.returncode == 0:
        pytest.fail("bench.py --gpus 2 succeeded without 2 GPUs: " + r.stdout[-500:])
    assert "GPU" in r.stderr, r.stderr[-800:]


def test_smt_topology_helpers():
    topo = bench.cpu_topology()
    assert topo and all(isinstance(v, tuple) and len(v) == 2 for v in topo.values())


def test_pmc_records_cover_both_auto_outcomes_of_the_headline():
    """bench.py's roofline PMC fields come from profiles/pmc_{valu,traffic}.json for the exact
    configuration run; the auto mode keeps two or four passes per lane on cornell1080 (64 or 32
    streams at 128-pass launches), so both outcomes must have a record of each kind."""
    for streams in (64, 32):
        for name in ("pmc_valu.json", "pmc_traffic.json"):
            rec = bench._pmc_record(name, "cornell1080", "cornell", 1921, 1081, 128.0, streams, True)
            assert rec is not None, (name, streams)
            assert rec["pass_streams"] == streams
    assert bench._pmc_record("pmc_valu.json", "cornell1080", "cornell", 1921, 1081, 128.0, 16, True) is None
