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


def test_scaling_breakdown_fields():
    """a multi-GPU line says where the time goes -- per-device kernel/path ms and
    owned samples, the reduce apart from the render, imbalance and the weak-efficiency estimate."""
    per_dev = [{"device": 0, "kernel_ms": 640.0, "path_ms": 660.0, "launches": 20, "owned_pixels": 1000},
               {"device": 1, "kernel_ms": 700.0, "path_ms": 720.0, "launches": 20, "owned_pixels": 1000}]
    s = bench.scaling_breakdown(per_dev, steps=20, dt=0.75, render_s=0.72, reduce_s=0.03, scaling="weak",
                                passes_per_step=256)
    assert [d["kernel_ms_per_step"] for d in s["per_device"]] == [32.0, 35.0]
    assert [d["path_ms_per_step"] for d in s["per_device"]] == [33.0, 36.0]
    assert s["per_device"][1]["samples_per_step"] == 256000
    assert s["reduce_s"] == 0.03 and s["reduce_frac"] == 0.04
    assert abs(s["imbalance_max_over_mean"] - 700 / 670) < 1e-4
    assert abs(s["weak_efficiency_vs_1gpu_estimate"] - 0.67 / 0.75) < 1e-4
    assert abs(s["host_gap_frac"] - 0.02 / 0.75) < 1e-4
    strong = bench.scaling_breakdown(per_dev, 20, 0.75, 0.72, 0.03, "strong", 128)
    assert "weak_efficiency_vs_1gpu_estimate" not in strong


def test_device_timing_through_the_abi():
    """bdpt_device_timing on a host-CPU context (the GPU contexts share the code): device id,
    the context's own accumulators and the pixels its shard owns."""
    import numpy as np
    import gpu_bidirectional_raytracer_amd as g
    from gpu_bidirectional_raytracer_amd import sharding as shd
    from conftest import SCENES
    W, H = 24, 40
    cam, sp = g.read_scene(os.path.join(SCENES, "simple.scn"))
    g.update_camera(cam, W, H)
    with g.Renderer(sp, W, H, cam, device=-1) as r:
        r.set_shard(1, 3, 8)
        r.light_pass(0)
        s = g.PassScheduler()
        s.light()
        sid, vlp = s.next(2)
        r.path_passes(sid, vlp)
        r.path_passes(sid, vlp)
        (d,) = r.device_timing()
        ms, n = r.kernel_timing()
        assert d["device"] == -1 and d["launches"] == n == 2 and abs(d["kernel_ms"] - ms) < 1e-9
        assert d["path_ms"] >= d["kernel_ms"] > 0
        assert d["owned_pixels"] == shd.owned_pixels(W, H, 1, 3, 8) == 16 * W    # bands 1 and 4
        assert g._lib.lib.bdpt_device_timing(r._h, 1, None, None, None, None, None) != 0   # one device only


def test_reduce_fallback_rule():
    """an in-process run on distinct GPUs whose frame reduce is not RCCL is a
    fallback (bench.py exits unless --allow-peer-reduce); repeated devices are a rehearsal."""
    assert bench.is_reduce_fallback("inproc", [0, 1], "peer", False)
    assert not bench.is_reduce_fallback("inproc", [0, 1], "rccl", False)
    assert not bench.is_reduce_fallback("inproc", [0, 0], "peer", False)
    assert not bench.is_reduce_fallback("single", [0], "none", False)
    assert bench.is_reduce_fallback("ranks", [0], "none", True)
    assert not bench.is_reduce_fallback("ranks", [0], "none", False)


def test_stream_choice_through_the_abi():
    """bdpt_stream_choice / bdpt_set_stream_choice / bdpt_device_mode on a host-CPU context: a
    choice applied without measuring reads back, a bad one or a non-auto stream mode is refused,
    and the per-device mode names S, the kernel features and the choice."""
    import gpu_bidirectional_raytracer_amd as g
    from gpu_bidirectional_raytracer_amd import _lib as L
    from conftest import SCENES
    cam, sp = g.read_scene(os.path.join(SCENES, "simple.scn"))
    g.update_camera(cam, 16, 8)
    with g.Renderer(sp, 16, 8, cam, device=-1) as r:
        assert r.stream_choice == 0                               # nothing measured yet
        ch = 1 | 16                                               # decided, pixel pools
        r.set_stream_choice(ch)
        assert r.stream_choice == ch
        assert r.device_mode(0)["choice"] == ["decided", "pools"]
        for bad in (0, 16, 64):                                   # not decided / unknown bits
            with pytest.raises(g.BdptError):
                r.set_stream_choice(bad)
        r.set_streams(1)                                          # fused fixed: no auto choice
        assert r.stream_choice == 0
        with pytest.raises(g.BdptError):
            r.set_stream_choice(ch)
        r.light_pass(0)
        sid, vlp = g.PassScheduler().next(2)
        r.path_passes(sid, vlp)
        m = r.device_mode(0)
        assert m["streams"] == 1 and m["choice"] == []
        with pytest.raises(g.BdptError):
            r.device_mode(1)
    assert L.CHOICES[16] == "pools"
