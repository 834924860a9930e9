"""bench.py's per-sample work constants (roofline numerators) match what the oracle counts on
the benchmark frame (cornell 1921x1081, the first pass of the reference schedule)."""
import os

import gpu_bidirectional_raytracer_amd as g
import oracle
from conftest import SCENES

import bench


import pytest


@pytest.mark.parametrize("name", sorted(bench.WORK))
def test_work_constants(name):
    W, H = 1921, 1081
    cam, sp = g.read_scene(os.path.join(SCENES, name + ".scn"))
    g.update_camera(cam, W, H)
    rnd = oracle.mt607(0)
    lp = oracle.light_pass(sp, rnd, 0)
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(1)
    step = bench.WORK[name].get("_rows_step", 1)
    st = {}
    for y0, y1 in ([(0, H)] if step == 1 else [(y, y + 1) for y in range(0, H, step)]):
        col, _, _, s1 = oracle.path_passes(sp, rnd, cam, W, H, lp, sid, vlp, rows=(y0, y1), stats=True)
        st = {k: st.get(k, 0) + v for k, v in s1.items()}
        st["nonzero"] = st.get("nonzero", 0) + int((col[y0:y1] != 0).any(axis=2).sum())
    n = st["samples"]
    assert n == W * len(range(0, H, step))
    for k, v in bench.WORK[name].items():
        if k.startswith("_"):
            continue
        assert abs(st[k] / n - v) <= 0.01 * abs(v) + 1e-3, (k, st[k] / n, v)
    if "_nonzero" in bench.WORK[name]:      # samples whose radiance is not +0 (pools' sparse radiance)
        assert abs(st["nonzero"] / n - bench.WORK[name]["_nonzero"]) < 2e-4, st["nonzero"] / n
    if name == "cornell":
        assert 3400 < bench.flop_per_sample(bench.WORK["cornell"]) < 3700
