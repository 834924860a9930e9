"""Multi-device contexts through the C-ABI (bdpt_create_multi, SURVEY.md 8(b) `devices[], ndev`):
pixel bands over the devices of one process, frame assembled on devices[0] by an in-process RCCL
reduce (distinct devices) or by peer copies (shards sharing a GPU).  The bar is the one-device
frame bit for bit.  The box has one MI355X: devices=[0] exercises the RCCL path (a communicator
of one), devices=[0, 0, ...] the band logic and the peer-copy reduce.  8-GPU runs are the
driver's (bench.py through torchrun)."""
import filecmp
import os
import subprocess

import numpy as np
import pytest

import gpu_bidirectional_raytracer_amd as g
from conftest import REPO, SCENES

pytestmark = pytest.mark.gpu
SMALLPT = os.path.join(REPO, "gpu_bidirectional_raytracer_amd", "smallpt")


def schedule(n):
    s = g.PassScheduler()
    s.light()
    return s.next(n)


def render(name, W, H, sid, vlp, streams=0, **kw):
    cam, sp = g.read_scene(os.path.join(SCENES, name + ".scn"))
    g.update_camera(cam, W, H)
    with g.Renderer(sp, W, H, cam, **kw) as r:
        r.set_streams(streams)
        r.light_pass(0)
        r.path_passes(sid, vlp)
        col, cnt = r.read_radiance()
        return col, cnt, r.read_pixels(), (r.num_devices, r.reduce_backend)


def same(a, b, what):
    assert a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8)), what


_RCCL_CHILD = r"""
import sys
sys.path.insert(0, {tests!r})
import numpy as np
import test_gpu_multi as t
gpu, streams = {gpu}, {streams}
sid, vlp = t.schedule(24)
ref = t.render("cornell", 257, 193, sid, vlp, streams, device=gpu)
got = t.render("cornell", 257, 193, sid, vlp, streams, devices=[gpu])
assert got[3] == (1, "rccl") and ref[3] == (1, "none"), (got[3], ref[3])
for a, b, w in zip(got[:3], ref[:3], ("colors", "counter", "pixels")):
    t.same(a, b, w)
print("RCCL_GROUP_OK")
"""


@pytest.mark.parametrize("streams", [0, 1])
def test_one_gpu_group_rccl_equals_single_context(gpu, streams):
    """A group of one distinct device: the in-process RCCL communicator (ncclCommInitAll) and
    ncclReduce path.  Run in a child process: RCCL's topology discovery on this shared pool
    (alt_rsmi reading the sysfs nodes of GPUs this box does not expose) aborted the whole test
    process twice in round 6, inside ncclCommInitAll; in a child an abort fails this test alone
    and keeps its stderr."""
    import sys
    code = _RCCL_CHILD.format(tests=os.path.dirname(os.path.abspath(__file__)), gpu=gpu, streams=streams)
    env = dict(os.environ, NCCL_DEBUG=os.environ.get("NCCL_DEBUG", "WARN"))
    p = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0 and "RCCL_GROUP_OK" in p.stdout, \
        f"rc={p.returncode}\nstdout: {p.stdout[-2000:]}\nstderr: {p.stderr[-4000:]}"


@pytest.mark.parametrize("name,ndev", [("cornell_glass", 2), ("caustic", 3), ("cornell", 8)])
def test_shards_on_one_gpu_peer_reduce_equals_single_context(gpu, name, ndev):
    sid, vlp = schedule(12)
    ref = render(name, 161, 121, sid, vlp, device=gpu)
    got = render(name, 161, 121, sid, vlp, devices=[gpu] * ndev)
    assert got[3] == (ndev, "peer")
    for a, b, w in zip(got[:3], ref[:3], ("colors", "counter", "pixels")):
        same(a, b, w)


def test_two_groups_as_shards_sum_to_the_frame(gpu):
    """bdpt_set_shard on a group: the group is shard s of n groups (e.g. one group per node)."""
    W, H = 129, 97
    sid, vlp = schedule(8)
    cam, sp = g.read_scene(os.path.join(SCENES, "cornell.scn"))
    g.update_camera(cam, W, H)
    ref = render("cornell", W, H, sid, vlp, device=gpu)
    acc_c, acc_n = np.zeros_like(ref[0]), np.zeros_like(ref[1])
    for grp in range(2):
        with g.Renderer(sp, W, H, cam, devices=[gpu, gpu]) as r:
            r.set_shard(grp, 2, 8)
            r.light_pass(0)
            r.path_passes(sid, vlp)
            c, n = r.read_radiance()
            own = (np.arange(H) // 8) % 4
            assert (n[(own == 2 * grp) | (own == 2 * grp + 1)] == 8).all()
            acc_c += c
            acc_n += n
    same(acc_c, ref[0], "group sum colors")
    same(acc_n, ref[1], "group sum counters")


def test_scene_edit_reset_and_more_passes(gpu):
    """ReInitScene / ReInit reach every device of the group; the frame is re-assembled."""
    W, H = 97, 73
    sid, vlp = schedule(10)
    cam, sp = g.read_scene(os.path.join(SCENES, "cornell.scn"))
    g.update_camera(cam, W, H)
    moved = sp.copy()
    moved[7]["p"][0] -= 5.0
    out = []
    for kw in ({"device": gpu}, {"devices": [gpu, gpu, gpu]}):
        with g.Renderer(sp, W, H, cam, **kw) as r:
            r.light_pass(0)
            r.path_passes(sid[:4], vlp[:4])
            first = r.read_radiance()[0]
            r.set_scene(moved)
            r.reset_accum()
            r.light_pass(0)
            r.path_passes(sid[4:], vlp[4:])
            out.append((first, r.read_radiance(), r.read_pixels()))
    same(out[0][0], out[1][0], "before the edit")
    same(out[0][1][0], out[1][1][0], "colors after the edit")
    same(out[0][1][1], out[1][1][1], "counters after the edit")
    same(out[0][2], out[1][2], "pixels after the edit")


@pytest.mark.parametrize("devs", ["0,0", "0"])
def test_smallpt_host_on_several_devices(gpu, tmp_path, devs):
    args = ["65", "49", os.path.join(SCENES, "cornell.scn"), "--spp", "6", "--batch", "4", "--keys", "w+4"]
    a, b = tmp_path / "one.ppm", tmp_path / "multi.ppm"
    subprocess.check_call([SMALLPT, *args, "--out", str(a)], cwd=REPO, timeout=120)
    r = subprocess.run([SMALLPT, *args, "--devices", devs, "--out", str(b)], cwd=REPO, timeout=120,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert ("rccl" if devs == "0" else "peer") in r.stderr
    assert filecmp.cmp(a, b, shallow=False)


def test_group_devices_follow_devices0_stream_choice(gpu):
    """the peers of a group take devices[0]'s auto stream-mode decision, so every
    device runs the same kernel; the frame still equals the one-device frame bit for bit."""
    W, H = 321, 241
    cam, sp = g.read_scene(os.path.join(SCENES, "caustic.scn"))
    g.update_camera(cam, W, H)
    sid, vlp = schedule(16 * 12)
    with g.Renderer(sp, W, H, cam, devices=[gpu, gpu, gpu]) as r:
        r.set_streams(0)
        r.light_pass(0)
        for k in range(12):                                       # 10 measured calls, then the choice
            r.path_passes(sid[16 * k:16 * (k + 1)], vlp[16 * k:16 * (k + 1)])
        modes = [r.device_mode(k) for k in range(3)]
        assert "decided" in modes[0]["choice"]
        assert all(m == modes[0] for m in modes), modes
        col, cnt = r.read_radiance()
        # a rank applies rank 0's choice: the same bits, no measurement
        r.set_stream_choice(r.stream_choice)
        assert r.device_mode(2)["choice"] == modes[0]["choice"]
    ref = render("caustic", W, H, sid, vlp, device=gpu)
    same(col, ref[0], "colors")
    same(cnt, ref[1], "counter")
