"""HIP kernels (through the C-ABI) vs the CPU oracle and the committed fixtures.

Bar: bit-exact for the MT607 table, the VLPs, the running-mean radiance, the counters and the
8-bit pixels on the same seeded inputs (both sides use one floating-point contract, see
DESIGN.md).  At full size (1080p) the checks are size-independent properties plus bit-exact
oracle rows.  The north-star tolerance (per-channel L-inf < 1e-3 after 1024 spp) is asserted too.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import gpu_bidirectional_raytracer_amd as g
import oracle
from conftest import GOLDEN, REPO, SCENES

pytestmark = pytest.mark.gpu

META = json.load(open(os.path.join(GOLDEN, "render_meta.json")))


@pytest.fixture(scope="module")
def rnd0():
    return oracle.mt607(0)


def scene(name):
    if name == "default":
        return g.default_scene()
    return g.read_scene(os.path.join(SCENES, name + ".scn"))


def make(name, W, H, gpu, light=True):
    cam, sp = scene(name)
    g.update_camera(cam, W, H)
    r = g.Renderer(sp, W, H, cam, device=gpu)
    if light:
        r.light_pass(0)
    return r, cam, sp


def schedule(npass):
    s = g.PassScheduler()
    s.light()
    return s.next(npass)


def assert_same(got, ref, what):
    if not np.array_equal(got, ref):
        bad = np.argwhere(got != ref)
        diff = np.abs(got.astype(np.float64) - ref.astype(np.float64))
        raise AssertionError(f"{what}: {len(bad)} mismatches of {got.size}, first {bad[:5].tolist()}, "
                             f"max |diff| {diff.max()}")


def test_mt607_table_bit_exact(gpu, rnd0):
    r, _, _ = make("cornell", 17, 9, gpu, light=False)
    ka = json.load(open(os.path.join(GOLDEN, "known_answers.json")))
    r.generate_rand(0)
    t = r.read_rand()
    assert_same(t, rnd0, "d_Rand seed 0")
    for k, v in ka["d_rand_seed0"].items():
        assert t[int(k)] == np.float32(v)
    r.generate_rand(5)
    assert_same(r.read_rand(), oracle.mt607(5), "d_Rand seed 5")
    r.close()


@pytest.mark.parametrize("name", ["cornell", "cornell_glass", "caustic", "simple", "cornell_2luci",
                                  "default", "cornell_multi", "hall_of_mirrors", "complex",
                                  "synthetic64"])
def test_light_pass_bit_exact(gpu, rnd0, name):
    r, cam, sp = make(name, 17, 9, gpu)
    ref = oracle.light_pass(sp, rnd0, 0)
    got = r.read_lightpaths()
    assert_same(got.view(np.float32), ref.view(np.float32), f"dev_lp {name}")
    r.close()


@pytest.mark.parametrize("name", META["scenes"])
def test_render_matches_golden_fixture(gpu, name):
    W, H = META["internal_size"]
    fx = np.load(os.path.join(GOLDEN, f"render_{name}.npz"))
    r, cam, sp = make(name, W, H, gpu)
    assert_same(r.read_lightpaths().view(np.float32).reshape(-1, 9), fx["lp"], "lp")
    r.path_passes(META["sid"], META["vlp"])
    col, cnt = r.read_radiance()
    assert_same(col, fx["colors"], f"colors {name}")
    assert_same(cnt, fx["counter"], f"counter {name}")
    assert_same(r.read_pixels(), fx["pixels"], f"pixels {name}")
    r.close()


@pytest.mark.parametrize("name,W,H,npass", [
    ("cornell", 61, 45, 24), ("cornell_glass", 53, 37, 24), ("caustic", 47, 35, 24),
    ("simple", 65, 33, 24), ("default", 33, 17, 16), ("cornell_2luci", 29, 21, 16),
    ("cornell_multi", 31, 23, 8), ("hall_of_mirrors", 31, 23, 8), ("gantz", 31, 23, 8),
    ("cornell_mirror_reflect", 25, 19, 8), ("complex", 17, 13, 2), ("mod_cornell", 13, 11, 2),
    ("open", 23, 17, 8), ("cornell", 1, 1, 5), ("simple", 16, 16, 3),
    ("synthetic64", 37, 21, 6),
])
def test_path_passes_bit_exact(gpu, rnd0, name, W, H, npass):
    r, cam, sp = make(name, W, H, gpu)
    sid, vlp = schedule(npass)
    r.path_passes(sid, vlp)
    col, cnt = r.read_radiance()
    lp = oracle.light_pass(sp, rnd0, 0)
    ocol, ocnt, opx = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)
    assert_same(cnt, ocnt, "counter")
    assert_same(col, ocol, f"colors {name}")
    assert_same(r.read_pixels(), opx, "pixels")
    r.close()


def test_split_launches_equal_one_launch(gpu):
    sid, vlp = schedule(9)
    a, _, _ = make("cornell", 40, 24, gpu)
    a.path_passes(sid, vlp)
    b, _, _ = make("cornell", 40, 24, gpu)
    b.path_passes(sid[:2], vlp[:2])
    b.path_passes(sid[2:7], vlp[2:7])
    b.path_passes(sid[7:], vlp[7:])
    for x, y in zip(a.read_radiance(), b.read_radiance()):
        assert_same(x, y, "split")
    a.close(); b.close()


@pytest.mark.parametrize("band,streams", [(16, 0), (8, 0), (8, 1), (5, 0), (24, 3)])
def test_shards_sum_to_full_frame(gpu, band, streams):
    """Bands that are whole tile rows launch only the shard's tiles (remapped grid rows); other
    band heights fall back to a per-pixel ownership test.  Either way the sum is the frame."""
    sid, vlp = schedule(4)
    full, _, _ = make("cornell_glass", 45, 70, gpu)
    full.set_streams(1)
    full.path_passes(sid, vlp)
    fc, fn = full.read_radiance()
    acc_c, acc_n = np.zeros_like(fc), np.zeros_like(fn)
    for s in range(3):
        r, _, _ = make("cornell_glass", 45, 70, gpu)
        r.set_shard(s, 3, band)
        r.set_streams(streams)
        r.path_passes(sid, vlp)
        c, n = r.read_radiance()
        owned = ((np.arange(70) // band) % 3 == s)
        assert (n[~owned] == 0).all() and (n[owned] == 4).all()
        acc_c += c
        acc_n += n
        r.close()
    assert_same(acc_c, fc, "shard sum colors")
    assert_same(acc_n, fn, "shard sum counter")
    full.close()


@pytest.mark.parametrize("streams", [1, 2, 3, 7, 16])
def test_pass_streams_bit_exact(gpu, rnd0, streams):
    """S lanes per pixel render passes s, s+S, ...; the ordered fold must give the oracle's
    running mean bit for bit, across split calls (11 passes: S clamps to the call's count)."""
    W, H = 37, 29
    r, cam, sp = make("cornell_glass", W, H, gpu)
    r.set_streams(streams)
    sid, vlp = schedule(16)
    r.path_passes(sid[:5], vlp[:5])
    assert r.last_streams == min(streams, 5)
    r.path_passes(sid[5:], vlp[5:])
    assert r.last_streams == min(streams, 11)
    col, cnt = r.read_radiance()
    lp = oracle.light_pass(sp, rnd0, 0)
    ocol, ocnt, opix = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)
    assert_same(cnt, ocnt, "counter")
    assert_same(col, ocol, "colors")
    assert_same(r.read_pixels(), opix, "pixels")
    r.close()


def test_per_lane_streams_policy(gpu):
    """-1: one pass per lane (S = passes in the launch, <= 128, launches of equal size); 1 forces
    the fused kernel."""
    r, _, _ = make("cornell", 1921, 1081, gpu)
    r.set_streams(-1)
    sid, vlp = schedule(200)
    r.path_passes(sid[:1], vlp[:1])
    assert r.last_streams == 1
    r.path_passes(sid[1:9], vlp[1:9])
    assert r.last_streams == 8
    r.path_passes(sid[9:200], vlp[9:200])                 # 191 passes: launches of 96 + 95
    assert r.last_streams == 96
    r.path_passes(sid[:128], vlp[:128])                   # 128 passes: one launch
    assert r.last_streams == 128
    r.set_shard(3, 8, 8)
    r.path_passes(sid[:8], vlp[:8])
    assert r.last_streams == 8
    r.set_streams(1)
    r.path_passes(sid[:8], vlp[:8])
    assert r.last_streams == 1
    r.close()
    s, _, _ = make("cornell", 65, 49, gpu)
    s.set_streams(-1)
    s.path_passes(sid[:8], vlp[:8])
    assert s.last_streams == 8
    s.close()


@pytest.mark.parametrize("name", ["cornell", "caustic"])
def test_auto_streams_measured(gpu, rnd0, name):
    """Auto (0): the first ten calls of >= 2 passes run pass streams with two passes per lane
    (launches of >= 4 passes), the fused kernel with paired segment loads, pass streams with four
    passes per lane (launches of >= 8), two per lane again, the fused kernel without pairing,
    four per lane again, twice pass streams with pixel pools (one pass per lane slice, S = the
    call's passes), and twice the ordered in-kernel fold (units; frames too small for it -- this
    one -- repeat two passes per lane there, and those calls decide nothing); later calls use the
    fastest pass-stream variant, or the faster fused one if it measured faster still; a scene
    change measures again.  Every call's result is the oracle's whatever was chosen."""
    W, H = 97, 65
    r, cam, sp = make(name, W, H, gpu)
    sid, vlp = schedule(112)
    r.path_passes(sid[:1], vlp[:1])                        # 1 pass: not a measurement
    assert r.last_streams == 1
    for k, want in enumerate((4, 1, 2, 4, 1, 2, 8, 8, 4, 4)):   # the ten measured calls of 8 passes
        a0 = 1 + 8 * k
        r.path_passes(sid[a0:a0 + 8], vlp[a0:a0 + 8])
        assert r.last_streams == want, (k, r.last_streams)
        if k in (6, 7):
            assert "pixel_pools" in r.last_features, (k, r.last_features)
        assert "unit_fold" not in r.last_features, (k, r.last_features)
    used = []
    for a0 in (81, 89):
        r.path_passes(sid[a0:a0 + 8], vlp[a0:a0 + 8])
        used.append(r.last_streams)
    assert used[0] == used[1] and used[0] in (1, 2, 4, 8), used
    assert "decided" in r.device_mode(0)["choice"] and "units" not in r.device_mode(0)["choice"]
    col, cnt = r.read_radiance()
    lp = oracle.light_pass(sp, rnd0, 0)
    ocol, ocnt, opix = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid[:97], vlp[:97])
    assert_same(cnt, ocnt, "counter")
    assert_same(col, ocol, "colors")
    assert_same(r.read_pixels(), opix, "pixels")
    r.set_scene(sp)                                        # ReInitScene: measure again
    r.path_passes(sid[97:104], vlp[97:104])
    assert r.last_streams == 4                             # 7 passes, two per lane
    r.close()


def test_auto_streams_measure_units(gpu, rnd0):
    """A frame with enough tile workgroups (1025 x 769: 33 x 97 = 3,201 >= 2 x CUs x 6): the
    ninth and tenth measured calls run the ordered in-kernel fold (units); every call's frame is
    still the oracle's (checked on a band of rows)."""
    W, H = 1025, 769
    r, cam, sp = make("cornell", W, H, gpu)
    sid, vlp = schedule(8 * 12)
    for k in range(12):
        r.path_passes(sid[8 * k:8 * (k + 1)], vlp[8 * k:8 * (k + 1)])
        if k in (8, 9):
            assert "unit_fold" in r.last_features, (k, r.last_features)
    col, cnt = r.read_radiance()
    assert (cnt == 96).all()
    lp = oracle.light_pass(sp, rnd0, 0)
    for y0 in (0, 384, 760):
        ocol, ocnt, opix = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp, rows=(y0, y0 + 2))
        assert_same(col[y0:y0 + 2], ocol[y0:y0 + 2], f"colors rows {y0}")
        assert_same(r.read_pixels()[y0:y0 + 2], opix[y0:y0 + 2], f"pixels rows {y0}")
    r.close()


def test_reset_accum_and_scene_edit(gpu, rnd0):
    """ReInit / ReInitScene semantics: counter restarts, new spheres, new light pass."""
    W, H = 31, 21
    r, cam, sp = make("cornell", W, H, gpu)
    sid, vlp = schedule(6)
    r.path_passes(sid[:3], vlp[:3])
    r.reset_accum()
    sp2 = sp.copy()
    assert g.sphere_key(sp2, 6, "4")
    r.set_scene(sp2)
    r.light_pass(0)
    r.path_passes(sid[3:], vlp[3:])
    col, cnt = r.read_radiance()
    lp = oracle.light_pass(sp2, rnd0, 0)
    ocol, ocnt, _ = oracle.path_passes(sp2, rnd0, cam, W, H, lp, sid[3:], vlp[3:])
    assert_same(cnt, ocnt, "counter after reset")
    assert_same(col, ocol, "colors after reset")
    r.close()


@pytest.mark.parametrize("streams", [0, 1])
def test_counter_cap_30000(gpu, rnd0, streams):
    W, H = 3, 2
    r, cam, sp = make("simple", W, H, gpu)
    r.set_streams(streams)
    sid, vlp = schedule(30004)
    r.path_passes(sid[:29990], vlp[:29990])
    r.path_passes(sid[29990:], vlp[29990:])   # the cap falls inside this call
    col, cnt = r.read_radiance()
    assert (cnt == 30000).all()
    lp = oracle.light_pass(sp, rnd0, 0)
    ocol, ocnt, _ = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)
    assert_same(col, ocol, "colors at cap")
    r.close()


def test_1080p_properties_and_oracle_rows(gpu, rnd0):
    """configs[*] at full size: counters, finiteness, pixel = toInt(colors), oracle rows."""
    W, H, npass = 1921, 1081, 3
    r, cam, sp = make("cornell", W, H, gpu)
    sid, vlp = schedule(npass)
    r.path_passes(sid, vlp)
    col, cnt = r.read_radiance()
    px = r.read_pixels()
    assert (cnt == npass).all()
    assert np.isfinite(col).all() and (col >= 0).all()
    assert (px[..., 3] == 0).all()
    thr = np.zeros(256, np.float32)
    g._lib.lib.bdpt_gamma_thresholds(g._lib.ctypes.c_void_p(thr.ctypes.data))
    k = np.searchsorted(thr, col.reshape(-1), side="right").reshape(col.shape) - 1
    assert_same(px[..., :3], k.astype(np.uint8), "pixels vs toInt(colors)")
    lp = oracle.light_pass(sp, rnd0, 0)
    for y in (0, 1, 540, 1079, 1080):
        ocol, ocnt, _ = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp, rows=(y, y + 1))
        assert_same(col[y], ocol[y], f"row {y}")
    r.close()


def test_linf_after_1024_spp(gpu, rnd0):
    """North-star tolerance: per-channel L-inf < 1e-3 vs the CPU path after 1024 spp."""
    W, H, npass = 24, 18, 1024
    r, cam, sp = make("cornell", W, H, gpu)
    sid, vlp = schedule(npass)
    r.path_passes(sid, vlp)
    col, _ = r.read_radiance()
    lp = oracle.light_pass(sp, rnd0, 0)
    ocol, _, _ = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)
    linf = float(np.abs(col - ocol).max())
    assert linf < 1e-3, linf
    assert np.array_equal(col, ocol)           # and in practice bit-exact
    r.close()


def test_update_pixels_after_external_reduce(gpu):
    r, _, _ = make("caustic", 20, 12, gpu)
    sid, vlp = schedule(2)
    r.path_passes(sid, vlp)
    px = r.read_pixels()
    r.update_pixels()
    assert_same(r.read_pixels(), px, "pixels recomputed")
    r.close()


def test_smallpt_mirror_and_host_program(gpu, tmp_path):
    """SmallPT (the Python mirror) and the C host program `smallpt` produce the same image."""
    spt = g.SmallPT(32, 24, os.path.join(SCENES, "cornell.scn"), device=gpu)
    spt.IdleFunc(1)                  # light pass + first path pass
    spt.IdleFunc(3)
    ppm_py = spt.SavePPM(str(tmp_path / "py.ppm"))
    exe = os.path.join(REPO, "gpu_bidirectional_raytracer_amd", "smallpt")
    out = tmp_path / "c.ppm"
    subprocess.check_call([exe, "32", "24", os.path.join(SCENES, "cornell.scn"), "--spp", "4",
                           "--batch", "1", "--out", str(out), "--dat",
                           os.path.join(REPO, "assets", "data", "MersenneTwister.dat")], cwd=tmp_path)
    assert open(ppm_py).read() == out.read_text()
    spt.FreeBuffers()


def test_rccl_frame_assembly_world1(gpu):
    """bench.py's N>1 assembly path on one GPU: torch tensors aliasing libbdpt's device buffers
    (__cuda_array_interface__) and an RCCL ("nccl") sum-reduce in a world-size-1 group."""
    import socket

    import torch
    import torch.distributed as dist

    from gpu_bidirectional_raytracer_amd import sharding as shd

    r, _, _ = make("cornell", 40, 24, gpu)
    sid, vlp = schedule(3)
    r.path_passes(sid, vlp)
    col, cnt = r.read_radiance()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(gpu)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", gpu))
    try:
        t_col, t_cnt = shd.device_tensors(r, f"cuda:{gpu}")
        assert np.array_equal(t_col.cpu().numpy().reshape(col.shape), col)
        assert np.array_equal(t_cnt.cpu().numpy().reshape(cnt.shape), cnt.astype(np.int32))
        shd.reduce_frame(t_col, t_cnt)
        torch.cuda.synchronize()
        col2, cnt2 = r.read_radiance()               # the reduce wrote into libbdpt's buffers
        assert_same(col2, col, "reduced colors")
        assert_same(cnt2, cnt, "reduced counters")
        r.update_pixels()
    finally:
        dist.destroy_process_group()
        r.close()


# ---- large scenes through the BVH (bdpt_bvh.cpp) --------------------------------
@pytest.mark.parametrize("name,W,H,npass", [("complex", 64, 48, 4), ("mod_cornell", 48, 36, 4),
                                            ("synthetic64", 40, 30, 4)])
def test_bvh_bit_exact_vs_oracle(gpu, rnd0, name, W, H, npass):
    r, cam, sp = make(name, W, H, gpu)
    assert r.has_bvh
    r.set_traversal("bvh")                    # synthetic64 (58 BVH spheres) is brute force in auto
    sid, vlp = schedule(npass)
    r.path_passes(sid, vlp)
    assert r.last_traversal == "bvh"
    col, cnt = r.read_radiance()
    lp = oracle.light_pass(sp, rnd0, 0)
    ocol, ocnt, opix = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)
    assert_same(cnt, ocnt, "counter")
    assert_same(col, ocol, "colors")
    assert_same(r.read_pixels(), opix, "pixels")
    r.close()


@pytest.mark.parametrize("name,keys", [("mod_cornell", ""), ("complex", ""), ("mod_cornell", "s" * 40),
                                       ("complex", "s" * 60 + "r" * 10)])
def test_bvh_equals_brute_force(gpu, name, keys):
    """Same frame through the BVH and through the reference's every-sphere loop, bit for bit;
    the camera moved far back (tiny spheres at long range: the margin's q*D^2 term)."""
    W, H = 241, 181
    sid, vlp = schedule(3)
    out = []
    for mode in ("bvh", "brute"):
        cam, sp = scene(name)
        g.update_camera(cam, W, H)
        for k in keys:
            g.camera_key(cam, k)
            g.update_camera(cam, W, H)
        r = g.Renderer(sp, W, H, cam, device=gpu)
        r.light_pass(0)
        r.set_traversal(mode)
        r.path_passes(sid, vlp)
        assert r.last_traversal == mode
        out.append(r.read_radiance())
        r.close()
    assert_same(out[0][1], out[1][1], "counter")
    assert_same(out[0][0], out[1][0], "colors")


def test_bvh_1080p_oracle_rows(gpu, rnd0):
    W, H = 1921, 1081
    r, cam, sp = make("mod_cornell", W, H, gpu)
    sid, vlp = schedule(2)
    r.path_passes(sid, vlp)
    col, cnt = r.read_radiance()
    assert (cnt == 2).all()
    lp = oracle.light_pass(sp, rnd0, 0)
    for y in (0, 333, 1080):
        ocol, _, _ = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp, rows=(y, y + 1))
        assert_same(col[y], ocol[y], f"row {y}")
    r.close()


# ---- edge cases: empty scene, no emitter, the N=16/17 kernel boundary, thin frames -----------
def _render_vs_oracle(gpu, rnd0, cam, sp, W, H, npass, streams=0):
    g.update_camera(cam, W, H)
    r = g.Renderer(sp, W, H, cam, device=gpu)
    r.light_pass(0)
    r.set_streams(streams)
    sid, vlp = schedule(npass)
    r.path_passes(sid, vlp)
    col, cnt = r.read_radiance()
    lp = oracle.light_pass(sp, rnd0, 0)
    assert_same(r.read_lightpaths()["hp"], lp["hp"], "vlp")
    ocol, ocnt, opix = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)
    assert_same(cnt, ocnt, "counter")
    assert_same(col, ocol, "colors")
    assert_same(r.read_pixels(), opix, "pixels")
    r.close()
    return col


@pytest.mark.parametrize("streams", [0, 1])
def test_scene_without_emitters(gpu, rnd0, streams):
    cam, sp = scene("cornell")
    sp = sp[np.all(sp["e"] == 0, axis=1)].copy()            # drop the light
    col = _render_vs_oracle(gpu, rnd0, cam, sp, 29, 17, 5, streams)
    assert (col == 0).all()                                   # no emitter, no light paths: black


def test_single_sphere_scene(gpu, rnd0):
    cam, sp = scene("cornell")
    _render_vs_oracle(gpu, rnd0, cam, sp[8:9].copy(), 23, 19, 4)   # the light alone


@pytest.mark.parametrize("n", [16, 17])
def test_template_boundary_16_17_spheres(gpu, rnd0, n):
    """16 spheres: the last compile-time instance (SGPR geometry); 17: the generic LDS kernel."""
    cam, sp = scene("synthetic64")
    _render_vs_oracle(gpu, rnd0, cam, np.ascontiguousarray(sp[-n:]), 31, 21, 4)


# Frame shapes for the packed edges (bdpt_kernels.hip BDPT_PACK_EDGES, tests/test_pixel_mapping.py):
# last workgroup column of <= 8 columns and/or last workgroup row of < 8 rows, both, neither, and
# a wide last column beside a packed last row (the corner workgroup keeps its own tile).
@pytest.mark.parametrize("W,H,streams", [(121, 89, 0), (121, 89, 1), (33, 17, 0), (40, 8, 0), (9, 3, 1),
                                         (64, 24, 0), (65, 25, 1), (100, 33, 0)])
def test_edge_packing_shapes(gpu, rnd0, W, H, streams):
    cam, sp = scene("cornell_glass")
    _render_vs_oracle(gpu, rnd0, cam, sp, W, H, 3, streams=streams)


@pytest.mark.parametrize("W,H", [(1921, 1), (1, 301), (37, 9)])
def test_thin_frames(gpu, rnd0, W, H):
    cam, sp = scene("cornell_glass")
    _render_vs_oracle(gpu, rnd0, cam, sp, W, H, 3)


def test_empty_scene(gpu, rnd0):
    cam, sp = scene("cornell")
    col = _render_vs_oracle(gpu, rnd0, cam, sp[:0].copy(), 13, 7, 3)
    assert (col == 0).all()
