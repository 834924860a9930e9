"""Seeded random scenes through the whole path (light pass, scene-specialised path kernel in both
kernel kinds) against the oracle, bit for bit.  The reference scenes fix a few geometries; these
vary what the specialised kernels' exact shortcuts depend on: wall boxes of radius 1e3 to 1e5
(det skips only for the small spheres), black surfaces with and without the host's black-exit
proof (bdpt_host.cpp jit_path_kernel), zero to three emitters, every material (DIFF, SPEC, REFR,
the LITE tag), spheres that overlap or contain the camera, and cameras inside and outside the
box.  Reference: device.cu:80-154 (sphere tests), :457-542 (NEE + VLP), :544-791 (path)."""
import os

import numpy as np
import pytest

import gpu_bidirectional_raytracer_amd as g
import oracle

pytestmark = pytest.mark.gpu

W, H, NPASS = 45, 31, 6
# seeds per test (BDPT_FUZZ_SEEDS=400 for a longer one-off sweep; the suite keeps 40)
SEEDS = int(os.environ.get("BDPT_FUZZ_SEEDS", "40"))


@pytest.fixture(scope="module")
def rnd0():
    return oracle.mt607(0)


def random_scene(seed):
    rng = np.random.default_rng(seed)
    f = np.float32
    box = np.array([100.0, 80.0, 170.0])
    rows = []
    nw = rng.choice([0, 4, 6])
    R = float(rng.choice([1e3, 1e4, 1e5]))
    walls = [((-R, 40, 80), (0.75, 0.25, 0.25)), ((100 + R, 40, 80), (0.25, 0.25, 0.75)),
             ((50, -R, 80), (0.75, 0.75, 0.75)), ((50, 80 + R, 80), (0.75, 0.75, 0.75)),
             ((50, 40, -R), (0.75, 0.75, 0.75)), ((50, 40, 170 + R), (0.0, 0.0, 0.0))]
    for k in rng.permutation(6)[:nw]:
        p, c = walls[k]
        rows.append((R, p, (0, 0, 0), c, 0))
    ns = int(rng.integers(1, 13))
    for _ in range(ns):
        r = float(np.exp(rng.uniform(np.log(0.5), np.log(20.0))))
        p = rng.uniform(0, 1, 3) * box
        c = (0.0, 0.0, 0.0) if rng.random() < 0.2 else tuple(rng.uniform(0, 1, 3))
        rows.append((r, tuple(p), (0, 0, 0), c, int(rng.choice(4, p=[0.5, 0.2, 0.2, 0.1]))))
    nl = int(rng.choice([0, 1, 1, 2, 2, 3, 3]))
    for k in rng.permutation(len(rows))[:nl]:
        if rows[k][0] >= 1e3:                                   # emitters among the small spheres
            continue
        r, p, _, c, m = rows[k]
        rows[k] = (r, p, tuple(rng.uniform(1, 30, 3)), c, m)
    sp = np.zeros(len(rows), g.SPHERE_DTYPE)
    for i, (r, p, e, c, m) in enumerate(rows):
        sp[i] = (f(r), np.array(p, f), np.array(e, f), np.array(c, f), m)
    cam = g.Camera()
    inside = rng.random() < 0.8
    o = rng.uniform(0.1, 0.9, 3) * box if inside else np.array([50.0, 45.0, 300.0])
    small = sp[sp["rad"] < 1e3]
    t = small["p"][rng.integers(len(small))] + rng.normal(0, 5, 3) if rng.random() < 0.6 else \
        rng.uniform(0.1, 0.9, 3) * box                            # towards a small sphere, or anywhere
    cam.orig.x, cam.orig.y, cam.orig.z = (float(v) for v in o)
    cam.target.x, cam.target.y, cam.target.z = (float(v) for v in t)
    return cam, sp


@pytest.mark.parametrize("streams", [0, 1])
@pytest.mark.parametrize("seed", range(SEEDS))
def test_random_scene_bit_exact(gpu, rnd0, seed, streams):
    cam, sp = random_scene(1000 + seed)
    g.update_camera(cam, W, H)
    r = g.Renderer(sp, W, H, cam, device=gpu)
    r.light_pass(0)
    r.set_streams(streams)
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(NPASS)
    r.path_passes(sid, vlp)
    col, cnt = r.read_radiance()
    px = r.read_pixels()
    specialized = r.last_specialized
    r.close()
    lp = oracle.light_pass(sp, rnd0, 0)
    ocol, ocnt, opx = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)
    assert specialized
    assert np.array_equal(cnt, ocnt)
    bad = int((col.view(np.uint32) != ocol.view(np.uint32)).sum())
    assert bad == 0, f"seed {seed} streams {streams}: {bad} colour values differ ({len(sp)} spheres)"
    assert np.array_equal(px, opx)


def random_large_scene(seed):
    """Cornell-like wall box (or none) with 150-400 small spheres: the BVH path (bdpt_bvh.cpp,
    kernel instance N = -1) and the generic every-sphere loop."""
    rng = np.random.default_rng(seed)
    cam, sp = random_scene(seed)
    walls = sp[sp["rad"] >= 1e3]
    n = int(rng.integers(150, 401))
    extra = np.zeros(n, g.SPHERE_DTYPE)
    extra["rad"] = np.exp(rng.uniform(np.log(0.3), np.log(6.0), n)).astype(np.float32)
    extra["p"] = (rng.uniform(0, 1, (n, 3)) * np.array([100.0, 80.0, 170.0])).astype(np.float32)
    extra["c"] = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    extra["c"][rng.random(n) < 0.1] = 0
    extra["refl"] = rng.choice(4, n, p=[0.6, 0.15, 0.15, 0.1])
    lit = rng.permutation(n)[:int(rng.integers(1, 4))]
    extra["e"][lit] = rng.uniform(1, 30, (len(lit), 3)).astype(np.float32)
    return cam, np.concatenate([walls, extra])


@pytest.mark.parametrize("traversal", ["bvh", "brute"])
@pytest.mark.parametrize("seed", range(max(6, SEEDS // 8)))
def test_random_large_scene_bit_exact(gpu, rnd0, seed, traversal):
    cam, sp = random_large_scene(2000 + seed)
    g.update_camera(cam, W, H)
    r = g.Renderer(sp, W, H, cam, device=gpu)
    r.set_traversal(traversal)
    r.light_pass(0)
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(4)
    r.path_passes(sid, vlp)
    col, cnt = r.read_radiance()
    px = r.read_pixels()
    has_bvh = r.has_bvh
    r.close()
    lp = oracle.light_pass(sp, rnd0, 0)
    ocol, ocnt, opx = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)
    assert has_bvh
    assert np.array_equal(cnt, ocnt)
    bad = int((col.view(np.uint32) != ocol.view(np.uint32)).sum())
    assert bad == 0, f"seed {seed} {traversal}: {bad} colour values differ ({len(sp)} spheres)"
    assert np.array_equal(px, opx)


@pytest.mark.parametrize("seed", range(max(8, SEEDS // 5)))
def test_random_call_sequence_bit_exact(gpu, rnd0, seed):
    """A random scene and frame size rendered by a random sequence of calls (1-40 passes each) in
    the auto stream mode, which measures pass streams and both fused variants on its first calls
    and then keeps one: passes rendered by different kernel kinds accumulate into one frame, which
    must equal the oracle's after every call."""
    rng = np.random.default_rng(3000 + seed)
    cam, sp = random_scene(3000 + seed)
    w, h = int(rng.integers(1, 80)), int(rng.integers(1, 50))
    g.update_camera(cam, w, h)
    r = g.Renderer(sp, w, h, cam, device=gpu)
    r.light_pass(0)
    r.set_streams(0)
    lp = oracle.light_pass(sp, rnd0, 0)
    s = g.PassScheduler()
    s.light()
    ocol = ocnt = None
    for call in range(7):
        n = int(rng.integers(1, 41))
        sid, vlp = s.next(n)
        r.path_passes(sid, vlp)
        ocol, ocnt, opx = oracle.path_passes(sp, rnd0, cam, w, h, lp, sid, vlp, colors=ocol, counter=ocnt)
        col, cnt = r.read_radiance()
        assert np.array_equal(cnt, ocnt), f"seed {seed} call {call}"
        bad = int((col.view(np.uint32) != ocol.view(np.uint32)).sum())
        assert bad == 0, f"seed {seed} call {call} ({n} passes, {w}x{h}, S={r.last_streams}): {bad} differ"
        assert np.array_equal(r.read_pixels(), opx)
    r.close()


@pytest.mark.parametrize("seed", range(max(6, SEEDS // 8)))
def test_random_shards_sum_to_oracle(gpu, rnd0, seed):
    """A random scene cut into 2-8 interleaved bands of 1-24 rows (bdpt_set_shard), each band set
    rendered by its own context in the auto stream mode: every pixel is rendered by exactly one
    shard, and the sum of the shards is the oracle's frame bit for bit."""
    rng = np.random.default_rng(4000 + seed)
    cam, sp = random_scene(4000 + seed)
    w, h = int(rng.integers(8, 70)), int(rng.integers(8, 60))
    nsh, band = int(rng.integers(2, 9)), int(rng.choice([1, 3, 8, 16, 24]))
    g.update_camera(cam, w, h)
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(int(rng.integers(2, 12)))
    acc_c = np.zeros((h, w, 3), np.float32)
    acc_n = np.zeros((h, w), np.uint32)
    for k in range(nsh):
        r = g.Renderer(sp, w, h, cam, device=gpu)
        r.set_shard(k, nsh, band)
        r.light_pass(0)
        r.path_passes(sid, vlp)
        c, n = r.read_radiance()
        r.close()
        owned = (np.arange(h) // band) % nsh == k
        assert (n[~owned] == 0).all() and (n[owned] == len(sid)).all()
        acc_c += c
        acc_n += n
    lp = oracle.light_pass(sp, rnd0, 0)
    ocol, ocnt, _ = oracle.path_passes(sp, rnd0, cam, w, h, lp, sid, vlp)
    assert np.array_equal(acc_n, ocnt)
    bad = int((acc_c.view(np.uint32) != ocol.view(np.uint32)).sum())
    assert bad == 0, f"seed {seed} ({nsh} shards of {band} rows, {w}x{h}): {bad} differ"
