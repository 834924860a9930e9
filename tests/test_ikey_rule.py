"""The integer-key form of the sphere tests (bdpt_kernels.hip `key_of`, BDPT_IKEY) against the
float form it replaces, on the host: for root pairs t1 <= t2 (or both NaN, as the kernel's roots
are), the closest-hit update `t2 > EPS && r < t` with r = t1 > EPS ? t1 : t2 (device.cu:106-124
through SphereIntersectDevice :80-104) must pick the same distance as min3(key(t), key(t1),
key(t2)), and the shadow test `t2 > EPS && r < maxt` must equal min(key(t1), key(t2)) <
maxt_key(maxt).  The GPU tests check the kernels bit for bit; this checks the rule itself on the
edge values (0, -0, EPS and its neighbours, +-inf, NaN, denormals) and on random roots."""
import numpy as np

EPS = np.float32(0.01)
KEYC = np.uint32(0x3C23D70B)                 # bits(0.01f) + 1


def key(x):
    return (np.asarray(x, np.float32).view(np.uint32) - KEYC).astype(np.uint32)


def maxt_key(m):
    m = np.asarray(m, np.float32)
    with np.errstate(invalid="ignore"):
        return np.where(m > EPS, key(m), np.uint32(0)).astype(np.uint32)


def float_rule(t1, t2, t):
    with np.errstate(invalid="ignore"):
        r = np.where(t1 > EPS, t1, t2)
        upd = (t2 > EPS) & (r < t)
    return np.where(upd, r, t), upd


def shadow_float(t1, t2, maxt):
    with np.errstate(invalid="ignore"):
        r = np.where(t1 > EPS, t1, t2)
        return (t2 > EPS) & (r < maxt)


def edge_values():
    f = np.float32
    eps_bits = np.array([EPS], np.float32).view(np.uint32)[0]
    near_eps = np.array([eps_bits - 1, eps_bits, eps_bits + 1], np.uint32).view(np.float32)
    vals = [f(0), f(-0.0), f(1e-45), f(-1e-45), f(1e-30), f(0.005), f(1), f(-1), f(1e20),
            f(3.4e38), f(-3.4e38), f(np.inf), f(-np.inf), f(np.nan), f(-np.nan), f(1e4), f(-1e4)]
    return np.concatenate([np.array(vals, np.float32), near_eps])


def ordered_pairs(v):
    """all (t1, t2) with t1 <= t2, plus the pairs fl(b - s), fl(b + s) forms with a NaN: both NaN,
    and b = -+inf with s = +inf (-inf, NaN) and (NaN, +inf)"""
    a, b = np.meshgrid(v, v, indexing="ij")
    a, b = a.ravel(), b.ravel()
    with np.errstate(invalid="ignore"):
        keep = a <= b
    nan, inf = np.float32(np.nan), np.float32(np.inf)
    t1 = np.concatenate([a[keep], [nan, -inf, nan]]).astype(np.float32)
    t2 = np.concatenate([b[keep], [nan, nan, inf]]).astype(np.float32)
    return t1, t2


def roots_from_spheres(n, seed):
    """roots the way the kernel forms them: b -+ fl(sqrt(det)) from random rays and spheres"""
    rng = np.random.default_rng(seed)
    o = rng.uniform(-50, 150, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    c = rng.uniform(-50, 150, (n, 3)).astype(np.float32)
    rad = np.exp(rng.uniform(np.log(0.5), np.log(1e4), n)).astype(np.float32)
    # a fifth of the origins on the sphere surface (hit points): roots near 0 and EPS
    on = rng.random(n) < 0.2
    o[on] = c[on] + rad[on, None] * d[on] * np.float32(-1)
    op = (c - o).astype(np.float32)
    b = (op[:, 0] * d[:, 0] + op[:, 1] * d[:, 1]).astype(np.float32) + (op[:, 2] * d[:, 2]).astype(np.float32)
    oo = (op[:, 0] * op[:, 0] + op[:, 1] * op[:, 1]).astype(np.float32) + (op[:, 2] * op[:, 2]).astype(np.float32)
    det = ((b * b).astype(np.float32) - oo).astype(np.float32) + (rad * rad).astype(np.float32)
    with np.errstate(invalid="ignore"):
        s = np.sqrt(det.astype(np.float32))
    return (b - s).astype(np.float32), (b + s).astype(np.float32)


def check(t1, t2, t):
    nt, upd = float_rule(t1, t2, t)
    kt = key(t)
    nk = np.minimum(kt, np.minimum(key(t1), key(t2)))
    assert np.array_equal(nk < kt, upd)
    # the running distance comes back from its key unchanged
    back = (nk + KEYC).astype(np.uint32).view(np.float32)
    assert np.array_equal(back.view(np.uint32), nt.astype(np.float32).view(np.uint32))


def test_closest_hit_rule_on_edge_values():
    t1, t2 = ordered_pairs(edge_values())
    # the running distance: the kernel's start (1e20) and earlier hits (> EPS, +inf included)
    for t in [np.float32(1e20), np.float32(0.0100001), np.float32(1.0), np.float32(np.inf),
              np.float32(3.4e38)]:
        if not t > EPS:
            continue
        check(t1, t2, np.full_like(t1, t))


def test_shadow_rule_on_edge_values():
    t1, t2 = ordered_pairs(edge_values())
    for m in edge_values():
        maxt = np.full_like(t1, m)
        got = np.minimum(key(t1), key(t2)) < maxt_key(maxt)
        assert np.array_equal(got, shadow_float(t1, t2, maxt)), f"maxt={m}"


def test_rules_on_sphere_roots():
    t1, t2 = roots_from_spheres(400_000, 7)
    with np.errstate(invalid="ignore"):
        assert not np.any(t1 > t2)                           # the ordering the proof rests on
    rng = np.random.default_rng(8)
    t = np.where(rng.random(t1.size) < 0.3, np.float32(1e20),
                 rng.uniform(0.011, 300, t1.size).astype(np.float32)).astype(np.float32)
    check(t1, t2, t)
    maxt = rng.uniform(-1, 300, t1.size).astype(np.float32)
    got = np.minimum(key(t1), key(t2)) < maxt_key(maxt)
    assert np.array_equal(got, shadow_float(t1, t2, maxt))
