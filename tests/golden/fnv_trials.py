"""Byte representations of the MT607 table tried against the survey's FNV digests.

SURVEY.md 8(c) records `fnv1a64 = 83acafc23249aada` (seed 0) and `26e65505c78a1645` (seed 5) for the
table the surveyor's host-compiled reference produced, without saying which bytes were hashed.  The
seven table values the survey also recorded (d_Rand[0..3], [4095], [4096], [RAND_N-1]) match the
oracle exactly, so the table itself agrees; this script hashes the oracle's table in every
representation we could think of and records the digests in known_answers.json["fnv_trials"], so
the mismatch is auditable.  None of them reproduces the survey's digests.

    python tests/golden/fnv_trials.py            # rewrite the record
    python tests/golden/fnv_trials.py --check    # recompute and compare (tests/test_oracle_pins.py)

TEST INFRASTRUCTURE: reads only the oracle and assets/data/MersenneTwister.dat.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
import oracle  # noqa: E402

SURVEY = {"0": "83acafc23249aada", "5": "26e65505c78a1645"}
MT_RNG_COUNT, N_PER_RNG, PATH_N = 4096, 1876, 7680000


def mt607_raw(seed):
    """The tempered uint32 outputs y of RandomGPU (MersenneTwister_kernel.cu:63-110) before the
    float conversion, lane-major like d_Rand (numpy, 4096 twisters in parallel).  The float table
    is ((float)y + 1.0f) / 2^32 of these; checked against oracle.mt607 by the caller."""
    p = oracle.load_mt_params().reshape(4096, 4).astype(np.uint32)
    a, mb, mc = p[:, 0], p[:, 1], p[:, 2]
    mt = np.zeros((19, 4096), np.uint32)
    mt[0] = seed
    for s in range(1, 19):
        mt[s] = (np.uint32(1812433253) * (mt[s - 1] ^ (mt[s - 1] >> np.uint32(30))) + np.uint32(s)).astype(np.uint32)
    out = np.empty((N_PER_RNG, 4096), np.uint32)
    st = 0
    for k in range(N_PER_RNG):
        s1, sm = (st + 1) % 19, (st + 9) % 19
        y = (mt[st] & np.uint32(0xFFFFFFFE)) | (mt[s1] & np.uint32(1))
        y = mt[sm] ^ (y >> np.uint32(1)) ^ np.where(y & np.uint32(1), a, np.uint32(0))
        mt[st] = y
        st = s1
        y = y ^ (y >> np.uint32(12))
        y = y ^ ((y << np.uint32(7)) & mb)
        y = y ^ ((y << np.uint32(15)) & mc)
        y = y ^ (y >> np.uint32(18))
        out[k] = y
    return out.reshape(-1)


def text(t, fmt):
    return "".join(fmt % float(v) for v in t).encode()


def trials(seed, with_text=True):
    t = oracle.mt607(seed)
    raw = mt607_raw(seed)
    conv = ((raw.astype(np.float32) + np.float32(1.0)) / np.float32(4294967296.0)).astype(np.float32)
    assert np.array_equal(conv.view(np.uint32), t.view(np.uint32)), "raw MT outputs disagree with the oracle"
    lane = t.reshape(N_PER_RNG, MT_RNG_COUNT).T.reshape(-1)        # d_Rand[tid * N_PER_RNG + k]
    f1a, f1 = oracle.fnv1a64, oracle.fnv1_64
    rec = {
        "fnv1a64 float32 LE, RAND_N = 7,684,096 entries (d_Rand as stored)": f1a(t),
        "fnv1a64 float32 BE": f1a(t.astype(">f4")),
        "fnv1a64 float64 LE of every entry": f1a(t.astype(np.float64)),
        "fnv1a64 float32 LE, first PATH_N = 7,680,000 entries": f1a(t[:PATH_N]),
        "fnv1a64 float32 LE, transposed (d_Rand[tid * N_PER_RNG + k])": f1a(lane),
        "fnv1a64 float32 LE, lane 0 only (N_PER_RNG entries)": f1a(t[::MT_RNG_COUNT]),
        "fnv1a64 float32 LE, first 4096 entries (one value per twister)": f1a(t[:MT_RNG_COUNT]),
        "fnv1a64 uint32 LE of the tempered MT outputs y (before (y + 1) / 2^32)": f1a(raw),
        "fnv1a64 uint32 BE of y": f1a(raw.astype(">u4")),
        "fnv1_64 (multiply first) float32 LE": f1(t),
        "fnv1_64 float32 BE": f1(t.astype(">f4")),
        "fnv1_64 float64 LE": f1(t.astype(np.float64)),
        "fnv1_64 uint32 LE of y": f1(raw),
    }
    if with_text:
        for fmt, name in (("%.9g\n", "'%.9g\\n'"), ("%g\n", "'%g\\n'"), ("%f\n", "'%f\\n'"),
                          ("%.8e\n", "'%.8e\\n'")):
            b = text(t, fmt)
            rec[f"fnv1a64 of the decimal text, one {name} line per entry"] = f1a(np.frombuffer(b, np.uint8))
    return {k: f"{v:016x}" for k, v in rec.items()}


def main():
    path = os.path.join(HERE, "known_answers.json")
    ka = json.load(open(path))
    got = {s: trials(int(s)) for s in ("0", "5")}
    if "--check" in sys.argv:
        assert got == ka["fnv_trials"]["digests"], "recorded trial digests do not reproduce"
        print("fnv trials reproduce")
        return
    hits = [(s, k) for s in got for k, v in got[s].items() if v == SURVEY[s]]
    ka["fnv_trials"] = {
        "_note": "tests/golden/fnv_trials.py: the oracle's MT607 table hashed in every representation tried; "
                 "the survey's digests (seed 0: 83acafc23249aada, seed 5: 26e65505c78a1645) are matched by "
                 + (", ".join(f"seed {s}: {k}" for s, k in hits) if hits else "none of them") +
                 ". The survey's seven table values match the oracle exactly (d_rand_seed0).",
        "survey": SURVEY, "digests": got}
    with open(path, "w") as f:
        json.dump(ka, f, indent=1)
        f.write("\n")
    print(json.dumps(ka["fnv_trials"], indent=1))


if __name__ == "__main__":
    main()
