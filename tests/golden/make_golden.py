"""Regenerate the committed golden fixtures in tests/golden/ (run from the repo root):

    python tests/golden/make_golden.py

Inputs are the scenes/MT parameters under assets/ and the reference's pass orchestration
(light pass at current_sample=0, then passes with sid = glibc rand() % RAND_N after srand(1)
and the flag/vlp_index state machine).  Outputs come from the CPU restatement in oracle/.
`known_answers.json` is NOT generated: it holds the values SURVEY.md 8(c) recorded from the
reference's own kernels, which pin the oracle.
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import oracle  # noqa: E402

SCENES = ["cornell", "cornell_glass", "caustic", "simple", "cornell_2luci"]
CLI_W, CLI_H, NPASS = 32, 24, 16          # internal 33 x 25 after the reference's +1


def glibc_rand(n, seed=1):
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(seed)
    return np.array([libc.rand() for _ in range(n)], dtype=np.int64)


def schedule(npass):
    """sid / vlp_index of passes 1..npass after the first light pass (smallpt_cpu.c:270,292)."""
    sid = (glibc_rand(npass) % oracle.RAND_N).astype(np.uint32)
    vlp, flag, v = [], 2, 1
    for _ in range(npass):
        vlp.append(v)
        if flag == 3:
            v, flag = v + 1, 1
        if flag < 3:
            flag += 1
    return sid, np.array(vlp, np.int32)


def read_scene_py(path):
    """Plain-Python parse of the .scn format (display_func.c:112-175 fscanf formats)."""
    with open(path) as f:
        toks = f.read().split()
    assert toks[0] == "camera"
    cam = [float(t) for t in toks[1:7]]
    assert toks[7] == "size"
    n = int(toks[8])
    sp = np.zeros(n, oracle.SPHERE_DTYPE)
    k = 9
    for i in range(n):
        assert toks[k] == "sphere"
        v = [float(t) for t in toks[k + 1:k + 11]]
        sp[i] = (v[0], v[1:4], v[4:7], v[7:10], int(toks[k + 11]))
        k += 12
    return np.array(cam[:3], np.float32), np.array(cam[3:], np.float32), sp


def main():
    params = oracle.load_mt_params()
    rnd0 = oracle.mt607(0, params)
    rnd5 = oracle.mt607(5, params)
    idx = np.arange(0, oracle.RAND_N, 997)
    np.savez_compressed(os.path.join(HERE, "mt607.npz"), idx=idx, seed0=rnd0[idx], seed5=rnd5[idx],
                        fnv_seed0=np.uint64(oracle.fnv1a64(rnd0)), fnv_seed5=np.uint64(oracle.fnv1a64(rnd5)))
    sid, vlp = schedule(NPASS)
    meta = {"cli_size": [CLI_W, CLI_H], "internal_size": [CLI_W + 1, CLI_H + 1], "npass": NPASS,
            "sid": sid.tolist(), "vlp": vlp.tolist(), "scenes": SCENES}
    for name in SCENES:
        orig, target, sp = read_scene_py(os.path.join(REPO, "assets", "scenes", name + ".scn"))
        W, H = CLI_W + 1, CLI_H + 1
        cam = oracle.update_camera(orig, target, W, H)
        lp = oracle.light_pass(sp, rnd0, 0)
        col, cnt, px = oracle.path_passes(sp, rnd0, cam, W, H, lp, sid, vlp)
        np.savez_compressed(os.path.join(HERE, f"render_{name}.npz"), lp=lp.view(np.float32).reshape(-1, 9),
                            colors=col, counter=cnt, pixels=px, camera=cam.view(np.float32).reshape(-1))
        print(name, "mean", col.mean(axis=(0, 1)), "lp written", int((lp["rad"].sum(1) != 0).sum()))
    with open(os.path.join(HERE, "render_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
