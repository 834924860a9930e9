"""Write the 64-sphere synthetic Cornell scene of BASELINE config 5 / SURVEY.md 8(d)5:
the cornell.scn camera and box (its 9 spheres) plus 55 spheres drawn with numpy seed 1234 --
radius U[2, 8], centre inside the box (x in [10, 90], y in [r, 80], z in [20, 150]), material
mix 60/20/20 DIFF/SPEC/REFR, DIFF colours U[0.2, 0.9] per channel, SPEC/REFR colour 0.9.
Output: assets/scenes/synthetic64.scn (the reference's .scn format, display_func.c:112-175)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(out=os.path.join(REPO, "assets", "scenes", "synthetic64.scn")):
    base = open(os.path.join(REPO, "assets", "scenes", "cornell.scn")).read().strip().splitlines()
    cam = base[0]
    spheres = [l for l in base[2:] if l.startswith("sphere")]
    rng = np.random.default_rng(1234)
    for _ in range(55):
        r = rng.uniform(2.0, 8.0)
        x, y, z = rng.uniform(10, 90), rng.uniform(r, 80), rng.uniform(20, 150)
        u = rng.random()
        mat = 0 if u < 0.6 else (1 if u < 0.8 else 2)
        c = rng.uniform(0.2, 0.9, 3) if mat == 0 else np.full(3, 0.9)
        spheres.append(f"sphere {r:.4f}  {x:.4f} {y:.4f} {z:.4f}  0 0 0  "
                       f"{c[0]:.4f} {c[1]:.4f} {c[2]:.4f}  {mat}")
    with open(out, "w") as f:
        f.write(cam + "\n")
        f.write(f"size {len(spheres)}\n")
        f.write("\n".join(spheres) + "\n")
    print(out, len(spheres), "spheres")


if __name__ == "__main__":
    main(*sys.argv[1:])
