"""Synthetic occluder-line inputs (SURVEY.md section 8(d) generator).

Region [0, W]^2 closed by four boundary walls, plus ``n`` random occluder segments whose centres
are uniform in [0.05W, 0.95W]^2, angles uniform in [0, pi) and lengths uniform in
[lmin*W, lmax*W] (so every segment lies inside the region).  The output CSV (header x1,y1,x2,y2)
is the committed fixture; nothing downstream depends on this RNG -- re-running the script is only
needed to regenerate a fixture.

    python tests/golden/gen_synthetic.py W n seed out.csv [lmin lmax]
"""
import math
import sys

import numpy as np


def make_lines(W, n, seed=1, lmin=0.02, lmax=0.10):
    rng = np.random.default_rng(seed)
    W = float(W)
    lines = [(0.0, 0.0, W, 0.0), (W, 0.0, W, W), (W, W, 0.0, W), (0.0, W, 0.0, 0.0)]
    for _ in range(n):
        cx, cy = rng.uniform(0.05 * W, 0.95 * W, size=2)
        a = rng.uniform(0.0, math.pi)
        half = 0.5 * rng.uniform(lmin * W, lmax * W)
        dx, dy = half * math.cos(a), half * math.sin(a)
        lines.append((cx - dx, cy - dy, cx + dx, cy + dy))
    return lines


def write_csv(path, lines):
    with open(path, "w") as f:
        f.write("x1,y1,x2,y2\n")
        for l in lines:
            f.write("%.6f,%.6f,%.6f,%.6f\n" % l)


if __name__ == "__main__":
    W, n, seed, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    lmin, lmax = (float(sys.argv[5]), float(sys.argv[6])) if len(sys.argv) > 6 else (0.02, 0.10)
    write_csv(out, make_lines(W, n, seed, lmin, lmax))
