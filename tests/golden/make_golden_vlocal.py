"""VGA visual local fixtures (-vl): runs oracle/_ref/ref_probe --vlocal (the reference's
VGAVisualLocal::run on salalib compiled from /root/reference) and saves the [N][3] columns as
tests/golden/<case>_vlocal.npy (Visual Clustering Coefficient, Visual Control, Visual
Controllability, node order).  The reference's per-source cost grows with k * sum |V(n)| * |total|
(std::find over vectors), so only cases it finishes in reasonable time are generated: kat, syn16,
syn32 take < 75 s (the default set); gallery takes ~130 s and syn64 about an hour, generated when
asked by name (gallery is committed).

Usage: python tests/golden/make_golden_vlocal.py [case ...]"""
import os
import subprocess
import sys
import tempfile

import numpy as np

from make_golden import CASES, HERE, PROBE, parse_grid


def run_case(name):
    src, spacing, fills, _vga, _rt, _keep = CASES[name]
    src_path = src if os.path.isabs(src) else os.path.join(HERE, src)
    with tempfile.TemporaryDirectory() as d:
        cmd = [PROBE, "--graph" if src_path.endswith(".graph") else "--lines", src_path, "--spacing", str(spacing),
               "--out", d, "--vlocal"]
        for p in fills:
            cmd += ["--fill", p]
        print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd, stdout=subprocess.DEVNULL)
        g = parse_grid(os.path.join(d, "grid.txt"))
        out = np.fromfile(os.path.join(d, "vlocal.bin"), dtype=np.float32).reshape(int(g["nodes"]), 3)
    np.save(os.path.join(HERE, name + "_vlocal.npy"), out)
    print(name, out.shape, "t_vlocal %.1f s" % g["t_vlocal"], flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or ["kat", "syn16", "syn32"]:
        run_case(n)
