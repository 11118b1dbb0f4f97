"""Diagnostic: VGA global radius 3 on the semi-filled gallery through the Python API, tile kernel (per-tile
column summaries) against vga_do, per source; bad sources re-run alone and in small ranges."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import depthmapx_amd as dmx  # noqa: E402
import test_semifill as ts  # noqa: E402
import tempfile  # noqa: E402

tmp = tempfile.mkdtemp()
ctx = dmx.Context(0)
region, lines = ts._drawing(ts._input(tmp, "gallery_empty.graph"))
pm = dmx.PointMap(region, lines, 0.04)
assert pm.make_points(*ts.SEMI_SEED, fill_type=pm.SEMIFILL)
g = pm.make_graph(ctx)
N = g.info()["nnodes"]
print("cols rows", pm.cols, pm.rows, "nodes", N, "special", len(g.special_nodes()), flush=True)


def run(env, **kw):
    old = dict(os.environ)
    os.environ.update(env)
    try:
        out, lv = g.vga_visual_global(radius=3, levels=True, **kw)
    finally:
        os.environ.clear()
        os.environ.update(old)
    return out, lv, ctx.last_stats()


ref, rlv, _ = run({"DMX_VGA_KERNEL": "do"})
for env in [{"DMX_VGA_RB": "0"}, {"DMX_VGA_RB": "0", "DMX_VGA_ALPHA": "0"}, {}]:
    for rep in range(3):
        out, lv, st = run(env)
        bad = np.flatnonzero(lv[:, 0] != rlv[:, 0])
        print(env, "rep", rep, "kernel", st["vga_kernel"], "bad", len(bad), bad[:8].tolist(),
              [(int(s), rlv[s].tolist(), lv[s].tolist()) for s in bad[:3]], flush=True)
        for s in bad[:3]:
            for lo in (s, max(0, s - 8), max(0, s - 64)):
                o2, l2, _ = run(env, src_begin=int(lo), src_end=int(s) + 1)
                print("   src", int(s), "range from", int(lo), "->", l2[s].tolist(), "ref", rlv[s].tolist(), flush=True)
            o3, l3, _ = run(dict(env, DMX_VGA_CHUNK="100000"), src_begin=max(0, int(s) - 64), src_end=int(s) + 1)
            print("   src", int(s), "one workgroup over 64 before ->", l3[s].tolist(), flush=True)
