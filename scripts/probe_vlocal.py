"""Time VGA visual local (-vl) on the bench's synthetic grid (default 256^2) on cuda:0."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import depthmapx_amd as dmx  # noqa: E402
from bench import load_lines  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=256)
args = ap.parse_args()
W = args.grid
ctx = dmx.Context(0)
pm = dmx.PointMap([0.0, 0.0, float(W), float(W)], load_lines(W, 50), 1.0)
assert pm.make_points(0.5, 0.5)
g = pm.make_graph(ctx)
g.vga_visual_local(src_begin=0, src_end=256)          # warm-up
t = time.perf_counter()
out = g.vga_visual_local()
wall = time.perf_counter() - t
st = ctx.last_stats()
n = out.shape[0]
print(json.dumps({"grid": W, "nodes": n, "kernel_s": ctx.last_timing()[1], "wall_s": wall,
                  "cells_per_s": n / ctx.last_timing()[1], "neighbour_runs": st["vga_runs_expanded"],
                  "sample": out[n // 2].tolist()}))
