"""Time VGA angular (-vm angular, all sources) on the bench's synthetic grid on cuda:0."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import depthmapx_amd as dmx  # noqa: E402
from bench import load_lines  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=128)
ap.add_argument("--sources", type=int, default=-1, help="first S sources only (-1: all)")
args = ap.parse_args()
W = args.grid
ctx = dmx.Context(0)
pm = dmx.PointMap([0.0, 0.0, float(W), float(W)], load_lines(W, 50), 1.0)
assert pm.make_points(0.5, 0.5)
g = pm.make_graph(ctx)
g.vga_angular(src_begin=0, src_end=64)   # warm-up
t = time.perf_counter()
out = g.vga_angular(src_end=args.sources)
wall = time.perf_counter() - t
n = out.shape[0]
ns = n if args.sources < 0 else min(n, args.sources)
print(json.dumps({"grid": W, "nodes": n, "sources": ns, "kernel_s": ctx.last_timing()[1], "wall_s": wall,
                  "sources_per_s": ns / ctx.last_timing()[1], "sample": out[ns // 2].tolist()}))
