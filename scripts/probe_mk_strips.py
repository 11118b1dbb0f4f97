"""makeGraph cost per strip of x columns (config 5 by default): where the edge shards of
probe_shard_balance.py spend their extra time.  DMX_VERBOSE=1 adds the per-attempt log (retries).

    python scripts/probe_mk_strips.py [--config 2|5] [--width 50] [--strips 0,1,2,...]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import depthmapx_amd as dmx  # noqa: E402
from bench import load_lines  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--width", type=int, default=50)
    ap.add_argument("--strips", default="")
    a = ap.parse_args()
    if a.config == 5:
        W, occ, lmin, lmax = 1999, 5000, 0.0025, 0.01
    else:
        W, occ, lmin, lmax = 1000, 50, 0.02, 0.10
    ctx = dmx.Context(0)
    pm = dmx.PointMap([0.0, 0.0, float(W), float(W)], load_lines(W, occ, lmin, lmax), 1.0)
    assert pm.make_points(0.5, 0.5)
    N = pm.info()["filled"]
    rows = N // (W + 1) if N % (W + 1) == 0 else None
    per_col = N / float(W + 1)
    nstrips = (W + 1 + a.width - 1) // a.width
    sel = [int(s) for s in a.strips.split(",")] if a.strips else list(range(nstrips))
    res = []
    for s in sel:
        b = int(round(s * a.width * per_col))
        e = min(N, int(round((s + 1) * a.width * per_col)))
        g = pm.make_graph(ctx, node_begin=b, node_end=e)
        t = ctx.last_timing()[0]
        st = ctx.last_stats()
        g.close()
        res.append({"strip": s, "x0": s * a.width, "nodes": e - b, "s": t, "us_per_src": 1e6 * t / max(e - b, 1),
                    "sieve_cells": st["mk_cells_examined"], "pairs": st["mk_visible_pairs"], "runs": st["mk_runs"],
                    "steps": st["mk_depth_steps"], "chunks": st["mk_chunks"]})
        r = res[-1]
        print("strip %3d x %4d..%4d  %7d src  %.3f s  %.2f us/src  sieve %.3g  pairs %.3g  runs %.3g  steps %.3g  "
              "chunks %.3g" % (s, r["x0"], r["x0"] + a.width, r["nodes"], t, r["us_per_src"], r["sieve_cells"],
                               r["pairs"], r["runs"], r["steps"], r["chunks"]),
            flush=True)
    print(json.dumps({"config": a.config, "N": N, "rows": rows, "strips": res}))


if __name__ == "__main__":
    main()
