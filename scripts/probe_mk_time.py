"""Whole-map makeGraph kernel time (ctx.last_timing) for A/B builds selected with DMX_LIB.

    DMX_LIB=depthmapx_amd/_lib_ab/<variant>/libdmx.so python scripts/probe_mk_time.py [--config 2|5] [--reps 2]
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
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    W, occ, lmin, lmax = (1999, 5000, 0.0025, 0.01) if a.config == 5 else (1000, 50, 0.02, 0.10)
    ctx = dmx.Context(0)
    pm = dmx.PointMap([0.0, 0.0, float(W), float(W)], load_lines(W, occ, lmin, lmax), 1.0)
    assert pm.make_points(0.5, 0.5)
    ts = []
    for _ in range(a.reps):
        g = pm.make_graph(ctx)
        ts.append(ctx.last_timing()[0])
        st = ctx.last_stats()
        g.close()
    print(json.dumps({"lib": os.environ.get("DMX_LIB", "default"), "tag": a.tag, "config": a.config, "mk_s": ts,
                      "pairs": st["mk_visible_pairs"], "runs": st["mk_runs"],
                      "reruns": st["mk_reruns"]}), flush=True)


if __name__ == "__main__":
    main()
