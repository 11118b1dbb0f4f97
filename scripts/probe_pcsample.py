"""Workload for PC sampling (rocprofv3 --pc-sampling-*): one whole 1000^2 makeGraph (configs[2]) and VGA
global on NSRC sources in the middle of the map, with the in-tree library or DMX_LIB (a -gline-tables-only
build maps samples to source lines).

    rocprofv3 --pc-sampling-beta-enabled ... -- python3 scripts/probe_pcsample.py [--nsrc 65536]
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
    ap.add_argument("--nsrc", type=int, default=65536)
    ap.add_argument("--skip-mk-timing", action="store_true")
    a = ap.parse_args()
    W = 1000
    ctx = dmx.Context(0)
    pm = dmx.PointMap([0.0, 0.0, float(W), float(W)], load_lines(W, 50, 0.02, 0.10), 1.0)
    assert pm.make_points(0.5, 0.5)
    g = pm.make_graph(ctx)
    mk = ctx.last_timing()[0]
    N = g.info()["nnodes"]
    b = N // 2 - a.nsrc // 2
    g.vga_visual_global(src_begin=b, src_end=b + a.nsrc)
    print(json.dumps({"makegraph_s": mk, "vga_s": ctx.last_timing()[1], "nsrc": a.nsrc,
                      "lib": os.environ.get("DMX_LIB", "default")}), flush=True)


if __name__ == "__main__":
    main()
