"""GPU probe: makeGraph kernel time on the synthetic W x W grid for a list of env settings.
    python scripts/probe_mk.py W [VAR=VALUE ...]   (each setting applied on top of the previous ones)"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import depthmapx_amd as dmx  # noqa: E402
from bench import load_lines  # noqa: E402

W = int(sys.argv[1])
ctx = dmx.Context(0)
pm = dmx.PointMap([0.0, 0.0, float(W), float(W)], load_lines(W, 50), 1.0)
assert pm.make_points(0.5, 0.5)
ref = None
for cfg in ["base"] + sys.argv[2:]:
    if cfg != "base":
        k, v = cfg.split("=")
        os.environ[k] = v
    g = pm.make_graph(ctx)
    t = ctx.last_timing()[0]
    st = ctx.last_stats()
    d = g.copy(runs=False) if W <= 1000 else None
    same = None
    if d is not None:
        if ref is None:
            ref = d
        else:
            same = all(bool((d[k] == ref[k]).all()) for k in ("bins", "gridconn")) and bool(
                (d["attrs"].view("u4") == ref["attrs"].view("u4")).all())
    print(json.dumps({"config": cfg, "makegraph_kernel_s": t, "runs": g.info()["nruns"], "same_as_base": same,
                      "cells_examined": st["mk_cells_examined"]}), flush=True)
    del g
