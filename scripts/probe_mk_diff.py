"""GPU probe: makeGraph of the config-5 grid (2000^2, 5000 occluders) under env settings; per-node run
counts compared with the first setting, differing nodes checked against the C restatement.
    python scripts/probe_mk_diff.py VAR=VALUE[,VAR=VALUE] ...   (each argument is one setting)"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import depthmapx_amd as dmx  # noqa: E402
from bench import load_lines  # noqa: E402

W = 1999
lines = load_lines(W, 5000, 0.0025, 0.01)
ctx = dmx.Context(0)
pm = dmx.PointMap([0.0, 0.0, float(W), float(W)], lines, 1.0)
assert pm.make_points(0.5, 0.5)
N = pm.info()["filled"]
base = None
keep = ["DMX_MK_GCAP", "DMX_MK_BCAP", "DMX_MK_WPE"]
for cfg in sys.argv[1:]:
    for k in keep:
        os.environ.pop(k, None)
    for kv in cfg.split(","):
        if kv and kv != "base":
            k, v = kv.split("=")
            os.environ[k] = v
    g = pm.make_graph(ctx)
    t = ctx.last_timing()[0]
    nr = np.zeros(N, dtype=np.int64)
    CH = 200000
    for b in range(0, N, CH):
        e = min(N, b + CH)
        d = g.copy_range(b, e, runs=False)
        nr[b:e] = d["bins"][:, :, 3].sum(axis=1)
    rec = {"config": cfg, "s": t, "runs": int(nr.sum())}
    if base is None:
        base = nr
    else:
        diff = np.nonzero(nr != base)[0]
        rec["nodes_differing"] = int(len(diff))
        rec["first"] = diff[:10].tolist()
        rec["delta"] = (nr[diff[:10]] - base[diff[:10]]).tolist()
        if len(diff):
            from pyoracle import OracleMap
            om = OracleMap([0.0, 0.0, float(W), float(W)], 1.0, lines)
            om.fill(0.5, 0.5)
            chk = []
            for k in diff[:5].tolist():
                om.make_graph(node_begin=k, node_end=k + 1)
                ob = om.graph()["bins"][k]
                chk.append({"node": k, "oracle_runs": int(ob[:, 3].sum()), "this": int(nr[k]), "base": int(base[k])})
            rec["oracle"] = chk
    print(json.dumps(rec), flush=True)
    del g
