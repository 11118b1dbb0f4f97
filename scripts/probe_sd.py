"""Probe: batched vs serial metric step depth on the reference fixture cases (diagnostics only)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"), os.path.join(os.path.dirname(__file__), "..")]
import numpy as np
import depthmapx_amd as dmx
from golden_io import load_case, case_input_lines

ctx = dmx.Context(0)
for name in sys.argv[1:]:
    meta, A = load_case(name)
    pm = dmx.PointMap(meta["region"], case_input_lines(meta), meta["spacing"])
    for f in meta["fills"]:
        pm.make_points(*f)
    g = pm.make_graph(ctx)
    pts = [tuple(float(v) for v in p.split(",")) for p in meta["stepdepth"]]
    os.environ.pop("DMX_SD_KERNEL", None)
    a = g.metric_step_depth(points=pts)
    sa = ctx.last_stepdepth()
    os.environ["DMX_SD_KERNEL"] = "serial"
    b = g.metric_step_depth(points=pts)
    sb = ctx.last_stepdepth()
    bad = [(a[:, j].view(np.uint32) != b[:, j].view(np.uint32)).sum() for j in range(3)]
    ref = [(a[:, j].view(np.uint32) != A["stepdepth"][:, j].view(np.uint32)).sum() for j in range(3)]
    print(name, "batched", sa, "\n   serial", sb, "\n   diff vs serial", bad, "vs fixture", ref,
          "unreached", int((a[:, 1] == -1).sum()), int((b[:, 1] == -1).sum()), flush=True)
