"""Diagnostic: VGA angular GPU vs oracle on the merge-test map, with and without the links."""
import sys
import numpy as np
sys.path[:0] = [".", "tests", "oracle"]
import depthmapx_amd as dmx
from test_merge_links import _synthetic

ctx = dmx.Context(0)
for seed in (1, 2):
    pm, om, pairs = _synthetic(seed, W=24, nlinks=8)
    g = pm.make_graph(ctx)
    om.make_graph()
    for linked in (False, True):
        if linked:
            g.set_merges(pairs)
            om.set_merges(pairs)
        got, ref = g.vga_angular(), om.vga_angular(threads=8)
        bad = np.flatnonzero((got.view(np.uint32) != ref.view(np.uint32)).any(axis=1))
        print("seed", seed, "linked", linked, "mismatching rows", bad.tolist())
        nc = np.flatnonzero(pm.state() & 2)
        for k in bad[:8]:
            print("  node", k, "cell", nc[k], "got", got[k].tolist(), "ref", ref[k].tolist())
        gm, rm = g.vga_metric(), om.vga_metric(threads=8)
        print("  metric mismatching rows", np.flatnonzero((gm.view(np.uint32) != rm.view(np.uint32)).any(axis=1)).tolist()[:10])
    print("pairs", pairs.tolist())
