"""How lossy is the .graph round trip at size?  PixelVec::write stores each run after the first of an H/V bin as
a 4-bit row shift (ngraph.cpp:536-583): a jump of more than 15 rows wraps and shifts every later run of the bin.
Counts, on the whole configs[2] / configs[4] graph: nodes with a wrapped jump, runs moved, and the cells those
moved runs cover (the nodes the re-read graph makes asymmetric).

    python scripts/probe_shift_overflow.py --config 2
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import depthmapx_amd as dmx  # noqa: E402
from bench import load_lines  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    a = ap.parse_args()
    W, occ, lmin, lmax = (1999, 5000, 0.0025, 0.01) if a.config == 5 else (1000, 50, 0.02, 0.10)
    ctx = dmx.Context(0)
    pm = dmx.PointMap([0.0, 0.0, float(W), float(W)], load_lines(W, occ, lmin, lmax), 1.0)
    assert pm.make_points(0.5, 0.5)
    g = pm.make_graph(ctx)
    N = g.info()["nnodes"]
    nodes_over = runs_moved = runs_total = 0
    chunk = 32768
    for b in range(0, N, chunk):
        e = min(N, b + chunk)
        c = g.copy_range(b, e)
        bins, runs = c["bins"], c["runs"].astype(np.int32)
        nr = bins[:, :, 3].reshape(-1).astype(np.int64)
        d = bins[:, :, 0].reshape(-1)
        start = np.concatenate([[0], np.cumsum(nr)[:-1]])
        binid = np.repeat(np.arange(len(nr)), nr)
        first = np.zeros(len(runs), bool)
        first[start[nr > 0]] = True
        dirr = np.repeat(d, nr)
        # H bins (dir 1): rows are y; V bins (dir 2): columns are x
        prim = np.where(dirr == 1, runs[:, 1], runs[:, 0])
        jump = np.zeros(len(runs), np.int64)
        jump[1:] = prim[1:] - prim[:-1]
        wrap = (~first) & ((dirr == 1) | (dirr == 2)) & ((jump < 0) | (jump > 15))
        # a wrap moves that run and every later run of its bin
        wb = np.zeros(len(nr), bool)
        wb[binid[wrap]] = True
        if wrap.any():
            firstwrap = np.full(len(nr), np.iinfo(np.int64).max)
            np.minimum.at(firstwrap, binid[wrap], np.nonzero(wrap)[0])
            idx = np.arange(len(runs))
            moved = idx >= firstwrap[binid]
            runs_moved += int(moved.sum())
        nodes_over += int(wb.reshape(-1, 32).any(axis=1).sum())
        runs_total += len(runs)
    print(json.dumps({"config": a.config, "nodes": N, "runs": runs_total, "nodes_with_wrap": nodes_over,
                      "runs_moved": runs_moved}), flush=True)


if __name__ == "__main__":
    main()
