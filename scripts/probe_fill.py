"""Times the VISPREP preparation at the benchmark sizes: host model (dmx_pointmap_fill) against the GPU
path (dmx_pointmap_fill_device: blockLines + the ordered flood fill), same inputs, results compared.
Usage: python scripts/probe_fill.py  -> one JSON line per configuration."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import depthmapx_amd as dmx  # noqa: E402
from golden_io import GOLDEN, read_csv_lines  # noqa: E402

ctx = dmx.Context(0)
for cfg, W in (("syn1000", 1000.0), ("syn2000_5000", 1999.0)):
    lines = read_csv_lines(os.path.join(GOLDEN, "inputs", cfg + ".csv"))
    region = [0.0, 0.0, W, W]
    # warm the GPU path once (first-launch costs), then time both
    dmx.PointMap(region, lines, 1.0).make_points(0.5, 0.5, ctx=ctx)
    a = dmx.PointMap(region, lines, 1.0)
    t = time.perf_counter()
    assert a.make_points(0.5, 0.5)
    host_s = time.perf_counter() - t
    b = dmx.PointMap(region, lines, 1.0)
    t = time.perf_counter()
    assert b.make_points(0.5, 0.5, ctx=ctx)
    dev_s = time.perf_counter() - t
    blk, fl, levels = ctx.last_fill()
    same = bool(np.array_equal(a.state(), b.state()))
    print(json.dumps({"config": cfg, "cells": a.state().size, "filled": b.info()["filled"], "host_fill_s": host_s,
                      "gpu_fill_call_s": dev_s, "gpu_blocklines_s": blk, "gpu_floodfill_s": fl, "levels": levels,
                      "states_equal": same}), flush=True)
