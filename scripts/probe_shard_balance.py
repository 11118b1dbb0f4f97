"""makeGraph cost per contiguous x-major source range (sharded.shard_range) at W = 2 / 4 / 8, on one GPU:
the kernel time each rank of a W-GPU node would spend on its shard.

    python scripts/probe_shard_balance.py [--config 2|5]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import depthmapx_amd as dmx  # noqa: E402
from bench import load_lines  # noqa: E402
from depthmapx_amd.sharded import shard_range  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--balanced", action="store_true", help="cost-balanced bounds (PointMap.shard_bounds)")
    ap.add_argument("--stride", type=int, default=256)
    a = ap.parse_args()
    if a.config == 5:
        W, occ, lmin, lmax = 1999, 5000, 0.0025, 0.01
    else:
        W, occ, lmin, lmax = 1000, 50, 0.02, 0.10
    ctx = dmx.Context(0)
    pm = dmx.PointMap([0.0, 0.0, float(W), float(W)], load_lines(W, occ, lmin, lmax), 1.0)
    assert pm.make_points(0.5, 0.5)
    N = pm.info()["filled"]
    g = pm.make_graph(ctx)
    whole = ctx.last_timing()[0]
    whole_runs = g.info()["nruns"]
    whole_blob = g.blob_size()
    g.close()
    res = {"config": a.config, "N": N, "whole_s": whole, "whole_runs": whole_runs, "whole_blob_bytes": whole_blob,
           "worlds": {}}
    for world in (2, 4, 8):
        ts = []
        if a.balanced:
            import time
            t0 = time.perf_counter()
            bounds = pm.shard_bounds(ctx, world, stride=a.stride)
            bal_s = time.perf_counter() - t0
            bal_k = ctx.last_timing()[0]
            print("W=%d balanced bounds %s (%.3f s wall, %.3f s kernels)" % (world, bounds, bal_s, bal_k), flush=True)
        blobs, runs = [], []
        for r in range(world):
            b, e = (bounds[r], bounds[r + 1]) if a.balanced else shard_range(N, r, world)
            s = pm.make_graph(ctx, node_begin=b, node_end=e)
            ts.append(ctx.last_timing()[0])
            blobs.append(s.blob_size())
            runs.append(s.info()["nruns"])
            s.close()
        mean = sum(ts) / len(ts)
        # the padded all-gather buffer every rank holds (sharded.exchange_graph): world x the largest blob
        res["worlds"][world] = {"rank_s": ts, "max_s": max(ts), "mean_s": mean, "spread": max(ts) / mean - 1.0,
                                "ideal_s": whole / world, "blob_bytes": blobs, "rank_runs": runs,
                                "exchange_buffer_bytes": world * max(blobs), "blob_total_bytes": sum(blobs),
                                "receive_bytes_max": sum(blobs) - min(blobs)}
        print("W=%d per-rank makeGraph s: %s  max %.3f  mean %.3f  spread %.1f%%  whole/W %.3f; blobs max %.2f GB, "
              "exchange buffer %.1f GB" % (world, " ".join("%.3f" % t for t in ts), max(ts), mean,
                                            100 * (max(ts) / mean - 1), whole / world, max(blobs) / 1e9,
                                            world * max(blobs) / 1e9), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
