"""configs[4] on one GPU: the 8-rank 2000^2/5000 choreography (makeGraph shards -> graph exchange -> metric
step depth), each rank emulated in turn, with the device-memory budget of one rank asserted.

BASELINE.json configs[4] runs makeGraph sharded over 8 MI355X and the metric step depth (a single search:
replicas only) on the whole graph.  Every rank therefore holds, at its peak, the
padded exchange buffer (world x the largest shard blob, filled by all_gather_into_tensor) and the assembled
graph (depthmapx_amd/sharded.py exchange_graph), plus the search's structures.  Here the 8 ranks' shards are
built one after another on one context (each blob parked on the host: a rank holds only its own shard), then
the padded buffer is filled as all_gather_into_tensor leaves it on every rank, so the device memory in use at
each phase end is a rank's:
  1. cost-balanced bounds (PointMap.shard_bounds), per-rank makeGraph -> its blob in its slot;
  2. assembly of the whole graph from the 8 blobs (the run count of the one-shot graph);
  3. metric step depth from the configs[4] cell on the assembled graph: bit-identical to the single-process
     run (itself pinned to the oracle's whole search at this size by test_gpu_scale.py).
The peak (torch.cuda.mem_get_info, libdmx's allocations included; cached blocks released between phases as
sharded.exchange_graph's caller does) must stay below 90 % of the device, and so must the analytic bound
world x max blob + assembled graph.  Reference path: vgametricdepth.cpp:23-92; bench.py --config 5."""
import os

import numpy as np
import pytest
import torch

import depthmapx_amd as dmx
from golden_io import GOLDEN, read_csv_lines

pytestmark = pytest.mark.gpu
W = 8


def _release():
    from depthmapx_amd import _native as N
    N.lib().dmx_release_cached_memory()
    torch.cuda.empty_cache()


def _in_use(dev):
    torch.cuda.synchronize(dev)
    free, total = torch.cuda.mem_get_info(dev)
    return total - free, total


def test_2000_sharded_choreography_fits_and_matches_single_run(ctx):
    import bench
    dev = torch.device("cuda", 0)
    lines = read_csv_lines(os.path.join(GOLDEN, "inputs", "syn2000_5000.csv"))
    pm = dmx.PointMap([0.0, 0.0, 1999.0, 1999.0], lines, 1.0)
    assert pm.make_points(0.5, 0.5)
    N = pm.info()["filled"]
    cell = bench.nearest_filled(pm, 1000.0, 1000.0)

    # the single-process run
    g1 = pm.make_graph(ctx)
    runs1 = g1.info()["nruns"]
    graph_bytes = g1.blob_size()
    ref = g1.metric_step_depth(cells=[cell])
    g1.close()
    _release()
    base, total = _in_use(dev)

    # 1. balanced bounds; each rank's shard -> its blob (kept on the host between the emulated ranks: a rank
    #    holds only its own shard, whose blob it writes into its slot of the exchange buffer)
    bounds = pm.shard_bounds(ctx, W)
    assert bounds[0] == 0 and bounds[-1] == N and bounds == pm.shard_bounds(ctx, W)
    sizes, blobs, shard_peak = [], [], 0
    for r in range(W):
        s = pm.make_graph(ctx, node_begin=bounds[r], node_end=bounds[r + 1])
        n = s.blob_size()
        t = torch.empty(n, dtype=torch.uint8, device=dev)
        s.write_blob_device(t.data_ptr(), n)
        shard_peak = max(shard_peak, _in_use(dev)[0])
        blobs.append(t.cpu())
        sizes.append(n)
        del t
        s.close()
        _release()
    mx = max(sizes)
    # a rank's peak: its shard next to the exchange buffer, or the buffer next to the assembled graph
    bound = max(shard_peak + W * mx, base + W * mx + graph_bytes)
    assert bound < 0.9 * total, (bound, total)
    flat = torch.empty(W * mx, dtype=torch.uint8, device=dev)
    for r in range(W):   # what all_gather_into_tensor leaves in every rank's buffer
        flat[r * mx:r * mx + sizes[r]].copy_(blobs[r].to(dev, non_blocking=False))
    del blobs
    peak = _in_use(dev)[0]

    # 2. assembly
    g = pm.assemble(ctx, [flat.data_ptr() + r * mx for r in range(W)], sizes)
    assert g.info()["nruns"] == runs1
    peak = max(peak, _in_use(dev)[0])
    del flat
    _release()

    # 3. the search on the assembled graph
    got = g.metric_step_depth(cells=[cell])
    peak = max(peak, _in_use(dev)[0])
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    g.close()
    _release()
    print("configs[4] one-rank budget: blobs max %.2f GB (spread %.1f %%), exchange buffer %.1f GB, graph %.1f GB, "
          "shard build peak %.1f GB, bound %.1f GB, peak in use after the build %.1f GB of %.1f GB (%.0f %%; %.1f GB "
          "before)" % (mx / 1e9, 100 * (mx / (sum(sizes) / W) - 1), W * mx / 1e9, graph_bytes / 1e9, shard_peak / 1e9,
                        bound / 1e9, peak / 1e9, total / 1e9, 100 * peak / total, base / 1e9))
    assert peak < 0.9 * total, (peak, total)
