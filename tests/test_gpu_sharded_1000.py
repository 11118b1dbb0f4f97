"""configs[3] on one GPU: the 8-rank (4 by default, below) sharded 1000^2 choreography of bench.py, each rank emulated
in turn.

BASELINE.json configs[3] shards the 1000^2 grid over 8 MI355X (per-GPU source-cell ranges + an
all-gather of the VGA columns).  A one-GPU box cannot run 8 processes' worth of device memory at once,
so the ranks run one after another on one context, through the same entry points bench.py's step()
calls on each rank (depthmapx_amd/sharded.py):
  1. makeGraph of the rank's contiguous node range (shard_range(N, r, 8)) -> its blob, written into
     the rank's slot of the padded exchange buffer (what all_gather_into_tensor fills over RCCL);
  2. assembly of the whole graph from the 8 blobs: byte-identical to the one-shot graph's blob;
  3. the VGA preparation split by node range (Graph.set_prep_shard): every rank's partial buffers are
     summed on the host call by call -- the in-process stand-in for the RCCL all-reduce, call k resolved
     in pass k over the ranks -- and the final graph receives the sums through the same callback;
  4. VGA global for each rank's interleaved source chunks (vga_nodes) into the shared [N][7] output
     (the row all-gather is pure data movement), which must be bit-identical to the single-process run.
Reference path: vgavisualglobal.cpp:23-216 (the single-process run is pinned to the oracle by
test_gpu_scale.py / test_gpu_parity.py); bench.py:286-337 (the choreography)."""
import os

import numpy as np
import pytest
import torch

import depthmapx_amd as dmx
from depthmapx_amd.sharded import device_view, shard_range, vga_nodes
from golden_io import GOLDEN, read_csv_lines

pytestmark = pytest.mark.gpu
# 8 ranks as configs[3] with DMX_SCALE_FULL=1; 4 by default, so that the driver's whole `-m gpu` run fits its 900 s
# limit (each rank re-assembles the whole graph once per all-reduce call of the emulated protocol; the protocol,
# the exchange and the per-rank source chunks are the same at any rank count; profiles/r6_gpu_scale_full.log)
W = 8 if os.environ.get("DMX_SCALE_FULL") == "1" else 4


def _release():
    from depthmapx_amd import _native as N
    N.lib().dmx_release_cached_memory()
    torch.cuda.empty_cache()


def _blob(g, dev):
    n = g.blob_size()
    t = torch.empty(n, dtype=torch.uint8, device=dev)
    g.write_blob_device(t.data_ptr(), n)
    return t


def test_1000_sharded_choreography_matches_single_run(ctx):
    dev = torch.device("cuda", 0)
    lines = read_csv_lines(os.path.join(GOLDEN, "inputs", "syn1000.csv"))
    pm = dmx.PointMap([0.0, 0.0, 1000.0, 1000.0], lines, 1.0)
    assert pm.make_points(0.5, 0.5)
    N = pm.info()["filled"]
    assert N == 998001

    # the single-process run: one-shot graph blob and VGA columns
    g1 = pm.make_graph(ctx)
    blob1 = _blob(g1, dev)
    ref = torch.full((N, 7), -1.0, dtype=torch.float32, device=dev)
    g1.vga_visual_global_device(ref.data_ptr())
    g1.close()
    _release()

    # 1. per-rank makeGraph shards into their slots of the padded exchange buffer
    ranges = [shard_range(N, r, W) for r in range(W)]
    shards = []
    for (b, e) in ranges:
        s = pm.make_graph(ctx, node_begin=b, node_end=e)
        shards.append((s, s.blob_size()))
    mx = max(n for _, n in shards)
    flat = torch.empty(W * mx, dtype=torch.uint8, device=dev)
    sizes = []
    for r, (s, n) in enumerate(shards):
        s.write_blob_device(flat.data_ptr() + r * mx, n)
        sizes.append(n)
        s.close()
    del shards
    _release()
    ptrs = [flat.data_ptr() + r * mx for r in range(W)]

    # 2. assembly == the one-shot graph, byte for byte
    g2 = pm.assemble(ctx, ptrs, sizes)
    blob2 = _blob(g2, dev)
    assert blob2.numel() == blob1.numel() and torch.equal(blob1, blob2)
    del blob1, blob2
    g2.close()
    _release()

    # 3. sharded preparation.  The all-reduce is a collective: a call returns only with the sum of every
    #    rank's partial buffer, and what a rank computes next may depend on it.  Emulated one rank at a
    #    time, call k is resolved in pass k: each rank replays the known sums of calls 0..k-1, hands in
    #    its partial for call k and stops there (the callback fails the preparation); the partials are
    #    summed on the host.  A pass in which no rank reaches call k ends the protocol.
    sums = []
    for k in range(16):
        reached = 0
        for r, (b, e) in enumerate(ranges):
            gr = pm.assemble(ctx, ptrs, sizes)
            calls = [0]

            def fn(ptr, count, dtype, k=k, calls=calls):
                i = calls[0]
                calls[0] += 1
                t = device_view(ptr, count, dtype, dev)
                if i < k:
                    assert t.numel() == sums[i].numel()
                    t.copy_(sums[i].to(dev))
                    torch.cuda.synchronize(dev)
                    return 0
                part = t.cpu()
                if len(sums) == k:
                    sums.append(part.clone())
                else:
                    assert sums[k].shape == part.shape and sums[k].dtype == part.dtype
                    sums[k] += part
                return -1                          # stop this rank's preparation at call k
            gr.set_prep_shard(b, e, fn)
            scratch = torch.empty((1, 7), dtype=torch.float32, device=dev)
            try:
                gr.vga_visual_global_device_list(scratch.data_ptr(), np.zeros(0, dtype=np.int64))
            except dmx.DmxError:
                pass
            reached += calls[0] > k
            gr.close()
            _release()
        assert reached in (0, W)                   # every rank makes the same calls
        if reached == 0:
            break
    ncalls = len(sums)
    assert ncalls >= 5                             # symmetry sums (2), veto, tile-visibility rows (2)

    # the final rank gets the sums through the callback, then every rank's sources run on its graph
    g = pm.assemble(ctx, ptrs, sizes)
    del flat
    served = [0]

    def apply(ptr, count, dtype):
        i = served[0]
        served[0] += 1
        t = device_view(ptr, count, dtype, dev)
        assert t.numel() == sums[i].numel()
        t.copy_(sums[i].to(dev))
        torch.cuda.synchronize(dev)
        return 0

    g.set_prep_shard(*ranges[0], apply)
    out = torch.full((N, 7), -1.0, dtype=torch.float32, device=dev)
    for r in range(W):
        g.vga_visual_global_device_list(out.data_ptr(), vga_nodes(N, r, W))
    assert served[0] == ncalls
    got = out.cpu().numpy()
    want = ref.cpu().numpy()
    assert (got[:, 5] > 0).all()
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    g.close()
    _release()
