"""Per-block digests of a makeGraph result (VERDICT r5 'do this' 2): the whole map pinned, not a sample.

A block is 64 consecutive nodes in x-major node order (the reference's attribute-row order).  Its digest
is the first 8 bytes (little-endian u64) of SHA-256 over, in this order:
  * the Bin headers   int32 [64][32][4]  (dir, count, far-distance float bits, run count) -- ngraph.h:48-60
  * the runs          int16 [R][4]       (x0, y0, x1, y1 of every PixelVec, bins 0..31 in Bin::make order)
  * the attributes    float32 bits [64][3] (Connectivity, Point First Moment, Point Second Moment)
  * addGridConnections u8 [64]          (pointdata.cpp:1735-1768)
exactly the arrays `OracleMap.make_graph_range` and `Graph.copy_range` return for those nodes.  The last
block of a map may hold fewer than 64 nodes.

Used by tests/golden/gen_mk_digests.py (the oracle, in the build container) and tests/test_gpu_digest.py
(the GPU graph).  Test infrastructure only.
"""
import hashlib

import numpy as np

BLOCK = 64


def _digest(bins, runs, attrs, gc):
    h = hashlib.sha256()
    h.update(bins.tobytes())
    h.update(runs.tobytes())
    h.update(attrs.tobytes())
    h.update(gc.tobytes())
    return np.frombuffer(h.digest()[:8], dtype="<u8")[0]


def block_digests(g, node_begin, pool=None):
    """Digests and run counts of the 64-node blocks of a node-range copy g (node_begin a multiple of BLOCK);
    pool: an optional concurrent.futures executor (hashlib releases the GIL on large buffers)."""
    assert node_begin % BLOCK == 0
    bins = np.ascontiguousarray(g["bins"], dtype="<i4")
    runs = np.ascontiguousarray(g["runs"], dtype="<i2")
    attrs = np.ascontiguousarray(g["attrs"], dtype=np.float32).view("<u4")
    gc = np.ascontiguousarray(g["gridconn"], dtype=np.uint8)
    n = bins.shape[0]
    per_node = bins[:, :, 3].astype(np.int64).sum(axis=1)
    off = np.concatenate([[0], np.cumsum(per_node)])
    assert off[-1] == runs.shape[0], (off[-1], runs.shape)
    nb = (n + BLOCK - 1) // BLOCK
    dig = np.zeros(nb, dtype=np.uint64)
    nr = np.zeros(nb, dtype=np.int64)
    args = []
    for i in range(nb):
        b, e = i * BLOCK, min(n, (i + 1) * BLOCK)
        args.append((bins[b:e], runs[off[b]:off[e]], attrs[b:e], gc[b:e]))
        nr[i] = off[e] - off[b]
    if pool is None:
        for i, a in enumerate(args):
            dig[i] = _digest(*a)
    else:
        for i, d in enumerate(pool.map(lambda a: _digest(*a), args)):
            dig[i] = d
    return dig, nr


def check_whole_map(g, path, N, chunk=65536, threads=16):
    """Every 64-node block of graph g (Graph.copy_range) against the committed digests at `path`; raises
    AssertionError naming the first mismatching block.  Returns the number of blocks checked."""
    from concurrent.futures import ThreadPoolExecutor
    z = np.load(path, allow_pickle=False)
    assert int(z["nnodes"]) == N, (int(z["nnodes"]), N)
    want, want_nr = z["digest"], z["nruns"]
    checked = 0
    with ThreadPoolExecutor(threads) as ex:
        for b in range(0, N, chunk):
            e = min(N, b + chunk)
            d, r = block_digests(g.copy_range(b, e), b, ex)
            i0 = b // BLOCK
            bad = np.nonzero((d != want[i0:i0 + len(d)]) | (r != want_nr[i0:i0 + len(r)]))[0]
            if len(bad):
                k = int(bad[0])
                raise AssertionError("block %d (nodes %d..%d): %d runs, digest %016x; expected %d runs, %016x (%d blocks differ "
                                     "in nodes %d..%d)" % (i0 + k, (i0 + k) * BLOCK, min(N, (i0 + k + 1) * BLOCK) - 1,
                                                           r[k], d[k], want_nr[i0 + k], want[i0 + k], len(bad), b, e - 1))
            checked += len(d)
    return checked
