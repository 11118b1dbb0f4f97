"""GPU parity at the benchmark sizes (BASELINE.json configs[2]/[3] 1000^2, configs[4] 2000^2/5000).

The oracle (oracle/dmx_oracle.c, pinned to the reference) cannot build these graphs whole in test
time, so the checks are seeded blocks and size-independent properties:
  * makeGraph (PointMap::sparkGraph2, salalib/pointdata.cpp:1246-1341): blocks of 64 sources --
    a corner, the middle, cells next to an occluder, seeded random blocks, and at 2000^2 the
    densest-occluder window (16 blocks) -- bin records, runs, the 3 float attributes and the grid
    connections bit-exact against OracleMap.make_graph on the same node range;
  * VGA global (VGAVisualGlobal::run, vgavisualglobal.cpp:23-216) at 1000^2: >= 256 sources targeted
    where the tile BFS's certificates could fail (asymmetric nodes and neighbours, occluder-adjacent
    cells, phase-C-heavy blocks, seeded random) against the oracle's BFS over the same graph (node
    counts exact, floats within 1e-6);
  * metric step depth at 2000^2/5000 (VGAMetricDepth::run, vgametricdepth.cpp:23-92): the
    whole-GPU batched search against the serial pop-order kernel (itself pinned to the reference
    fixtures at small sizes), bit-exact on every column, plus invariants of the result.
"""
import os

import numpy as np
import pytest

import depthmapx_amd as dmx
from golden_io import GOLDEN, read_csv_lines

pytestmark = pytest.mark.gpu

BLOCK = 64
FILLED, BLOCKED = 2, 4


def _blocks(pm, N, seed):
    """Node ranges: a corner, the middle, the node of an occluder-adjacent cell, a seeded random one."""
    st = pm.state()
    filled = np.nonzero(st & FILLED)[0]          # node k <-> cell filled[k] (x-major)
    blocked = np.nonzero(st & BLOCKED)[0]
    near = blocked[len(blocked) // 2]             # a cell on an occluder near the middle of the list
    k_near = min(max(0, int(np.searchsorted(filled, near)) - BLOCK // 2), N - BLOCK)
    rng = np.random.default_rng(seed)
    starts = [0, N // 2 - BLOCK // 2, k_near, int(rng.integers(0, N - BLOCK))]
    return [(b, b + BLOCK) for b in starts]


def _check_makegraph_blocks(pm, g, om, blocks, threads=16):
    for (b, e) in blocks:
        got = g.copy_range(b, e)
        om.make_graph(node_begin=b, node_end=e, threads=threads)
        ref = om.graph()
        rb = ref["bins"][b:e]
        off = np.concatenate([[0], np.cumsum(ref["bins"][:, :, 3].sum(axis=1))])
        rr = ref["runs"][off[b]:off[e]]
        np.testing.assert_array_equal(got["bins"], rb, err_msg="bins of nodes [%d,%d)" % (b, e))
        np.testing.assert_array_equal(got["runs"], rr, err_msg="runs of nodes [%d,%d)" % (b, e))
        np.testing.assert_array_equal(got["attrs"].view(np.uint32), ref["attrs"][b:e].view(np.uint32))
        np.testing.assert_array_equal(got["gridconn"], ref["gridconn"][b:e])
        assert got["bins"][:, :, 3].sum() > 0


def _ranges(nodes):
    """Sorted unique node indices as maximal contiguous [b, e) ranges."""
    nodes = np.unique(np.asarray(nodes, dtype=np.int64))
    if len(nodes) == 0:
        return []
    cut = np.nonzero(np.diff(nodes) != 1)[0] + 1
    return [(int(p[0]), int(p[-1]) + 1) for p in np.split(nodes, cut)]


def _check_makegraph_sample(g, om, nodes, threads=16):
    """Bins, runs and the 3 float attributes of every listed node bit-exact against the oracle's sparkPixel2
    of the same nodes (OracleMap.make_graph_sample: the node list only, 16 threads)."""
    nodes = np.unique(np.asarray(nodes, dtype=np.int64))
    om.make_graph_sample(nodes, threads=threads)
    ref = om.graph()
    off = np.concatenate([[0], np.cumsum(ref["bins"][:, :, 3].sum(axis=1))])
    for (b, e) in _ranges(nodes):
        got = g.copy_range(b, e)
        np.testing.assert_array_equal(got["bins"], ref["bins"][b:e], err_msg="bins of nodes [%d,%d)" % (b, e))
        np.testing.assert_array_equal(got["runs"], ref["runs"][off[b]:off[e]], err_msg="runs of nodes [%d,%d)" % (b, e))
        np.testing.assert_array_equal(got["attrs"].view(np.uint32), ref["attrs"][b:e].view(np.uint32),
                                      err_msg="attributes of nodes [%d,%d)" % (b, e))
    return len(nodes)


def _mk_wide_sample(N, nblocks, seed, reruns):
    """nblocks blocks of 64 sources spread over the map (seeded) plus every source the whole-map build
    re-ran (moment certificate or capacity): the paths whose bit-exactness rests on a certificate."""
    rng = np.random.default_rng(seed)
    starts = np.unique(np.concatenate([np.linspace(0, N - BLOCK, nblocks // 2).astype(np.int64),
                                       rng.integers(0, N - BLOCK, size=nblocks - nblocks // 2)]))
    blocks = np.concatenate([np.arange(b, b + BLOCK) for b in starts])
    return np.unique(np.concatenate([blocks] + [np.asarray(r, dtype=np.int64) for r in reruns])), len(starts)


def _release(ctx, *objs):
    for o in objs:
        o.close()
    import ctypes  # noqa: F401
    from depthmapx_amd import _native as N
    N.lib().dmx_release_cached_memory()


# The driver's round-end `-m gpu` run has a 900 s limit for the whole suite: by default the oracle samples below
# are sized to fit it (the oracle's BFS is ~8.7 s of CPU a source at 1000^2, ~30 s at 2000^2, on 16 threads of the
# box); DMX_SCALE_FULL=1 runs the larger samples of earlier rounds (>= 256 targeted sources at 1000^2, 64 at
# 2000^2, the serial step-depth kernel at 2000^2), whose logs are under profiles/.
FULL = os.environ.get("DMX_SCALE_FULL") == "1"

# module-scoped graphs still alive; the 2000^2 fixture closes the 1000^2 one first (the 1000^2 tests come first in
# this file): its ~90 GB would otherwise leave no room for the 2000^2 partial-tile masks
_LIVE = {}


@pytest.fixture(scope="module")
def big1000(ctx):
    from pyoracle import OracleMap
    lines = read_csv_lines(os.path.join(GOLDEN, "inputs", "syn1000.csv"))
    region = [0.0, 0.0, 1000.0, 1000.0]
    pm = dmx.PointMap(region, lines, 1.0)
    assert pm.make_points(0.5, 0.5)
    g = pm.make_graph(ctx)
    g.reruns = ctx.last_mk_reruns()
    om = OracleMap(region, 1.0, lines)
    assert om.fill(0.5, 0.5)
    _LIVE["1000"] = g
    yield pm, g, om
    if _LIVE.pop("1000", None) is not None:
        _release(ctx, g)


def test_1000_makegraph_blocks_match_oracle(big1000):
    """configs[2]: 1001^2 cells, 50 occluders.  Node count, run total and 4 blocks bit-exact."""
    pm, g, om = big1000
    info = g.info()
    assert info["nnodes"] == pm.info()["filled"] == 998001
    np.testing.assert_array_equal(pm.state(), om.state())
    _check_makegraph_blocks(pm, g, om, _blocks(pm, info["nnodes"], seed=1000))


def test_1000_makegraph_wide_sample_matches_oracle(big1000):
    """configs[2] makeGraph on >= 8,192 sources (128 spread blocks of 64) plus every source the whole-map build
    swept again -- the ~0.4 % whose certified moment sums straddled a float rounding and any capacity
    re-runs -- bit-exact against the oracle (~0.8 ms a source on 16 threads)."""
    pm, g, om = big1000
    N = g.info()["nnodes"]
    cert, cap = g.reruns
    assert len(cert) > 0, "the whole-map build took no certificate re-run"
    nodes, nb = _mk_wide_sample(N, 128, 1001, [cert, cap])
    assert nb * BLOCK >= 8192
    n = _check_makegraph_sample(g, om, nodes)
    print("1000^2 makeGraph sample: %d sources (%d certificate re-runs, %d capacity re-runs)" % (n, len(cert), len(cap)))


def _digests_or_skip(name):
    path = os.path.join(GOLDEN, "digests", "mk_%s.npz" % name)
    if not os.path.exists(path):
        pytest.skip("no whole-map digests at %s (tests/golden/gen_mk_digests.py --map %s)" % (path, name))
    return path


def test_1000_makegraph_whole_map_matches_oracle_digests(big1000):
    """configs[2] makeGraph on EVERY source: each 64-node block's bins, runs, attributes and grid connections
    hashed (tests/mk_digest.py) against the pinned oracle's whole-map sweep (tests/golden/gen_mk_digests.py,
    oracle/dmx_oracle.c sparkGraph2 + addGridConnections over all 998,001 sources)."""
    from mk_digest import check_whole_map
    pm, g, om = big1000
    N = g.info()["nnodes"]
    n = check_whole_map(g, _digests_or_skip("1000"), N)
    print("1000^2 makeGraph: all %d blocks of 64 nodes equal the oracle's" % n)


def _neighbour_nodes(pm, cells, N):
    """Nodes of the filled 8-neighbours of the given cells."""
    st = pm.state()
    rows, cols = pm.rows, pm.cols
    filled = np.nonzero(st & FILLED)[0]
    out = set()
    for c in cells:
        x, y = divmod(int(c), rows)
        for dx in (-1, 0, 1):
            for dy in (-1, 0, 1):
                if (dx or dy) and 0 <= x + dx < cols and 0 <= y + dy < rows:
                    cc = (x + dx) * rows + y + dy
                    if st[cc] & FILLED:
                        out.add(int(np.searchsorted(filled, cc)))
    return sorted(out)


def _vga_targeted_sources(pm, g, ctx, N, total):
    """Sources where the tile BFS's certificates could fail (VERDICT r3 'do this' 2), in 4 equal groups of
    total / 4 (total 96 by default, 256 with DMX_SCALE_FULL=1):
      - the asymmetric (special) nodes and their neighbours (exact in-set corrections);
      - sources on cells next to an occluder (partly seen tiles, masks);
      - the spread blocks whose BFS sends the most cells to phase C (the mask test);
      - seeded random sources to the total and beyond."""
    q = total // 4
    rng = np.random.default_rng(1000)
    st = pm.state()
    filled = np.nonzero(st & FILLED)[0]
    special = [int(k) for k in g.special_nodes()]
    picks = special[:q // 2]
    picks += _neighbour_nodes(pm, [filled[k] for k in special[:q // 2]], N)[:q - len(picks)]
    near = np.nonzero(((st & FILLED) != 0) & ((st & BLOCKED) != 0))[0]
    adj = _neighbour_nodes(pm, rng.choice(near, size=min(len(near), 200), replace=False), N)
    picks += [int(v) for v in rng.choice(adj, size=q, replace=False)]
    # phase-C-heavy: 96 spread blocks of 32 sources, the q / 32 with the most phase-C cells
    heavy = []
    for b in np.linspace(0, N - 32, 96).astype(int):
        g.vga_visual_global(src_begin=int(b), src_end=int(b) + 32)
        heavy.append((ctx.last_stats()["vga_hard_cells"], int(b)))
    heavy.sort(reverse=True)
    for _, b in heavy[:max(1, q // 32)]:
        picks += list(range(b, b + 32))
    picks = sorted(set(picks))
    picks += [int(v) for v in rng.choice(N, size=max(0, total - len(picks)) + q // 2, replace=False)]
    return np.array(sorted(set(picks)), dtype=np.int64), special


def test_1000_vga_targeted_sources_match_oracle(big1000, ctx):
    """configs[2] VGA global against the oracle's BFS over the same graph (the GPU graph copied to the
    host; its makeGraph blocks are pinned by the test above) on >= 96 targeted sources (>= 256 with
    DMX_SCALE_FULL=1; profiles/r6_gpu_scale_full.log): node counts and
    level sums exact, floats within 1e-6.  The sample must exercise every path of the tile BFS: tiles
    resolved by common runs (phase A), head and hint tests (B), hard cells (C), partial-tile masks, and --
    where the graph has asymmetric nodes -- the special-node corrections."""
    import torch
    pm, g, om = big1000
    N = g.info()["nnodes"]
    total = 256 if FULL else 96
    src, special = _vga_targeted_sources(pm, g, ctx, N, total)
    assert len(src) >= total
    out = torch.full((N, 7), -1.0, dtype=torch.float32, device="cuda:0")
    g.vga_visual_global_device_list(out.data_ptr(), src)
    torch.cuda.synchronize()
    st = ctx.last_stats()
    cyc = ctx.last_phase_cycles()
    assert st["vga_kernel"] == "tile-resolved"
    assert cyc["tile_common"] > 0 and cyc["heads"] > 0 and cyc["hard"] > 0, cyc   # phases A, B, C ran
    assert st["vga_cr_tiles"] > 0 and st["vga_hard_cells"] > 0 and st["vga_pmask_cells"] > 0, st
    if special:
        assert st["vga_n_spec"] > 0, st                      # special-node tests in phase C
    got = out.cpu().numpy()[src].astype(np.float64)
    del out
    full = g.copy(runs=True)
    om.set_graph_view(full["bins"], full["runs"])
    ref, _ = om.vga_global_sample(src, threads=16)
    want = ref[src].astype(np.float64)
    del full
    np.testing.assert_array_equal(got[:, 5], want[:, 5])            # node count: exact
    assert (np.abs(got - want) <= 1e-6 * np.maximum(1.0, np.abs(want))).all()
    print("targeted VGA sample: %d sources (%d special nodes in the graph), stats %s" % (len(src), len(special), st))


def _spread_blocks(N, n, size, seed):
    rng = np.random.default_rng(seed)
    starts = sorted(set([0, N - size] + [int(v) for v in rng.integers(0, N - size, size=n - 2)]))
    return [(b, b + size) for b in starts]


def test_1000_vga_kernels_agree_at_size(big1000, ctx, monkeypatch):
    """The tile-resolved BFS (line summaries, tile-visibility rows, partial-tile masks) against the
    direction-optimising kernel, which shares none of those certificates, bit-for-bit on 4 blocks of
    256 sources spread over the map (the direction-optimising kernel keeps its bitmaps in HBM at this
    size: ~100 sources/s, so the wide sample is the run-scan comparison below)."""
    pm, g, om = big1000
    N = g.info()["nnodes"]
    blocks = _spread_blocks(N, 4, 256, seed=31)
    a = [g.vga_visual_global(src_begin=b, src_end=e) for (b, e) in blocks]
    st = ctx.last_stats()
    assert st["vga_kernel"] == "tile-resolved"
    monkeypatch.setenv("DMX_VGA_KERNEL", "do")
    g2 = pm.make_graph(ctx)
    for (b, e), ai in zip(blocks, a):
        c = g2.vga_visual_global(src_begin=b, src_end=e)
        np.testing.assert_array_equal(ai[b:e].view(np.uint32), c[b:e].view(np.uint32), err_msg="sources [%d,%d)" % (b, e))
    _release(ctx, g2)


def test_1000_vga_partial_tile_masks_agree_with_run_scan(big1000, ctx, monkeypatch):
    """Phase C's exact partial-tile-mask test (default) against its run scan (DMX_VGA_PMASK=0, a
    launch-time switch on the same graph), bit-for-bit on 16 blocks of 8192 sources (131,072 sources,
    13 % of the map: the rare-cell cases the certificates could hide show up here before they show up
    in a 32-source oracle block); the masks must have decided cells on these blocks."""
    pm, g, om = big1000
    N = g.info()["nnodes"]
    blocks = _spread_blocks(N, 16, 8192, seed=32)
    a, used = [], 0
    for (b, e) in blocks:
        a.append(g.vga_visual_global(src_begin=b, src_end=e))
        used += ctx.last_stats()["vga_pmask_cells"]
    assert used > 0
    monkeypatch.setenv("DMX_VGA_PMASK", "0")
    for (b, e), ai in zip(blocks, a):
        c = g.vga_visual_global(src_begin=b, src_end=e)
        assert ctx.last_stats()["vga_pmask_cells"] == 0
        np.testing.assert_array_equal(ai[b:e].view(np.uint32), c[b:e].view(np.uint32), err_msg="sources [%d,%d)" % (b, e))


def test_1000_vga_per_tile_summary_path_agrees(big1000, ctx, monkeypatch):
    """The coarser per-tile frontier summary (what grids above ~1010^2 use when the line-resolved
    summaries no longer fit the LDS), forced at 1000^2 with DMX_VGA_RB=0: bit-identical to the
    default line-summary run on a block of 256 sources."""
    pm, g, om = big1000
    N = g.info()["nnodes"]
    b, e = 2 * N // 3, 2 * N // 3 + 256
    a = g.vga_visual_global(src_begin=b, src_end=e)
    monkeypatch.setenv("DMX_VGA_RB", "0")
    c = g.vga_visual_global(src_begin=b, src_end=e)
    np.testing.assert_array_equal(a[b:e].view(np.uint32), c[b:e].view(np.uint32))


@pytest.fixture(scope="module")
def big2000(ctx):
    g1000 = _LIVE.pop("1000", None)
    if g1000 is not None:
        _release(ctx, g1000)
    from pyoracle import OracleMap
    lines = read_csv_lines(os.path.join(GOLDEN, "inputs", "syn2000_5000.csv"))
    region = [0.0, 0.0, 1999.0, 1999.0]
    pm = dmx.PointMap(region, lines, 1.0)
    assert pm.make_points(0.5, 0.5)
    g = pm.make_graph(ctx)
    g.reruns = ctx.last_mk_reruns()
    om = OracleMap(region, 1.0, lines)
    assert om.fill(0.5, 0.5)
    yield pm, g, om
    _release(ctx, g)


def _densest_block(pm, N, win=64):
    """The 64-node block centred on the cell whose win x win window holds the most blocked cells."""
    st = pm.state()
    cols, rows = pm.cols, pm.rows
    blk = ((st & BLOCKED) != 0).reshape(cols, rows).astype(np.int64)
    ii = np.zeros((cols + 1, rows + 1), dtype=np.int64)
    ii[1:, 1:] = blk.cumsum(0).cumsum(1)
    dens = ii[win:, win:] - ii[:-win, win:] - ii[win:, :-win] + ii[:-win, :-win]
    x, y = np.unravel_index(int(np.argmax(dens)), dens.shape)
    cx, cy = x + win // 2, y + win // 2
    filled = np.nonzero(st & FILLED)[0]
    k = int(np.searchsorted(filled, cx * rows + cy))
    k = min(max(0, k - BLOCK // 2), N - BLOCK)
    return (k, k + BLOCK), int(dens.max())


def test_2000_makegraph_blocks_match_oracle(big2000):
    """configs[4]: 2000^2 cells, 5000 short occluders (dense): 16 blocks of 64 sources bit-exact -- the
    corner, the middle, an occluder cell, the densest-occluder window (most blocked cells in 64 x 64) and
    12 seeded random blocks."""
    pm, g, om = big2000
    info = g.info()
    N = info["nnodes"]
    assert N == pm.info()["filled"]
    assert N > 3_900_000
    np.testing.assert_array_equal(pm.state(), om.state())
    blocks = _blocks(pm, N, seed=2000)
    dense, nblocked = _densest_block(pm, N)
    assert nblocked > 100
    blocks.append(dense)
    rng = np.random.default_rng(2001)
    blocks += [(int(b), int(b) + BLOCK) for b in rng.integers(0, N - BLOCK, size=16 - len(blocks))]
    assert len(blocks) == 16
    _check_makegraph_blocks(pm, g, om, blocks)


def test_2000_makegraph_wide_sample_matches_oracle(big2000):
    """configs[4] makeGraph on >= 4,096 sources (64 spread blocks of 64) plus every source the whole-map build
    swept again (moment certificate, capacity), bit-exact against the oracle."""
    pm, g, om = big2000
    N = g.info()["nnodes"]
    cert, cap = g.reruns
    assert len(cert) > 0, "the whole-map build took no certificate re-run"
    nodes, nb = _mk_wide_sample(N, 64, 2002, [cert, cap])
    assert nb * BLOCK >= 4096
    n = _check_makegraph_sample(g, om, nodes)
    print("2000^2 makeGraph sample: %d sources (%d certificate re-runs, %d capacity re-runs)" % (n, len(cert), len(cap)))


def test_2000_makegraph_whole_map_matches_oracle_digests(big2000):
    """configs[4] makeGraph on EVERY source (3,991,912): every 64-node block against the oracle's whole-map
    digests."""
    from mk_digest import check_whole_map
    pm, g, om = big2000
    N = g.info()["nnodes"]
    n = check_whole_map(g, _digests_or_skip("2000"), N)
    print("2000^2 makeGraph: all %d blocks of 64 nodes equal the oracle's" % n)


def test_2000_metric_stepdepth_batched_equals_serial(big2000, ctx, monkeypatch):
    """configs[4] step depth from the cell nearest the centre: the result's invariants (every reached cell's
    length >= its straight-line distance; the selected cell at 0), and with DMX_SCALE_FULL=1 batched == serial on
    every column with the expander count and relaxations identical (the serial kernel takes ~40 s here; batched ==
    serial is checked on every small map in test_gpu_parity.py)."""
    import bench
    pm, g, om = big2000
    cell = bench.nearest_filled(pm, 1000.0, 1000.0)
    monkeypatch.delenv("DMX_SD_KERNEL", raising=False)
    a = g.metric_step_depth(cells=[cell])
    sa = ctx.last_stepdepth()
    assert sa["mode"] == "batched"
    if FULL:
        monkeypatch.setenv("DMX_SD_KERNEL", "serial")
        b = g.metric_step_depth(cells=[cell])
        sb = ctx.last_stepdepth()
        assert sb["mode"] == "serial"
        assert (sa["expanders_popped"], sa["cells_relaxed"]) == (sb["expanders_popped"], sb["cells_relaxed"])
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    reached = a[:, 1] >= 0
    assert reached.mean() > 0.99
    assert (a[reached, 1] >= a[reached, 2] * (1 - 1e-6)).all()
    st = pm.state()
    k_sel = int(np.searchsorted(np.nonzero(st & FILLED)[0], cell))
    assert a[k_sel, 1] == 0.0 and a[k_sel, 2] == 0.0


def test_2000_vga_sources_match_oracle(big2000, ctx):
    """configs[4] grid (2000^2, above the 1024^2 that an LDS frontier holds): the tile BFS with its frontier in
    HBM and its line summaries in LDS, on seeded sources -- a block in the middle of the map, one next to the
    densest occluders and random ones -- against the oracle's BFS over the same graph (node count exact,
    floats within 1e-6).  16 sources (64 with DMX_SCALE_FULL=1: one oracle BFS is ~30 s of CPU here)."""
    import torch
    pm, g, om = big2000
    N = g.info()["nnodes"]
    n = 64 if FULL else 16
    rng = np.random.default_rng(2000)
    (db, _), _ = _densest_block(pm, N)
    fixed = [N // 2, N // 2 + 1, db, db + 1]
    src = sorted(set(fixed + [int(v) for v in rng.integers(0, N, size=n - len(fixed))]))
    src = np.array(src, dtype=np.int64)
    out = torch.full((N, 7), -1.0, dtype=torch.float32, device="cuda:0")
    g.vga_visual_global_device_list(out.data_ptr(), src)
    torch.cuda.synchronize()
    st = ctx.last_stats()
    assert st["vga_kernel"] == "tile-resolved" and st["vga_frontier_hbm"] == 1, st
    got = out.cpu().numpy()[src].astype(np.float64)
    del out
    full = g.copy(runs=True)
    om.set_graph_view(full["bins"], full["runs"])
    ref, _ = om.vga_global_sample(src, threads=16)
    want = ref[src].astype(np.float64)
    del full
    np.testing.assert_array_equal(got[:, 5], want[:, 5])
    assert (np.abs(got - want) <= 1e-6 * np.maximum(1.0, np.abs(want))).all()
    assert (want[:, 5] > 0.5 * N).all()
    # the wide-grid partial-tile masks (in the scan order's place at this size) were built and decided cells: the
    # path behind the bench's 2000^2 figure (the fixture closed the 1000^2 graph to leave them room)
    assert st["vga_pmask_bytes"] > 0 and st["vga_pmask_cells"] > 0, st
    assert st["vga_scan_released"] == 1, st
    print("2000^2 VGA: partial-tile masks %.1f GB, %d cells decided by them" % (st["vga_pmask_bytes"] / 1e9,
                                                                              st["vga_pmask_cells"]))


def test_2000_vga_masks_release_restore_and_recover(big2000, ctx, monkeypatch):
    """Above 1024^2 the partial-tile masks take the scan order's memory (prepare_pmask releases it and the tile
    search reads runs in pool order); the direction-optimising kernel reads the scan order itself, so a vga_do
    call frees the tile data and rebuilds it (restore_scan_order), and the next tile call builds the masks
    again.  A preparation that fails after the release (a test hook injects it) leaves the graph usable: the next
    tile search rebuilds the scan order and the tile data (a second call used to read the released
    scan order).  All answers on the same sources are bit-identical."""
    from depthmapx_amd._native import DmxError
    pm, g, om = big2000
    N = g.info()["nnodes"]
    s0 = N // 3   # (the source-range entry point honours DMX_VGA_KERNEL; the list entry point takes the tile path)

    def run(n=4):
        out = g.vga_visual_global(src_begin=s0, src_end=s0 + n)
        return out[s0:s0 + n].copy(), ctx.last_stats()

    a, st_a = run()
    assert st_a["vga_pmask_bytes"] > 0, st_a
    assert st_a["vga_kernel"] == "tile-resolved" and st_a["vga_pmask_cells"] > 0, st_a
    monkeypatch.setenv("DMX_VGA_KERNEL", "do")
    b, st_b = run(4 if FULL else 1)   # (the direction-optimising kernel with its bitmaps in HBM: ~20 s a source here)
    assert st_b["vga_kernel"] != "tile-resolved", st_b
    monkeypatch.delenv("DMX_VGA_KERNEL")
    # the next tile preparation releases the scan order again and then fails: the call raises
    monkeypatch.setenv("DMX_VGA_PMASK_FAIL", "1")
    with pytest.raises(DmxError):
        run()
    monkeypatch.delenv("DMX_VGA_PMASK_FAIL")
    c, st_c = run()
    assert st_c["vga_kernel"] == "tile-resolved" and st_c["vga_pmask_cells"] > 0, st_c
    np.testing.assert_array_equal(a[:len(b)].view(np.uint32), b.view(np.uint32))
    np.testing.assert_array_equal(a.view(np.uint32), c.view(np.uint32))
    # phase B past the heads (DMX_VGA_BEXT) while the runs are read in pool order: only the heads are tested
    # there, so the answer stays the same (positions past the heads are not scan order then)
    monkeypatch.setenv("DMX_VGA_BEXT", "4")
    d, st_d = run()
    assert st_d["vga_scan_released"] == 1, st_d
    np.testing.assert_array_equal(a.view(np.uint32), d.view(np.uint32))
    monkeypatch.delenv("DMX_VGA_BEXT")


def test_2000_metric_stepdepth_matches_oracle(big2000, ctx):
    """configs[4] step depth at size against the pinned oracle: the C restatement's std::set search
    (oracle/dmx_oracle.c metric_search, vgametricdepth.cpp:23-92) over the same 2000^2 graph from the
    same cell.  Lengths and straight-line distances bit-exact, angles within 1e-6 (north_star)."""
    import time
    import bench
    pm, g, om = big2000
    cell = bench.nearest_filled(pm, 1000.0, 1000.0)
    a = g.metric_step_depth(cells=[cell])
    assert ctx.last_stepdepth()["mode"] == "batched"
    if getattr(om, "_borrowed", None) is None:
        full = g.copy(runs=True)
        om.set_graph_view(full["bins"], full["runs"])
        del full
    t0 = time.perf_counter()
    ref = om.metric_stepdepth([cell])
    print("oracle metric step depth at 2000^2/5000: %.1f s" % (time.perf_counter() - t0))
    np.testing.assert_array_equal(a[:, 1:].view(np.uint32), ref[:, 1:].view(np.uint32))
    reached = ref[:, 1] >= 0
    assert reached.mean() > 0.99
    ga, ra = a[reached, 0], ref[reached, 0]
    # acos of a rounded cosine above 1 is NaN in the reference too (pixelref.h:121-131)
    assert np.array_equal(np.isnan(ga), np.isnan(ra)), (int(np.isnan(ga).sum()), int(np.isnan(ra).sum()))
    fin = ~np.isnan(ra)
    bad = ~np.isclose(ga[fin], ra[fin], rtol=1e-6, atol=1e-6)
    assert not bad.any(), (int(bad.sum()), float(np.abs(ga[fin] - ra[fin]).max()))
    np.testing.assert_array_equal(a[~reached], ref[~reached])
