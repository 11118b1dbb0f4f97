"""GPU parity: the HIP makeGraph / VGA-global path against (a) the golden fixtures produced by the
real reference (oracle/_ref/ref_probe) and (b) the C restatement (oracle/) on seeded inputs.

Bar: bit-exact for everything integer (states, bins, run lists, node counts, grid connections) and
for the makeGraph float attributes; VGA float measures within 1e-6 relative (north_star), with the
bit-exact fraction asserted separately to catch silent drift."""
import os

import numpy as np
import pytest

import depthmapx_amd as dmx
from golden_io import case_input_lines, load_case, node_digests

HERE = os.path.dirname(os.path.abspath(__file__))

pytestmark = pytest.mark.gpu

MK_CASES = ["kat", "syn16", "syn32", "gallery", "syn64", "barnsbury", "syn256mk"]
VGA_CASES = ["kat", "syn16", "syn32", "gallery", "syn64", "barnsbury", "syn128"]
VGA_RTOL = 1e-6


def _map(meta):
    pm = dmx.PointMap(meta["region"], case_input_lines(meta), meta["spacing"])
    for f in meta["fills"]:
        assert pm.make_points(*f)
    return pm


def _assert_graph_equal(got, A, runs_full):
    if "bins" in A:
        np.testing.assert_array_equal(got["bins"], A["bins"])
    np.testing.assert_array_equal(got["bins"][:, :, 3].sum(axis=1), A["nruns"] if "nruns" in A else A["bins"][:, :, 3].sum(axis=1))
    np.testing.assert_array_equal(got["attrs"].view(np.uint32), A["attrs"].view(np.uint32))
    np.testing.assert_array_equal(got["gridconn"], A["gridconn"])
    if runs_full:
        np.testing.assert_array_equal(got["runs"], A["runs"])
    np.testing.assert_array_equal(node_digests(got["bins"], got["runs"]), A["digests"])


def _assert_vga_close(got, want):
    want = want.astype(np.float64)
    got = got.astype(np.float64)
    tol = VGA_RTOL * np.maximum(1.0, np.abs(want))
    bad = np.abs(got - want) > tol
    assert not bad.any(), "VGA mismatch at %d cells, first %s" % (bad.sum(), np.argwhere(bad)[:5].tolist())
    return float((got == want).mean())


@pytest.mark.parametrize("name", MK_CASES)
def test_makegraph_matches_reference(ctx, name):
    try:
        meta, A = load_case(name)
    except FileNotFoundError:
        pytest.skip("fixture not generated")
    pm = _map(meta)
    np.testing.assert_array_equal(pm.state(), A["state"])
    g = pm.make_graph(ctx)
    info = g.info()
    assert info["nnodes"] == meta["nodes"]
    assert info["nruns"] == meta["runs"]
    got = g.copy(runs=True)
    _assert_graph_equal(got, A, meta["full_runs"])


@pytest.mark.parametrize("name", VGA_CASES)
def test_vga_global_matches_reference(ctx, name):
    try:
        meta, A = load_case(name)
    except FileNotFoundError:
        pytest.skip("fixture not generated")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    out = g.vga_visual_global(radius=-1)
    exact = _assert_vga_close(out, A["vga"])
    # integer columns (node count) must be bit-exact; floats nearly always are
    np.testing.assert_array_equal(out[:, 5], A["vga"][:, 5])
    assert exact > 0.99


def test_vga_levels_match_oracle(ctx):
    from pyoracle import OracleMap
    meta, A = load_case("syn32")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    out, lv = g.vga_visual_global(levels=True)
    om = OracleMap(meta["region"], meta["spacing"], case_input_lines(meta))
    for f in meta["fills"]:
        om.fill(*f)
    om.make_graph()
    ref, rlv = om.vga_global(levels=True)
    np.testing.assert_array_equal(lv[:, :2], rlv[:, :2])
    _assert_vga_close(out, ref)


@pytest.mark.parametrize("seed", [3, 7, 11])
def test_random_occluders_match_oracle(ctx, seed):
    """Seeded random drawings (dense short occluders -> many gaps/blocks per depth)."""
    from pyoracle import OracleMap
    from golden.gen_synthetic import make_lines
    W = 40
    lines = np.array(make_lines(W, 60, seed=seed, lmin=0.02, lmax=0.3), dtype=np.float64)
    region = [0.0, 0.0, float(W), float(W)]
    pm = dmx.PointMap(region, lines, 1.0)
    om = OracleMap(region, 1.0, lines)
    assert pm.make_points(0.5, 0.5) == om.fill(0.5, 0.5)
    np.testing.assert_array_equal(pm.state(), om.state())
    g = pm.make_graph(ctx)
    om.make_graph(threads=8)
    ref = om.graph()
    got = g.copy(runs=True)
    np.testing.assert_array_equal(got["bins"], ref["bins"])
    np.testing.assert_array_equal(got["runs"], ref["runs"])
    np.testing.assert_array_equal(got["attrs"].view(np.uint32), ref["attrs"].view(np.uint32))
    np.testing.assert_array_equal(got["gridconn"], ref["gridconn"])
    _assert_vga_close(g.vga_visual_global(), om.vga_global(threads=8))


@pytest.mark.parametrize("shape", [(1300, 5), (6, 1300)])
def test_far_rows_past_lds_match_oracle(ctx, shape):
    """Sight lines longer than 1024 cells: the open-run state of rows past MK_OPEN_LDS lives in scratch
    memory (makegraph.hip).  A long narrow corridor with a few occluders, both orientations (rows are
    x-rows in the horizontal octants, y-rows in the vertical ones)."""
    from pyoracle import OracleMap
    W, H = shape
    rng = np.random.default_rng(5)
    lines = []
    for _ in range(6):
        x = rng.uniform(0.1, 0.9) * W
        y = rng.uniform(0.1, 0.9) * H
        lines.append([x, y, x + (0.7 if W > H else 0.3), y + (0.3 if W > H else 0.7)])
    lines = np.array(lines, dtype=np.float64)
    region = [0.0, 0.0, float(W), float(H)]
    pm = dmx.PointMap(region, lines, 1.0)
    om = OracleMap(region, 1.0, lines)
    assert pm.make_points(0.5, 0.5) == om.fill(0.5, 0.5)
    g = pm.make_graph(ctx)
    om.make_graph(threads=8)
    ref = om.graph()
    got = g.copy(runs=True)
    np.testing.assert_array_equal(got["bins"], ref["bins"])
    np.testing.assert_array_equal(got["runs"], ref["runs"])
    np.testing.assert_array_equal(got["attrs"].view(np.uint32), ref["attrs"].view(np.uint32))
    assert int(np.abs(got["runs"][:, 0].astype(np.int64) - got["runs"][:, 2]).max()) > 1024 or \
        int(np.abs(got["runs"][:, 1].astype(np.int64) - got["runs"][:, 3]).max()) > 1024


def test_maxdist_and_radius_match_oracle(ctx):
    from pyoracle import OracleMap
    meta, _ = load_case("syn32")
    lines = case_input_lines(meta)
    pm = _map(meta)
    om = OracleMap(meta["region"], meta["spacing"], lines)
    for f in meta["fills"]:
        om.fill(*f)
    g = pm.make_graph(ctx, maxdist=9.5)
    om.make_graph(maxdist=9.5)
    ref = om.graph()
    got = g.copy()
    np.testing.assert_array_equal(got["bins"], ref["bins"])
    np.testing.assert_array_equal(got["runs"], ref["runs"])
    for r in (1, 2, 3):
        _assert_vga_close(g.vga_visual_global(radius=r), om.vga_global(radius=r))


def test_shards_assemble_to_whole_graph(ctx):
    """Source-range shards (one per rank in multi-GPU runs) reassembled == one-shot graph."""
    import torch
    meta, A = load_case("gallery")
    pm = _map(meta)
    n = meta["nodes"]
    cuts = [0, n // 3, (2 * n) // 3, n]
    shards = [pm.make_graph(ctx, node_begin=cuts[i], node_end=cuts[i + 1]) for i in range(3)]
    blobs = []
    for s in shards:
        t = torch.empty(s.blob_size(), dtype=torch.uint8, device="cuda:0")
        s.write_blob_device(t.data_ptr(), t.numel())
        blobs.append(t)
    torch.cuda.synchronize()
    g = pm.assemble(ctx, [b.data_ptr() for b in blobs[::-1]], [b.numel() for b in blobs[::-1]])
    got = g.copy()
    _assert_graph_equal(got, A, True)
    out = torch.full((n, 7), -1.0, dtype=torch.float32, device="cuda:0")
    g.vga_visual_global_device(out.data_ptr(), src_begin=100, src_end=900)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    _assert_vga_close(o[100:900], A["vga"][100:900])
    assert (o[:100] == -1).all() and (o[900:] == -1).all()


@pytest.mark.parametrize("stride", [1, 7, 64])
def test_balanced_shard_bounds_assemble_to_whole_graph(ctx, stride):
    """dmx_makegraph_balance: bounds cover [0, N) in order, repeat exactly (every rank computes them on
    its own), and the shards they cut reassemble to the one-shot graph."""
    import torch
    meta, A = load_case("gallery")
    pm = _map(meta)
    n = meta["nodes"]
    b = pm.shard_bounds(ctx, 4, stride=stride)
    assert b[0] == 0 and b[-1] == n and all(x <= y for x, y in zip(b, b[1:]))
    assert pm.shard_bounds(ctx, 4, stride=stride) == b
    assert pm.shard_bounds(ctx, 1, stride=stride) == [0, n]
    blobs = []
    for i in range(4):
        s = pm.make_graph(ctx, node_begin=b[i], node_end=b[i + 1])
        t = torch.empty(s.blob_size(), dtype=torch.uint8, device="cuda:0")
        s.write_blob_device(t.data_ptr(), t.numel())
        blobs.append(t)
        s.close()
    torch.cuda.synchronize()
    g = pm.assemble(ctx, [t.data_ptr() for t in blobs], [t.numel() for t in blobs])
    _assert_graph_equal(g.copy(), A, True)


def test_balanced_shard_bounds_do_not_depend_on_verbose(ctx, tmp_path):
    """DMX_VERBOSE=1 selects the makeGraph kernels with per-phase clocks; the cost sample of
    dmx_makegraph_balance must still count every sampled source, so the bounds are the same (every rank
    relies on computing identical bounds).  The flag is read once per process: a child process runs it."""
    import subprocess
    import sys
    meta, A = load_case("gallery")
    pm = _map(meta)
    want = pm.shard_bounds(ctx, 4, stride=7)
    code = ("import sys; sys.path[:0] = %r\n"
            "import depthmapx_amd as dmx\n"
            "from golden_io import load_case, case_input_lines\n"
            "meta, A = load_case('gallery')\n"
            "pm = dmx.PointMap(meta['region'], case_input_lines(meta), meta['spacing'])\n"
            "[pm.make_points(*f) for f in meta['fills']]\n"
            "print(pm.shard_bounds(dmx.Context(0), 4, stride=7))\n") % ([os.path.dirname(HERE), HERE],)
    env = dict(os.environ, DMX_VERBOSE="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == str(want)


@pytest.mark.parametrize("kernel", ["v1", "topdown", "do"])
def test_vga_kernels_agree(ctx, kernel, monkeypatch):
    """The tile-resolved BFS (default), the direction-optimising BFS, its top-down-only mode and
    the v1 top-down kernel agree bit-for-bit (levels and measures)."""
    meta, A = load_case("gallery")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    out_do, lv_do = g.vga_visual_global(levels=True)
    assert ctx.last_stats()["vga_kernel"] == "tile-resolved"
    monkeypatch.setenv("DMX_VGA_KERNEL", kernel)
    g2 = pm.make_graph(ctx)
    out2, lv2 = g2.vga_visual_global(levels=True)
    np.testing.assert_array_equal(lv_do, lv2)
    np.testing.assert_array_equal(out_do.view(np.uint32), out2.view(np.uint32))


def test_vga_asymmetric_graph_corrections(ctx, monkeypatch):
    """syn256 has 2 asymmetric visibility pairs (found by an exhaustive check): the bottom-up BFS
    must route the 4 nodes involved through exact in-set corrections and still agree bit-for-bit
    with the pure top-down kernel on sources around them."""
    lines = np.loadtxt(__import__("os").path.join(__import__("golden_io").GOLDEN, "inputs", "syn256.csv"),
                       delimiter=",", skiprows=1)
    pm = dmx.PointMap([0.0, 0.0, 256.0, 256.0], lines, 1.0)
    assert pm.make_points(0.5, 0.5)
    g = pm.make_graph(ctx)
    ranges = [(21900, 22100), (34000, 34200), (48050, 48200)]
    outs = []
    for (b, e) in ranges:
        outs.append(g.vga_visual_global(src_begin=b, src_end=e, levels=True))
    st = ctx.last_stats()
    assert st["vga_kernel"] == "tile-resolved" and st["vga_special_nodes"] == 4
    monkeypatch.setenv("DMX_VGA_KERNEL", "v1")
    g2 = pm.make_graph(ctx)
    for (b, e), (o, lv) in zip(ranges, outs):
        o2, lv2 = g2.vga_visual_global(src_begin=b, src_end=e, levels=True)
        np.testing.assert_array_equal(lv[b:e], lv2[b:e])
        np.testing.assert_array_equal(o[b:e].view(np.uint32), o2[b:e].view(np.uint32))


def test_symmetry_scatter_in_makegraph_equals_separate_pass(ctx, monkeypatch):
    """A whole-graph makeGraph does the symmetry certificate's scatter (per-node out-hash, range adds of the
    in-hash) as each source publishes its runs; DMX_MK_NOSYM leaves it to the VGA preparation's pass over the
    pool, as a shard or an assembled graph does.  Same special nodes (syn256: the 4 of its 2 asymmetric
    pairs) and bit-identical VGA on sources around them."""
    lines = np.loadtxt(__import__("os").path.join(__import__("golden_io").GOLDEN, "inputs", "syn256.csv"),
                       delimiter=",", skiprows=1)
    pm = dmx.PointMap([0.0, 0.0, 256.0, 256.0], lines, 1.0)
    assert pm.make_points(0.5, 0.5)
    res = []
    for nosym in (False, True):
        if nosym:
            monkeypatch.setenv("DMX_MK_NOSYM", "1")
        g = pm.make_graph(ctx)
        o, lv = g.vga_visual_global(src_begin=21900, src_end=22100, levels=True)
        res.append((g.special_nodes(), o[21900:22100].copy(), lv[21900:22100].copy()))
        g.close()
    assert len(res[0][0]) == 4 and list(res[0][0]) == list(res[1][0])
    np.testing.assert_array_equal(res[0][1].view(np.uint32), res[1][1].view(np.uint32))
    np.testing.assert_array_equal(res[0][2], res[1][2])


SD_CASES = ["kat", "syn16", "syn32", "syn64", "gallery"]


def _assert_stepdepth(got, want):
    # path length and straight-line distance: float sums of correctly rounded sqrt -> bit-exact;
    # cumulative angle: acos is libm vs device-libm (1 ulp) -> within 1e-6 relative
    np.testing.assert_array_equal(got[:, 1].view(np.uint32), want[:, 1].view(np.uint32))
    np.testing.assert_array_equal(got[:, 2].view(np.uint32), want[:, 2].view(np.uint32))
    tol = 1e-6 * np.maximum(1.0, np.abs(want[:, 0]))
    assert (np.abs(got[:, 0] - want[:, 0]) <= tol).all()


@pytest.mark.parametrize("name", SD_CASES)
def test_metric_stepdepth_matches_reference(ctx, name):
    meta, A = load_case(name)
    if "stepdepth" not in A:
        pytest.skip("fixture without step depth")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    pts = [tuple(float(v) for v in p.split(",")) for p in meta["stepdepth"]]
    got = g.metric_step_depth(points=pts)
    _assert_stepdepth(got, A["stepdepth"])
    sd = ctx.last_stepdepth()
    assert sd["expanders_popped"] > 0


@pytest.mark.parametrize("seed", [3, 7])
def test_metric_stepdepth_random_matches_oracle(ctx, seed):
    from pyoracle import OracleMap
    from golden.gen_synthetic import make_lines
    W = 48
    lines = np.array(make_lines(W, 80, seed=seed, lmin=0.02, lmax=0.3), dtype=np.float64)
    region = [0.0, 0.0, float(W), float(W)]
    pm = dmx.PointMap(region, lines, 1.0)
    om = OracleMap(region, 1.0, lines)
    assert pm.make_points(0.5, 0.5) and om.fill(0.5, 0.5)
    g = pm.make_graph(ctx)
    om.make_graph(threads=8)
    st = pm.state()
    rng = np.random.default_rng(seed)
    filled = np.nonzero(st & 2)[0]
    for nsel in (1, 3):
        cells = np.sort(rng.choice(filled, nsel, replace=False))
        got = g.metric_step_depth(cells=cells)
        rows = pm.rows
        order = np.argsort((cells // rows) * 65536 + cells % rows)
        want = om.metric_stepdepth(cells[order])
        _assert_stepdepth(got, want)


@pytest.mark.parametrize("name", SD_CASES + ["barnsbury", "syn128sd"])
def test_visual_stepdepth_matches_reference(ctx, name):
    """STEPDEPTH -sdt visual: the tile-resolved BFS in seed mode against the reference's column."""
    meta, A = load_case(name)
    if "vstepdepth" not in A:
        pytest.skip("fixture without visual step depth")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    pts = [tuple(float(v) for v in p.split(",")) for p in meta["stepdepth"]]
    got = g.visual_step_depth(points=pts)
    np.testing.assert_array_equal(got.view(np.uint32), A["vstepdepth"].view(np.uint32))


@pytest.mark.parametrize("seed", [3, 7])
def test_visual_stepdepth_random_matches_oracle(ctx, seed):
    from pyoracle import OracleMap
    from golden.gen_synthetic import make_lines
    W = 64
    lines = np.array(make_lines(W, 120, seed=seed, lmin=0.02, lmax=0.3), dtype=np.float64)
    region = [0.0, 0.0, float(W), float(W)]
    pm = dmx.PointMap(region, lines, 1.0)
    om = OracleMap(region, 1.0, lines)
    assert pm.make_points(0.5, 0.5) and om.fill(0.5, 0.5)
    g = pm.make_graph(ctx)
    om.make_graph(threads=8)
    filled = np.nonzero(pm.state() & 2)[0]
    rng = np.random.default_rng(seed)
    for nsel in (1, 4, 32):
        cells = np.sort(rng.choice(filled, nsel, replace=False))
        got = g.visual_step_depth(cells=cells)
        want = om.visual_stepdepth(cells)
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
        assert got.max() >= 2


def _dense_map(W, nocc, seed, lmin=0.0025, lmax=0.01):
    from golden.gen_synthetic import make_lines
    lines = np.array(make_lines(W, nocc, seed=seed, lmin=lmin, lmax=lmax), dtype=np.float64)
    pm = dmx.PointMap([0.0, 0.0, float(W), float(W)], lines, 1.0)
    assert pm.make_points(0.5, 0.5)
    return pm


@pytest.mark.parametrize("W,nocc,seed", [(48, 80, 3), (160, 400, 5), (300, 1500, 9)])
def test_metric_stepdepth_batched_equals_serial(ctx, monkeypatch, W, nocc, seed):
    """The whole-GPU batched search (distance windows of 1 grid unit, certified single winners,
    sequential fold of ambiguous cells) reproduces the serial pop-order kernel bit-for-bit on all three
    columns, for 1 and several selected cells (dense short occluders: many expanders)."""
    pm = _dense_map(W, nocc, seed, lmin=0.01 if W < 100 else 0.0025, lmax=0.05 if W < 100 else 0.01)
    g = pm.make_graph(ctx)
    filled = np.nonzero(pm.state() & 2)[0]
    rng = np.random.default_rng(seed)
    for nsel in (1, 5):
        cells = np.sort(rng.choice(filled, nsel, replace=False))
        monkeypatch.delenv("DMX_SD_KERNEL", raising=False)
        got = g.metric_step_depth(cells=cells)
        sd = ctx.last_stepdepth()
        assert sd["mode"] == "batched" and sd["batches"] > 1, sd
        monkeypatch.setenv("DMX_SD_KERNEL", "serial")
        want = g.metric_step_depth(cells=cells)
        sd2 = ctx.last_stepdepth()
        assert sd2["mode"] == "serial"
        assert sd["expanders_popped"] == sd2["expanders_popped"]
        assert sd["cells_relaxed"] == sd2["cells_relaxed"]
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def test_metric_stepdepth_errors(ctx):
    meta, _ = load_case("syn32")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    with pytest.raises(dmx.DmxError):
        g.metric_step_depth(points=[(-5.0, 1.0)])   # outside the region


CHUNK_CASES = ["kat", "syn16", "syn32", "gallery", "syn64"]


@pytest.mark.parametrize("name", CHUNK_CASES)
def test_gpu_graph_chunk_bytes_match_reference(ctx, name):
    """VISPREP's output: the PointMap chunk written from the GPU graph is byte-identical to the one
    the reference writes (PointMap::write)."""
    import hashlib
    from depthmapx_amd import graphio
    meta, A = load_case(name)
    pm = _map(meta)
    g = pm.make_graph(ctx)
    c = g.copy(runs=True)
    cols = [(n, c["attrs"][:, j], j == 0) for j, n in enumerate(dmx.MAKEGRAPH_COLUMNS)]
    blob = graphio.write_chunk(pm, c["bins"], c["runs"], c["gridconn"], cols, displayed=0)
    assert len(blob) == int(A["pm_chunk_size"][0])
    assert hashlib.sha256(blob).digest() == A["pm_chunk_sha256"].tobytes()


@pytest.mark.parametrize("name", [n for n in CHUNK_CASES if n != "syn64"])
def test_vga_after_graph_roundtrip_matches_reference_cli(ctx, name):
    """The reference CLI runs VGA on the graph re-read from the .graph file (4-bit shift quirk):
    VISPREP chunk -> decode -> GPU VGA == the reference's VGA after its own round trip."""
    from depthmapx_amd import graphio
    meta, A = load_case(name)
    if "vga_rt" not in A:
        pytest.skip("no round-trip fixture")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    c = g.copy(runs=True)
    cols = [(n, c["attrs"][:, j], j == 0) for j, n in enumerate(dmx.MAKEGRAPH_COLUMNS)]
    blob = graphio.write_chunk(pm, c["bins"], c["runs"], c["gridconn"], cols, displayed=0)
    pm2, g2 = graphio.load_chunk(ctx, blob, meta["region"])
    out = g2.vga_visual_global(radius=-1)
    _assert_vga_close(out, A["vga_rt"])
    np.testing.assert_array_equal(out[:, 5], A["vga_rt"][:, 5])


@pytest.mark.parametrize("gcap,bcap,spill", [("2", "2", None), ("128", "2", "2")])
def test_makegraph_capacity_retries_are_exact(ctx, monkeypatch, gcap, bcap, spill):
    """Blocks past the LDS capacity go to the wave's HBM spill area; sources that overflow the gap
    capacity or the spill area are re-run with larger capacities.  With tiny initial capacities
    almost every source takes those paths and the graph is still exact."""
    meta, A = load_case("gallery")
    monkeypatch.setenv("DMX_MK_GCAP", gcap)
    monkeypatch.setenv("DMX_MK_BCAP", bcap)
    if spill:
        monkeypatch.setenv("DMX_MK_SPILL", spill)
    pm = _map(meta)
    g = pm.make_graph(ctx)
    _assert_graph_equal(g.copy(runs=True), A, True)


def test_makegraph_sampled_pool_is_exact(ctx, monkeypatch):
    """Run-pool sizing from a sample pass (forced with DMX_MK_SAMPLE; automatic when the worst-case pool
    would take over 40 % of the device, e.g. 2000^2): the graph is bit-identical to the reference's."""
    meta, A = load_case("syn256mk")
    monkeypatch.setenv("DMX_MK_SAMPLE", "1")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    _assert_graph_equal(g.copy(runs=True), A, meta["full_runs"])


def test_makegraph_certified_moments_equal_serial_chains(ctx, monkeypatch):
    """The first makeGraph pass sums the moments in parallel (double-double) and keeps a float only
    when the reference's serial FP64 chain provably rounds to it; the rest are re-run with the
    serial chains.  Both modes must give the same bits on every node (65k sources)."""
    meta, A = load_case("syn256mk")
    pm = _map(meta)
    fast = pm.make_graph(ctx).copy(runs=False)["attrs"]
    monkeypatch.setenv("DMX_MK_EXACT", "1")
    serial = pm.make_graph(ctx).copy(runs=False)["attrs"]
    np.testing.assert_array_equal(fast.view(np.uint32), serial.view(np.uint32))
    np.testing.assert_array_equal(fast.view(np.uint32), A["attrs"].view(np.uint32))


def test_makegraph_spans_equal_cell_by_cell(ctx, monkeypatch):
    """Occluder-free depth spans (makegraph.hip, span.hpp) against the cell-by-cell sweep of the same kernel
    (DMX_MK_NOSPAN) and the reference's own graph of syn256mk: bins, runs, attributes and grid connections
    bit for bit, with spans of every length taken (DMX_MK_SPAN=1)."""
    meta, A = load_case("syn256mk")
    pm = _map(meta)
    monkeypatch.setenv("DMX_MK_SPAN", "1")
    a = pm.make_graph(ctx).copy(runs=True)
    monkeypatch.delenv("DMX_MK_SPAN")
    monkeypatch.setenv("DMX_MK_NOSPAN", "1")
    b = pm.make_graph(ctx).copy(runs=True)
    for k in ("bins", "runs", "gridconn"):
        np.testing.assert_array_equal(a[k], b[k])
    np.testing.assert_array_equal(a["attrs"].view(np.uint32), b["attrs"].view(np.uint32))
    np.testing.assert_array_equal(a["attrs"].view(np.uint32), A["attrs"].view(np.uint32))


def test_makegraph_without_the_certified_sums_is_exact(ctx, monkeypatch):
    """A device square root too coarse for the moment certificate (forced with DMX_MK_SQRT_BAD) no longer fails
    makeGraph: every source takes the serial chains from the first pass, with the same bits."""
    meta, A = load_case("syn64")
    pm = _map(meta)
    monkeypatch.setenv("DMX_MK_SQRT_BAD", "1")
    g = pm.make_graph(ctx)
    _assert_graph_equal(g.copy(runs=True), A, False)


def test_vga_source_list_matches_full_run(ctx):
    """dmx_vga_global_device_list (the interleaved multi-GPU shards): listed rows equal the full
    run's rows bit for bit, every other row is left untouched."""
    import torch
    meta, A = load_case("syn64")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    full = g.vga_visual_global()
    n = full.shape[0]
    rng = np.random.default_rng(5)
    nodes = np.sort(rng.choice(n, n // 3, replace=False))
    out = torch.full((n, 7), -7.0, dtype=torch.float32, device="cuda")
    g.vga_visual_global_device_list(out.data_ptr(), nodes)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    np.testing.assert_array_equal(got[nodes].view(np.uint32), full[nodes].view(np.uint32))
    rest = np.setdiff1d(np.arange(n), nodes)
    assert (got[rest] == -7.0).all()


def test_vga_prep_shard_single_rank_identity(ctx, monkeypatch):
    """dmx_graph_set_prep_shard with a world of one (the all-reduce is the identity): same columns
    as the unsharded run, and the callback sees the partial buffers in order: the in-set hash
    difference arrays, the out-set hashes, the special-node veto, then the tvis / ftvis rows (each rank
    builds the partial-tile masks of every node itself: no collective).  A graph whose makeGraph swept
    every source did the hash scatter as it published the runs: complete on every rank, so the hashes
    are not all-reduced (the veto and the rows still are)."""
    import torch
    meta, A = load_case("gallery")
    pm = _map(meta)
    full = pm.make_graph(ctx).vga_visual_global()
    n = full.shape[0]
    C = meta["cols"] * meta["rows"]
    for nosym in (True, False):
        if nosym:
            monkeypatch.setenv("DMX_MK_NOSYM", "1")
        else:
            monkeypatch.delenv("DMX_MK_NOSYM", raising=False)
        g = pm.make_graph(ctx)
        calls = []
        g.set_prep_shard(0, n, lambda ptr, count, dtype: calls.append((count, dtype)) or 0)
        out = torch.full((n, 7), -1.0, dtype=torch.float32, device="cuda")
        g.vga_visual_global_device_list(out.data_ptr(), np.arange(n))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), full.view(np.uint32))
        if nosym:
            assert calls[:3] == [(4 * C, 1), (n, 1), (1, 1)]
            assert len(calls) == 5 and calls[3] == calls[4] and calls[3][1] == 1
        else:
            assert calls[0] == (1, 1) and len(calls) == 3 and calls[1] == calls[2] and calls[1][1] == 1
        g.close()


@pytest.mark.parametrize("name", ["gallery", "syn64"])
def test_vga_prep_shard_two_ranks_threads(ctx, name):
    """Two emulated ranks (threads, each with its own context and stream on cuda:0) split the VGA
    preparation by node range and sum the partial buffers through a barrier -- the all-reduce that
    bench.py does with RCCL; each rank's interleaved source rows must equal the unsharded run."""
    import threading
    import torch
    from depthmapx_amd.sharded import device_view, shard_range, vga_nodes
    meta, A = load_case(name)
    pm = _map(meta)
    full = pm.make_graph(ctx).vga_visual_global()
    n = full.shape[0]
    ctxs = [dmx.Context(0), dmx.Context(0)]
    graphs = [pm.make_graph(c) for c in ctxs]
    bar = threading.Barrier(2, timeout=60)
    slots = [None, None]
    dev = torch.device("cuda", 0)

    def make_fn(r):
        def fn(ptr, count, dtype):
            t = device_view(ptr, count, dtype, dev)
            slots[r] = t.clone()
            torch.cuda.synchronize()
            bar.wait()
            t.copy_(slots[0] + slots[1])
            torch.cuda.synchronize()
            bar.wait()
            return 0
        return fn

    outs = [torch.full((n, 7), -1.0, dtype=torch.float32, device="cuda") for _ in range(2)]
    lists = [vga_nodes(n, r, 2, chunk=256) for r in range(2)]
    errs = [None, None]
    for r in range(2):
        graphs[r].set_prep_shard(*shard_range(n, r, 2), make_fn(r))

    def run(r):
        try:
            graphs[r].vga_visual_global_device_list(outs[r].data_ptr(), lists[r])
        except Exception as ex:   # surfaced below
            errs[r] = ex
            bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert errs == [None, None], errs
    torch.cuda.synchronize()
    got = np.full_like(full, -1.0)
    for r in range(2):
        got[lists[r]] = outs[r].cpu().numpy()[lists[r]]
    np.testing.assert_array_equal(got.view(np.uint32), full.view(np.uint32))


@pytest.mark.parametrize("name", ["kat", "syn16", "syn32", "syn64", "gallery"])
def test_vga_local_matches_reference_and_oracle(ctx, name):
    """VGA -vl on the GPU: bit-exact against the reference's columns where a fixture exists
    (make_golden_vga_modes.py) and against the C restatement (itself pinned on those fixtures)."""
    import os
    from golden_io import GOLDEN
    from pyoracle import OracleMap
    meta, A = load_case(name)
    pm = _map(meta)
    got = pm.make_graph(ctx).vga_visual_local()
    path = os.path.join(GOLDEN, name + "_vlocal.npy")
    if os.path.exists(path):
        np.testing.assert_array_equal(got.view(np.uint32), np.load(path).view(np.uint32))
    om = OracleMap(meta["region"], meta["spacing"], case_input_lines(meta))
    for f in meta["fills"]:
        om.fill(*f)
    om.make_graph(threads=8)
    np.testing.assert_array_equal(got.view(np.uint32), om.vga_local(threads=8).view(np.uint32))


def test_vga_local_ranges_and_gates_only(ctx):
    """Source ranges leave other rows untouched; gates_only skips every source (-1)."""
    meta, A = load_case("syn32")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    full = g.vga_visual_local()
    n = full.shape[0]
    part = g.vga_visual_local(src_begin=100, src_end=300)
    np.testing.assert_array_equal(part[100:300].view(np.uint32), full[100:300].view(np.uint32))
    assert (part[:100] == -1).all() and (part[300:] == -1).all()
    assert (g.vga_visual_local(gates_only=True) == -1).all()


@pytest.mark.parametrize("name,radius", [("kat", -1.0), ("syn16", -1.0), ("syn32", -1.0), ("syn32", 10.0),
                                         ("gallery", -1.0), ("syn64", -1.0), ("syn64", 7.5)])
def test_vga_metric_matches_reference_and_oracle(ctx, name, radius):
    """VGA -vm metric on the GPU (all sources, ordered float totals): bit-exact against the
    reference's columns where a fixture exists and against the C restatement."""
    import os
    from golden_io import GOLDEN
    from pyoracle import OracleMap
    meta, A = load_case(name)
    pm = _map(meta)
    got = pm.make_graph(ctx).vga_metric(radius=radius)
    path = os.path.join(GOLDEN, name + "_vmetric" + ("" if radius < 0 else "_r%g" % radius) + ".npy")
    if os.path.exists(path):
        np.testing.assert_array_equal(got.view(np.uint32), np.load(path).view(np.uint32))
    om = OracleMap(meta["region"], meta["spacing"], case_input_lines(meta))
    for f in meta["fills"]:
        om.fill(*f)
    om.make_graph(threads=8)
    np.testing.assert_array_equal(got.view(np.uint32), om.vga_metric(radius=radius, threads=8).view(np.uint32))


def test_vga_metric_ranges_and_gates_only(ctx):
    meta, A = load_case("syn32")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    full = g.vga_metric()
    part = g.vga_metric(src_begin=200, src_end=500)
    np.testing.assert_array_equal(part[200:500].view(np.uint32), full[200:500].view(np.uint32))
    assert (part[:200] == -1).all() and (part[500:] == -1).all()
    assert (g.vga_metric(gates_only=True) == -1).all()


def test_vga_metric_syn128_sources_match_oracle(ctx):
    """A block of sources in the middle of the 128^2 synthetic plan (16k nodes, long float chains
    and NaN angles from acos of a rounded-up cosine, as in the reference) against the oracle."""
    from pyoracle import OracleMap
    meta, A = load_case("syn128sd")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    n = g.info()["nnodes"]
    b, e = n // 2 - 48, n // 2 + 48
    got = g.vga_metric(src_begin=b, src_end=e)
    om = OracleMap(meta["region"], meta["spacing"], case_input_lines(meta))
    for f in meta["fills"]:
        om.fill(*f)
    om.make_graph(threads=8)
    want = om.vga_metric(node_begin=b, node_end=e, threads=8)
    np.testing.assert_array_equal(got[b:e].view(np.uint32), want[b:e].view(np.uint32))


@pytest.mark.parametrize("name,radius", [("kat", -1.0), ("syn16", -1.0), ("syn32", -1.0), ("syn32", 1.5),
                                         ("gallery", -1.0), ("syn64", -1.0), ("syn64", 0.5)])
def test_vga_angular_matches_reference_and_oracle(ctx, name, radius):
    """VGA -vm angular on the GPU (all sources; cells reached at angle 0 expand too): bit-exact
    against the reference's columns where a fixture exists and against the C restatement."""
    import os
    from golden_io import GOLDEN
    from pyoracle import OracleMap
    meta, A = load_case(name)
    pm = _map(meta)
    got = pm.make_graph(ctx).vga_angular(radius=radius)
    path = os.path.join(GOLDEN, name + "_vangular" + ("" if radius < 0 else "_r%g" % radius) + ".npy")
    if os.path.exists(path):
        np.testing.assert_array_equal(got.view(np.uint32), np.load(path).view(np.uint32))
    om = OracleMap(meta["region"], meta["spacing"], case_input_lines(meta))
    for f in meta["fills"]:
        om.fill(*f)
    om.make_graph(threads=8)
    np.testing.assert_array_equal(got.view(np.uint32), om.vga_angular(radius=radius, threads=8).view(np.uint32))


@pytest.mark.parametrize("name", ["kat", "syn16", "syn32", "syn64", "gallery", "barnsbury", "syn128sd"])
def test_angular_stepdepth_matches_reference(ctx, name):
    """STEPDEPTH -sdt angular on the GPU: the reference's column (fixtures) / the oracle (syn128sd)."""
    import os
    from golden_io import GOLDEN
    from pyoracle import OracleMap
    meta, A = load_case(name)
    pm = _map(meta)
    g = pm.make_graph(ctx)
    sel = A["stepdepth_sel"]
    cells = (sel >> 16) * meta["rows"] + (sel & 0xFFFF)
    got = g.angular_step_depth(cells=cells)
    path = os.path.join(GOLDEN, name + "_astepdepth.npy")
    if os.path.exists(path):
        want = np.load(path)
    else:
        om = OracleMap(meta["region"], meta["spacing"], case_input_lines(meta))
        for f in meta["fills"]:
            om.fill(*f)
        om.make_graph(threads=8)
        want = om.angular_stepdepth(cells)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    assert (got >= 0).sum() > 0


def test_vga_angular_syn128_sources_match_oracle(ctx):
    """A block of sources of the 128^2 plan against the oracle: thousands of cells sit at angle 0
    (seen straight from the source), more than one LDS sort window -- the HBM sort path."""
    from pyoracle import OracleMap
    meta, A = load_case("syn128sd")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    n = g.info()["nnodes"]
    b, e = n // 2 - 48, n // 2 + 48
    got = g.vga_angular(src_begin=b, src_end=e)
    om = OracleMap(meta["region"], meta["spacing"], case_input_lines(meta))
    for f in meta["fills"]:
        om.fill(*f)
    om.make_graph(threads=8)
    want = om.vga_angular(node_begin=b, node_end=e, threads=8)
    np.testing.assert_array_equal(got[b:e].view(np.uint32), want[b:e].view(np.uint32))
    assert (got[b:e, 2] > 8192).any()


@pytest.mark.parametrize("kind", ["metric", "angular"])
def test_vga_metric_angular_overflow_rerun_is_exact(ctx, kind, monkeypatch):
    """A per-workgroup overflow list far too small (DMX_SD_CAP test hook): the sources whose search
    outgrows it stop, are listed, and only they run again with a 4x list -- same bits as one pass."""
    meta, A = load_case("syn64")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    run = g.vga_metric if kind == "metric" else g.vga_angular
    want = run()
    assert ctx.last_stats()["vga_fail_cells"] == 0
    monkeypatch.setenv("DMX_SD_CAP", "64")
    got = run()
    if kind == "angular":   # cells seen at angle 0 are all queued: the 64-entry list overflows
        assert ctx.last_stats()["vga_fail_cells"] > 0
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def test_vga_global_gates_only_matches_oracle(ctx):
    """VGA -vg with gates_only: VGAVisualGlobal::run skips every source (vgavisualglobal.cpp:72-75), so
    no column value is set -- the same rows as the restatement."""
    from pyoracle import OracleMap
    meta, A = load_case("syn32")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    got = g.vga_visual_global(gates_only=True)
    om = OracleMap(meta["region"], meta["spacing"], case_input_lines(meta))
    for f in meta["fills"]:
        om.fill(*f)
    om.make_graph(threads=8)
    want = om.vga_global(gates_only=True, threads=8)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    assert (got == -1).all()
