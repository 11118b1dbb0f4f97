"""Merge links (Point::m_merge, set by depthmapXcli's LINK mode / PointMap::mergePixels,
salalib/pointdata.cpp:1653-1680) in every search that follows them.

The reference's own VGA / STEPDEPTH regression cases (RegressionTest/regressionconfig.json) all run on
maps with merge links (gallery_connected.graph: 2 links, turns_connected.graph: 1).  The partner
bookkeeping being restated:
  VGA global         vgavisualglobal.cpp:113-122      partner extracted at the same level, not counted
  visual step depth  vgavisualglobaldepth.cpp:55-63   partner takes the level, extracted
  VGA metric/angular vgametric.cpp:97-105, vgaangular.cpp:95-104       partner extracted, not counted
  metric/angular SD  vgametricdepth.cpp:68-83, vgaangulardepth.cpp:57-67 partner row written, extracted

CPU: the C restatement (oracle/) against the columns the real reference wrote for those cases
(tests/golden/graphfiles/*_cols.npz, made by tests/golden/make_golden_graphfiles.py from the reference
built from source) -- this pins the oracle's merge semantics.  GPU: the HIP kernels against the pinned
oracle on seeded synthetic maps with random merge links (every kernel family: tile-resolved BFS,
direction-optimising BFS, top-down visual step depth, the serial metric / angular searches), and the
exact handling of links with a context-filled end, in the reference's own level order where its pop order
decides (kernels/vga_ordered.hip)."""
import json
import lzma
import os

import numpy as np
import pytest

import graphfile_util as gu

HERE = os.path.dirname(os.path.abspath(__file__))
GF = os.path.join(HERE, "golden", "graphfiles")
CASES = json.load(open(os.path.join(GF, "cases.json")))
EXACT = {"Visual Node Count", "Metric Node Count", "Angular Node Count", "Visual Step Depth",
         "Metric Step Shortest-Path Length", "Metric Straight-Line Distance", "Angular Step Depth",
         "Angular Total Depth"}
VGA_VIS = ["Visual Entropy", "Visual Integration [HH]", "Visual Integration [P-value]", "Visual Integration [Tekl]",
           "Visual Mean Depth", "Visual Node Count", "Visual Relativised Entropy"]
SD_METRIC = ["Metric Step Shortest-Path Angle", "Metric Step Shortest-Path Length", "Metric Straight-Line Distance"]
VGA_METRIC = ["Metric Mean Shortest-Path Angle", "Metric Mean Shortest-Path Distance",
              "Metric Mean Straight-Line Distance", "Metric Node Count"]
VGA_ANGULAR = ["Angular Mean Depth", "Angular Total Depth", "Angular Node Count"]


def _graph_input(tmp_path, name):
    dst = os.path.join(str(tmp_path), name)
    if not os.path.exists(dst):
        with lzma.open(os.path.join(GF, "inputs", name + ".xz")) as f, open(dst, "wb") as o:
            o.write(f.read())
    return dst


def _oracle_for(pmd):
    from pyoracle import OracleMap
    om = OracleMap.from_grid(pmd["cols"], pmd["rows"], pmd["spacing"], pmd["bottom_left"], pmd["state"])
    om.set_graph(pmd["bins"], pmd["runs"])
    om.set_merges(pmd["merges"])
    return om


def _pixelate(pmd, x, y):
    """PointMap::pixelate(p, constrain=true) (pointdata.cpp:263-283) -> x-major cell."""
    s, (bx, by) = pmd["spacing"], pmd["bottom_left"]
    px = min(max(int(np.floor((x - bx + s / 2.0) / s)), 0), pmd["cols"] - 1)
    py = min(max(int(np.floor((y - by + s / 2.0) / s)), 0), pmd["rows"] - 1)
    return px * pmd["rows"] + py


def _compare(got, ref, cols, rows=None):
    for j, col in enumerate(cols):
        a = got[:, j] if got.ndim == 2 else got
        r = ref[col]
        if rows is not None:
            a, r = a[rows], r[rows]
        if col.split(" R")[0] in EXACT:
            assert np.array_equal(a.view(np.uint32), r.view(np.uint32)), (col, np.flatnonzero(a != r)[:8])
        else:
            fin = np.isfinite(r)
            assert np.array_equal(np.isfinite(a), fin), col
            assert np.allclose(a[fin], r[fin], rtol=1e-6, atol=1e-6), (col, float(np.abs(a[fin] - r[fin]).max()))


def _ref_cols(case):
    return np.load(os.path.join(GF, case + "_cols.npz"), allow_pickle=False)


def test_merge_fixtures_hold_links():
    """The reference inputs carry merge links and every merge case has the reference's output columns."""
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:
        for graph, nlinks in [("gallery_connected.graph", 2), ("turns_connected.graph", 1)]:
            pmd = gu.load_pointmap(_graph_input(tmp, graph))
            assert len(pmd["merges"]) == nlinks, graph
            filled = (pmd["state"] & 2) != 0
            assert filled[pmd["merges"].ravel()].all()
    for name, m in CASES.items():
        if name.startswith("merge_") and m["columns"]:
            assert os.path.exists(os.path.join(GF, name + "_cols.npz")), name


@pytest.mark.parametrize("case,radius", [("merge_vis_global_n", -1), ("merge_vis_global_3", 3)])
def test_oracle_vga_global_with_merges_matches_reference(tmp_path, case, radius):
    pmd = gu.load_pointmap(_graph_input(tmp_path, CASES[case]["input"]))
    om = _oracle_for(pmd)
    out = om.vga_global(radius=radius, threads=8)
    cols = VGA_VIS if radius < 0 else [c + " R3" for c in VGA_VIS]
    _compare(out, _ref_cols(case), cols)


def test_oracle_step_depths_with_merges_match_reference(tmp_path):
    pmd = gu.load_pointmap(_graph_input(tmp_path, "gallery_connected.graph"))
    om = _oracle_for(pmd)
    sel = [_pixelate(pmd, 3.0, 5.0)]
    assert pmd["state"][sel[0]] & 2
    _compare(om.visual_stepdepth(sel), _ref_cols("merge_sd_visual"), ["Visual Step Depth"])
    _compare(om.metric_stepdepth(sel), _ref_cols("merge_sd_metric"), SD_METRIC)
    _compare(om.angular_stepdepth(sel), _ref_cols("merge_sd_angular"), ["Angular Step Depth"])


@pytest.mark.parametrize("case,kind", [("merge_vga_metric", "metric"), ("merge_vga_angular", "angular")])
def test_oracle_vga_metric_angular_with_merges_match_reference_turns(tmp_path, case, kind):
    pmd = gu.load_pointmap(_graph_input(tmp_path, CASES[case]["input"]))
    om = _oracle_for(pmd)
    out = om.vga_metric(threads=8) if kind == "metric" else om.vga_angular(threads=8)
    _compare(out, _ref_cols(case), VGA_METRIC if kind == "metric" else VGA_ANGULAR)


@pytest.mark.parametrize("case,kind", [("merge_vga_metric_gallery", "metric"), ("merge_vga_angular_gallery", "angular")])
def test_oracle_vga_metric_angular_with_merges_match_reference_gallery(tmp_path, case, kind):
    """Gallery: the sources around the linked cells and a sample elsewhere (the full all-pairs search is
    minutes of CPU)."""
    pmd = gu.load_pointmap(_graph_input(tmp_path, "gallery_connected.graph"))
    om = _oracle_for(pmd)
    N = int((pmd["state"] & 2).astype(bool).sum())
    cell_node = np.cumsum((pmd["state"] & 2) != 0) - 1
    linked = sorted(set(int(cell_node[c]) for c in pmd["merges"].ravel()))
    rows = sorted(set(linked + list(range(0, N, 97))))
    out = np.full((N, 4 if kind == "metric" else 3), -1.0, dtype=np.float32)
    for k in rows:
        part = om.vga_metric(node_begin=k, node_end=k + 1) if kind == "metric" else om.vga_angular(node_begin=k,
                                                                                                  node_end=k + 1)
        out[k] = part[k]
    _compare(out, _ref_cols(case), VGA_METRIC if kind == "metric" else VGA_ANGULAR, rows=rows)


# ---------------------------------------------------------------- GPU vs the pinned oracle
def _synthetic(seed, W=40, nlinks=12):
    """A seeded map with random merge links between filled cells (disjoint pairs)."""
    from golden.gen_synthetic import make_lines
    from pyoracle import OracleMap
    import depthmapx_amd as dmx
    lines = np.array(make_lines(W, 40, seed=seed, lmin=0.04, lmax=0.25), dtype=np.float64)
    region = [0.0, 0.0, float(W), float(W)]
    pm = dmx.PointMap(region, lines, 1.0)
    om = OracleMap(region, 1.0, lines)
    assert pm.make_points(0.5, 0.5) and om.fill(0.5, 0.5)
    st = pm.state()
    filled = np.flatnonzero(st & 2)
    rng = np.random.default_rng(seed)
    cells = rng.choice(filled, size=2 * nlinks, replace=False)
    pairs = cells.reshape(-1, 2).astype(np.int32)
    return pm, om, pairs


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 5])
@pytest.mark.parametrize("kernel", ["tile", "do", "do_topdown"])
def test_gpu_vga_global_with_merges_matches_oracle(ctx, monkeypatch, seed, kernel):
    if kernel == "do":
        monkeypatch.setenv("DMX_VGA_KERNEL", "do")
    elif kernel == "do_topdown":
        monkeypatch.setenv("DMX_VGA_KERNEL", "topdown")
    pm, om, pairs = _synthetic(seed)
    pm.set_merges(pairs)
    g = pm.make_graph(ctx)
    om.make_graph()
    om.set_merges(pairs)
    for radius in (-1, 3):
        got, lv = g.vga_visual_global(radius=radius, levels=True)
        ref, rlv = om.vga_global(radius=radius, threads=8, levels=True)
        np.testing.assert_array_equal(lv[:, :2], rlv[:, :2])
        np.testing.assert_array_equal(got[:, 5], ref[:, 5])
        assert np.allclose(got, ref, rtol=1e-6, atol=1e-6)
    # the links change the result (the comparison above would hold vacuously otherwise)
    om.set_merges(np.zeros((0, 2), dtype=np.int32))
    _, plain = om.vga_global(radius=-1, threads=8, levels=True)
    _, linked = g.vga_visual_global(radius=-1, levels=True)
    assert (plain[:, 1] != linked[:, 1]).any()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("topdown", [False, True])
def test_gpu_visual_step_depth_with_merges_matches_oracle(ctx, monkeypatch, seed, topdown):
    if topdown:
        monkeypatch.setenv("DMX_VSD_TOPDOWN", "1")
    pm, om, pairs = _synthetic(seed)
    pm.set_merges(pairs)
    g = pm.make_graph(ctx)
    om.make_graph()
    om.set_merges(pairs)
    for sel in ([int(pairs[0, 0])], [int(pairs[1, 1]), int(pairs[3, 0])], [pm.pixelate(20.5, 20.5)]):
        if not (pm.state()[sel] & 2).all():
            continue
        got = g.visual_step_depth(cells=sel)
        ref = om.visual_stepdepth(sorted(sel))
        np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_metric_angular_step_depth_with_merges_match_oracle(ctx, seed):
    pm, om, pairs = _synthetic(seed)
    pm.set_merges(pairs)
    g = pm.make_graph(ctx)
    om.make_graph()
    om.set_merges(pairs)
    for sel in ([int(pairs[0, 0])], [int(pairs[2, 1]), int(pairs[4, 0])]):
        got = g.metric_step_depth(cells=sel)
        ref = om.metric_stepdepth(sorted(sel, key=lambda c: ((c // pm.rows) << 16) + c % pm.rows))
        np.testing.assert_array_equal(got[:, 1:].view(np.uint32), ref[:, 1:].view(np.uint32))
        assert np.allclose(got[:, 0], ref[:, 0], rtol=1e-6, atol=1e-6, equal_nan=True)
        gota = g.angular_step_depth(cells=sel)
        refa = om.angular_stepdepth(sorted(sel, key=lambda c: ((c // pm.rows) << 16) + c % pm.rows))
        np.testing.assert_array_equal(gota.view(np.uint32), refa.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_vga_metric_angular_with_merges_match_oracle(ctx, seed):
    pm, om, pairs = _synthetic(seed, W=24, nlinks=8)
    pm.set_merges(pairs)
    g = pm.make_graph(ctx)
    om.make_graph()
    om.set_merges(pairs)
    got, ref = g.vga_metric(), om.vga_metric(threads=8)
    np.testing.assert_array_equal(got[:, 3], ref[:, 3])
    np.testing.assert_array_equal(got[:, 1:3].view(np.uint32), ref[:, 1:3].view(np.uint32))
    assert np.allclose(got[:, 0], ref[:, 0], rtol=1e-6, atol=1e-6, equal_nan=True)
    got, ref = g.vga_angular(), om.vga_angular(threads=8)
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))


def _contextfilled_links(seed):
    """A seeded map whose links all have one end context-filled at an odd PixelRef (SEMIFILL)."""
    import depthmapx_amd as dmx
    pm, om, pairs = _synthetic(seed, nlinks=16)
    rows = pm.rows
    st = np.ascontiguousarray(pm.state(), dtype=np.int32)
    for a, _ in pairs:
        x, y = divmod(int(a), rows)
        if x % 2 or y % 2:
            st[a] |= 0x8   # Point::CONTEXTFILLED
    N = dmx._native
    N.check(N.lib().dmx_pointmap_set_state(pm.h, N.ptr(st)))
    from pyoracle import OracleMap
    om2 = OracleMap.from_grid(pm.cols, rows, 1.0, pm.info()["bottom_left"], st)
    return pm, om, om2, pairs


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 4, 6])
@pytest.mark.parametrize("kernel", ["tile", "do"])
def test_gpu_contextfilled_links_exact_where_order_matters(ctx, monkeypatch, seed, kernel):
    """Merge links with a context-filled odd end under a radius: the GPU answers exactly what the reference
    computes.  Where some source finds both ends at one level the reference's count depends on its pop order
    inside the level (the oracle's two orders differ): the level-synchronous kernel flags those sources and
    they run again in the reference's order (vga_order_reruns > 0); elsewhere nothing is re-run.  Radius n
    expands every cell."""
    import pyoracle
    if kernel == "do":
        monkeypatch.setenv("DMX_VGA_KERNEL", "do")
    pm, om, om2, pairs = _contextfilled_links(seed)
    pm.set_merges(pairs)
    g = pm.make_graph(ctx)
    om.make_graph()
    b = om.graph()
    om2.set_graph(b["bins"], b["runs"])
    om2.set_merges(pairs)
    got = g.vga_visual_global(radius=-1)
    assert np.allclose(got, om2.vga_global(radius=-1, threads=8), rtol=1e-6, atol=1e-6)
    outcomes = []
    for radius in (2, 3, 5):
        ref = om2.vga_global(radius=radius, threads=8)
        try:
            pyoracle.set_pop_forward(True)
            fwd = om2.vga_global(radius=radius, threads=8)
        finally:
            pyoracle.set_pop_forward(False)
        order_free = np.array_equal(ref.view(np.uint32), fwd.view(np.uint32))
        got = g.vga_visual_global(radius=radius)
        reruns = ctx.last_stats()["vga_order_reruns"]
        np.testing.assert_array_equal(got[:, 5], ref[:, 5])
        assert np.allclose(got, ref, rtol=1e-6, atol=1e-6)
        if not order_free:
            assert reruns > 0, radius
        outcomes.append("reference order" if reruns else "level-synchronous")
    assert len(outcomes) == 3


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 4, 6])
def test_gpu_visual_step_depth_with_contextfilled_links(ctx, seed):
    """Visual step depth with context-filled odd link ends: exact (bit for bit with the oracle).  Where
    extracting an unexpanded end would reach a new cell (the two pop orders can differ) the search runs in the
    reference's order (vga_order_reruns == 1)."""
    import pyoracle
    pm, om, om2, pairs = _contextfilled_links(seed)
    pm.set_merges(pairs)
    g = pm.make_graph(ctx)
    om.make_graph()
    b = om.graph()
    om2.set_graph(b["bins"], b["runs"])
    om2.set_merges(pairs)
    st = pm.state()
    cells = [int(pairs[0, 1]), int(pairs[1, 0]), pm.pixelate(20.5, 20.5), int(pairs[5, 1])]
    ran = 0
    for c in cells:
        if not st[c] & 2:
            continue
        ref = om2.visual_stepdepth([c])
        try:
            pyoracle.set_pop_forward(True)
            fwd = om2.visual_stepdepth([c])
        finally:
            pyoracle.set_pop_forward(False)
        got = g.visual_step_depth(cells=[c])
        if not np.array_equal(ref.view(np.uint32), fwd.view(np.uint32)):
            assert ctx.last_stats()["vga_order_reruns"] == 1
        np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
        ran += 1
    assert ran > 0


def _deep_serpentine_links(W=320, H=12, pitch=4, gap=3):
    """A serpentine corridor (walls every `pitch` cells, openings alternating top / bottom): visual depths past
    64 levels from the ends.  Merge links join neighbouring cells of one corridor, the odd-x end context-filled
    (SEMIFILL), so a search finds both ends at one level and the reference's pop order decides the count."""
    import depthmapx_amd as dmx
    from pyoracle import OracleMap
    lines = [(0.0, 0.0, W, 0.0), (W, 0.0, W, H), (W, H, 0.0, H), (0.0, H, 0.0, 0.0)]
    for k, x in enumerate(range(pitch, W, pitch)):
        lines.append((x, 0.0, x, H - gap) if k % 2 == 0 else (x, gap, x, H))
    lines = np.array(lines, dtype=np.float64)
    region = [0.0, 0.0, float(W), float(H)]
    pm = dmx.PointMap(region, lines, 1.0)
    om = OracleMap(region, 1.0, lines)
    assert pm.make_points(1.5, 1.5) and om.fill(1.5, 1.5)
    rows = pm.rows
    st = np.ascontiguousarray(pm.state(), dtype=np.int32)
    pairs = []
    for x in range(pitch + 1, W - pitch, 3 * pitch):
        a, b = x * rows + 5, (x + 1) * rows + 5
        if st[a] & 2 and st[b] & 2:
            st[a] |= 0x8   # Point::CONTEXTFILLED at an odd PixelRef
            pairs.append((a, b))
    pairs = np.array(pairs, dtype=np.int32)
    N = dmx._native
    N.check(N.lib().dmx_pointmap_set_state(pm.h, N.ptr(st)))
    om2 = OracleMap.from_grid(pm.cols, rows, 1.0, pm.info()["bottom_left"], st)
    return pm, om, om2, pairs


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["tile", "do"])
def test_gpu_contextfilled_links_reference_order_past_64_levels(ctx, monkeypatch, kernel):
    """The reference-order re-run (vga_ordered.hip) keeps as many levels as the radius needs (it kept
    64, so a flagged source whose search went deeper failed the whole call): a radius-100 search on a serpentine
    map deeper than 64 levels, with order-dependent links, equals the reference's order (the oracle)."""
    if kernel == "do":
        monkeypatch.setenv("DMX_VGA_KERNEL", "do")
    pm, om, om2, pairs = _deep_serpentine_links()
    assert len(pairs) >= 8
    pm.set_merges(pairs)
    g = pm.make_graph(ctx)
    om.make_graph(threads=8)
    b = om.graph()
    om2.set_graph(b["bins"], b["runs"])
    om2.set_merges(pairs)
    ref, rlv = om2.vga_global(radius=100, threads=8, levels=True)
    assert rlv[:, 2].max() > 64
    got, lv = g.vga_visual_global(radius=100, levels=True)
    assert ctx.last_stats()["vga_order_reruns"] > 0
    np.testing.assert_array_equal(lv[:, :2], rlv[:, :2])
    np.testing.assert_array_equal(got[:, 5], ref[:, 5])
    assert np.allclose(got, ref, rtol=1e-6, atol=1e-6)
