"""Context-filled maps: PointMap::makePoints(p, fill_type) with the GUI's SEMIFILL and AUGMENT modes
(salalib/pointdata.cpp:402-481, depthmapX/views/depthmapview/depthmapview.h:75), and every analysis on
maps that carry Point::CONTEXTFILLED cells.

The clauses being pinned:
  VGA global         vgavisualglobal.cpp:75   context-filled odd sources are skipped
                     vgavisualglobal.cpp:110  ... and not expanded under a radius
  visual step depth  vgavisualglobaldepth.cpp:52  context-filled odd cells are not expanded (but level 0)
  VGA local          vgavisuallocal.cpp:43    context-filled odd sources are skipped
Fixtures (tests/golden/make_golden_graphfiles.py, the reference built from source): semi_gallery (one SEMIFILL
seed), mixed_gallery (plus a block of FULL cells drawn with the pencil tool, PointMap::fillPoint), mixed_made
(the reference's makeGraph of it) and mixed_link (plus merge links from LINK mode: a context-filled odd cell to
a full cell, a context-filled even cell to an odd one).  The .graph regression cases on them (semi_*, mixed_*,
link_*) run through dmxcli in test_graphfile.py; here: the fill itself, the oracle pinned on every case, the
three BFS kernels on the reference's graph, and the order dependence of link_vis_global_3, which the engine
answers in the reference's own level order (kernels/vga_ordered.hip).
"""
import ctypes
import json
import lzma
import os

import numpy as np
import pytest

import graphfile_util as gu

HERE = os.path.dirname(os.path.abspath(__file__))
GF = os.path.join(HERE, "golden", "graphfiles")
CASES = json.load(open(os.path.join(GF, "cases.json")))
VGA_VIS = ["Visual Entropy", "Visual Integration [HH]", "Visual Integration [P-value]", "Visual Integration [Tekl]",
           "Visual Mean Depth", "Visual Node Count", "Visual Relativised Entropy"]
SD_METRIC = ["Metric Step Shortest-Path Angle", "Metric Step Shortest-Path Length", "Metric Straight-Line Distance"]
VGA_LOCAL = ["Visual Clustering Coefficient", "Visual Control", "Visual Controllability"]
EXACT = {"Visual Node Count", "Metric Node Count", "Angular Node Count", "Visual Step Depth",
         "Metric Step Shortest-Path Length", "Metric Straight-Line Distance", "Angular Step Depth",
         "Angular Total Depth", "Visual Clustering Coefficient", "Visual Control", "Visual Controllability"}
SEMI_SEED = (1.32, 7.24)


def _input(tmp_path, name):
    dst = os.path.join(str(tmp_path), name)
    if not os.path.exists(dst):
        with lzma.open(os.path.join(GF, "inputs", name + ".xz")) as f, open(dst, "wb") as o:
            o.write(f.read())
    return dst


def _ref_cols(case):
    return np.load(os.path.join(GF, case + "_cols.npz"), allow_pickle=False)


def _compare(got, ref, cols):
    for j, col in enumerate(cols):
        a = got[:, j] if got.ndim == 2 else got
        r = ref[col]
        if col.split(" R")[0] in EXACT:
            assert np.array_equal(a.view(np.uint32), r.view(np.uint32)), (col, np.flatnonzero(a != r)[:8])
        else:
            fin = np.isfinite(r)
            assert np.array_equal(np.isfinite(a), fin), col
            assert np.allclose(a[fin], r[fin], rtol=1e-6, atol=1e-6), (col, float(np.abs(a[fin] - r[fin]).max()))


def _drawing(path):
    """region and drawing lines of a .graph (what PointMap::blockLines reads)."""
    from depthmapx_amd import _native as N
    lib = N.lib()
    h = ctypes.c_void_p()
    N.check(lib.dmx_graphfile_read(path.encode(), ctypes.byref(h)))
    try:
        n = ctypes.c_int64()
        region = np.zeros(4)
        N.check(lib.dmx_graphfile_info(h, None, None, N.ptr(region), ctypes.byref(n), None, None))
        lines = np.zeros((n.value, 4))
        N.check(lib.dmx_graphfile_lines(h, N.ptr(lines)))
    finally:
        lib.dmx_graphfile_free(h)
    return region, lines


def _oracle_for(pmd):
    from pyoracle import OracleMap
    om = OracleMap.from_grid(pmd["cols"], pmd["rows"], pmd["spacing"], pmd["bottom_left"], pmd["state"])
    om.set_graph(pmd["bins"], pmd["runs"])
    om.set_merges(pmd["merges"])
    return om


def _cell(pmd, x, y):
    s, (bx, by) = pmd["spacing"], pmd["bottom_left"]
    return int(np.floor((x - bx + s / 2.0) / s)) * pmd["rows"] + int(np.floor((y - by + s / 2.0) / s))


# ---------------------------------------------------------------- the fill (host model, CPU)
def test_fixtures_carry_contextfilled_cells(tmp_path):
    """semi_gallery is context-filled throughout; mixed_gallery also has full cells; mixed_link has merge links
    on a context-filled odd cell and between a context-filled even and odd cell."""
    semi = gu.load_pointmap(_input(tmp_path, "semi_gallery.graph"))
    filled = (semi["state"] & 2) != 0
    assert filled.sum() > 4000 and ((semi["state"][filled] & 8) != 0).all()
    mixed = gu.load_pointmap(_input(tmp_path, "mixed_gallery.graph"))
    f = (mixed["state"] & 2) != 0
    full = f & ((mixed["state"] & 8) == 0)
    assert 50 < full.sum() < f.sum()
    link = gu.load_pointmap(_input(tmp_path, "mixed_link.graph"))
    assert len(link["merges"]) == 2
    rows = link["rows"]
    kinds = set()
    for a, b in link["merges"]:
        for c in (a, b):
            x, y = divmod(int(c), rows)
            cf = bool(link["state"][c] & 8)
            kinds.add((cf, cf and (x % 2 or y % 2)))
    assert (True, True) in kinds and (False, False) in kinds and (True, False) in kinds


def test_semifill_states_match_reference(tmp_path):
    """dmx_pointmap_make_points(fill_type 1) on the gallery grid sets the states the reference's SEMIFILL did
    (FILLED | CONTEXTFILLED, EDGE in expand order, BLOCKED kept) and counts the filled points as it does."""
    import depthmapx_amd as dmx
    region, lines = _drawing(_input(tmp_path, "gallery_empty.graph"))
    pm = dmx.PointMap(region, lines, 0.04)
    assert pm.make_points(*SEMI_SEED, fill_type=pm.SEMIFILL)
    path = _input(tmp_path, "semi_gallery.graph")
    ref = gu.load_pointmap(path)
    assert np.array_equal(pm.state(), ref["state"])
    assert pm.info()["filled"] == gu.parse(open(path, "rb").read())["maps"][0]["filled"]
    # a second fill of an already filled cell is refused, as makePoints returns false
    assert not pm.make_points(*SEMI_SEED, fill_type=pm.SEMIFILL)


def test_semifill_oracle_matches_reference(tmp_path):
    from pyoracle import OracleMap
    region, lines = _drawing(_input(tmp_path, "gallery_empty.graph"))
    om = OracleMap(region, 0.04, lines)
    assert om.fill(*SEMI_SEED, fill_type=1)
    assert np.array_equal(om.state(), gu.load_pointmap(_input(tmp_path, "semi_gallery.graph"))["state"])


def test_augment_fill_refused_exactly_where_the_reference_never_ends(tmp_path):
    """AUGMENT sets Point::AUGMENTED without FILLED, and expand stops only at FILLED cells
    (pointdata.cpp:489), so the reference's loop never ends once the seed expands anywhere (the reference
    built here runs until killed on the gallery; the oracle's literal loop is cut and says so).  The engine
    refuses exactly those fills, and sets the seed alone where the seed cannot expand."""
    import depthmapx_amd as dmx
    from pyoracle import OracleMap
    region, lines = _drawing(_input(tmp_path, "gallery_empty.graph"))
    pm = dmx.PointMap(region, lines, 0.04)
    om = OracleMap(region, 0.04, lines)
    with pytest.raises(dmx.DmxError) as e:
        pm.make_points(*SEMI_SEED, fill_type=pm.AUGMENT)
    assert e.value.status == -5
    assert om.fill(*SEMI_SEED, fill_type=2) is None
    assert not (pm.state() & 0x8002).any()
    # a seed boxed into its own cell: the fill ends at once in the reference
    box = np.array([[4.6, 4.6, 5.4, 4.6], [5.4, 4.6, 5.4, 5.4], [5.4, 5.4, 4.6, 5.4], [4.6, 5.4, 4.6, 4.6],
                    [0.0, 0.0, 10.0, 0.0]], dtype=np.float64)
    reg = [0.0, 0.0, 10.0, 10.0]
    pm2, om2 = dmx.PointMap(reg, box, 1.0), OracleMap(reg, 1.0, box)
    assert pm2.make_points(5.0, 5.0, fill_type=pm2.AUGMENT)
    assert om2.fill(5.0, 5.0, fill_type=2) is True
    st = pm2.state()
    assert np.array_equal(st, om2.state())
    assert ((st & 0x8000) != 0).sum() == 1 and not (st & 2).any()
    assert pm2.info()["filled"] == 1      # m_filled_point_count++ (pointdata.cpp:444)
    # a full fill from a neighbouring region is unaffected; the augmented cell can be filled over later
    assert pm2.make_points(1.0, 1.0) and om2.fill(1.0, 1.0)
    assert np.array_equal(pm2.state(), om2.state())
    with pytest.raises(dmx.DmxError):
        pm2.make_points(1.0, 1.0, fill_type=7)


# ---------------------------------------------------------------- the oracle pinned on every case (CPU)
SEMI_CASES = [n for n in CASES if n.split("_")[0] in ("semi", "mixed", "link") and CASES[n]["columns"]]


def _made_graph(tmp_path, case):
    """The graph a case analyses: the reference's own makeGraph output of the case's map."""
    inp = CASES[case]["input"]
    if inp.startswith("@"):
        src = CASES[inp[1:]]["input"]
        assert CASES[inp[1:]]["args"] == ["-m", "VISPREP", "-pm"], case
        # semi_make / mixed_make are byte-identical to the reference's (test_graphfile); the reference made
        # mixed_made itself, semi is made here by the oracle from the reference's fill
        return src
    return inp


def _oracle_map(tmp_path, case):
    g = _made_graph(tmp_path, case)
    if g == "semi_gallery.graph":   # the reference's fill; make the graph with the oracle
        from pyoracle import OracleMap
        pmd = gu.load_pointmap(_input(tmp_path, g))
        region, lines = _drawing(_input(tmp_path, "gallery_empty.graph"))
        om = OracleMap(region, 0.04, lines)
        assert om.fill(*SEMI_SEED, fill_type=1)
        assert np.array_equal(om.state(), pmd["state"])
        om.make_graph(threads=8)
        return om, pmd
    name = "mixed_made.graph" if g == "mixed_gallery.graph" else g
    pmd = gu.load_pointmap(_input(tmp_path, name))
    return _oracle_for(pmd), pmd


def _oracle_run(om, pmd, args):
    a, i = {}, 0
    while i < len(args):   # flags with a value; -s, -vg, -vl stand alone
        if args[i] in ("-m", "-vm", "-vr", "-sdt", "-sdp"):
            a[args[i]] = args[i + 1]
            i += 2
        else:
            i += 1
    if a["-m"] == "STEPDEPTH":
        x, y = (float(v) for v in a["-sdp"].split(","))
        sel = [_cell(pmd, x, y)]
        return {"visual": om.visual_stepdepth, "metric": om.metric_stepdepth,
                "angular": om.angular_stepdepth}[a["-sdt"]](sel)
    if a["-vm"] == "visibility":
        if "-vl" in args:
            return om.vga_local(threads=8)
        r = a["-vr"]
        return om.vga_global(radius=-1 if r == "n" else int(r), threads=8)
    if a["-vm"] == "metric":
        return om.vga_metric(threads=8)
    return om.vga_angular(threads=8)


@pytest.mark.parametrize("case", SEMI_CASES)
def test_oracle_matches_reference_on_contextfilled_case(tmp_path, case):
    om, pmd = _oracle_map(tmp_path, case)
    args = CASES[case]["args"]
    out = _oracle_run(om, pmd, args)
    cols = CASES[case]["columns"]
    if "-s" in args:   # simple mode: the HH column only
        out = out[:, 1]
    _compare(out, _ref_cols(case), cols)


def _both_orders(om, pmd, args):
    """The oracle's result with the reference's pop order (back to front) and front to back, with the merge
    links and without them."""
    import pyoracle
    try:
        pyoracle.set_pop_forward(True)
        fwd = _oracle_run(om, pmd, args)
        om.set_merges(np.zeros((0, 2), dtype=np.int32))
        fwd_nolink = _oracle_run(om, pmd, args)
        pyoracle.set_pop_forward(False)
        back_nolink = _oracle_run(om, pmd, args)
        om.set_merges(pmd["merges"])
        back = _oracle_run(om, pmd, args)
    finally:
        pyoracle.set_pop_forward(False)
    return fwd, back, fwd_nolink, back_nolink


def test_order_dependent_case_depends_on_the_pop_order(tmp_path):
    """What link_vis_global_3 computes changes with the order the reference pops a level in: the oracle with
    the reference's order (back to front) reproduces the reference's columns, front to back it does not (a
    source finds a context-filled odd cell and its linked full cell at one level: popped first, the full
    cell extracts its partner, which is then never counted).  On the same map without the links the order
    changes nothing.  The engine runs such sources in the reference's order (test_graphfile runs the case and
    compares it with the reference's output; test_merge_links covers seeded maps)."""
    case = "link_vis_global_3"
    assert not CASES[case].get("refused")
    om, pmd = _oracle_map(tmp_path, case)
    fwd, back, fwd_nolink, back_nolink = _both_orders(om, pmd, CASES[case]["args"])
    _compare(back, _ref_cols(case), CASES[case]["columns"])
    assert np.array_equal(fwd_nolink.view(np.uint32), back_nolink.view(np.uint32))
    assert not np.array_equal(fwd.view(np.uint32), back.view(np.uint32))


def test_visual_step_depth_with_contextfilled_links_is_order_free_here(tmp_path):
    """link_sd_visual: both links have their two ends at one level, but extracting the unexpanded
    context-filled end finds no cell that is not reached at the next level anyway, so both pop orders give
    the reference's columns -- the case the GPU search checks before it answers (vsd_pending_kernel) and
    then runs (test_graphfile)."""
    case = "link_sd_visual"
    assert not CASES[case].get("refused")
    om, pmd = _oracle_map(tmp_path, case)
    fwd, back, _, _ = _both_orders(om, pmd, CASES[case]["args"])
    _compare(back, _ref_cols(case), CASES[case]["columns"])
    _compare(fwd, _ref_cols(case), CASES[case]["columns"])


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_semifill_states_match_reference(ctx, tmp_path):
    """The GPU flood fill (dmx_pointmap_make_points_device, fill_type 1) leaves the reference's states."""
    import depthmapx_amd as dmx
    region, lines = _drawing(_input(tmp_path, "gallery_empty.graph"))
    pm = dmx.PointMap(region, lines, 0.04)
    assert pm.make_points(*SEMI_SEED, ctx=ctx, fill_type=pm.SEMIFILL)
    path = _input(tmp_path, "semi_gallery.graph")
    assert np.array_equal(pm.state(), gu.load_pointmap(path)["state"])
    assert pm.info()["filled"] == gu.parse(open(path, "rb").read())["maps"][0]["filled"]


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["tile", "tile_fsc", "do", "topdown"])
@pytest.mark.parametrize("case", ["mixed_vis_global_n", "mixed_vis_global_3", "semi_vis_global_3",
                                  "link_vis_global_n"])
def test_gpu_vga_global_kernels_on_contextfilled_maps(ctx, monkeypatch, tmp_path, kernel, case):
    """Every BFS kernel family on the reference's own graph of a context-filled map, against the columns the
    reference wrote (the regression cases run the default kernel through dmxcli).  tile_fsc: the tile kernel
    with per-tile column summaries, run twice -- the radius-3 cases have small frontiers that take the
    top-down levels, where a leader-thread reset of the level counters once raced the next level's first
    appends (tens of sources a run lost their frontier)."""
    from depthmapx_amd import graphio
    if kernel == "tile_fsc":
        monkeypatch.setenv("DMX_VGA_RB", "0")
    elif kernel != "tile":
        monkeypatch.setenv("DMX_VGA_KERNEL", kernel)
    g = _made_graph(tmp_path, case)
    if g == "semi_gallery.graph":
        import depthmapx_amd as dmx
        region, lines = _drawing(_input(tmp_path, "gallery_empty.graph"))
        pm = dmx.PointMap(region, lines, 0.04)
        assert pm.make_points(*SEMI_SEED, fill_type=pm.SEMIFILL)
        graph = pm.make_graph(ctx)
    else:
        name = "mixed_made.graph" if g == "mixed_gallery.graph" else g
        path = _input(tmp_path, name)
        region, _ = _drawing(path)
        pmd_blob = _chunk_bytes(path)
        _, graph = graphio.load_chunk(ctx, pmd_blob, region)
    r = CASES[case]["args"][CASES[case]["args"].index("-vr") + 1]
    for _ in range(2 if kernel == "tile_fsc" else 1):
        got = graph.vga_visual_global(radius=-1 if r == "n" else int(r))
        _compare(got, _ref_cols(case), CASES[case]["columns"])


@pytest.mark.gpu
@pytest.mark.parametrize("topdown", [False, True])
@pytest.mark.parametrize("case", ["mixed_sd_visual", "mixed_sd_visual_full_seed", "semi_sd_visual"])
def test_gpu_visual_step_depth_on_contextfilled_maps(ctx, monkeypatch, tmp_path, topdown, case):
    from depthmapx_amd import graphio
    if topdown:
        monkeypatch.setenv("DMX_VSD_TOPDOWN", "1")
    g = _made_graph(tmp_path, case)
    if g == "semi_gallery.graph":
        import depthmapx_amd as dmx
        region, lines = _drawing(_input(tmp_path, "gallery_empty.graph"))
        pm = dmx.PointMap(region, lines, 0.04)
        assert pm.make_points(*SEMI_SEED, fill_type=pm.SEMIFILL)
        graph = pm.make_graph(ctx)
        pmd = {"spacing": 0.04, "bottom_left": pm.info()["bottom_left"], "rows": pm.rows}
    else:
        path = _input(tmp_path, "mixed_made.graph")
        region, _ = _drawing(path)
        _, graph = graphio.load_chunk(ctx, _chunk_bytes(path), region)
        pmd = gu.load_pointmap(path)
    x, y = (float(v) for v in CASES[case]["args"][-1].split(","))
    got = graph.visual_step_depth(cells=[_cell(pmd, x, y)])
    _compare(got, _ref_cols(case), ["Visual Step Depth"])


def _chunk_bytes(path):
    from depthmapx_amd import _native as N
    lib = N.lib()
    h = ctypes.c_void_p()
    N.check(lib.dmx_graphfile_read(path.encode(), ctypes.byref(h)))
    try:
        npm, disp = ctypes.c_int32(), ctypes.c_int32()
        N.check(lib.dmx_graphfile_info(h, None, None, None, None, ctypes.byref(npm), ctypes.byref(disp)))
        buf, size = ctypes.POINTER(ctypes.c_uint8)(), ctypes.c_int64()
        N.check(lib.dmx_graphfile_pointmap(h, disp.value, ctypes.byref(buf), ctypes.byref(size)))
        return ctypes.string_at(buf, size.value)
    finally:
        lib.dmx_graphfile_free(h)
