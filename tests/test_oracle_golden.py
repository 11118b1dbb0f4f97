"""The C restatement (oracle/) against the REAL reference's outputs (tests/golden/, produced by
oracle/_ref/ref_probe = salalib compiled from source).  This pins the oracle before it is trusted
as the GPU checker."""
import numpy as np
import pytest

from golden_io import case_input_lines, load_case, node_digests, roundtrip_runs
from pyoracle import OracleMap

CASES = ["kat", "syn16", "syn32", "gallery", "syn64", "barnsbury"]


def _oracle(meta, threads=8):
    om = OracleMap(meta["region"], meta["spacing"], case_input_lines(meta))
    assert (om.cols, om.rows) == (meta["cols"], meta["rows"])
    assert np.allclose(om.bottom_left, meta["bottom_left"])
    for f in meta["fills"]:
        assert om.fill(*f)
    return om


@pytest.mark.parametrize("name", CASES)
def test_prep_matches_reference(name):
    meta, A = load_case(name)
    om = _oracle(meta)
    counts, pieces = om.cell_lines()
    np.testing.assert_array_equal(counts, A["celllines_n"])
    np.testing.assert_array_equal(pieces, A["celllines"])
    np.testing.assert_array_equal(om.state(), A["state"])


@pytest.mark.parametrize("name", CASES + ["syn256mk"])
def test_makegraph_matches_reference(name):
    meta, A = load_case(name)
    om = _oracle(meta)
    om.make_graph(threads=8)
    assert om.num_nodes == meta["nodes"]
    g = om.graph()
    assert len(g["runs"]) == meta["runs"]
    np.testing.assert_array_equal(g["attrs"].view(np.uint32), A["attrs"].view(np.uint32))
    np.testing.assert_array_equal(g["gridconn"], A["gridconn"])
    if "bins" in A:
        np.testing.assert_array_equal(g["bins"], A["bins"])
        np.testing.assert_array_equal(g["runs"], A["runs"])
    np.testing.assert_array_equal(g["bins"][:, :, 3].sum(axis=1), A["nruns"])
    np.testing.assert_array_equal(node_digests(g["bins"], g["runs"]), A["digests"])


@pytest.mark.parametrize("name", ["kat", "syn16", "syn32", "gallery", "syn64"])
def test_vga_global_matches_reference_bitexact(name):
    meta, A = load_case(name)
    om = _oracle(meta)
    om.make_graph(threads=8)
    out = om.vga_global(threads=8)
    np.testing.assert_array_equal(out.view(np.uint32), A["vga"].view(np.uint32))


@pytest.mark.slow
def test_vga_global_barnsbury_bitexact():
    meta, A = load_case("barnsbury")
    om = _oracle(meta)
    om.make_graph(threads=8)
    out = om.vga_global(threads=8)
    np.testing.assert_array_equal(out.view(np.uint32), A["vga"].view(np.uint32))


@pytest.mark.parametrize("name", ["syn32", "gallery", "syn64"])
def test_graph_file_roundtrip_quirk(name):
    """VGA in the CLI pipeline runs on the re-read .graph whose runs went through the lossy 4-bit
    row shift; the reference's post-round-trip VGA columns (vga_rt) are reproduced by
    applying that transform to the runs."""
    meta, A = load_case(name)
    om = _oracle(meta)
    om.make_graph(threads=8)
    g = om.graph()
    rt = roundtrip_runs(g["bins"], g["runs"])
    om.set_graph(g["bins"], rt)
    out = om.vga_global(threads=8)
    np.testing.assert_array_equal(out.view(np.uint32), A["vga_rt"].view(np.uint32))


def test_kat_connections_from_reference_test():
    """salaTest/testpointmap.cpp:400-451: node iteration order of the 2x2 KAT (PixelRef ints)."""
    expected = {65537: [131073, 131074, 65538], 65538: [131074, 65537, 131073],
                131073: [131074, 65538, 65537], 131074: [65538, 65537, 131073]}
    meta, _ = load_case("kat")
    om = _oracle(meta)
    om.make_graph()
    g = om.graph()
    ro = 0
    st = om.state()
    nodes = [c for c in range(len(st)) if st[c] & 2]
    for k, c in enumerate(nodes):
        x, y = divmod(c, om.rows)
        conn = []
        for b in range(32):
            for r in g["runs"][ro:ro + g["bins"][k, b, 3]]:
                x0, y0, x1, y1 = map(int, r)
                dx = 1 if x1 > x0 else 0
                dy = 0 if y0 == y1 else (1 if x0 == x1 else (1 if y1 > y0 else -1))
                px, py = x0, y0
                while True:
                    conn.append((px << 16) | py)
                    if (px, py) == (x1, y1):
                        break
                    px += dx
                    py += dy
            ro += g["bins"][k, b, 3]
        assert conn == expected[(x << 16) | y]


def test_reference_gallery_attributes_file():
    """testdata/gallery_graph_vga.txt (the reference's own expected Connectivity / moments for
    gallery_empty.graph -pg 0.04 -pp 1.32,7.24) vs the golden probe dump."""
    import os
    from golden_io import GOLDEN
    meta, A = load_case("gallery")
    rows = np.loadtxt(os.path.join(GOLDEN, "gallery_graph_vga.txt"), skiprows=1)
    assert len(rows) == meta["nodes"]
    np.testing.assert_array_equal(rows[:, 3], A["attrs"][:, 0])
    np.testing.assert_allclose(rows[:, 4:6], A["attrs"][:, 1:3], rtol=1e-6)


@pytest.mark.parametrize("name", ["kat", "syn16", "syn32", "syn64", "gallery"])
def test_metric_stepdepth_matches_reference_bitexact(name):
    """VGAMetricDepth::run restatement vs the reference's STEPDEPTH -sdt metric columns
    (ref_probe --stepdepth, runStepDepth semantics: setCurSel at each point)."""
    meta, A = load_case(name)
    om = _oracle(meta)
    om.make_graph(threads=8)
    sel = A["stepdepth_sel"]                         # std::set<int> of PixelRef ints
    cells = (sel >> 16) * meta["rows"] + (sel & 0xFFFF)
    got = om.metric_stepdepth(cells)
    np.testing.assert_array_equal(got.view(np.uint32), A["stepdepth"].view(np.uint32))
    assert (A["stepdepth"][:, 1] >= 0).sum() > 0


@pytest.mark.parametrize("name", ["kat", "syn16", "syn32", "syn64", "gallery", "syn128sd"])
def test_visual_stepdepth_matches_reference_bitexact(name):
    """VGAVisualGlobalDepth::run restatement vs the reference's STEPDEPTH -sdt visual column
    (ref_probe --stepdepth runs both step types on the same setCurSel selection)."""
    meta, A = load_case(name)
    if "vstepdepth" not in A:
        pytest.skip("fixture without visual step depth")
    om = _oracle(meta)
    om.make_graph(threads=8)
    sel = A["stepdepth_sel"]
    cells = (sel >> 16) * meta["rows"] + (sel & 0xFFFF)
    got = om.visual_stepdepth(cells)
    np.testing.assert_array_equal(got.view(np.uint32), A["vstepdepth"].view(np.uint32))
    assert (A["vstepdepth"] >= 1).sum() > 0


@pytest.mark.parametrize("name", ["kat", "syn16", "syn32", "syn64", "gallery"])
def test_vga_local_matches_reference_bitexact(name):
    """VGAVisualLocal::run restatement vs the reference's -vl columns (ref_probe --vlocal,
    tests/golden/make_golden_vga_modes.py): clustering coefficient, control, controllability."""
    import os
    from golden_io import GOLDEN
    path = os.path.join(GOLDEN, name + "_vlocal.npy")
    if not os.path.exists(path):
        pytest.skip("no -vl fixture for this case (the reference takes hours on it)")
    meta, A = load_case(name)
    om = _oracle(meta)
    om.make_graph(threads=8)
    want = np.load(path)
    got = om.vga_local(threads=8)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    assert (want[:, 0] >= 0).sum() > 0


VMETRIC_CASES = [("kat", -1.0), ("syn16", -1.0), ("syn32", -1.0), ("syn32", 10.0), ("gallery", -1.0)]


def _vmetric_fixture(name, radius):
    import os
    from golden_io import GOLDEN
    return os.path.join(GOLDEN, name + "_vmetric" + ("" if radius < 0 else "_r%g" % radius) + ".npy")


@pytest.mark.parametrize("name,radius", VMETRIC_CASES)
def test_vga_metric_matches_reference_bitexact(name, radius):
    """VGAMetric::run restatement vs the reference's -vm metric columns (ref_probe --vmetric,
    tests/golden/make_golden_vga_modes.py): mean angle, mean path distance, mean straight-line
    distance, node count -- float totals accumulated in the reference's pop order."""
    meta, A = load_case(name)
    om = _oracle(meta)
    om.make_graph(threads=8)
    want = np.load(_vmetric_fixture(name, radius))
    got = om.vga_metric(radius=radius, threads=8)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("name,radius", [("kat", -1.0), ("syn16", -1.0), ("syn32", -1.0), ("syn32", 1.5),
                                         ("gallery", -1.0)])
def test_vga_angular_matches_reference_bitexact(name, radius):
    """VGAAngular::run restatement vs the reference's -vm angular columns (ref_probe --vangular)."""
    import os
    from golden_io import GOLDEN
    meta, A = load_case(name)
    om = _oracle(meta)
    om.make_graph(threads=8)
    want = np.load(os.path.join(GOLDEN, name + "_vangular" + ("" if radius < 0 else "_r%g" % radius) + ".npy"))
    got = om.vga_angular(radius=radius, threads=8)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("name", ["kat", "syn16", "syn32", "syn64", "gallery", "barnsbury"])
def test_angular_stepdepth_matches_reference_bitexact(name):
    """VGAAngularDepth::run restatement vs the reference's STEPDEPTH -sdt angular column on the
    same selection as the metric / visual step depth fixtures."""
    import os
    from golden_io import GOLDEN
    meta, A = load_case(name)
    om = _oracle(meta)
    om.make_graph(threads=8)
    sel = A["stepdepth_sel"]
    cells = (sel >> 16) * meta["rows"] + (sel & 0xFFFF)
    want = np.load(os.path.join(GOLDEN, name + "_astepdepth.npy"))
    np.testing.assert_array_equal(om.angular_stepdepth(cells).view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("name", ["syn32", "gallery", "syn64"])
def test_batched_stepdepth_schedule_matches_reference(name):
    """The batched metric step-depth schedule (distance windows, certified single winners, ambiguous
    cells folded in pop order), modelled in pure Python (tests/sd_batched_model.py), reproduces the
    reference's VGAMetricDepth columns bit-for-bit.  Pins the schedule's mathematics on the CPU; the
    GPU tests then pin the kernels to the serial pop-order kernel."""
    from sd_batched_model import batched_metric_stepdepth
    meta, A = load_case(name)
    om = _oracle(meta)
    om.make_graph(threads=8)
    gr = om.graph()
    sel = A["stepdepth_sel"]
    cells = (sel >> 16) * meta["rows"] + (sel & 0xFFFF)
    got, stats = batched_metric_stepdepth(om.state(), meta["rows"], meta["cols"], gr["bins"], gr["runs"], cells,
                                          meta["spacing"])
    assert stats["batches"] > 1
    np.testing.assert_array_equal(got.view(np.uint32), A["stepdepth"].view(np.uint32))
