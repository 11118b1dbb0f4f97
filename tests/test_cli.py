"""dmxcli: the depthmapXcli mode-parser surface for VISPREP / VGA / STEPDEPTH
(depthmapXcli/commandlineparser.cpp:51-142, visprepparser.cpp:26-172, vgaparser.cpp:29-106,
stepdepthparser.cpp:26-100, main.cpp:47-52).  CPU tests cover flag validation (no GPU needed: a
failing parse never reaches the device); the GPU test runs the whole CLI pipeline."""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "depthmapx_amd", "_lib", "dmxcli")
GOLDEN = os.path.join(REPO, "tests", "golden")


def run(*args):
    p = subprocess.run([CLI] + list(args), capture_output=True, text=True)
    return p.returncode, p.stdout


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(CLI):
        from depthmapx_amd import build
        build.build()


@pytest.mark.parametrize("args,message", [
    ([], "No commandline parameters provided - don't know what to do"),
    (["-m", "NOPE", "-f", "a", "-o", "b"], "Invalid mode: NOPE"),
    (["-m", "VISPREP", "-m", "VGA"], "-m can only be used once"),
    (["-f", "a", "-o", "b"], "-m for mode is required"),
    (["-m", "VGA", "-o", "b"], "-f for input file is required"),
    (["-m", "VGA", "-f", "a"], "-o for output file is required"),
    (["-m", "VISPREP", "-f", "a", "-o", "b"], "Nothing to do"),
    (["-m", "VISPREP", "-f", "a", "-o", "b", "-pg", "1", "-pg", "2"], "-pg can only be used once"),
    (["-m", "VISPREP", "-f", "a", "-o", "b", "-pg", "0"], "-pg must be a number >0, got 0"),
    (["-m", "VISPREP", "-f", "a", "-o", "b", "-pg", "1", "-pm"],
     "Creating a graph for an unfilled grid is not possible. Either -pp or -pf must be given"),
    (["-m", "VISPREP", "-f", "a", "-o", "b", "-pp", "1a,2"],
     "Invalid fill point provided (1a,2). Should only contain digits dots and commas"),
    (["-m", "VISPREP", "-f", "a", "-o", "b", "-pm", "-pu"], "-pu cannot be used together with -pm"),
    (["-m", "VISPREP", "-f", "a", "-o", "b", "-pr", "0", "-pm"],
     "Restricted visibility of '0' makes no sense, use a positive number or -1 for unrestricted"),
    (["-m", "VISPREP", "-f", "a", "-o", "b", "-pg"], "-pg requires an argument"),
    (["-m", "VGA", "-f", "a", "-o", "b", "-vm", "visibility", "-vg"],
     "Global measures in VGA/visibility analysis require a radius, use -vr <radius>"),
    (["-m", "VGA", "-f", "a", "-o", "b", "-vm", "visibility", "-vg", "-vr", "x"],
     "Radius must be a positive integer number or n, got x"),
    (["-m", "VGA", "-f", "a", "-o", "b", "-vm", "nope"], "Invalid VGA mode: nope"),
    (["-m", "VGA", "-f", "a", "-o", "b", "-vm", "metric"], "Metric vga requires a radius, use -vr <radius>"),
    (["-m", "STEPDEPTH", "-f", "a", "-o", "b", "-sdt", "metric"], "Either -sdp or -sdf must be given"),
    (["-m", "STEPDEPTH", "-f", "a", "-o", "b", "-sdp", "1,1"], "Step depth type (-sdt) must be provided"),
    (["-m", "STEPDEPTH", "-f", "a", "-o", "b", "-sdp", "1,1", "-sdt", "odd"], "Invalid step type: odd"),
])
def test_parser_messages_like_depthmapxcli(args, message):
    rc, out = run(*args)
    assert rc == 255, out   # main returns -1
    assert out.splitlines() == [message, "Type 'depthmapXcli -h' for help"]


def test_help_and_missing_file(tmp_path):
    rc, out = run("-h")
    assert rc == 0 and "VISPREP" in out
    rc, out = run("-m", "VISPREP", "-f", str(tmp_path / "none.csv"), "-o", str(tmp_path / "o.dmxg"), "-pg", "1",
                  "-pp", "0.5,0.5", "-pm")
    assert rc == 255 and "Failed to load graph from file" in out


def test_remaking_a_processed_map_is_an_error(tmp_path):
    """VISPREP -pm on a map that already has a graph: the reference's sparkGraph2 re-adds attribute rows
    that exist and AttributeTable::addRow throws a pointer (`throw new std::invalid_argument("Duplicate
    key")`, salalib/attributetable.cpp:278) that main's catch (std::exception&) (depthmapXcli/main.cpp:47)
    does not catch, so depthmapXcli aborts (SIGABRT; oracle/_ref/ref_cli reproduces it in this container).
    dmxcli reports an error with the CLI's exit code instead, before touching the GPU, and writes nothing."""
    import lzma
    src = tmp_path / "gallery_connected.graph"
    with lzma.open(os.path.join(GOLDEN, "graphfiles", "inputs", "gallery_connected.graph.xz")) as f:
        src.write_bytes(f.read())
    out = tmp_path / "out.graph"
    rc, msg = run("-f", str(src), "-o", str(out), "-m", "VISPREP", "-pm")
    assert rc == 255 and "already has a graph" in msg and "Type 'depthmapXcli -h' for help" in msg, msg
    assert not out.exists()
    ref_cli = os.path.join(REPO, "oracle", "_ref", "ref_cli")
    if os.path.exists(ref_cli):
        p = subprocess.run([ref_cli, "-f", str(src), "-o", str(tmp_path / "ref.graph"), "-m", "VISPREP", "-pm"],
                           capture_output=True, text=True)
        assert p.returncode == -6 and "invalid_argument" in p.stderr


@pytest.mark.gpu
def test_cli_pipeline_matches_reference(tmp_path):
    """VISPREP -pg 1 -pp 0.5,0.5 -pm -> VGA -vm visibility -vg -vr n -> STEPDEPTH -sdt metric on the
    synthetic 32^2 drawing: the VISPREP PointMap chunk is byte-identical to the reference's, the
    VGA columns equal the reference CLI's (VGA on the re-read graph), step depth matches the C
    restatement on the same re-read graph, and the -t CSV carries the reference's action names."""
    import hashlib
    import sys
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from depthmapx_amd import graphio
    from golden_io import load_case
    from pyoracle import OracleMap
    meta, A = load_case("syn32")
    src = os.path.join(GOLDEN, "inputs", "syn32.csv")
    g1, g2, g3 = (str(tmp_path / n) for n in ("a.dmxg", "b.dmxg", "c.dmxg"))
    t1 = str(tmp_path / "t1.csv")
    rc, out = run("-m", "VISPREP", "-f", src, "-o", g1, "-pg", "1", "-pp", "0.5,0.5", "-pm", "-t", t1)
    assert rc == 0, out
    assert [l.split(",")[0] for l in open(t1).read().splitlines()] == [
        '"action"', '"Load graph file"', '"Setting grid"', '"Filling grid"', '"Making graph"', '"Writing graph"']

    def chunk(path):
        b = open(path, "rb").read()
        nl = int(np.frombuffer(b[40:48], np.int64)[0])
        o = 48 + nl * 32 + 1
        n = int(np.frombuffer(b[o:o + 8], np.int64)[0])
        return b[o + 8:o + 8 + n]
    c1 = chunk(g1)
    assert hashlib.sha256(c1).digest() == A["pm_chunk_sha256"].tobytes()
    rc, out = run("-m", "VGA", "-f", g1, "-o", g2, "-vm", "visibility", "-vg", "-vr", "n")
    assert rc == 0, out
    doc = graphio.read_chunk(chunk(g2))
    names = [c[0] for c in doc["columns"]]
    assert names[:3] == ["Connectivity", "Point First Moment", "Point Second Moment"]
    from depthmapx_amd import VGA_COLUMNS
    assert names[3:] == VGA_COLUMNS
    got = np.stack([c[1] for c in doc["columns"][3:]], axis=1)
    want = A["vga_rt"]
    assert (np.abs(got.astype(np.float64) - want) <= 1e-6 * np.maximum(1.0, np.abs(want))).all()
    rc, out = run("-m", "STEPDEPTH", "-f", g2, "-o", g3, "-sdt", "metric", "-sdp", "16.5,16.5")
    assert rc == 0, out
    d3 = graphio.read_chunk(chunk(g3))
    cols = {c[0]: c[1] for c in d3["columns"]}
    om = OracleMap(meta["region"], meta["spacing"], np.load(os.path.join(GOLDEN, meta["lines_npy"])))
    for f in meta["fills"]:
        om.fill(*f)
    om.make_graph()
    om.set_graph(doc["bins"], doc["runs"])
    rows = meta["rows"]
    # PointMap::pixelate(16.5, 16.5) at spacing 1 from bottom-left (0, 0): floor(16.5 + 0.5) = 17
    ref = om.metric_stepdepth(np.array([17 * rows + 17], np.int32))
    np.testing.assert_array_equal(cols["Metric Step Shortest-Path Length"], ref[:, 1])
    np.testing.assert_array_equal(cols["Metric Straight-Line Distance"], ref[:, 2])
    assert np.allclose(cols["Metric Step Shortest-Path Angle"], ref[:, 0], rtol=1e-6, atol=1e-6)
    # STEPDEPTH -sdt visual on the same graph (VGAVisualGlobalDepth::run): one column, -1 unreached
    g4 = str(tmp_path / "d.dmxg")
    rc, out = run("-m", "STEPDEPTH", "-f", g2, "-o", g4, "-sdt", "visual", "-sdp", "16.5,16.5")
    assert rc == 0, out
    cols4 = {c[0]: c[1] for c in graphio.read_chunk(chunk(g4))["columns"]}
    want = om.visual_stepdepth(np.array([17 * rows + 17], np.int32))
    np.testing.assert_array_equal(cols4["Visual Step Depth"], want)


@pytest.mark.gpu
def test_cli_vga_local_and_global(tmp_path):
    """VGA -vm visibility -vl -vg -vr n: the local columns come first (VGAVisualLocal runs before
    VGAVisualGlobal, mgraph.cpp:349-356) and equal the C restatement on the re-read graph; the
    global columns equal the reference CLI's."""
    from depthmapx_amd import VGA_COLUMNS, VGA_LOCAL_COLUMNS, graphio
    from golden_io import load_case
    from pyoracle import OracleMap
    meta, A = load_case("syn32")
    src = os.path.join(GOLDEN, "inputs", "syn32.csv")
    g1, g2 = str(tmp_path / "a.dmxg"), str(tmp_path / "b.dmxg")
    rc, out = run("-m", "VISPREP", "-f", src, "-o", g1, "-pg", "1", "-pp", "0.5,0.5", "-pm")
    assert rc == 0, out
    rc, out = run("-m", "VGA", "-f", g1, "-o", g2, "-vm", "visibility", "-vl", "-vg", "-vr", "n")
    assert rc == 0, out

    def chunk(path):
        b = open(path, "rb").read()
        nl = int(np.frombuffer(b[40:48], np.int64)[0])
        o = 48 + nl * 32 + 1
        n = int(np.frombuffer(b[o:o + 8], np.int64)[0])
        return b[o + 8:o + 8 + n]
    doc = graphio.read_chunk(chunk(g2))
    names = [c[0] for c in doc["columns"]]
    assert names == ["Connectivity", "Point First Moment", "Point Second Moment"] + VGA_LOCAL_COLUMNS + VGA_COLUMNS
    om = OracleMap(meta["region"], meta["spacing"], np.load(os.path.join(GOLDEN, meta["lines_npy"])))
    for f in meta["fills"]:
        om.fill(*f)
    om.make_graph()
    om.set_graph(doc["bins"], doc["runs"])
    want = om.vga_local(threads=8)
    got = np.stack([c[1] for c in doc["columns"][3:6]], axis=1)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    glob = np.stack([c[1] for c in doc["columns"][6:]], axis=1)
    assert (np.abs(glob.astype(np.float64) - A["vga_rt"]) <= 1e-6 * np.maximum(1.0, np.abs(A["vga_rt"]))).all()


@pytest.mark.gpu
@pytest.mark.parametrize("radius", ["n", "10"])
def test_cli_vga_metric(tmp_path, radius):
    """VGA -vm metric -vr <n|r> (runVga METRIC branch -> VGAMetric::run): four columns with the
    reference's radius suffix, equal to the C restatement on the re-read graph."""
    from depthmapx_amd import VGA_METRIC_COLUMNS, graphio
    from golden_io import load_case
    from pyoracle import OracleMap
    meta, A = load_case("syn32")
    src = os.path.join(GOLDEN, "inputs", "syn32.csv")
    g1, g2 = str(tmp_path / "a.dmxg"), str(tmp_path / "b.dmxg")
    rc, out = run("-m", "VISPREP", "-f", src, "-o", g1, "-pg", "1", "-pp", "0.5,0.5", "-pm")
    assert rc == 0, out
    rc, out = run("-m", "VGA", "-f", g1, "-o", g2, "-vm", "metric", "-vr", radius)
    assert rc == 0, out

    def chunk(path):
        b = open(path, "rb").read()
        nl = int(np.frombuffer(b[40:48], np.int64)[0])
        o = 48 + nl * 32 + 1
        n = int(np.frombuffer(b[o:o + 8], np.int64)[0])
        return b[o + 8:o + 8 + n]
    doc = graphio.read_chunk(chunk(g2))
    suffix = "" if radius == "n" else " R10.00"
    names = [c[0] for c in doc["columns"]]
    assert names == ["Connectivity", "Point First Moment", "Point Second Moment"] + [n + suffix for n in VGA_METRIC_COLUMNS]
    om = OracleMap(meta["region"], meta["spacing"], np.load(os.path.join(GOLDEN, meta["lines_npy"])))
    for f in meta["fills"]:
        om.fill(*f)
    om.make_graph()
    om.set_graph(doc["bins"], doc["runs"])
    want = om.vga_metric(radius=-1.0 if radius == "n" else float(radius), threads=8)
    got = np.stack([c[1] for c in doc["columns"][3:]], axis=1)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_cli_vga_metric_radius_errors(tmp_path):
    src = os.path.join(GOLDEN, "inputs", "syn16.csv")
    g1 = str(tmp_path / "a.dmxg")
    rc, out = run("-m", "VISPREP", "-f", src, "-o", g1, "-pg", "1", "-pp", "0.5,0.5", "-pm")
    assert rc == 0, out
    rc, out = run("-m", "VGA", "-f", g1, "-o", str(tmp_path / "b.dmxg"), "-vm", "metric", "-vr", "-3")
    assert rc == 255 and "Radius for metric vga must be n for the whole range or a positive number. Got -3" in out


@pytest.mark.gpu
def test_cli_vga_angular_and_angular_stepdepth(tmp_path):
    """VGA -vm angular (VGAAngular::run) and STEPDEPTH -sdt angular (VGAAngularDepth::run) through
    the CLI, against the C restatement on the re-read graph."""
    from depthmapx_amd import VGA_ANGULAR_COLUMNS, graphio
    from golden_io import load_case
    from pyoracle import OracleMap
    meta, A = load_case("syn32")
    src = os.path.join(GOLDEN, "inputs", "syn32.csv")
    g1, g2, g3 = (str(tmp_path / n) for n in ("a.dmxg", "b.dmxg", "c.dmxg"))
    rc, out = run("-m", "VISPREP", "-f", src, "-o", g1, "-pg", "1", "-pp", "0.5,0.5", "-pm")
    assert rc == 0, out
    rc, out = run("-m", "VGA", "-f", g1, "-o", g2, "-vm", "angular")
    assert rc == 0, out
    rc, out = run("-m", "STEPDEPTH", "-f", g1, "-o", g3, "-sdt", "angular", "-sdp", "16.5,16.5")
    assert rc == 0, out

    def chunk(path):
        b = open(path, "rb").read()
        nl = int(np.frombuffer(b[40:48], np.int64)[0])
        o = 48 + nl * 32 + 1
        n = int(np.frombuffer(b[o:o + 8], np.int64)[0])
        return b[o + 8:o + 8 + n]
    doc = graphio.read_chunk(chunk(g2))
    assert [c[0] for c in doc["columns"]][3:] == VGA_ANGULAR_COLUMNS
    om = OracleMap(meta["region"], meta["spacing"], np.load(os.path.join(GOLDEN, meta["lines_npy"])))
    for f in meta["fills"]:
        om.fill(*f)
    om.make_graph()
    om.set_graph(doc["bins"], doc["runs"])
    got = np.stack([c[1] for c in doc["columns"][3:]], axis=1)
    np.testing.assert_array_equal(got.view(np.uint32), om.vga_angular(threads=8).view(np.uint32))
    cols3 = {c[0]: c[1] for c in graphio.read_chunk(chunk(g3))["columns"]}
    want = om.angular_stepdepth(np.array([17 * meta["rows"] + 17], np.int32))
    np.testing.assert_array_equal(cols3["Angular Step Depth"], want)
