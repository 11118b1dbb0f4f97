""".graph drop-in: dmxcli reads depthmapX .graph files and writes them the way depthmapXcli does.

The regression method of the reference (RegressionTest/depthmaprunner.py:72-75) is a byte compare of the
output .graph files of the same command run by the baseline and the test binary.  The fixtures under
tests/golden/graphfiles/ hold the reference's outputs for the VISPREP / VGA / STEPDEPTH regression cases
(regressionconfig.json) as sha256 digests, written by tests/golden/make_golden_graphfiles.py from the real
reference built from source (oracle/_ref/ref_cli).  Cases without floating-point analysis columns must be
byte-identical.  Cases with analysis columns are byte-identical or, where a GPU float differs in its last
bits, identical outside those columns with the columns within the north-star tolerance (1e-6 relative).
"""
import hashlib
import json
import lzma
import os
import subprocess

import numpy as np
import pytest

import graphfile_util as gu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GF = os.path.join(HERE, "golden", "graphfiles")
CLI = os.path.join(REPO, "depthmapx_amd", "_lib", "dmxcli")
CASES = json.load(open(os.path.join(GF, "cases.json")))
# columns compared exactly even when the file is not byte-identical (integer-valued or bit-exact paths)
EXACT = {"Visual Node Count", "Metric Node Count", "Angular Node Count", "Visual Step Depth",
         "Metric Step Shortest-Path Length", "Metric Straight-Line Distance", "Visual Clustering Coefficient",
         "Visual Control", "Visual Controllability", "Angular Step Depth", "Angular Total Depth"}


def _input(tmp, name, made):
    if name.startswith("@"):
        return made[name[1:]]
    dst = os.path.join(tmp, name)
    if not os.path.exists(dst):
        with lzma.open(os.path.join(GF, "inputs", name + ".xz")) as f, open(dst, "wb") as o:
            o.write(f.read())
    return dst


def _run_chain(tmp, target, expect_fail=False):
    """Run the case and the cases its input chain needs (each through dmxcli); returns the paths (for a
    case expected to fail: the CompletedProcess of its run)."""
    made = {}
    order = []
    c = target
    while True:
        order.append(c)
        inp = CASES[c]["input"]
        if not inp.startswith("@"):
            break
        c = inp[1:]
    for name in reversed(order):
        src = _input(tmp, CASES[name]["input"], made)
        dst = os.path.join(tmp, name + ".graph")
        r = subprocess.run([CLI, "-f", src, "-o", dst] + CASES[name]["args"], capture_output=True, text=True, timeout=600)
        if expect_fail and name == target:
            return r
        assert r.returncode == 0, r.stdout + r.stderr
        made[name] = dst
    return made


def _check_case(tmp, name):
    m = CASES[name]
    if m.get("refused"):
        # the engine refuses it (DMX_ERR_UNSUPPORTED, see the case's note), with the CLI's error exit
        r = _run_chain(str(tmp), name, expect_fail=True)
        assert r.returncode != 0 and m["refused"] in (r.stdout + r.stderr), r.stdout + r.stderr
        return "refused"
    made = _run_chain(str(tmp), name)
    b = open(made[name], "rb").read()
    if hashlib.sha256(b).hexdigest() == m["sha256"]:
        assert len(b) == m["size"]
        return "identical"
    assert m["columns"], "%s: output differs from the reference's (%d vs %d bytes)" % (name, len(b), m["size"])
    assert gu.masked_digest(b, m["columns"]) == m["masked_sha256"], "%s differs outside the analysis columns" % name
    ref = np.load(os.path.join(GF, name + "_cols.npz"), allow_pickle=False)
    got = gu.columns(b, m["columns"])
    for col in m["columns"]:
        a, r = got[col], ref[col]
        if col in EXACT or col.split(" R")[0] in EXACT:
            assert np.array_equal(a.view(np.uint32), r.view(np.uint32)), col
        else:
            fin = np.isfinite(r)
            assert np.array_equal(np.isfinite(a), fin), col
            assert np.allclose(a[fin], r[fin], rtol=1e-6, atol=1e-6), (col, float(np.abs(a[fin] - r[fin]).max()))
    return "within tolerance"


CPU_CASES = [n for n, m in CASES.items() if not m["gpu"] and not any(
    CASES.get(c, {}).get("gpu") for c in [m["input"][1:]] if m["input"].startswith("@"))]
GPU_CASES = [n for n in CASES if n not in CPU_CASES]


@pytest.mark.parametrize("name", CPU_CASES)
def test_graph_visprep_matches_reference_bytes(tmp_path, name):
    """VISPREP grid / fill (host path, no GPU): the output .graph equals the reference's byte for byte."""
    assert _check_case(tmp_path, name) == "identical"


@pytest.mark.gpu
@pytest.mark.parametrize("name", GPU_CASES)
def test_graph_regression_case_matches_reference(tmp_path, name):
    """The regression cases that run makeGraph / VGA / step depth on the GPU."""
    how = _check_case(tmp_path, name)
    if not CASES[name]["columns"]:
        assert how == "identical"


def test_graph_drawing_lines_match_reference():
    """The drawing lines the reader hands to PointMap::blockLines equal the reference's (ref_probe dump for
    gallery and barnsbury, tests/golden/*_lines.npy)."""
    import ctypes
    import tempfile
    from depthmapx_amd import _native as N
    lib = N.lib()
    for graph, lines_npy in [("gallery_empty.graph", "gallery_lines.npy"), ("barnsbury_drawing.graph", "barnsbury_lines.npy")]:
        with tempfile.TemporaryDirectory() as tmp:
            path = _input(tmp, graph, {})
            h = ctypes.c_void_p()
            N.check(lib.dmx_graphfile_read(path.encode(), ctypes.byref(h)))
            try:
                n = ctypes.c_int64()
                region = np.zeros(4)
                N.check(lib.dmx_graphfile_info(h, None, None, N.ptr(region), ctypes.byref(n), None, None))
                got = np.zeros((n.value, 4))
                N.check(lib.dmx_graphfile_lines(h, N.ptr(got)))
            finally:
                lib.dmx_graphfile_free(h)
        ref = np.load(os.path.join(HERE, "golden", lines_npy), allow_pickle=False)
        assert got.shape == ref.shape and np.array_equal(got, ref), graph


def test_graph_roundtrip_rejects_legacy_and_garbage(tmp_path):
    """Files older than METAGRAPH_VERSION 440 need the reference's mgraph440 reader: refused, not misread."""
    import ctypes
    from depthmapx_amd import _native as N
    lib = N.lib()
    src = _input(str(tmp_path), "rect1x1.graph", {})
    b = bytearray(open(src, "rb").read())
    b[3:7] = (430).to_bytes(4, "little")
    old = tmp_path / "old.graph"
    old.write_bytes(bytes(b))
    h = ctypes.c_void_p()
    assert lib.dmx_graphfile_read(str(old).encode(), ctypes.byref(h)) == -5   # DMX_ERR_UNSUPPORTED
    bad = tmp_path / "bad.graph"
    bad.write_bytes(b"grf" + (440).to_bytes(4, "little") + b"\x00\x00")
    assert lib.dmx_graphfile_read(str(bad).encode(), ctypes.byref(h)) < 0


@pytest.mark.parametrize("nodes,count", [(-1, 0), (1, -1), (1, -(1 << 30)), (2, 1 << 30)])
def test_graph_virtual_section_bad_counts_are_rejected(tmp_path, nodes, count):
    """skipVirtualMem (mgraph.cpp:2760-2774) with a negative node count, a negative per-node count or a
    count past the end of the file: rejected as damaged, never a backwards or wrapped seek."""
    import ctypes
    import struct
    from depthmapx_amd import _native as N
    lib = N.lib()
    body = b"grf" + struct.pack("<iii", 440, 0, 0) + b"\x00\x00" + b"v" + struct.pack("<ii", nodes, count)
    bad = tmp_path / "virtual.graph"
    bad.write_bytes(body + b"\x00" * 64)
    h = ctypes.c_void_p()
    assert lib.dmx_graphfile_read(str(bad).encode(), ctypes.byref(h)) == -1   # DMX_ERR_ARG: damaged
    assert b"virtual graph" in lib.dmx_last_error()
