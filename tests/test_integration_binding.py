"""The reference-side binding (integration/dmx_salalib.cpp, the code INTEGRATION.md tells a maintainer to
add to salalib) compiles as a real translation unit against the reference headers and links with the
reference library built from /root/reference (oracle/Makefile) and libdmx.so.  The check driver then
runs the map-image round trip the binding is built on: the reference's PointMap::write image, parsed and
re-serialized by the engine, read back by the reference's PointMap::read, written again -- identical
bytes.  (The GPU half of the binding -- makeGraph / VGA through the engine -- is the same chunk path the
.graph regression tests cover in -m gpu.)  Build container only: skipped where /root/reference or the
reference library is absent (the GPU box)."""
import lzma
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REFLIB = os.path.join(REPO, "oracle", "_ref", "libsalaref.a")


@pytest.mark.skipif(not (os.path.isdir("/root/reference") and os.path.exists(REFLIB)),
                    reason="needs the reference sources and oracle/_ref (build container only)")
@pytest.mark.parametrize("graph,spacing,fill", [("gallery_empty.graph", "0.04", "1.32,7.24"),
                                                ("barnsbury_drawing.graph", "2", "531000,184000")])
def test_binding_compiles_against_reference_and_round_trips(tmp_path, graph, spacing, fill):
    r = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "integration"), "check"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "warning" not in r.stderr.lower(), r.stderr
    src = tmp_path / graph
    with lzma.open(os.path.join(HERE, "golden", "graphfiles", "inputs", graph + ".xz")) as f:
        src.write_bytes(f.read())
    exe = os.path.join(REPO, "integration", "_build", "bind_check")
    r = subprocess.run([exe, str(src), spacing, fill], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "engine chunk parse/serialize: identical" in r.stdout
    assert "reference PointMap::read of the engine image: identical" in r.stdout
