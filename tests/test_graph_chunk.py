"""The .graph PointMap chunk (depthmapx_amd.graphio over dmx_chunk_*): byte-for-byte against the
chunk the REAL reference writes after VISPREP (ref_probe: PointMap::write, pointdata.cpp:1158-1188),
and the decoder's 4-bit shift quirk against the reference's own round trip.  Host-only (no GPU):
the graph comes from the C restatement, which is pinned to the same fixtures."""
import hashlib

import numpy as np
import pytest

import depthmapx_amd as dmx
from depthmapx_amd import graphio
from golden_io import case_input_lines, load_case, roundtrip_runs
from pyoracle import OracleMap

CASES = ["kat", "syn16", "syn32", "gallery", "syn64"]


def _maps(meta):
    lines = case_input_lines(meta)
    pm = dmx.PointMap(meta["region"], lines, meta["spacing"])
    om = OracleMap(meta["region"], meta["spacing"], lines)
    for f in meta["fills"]:
        assert pm.make_points(*f) and om.fill(*f)
    pm.cell_lines()   # blockLines (sets BLOCKED like sparkGraph2 leaves it)
    om.make_graph(threads=8)
    return pm, om.graph()


def _chunk(pm, g):
    cols = [(name, g["attrs"][:, j], j == 0) for j, name in enumerate(dmx.MAKEGRAPH_COLUMNS)]
    return graphio.write_chunk(pm, g["bins"], g["runs"], g["gridconn"], cols, displayed=0)


@pytest.mark.parametrize("name", CASES)
def test_chunk_bytes_match_reference(name):
    meta, A = load_case(name)
    pm, g = _maps(meta)
    np.testing.assert_array_equal(pm.state(), A["state"])
    blob = _chunk(pm, g)
    assert len(blob) == int(A["pm_chunk_size"][0])
    if "pm_chunk" in A:
        ref = A["pm_chunk"].tobytes()
        first = next((i for i in range(len(ref)) if blob[i] != ref[i]), None)
        assert first is None, "first differing byte at %s" % first
    assert hashlib.sha256(blob).digest() == A["pm_chunk_sha256"].tobytes()


@pytest.mark.parametrize("name", CASES)
def test_chunk_read_applies_shift_quirk(name):
    meta, A = load_case(name)
    pm, g = _maps(meta)
    doc = graphio.read_chunk(_chunk(pm, g))
    assert (doc["cols"], doc["rows"]) == (meta["cols"], meta["rows"])
    np.testing.assert_array_equal(doc["state"], A["state"])
    np.testing.assert_array_equal(doc["gridconn"], g["gridconn"])
    np.testing.assert_array_equal(doc["bins"][:, :, 3], g["bins"][:, :, 3])
    np.testing.assert_array_equal(doc["runs"], roundtrip_runs(g["bins"], g["runs"]))
    names = [c[0] for c in doc["columns"]]
    assert names == dmx.MAKEGRAPH_COLUMNS
    for j, c in enumerate(doc["columns"]):
        np.testing.assert_array_equal(c[1].view(np.uint32), g["attrs"][:, j].view(np.uint32))
    # a decoded chunk re-encodes to the same bytes (the quirk is idempotent)
    assert graphio.write_chunk(pm, doc["bins"], doc["runs"], doc["gridconn"],
                               [(n, v, lk) for (n, v, lk) in doc["columns"]]) == _chunk(pm, dict(g, runs=doc["runs"]))
