"""VGA global on a graph read back from a .graph PointMap chunk (the CLI drop-in: VISPREP writes the map, the VGA
step reads it).  PixelVec::write stores a bin's runs after the first as a 4-bit row shift (salalib/ngraph.cpp:
536-583), so a jump of more than 15 rows moves the later runs of the bin, and Bin::write drops the runs of a bin of
65536 k cells (:447-472): the re-read graph is asymmetric, at 1000^2 in 996,278 of 998,001 nodes.  The reference's
VGA walks it as it is (vgavisualglobal.cpp:96-128).

The engine's asymmetric mode (dmx_graph_set_drawing; vga_tile.hip) makes the map's graph again from the drawing as
a symmetric reference R, runs the tile search on R with the frontier limited to cells outside A (the nodes whose
re-read runs differ from R's, plus R's own asymmetric nodes) and lets A's frontier cells push their re-read runs.
Checked here on the golden maps written and re-read through the chunk codec, every source, against the oracle's
BFS over the same decoded runs (node counts exact, floats within 1e-6), at radius n and 3; the mode is forced
(DMX_VGA_ASYM) where the in-set correction lists would otherwise take the few asymmetric nodes.
"""
import numpy as np
import pytest

import depthmapx_amd as dmx
from depthmapx_amd import graphio
from golden_io import case_input_lines, load_case

pytestmark = pytest.mark.gpu

MAKEGRAPH_COLUMNS = ["Connectivity", "Point First Moment", "Point Second Moment"]


def _reread(ctx, name):
    meta, _ = load_case(name)
    lines = case_input_lines(meta)
    pm = dmx.PointMap(meta["region"], lines, meta["spacing"])
    for f in meta["fills"]:
        assert pm.make_points(*f)
    g = pm.make_graph(ctx)
    c = g.copy(runs=True)
    cols = [(n, c["attrs"][:, i], False) for i, n in enumerate(MAKEGRAPH_COLUMNS)]
    blob = graphio.write_chunk(pm, c["bins"], c["runs"], c["gridconn"], cols)
    info = graphio.read_chunk(blob)
    moved = int(np.any(info["runs"] != c["runs"], axis=1).sum()) if len(info["runs"]) == len(c["runs"]) else -1
    pm2, g2 = graphio.load_chunk(ctx, blob, meta["region"], lines=lines)
    return meta, info, g2, moved, (pm, g, pm2)


def _oracle(info):
    from pyoracle import OracleMap
    om = OracleMap.from_grid(info["cols"], info["rows"], info["spacing"], info["bottom_left"], info["state"])
    om.set_graph(info["bins"], info["runs"])
    return om


@pytest.mark.parametrize("name", ["syn128", "barnsbury"])
def test_vga_on_reread_graph_asymmetric_mode_equals_oracle(ctx, monkeypatch, name):
    meta, info, g2, moved, keep = _reread(ctx, name)
    assert moved > 0, "the round trip moved no run: nothing to test"
    om = _oracle(info)
    monkeypatch.setenv("DMX_VGA_ASYM", "1")
    for radius in (-1, 3):
        got, lv = g2.vga_visual_global(radius=radius, levels=True)
        st = ctx.last_stats()
        assert st["vga_kernel"] == "tile-resolved" and st["vga_asym_mode"] == 1, st
        assert st["vga_asym_nodes"] > 0, st
        ref, rlv = om.vga_global(radius=radius, threads=16, levels=True)
        np.testing.assert_array_equal(lv[:, :2], rlv[:, :2])
        np.testing.assert_array_equal(got[:, 5], ref[:, 5])
        assert np.allclose(got, ref, rtol=1e-6, atol=1e-6)
    # the same graph without the mode (the in-set correction lists where the asymmetric nodes are few, else the
    # top-down search) gives the same bits
    asym = g2.vga_visual_global(radius=-1)
    monkeypatch.delenv("DMX_VGA_ASYM")
    monkeypatch.setenv("DMX_VGA_NOASYM", "1")
    plain = g2.vga_visual_global(radius=-1)
    assert ctx.last_stats()["vga_asym_mode"] == 0
    np.testing.assert_array_equal(asym.view(np.uint32), plain.view(np.uint32))
