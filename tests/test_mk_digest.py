"""The whole-map makeGraph digests (tests/mk_digest.py, tests/golden/gen_mk_digests.py): the oracle's chunked
sweep (OracleMap.make_graph_range) hashes exactly as its one-shot sweep does, and the committed digest files
describe the benchmark maps (block count, node count)."""
import os

import numpy as np
import pytest

from golden_io import GOLDEN, read_csv_lines
from mk_digest import BLOCK, block_digests


def _map(name, W):
    from pyoracle import OracleMap
    lines = read_csv_lines(os.path.join(GOLDEN, "inputs", name))
    om = OracleMap([0.0, 0.0, float(W), float(W)], 1.0, lines)
    assert om.fill(0.5, 0.5)
    return om


def test_chunked_oracle_sweep_hashes_as_the_whole_sweep():
    om = _map("syn64.csv", 64)
    om.make_graph(threads=4)
    whole = om.graph()
    N = len(whole["bins"])
    want, want_nr = block_digests(whole, 0)
    om2 = _map("syn64.csv", 64)
    got, got_nr = [], []
    for b in range(0, N, 3 * BLOCK):   # chunks of 192 nodes, the last one ragged
        d, r = block_digests(om2.make_graph_range(b, min(N, b + 3 * BLOCK), threads=4), b)
        got.append(d)
        got_nr.append(r)
    np.testing.assert_array_equal(np.concatenate(got), want)
    np.testing.assert_array_equal(np.concatenate(got_nr), want_nr)
    assert want_nr.sum() == len(whole["runs"])
    # any change to one run changes its block's digest only
    bad = dict(whole)
    bad["runs"] = whole["runs"].copy()
    bad["runs"][len(bad["runs"]) // 2, 2] += 1
    d, _ = block_digests(bad, 0)
    assert (d != want).sum() == 1


@pytest.mark.parametrize("name,nnodes", [("1000", 998001), ("2000", 3991912)])
def test_committed_digests_cover_the_benchmark_maps(name, nnodes):
    path = os.path.join(GOLDEN, "digests", "mk_%s.npz" % name)
    if not os.path.exists(path):
        pytest.skip("not generated yet: python tests/golden/gen_mk_digests.py --map %s" % name)
    z = np.load(path, allow_pickle=False)
    assert int(z["nnodes"]) == nnodes and int(z["block"]) == BLOCK
    assert len(z["digest"]) == len(z["nruns"]) == (nnodes + BLOCK - 1) // BLOCK
    assert (z["nruns"] > 0).all()
