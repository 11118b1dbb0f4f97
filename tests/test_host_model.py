"""CPU-side checks of the product library (no GPU compute): libdmx.so loads, exports every symbol
include/dmx.h declares, and its host VISPREP model (grid, occluder rasterisation, flood fill) is
bit-exact against the reference's fixtures; CLI-facing error behaviour matches the reference."""
import os
import re

import numpy as np
import pytest

import depthmapx_amd as dmx
from depthmapx_amd import _native
from golden_io import case_input_lines, load_case

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def built():
    from depthmapx_amd import build
    build.build(verbose=False)


def test_library_exports_every_declared_symbol():
    hdr = open(os.path.join(REPO, "include", "dmx.h")).read()
    declared = set(re.findall(r"^\s*(?:int|int32_t|const char\*)\s+(dmx_\w+)\s*\(", hdr, re.M))
    assert declared and declared == set(_native.SIGNATURES)
    L = _native.lib()
    for name in declared:
        assert getattr(L, name) is not None
    assert L.dmx_abi_version() == 1


@pytest.mark.parametrize("name", ["kat", "syn16", "syn32", "gallery", "syn64", "barnsbury", "syn256mk"])
def test_host_prep_matches_reference(name):
    meta, A = load_case(name)
    pm = dmx.PointMap(meta["region"], case_input_lines(meta), meta["spacing"])
    i = pm.info()
    assert (i["cols"], i["rows"]) == (meta["cols"], meta["rows"])
    assert np.allclose(i["bottom_left"], meta["bottom_left"])
    for f in meta["fills"]:
        assert pm.make_points(*f)
    counts, pieces = pm.cell_lines()
    np.testing.assert_array_equal(counts, A["celllines_n"])
    np.testing.assert_array_equal(pieces, A["celllines"])
    np.testing.assert_array_equal(pm.state(), A["state"])
    assert pm.info()["filled"] == meta["nodes"]


def test_fill_errors_like_the_cli():
    meta, _ = load_case("syn16")
    pm = dmx.PointMap(meta["region"], case_input_lines(meta), meta["spacing"])
    with pytest.raises(dmx.DmxError) as e:                 # runmethods.cpp:271-275
        pm.make_points(-5.0, 3.0)
    assert e.value.status == -6 and "outside" in str(e.value)
    assert pm.make_points(0.5, 0.5)
    assert not pm.make_points(0.5, 0.5)                    # already filled: makePoints false
    with pytest.raises(dmx.DmxError):
        dmx.PointMap(meta["region"], case_input_lines(meta), 0.0)


def test_no_gpu_compute_without_device():
    """On a box without a GPU the compute entry points fail loudly (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(dmx.DmxError) as e:
        dmx.Context(0)
    assert e.value.status in (-1, -2)
