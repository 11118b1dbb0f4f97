"""Progress callback and cancellation (dmx_ctx_set_progress / dmx_ctx_cancel): the reference's
Communicator contract (genlib/comm.h:59-142) as sparkGraph2 (salalib/pointdata.cpp:1301-1316) and
VGAVisualGlobal::run (salalib/vgavisualglobal.cpp:195-202) use it: the record count is posted while the
analysis runs, and a cancel stops it with no result.  A cancelled call must leave the context usable and
the next call bit-exact."""
import numpy as np
import pytest

import depthmapx_amd as dmx
from depthmapx_amd import _native as N
from golden_io import case_input_lines, load_case


def _map(meta):
    pm = dmx.PointMap(meta["region"], case_input_lines(meta), meta["spacing"])
    for f in meta["fills"]:
        assert pm.make_points(*f)
    return pm


def test_abi_constants():
    assert N.STATUS_NAMES[-7] == "DMX_ERR_CANCELLED"
    for sym in ("dmx_ctx_set_progress", "dmx_ctx_cancel"):
        assert hasattr(N.lib(), sym)


@pytest.mark.gpu
def test_progress_reports_and_leaves_results_unchanged(ctx):
    meta, A = load_case("syn64")
    pm = _map(meta)
    ref = pm.make_graph(ctx)
    ref_vga = ref.vga_visual_global()
    calls = []
    ctx.set_progress(lambda phase, done, total: calls.append((phase, done, total)) and False, interval_s=0.001)
    try:
        g = pm.make_graph(ctx)
        out = g.vga_visual_global()
    finally:
        ctx.set_progress(None)
    n = meta["nodes"]
    mk = [c for c in calls if c[0] == 1]
    vg = [c for c in calls if c[0] == 2]
    assert mk and vg
    assert mk[-1] == (1, n, n) and vg[-1] == (2, n, n)
    assert all(0 <= d <= t == n for _, d, t in calls)
    np.testing.assert_array_equal(g.copy(runs=True)["runs"], ref.copy(runs=True)["runs"])
    np.testing.assert_array_equal(out.view(np.uint32), ref_vga.view(np.uint32))


@pytest.mark.gpu
def test_callback_cancels_then_context_recovers(ctx):
    meta, A = load_case("syn64")
    pm = _map(meta)
    ctx.set_progress(lambda phase, done, total: True, interval_s=0.001)
    try:
        with pytest.raises(N.DmxError) as ei:
            pm.make_graph(ctx)
        assert ei.value.status == -7
    finally:
        ctx.set_progress(None)
    g = pm.make_graph(ctx)
    assert g.info()["nruns"] == meta["runs"]
    np.testing.assert_array_equal(g.copy()["attrs"].view(np.uint32), A["attrs"].view(np.uint32))
    ref = g.vga_visual_global()
    # cancel the VGA phase only
    ctx.set_progress(lambda phase, done, total: phase == 2, interval_s=0.001)
    try:
        with pytest.raises(N.DmxError) as ei:
            g.vga_visual_global()
        assert ei.value.status == -7
    finally:
        ctx.set_progress(None)
    out = g.vga_visual_global()
    np.testing.assert_array_equal(out.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
def test_pending_cancel_stops_next_call_once(ctx):
    meta, A = load_case("syn32")
    pm = _map(meta)
    ctx.cancel()
    with pytest.raises(N.DmxError) as ei:
        pm.make_graph(ctx)
    assert ei.value.status == -7
    g = pm.make_graph(ctx)          # the request was consumed
    assert g.info()["nruns"] == meta["runs"]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["metric", "angular", "visual"])
def test_pending_cancel_stops_next_stepdepth_once(ctx, kind):
    """A cancel made while nothing runs is consumed by the next step-depth call of every type (dmx.h),
    before it writes its output, and does not linger to abort a later call."""
    meta, A = load_case("syn32")
    pm = _map(meta)
    g = pm.make_graph(ctx)
    sel = A["stepdepth_sel"]
    cells = (sel >> 16) * meta["rows"] + (sel & 0xFFFF)
    fn = {"metric": g.metric_step_depth, "angular": g.angular_step_depth, "visual": g.visual_step_depth}[kind]

    def run(c):
        return fn(cells=c)
    ref = run(cells)
    ctx.cancel()
    with pytest.raises(N.DmxError) as ei:
        run(cells)
    assert ei.value.status == -7
    np.testing.assert_array_equal(run(cells).view(np.uint32), ref.view(np.uint32))


def test_progress_interval_contract():
    """interval_s <= 0 means the default 0.5 s (dmx.h); only NaN is refused.  No GPU needed: the context
    is never created, the argument check runs first."""
    lib = N.lib()
    assert lib.dmx_ctx_set_progress(None, N.PROGRESS_FN(0), None, -1.0) == -1   # NULL context
