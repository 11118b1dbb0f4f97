"""depthmapx_amd -- MI355X-native visibility-graph engine for the depthmapX VISPREP makeGraph +
VGA global path.  The compute path is libdmx.so (hand-written HIP for gfx950)
behind the C ABI in include/dmx.h; this package is its Python host binding."""
from ._native import DmxError, lib  # noqa: F401
from .engine import MAKEGRAPH_COLUMNS, STEPDEPTH_COLUMNS, VGA_COLUMNS, VGA_LOCAL_COLUMNS, VGA_METRIC_COLUMNS, VGA_ANGULAR_COLUMNS, Context, Graph, PointMap  # noqa: F401

__all__ = ["Context", "PointMap", "Graph", "DmxError", "MAKEGRAPH_COLUMNS", "VGA_COLUMNS", "VGA_LOCAL_COLUMNS", "VGA_METRIC_COLUMNS", "VGA_ANGULAR_COLUMNS", "STEPDEPTH_COLUMNS"]
