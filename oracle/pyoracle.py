"""ctypes wrapper around oracle/_build/libdmx_oracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libdmx_oracle.so")
_lib = None


def build():
    """Compile the C restatement (plain gcc; no reference sources involved)."""
    subprocess.check_call(["make", "-s", "-C", _HERE, "port"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i64, i32, dbl = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double
        L.dmxo_create.restype = vp
        L.dmxo_create.argtypes = [vp, dbl, vp, i64]
        L.dmxo_free.argtypes = [vp]
        L.dmxo_grid_info.argtypes = [vp, vp, vp, vp, vp]
        L.dmxo_fill.restype = i32
        L.dmxo_fill.argtypes = [vp, dbl, dbl]
        L.dmxo_fill_type.restype = i32
        L.dmxo_fill_type.argtypes = [vp, dbl, dbl, i32]
        L.dmxo_set_pop_forward.restype = None
        L.dmxo_set_pop_forward.argtypes = [i32]
        L.dmxo_get_state.argtypes = [vp, vp]
        L.dmxo_cell_lines_count.restype = i64
        L.dmxo_cell_lines_count.argtypes = [vp]
        L.dmxo_get_cell_lines.argtypes = [vp, vp, vp]
        L.dmxo_makegraph.restype = i32
        L.dmxo_makegraph.argtypes = [vp, dbl, i32, i64, i64, i32]
        L.dmxo_num_nodes.restype = i64
        L.dmxo_num_nodes.argtypes = [vp]
        L.dmxo_num_runs.restype = i64
        L.dmxo_num_runs.argtypes = [vp]
        L.dmxo_get_graph.argtypes = [vp, vp, vp, vp, vp]
        L.dmxo_set_graph.restype = i32
        L.dmxo_set_graph.argtypes = [vp, vp, vp, i64]
        L.dmxo_metric_stepdepth.restype = i32
        L.dmxo_metric_stepdepth.argtypes = [vp, vp, i64, vp]
        L.dmxo_visual_stepdepth.restype = i32
        L.dmxo_visual_stepdepth.argtypes = [vp, vp, i64, vp]
        L.dmxo_vga_metric.restype = i32
        L.dmxo_vga_metric.argtypes = [vp, dbl, i32, i64, i64, i32, vp]
        L.dmxo_vga_angular.restype = i32
        L.dmxo_vga_angular.argtypes = [vp, dbl, i32, i64, i64, i32, vp]
        L.dmxo_angular_stepdepth.restype = i32
        L.dmxo_angular_stepdepth.argtypes = [vp, vp, i64, vp]
        L.dmxo_vga_local.restype = i32
        L.dmxo_vga_local.argtypes = [vp, i32, i64, i64, i32, vp]
        L.dmxo_vga_global.restype = i32
        L.dmxo_vga_global.argtypes = [vp, dbl, i32, i64, i64, i32, vp, vp]
        L.dmxo_set_graph_view.restype = i32
        L.dmxo_set_graph_view.argtypes = [vp, vp, vp, i64]
        L.dmxo_makegraph_sample.restype = i32
        L.dmxo_makegraph_sample.argtypes = [vp, dbl, vp, i64, i32, vp]
        L.dmxo_vga_global_sample.restype = i32
        L.dmxo_vga_global_sample.argtypes = [vp, dbl, vp, i64, i32, vp, vp]
        L.dmxo_create_grid.restype = vp
        L.dmxo_create_grid.argtypes = [i32, i32, dbl, dbl, dbl]
        L.dmxo_set_state.restype = None
        L.dmxo_set_state.argtypes = [vp, vp]
        L.dmxo_set_merges.restype = i32
        L.dmxo_set_merges.argtypes = [vp, vp, i64]
        L.dmxo_set_graph.restype = i32
        L.dmxo_set_graph.argtypes = [vp, vp, vp, i64]
        L.dmxo_makegraph_range.restype = i32
        L.dmxo_makegraph_range.argtypes = [vp, dbl, i64, i64, i32]
        L.dmxo_num_runs_range.restype = i64
        L.dmxo_num_runs_range.argtypes = [vp, i64, i64]
        L.dmxo_get_graph_range.restype = None
        L.dmxo_get_graph_range.argtypes = [vp, i64, i64, vp, vp, vp, vp]
        L.dmxo_release_range.restype = None
        L.dmxo_release_range.argtypes = [vp, i64, i64]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleMap:
    """CPU restatement of one PointMap: setGrid -> fill -> makeGraph -> VGA global."""

    def __init__(self, region, spacing, lines):
        L = lib()
        self._region = np.ascontiguousarray(region, dtype=np.float64)
        self._lines = np.ascontiguousarray(lines, dtype=np.float64).reshape(-1, 4)
        self.h = L.dmxo_create(_p(self._region), float(spacing), _p(self._lines), len(self._lines))
        c, r = ctypes.c_int32(), ctypes.c_int32()
        bx, by = ctypes.c_double(), ctypes.c_double()
        L.dmxo_grid_info(self.h, ctypes.byref(c), ctypes.byref(r), ctypes.byref(bx), ctypes.byref(by))
        self.cols, self.rows = c.value, r.value
        self.bottom_left = (bx.value, by.value)

    @classmethod
    def from_grid(cls, cols, rows, spacing, bottom_left, state):
        """A map as a .graph PointMap chunk stores it (grid + cell states, no drawing): for analysing a
        graph handed over with set_graph."""
        L = lib()
        self = cls.__new__(cls)
        self.h = L.dmxo_create_grid(int(cols), int(rows), float(spacing), float(bottom_left[0]), float(bottom_left[1]))
        self.cols, self.rows = int(cols), int(rows)
        self.bottom_left = tuple(bottom_left)
        st = np.ascontiguousarray(state, dtype=np.int32)
        L.dmxo_set_state(self.h, _p(st))
        return self

    def set_merges(self, cell_pairs):
        """Merge links (Point::m_merge): pairs of x-major cells, followed by the VGA searches."""
        arr = np.ascontiguousarray(cell_pairs, dtype=np.int32).reshape(-1, 2)
        if lib().dmxo_set_merges(self.h, _p(arr), len(arr)):
            raise ValueError("bad merge pair")

    def __del__(self):
        if getattr(self, "h", None):
            lib().dmxo_free(self.h)
            self.h = None

    def fill(self, x, y, fill_type=0):
        """True if makePoints filled; None for an AUGMENT fill that never ends in the reference."""
        r = lib().dmxo_fill_type(self.h, float(x), float(y), int(fill_type))
        return None if r < 0 else bool(r)

    def state(self):
        out = np.zeros(self.cols * self.rows, dtype=np.int32)
        lib().dmxo_get_state(self.h, _p(out))
        return out

    def cell_lines(self):
        n = lib().dmxo_cell_lines_count(self.h)
        counts = np.zeros(self.cols * self.rows, dtype=np.int32)
        lines = np.zeros((max(n, 1), 4), dtype=np.float64)
        lib().dmxo_get_cell_lines(self.h, _p(counts), _p(lines))
        return counts, lines[:n]

    def make_graph(self, maxdist=-1.0, boundary=False, node_begin=0, node_end=-1, threads=1):
        return lib().dmxo_makegraph(self.h, float(maxdist), int(boundary), node_begin, node_end, threads)

    @property
    def num_nodes(self):
        return lib().dmxo_num_nodes(self.h)

    def graph(self):
        N = self.num_nodes
        R = lib().dmxo_num_runs(self.h)
        attrs = np.zeros((N, 3), dtype=np.float32)
        bins = np.zeros((N, 32, 4), dtype=np.int32)
        runs = np.zeros((max(R, 1), 4), dtype=np.int16)
        gc = np.zeros(N, dtype=np.uint8)
        lib().dmxo_get_graph(self.h, _p(attrs), _p(bins), _p(runs), _p(gc))
        return dict(attrs=attrs, bins=bins, runs=runs[:R], gridconn=gc)

    def set_graph(self, bins, runs):
        bins = np.ascontiguousarray(bins, dtype=np.int32)
        runs = np.ascontiguousarray(runs, dtype=np.int16)
        rc = lib().dmxo_set_graph(self.h, _p(bins), _p(runs), len(runs))
        if rc:
            raise ValueError("bins/runs inconsistent")
        self._borrowed = None

    def set_graph_view(self, bins, runs):
        """set_graph without copying the runs: the map keeps a reference to `runs` and reads it in place."""
        bins = np.ascontiguousarray(bins, dtype=np.int32)
        runs = np.ascontiguousarray(runs, dtype=np.int16)
        if lib().dmxo_set_graph_view(self.h, _p(bins), _p(runs), len(runs)):
            raise ValueError("bins/runs inconsistent")
        self._borrowed = runs

    def vga_global(self, radius=-1.0, gates_only=False, node_begin=0, node_end=-1, threads=1, levels=False):
        N = self.num_nodes
        out = np.full((N, 7), -1.0, dtype=np.float32)
        lv = np.zeros((N, 3), dtype=np.int64) if levels else None
        lib().dmxo_vga_global(self.h, float(radius), int(gates_only), node_begin, node_end, threads, _p(out),
                              _p(lv) if lv is not None else None)
        return (out, lv) if levels else out

    def metric_stepdepth(self, sel_cells):
        """VGAMetricDepth::run from x-major cell indices (std::set<int> PixelRef order).  [N][3]:
        Shortest-Path Angle, Shortest-Path Length, Straight-Line Distance (single selection)."""
        sel = np.ascontiguousarray(sel_cells, dtype=np.int32)
        out = np.full((self.num_nodes, 3), -1.0, dtype=np.float32)
        lib().dmxo_metric_stepdepth(self.h, _p(sel), len(sel), _p(out))
        return out

    def visual_stepdepth(self, sel_cells):
        """VGAVisualGlobalDepth::run from x-major cell indices of the (filled) selection, in
        std::set<int> PixelRef order.  [N] Visual Step Depth, -1 where not reached."""
        sel = np.ascontiguousarray(sel_cells, dtype=np.int32)
        out = np.full(self.num_nodes, -1.0, dtype=np.float32)
        lib().dmxo_visual_stepdepth(self.h, _p(sel), len(sel), _p(out))
        return out

    def vga_local(self, gates_only=False, node_begin=0, node_end=-1, threads=1):
        """VGAVisualLocal::run: [N][3] Visual Clustering Coefficient, Visual Control, Visual
        Controllability (-1: skipped source or neighbourhood of <= 1 cell)."""
        out = np.full((self.num_nodes, 3), -1.0, dtype=np.float32)
        lib().dmxo_vga_local(self.h, int(gates_only), node_begin, node_end, threads, _p(out))
        return out

    def vga_metric(self, radius=-1.0, gates_only=False, node_begin=0, node_end=-1, threads=1):
        """VGAMetric::run: [N][4] Metric Mean Shortest-Path Angle, Mean Shortest-Path Distance, Mean
        Straight-Line Distance, Node Count."""
        out = np.full((self.num_nodes, 4), -1.0, dtype=np.float32)
        lib().dmxo_vga_metric(self.h, float(radius), int(gates_only), node_begin, node_end, threads, _p(out))
        return out

    def vga_angular(self, radius=-1.0, gates_only=False, node_begin=0, node_end=-1, threads=1):
        """VGAAngular::run: [N][3] Angular Mean Depth, Angular Total Depth, Angular Node Count."""
        out = np.full((self.num_nodes, 3), -1.0, dtype=np.float32)
        lib().dmxo_vga_angular(self.h, float(radius), int(gates_only), node_begin, node_end, threads, _p(out))
        return out

    def angular_stepdepth(self, sel_cells):
        """VGAAngularDepth::run from x-major cell indices (std::set<int> PixelRef order): [N] Angular
        Step Depth, -1 where not reached."""
        sel = np.ascontiguousarray(sel_cells, dtype=np.int32)
        out = np.full(self.num_nodes, -1.0, dtype=np.float32)
        lib().dmxo_angular_stepdepth(self.h, _p(sel), len(sel), _p(out))
        return out

    def make_graph_range(self, node_begin, node_end, maxdist=-1.0, threads=1):
        """sparkGraph2 + addGridConnections of nodes [node_begin, node_end) only, returned in graph()'s layout
        for those nodes, and their runs freed again: a whole-map sweep in chunks (gen_mk_digests.py)."""
        L = lib()
        if L.dmxo_makegraph_range(self.h, float(maxdist), int(node_begin), int(node_end), int(threads)):
            raise ValueError("node range out of bounds")
        n = node_end - node_begin
        R = L.dmxo_num_runs_range(self.h, int(node_begin), int(node_end))
        attrs = np.zeros((n, 3), dtype=np.float32)
        bins = np.zeros((n, 32, 4), dtype=np.int32)
        runs = np.zeros((max(R, 1), 4), dtype=np.int16)
        gc = np.zeros(n, dtype=np.uint8)
        L.dmxo_get_graph_range(self.h, int(node_begin), int(node_end), _p(attrs), _p(bins), _p(runs), _p(gc))
        L.dmxo_release_range(self.h, int(node_begin), int(node_end))
        return dict(attrs=attrs, bins=bins, runs=runs[:R], gridconn=gc)

    def make_graph_sample(self, nodes, maxdist=-1.0, threads=1):
        """sparkPixel2 for each listed node (one node per thread); per-node seconds."""
        nodes = np.ascontiguousarray(nodes, dtype=np.int64)
        secs = np.zeros(len(nodes))
        if lib().dmxo_makegraph_sample(self.h, float(maxdist), _p(nodes), len(nodes), int(threads), _p(secs)):
            raise ValueError("node out of range")
        return secs

    def vga_global_sample(self, nodes, radius=-1.0, threads=1):
        """VGA global BFS from each listed source (one source per thread): ([N][7] rows, per-source seconds)."""
        nodes = np.ascontiguousarray(nodes, dtype=np.int64)
        out = np.full((self.num_nodes, 7), -1.0, dtype=np.float32)
        secs = np.zeros(len(nodes))
        if lib().dmxo_vga_global_sample(self.h, float(radius), _p(nodes), len(nodes), int(threads), _p(out), _p(secs)):
            raise ValueError("node out of range")
        return out, secs


def set_pop_forward(forward):
    """Test knob: the oracle's BFS walks each level front to back (True) instead of the reference's back
    to front.  Only to show which results depend on the order inside a level."""
    lib().dmxo_set_pop_forward(1 if forward else 0)
