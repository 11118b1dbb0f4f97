"""Python host mirror of the depthmapX VISPREP / VGA operator surface over the C ABI (include/dmx.h).

    ctx = Context(0)
    pm = PointMap(region, lines, spacing)            # MetaGraph::addNewPointMap + setGrid
    pm.make_points(x, y)                              # PointMap::makePoints (FULLFILL)
    g = pm.make_graph(ctx)                            # MetaGraph::makeGraph -> sparkGraph2 (GPU)
    cols = g.vga_visual_global(radius=-1)             # VGAVisualGlobal::run (GPU)

Column orders follow the reference attribute tables (see VGA_COLUMNS / MAKEGRAPH_COLUMNS).
"""
import ctypes

import numpy as np

from . import _native as N

MAKEGRAPH_COLUMNS = ["Connectivity", "Point First Moment", "Point Second Moment"]
STEPDEPTH_COLUMNS = ["Metric Step Shortest-Path Angle", "Metric Step Shortest-Path Length",
                     "Metric Straight-Line Distance"]
# VGAVisualLocal column insertion order (vgavisuallocal.cpp:31-35), also alphabetical
VGA_LOCAL_COLUMNS = ["Visual Clustering Coefficient", "Visual Control", "Visual Controllability"]
# VGAMetric columns (vgametric.cpp:45-54, inserted in this alphabetical order; " R<r>" suffix)
VGA_METRIC_COLUMNS = ["Metric Mean Shortest-Path Angle", "Metric Mean Shortest-Path Distance",
                      "Metric Mean Straight-Line Distance", "Metric Node Count"]
# VGAAngular columns (vgaangular.cpp:43-48; " R<r>" suffix)
VGA_ANGULAR_COLUMNS = ["Angular Mean Depth", "Angular Total Depth", "Angular Node Count"]
VGA_COLUMNS = ["Visual Entropy", "Visual Integration [HH]", "Visual Integration [P-value]",
               "Visual Integration [Tekl]", "Visual Mean Depth", "Visual Node Count",
               "Visual Relativised Entropy"]


class Context:
    """One HIP device (one process per GPU)."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        N.check(N.lib().dmx_ctx_create(int(device), ctypes.byref(h)))
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            N.lib().dmx_ctx_free(self.h)
            self.h = None

    __del__ = close

    def set_progress(self, fn, interval_s=0.5):
        """fn(phase, done, total) -> truthy to cancel, called while makeGraph / VGA-global kernels run
        (dmx_ctx_set_progress; the reference's Communicator, genlib/comm.h:59-142).  None removes it."""
        if fn is None:
            self._progress = None
            N.check(N.lib().dmx_ctx_set_progress(self.h, N.PROGRESS_FN(), None, 0.0))
            return

        def tramp(_user, phase, done, total):
            try:
                return 1 if fn(int(phase), int(done), int(total)) else 0
            except Exception:
                return 1
        self._progress = N.PROGRESS_FN(tramp)   # kept alive while registered
        N.check(N.lib().dmx_ctx_set_progress(self.h, self._progress, None, float(interval_s)))

    def cancel(self):
        """Cancel the running (or next) makeGraph / VGA-global / step-depth call (any thread)."""
        N.check(N.lib().dmx_ctx_cancel(self.h))

    def last_fill(self):
        """(blockLines s, flood fill s, levels) of the last GPU fill."""
        b, f, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
        N.check(N.lib().dmx_ctx_last_fill(self.h, ctypes.byref(b), ctypes.byref(f), ctypes.byref(n)))
        return b.value, f.value, n.value

    def last_timing(self):
        mk, vg = ctypes.c_double(), ctypes.c_double()
        N.check(N.lib().dmx_ctx_last_timing(self.h, ctypes.byref(mk), ctypes.byref(vg)))
        return mk.value, vg.value

    def last_stepdepth(self):
        t, p, r = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
        N.check(N.lib().dmx_ctx_last_stepdepth(self.h, ctypes.byref(t), ctypes.byref(p), ctypes.byref(r)))
        d = np.zeros(4, dtype=np.int64)
        N.check(N.lib().dmx_ctx_last_stepdepth_detail(self.h, N.ptr(d)))
        return dict(seconds=t.value, expanders_popped=p.value, cells_relaxed=r.value,
                    mode=["serial", "batched", "batched-overflow-serial"][int(d[0])], batches=int(d[1]),
                    improved=int(d[2]), ambiguous=int(d[3]))

    def last_mk_reruns(self):
        """The sources the last makeGraph swept again: (certificate re-runs, capacity re-runs), node indices
        (dmx_ctx_last_mk_reruns)."""
        n = ctypes.c_int64()
        N.check(N.lib().dmx_ctx_last_mk_reruns(self.h, None, 0, ctypes.byref(n)))
        out = np.zeros(max(n.value, 1), dtype=np.int64)
        N.check(N.lib().dmx_ctx_last_mk_reruns(self.h, N.ptr(out), n.value, ctypes.byref(n)))
        out = out[:n.value]
        cap = (out >> 62) & 1
        nodes = out & ((1 << 62) - 1)
        return np.unique(nodes[cap == 0]), np.unique(nodes[cap == 1])

    def last_phase_cycles(self):
        out = np.zeros(5, dtype=np.int64)
        N.check(N.lib().dmx_ctx_last_phase_cycles(self.h, N.ptr(out)))
        return dict(zip(["level1", "tile_common", "heads", "hard", "bookkeeping"], (int(v) for v in out)))

    def last_stats(self):
        out = np.zeros(48, dtype=np.int64)
        N.check(N.lib().dmx_ctx_last_stats(self.h, N.ptr(out), 48))
        keys = ["mk_cells_examined", "mk_visible_pairs", "mk_runs", "vga_kernel", "vga_runs_expanded", "vga_levels",
                "vga_cells_reached", "vga_sources", "vga_fail_cells", "vga_fail_runs", "vga_hbm_bitmaps",
                "vga_cr_tiles", "vga_launch", "vga_pruned_cells", "vga_tvis_bytes", "vga_hard_runs", "vga_hard_hits",
                "vga_hard_cells", "vga_hard_certain", "vga_topdown_cycles", "vga_b_tiles", "vga_b_cells", "vga_tt_tiles", "vga_c_busy", "vga_c_scan", "vga_c_spec", "vga_n_spec", "vga_tt_pruned", "vga_b_row_cycles", "vga_b_cell_tiles",
                "vga_b_cell_cycles", "vga_b_ext_cells", "mk_depth_steps", "mk_chunks", "mk_reruns", "vga_pmask_loads", "vga_pmask_cells", "vga_pmask_bytes",
                "vga_order_reruns", "vga_sym_scatter_us", "vga_prep_flags", "vga_tile_rows_bytes", "vga_scan_bytes",
                "vga_asym_nodes"]
        # vga_c_scan, vga_c_spec, vga_b_row_cycles and vga_b_cell_cycles stay 0: the kernel no longer reads
        # the clock per hard cell or per tile (2.6 % of the 1000^2 VGA); the per-phase clocks remain
        d = {k: int(v) for k, v in zip(keys, out)}
        lv = d.pop("vga_levels")
        d["vga_bottom_up_levels"], d["vga_top_down_levels"] = lv & 0xFFFFFFFF, lv >> 32
        d["vga_special_nodes"] = d["vga_kernel"] >> 8
        d["vga_frontier_hbm"] = (d["vga_launch"] >> 56) & 1   # tile BFS with its frontier in HBM (grids > 1024^2)
        d["vga_launch"] &= (1 << 56) - 1
        f = d["vga_prep_flags"]   # the memory-dependent preparation the last VGA search ran with
        d["vga_scan_order"], d["vga_scan_released"] = f & 1, (f >> 1) & 1
        d["vga_prep"] = "+".join(n for b, n in enumerate(["scan", "scan-released", "tvis", "ftvis", "ttvis", "masks",
                                                            "tvsum", "asymmetric-mode"]) if (f >> b) & 1) or "none"
        d["vga_asym_mode"] = (f >> 7) & 1
        d["vga_kernel"] = ["topdown-v1", "direction-optimizing(top-down only)",
                           "direction-optimizing", "tile-resolved"][d["vga_kernel"] & 0xFF]
        return d


class PointMap:
    """A VGA point map: grid over the drawing region, occluder pieces per cell, filled cells."""

    def __init__(self, region, lines, spacing):
        self._region = np.ascontiguousarray(region, dtype=np.float64)
        self._lines = np.ascontiguousarray(lines, dtype=np.float64).reshape(-1, 4)
        h = ctypes.c_void_p()
        N.check(N.lib().dmx_pointmap_create(N.ptr(self._region), float(spacing), N.ptr(self._lines),
                                            len(self._lines), ctypes.byref(h)))
        self.h = h
        self.spacing = float(spacing)

    def close(self):
        if getattr(self, "h", None):
            N.lib().dmx_pointmap_free(self.h)
            self.h = None

    __del__ = close

    def info(self):
        c, r, f = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        bx, by = ctypes.c_double(), ctypes.c_double()
        N.check(N.lib().dmx_pointmap_info(self.h, ctypes.byref(c), ctypes.byref(r), ctypes.byref(bx),
                                          ctypes.byref(by), ctypes.byref(f)))
        return dict(cols=c.value, rows=r.value, bottom_left=(bx.value, by.value), filled=f.value)

    @property
    def cols(self):
        return self.info()["cols"]

    @property
    def rows(self):
        return self.info()["rows"]

    FULLFILL, SEMIFILL, AUGMENT = 0, 1, 2   # QDepthmapView fill modes (depthmapview.h:75)

    def make_points(self, x, y, ctx=None, fill_type=0):
        """runmethods fillGraph + PointMap::makePoints(p, fill_type) (pointdata.cpp:402-481); raises
        DmxError(DMX_ERR_OUTSIDE) like the CLI's 'Point outside of target region'; returns False where
        makePoints returns false.  fill_type 1 (SEMIFILL) marks the cells CONTEXTFILLED; 2 (AUGMENT)
        raises DMX_ERR_UNSUPPORTED where the reference's fill would never end.  With a Context the
        rasterisation and the flood fill run on its GPU (dmx_pointmap_make_points_device)."""
        made = ctypes.c_int()
        if ctx is None:
            N.check(N.lib().dmx_pointmap_make_points(self.h, float(x), float(y), int(fill_type), ctypes.byref(made)))
        else:
            N.check(N.lib().dmx_pointmap_make_points_device(ctx.h, self.h, float(x), float(y), int(fill_type),
                                                            ctypes.byref(made)))
        return bool(made.value)

    def state(self):
        i = self.info()
        out = np.zeros(i["cols"] * i["rows"], dtype=np.int32)
        N.check(N.lib().dmx_pointmap_state(self.h, N.ptr(out)))
        return out

    def pixelate(self, x, y):
        """PointMap::pixelate(p, constrain=true) (salalib/pointdata.cpp:263-283) -> x-major cell index."""
        i = self.info()
        blx, bly = i["bottom_left"]
        px = int(np.floor((x - blx + self.spacing / 2.0) / self.spacing))
        py = int(np.floor((y - bly + self.spacing / 2.0) / self.spacing))
        px = min(max(px, 0), i["cols"] - 1)
        py = min(max(py, 0), i["rows"] - 1)
        return px * i["rows"] + py

    def region_contains(self, x, y):
        r = self._region
        return r[0] <= x <= r[2] and r[1] <= y <= r[3]

    def cell_lines(self):
        i = self.info()
        total = ctypes.c_int64()
        N.check(N.lib().dmx_pointmap_cell_lines(self.h, None, None, ctypes.byref(total)))
        counts = np.zeros(i["cols"] * i["rows"], dtype=np.int32)
        pieces = np.zeros((max(total.value, 1), 4), dtype=np.float64)
        N.check(N.lib().dmx_pointmap_cell_lines(self.h, N.ptr(counts), N.ptr(pieces), ctypes.byref(total)))
        return counts, pieces[:total.value]

    def set_merges(self, cell_pairs):
        """Merge links (Point::m_merge; PointMap::mergePixels, salalib/pointdata.cpp:1653-1680): pairs of
        x-major cells.  Written into the map's .graph chunk and followed by the graphs made from it."""
        arr = np.ascontiguousarray(cell_pairs, dtype=np.int32).reshape(-1, 2)
        N.check(N.lib().dmx_pointmap_set_merges(self.h, N.ptr(arr), len(arr)))

    def make_graph(self, ctx, boundarygraph=False, maxdist=-1.0, node_begin=0, node_end=-1):
        h = ctypes.c_void_p()
        N.check(N.lib().dmx_makegraph(ctx.h, self.h, float(maxdist), int(bool(boundarygraph)), int(node_begin),
                                      int(node_end), ctypes.byref(h)))
        return Graph(h, ctx, self)

    def shard_bounds(self, ctx, world, stride=256, boundarygraph=False, maxdist=-1.0):
        """Contiguous node ranges of equal modelled makeGraph cost for `world` ranks (dmx_makegraph_balance):
        a list of world + 1 bounds, the same on every rank."""
        b = np.zeros(int(world) + 1, dtype=np.int64)
        N.check(N.lib().dmx_makegraph_balance(ctx.h, self.h, float(maxdist), int(bool(boundarygraph)), int(world),
                                              int(stride), N.ptr(b)))
        return [int(v) for v in b]

    def assemble(self, ctx, blob_ptrs, blob_sizes):
        """Whole-map graph from shard blobs living in device memory (e.g. all-gathered torch tensors)."""
        ptrs = (ctypes.c_void_p * len(blob_ptrs))(*blob_ptrs)
        sizes = np.ascontiguousarray(blob_sizes, dtype=np.int64)
        h = ctypes.c_void_p()
        N.check(N.lib().dmx_graph_assemble_device(ctx.h, self.h, ptrs, N.ptr(sizes), len(blob_ptrs),
                                                  ctypes.byref(h)))
        return Graph(h, ctx, self)


class Graph:
    """The run-length visibility graph (device resident)."""

    def __init__(self, h, ctx, pm):
        self.h, self.ctx, self.pm = h, ctx, pm

    def close(self):
        if getattr(self, "h", None):
            N.lib().dmx_graph_free(self.h)
            self.h = None

    __del__ = close

    def info(self):
        n, b, e, r = (ctypes.c_int64() for _ in range(4))
        N.check(N.lib().dmx_graph_info(self.h, ctypes.byref(n), ctypes.byref(b), ctypes.byref(e), ctypes.byref(r)))
        return dict(nnodes=n.value, node_begin=b.value, node_end=e.value, nruns=r.value)

    def special_nodes(self):
        """Nodes with an asymmetric visible set (dmx_graph_special_nodes)."""
        n = ctypes.c_int64(0)
        N.check(N.lib().dmx_graph_special_nodes(self.h, None, ctypes.byref(n)))
        out = np.zeros(max(n.value, 1), dtype=np.int32)
        N.check(N.lib().dmx_graph_special_nodes(self.h, N.ptr(out), ctypes.byref(n)))
        return out[:n.value]

    def copy(self, runs=True):
        i = self.info()
        n = i["node_end"] - i["node_begin"]
        attrs = np.zeros((n, 3), dtype=np.float32)
        bins = np.zeros((n, 32, 4), dtype=np.int32)
        gc = np.zeros(n, dtype=np.uint8)
        rr = np.zeros((max(i["nruns"], 1), 4), dtype=np.int16) if runs else None
        N.check(N.lib().dmx_graph_copy(self.h, N.ptr(attrs), N.ptr(bins), N.ptr(rr), N.ptr(gc)))
        out = dict(attrs=attrs, bins=bins, gridconn=gc)
        if runs:
            out["runs"] = rr[:i["nruns"]]
        return out

    def copy_range(self, node_begin, node_end, runs=True):
        """bins/attrs/gridconn (and node-ordered runs) of the local nodes [node_begin, node_end) only:
        block checks at 1000^2+ without moving the whole 36-90 GB run pool to the host."""
        n = node_end - node_begin
        attrs = np.zeros((n, 3), dtype=np.float32)
        bins = np.zeros((n, 32, 4), dtype=np.int32)
        gc = np.zeros(n, dtype=np.uint8)
        nr = ctypes.c_int64()
        N.check(N.lib().dmx_graph_copy_range(self.h, int(node_begin), int(node_end), N.ptr(attrs), N.ptr(bins), None,
                                             -1, ctypes.byref(nr), N.ptr(gc)))
        out = dict(attrs=attrs, bins=bins, gridconn=gc)
        if runs:
            rr = np.zeros((max(nr.value, 1), 4), dtype=np.int16)
            N.check(N.lib().dmx_graph_copy_range(self.h, int(node_begin), int(node_end), None, None, N.ptr(rr),
                                                 len(rr), None, None))
            out["runs"] = rr[:nr.value]
        return out

    def set_merges(self, cell_pairs):
        """Merge links followed by VGA global, visual / metric / angular step depth and VGA metric /
        angular (the getMergePixel blocks of salalib/vgamodules); pairs of x-major cells."""
        arr = np.ascontiguousarray(cell_pairs, dtype=np.int32).reshape(-1, 2)
        N.check(N.lib().dmx_graph_set_merges(self.h, N.ptr(arr), len(arr)))

    def set_drawing(self, lines):
        """The drawing lines ([n][4]) the graph's map was made from: VGA global on a graph re-read from a .graph file
        (asymmetric: 4-bit row shifts, 16-bit bin counts) then runs in the asymmetric mode (dmx_graph_set_drawing)."""
        arr = np.ascontiguousarray(lines, dtype=np.float64).reshape(-1, 4)
        self._drawing = arr
        N.check(N.lib().dmx_graph_set_drawing(self.h, N.ptr(arr), len(arr)))

    def blob_size(self):
        b = ctypes.c_int64()
        N.check(N.lib().dmx_graph_blob_size(self.h, ctypes.byref(b)))
        return b.value

    def write_blob_device(self, dev_ptr, nbytes):
        N.check(N.lib().dmx_graph_blob_write_device(self.h, ctypes.c_void_p(dev_ptr), int(nbytes)))

    def vga_visual_global(self, radius=-1.0, gates_only=False, src_begin=0, src_end=-1, levels=False):
        n = self.info()["nnodes"]
        out = np.full((n, 7), -1.0, dtype=np.float32)
        lv = np.zeros((n, 3), dtype=np.int64) if levels else None
        N.check(N.lib().dmx_vga_global(self.ctx.h, self.h, float(radius), int(bool(gates_only)), int(src_begin),
                                       int(src_end), N.ptr(out), N.ptr(lv)))
        return (out, lv) if levels else out

    def vga_metric(self, radius=-1.0, gates_only=False, src_begin=0, src_end=-1):
        """VGA -vm metric -vr <radius|n> (VGAMetric::run, vgamodules/vgametric.cpp:26-136) on the GPU:
        [N][4] float32 in VGA_METRIC_COLUMNS order (radius < 0: n)."""
        n = self.info()["nnodes"]
        out = np.full((n, 4), -1.0, dtype=np.float32)
        N.check(N.lib().dmx_vga_metric(self.ctx.h, self.h, float(radius), int(bool(gates_only)), int(src_begin),
                                       int(src_end), N.ptr(out)))
        return out

    def vga_angular(self, radius=-1.0, gates_only=False, src_begin=0, src_end=-1):
        """VGA -vm angular (VGAAngular::run, vgamodules/vgaangular.cpp:26-133) on the GPU: [N][3]
        float32 in VGA_ANGULAR_COLUMNS order (radius < 0: n)."""
        n = self.info()["nnodes"]
        out = np.full((n, 3), -1.0, dtype=np.float32)
        N.check(N.lib().dmx_vga_angular(self.ctx.h, self.h, float(radius), int(bool(gates_only)), int(src_begin),
                                        int(src_end), N.ptr(out)))
        return out

    def angular_step_depth(self, points=None, cells=None):
        """STEPDEPTH -sdt angular (VGAAngularDepth::run): [N] Angular Step Depth (-1: not reached)."""
        sel = [] if cells is None else [int(c) for c in cells]
        for (x, y) in (points or []):
            if not self.pm.region_contains(x, y):
                raise N.DmxError(-6, "Point outside of target region")
            sel.append(self.pm.pixelate(x, y))
        arr = np.ascontiguousarray(sel, dtype=np.int32)
        out = np.full(self.info()["nnodes"], -1.0, dtype=np.float32)
        N.check(N.lib().dmx_angular_stepdepth(self.ctx.h, self.h, N.ptr(arr), len(arr), N.ptr(out)))
        return out

    def vga_visual_local(self, gates_only=False, src_begin=0, src_end=-1):
        """VGA -vm visibility -vl (VGAVisualLocal::run, vgamodules/vgavisuallocal.cpp:23-117) on the
        GPU: [N][3] float32 in VGA_LOCAL_COLUMNS order (-1: skipped source or neighbourhood <= 1)."""
        n = self.info()["nnodes"]
        out = np.full((n, 3), -1.0, dtype=np.float32)
        N.check(N.lib().dmx_vga_local(self.ctx.h, self.h, int(bool(gates_only)), int(src_begin), int(src_end),
                                      N.ptr(out)))
        return out

    def metric_step_depth(self, points=None, cells=None):
        """STEPDEPTH -sdt metric (dm_runmethods::runStepDepth, depthmapXcli/runmethods.cpp:735-778):
        select the cell under each point (MetaGraph::setCurSel; 'Point outside of target region'
        like the CLI), then VGAMetricDepth::run on the GPU.  Returns [N][3] float32 in
        STEPDEPTH_COLUMNS order."""
        sel = [] if cells is None else [int(c) for c in cells]
        for (x, y) in (points or []):
            if not self.pm.region_contains(x, y):
                raise N.DmxError(-6, "Point outside of target region")
            sel.append(self.pm.pixelate(x, y))
        arr = np.ascontiguousarray(sel, dtype=np.int32)
        n = self.info()["nnodes"]
        out = np.full((n, 3), -1.0, dtype=np.float32)
        N.check(N.lib().dmx_metric_stepdepth(self.ctx.h, self.h, N.ptr(arr), len(arr), N.ptr(out)))
        return out

    def visual_step_depth(self, points=None, cells=None):
        """STEPDEPTH -sdt visual (dm_runmethods::runStepDepth, depthmapXcli/runmethods.cpp:767-769):
        select the cell under each point, then VGAVisualGlobalDepth::run
        (salalib/vgamodules/vgavisualglobaldepth.cpp:23-77) on the GPU.  Returns [N] float32
        "Visual Step Depth" (-1: not reached)."""
        sel = [] if cells is None else [int(c) for c in cells]
        for (x, y) in (points or []):
            if not self.pm.region_contains(x, y):
                raise N.DmxError(-6, "Point outside of target region")
            sel.append(self.pm.pixelate(x, y))
        arr = np.ascontiguousarray(sel, dtype=np.int32)
        n = self.info()["nnodes"]
        out = np.full(n, -1.0, dtype=np.float32)
        N.check(N.lib().dmx_visual_stepdepth(self.ctx.h, self.h, N.ptr(arr), len(arr), N.ptr(out)))
        return out

    def set_prep_shard(self, node_begin, node_end, allreduce):
        """Split the VGA preparation over ranks (dmx_graph_set_prep_shard): this rank scatters nodes
        [node_begin, node_end); allreduce(ptr, count, dtype) must sum the device buffer in place over
        all ranks (dtype 0 = int32, 1 = int64) and return 0.  allreduce=None undoes it."""
        if allreduce is None:
            self._prep_cb = None
            N.check(N.lib().dmx_graph_set_prep_shard(self.h, 0, 0, None, None))
            return

        def cb(ptr, count, dtype, user):
            try:
                return int(allreduce(ptr, count, dtype) or 0)
            except Exception:                     # an exception must not unwind through C
                import traceback
                traceback.print_exc()
                return -1
        self._prep_cb = N.ALLREDUCE_FN(cb)        # kept alive as long as the graph
        N.check(N.lib().dmx_graph_set_prep_shard(self.h, int(node_begin), int(node_end),
                                                 ctypes.cast(self._prep_cb, ctypes.c_void_p), None))

    def vga_visual_global_device_list(self, out_dev_ptr, nodes, radius=-1.0, gates_only=False):
        """VGA global for the listed source nodes only (rows of the others untouched); device output."""
        arr = np.ascontiguousarray(nodes, dtype=np.int64)
        N.check(N.lib().dmx_vga_global_device_list(self.ctx.h, self.h, float(radius), int(bool(gates_only)),
                                                   N.ptr(arr), len(arr), ctypes.c_void_p(out_dev_ptr)))

    def vga_visual_global_device(self, out_dev_ptr, radius=-1.0, gates_only=False, src_begin=0, src_end=-1):
        N.check(N.lib().dmx_vga_global_device(self.ctx.h, self.h, float(radius), int(bool(gates_only)),
                                              int(src_begin), int(src_end), ctypes.c_void_p(out_dev_ptr)))
