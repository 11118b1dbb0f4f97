"""The PointMap chunk of a depthmapX .graph file (PointMap::write / PointMap::read,
salalib/pointdata.cpp:1073-1188), byte-exact, through the C ABI (include/dmx.h dmx_chunk_*).

    blob = write_chunk(pm, graph_arrays, columns, displayed=0)   # bytes
    doc = read_chunk(blob)                                        # dict of numpy arrays
    pm2, g2 = load_chunk(ctx, blob, region)                       # state-only map + device graph
"""
import ctypes

import numpy as np

from . import _native as N


def write_chunk(pm, bins, runs, gridconn, columns, displayed=0, boundary=False):
    """columns: list of (name, values[N] float32, locked[, setmask[N]]) in insertion order
    (MAKEGRAPH_COLUMNS after VISPREP, then the VGA columns); displayed indexes that list."""
    bins = np.ascontiguousarray(bins, dtype=np.int32)
    runs = np.ascontiguousarray(runs, dtype=np.int16).reshape(-1, 4)
    gridconn = np.ascontiguousarray(gridconn, dtype=np.uint8)
    n = bins.shape[0]
    names = (ctypes.c_char_p * max(len(columns), 1))(*[c[0].encode() for c in columns])
    vals = np.ascontiguousarray(np.stack([np.asarray(c[1], dtype=np.float32) for c in columns]) if columns
                                else np.zeros((0, n), np.float32))
    locked = np.ascontiguousarray([1 if (len(c) > 2 and c[2]) else 0 for c in columns] or [0], dtype=np.uint8)
    masks = None
    if any(len(c) > 3 and c[3] is not None for c in columns):
        masks = np.ascontiguousarray(np.stack([np.asarray(c[3], dtype=np.uint8) if (len(c) > 3 and c[3] is not None)
                                               else np.ones(n, np.uint8) for c in columns]))
    size = ctypes.c_int64()
    args = [pm.h, n, N.ptr(bins), N.ptr(runs), len(runs), N.ptr(gridconn), len(columns), names, N.ptr(vals),
            N.ptr(locked), N.ptr(masks), int(displayed), int(bool(boundary))]
    N.check(N.lib().dmx_chunk_write(*args, None, 0, ctypes.byref(size)))
    buf = np.zeros(size.value, dtype=np.uint8)
    N.check(N.lib().dmx_chunk_write(*args, N.ptr(buf), size.value, ctypes.byref(size)))
    return buf.tobytes()


class _Chunk:
    def __init__(self, blob):
        self.buf = np.frombuffer(blob, dtype=np.uint8).copy()
        h = ctypes.c_void_p()
        N.check(N.lib().dmx_chunk_parse(N.ptr(self.buf), len(self.buf), ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            N.lib().dmx_chunk_free(self.h)
            self.h = None

    __del__ = close


def read_chunk(blob):
    c = _Chunk(blob)
    cols, rows, nc, disp = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    sp = ctypes.c_double()
    bl = np.zeros(2)
    nn, nr, used = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    N.check(N.lib().dmx_chunk_info(c.h, ctypes.byref(cols), ctypes.byref(rows), ctypes.byref(sp), N.ptr(bl),
                                   ctypes.byref(nn), ctypes.byref(nr), ctypes.byref(nc), ctypes.byref(disp),
                                   ctypes.byref(used)))
    n = nn.value
    state = np.zeros(cols.value * rows.value, dtype=np.int32)
    bins = np.zeros((n, 32, 4), dtype=np.int32)
    runs = np.zeros((max(nr.value, 1), 4), dtype=np.int16)
    gc = np.zeros(n, dtype=np.uint8)
    N.check(N.lib().dmx_chunk_arrays(c.h, N.ptr(state), N.ptr(bins), N.ptr(runs), N.ptr(gc)))
    columns = []
    for i in range(nc.value):
        name = ctypes.create_string_buffer(512)
        vals = np.zeros(n, dtype=np.float32)
        lk = ctypes.c_int()
        N.check(N.lib().dmx_chunk_column(c.h, i, name, 512, N.ptr(vals), ctypes.byref(lk)))
        columns.append((name.value.decode(), vals, bool(lk.value)))
    return dict(cols=cols.value, rows=rows.value, spacing=sp.value, bottom_left=tuple(bl), nnodes=n,
                state=state, bins=bins, runs=runs[:nr.value], gridconn=gc, columns=columns,
                displayed_sorted=disp.value, bytes_used=used.value)


def load_chunk(ctx, blob, region, lines=None):
    """(PointMap-like handle, Graph) analysing what the reference CLI's VGA / STEPDEPTH step would
    after loading the .graph (the run-length graph as decoded, 4-bit shift quirk included).  lines: the
    document's drawing, for VGA global's asymmetric mode (Graph.set_drawing)."""
    from .engine import Graph, PointMap
    c = _Chunk(blob)
    reg = np.ascontiguousarray(region, dtype=np.float64)
    hp, hg = ctypes.c_void_p(), ctypes.c_void_p()
    N.check(N.lib().dmx_chunk_load(ctx.h, c.h, N.ptr(reg), ctypes.byref(hp), ctypes.byref(hg)))
    pm = PointMap.__new__(PointMap)
    pm._region = reg
    pm._lines = np.zeros((0, 4))
    pm.h = hp
    info = read_chunk(blob)
    pm.spacing = info["spacing"]
    g = Graph(hg, ctx, pm)
    if lines is not None:
        g.set_drawing(lines)
    return pm, g
