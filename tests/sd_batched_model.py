"""Pure-Python model of the batched metric step-depth schedule (depthmapx_amd/csrc/kernels/stepdepth.hip,
"batched metric step depth"): distance windows of one grid unit, a certified single winner per cell,
and a sequential pop-order fold for the ambiguous cells.  Test infrastructure only: it checks the
schedule's mathematics against the serial restatement (oracle/, pinned to the reference's
VGAMetricDepth::run, salalib/vgamodules/vgametricdepth.cpp:23-92) on small maps, independently of the
HIP kernels."""
import math

import numpy as np

F32 = np.float32
INF = (1 << 64) - 1
W_REL = 2.0 ** -20
FILLED, BLOCKED = 2, 4


def _key(d, pix):
    return (int(np.array(d, dtype=np.float32).view(np.uint32)) << 32) | (pix & 0xFFFFFFFF)


def _kdist(k):
    return float(np.array(k >> 32, dtype=np.uint32).view(np.float32))


def _turn(dx, dy, ux, uy, lastu):
    if lastu == -1:
        return F32(0.0)
    lx, ly = lastu >> 16, lastu & 0xFFFF
    ex, ey = ux - lx, uy - ly
    v = math.acos((dx * ex + dy * ey) / (math.sqrt(dx * dx + dy * dy) * math.sqrt(ex * ex + ey * ey) + 1e-12))
    return F32(v / (math.pi * 0.5))


def _cells(run):
    x0, y0, x1, y1 = (int(v) for v in run)
    dxs = 1 if x1 > x0 else 0
    dys = 0 if y0 == y1 else (1 if x0 == x1 else (1 if y1 > y0 else -1))
    n = max(x1 - x0, y1 - y0, y0 - y1) + 1
    return [(x0 + k * dxs, y0 + k * dys) for k in range(n)]


def batched_metric_stepdepth(state, rows, cols, bins, runs, sel_cells, spacing=1.0):
    """state: [C] cell state (x-major), bins/runs: the graph as OracleMap.graph() returns it.
    Returns ([N][3] like OracleMap.metric_stepdepth, stats)."""
    C = rows * cols
    filled = [c for c in range(C) if state[c] & FILLED]
    node_of = {c: k for k, c in enumerate(filled)}
    nr = bins[:, :, 3].sum(axis=1)
    start = np.concatenate([[0], np.cumsum(nr)])

    def blocked_adj(x, y):
        for dx in (-1, 0, 1):
            for dy in (-1, 0, 1):
                xx, yy = x + dx, y + dy
                if 0 <= xx < cols and 0 <= yy < rows and (state[xx * rows + yy] & BLOCKED):
                    return True
        return False

    sel = sorted(set(int(c) for c in sel_cells if state[c] & FILLED), key=lambda c: ((c // rows) << 16) + c % rows)
    expand = {c for c in filled if blocked_adj(c // rows, c % rows)} | set(sel)
    key = {c: INF for c in filled}
    md = {c: F32(-1.0) for c in filled}
    cum = {c: F32(0.0) for c in filled}
    last = {c: -1 for c in filled}
    for c in sel:
        key[c] = _key(0.0, ((c // rows) << 16) + c % rows)
    done = set()
    stats = dict(batches=0, ambiguous=0)

    def update(c, u):
        x, y, ux, uy = c // rows, c % rows, u // rows, u % rows
        dx, dy = x - ux, y - uy
        dd = math.sqrt(dx * dx + dy * dy)
        du = F32(_kdist(key[u]))
        if md[c] == F32(-1.0) or float(du) + dd < float(md[c]):
            nd = F32(du + F32(dd))
            md[c] = nd
            cum[c] = F32(cum[u] + _turn(dx, dy, ux, uy, last[u]))
            nk = _key(nd, (x << 16) + y)
            if nk < key[c]:
                key[c] = nk
                last[c] = (ux << 16) + uy

    while True:
        live = [c for c in expand if c not in done and key[c] != INF]
        if not live:
            break
        g = min(key[c] for c in live)
        lim = _kdist(g) + 1.0
        batch = sorted((c for c in live if _kdist(key[c]) < lim - lim * 2.0 ** -18), key=lambda c: key[c])
        stats["batches"] += 1
        done.update(batch)
        # candidates per cell: (s, pop rank) of every relaxer; md/key are the pre-batch values
        cand = {}
        for rank, u in enumerate(batch):
            ux, uy, ku = u // rows, u % rows, key[u]
            du = _kdist(ku)
            k = node_of[u]
            for r in runs[start[k]:start[k + 1]]:
                for (x, y) in _cells(r):
                    c = x * rows + y
                    if not (state[c] & FILLED) or key[c] < ku:
                        continue
                    s = du + math.sqrt((x - ux) ** 2 + (y - uy) ** 2)
                    cand.setdefault(c, []).append((rank, s, u))
        for c, lst in cand.items():
            m0 = float(md[c])
            near = [e for e in lst if m0 == -1.0 or e[1] <= m0 + m0 * W_REL]
            if not near:
                continue
            best = min(e[1] for e in near)
            rivals = [e for e in near if e[1] <= best + best * W_REL]
            if len(rivals) == 1:
                update(c, rivals[0][2])
            else:
                stats["ambiguous"] += 1
                for e in sorted(lst):
                    update(c, e[2])
    out = np.full((len(filled), 3), -1.0, dtype=np.float32)
    single = len(sel) == 1
    for k, c in enumerate(filled):
        if key[c] == INF:
            continue
        d = _kdist(key[c])
        out[k, 0] = cum[c]
        out[k, 1] = F32(spacing * d)
        if single:
            dx, dy = c // rows - sel[0] // rows, c % rows - sel[0] % rows
            out[k, 2] = F32(spacing * math.sqrt(dx * dx + dy * dy))
    return out, stats
