#!/usr/bin/env python3
"""Headline benchmark: grid cells/s for VISPREP makeGraph + VGA global (radius n) on a synthetic
W x W open-plan grid with 50 random occluders (BASELINE.json metric).

One step = the whole hot path for every filled cell of the grid:
  makeGraph (sparkGraph2) -> VGA global BFS + measures (VGAVisualGlobal::run) for every source.
Multi-GPU (one process per GPU, RCCL): makeGraph sources are split into contiguous x-major ranges of
equal modelled cost (--balance cost: PointMap.shard_bounds, a sampled sweep every rank runs alike; the
time is reported as graph_exchange.balance_s).  The VGA BFS of any source walks the whole graph, so every
rank needs all of it:
  --mk-mode shard:     each rank builds its source range, the run-length shards are all-gathered
                       over RCCL and assembled (bytes ~ 8 B/run: 574 MB at 256^2, 36 GB at 1000^2);
  --mk-mode replicate: every rank builds the whole graph (no data-path collective);
  auto (default):      the first warm-up step runs sharded and measures the shard build and the
                       exchange (max over ranks); every rank then keeps the mode that measurement
                       predicts faster (sharded.choose_mk_mode).  With no warm-up step it stays sharded.
then VGA for the rank's sources and one RCCL all-gather of the 7 float columns.
Inputs (grid state + occluder pieces) are resident in HBM before the timed region; value =
filled cells / step time (max over ranks).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--grid 1000|256]
The default workload is BASELINE.json configs[2]: the 1000 x 1000 synthetic grid (1001^2 cells),
makeGraph + VGA global (radius n) on one MI355X; configs[1] (256^2) is --grid 256.
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)


def load_lines(W, occluders, lmin=0.02, lmax=0.10):
    p = os.path.join(REPO, "tests", "golden", "inputs", ("syn%d.csv" % W) if occluders == 50 else
                     ("syn%d_%d.csv" % (W + 1, occluders)))
    if os.path.exists(p):
        from tests.golden_io import read_csv_lines
        return read_csv_lines(p)
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    from gen_synthetic import make_lines
    return np.array(make_lines(W, occluders, seed=1, lmin=lmin, lmax=lmax), dtype=np.float64)


def nearest_filled(pm, x, y):
    """STEPDEPTH -sdp x,y on the synthetic config-5 grid: the cell under (x, y), moved to the nearest
    FILLED cell when an occluder blocks it."""
    i = pm.info()
    rows, cols = i["rows"], i["cols"]
    st = pm.state()
    c0 = pm.pixelate(x, y)
    x0, y0 = c0 // rows, c0 % rows
    for r in range(max(rows, cols)):
        best = None
        for dx in range(-r, r + 1):
            for dy in range(-r, r + 1):
                if max(abs(dx), abs(dy)) != r:
                    continue
                xx, yy = x0 + dx, y0 + dy
                if 0 <= xx < cols and 0 <= yy < rows and (st[xx * rows + yy] & 2):
                    d = dx * dx + dy * dy
                    if best is None or d < best[0]:
                        best = (d, xx * rows + yy)
        if best is not None:
            return best[1]
    raise RuntimeError("no filled cell")


# the newest round's PMC summary of the shipped build (scripts/gpu_evidence.sh ROUND=6 writes r6)
PMC_SUMMARY = next((p for p in (os.path.join(REPO, "profiles", "r%d_pmc.json" % r) for r in (6, 5, 4, 3)) if os.path.exists(p)),
                   os.path.join(REPO, "profiles", "r6_pmc.json"))
FP64_PEAK_TF = 78.6    # MI355X FP64 vector (MI355X_MICROARCH.md)


def load_pmc(workload):
    """Per-kernel PMC summary of the same workload and build (scripts/gpu_pmc.sh -> scripts/pmc_summary.py ->
    profiles/r<round>_pmc.json): HBM bytes raw and 2x-FETCH corrected, L2 hit rate, VALU issue, FP64 instruction
    counts."""
    if not os.path.exists(PMC_SUMMARY):
        return {}
    try:
        return json.load(open(PMC_SUMMARY)).get(workload, {})
    except Exception:
        return {}


def cpu_threads():
    """Threads for the all-cores leg: the job's CPU share (OMP_NUM_THREADS, 16 on the GPU box), at most the
    affinity set."""
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, min(n, 16))


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def calibration():
    """ref_over_port: the reference (oracle/_ref, built from /root/reference) over the C restatement, seconds
    on identical inputs in the build container (scripts/calibrate_oracle.py -> tests/golden/oracle_calibration.json)."""
    p = os.path.join(REPO, "tests", "golden", "oracle_calibration.json")
    try:
        d = json.load(open(p))
        out = {"makegraph": d["ref_over_port_makegraph"], "vga": d["ref_over_port_vga"], "measured_on": d["cpu"]}
        if "ref_over_port_stepdepth" in d:
            out["stepdepth"] = d["ref_over_port_stepdepth"]
        return out
    except Exception:
        return None


def _oracle_map(region, lines, spacing, fill):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from pyoracle import OracleMap
    om = OracleMap(region, spacing, lines)
    om.fill(*fill)
    return om


def _legs(mk1, mkT, v1=None, vT=None):
    """cells/s of a whole step from per-source seconds: every cell is one makeGraph source and one BFS source."""
    one = 1.0 / (mk1 + (v1 or 0.0))
    allc = 1.0 / (mkT + (vT or 0.0))
    return one, allc


def cpu_baseline(region, lines, spacing, fill, g, budget_s, seed=2026, stepdepth=False, N=None, sd_cell=None):
    """The C restatement (oracle/dmx_oracle.c, bit-exact vs the reference) on the GPU box's host cores, on a
    bounded seeded sample of the same workload:
      makeGraph: S=200 random sources (seed 2026): one thread, then all cores (OpenMP over sources);
      VGA global BFS (over the whole graph, copied from the GPU and read in place): S=20 random sources on all
      cores (per-source times recorded on their threads), then the first source alone on one thread.
    value = the all-cores rate; `single_thread` = the one-thread rate (the reference is single-threaded);
    `reference_equivalent` = the one-thread rate divided by the committed reference/restatement ratio."""
    om = _oracle_map(region, lines, spacing, fill)
    N = N if N is not None else g.info()["nnodes"]
    rng = np.random.default_rng(seed)
    mk_nodes = np.sort(rng.choice(N, size=min(200, N), replace=False))
    bfs_nodes = np.sort(rng.choice(N, size=min(20, N), replace=False))
    T = cpu_threads()
    print("[bench] CPU baseline: makeGraph sample", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    mk_secs = om.make_graph_sample(mk_nodes, threads=1)
    mk1_wall = time.perf_counter() - t0
    t0 = time.perf_counter()
    om.make_graph_sample(mk_nodes, threads=T)
    mkT_wall = time.perf_counter() - t0
    mk1, mkT = mk1_wall / len(mk_nodes), mkT_wall / len(mk_nodes)
    rec = {"unit": "cells/s", "kind": "port", "cores": T, "nproc": os.cpu_count(), "cpu_model": cpu_model(),
           "seed": seed, "makegraph": {"sources": len(mk_nodes), "one_thread_s": mk1_wall, "all_cores_s": mkT_wall,
                                       "s_per_source_one_thread": mk1, "source_s_mean": float(mk_secs.mean()),
                                       "source_s_max": float(mk_secs.max())}}
    cal = calibration()
    if stepdepth:
        # config 5: the metric step depth from the config cell over the whole graph (~94 GB, copied from the
        # GPU and read in place): one search, single-threaded like the reference, run in full (not sampled)
        print("[bench] CPU baseline: graph copy + metric step depth", file=sys.stderr, flush=True)
        gn = g.copy(runs=True)
        om.set_graph_view(gn["bins"], gn["runs"])
        t0 = time.perf_counter()
        om.metric_stepdepth([sd_cell])
        sd_s = time.perf_counter() - t0
        del om, gn
        # a step = every cell's makeGraph sweep + the one search: per-cell cost mk + sd / N
        one, allc = _legs(mk1 + sd_s / N, mkT + sd_s / N)
        rec["stepdepth"] = {"cell": int(sd_cell), "one_thread_s": sd_s}
        rec["sample"] = ("oracle/dmx_oracle.c: makeGraph on %d seeded random sources (1 thread %.2f s, %d threads "
                         "%.2f s) + the whole metric step depth from cell %d on 1 thread (%.1f s; the search is "
                         "sequential on every core count)" % (len(mk_nodes), mk1_wall, T, mkT_wall, sd_cell, sd_s))
    else:
        print("[bench] CPU baseline: graph copy + BFS sample", file=sys.stderr, flush=True)
        gn = g.copy(runs=True)
        om.set_graph_view(gn["bins"], gn["runs"])
        # all S sources on T threads (each source's own time recorded on its thread), then the first of
        # them alone on one thread: the 1-thread cost per source is the loaded mean scaled by that
        # source's alone / loaded ratio (the memory-bound BFS slows a little under load)
        t0 = time.perf_counter()
        _, secs = om.vga_global_sample(bfs_nodes, threads=T)
        vT_wall = time.perf_counter() - t0
        _, sec1 = om.vga_global_sample(bfs_nodes[:1], threads=1)
        del om, gn
        alone = float(sec1[0])
        v1 = float(secs.mean()) * alone / float(secs[0])
        vT = vT_wall / len(bfs_nodes)
        one, allc = _legs(mk1, mkT, v1, vT)
        rec["vga"] = {"sources": len(bfs_nodes), "s_per_source_one_thread": v1, "first_source_alone_s": alone,
                      "first_source_loaded_s": float(secs[0]), "source_s_mean_loaded": float(secs.mean()),
                      "all_cores_s": vT_wall, "s_per_source_all_cores": vT}
        rec["sample"] = ("oracle/dmx_oracle.c on seeded random sources (seed %d): makeGraph S=%d (1 thread %.2f s, "
                         "%d threads %.2f s); VGA global BFS over the full graph S=%d on %d threads (%.2f s), the "
                         "first source again alone on 1 thread (%.2f s); per-source seconds -> cells/s"
                         % (seed, len(mk_nodes), mk1_wall, T, mkT_wall, len(bfs_nodes), T, vT_wall, alone))
    rec["value"] = allc
    rec["single_thread"] = {"value": one, "cores": 1}
    if cal:
        if stepdepth:
            ref = 1.0 / (mk1 * cal["makegraph"] + rec["stepdepth"]["one_thread_s"] * cal.get("stepdepth", 1.0) / N)
        else:
            ref = 1.0 / (mk1 * cal["makegraph"] + rec["vga"]["s_per_source_one_thread"] * cal["vga"])
        rec["reference_equivalent"] = {"value": ref, "cores": 1, "ref_over_port": cal,
                                       "note": "one-thread rate / the reference-over-restatement ratio measured on "
                                               "identical inputs (tests/golden/oracle_calibration.json)"}
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, choices=[1, 2, 5], default=2,
                    help="BASELINE.json configs[i]: 2 = 1000^2 makeGraph + VGA global (default), 1 = 256^2, "
                         "5 = 2000^2/5000 occluders makeGraph + metric step depth")
    ap.add_argument("--grid", type=int, default=None, help="W: region [0,W]^2 at spacing 1 -> (W+1)^2 cells")
    ap.add_argument("--occluders", type=int, default=50)
    ap.add_argument("--mk-mode", choices=["auto", "shard", "replicate"], default="auto")
    ap.add_argument("--balance", choices=["cost", "even"], default="cost",
                    help="makeGraph shard bounds: equal modelled cost (PointMap.shard_bounds) or equal node counts")
    ap.add_argument("--prep-mode", choices=["shard", "replicate"], default="shard",
                    help="N>1: split the VGA pre-passes by node range (partials all-reduced) or repeat them")
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="unused (the CPU sample is fixed: S=200 / S=20)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dump-out", default=None, help="rank 0 saves the gathered [N][7] VGA columns (.npy)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (not used by the driver): several ranks on one GPU over gloo
    if os.environ.get("DMX_FORCE_DEVICE") is not None:
        local = int(os.environ["DMX_FORCE_DEVICE"])
    backend = os.environ.get("DMX_DIST_BACKEND", "nccl")   # nccl = RCCL on ROCm
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world == 1 and args.mk_mode == "shard":
        # one-rank rehearsal of the sharded path: blob write, RCCL all-gather (a local copy at world 1) and
        # assembly are all timed; only the xGMI transfer itself is absent
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    dist_on = world > 1 or args.mk_mode == "shard"
    if dist_on:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    import depthmapx_amd as dmx
    from depthmapx_amd.sharded import (allgather_rows_chunked, choose_mk_mode, exchange_graph, prep_allreduce,
                                       shard_range, vga_nodes)

    stepdepth = args.config == 5
    if stepdepth:
        W, args.occluders, lmin, lmax = 1999, 5000, 0.0025, 0.01
    else:
        W, lmin, lmax = args.grid or (256 if args.config == 1 else 1000), 0.02, 0.10
    # makeGraph across ranks: "auto" runs the first warm-up step sharded, measures the shard build and the
    # graph exchange, then keeps whichever of shard / replicate the measurement predicts faster (max over
    # ranks: sharded.choose_mk_mode).  With no warm-up step it stays sharded.  The exchange over xGMI is not
    # measured on a one-GPU box: DESIGN.md section 5 gives the prediction per world size.
    mk_mode = args.mk_mode
    mk_auto = None
    if world == 1 and mk_mode == "auto":
        mk_mode = "replicate"
    elif mk_mode == "auto":
        mk_mode = "shard"
        mk_auto = {}
    lines = load_lines(W, args.occluders, lmin, lmax)
    region = [0.0, 0.0, float(W), float(W)]
    fill = (0.5, 0.5)
    ctx = dmx.Context(local)
    pm = dmx.PointMap(region, lines, 1.0)
    assert pm.make_points(*fill)
    info = pm.info()
    N = info["filled"]
    shard_be = list(shard_range(N, rank, world))   # [b, e): makeGraph sources of this rank (re-cut by cost each step)
    bal_stride = max(1, N // 4096)              # ~4096 sampled sources: one wave each, one round of the GPU
    vnodes = vga_nodes(N, rank, world) if world > 1 else None   # VGA sources of this rank
    workload = "synthetic-%d/%d-occluders VISPREP -pg 1 -pp 0.5,0.5 -pm + VGA -vm visibility -vg -vr n" % (
        W, args.occluders)
    sd_cell = None
    if stepdepth:
        sd_cell = nearest_filled(pm, W / 2 + 0.5, W / 2 + 0.5)
        workload = ("synthetic-%d/%d-occluders VISPREP -pg 1 -pp 0.5,0.5 -pm + STEPDEPTH -sdt metric -sdp "
                    "%g,%g (cell %d)" % (W, args.occluders, W / 2 + 0.5, W / 2 + 0.5, sd_cell))

    out_full = None if stepdepth else torch.full((N, 7), -1.0, dtype=torch.float32, device=dev)
    sd_out = [None]
    kt = {"makegraph_s": 0.0, "vga_s": 0.0, "n": 0, "exchange_s": 0.0, "allgather_s": 0.0, "xbytes": 0,
          "balance_s": 0.0}
    stats = {}

    def step(record):
        # 1. makeGraph: this rank's sources (shard) or all of them (replicate).  Sharded over several ranks,
        #    the contiguous ranges are cut at equal modelled cost (dmx_makegraph_balance: a sampled sweep,
        #    deterministic, so every rank cuts the same bounds without a collective)
        if mk_mode == "shard":
            if world > 1 and args.balance == "cost":
                bounds = pm.shard_bounds(ctx, world, stride=bal_stride)
                shard_be[:] = bounds[rank:rank + 2]
                if record:
                    kt["balance_s"] += ctx.last_timing()[0]
                    kt["bounds"] = bounds
            shard = pm.make_graph(ctx, node_begin=shard_be[0], node_end=shard_be[1])
        else:
            shard = pm.make_graph(ctx)
        t_mk = ctx.last_timing()[0]
        st = dict(ctx.last_stats())
        if mk_mode == "shard":
            # 2. all-gather the run-length graph shards (RCCL), assemble the whole graph
            g, xt = exchange_graph(pm, ctx, shard, dist, dev)
            del shard
            if mk_auto is not None and not mk_auto:
                mk_auto.update(xt)
                mk_auto["mk_shard_s"] = t_mk
            if record:
                kt["exchange_s"] += xt["blob_s"] + xt["allgather_s"] + xt["assemble_s"]
                kt["allgather_s"] += xt["allgather_s"]
                kt["xbytes"] = xt["bytes"]
                kt["xpeak"] = max(kt.get("xpeak") or 0, xt.get("device_peak_bytes") or 0)
        else:
            g = shard
        if stepdepth:
            # 3'. metric step depth from one cell: a single-source Dijkstra, replicas only (every rank
            #     holds the whole graph and runs the same selection)
            sd_out[0] = g.metric_step_depth(cells=[sd_cell])
            t_sd = ctx.last_stepdepth()["seconds"]
            if record:
                kt["makegraph_s"] += t_mk
                kt["vga_s"] += t_sd
                kt["n"] += 1
                st.update({"sd_" + k: v for k, v in ctx.last_stepdepth().items()})
                stats.update(st)
            return g
        # 3. VGA global for this rank's sources (node chunks dealt round-robin: balanced BFS cost);
        #    the O(runs) pre-passes are split by contiguous node range, partials all-reduced
        if world > 1:
            if args.prep_mode == "shard":
                g.set_prep_shard(shard_be[0], shard_be[1], prep_allreduce(dist, dev))
            g.vga_visual_global_device_list(out_full.data_ptr(), vnodes)
        else:
            g.vga_visual_global_device(out_full.data_ptr())
        t_vga = ctx.last_timing()[1]
        st.update({k: v for k, v in ctx.last_stats().items() if k.startswith("vga")})
        if mk_auto is not None and "sym_s" not in mk_auto and "mk_shard_s" in mk_auto:
            mk_auto["sym_s"] = st.get("vga_sym_scatter_us", 0) * 1e-6   # the sharded warm-up's scatter
        # 4. all-gather the 7 float columns
        if world > 1:
            allgather_rows_chunked(out_full, N, dist)
        if record:
            kt["makegraph_s"] += t_mk
            kt["vga_s"] += t_vga
            kt["n"] += 1
            stats.update(st)
        return g

    def progress(what):
        # one stderr line per step (stdout carries only the JSON result line)
        if rank == 0:
            print("[bench] %s %.1f s" % (what, time.perf_counter() - t_start), file=sys.stderr, flush=True)

    t_start = time.perf_counter()
    for w in range(args.warmup):
        g = step(False)
        del g
        progress("warm-up step %d/%d" % (w + 1, args.warmup))
        if w == 0 and mk_auto is not None:
            mk_mode, dec = choose_mk_mode(dist, dev, world, mk_auto["mk_shard_s"], mk_auto["blob_s"] +
                                          mk_auto["allgather_s"] + mk_auto["assemble_s"],
                                          (shard_be[1] - shard_be[0]) / max(N, 1), mk_auto.get("sym_s", 0.0))
            mk_auto.update(dec)
            mk_auto["chosen"] = mk_mode
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        g = step(True)
        if i != args.steps - 1:
            del g
        progress("step %d/%d" % (i + 1, args.steps))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    if rank == 0:
        steps = max(args.steps, 1)
        mk_s = kt["makegraph_s"] / max(kt["n"], 1)
        vga_s = kt["vga_s"] / max(kt["n"], 1)
        nsrc = len(vnodes) if world > 1 else N
        # algorithmic bytes per launch
        mk_bytes = 8 * stats.get("mk_runs", 0) + 4 * stats.get("mk_cells_examined", 0)
        tw, th = (info["cols"] + 7) // 8, (info["rows"] + 7) // 8
        levels = stats.get("vga_bottom_up_levels", 0) + stats.get("vga_top_down_levels", 0)
        # run records tested + V/X reset and per-level read/write + the tile-visibility rows read by
        # phase C (tvis and ftvis) and phase B (tile-to-tile rows)
        tvw = th * ((tw + 63) // 64)
        vga_bytes = (8 * stats.get("vga_runs_expanded", 0) + 16 * tw * th * nsrc + 32 * tw * th * levels +
                     2 * stats.get("vga_tvis_bytes", 0) + 8 * tvw * stats.get("vga_b_tiles", 0) +
                     8 * stats.get("vga_pmask_loads", 0))
        second = "vga_tile_kernel"
        if stepdepth:
            # expanders' run records (average runs per node: the per-expander counts are not exported)
            # + one 8 B relaxation record per relaxed cell
            runs_per_node = g.info()["nruns"] / max(N, 1)
            vga_bytes = int(8 * runs_per_node * stats.get("sd_expanders_popped", 0) +
                            8 * stats.get("sd_cells_relaxed", 0))
            second = "stepdepth_kernel"
        dominant = second if vga_s >= mk_s else "makegraph_kernel"
        dom_bytes, dom_s = (vga_bytes, vga_s) if vga_s >= mk_s else (mk_bytes, mk_s)
        work_rate = dom_bytes / dom_s / 1e9 if dom_s > 0 else 0.0
        pmc = load_pmc(workload) if world == 1 else {}
        dpm = pmc.get(dominant, {})
        dps = dpm.get("per_step", {})
        traffic = dps.get("hbm_bytes_raw", dpm.get("hbm_bytes_raw"))
        traffic_2x = dps.get("hbm_bytes_corrected", dpm.get("hbm_bytes_corrected"))
        # achieved = HBM bytes the counters measured for the dominant kernel (FETCH_SIZE + WRITE_SIZE per step,
        # PMC passes of this workload and build) over its live time; the 2x-FETCH figure (the guide's
        # correction for 16 B/lane streaming loads, which neither kernel issues) bounds it from above.  The
        # kernels' work models (bytes of run records, bitmap words and rows they read, most of them served
        # by the L2 / MALL / LDS) are reported as work_model_rate.  The binding limit
        # is instruction issue and memory latency, not HBM bandwidth: bound = "issue".
        if traffic:
            achieved, basis = traffic / dom_s / 1e9, "pmc FETCH_SIZE + WRITE_SIZE per step / live kernel time"
        else:
            achieved, basis = work_rate, "work model (no PMC summary of this workload and build)"
        roof = {"bound": "issue", "kernel": dominant, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "achieved_basis": basis,
                "frac_upper_2x_fetch": traffic_2x / dom_s / 1e9 / HBM_PEAK_GBS if traffic_2x else None,
                "traffic": traffic, "traffic_corrected_2x_fetch": traffic_2x,
                "traffic_source": os.path.relpath(PMC_SUMMARY, REPO) if dpm else None,
                "l2_hit_rate": dpm.get("l2_hit_rate"),
                "algorithmic_bytes": dom_bytes, "work_model_rate": work_rate,
                "launches_per_step": dpm.get("calls"), "kernel_s_live": dom_s,
                "kernel_s_rocprof": dps.get("duration_ns", dpm.get("duration_ns", 0)) * 1e-9 if dpm else None}
        vga_model = ("8 B x run records tested + 16 B x tiles x sources (V/X reset) + 32 B x tiles x levels + "
                     "tile-visibility rows read + 8 B x partial-tile masks read (DESIGN.md section 3)")
        mk_model = "B_mk = 8 B x runs written + 4 B x sieve cells examined (DESIGN.md section 2)"
        roof["work_model"] = mk_model if dominant == "makegraph_kernel" else (vga_model if not stepdepth else
                                                                              "8 B x expander runs + 8 B x relaxations")
        # the other hot kernel of the step, the same figures (the two are within a few % of each other at 1000^2)
        okern, obytes, osecs = ((second, vga_bytes, vga_s) if dominant == "makegraph_kernel" else
                                ("makegraph_kernel", mk_bytes, mk_s))
        opm = pmc.get(okern, {})
        otraffic = opm.get("per_step", {}).get("hbm_bytes_raw", opm.get("hbm_bytes_raw"))
        if osecs:
            roof["other_kernel"] = {"kernel": okern, "kernel_s_live": osecs,
                                    "achieved": otraffic / osecs / 1e9 if otraffic else None,
                                    "frac": otraffic / osecs / 1e9 / HBM_PEAK_GBS if otraffic else None,
                                    "traffic": otraffic, "l2_hit_rate": opm.get("l2_hit_rate"),
                                    "algorithmic_bytes": obytes, "work_model_rate": obytes / osecs / 1e9,
                                    "work_model": mk_model if okern == "makegraph_kernel" else (
                                        vga_model if not stepdepth else "8 B x expander runs + 8 B x relaxations")}
        if not stepdepth:
            # SURVEY.md section 8(d) B_vga at batch size 1 = the reference's BFS work (every source reads every
            # reached node's run records and touches N cells): the bytes a run-by-run BFS would move
            b_vga = nsrc * (8 * int(g.info()["nruns"]) + 4 * N)
            roof["b_vga_reference_work"] = b_vga
            roof["b_vga_rate_GBs"] = b_vga / vga_s / 1e9 if vga_s else None
        # issue-rate roofline (VALU) for the two hot kernels, and makeGraph's FP64 rate
        issue = {}
        for kname in ("makegraph_kernel", "vga_tile_kernel", "stepdepth_kernel"):
            kp = pmc.get(kname)
            if kp and "valu_active_frac" in kp:
                issue[kname] = {"valu_busy_frac": kp["valu_active_frac"], "valu_issue_frac": kp.get("valu_issue_frac"),
                                "wave_cycles_split": kp.get("wave_cycles_split"), "clock_ghz": kp.get("clock_ghz"),
                                "l2_hit_rate": kp.get("l2_hit_rate")}
        if issue:
            roof["issue"] = issue
        mkp = pmc.get("makegraph_kernel", {})
        if "per_step" in mkp and "fp64_flops" in mkp["per_step"] and mk_s:
            f = mkp["per_step"]["fp64_flops"]
            roof["makegraph_fp64"] = {"flops": f, "achieved": f / mk_s / 1e12, "peak": FP64_PEAK_TF,
                                      "unit": "TFLOP/s", "frac": f / mk_s / 1e12 / FP64_PEAK_TF,
                                      "note": "64 x (ADD+MUL+TRANS+2 FMA) F64 wave instructions (PMC), over the "
                                              "live makeGraph time"}
        rec = {
            "metric": "grid cells/sec for VISPREP makeGraph + VGA global on N×N grid",
            "value": N * steps / elapsed,
            "unit": "cells/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (committed occluder CSV, seed 1)",
            "config": {"workload": workload, "grid": "%dx%d" % (info["cols"], info["rows"]), "filled_cells": N,
                       "runs": int(g.info()["nruns"]),
                       "parallelism": "source-shard x%d (makeGraph %s, VGA prep %s)" % (
                           world, mk_mode, args.prep_mode if world > 1 else "local")},
            "kernels": {"makegraph_s": mk_s, "vga_s": vga_s,
                        "makegraph_cells_per_s": (N if mk_mode == "replicate" or world == 1 else shard_be[1] - shard_be[0]) / mk_s
                        if mk_s else None,
                        "visible_pairs": stats.get("mk_visible_pairs"),
                        "vga_kernel": stats.get("vga_kernel"),
                        "vga_runs_tested": stats.get("vga_runs_expanded"),
                        "vga_tiles_resolved_by_common_runs": stats.get("vga_cr_tiles"),
                        "vga_hard_cells_rejected_by_tile_visibility": stats.get("vga_pruned_cells"),
                        "vga_levels_bottom_up": stats.get("vga_bottom_up_levels"),
                        "vga_levels_top_down": stats.get("vga_top_down_levels"),
                        "vga_cells_decided_by_partial_tile_masks": stats.get("vga_pmask_cells"),
                        "vga_partial_tile_mask_loads": stats.get("vga_pmask_loads"),
                        "vga_partial_tile_mask_bytes": stats.get("vga_pmask_bytes"),
                        # the memory-dependent preparation this VGA ran with (DESIGN.md sections 1 and 5): scan order
                        # (or released for the masks), tile-visibility rows, fully-seen rows, tile-to-tile rows,
                        # partial-tile masks, row summaries
                        "vga_path": stats.get("vga_prep"),
                        "vga_tile_rows_bytes": stats.get("vga_tile_rows_bytes"),
                        "vga_scan_order_bytes": stats.get("vga_scan_bytes"),
                        "vga_runs_full_bfs_equiv": int(g.info()["nruns"]) * nsrc,
                        "makegraph_algorithmic_bytes": mk_bytes, "vga_algorithmic_bytes": vga_bytes,
                        # the bottom-up BFS's symmetry test and early-exit universe rest on 64-bit random-weight
                        # sums (prep): a node misclassified with probability 2^-64 each
                        "vga_certificate_failure_bound": 2.0 * N / 2.0 ** 64 if not stepdepth else None},
            "roofline": roof,
        }
        if kt["exchange_s"] or mk_auto:
            rec["kernels"]["graph_exchange"] = {
                "s_per_step": kt["exchange_s"] / max(kt["n"], 1), "allgather_s": kt["allgather_s"] / max(kt["n"], 1),
                "bytes": kt["xbytes"], "device_peak_bytes": kt.get("xpeak"), "auto": mk_auto,
                "balance": args.balance, "balance_s": kt["balance_s"] / max(kt["n"], 1), "bounds": kt.get("bounds")}
        if stepdepth:
            rec["metric"] = "grid cells/sec for VISPREP makeGraph + metric step depth on N×N grid"
            kk = rec["kernels"]
            for k in [k for k in kk if k.startswith("vga")]:
                del kk[k]
            kk.update({"stepdepth_s": vga_s, "stepdepth_expanders_popped": stats.get("sd_expanders_popped"),
                       "stepdepth_cells_relaxed": stats.get("sd_cells_relaxed"),
                       "stepdepth_algorithmic_bytes": vga_bytes,
                       "stepdepth_reached_cells": int((sd_out[0][:, 0] >= 0).sum())})
        if not args.no_cpu_baseline and world == 1:
            rec["cpu_baseline"] = cpu_baseline(region, lines, 1.0, fill, g, args.cpu_budget, stepdepth=stepdepth,
                                               N=N, sd_cell=sd_cell)
            rec["vs_cpu_baseline"] = rec["value"] / rec["cpu_baseline"]["value"]
        print(json.dumps(rec), flush=True)
        if args.dump_out and out_full is not None:
            np.save(args.dump_out, out_full.cpu().numpy())
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
