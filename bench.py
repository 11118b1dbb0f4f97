#!/usr/bin/env python3
"""Headline benchmark: grid cells/s for VISPREP makeGraph + VGA global (radius n) on a synthetic
W x W open-plan grid with 50 random occluders (BASELINE.json metric).

One step = the whole hot path for every filled cell of the grid:
  makeGraph (sparkGraph2) -> VGA global BFS + measures (VGAVisualGlobal::run) for every source.
Multi-GPU (one process per GPU, RCCL): sources are split into contiguous x-major ranges.  The VGA
BFS of any source walks the whole graph, so every rank needs all of it:
  --mk-mode shard:     each rank builds its source range, the run-length shards are all-gathered
                       over RCCL and assembled (bytes ~ 8 B/run: 574 MB at 256^2, 36 GB at 1000^2);
  --mk-mode replicate: every rank builds the whole graph (no data-path collective);
  auto:                shard (the all-gather moves ~36 GB at 1000^2, well under a second over xGMI,
                       against ~10 s of makeGraph that replicate would repeat on every rank).
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


def load_traffic(workload):
    """HBM bytes per launch from a committed rocprofv3 --pmc pass (profiles/pmc_traffic.json)."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p)).get(workload)
    except Exception:
        return None


def cpu_baseline(region, lines, spacing, fill, g, budget_s):
    """The C restatement (oracle/, bit-exact vs the reference) timed single-threaded on a bounded
    sample of the same workload: makeGraph on a contiguous block of sources, then VGA global BFS
    on a block of sources over the full graph (copied from the GPU result, identical bits)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from pyoracle import OracleMap
    om = OracleMap(region, spacing, lines)
    om.fill(*fill)
    N = g.info()["nnodes"]
    mid = N // 2
    k, t_mk = 4, 0.0
    while True:
        t0 = time.perf_counter()
        om.make_graph(node_begin=mid, node_end=min(N, mid + k), threads=1)
        t_mk = time.perf_counter() - t0
        if t_mk > 0.3 * budget_s or mid + k >= N:
            break
        k = min(N - mid, max(k * 2, int(k * 0.3 * budget_s / max(t_mk, 1e-3))))
    mk_per_src = t_mk / min(k, N - mid)
    gn = g.copy(runs=True)
    om.set_graph(gn["bins"], gn["runs"])
    del gn
    kv, t_v = 1, 0.0
    while True:
        t0 = time.perf_counter()
        om.vga_global(node_begin=mid, node_end=min(N, mid + kv), threads=1)
        t_v = time.perf_counter() - t0
        if t_v > 0.4 * budget_s or mid + kv >= N:
            break
        kv = min(N - mid, max(kv * 2, int(kv * 0.4 * budget_s / max(t_v, 1e-3))))
    vga_per_src = t_v / min(kv, N - mid)
    return {"value": 1.0 / (mk_per_src + vga_per_src), "unit": "cells/s", "cores": 1, "kind": "port",
            "sample": "oracle/dmx_oracle.c single thread: makeGraph on %d sources (%.2f s) + VGA global BFS "
                      "on %d sources (%.2f s) from node %d over the full graph; per-source times -> cells/s"
                      % (min(k, N - mid), t_mk, min(kv, N - mid), t_v, mid),
            "makegraph_s_per_source": mk_per_src, "vga_s_per_source": vga_per_src}


def cpu_baseline_mk(region, lines, spacing, fill, N, budget_s):
    """Config 5: the C restatement's makeGraph timed single-threaded on a contiguous source block.
    The step-depth leg is not sampled (it needs the whole ~94 GB graph on the host), so the CPU
    figure omits it and overstates the CPU rate."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from pyoracle import OracleMap
    om = OracleMap(region, spacing, lines)
    om.fill(*fill)
    mid, k = N // 2, 4
    while True:
        t0 = time.perf_counter()
        om.make_graph(node_begin=mid, node_end=min(N, mid + k), threads=1)
        t_mk = time.perf_counter() - t0
        if t_mk > 0.5 * budget_s or mid + k >= N:
            break
        k = min(N - mid, max(k * 2, int(k * 0.5 * budget_s / max(t_mk, 1e-3))))
    k = min(k, N - mid)
    return {"value": k / t_mk, "unit": "cells/s", "cores": 1, "kind": "port",
            "sample": "oracle/dmx_oracle.c single thread: makeGraph on %d sources (%.2f s) from node %d; "
                      "step depth not sampled (CPU rate overstated)" % (k, t_mk, mid),
            "makegraph_s_per_source": t_mk / k}


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
    ap.add_argument("--prep-mode", choices=["shard", "replicate"], default="shard",
                    help="N>1: split the VGA pre-passes by node range (partials all-reduced) or repeat them")
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of CPU baseline sampling")
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
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    import depthmapx_amd as dmx
    from depthmapx_amd.sharded import (allgather_blobs, allgather_rows_chunked, prep_allreduce, shard_range,
                                       vga_nodes)

    stepdepth = args.config == 5
    if stepdepth:
        W, args.occluders, lmin, lmax = 1999, 5000, 0.0025, 0.01
    else:
        W, lmin, lmax = args.grid or (256 if args.config == 1 else 1000), 0.02, 0.10
    mk_mode = args.mk_mode
    if mk_mode == "auto":
        mk_mode = "shard"
    lines = load_lines(W, args.occluders, lmin, lmax)
    region = [0.0, 0.0, float(W), float(W)]
    fill = (0.5, 0.5)
    ctx = dmx.Context(local)
    pm = dmx.PointMap(region, lines, 1.0)
    assert pm.make_points(*fill)
    info = pm.info()
    N = info["filled"]
    b, e = shard_range(N, rank, world)          # makeGraph sources of this rank
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
    kt = {"makegraph_s": 0.0, "vga_s": 0.0, "n": 0}
    stats = {}

    def step(record):
        # 1. makeGraph: this rank's sources (shard) or all of them (replicate)
        if world > 1 and mk_mode == "shard":
            shard = pm.make_graph(ctx, node_begin=b, node_end=e)
        else:
            shard = pm.make_graph(ctx)
        t_mk = ctx.last_timing()[0]
        st = dict(ctx.last_stats())
        if world > 1 and mk_mode == "shard":
            # 2. all-gather the run-length graph shards (RCCL), assemble the whole graph
            blob = torch.empty(shard.blob_size(), dtype=torch.uint8, device=dev)
            shard.write_blob_device(blob.data_ptr(), blob.numel())
            flat, mx, sizes = allgather_blobs(blob, dist)
            torch.cuda.synchronize()
            g = pm.assemble(ctx, [flat.data_ptr() + i * mx for i in range(world)], sizes)
            del flat, blob, shard
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
                g.set_prep_shard(b, e, prep_allreduce(dist, dev))
            g.vga_visual_global_device_list(out_full.data_ptr(), vnodes)
        else:
            g.vga_visual_global_device(out_full.data_ptr())
        t_vga = ctx.last_timing()[1]
        st.update({k: v for k, v in ctx.last_stats().items() if k.startswith("vga")})
        # 4. all-gather the 7 float columns
        if world > 1:
            allgather_rows_chunked(out_full, N, dist)
        if record:
            kt["makegraph_s"] += t_mk
            kt["vga_s"] += t_vga
            kt["n"] += 1
            stats.update(st)
        return g

    for _ in range(args.warmup):
        g = step(False)
        del g
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        g = step(True)
        if i != args.steps - 1:
            del g
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
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
        # phase C (tvis and ftvis) and phase B1 (tile-to-tile rows)
        tvw = th * ((tw + 63) // 64)
        vga_bytes = (8 * stats.get("vga_runs_expanded", 0) + 16 * tw * th * nsrc + 32 * tw * th * levels +
                     2 * stats.get("vga_tvis_bytes", 0) + 8 * tvw * stats.get("vga_b_tiles", 0))
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
        achieved = dom_bytes / dom_s / 1e9 if dom_s > 0 else 0.0
        traffic = load_traffic(workload)
        tr = traffic.get(dominant) if isinstance(traffic, dict) else None
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
                        "makegraph_cells_per_s": (N if mk_mode == "replicate" or world == 1 else e - b) / mk_s
                        if mk_s else None,
                        "visible_pairs": stats.get("mk_visible_pairs"),
                        "vga_kernel": stats.get("vga_kernel"),
                        "vga_runs_tested": stats.get("vga_runs_expanded"),
                        "vga_tiles_resolved_by_common_runs": stats.get("vga_cr_tiles"),
                        "vga_hard_cells_rejected_by_tile_visibility": stats.get("vga_pruned_cells"),
                        "vga_levels_bottom_up": stats.get("vga_bottom_up_levels"),
                        "vga_levels_top_down": stats.get("vga_top_down_levels"),
                        "vga_runs_full_bfs_equiv": int(g.info()["nruns"]) * nsrc,
                        "makegraph_algorithmic_bytes": mk_bytes, "vga_algorithmic_bytes": vga_bytes},
            "roofline": {"bound": "hbm", "kernel": dominant, "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": tr},
        }
        if stepdepth:
            rec["metric"] = "grid cells/sec for VISPREP makeGraph + metric step depth on N×N grid"
            kk = rec["kernels"]
            for k in [k for k in kk if k.startswith("vga")]:
                del kk[k]
            kk.update({"stepdepth_s": vga_s, "stepdepth_expanders_popped": stats.get("sd_expanders_popped"),
                       "stepdepth_cells_relaxed": stats.get("sd_cells_relaxed"),
                       "stepdepth_algorithmic_bytes": vga_bytes,
                       "stepdepth_reached_cells": int((sd_out[0][:, 0] >= 0).sum())})
        if not args.no_cpu_baseline and world == 1 and stepdepth:
            rec["cpu_baseline"] = cpu_baseline_mk(region, lines, 1.0, fill, N, args.cpu_budget)
            rec["vs_cpu_baseline"] = rec["value"] / rec["cpu_baseline"]["value"]
        elif not args.no_cpu_baseline and world == 1:
            rec["cpu_baseline"] = cpu_baseline(region, lines, 1.0, fill, g, args.cpu_budget)
            rec["vs_cpu_baseline"] = rec["value"] / rec["cpu_baseline"]["value"]
        print(json.dumps(rec), flush=True)
        if args.dump_out and out_full is not None:
            np.save(args.dump_out, out_full.cpu().numpy())
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
