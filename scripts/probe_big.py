"""GPU probe: makeGraph + VGA global on a contiguous block of sources of the synthetic W x W grid;
prints timings and the BFS work counters.  python scripts/probe_big.py W nsources [kernel]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import depthmapx_amd as dmx  # noqa: E402
from bench import load_lines  # noqa: E402

W = int(sys.argv[1])
ns = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
if len(sys.argv) > 3:
    os.environ["DMX_VGA_KERNEL"] = sys.argv[3]  # "" keeps the default
ctx = dmx.Context(0)
pm = dmx.PointMap([0.0, 0.0, float(W), float(W)], load_lines(W, 50), 1.0)
assert pm.make_points(0.5, 0.5)
N = pm.info()["filled"]
t0 = time.time()
g = pm.make_graph(ctx)
t1 = time.time()
print(json.dumps({"W": W, "N": N, "runs": g.info()["nruns"], "makegraph_kernel_s": ctx.last_timing()[0],
                  "makegraph_wall_s": t1 - t0}), flush=True)
b = max(0, N // 2 - ns // 2)
e = min(N, b + ns)
t0 = time.time()
g.vga_visual_global(src_begin=b, src_end=b + 1)   # prep (uf, symmetry, tiles)
print(json.dumps({"prep_wall_s": time.time() - t0}), flush=True)
configs = [c.split("=") for c in (sys.argv[4:] if len(sys.argv) > 4 else ["DMX_VGA_CHUNK=1"])]
ref_out = None
for k, v in configs:
    os.environ[k] = v
    out = g.vga_visual_global(src_begin=b, src_end=e)
    same = None
    if ref_out is None:
        ref_out = out.copy()
    else:
        same = bool((out.view("u4") == ref_out.view("u4")).all())
    st = ctx.last_stats()
    nsrc = e - b
    tk = ctx.last_timing()[1]
    print(json.dumps({"config": "%s=%s" % (k, v), "same_as_first": same, "vga_sources": nsrc, "vga_kernel_s": tk,
                      "vga_s_per_source": tk / nsrc, "est_full_vga_s": tk / nsrc * N,
                      "runs_read_per_src": st["vga_runs_expanded"] / nsrc,
                      "fail_cells_per_src": st["vga_fail_cells"] / nsrc,
                      "fail_runs_per_src": st["vga_fail_runs"] / nsrc, "cr_tiles_per_src": st["vga_cr_tiles"] / nsrc,
                      "pruned_cells_per_src": st["vga_pruned_cells"] / nsrc,
                      "hard_cells_per_src": st["vga_hard_cells"] / nsrc, "hard_hits_per_src": st["vga_hard_hits"] / nsrc,
                      "hard_runs_per_src": st["vga_hard_runs"] / nsrc, "hard_certain_per_src": st["vga_hard_certain"] / nsrc,
                      "topdown_cycles_per_src": st["vga_topdown_cycles"] / nsrc,
                      "b_tiles_per_src": st["vga_b_tiles"] / nsrc, "b_cells_per_src": st["vga_b_cells"] / nsrc,
                      "tt_tiles_per_src": st["vga_tt_tiles"] / nsrc, "tt_pruned_per_src": st["vga_tt_pruned"] / nsrc,
                      "b_row_cycles_per_src": st["vga_b_row_cycles"] / nsrc, "b_cell_tiles_per_src": st["vga_b_cell_tiles"] / nsrc,
                      "b_cell_cycles_per_src": st["vga_b_cell_cycles"] / nsrc, "b_ext_cells_per_src": st["vga_b_ext_cells"] / nsrc,
                      "c_busy_per_src": st["vga_c_busy"] / nsrc, "c_scan_per_src": st["vga_c_scan"] / nsrc,
                      "c_spec_per_src": st["vga_c_spec"] / nsrc, "n_spec_per_src": st["vga_n_spec"] / nsrc,
                      "levels_bu_per_src": st["vga_bottom_up_levels"] / nsrc, "kernel": st["vga_kernel"], "special_nodes": st["vga_special_nodes"],
                      "launch_blocks": st["vga_launch"] & 0xFFFFFFFF,
                      "phase_cycles_per_src": {kk: vv / nsrc for kk, vv in ctx.last_phase_cycles().items()}}),
          flush=True)
