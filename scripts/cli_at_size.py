"""The CLI drop-in at configs[2] size (VERDICT r5 'do this' 3): VISPREP through dmxcli on the 1000^2 drawing, the
written map read back the way the next dmxcli step (VGA) reads it -- PointMap chunk, lossy 4-bit ShiftLength
decode (salalib/ngraph.cpp:536-583) -- and VGA global on that re-read graph, checked against the oracle's BFS over
the same decoded runs on a block of sources.

    python scripts/cli_at_size.py --workdir /tmp/cli1000 --nsrc 256 [--cli-vga-seconds 300]

Records: the map file's size, dmxcli's -t timings (makeGraph, write), the read + decode + upload time, the runs
the round trip moved and the nodes they belong to, the re-read graph's special (asymmetric) node count and
symmetry status, the VGA kernel it takes and its time per source, and the oracle check.  Optionally runs the real
dmxcli VGA step under a time limit for its load time and progress rate.
"""
import argparse
import csv
import json
import os
import struct
import subprocess
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")]
import depthmapx_amd as dmx  # noqa: E402
from depthmapx_amd import graphio  # noqa: E402
from depthmapx_amd.build import CLI_OUT  # noqa: E402


def log(*a):
    print("[cli_at_size %.0fs]" % (time.time() - T0), *a, flush=True)


def run_cli(args, limit=None):
    """dmxcli with a heartbeat line every 30 s (a silent GPU command is taken for hung)."""
    p = subprocess.Popen([CLI_OUT] + args, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    out = []
    stop = threading.Event()

    def beat():
        while not stop.wait(30):
            log("dmxcli running:", " ".join(args[-6:]), "| last output:", (out[-1].strip() if out else "")[-120:])
    threading.Thread(target=beat, daemon=True).start()
    t0 = time.time()
    timed_out = False
    try:
        for line in p.stdout:
            out.append(line)
            if limit and time.time() - t0 > limit:
                timed_out = True
                p.kill()
                break
        p.wait(timeout=60)
    finally:
        stop.set()
    return p.returncode, "".join(out), time.time() - t0, timed_out


def read_dmxg(path):
    """dmxcli's container for a CSV drawing: region, drawing lines, one PointMap chunk of the .graph format"""
    with open(path, "rb") as f:
        assert f.read(4) == b"DMXG"
        f.read(4)
        region = struct.unpack("<4d", f.read(32))
        nl = struct.unpack("<q", f.read(8))[0]
        lines = np.frombuffer(f.read(nl * 32), dtype="<f8").reshape(-1, 4).copy()
        assert f.read(1) == b"\x01"
        n = struct.unpack("<q", f.read(8))[0]
        return list(region), lines, f.read(n)


def heartbeat():
    """a line every 30 s while the script works in-process (a silent GPU command is taken for hung)"""
    def beat():
        while True:
            time.sleep(30)
            log("working")
    threading.Thread(target=beat, daemon=True).start()


def main():
    heartbeat()
    ap = argparse.ArgumentParser()
    ap.add_argument("--workdir", default="/tmp/cli1000")
    ap.add_argument("--nsrc", type=int, default=256)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--cli-vga-seconds", type=float, default=0)
    ap.add_argument("--no-drawing", action="store_true", help="without the drawing: the top-down search")
    ap.add_argument("--skip-oracle", action="store_true", help="time the VGA block only (no oracle check)")
    a = ap.parse_args()
    os.makedirs(a.workdir, exist_ok=True)
    rec = {"workload": "dmxcli VISPREP -pg 1 -pp 0.5,0.5 -pm on syn1000 (configs[2] drawing) -> map file -> VGA -vm "
                       "visibility -vg -vr n on the re-read graph"}
    drawing = os.path.join(REPO, "tests", "golden", "inputs", "syn1000.csv")
    vp = os.path.join(a.workdir, "vp.dmxg")
    times = os.path.join(a.workdir, "vp_times.csv")
    rc, out, secs, _ = run_cli(["-f", drawing, "-o", vp, "-m", "VISPREP", "-pg", "1", "-pp", "0.5,0.5", "-pm", "-t", times])
    assert rc == 0, out[-2000:]
    rec["visprep_wall_s"] = secs
    rec["visprep_times"] = {r[0]: float(r[1]) for r in csv.reader(open(times)) if len(r) >= 2 and r[0] != "action"}
    rec["map_file_bytes"] = os.path.getsize(vp)
    log("VISPREP", rec["visprep_times"], "file %.2f GB" % (rec["map_file_bytes"] / 1e9))

    t0 = time.time()
    region, lines, blob = read_dmxg(vp)
    rec["file_read_s"] = time.time() - t0
    ctx = dmx.Context(0)
    t0 = time.time()
    # parse + ShiftLength decode + upload, and the drawing: what dmxcli's VGA step loads
    pm2, g2 = graphio.load_chunk(ctx, blob, region, lines=None if a.no_drawing else lines)
    rec["decode_upload_s"] = time.time() - t0
    N = g2.info()["nnodes"]
    rec["nnodes"], rec["nruns"] = N, g2.info()["nruns"]
    log("re-read graph: %d nodes, %d runs, decode + upload %.1f s" % (N, rec["nruns"], rec["decode_upload_s"]))

    # what the round trip moved: the decoded runs against the engine's makeGraph of the same map
    from bench import load_lines
    pm = dmx.PointMap([0.0, 0.0, 1000.0, 1000.0], load_lines(1000, 50), 1.0)
    assert pm.make_points(0.5, 0.5)
    g = pm.make_graph(ctx)
    # Bin::write stores the node count as unsigned short and writes a bin's runs only if it is non-zero
    # (ngraph.cpp:447-472): a bin of exactly 65536 k cells is read back empty
    moved = nodes_moved = dropped_bins = dropped_runs = 0
    for b in range(0, N, 65536):
        e = min(N, b + 65536)
        x, y = g.copy_range(b, e), g2.copy_range(b, e)
        np.testing.assert_array_equal(x["bins"][:, :, 1:3], y["bins"][:, :, 1:3])   # node counts, far distances
        nx, ny = x["bins"][:, :, 3].reshape(-1), y["bins"][:, :, 3].reshape(-1)
        drop = nx != ny
        # (a dropped bin reads back as direction 0 here: Graph.copy_range derives it from the run count)
        np.testing.assert_array_equal(x["bins"][:, :, 0].reshape(-1)[~drop], y["bins"][:, :, 0].reshape(-1)[~drop])
        assert (ny[drop] == 0).all() and (x["bins"][:, :, 1].reshape(-1)[drop] == 0).all()
        dropped_bins += int(drop.sum())
        dropped_runs += int(nx[drop].sum())
        keep = np.repeat(~drop, nx)
        xr = x["runs"][keep]
        assert len(xr) == len(y["runs"])
        d = np.any(xr != y["runs"], axis=1)
        moved += int(d.sum())
        per = np.repeat(np.arange(e - b), ny.reshape(-1, 32).sum(axis=1))
        nodes_moved += len(np.unique(per[d]))
    rec["runs_moved_by_roundtrip"], rec["nodes_with_moved_runs"] = moved, nodes_moved
    rec["bins_dropped_by_count_wrap"], rec["runs_dropped_by_count_wrap"] = dropped_bins, dropped_runs
    g.close()
    log("round trip moved %d runs of %d nodes; %d bins (%d runs) dropped by the 16-bit count" % (
        moved, nodes_moved, dropped_bins, dropped_runs))

    rng = np.random.default_rng(1000)
    b0 = int(rng.integers(0, N - a.nsrc))
    ctx.set_progress(lambda ph, done, total: log("VGA progress %d / %d" % (done, total)) and False, 20.0)
    t0 = time.time()
    got, lv = g2.vga_visual_global(src_begin=b0, src_end=b0 + a.nsrc, levels=True)
    secs = time.time() - t0
    st = ctx.last_stats()
    rec["vga_block"] = [b0, b0 + a.nsrc]
    rec["vga_wall_s_block"] = secs
    rec["vga_kernel_s_block"] = ctx.last_timing()[1]
    rec["vga_ms_per_source"] = 1e3 * rec["vga_kernel_s_block"] / a.nsrc
    rec["vga_kernel"] = st["vga_kernel"]
    rec["vga_special_nodes"] = st["vga_special_nodes"]
    rec["vga_prep"] = st["vga_prep"]
    rec["vga_asym_mode"], rec["vga_asym_nodes"] = st["vga_asym_mode"], st["vga_asym_nodes"]
    rec["vga_projected_whole_map_s"] = rec["vga_ms_per_source"] * 1e-3 * N
    log("VGA on the re-read graph:", st["vga_kernel"], "special nodes", st["vga_special_nodes"],
        "%.3f ms a source" % rec["vga_ms_per_source"])

    if a.skip_oracle:
        print(json.dumps(rec), flush=True)
        return
    # the oracle's BFS over the same decoded runs (the chunk's arrays), same sources
    from pyoracle import OracleMap
    info = graphio.read_chunk(blob)
    del blob
    om = OracleMap.from_grid(info["cols"], info["rows"], info["spacing"], info["bottom_left"], info["state"])
    om.set_graph_view(info["bins"], info["runs"])
    src = np.arange(b0, b0 + a.nsrc, dtype=np.int64)
    t0 = time.time()
    ref, _ = om.vga_global_sample(src, threads=a.threads)
    rec["oracle_s"] = time.time() - t0
    want = ref[src].astype(np.float64)
    gotb = got[src].astype(np.float64)
    rec["oracle_node_count_equal"] = bool(np.array_equal(gotb[:, 5], want[:, 5]))
    rec["oracle_max_rel_err"] = float(np.max(np.abs(gotb - want) / np.maximum(1.0, np.abs(want))))
    rec["oracle_ok"] = rec["oracle_node_count_equal"] and rec["oracle_max_rel_err"] <= 1e-6
    log("oracle check on %d sources: %s (max rel err %.2e, %.0f s)" % (a.nsrc, rec["oracle_ok"],
                                                                        rec["oracle_max_rel_err"], rec["oracle_s"]))
    del info, om

    if a.cli_vga_seconds > 0:
        vga = os.path.join(a.workdir, "vga.dmxg")
        rc, out, secs, timed_out = run_cli(["-f", vp, "-o", vga, "-m", "VGA", "-vm", "visibility", "-vg", "-vr", "n",
                                            "-p"], limit=a.cli_vga_seconds)
        rec["cli_vga"] = {"rc": rc, "seconds": secs, "timed_out": timed_out, "tail": out[-1500:]}
    print(json.dumps(rec), flush=True)
    assert rec["oracle_ok"], rec


if __name__ == "__main__":
    T0 = time.time()
    main()
