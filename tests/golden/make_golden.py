"""Generate the golden fixtures from the REAL reference (this container only).

Runs oracle/_ref/ref_probe (depthmapX salalib compiled from /root/reference by oracle/Makefile)
on each case below and stores its dumps as compressed .npz fixtures + cases.json.  The fixtures are
data (inputs and the reference's outputs); no reference source is copied.

    make -C oracle ref && python tests/golden/make_golden.py [case ...]
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PROBE = os.path.join(REPO, "oracle", "_ref", "ref_probe")
REF = "/root/reference"

# name: (input, spacing, fill points, vga?, roundtrip?, keep full runs?)
CASES = {
    "kat": ("inputs/kat_square.csv", 0.5, ["0.25,0.25"], True, True, True),
    "syn16": ("inputs/syn16.csv", 1.0, ["0.5,0.5"], True, True, True),
    "syn32": ("inputs/syn32.csv", 1.0, ["0.5,0.5"], True, True, True),
    "syn64": ("inputs/syn64.csv", 1.0, ["0.5,0.5"], True, True, False),
    "gallery": (REF + "/testdata/gallery_empty.graph", 0.04, ["1.32,7.24"], True, True, True),
    "barnsbury": (REF + "/testdata/barnsbury_drawing.graph", 2.0, ["531000,184000"], True, False, False),
    "syn128": ("inputs/syn128.csv", 1.0, ["0.5,0.5"], True, False, False),
    "syn256mk": ("inputs/syn256.csv", 1.0, ["0.5,0.5"], False, False, False),
    "syn128sd": ("inputs/syn128.csv", 1.0, ["0.5,0.5"], False, False, False),   # step depths only
}

# step depth selections per case (STEPDEPTH -sdt metric|visual -sdp x,y [-sdp ...]); the probe runs
# both step types on the same selection
STEPDEPTH = {
    "kat": ["0.25,0.25"],
    "syn16": ["8.5,8.5"],
    "syn32": ["16.5,16.5"],
    "syn64": ["32.5,32.5", "10.5,50.5"],
    "gallery": ["1.32,7.24"],
    "barnsbury": ["531000,184000"],
    "syn128sd": ["64.5,64.5", "3.5,120.5"],
}


def node_digests(bins, runs):
    """64-bit blake2b per node over its 32 bin records (int32 x4) and its runs (int16 x4)."""
    out = np.zeros(len(bins), dtype=np.uint64)
    ro = 0
    for k in range(len(bins)):
        nr = int(bins[k, :, 3].sum())
        h = hashlib.blake2b(digest_size=8)
        h.update(np.ascontiguousarray(bins[k]).tobytes())
        h.update(np.ascontiguousarray(runs[ro:ro + nr]).tobytes())
        out[k] = np.frombuffer(h.digest(), dtype=np.uint64)[0]
        ro += nr
    return out


def parse_grid(path):
    meta = {}
    with open(path) as f:
        for line in f:
            k, *v = line.split()
            meta[k] = [float(x) for x in v] if len(v) > 1 else float(v[0])
    return meta


def run_case(name):
    src, spacing, fills, vga, rt, keep = CASES[name]
    src_path = src if os.path.isabs(src) else os.path.join(HERE, src)
    with tempfile.TemporaryDirectory() as d:
        cmd = [PROBE, "--graph" if src_path.endswith(".graph") else "--lines", src_path,
               "--spacing", str(spacing), "--out", d]
        for p in fills:
            cmd += ["--fill", p]
        if vga:
            cmd += ["--vga"]
        if rt:
            cmd += ["--roundtrip"]
        for p in STEPDEPTH.get(name, []):
            cmd += ["--stepdepth", p]
        print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        g = parse_grid(os.path.join(d, "grid.txt"))
        rd = lambda f, dt: np.fromfile(os.path.join(d, f), dtype=dt)
        N = int(g["nodes"])
        C = int(g["cols"]) * int(g["rows"])
        lines = rd("lines.bin", np.float64).reshape(-1, 4)
        state = rd("state.bin", np.int32)
        cln = rd("celllines_n.bin", np.int32)
        cl = rd("celllines.bin", np.float64).reshape(-1, 4)
        attrs = rd("attrs.bin", np.float32).reshape(N, 3)
        bins = rd("bins.bin", np.int32).reshape(N, 32, 4)
        runs = rd("runs.bin", np.int16).reshape(-1, 4)
        gc = rd("gridconn.bin", np.uint8)
        assert len(state) == C
        arrays = dict(state=state, celllines_n=cln, celllines=cl, attrs=attrs, gridconn=gc,
                      digests=node_digests(bins, runs), nruns=bins[:, :, 3].sum(axis=1).astype(np.int32))
        if keep:  # small cases: full bin records and runs; large ones: per-node digests only
            arrays["bins"] = bins
            arrays["runs"] = runs
        if vga:
            arrays["vga"] = rd("vga.bin", np.float32).reshape(N, 7)
        if rt:
            arrays["vga_rt"] = rd("vga_rt.bin", np.float32).reshape(N, 7)
        chunk = open(os.path.join(d, "pm_chunk_mk.bin"), "rb").read()
        arrays["pm_chunk_sha256"] = np.frombuffer(hashlib.sha256(chunk).digest(), dtype=np.uint8)
        arrays["pm_chunk_size"] = np.array([len(chunk)], dtype=np.int64)
        if len(chunk) <= 64 * 1024:
            arrays["pm_chunk"] = np.frombuffer(chunk, dtype=np.uint8)
        if name in STEPDEPTH:
            arrays["stepdepth"] = rd("stepdepth.bin", np.float32).reshape(N, 3)
            arrays["stepdepth_sel"] = rd("stepdepth_sel.bin", np.int32)
            arrays["vstepdepth"] = rd("vstepdepth.bin", np.float32)
    lines_npy = name + "_lines.npy"
    np.save(os.path.join(HERE, lines_npy), lines)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
    meta = dict(source=os.path.basename(src), spacing=spacing, fills=[[float(v) for v in p.split(",")] for p in fills],
                region=g["region"], cols=int(g["cols"]), rows=int(g["rows"]), bottom_left=g["bottom_left"],
                nodes=N, runs=int(g["runs"]), lines_npy=lines_npy, vga=vga, roundtrip=rt, full_runs=keep,
                stepdepth=STEPDEPTH.get(name, []),
                ref_seconds=dict(makegraph=g["t_makegraph"], vga=g["t_vga"], stepdepth=g.get("t_stepdepth", 0.0),
                                 vstepdepth=g.get("t_vstepdepth", 0.0)))
    return meta


def main(names):
    path = os.path.join(HERE, "cases.json")
    allmeta = json.load(open(path)) if os.path.exists(path) else {}
    for n in names:
        allmeta[n] = run_case(n)
        json.dump(allmeta, open(path, "w"), indent=1, sort_keys=True)
        print(n, allmeta[n]["nodes"], "nodes", allmeta[n]["runs"], "runs", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or [k for k in CASES if k not in ("syn128", "barnsbury")])
