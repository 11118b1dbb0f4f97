"""Whole-map makeGraph digests of the benchmark maps, from the pinned oracle (oracle/dmx_oracle.c).

    python tests/golden/gen_mk_digests.py --map 1000 --threads 6
    python tests/golden/gen_mk_digests.py --map 2000 --threads 6

Sweeps every source of configs[2] (syn1000, 998,001 nodes) or configs[4] (syn2000_5000, 3,991,912 nodes) with
the C restatement of sparkGraph2 + addGridConnections (pointdata.cpp:1246-1341, 1735-1768) in chunks, hashes
each 64-node block (tests/mk_digest.py) and writes tests/golden/digests/mk_<map>.npz: `digest` u64 and `nruns`
i64 per block, plus the node count.  Progress is checkpointed to a .partial.npz next to it, so a killed run
resumes where it stopped.  Hours of CPU at 1000^2 (the reference's 92.7 ms a source / 2.15 for the
restatement), so it runs once, here, and the GPU test compares against the committed file.
"""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))

from golden_io import read_csv_lines  # noqa: E402
from mk_digest import BLOCK, block_digests  # noqa: E402

MAPS = {
    "1000": ("syn1000.csv", [0.0, 0.0, 1000.0, 1000.0]),
    "2000": ("syn2000_5000.csv", [0.0, 0.0, 1999.0, 1999.0]),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--map", choices=sorted(MAPS), required=True)
    ap.add_argument("--threads", type=int, default=6)
    ap.add_argument("--chunk", type=int, default=8192)
    ap.add_argument("--limit", type=int, default=-1, help="stop after this many nodes (a timing probe)")
    a = ap.parse_args()
    from pyoracle import OracleMap
    csv, region = MAPS[a.map]
    om = OracleMap(region, 1.0, read_csv_lines(os.path.join(HERE, "inputs", csv)))
    assert om.fill(0.5, 0.5)
    N = int((om.state() & 2).astype(bool).sum())
    out = os.path.join(HERE, "digests", "mk_%s.npz" % a.map)
    part = out.replace(".npz", ".partial.npz")
    nblk = (N + BLOCK - 1) // BLOCK
    dig = np.zeros(nblk, dtype=np.uint64)
    nr = np.zeros(nblk, dtype=np.int64)
    done = 0
    if os.path.exists(part):
        z = np.load(part)
        done = int(z["done"])
        dig[:], nr[:] = z["digest"], z["nruns"]
        print("resuming at node %d" % done, flush=True)
    chunk = a.chunk - a.chunk % BLOCK
    end = N if a.limit < 0 else min(N, done + a.limit)
    t0 = time.time()
    start = done
    while done < end:
        e = min(end, done + chunk)
        g = om.make_graph_range(done, e, threads=a.threads)
        d, r = block_digests(g, done)
        dig[done // BLOCK: done // BLOCK + len(d)] = d
        nr[done // BLOCK: done // BLOCK + len(r)] = r
        done = e
        del g
        el = time.time() - t0
        rate = (done - start) / el
        print("%s: %d / %d nodes, %.1f nodes/s, %.0f s left" % (a.map, done, N, rate, (N - done) / rate), flush=True)
        if done % BLOCK == 0 or done == N:
            np.savez(part, digest=dig, nruns=nr, done=np.int64(done))
    if done == N:
        np.savez(out, digest=dig, nruns=nr, nnodes=np.int64(N), block=np.int64(BLOCK))
        os.remove(part)
        print("wrote %s: %d blocks, %d runs" % (out, nblk, int(nr.sum())), flush=True)


if __name__ == "__main__":
    main()
