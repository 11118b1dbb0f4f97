"""Readers for the golden fixtures under tests/golden/ (written by tests/golden/make_golden.py from
the real reference, oracle/_ref/ref_probe)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

VGA_COLUMNS = ["Visual Entropy", "Visual Integration [HH]", "Visual Integration [P-value]",
               "Visual Integration [Tekl]", "Visual Mean Depth", "Visual Node Count",
               "Visual Relativised Entropy"]


def read_csv_lines(path):
    rows = []
    with open(path) as f:
        next(f)
        for line in f:
            if line.strip():
                rows.append([float(v) for v in line.split(",")[:4]])
    return np.array(rows, dtype=np.float64).reshape(-1, 4)


def case_names():
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        return list(json.load(f).keys())


def load_case(name):
    """Returns (meta, arrays) for a committed golden case."""
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        meta = json.load(f)[name]
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    arrays = {k: z[k] for k in z.files}
    return meta, arrays


def case_input_lines(meta):
    return np.load(os.path.join(GOLDEN, meta["lines_npy"]), allow_pickle=False)


def node_digests(bins, runs):
    """64-bit blake2b per node over its 32 bin records (int32 x4) and its runs (int16 x4) -- the
    same digest tests/golden/make_golden.py stores for cases too large to commit run-by-run."""
    import hashlib
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


def roundtrip_runs(bins, runs):
    """Apply the .graph write/read round trip to a run list: inside each H/V bin,
    run i>0 is stored as (primary coordinate, ShiftLength{shift:4, runlength:12}) relative to run
    i-1 (ngraph.cpp:536-583), so row/column jumps > 15 wrap on re-read and the error propagates.
    Diagonal bins keep their single span.  Returns the runs VGA sees after VISPREP -> file -> VGA."""
    out = runs.astype(np.int32).copy()
    ro = 0
    for k in range(len(bins)):
        for b in range(32):
            d, n = int(bins[k, b, 0]), int(bins[k, b, 3])
            if n and d in (1, 2):
                for i in range(ro + 1, ro + n):
                    if d == 1:  # HORIZONTAL: primary x, shift in y, length in x
                        y = out[i - 1, 1] + ((int(runs[i, 1]) - int(runs[i - 1, 1])) & 15)
                        x0 = int(runs[i, 0])
                        out[i] = (x0, y, x0 + ((int(runs[i, 2]) - x0) & 4095), y)
                    else:       # VERTICAL: primary y, shift in x, length in y
                        x = out[i - 1, 0] + ((int(runs[i, 0]) - int(runs[i - 1, 0])) & 15)
                        y0 = int(runs[i, 1])
                        out[i] = (x, y0, x, y0 + ((int(runs[i, 3]) - y0) & 4095))
            ro += n
    return out.astype(np.int16)
