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
