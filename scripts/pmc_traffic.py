"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_traffic.json.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md ("HBM [CDNA4]": FETCH_SIZE reports half the bytes of wide
coalesced reads; WRITE_SIZE reads exactly).  Usage:
    python scripts/pmc_traffic.py <workload> <fetch_counter_collection.csv> <write_counter_collection.csv> [tag]
"""
import collections
import csv
import json
import os
import sys

KERNELS = {"vga_tile_kernel": "vga_tile_kernel", "makegraph_kernel": "makegraph_kernel",
           "vga_do_kernel": "vga_do_kernel", "stepdepth_kernel": "stepdepth_kernel"}


def per_launch(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        for k in KERNELS:
            if k in r["Kernel_Name"]:
                acc[k].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    workload, fetch, write = sys.argv[1:4]
    tag = sys.argv[4] if len(sys.argv) > 4 else "r1"
    f = per_launch(fetch, "FETCH_SIZE")
    w = per_launch(write, "WRITE_SIZE")
    out_p = os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json")
    db = json.load(open(out_p)) if os.path.exists(out_p) else {}
    ent = {}
    for k in f:
        if k in w:
            ent[k] = 2.0 * f[k] + w[k]
            ent[k + "_detail"] = {"fetch_size_bytes_raw": f[k], "write_size_bytes": w[k], "tag": tag,
                                  "formula": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE half-count correction)"}
    db[workload] = ent
    json.dump(db, open(out_p, "w"), indent=1, sort_keys=True)
    print(json.dumps(ent, indent=1))


if __name__ == "__main__":
    main()
