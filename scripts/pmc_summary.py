"""Summarise the rocprofv3 passes of scripts/gpu_pmc.sh into one per-kernel JSON under profiles/.

    python scripts/pmc_summary.py <gpurun_out/TAG> <workload> <profiles/OUT.json>

Per kernel (makegraph_kernel, vga_tile_kernel, ...), averaged per launch:
  duration_ns (kernel-trace pass), FETCH_SIZE / WRITE_SIZE bytes (KiB x 1024), the VALU issue counters
  and the FP64 instruction counts, plus the derived figures bench.py reports:
  hbm_bytes_raw       = FETCH_SIZE + WRITE_SIZE  (the counters as read)
  hbm_bytes_corrected = 2 x FETCH_SIZE + WRITE_SIZE.  MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE
                        reads 1/2 of the bytes of 16-B-per-lane streaming loads; other widths are
                        uncalibrated.  Neither kernel streams 16 B/lane (makeGraph: 4-8 B gathers,
                        VGA: 8 B run records and 8 B bitmap words), so the raw figure is the reported
                        traffic and the corrected one an upper bound.
  l2_hit_rate         = TCC_HIT / (TCC_HIT + TCC_MISS) (guide, "L2 (per XCD)")
  clock_ghz           = GRBM_GUI_ACTIVE / 8 XCDs / duration (guide, "DVFS give-back")
  valu_issue_frac     = SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x cycles): a wave64 VALU instruction
                        occupies its SIMD for 2 cycles (guide, "SIMD-32"), so 1.0 = every SIMD issuing
                        VALU every cycle
  valu_active_frac    = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x cycles): the gfx9 "VALUBusy" formula
                        (quad-cycle units), with cycles per XCD since GRBM_GUI_ACTIVE sums the 8 XCDs
  fp64_flops          = 64 x (ADD + MUL + TRANS + 2 x FMA) F64 wave-instructions (an upper bound: the
                        counters count wave instructions, partially-masked waves count 64 lanes)
  fp64_tflops         = fp64_flops / duration, against the 78.6 TF FP64 vector peak
  lds_conflict_*      = SQ_LDS_BANK_CONFLICT per SQ_INSTS_LDS, and as a share of SQ_LDS_IDX_ACTIVE
"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = ["vga_tile_kernel", "makegraph_kernel", "vga_measures_kernel", "gridconn_kernel", "vga_do_kernel",
           "stepdepth_kernel", "vga_prep"]
N_XCD, N_CU, N_SIMD = 8, 256, 1024
FP64_PEAK_TF = 78.6


def kname(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def counters(root):
    """{kernel: {counter: [per-dispatch values]}} over every counter_collection.csv under root."""
    acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for p in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            k = kname(r["Kernel_Name"])
            if k is None:
                continue
            acc[k][r["Counter_Name"]][(p, r.get("Dispatch_Id") or r.get("Correlation_Id"))] += float(
                r["Counter_Value"])
    return {k: {c: list(v.values()) for c, v in d.items()} for k, d in acc.items()}


def durations(root):
    """{kernel: calls, total and average duration} summed over every row whose name maps to the kernel: the
    template variants of one kernel (makeGraph's first pass and its capacity re-run) are separate rows of the
    kernel-trace stats, and the counter passes average over all their launches alike."""
    out = {}
    for p in glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            k = kname(r["Name"])
            if k is None:
                continue
            e = out.setdefault(k, {"calls": 0, "total_ns": 0.0})
            e["calls"] += int(r["Calls"])
            e["total_ns"] += float(r["TotalDurationNs"])
    for e in out.values():
        e["avg_ns"] = e["total_ns"] / max(e["calls"], 1)
    return out


def main():
    root, workload, out_p = sys.argv[1:4]
    C = counters(root)
    D = durations(root)
    res = {}
    for k in sorted(set(C) | set(D)):
        c = {name: sum(v) / len(v) for name, v in C.get(k, {}).items()}
        e = {"launches_profiled": {name: len(v) for name, v in C.get(k, {}).items()}, "counters": c}
        if k in D:
            e["duration_ns"] = D[k]["avg_ns"]
            e["calls"] = D[k]["calls"]
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            f, w = 1024.0 * c["FETCH_SIZE"], 1024.0 * c["WRITE_SIZE"]
            e["fetch_bytes"], e["write_bytes"] = f, w
            e["hbm_bytes_raw"], e["hbm_bytes_corrected"] = f + w, 2.0 * f + w
        hit, miss = c.get("TCC_HIT_sum", c.get("TCC_HIT")), c.get("TCC_MISS_sum", c.get("TCC_MISS"))
        if hit is not None and miss is not None and hit + miss > 0:
            e["l2_hit_rate"] = hit / (hit + miss)   # MI355X_MICROARCH.md "L2 (per XCD)"
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / N_XCD
        if cyc > 0:
            e["cycles"] = cyc
            if "duration_ns" in e:
                e["clock_ghz"] = cyc / e["duration_ns"]
            if "SQ_INSTS_VALU" in c:
                e["valu_issue_frac"] = c["SQ_INSTS_VALU"] * 2.0 / (N_SIMD * cyc)
            if "SQ_ACTIVE_INST_VALU" in c:
                e["valu_active_frac"] = c["SQ_ACTIVE_INST_VALU"] / (N_CU * cyc)
            if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"] > 0:
                wc = c["SQ_WAVE_CYCLES"]
                e["wave_cycles_split"] = {"active_inst_any": c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                                          "wait_any": c.get("SQ_WAIT_ANY", 0) / wc,
                                          "wait_inst_any": c.get("SQ_WAIT_INST_ANY", 0) / wc}
        if c.get("SQ_INSTS_LDS"):
            # conflict cycles per LDS instruction, and their share of the cycles the LDS was busy indexing
            e["lds_conflict_cycles_per_inst"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_INSTS_LDS"]
            if c.get("SQ_LDS_IDX_ACTIVE"):
                e["lds_conflict_frac_of_idx_active"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"]
        f64 = [c.get("SQ_INSTS_VALU_%s_F64" % t) for t in ("ADD", "MUL", "FMA", "TRANS")]
        if all(x is not None for x in f64):
            flops = 64.0 * (f64[0] + f64[1] + 2.0 * f64[2] + f64[3])
            e["fp64_flops"] = flops
            if "duration_ns" in e:
                e["fp64_tflops"] = flops / e["duration_ns"] / 1e3
                e["fp64_frac"] = e["fp64_tflops"] / FP64_PEAK_TF
        if "calls" in e:   # the step's total over its launches (makeGraph: main launch + capacity retry)
            e["per_step"] = {x: e[x] * e["calls"] for x in ("duration_ns", "hbm_bytes_raw", "hbm_bytes_corrected",
                                                              "fp64_flops") if x in e}
        res[k] = e
    db = json.load(open(out_p)) if os.path.exists(out_p) else {}
    db[workload] = res
    json.dump(db, open(out_p, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: {x: v[x] for x in v if x != "counters" and x != "launches_profiled"} for k, v in res.items()},
                     indent=1))


if __name__ == "__main__":
    main()
