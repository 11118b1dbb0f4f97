"""Restatement-vs-reference speed ratio: the C restatement (oracle/, 1 thread)
timed here on the inputs whose reference (salalib built from source, oracle/_ref) timings are in
tests/golden/cases.json `ref_seconds`, both measured in this container: makeGraph, VGA global (syn64,
gallery, barnsbury, syn128: up to 16,129 sources) and metric step depth.  Writes
tests/golden/oracle_calibration.json; bench.py reports the ratio next to its CPU baseline.
    python scripts/calibrate_oracle.py"""
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from golden_io import case_input_lines, load_case  # noqa: E402
from pyoracle import OracleMap  # noqa: E402


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    out = {"cpu": cpu_model(), "nproc": os.cpu_count(), "cases": {}}
    # makeGraph, VGA global (every source of the map) and metric step depth (the fixture's selection), each on
    # one thread, against the reference's own timings of the same runs (oracle/_ref/ref_probe, cases.json)
    plan = [("syn64", ("makegraph", "vga", "stepdepth")), ("gallery", ("makegraph", "vga", "stepdepth")),
            ("barnsbury", ("makegraph", "vga", "stepdepth")), ("syn128", ("makegraph", "vga")),
            ("syn128sd", ("stepdepth",)), ("syn32", ("stepdepth",))]
    for name, legs in plan:
        meta, A = load_case(name)
        om = OracleMap(meta["region"], meta["spacing"], case_input_lines(meta))
        for f in meta["fills"]:
            om.fill(*f)
        rec = {}
        t0 = time.perf_counter()
        om.make_graph(threads=1)
        t = time.perf_counter() - t0
        if "makegraph" in legs:
            rec["makegraph"] = {"port_s": t, "ref_s": meta["ref_seconds"]["makegraph"]}
        if "vga" in legs:
            t0 = time.perf_counter()
            om.vga_global(threads=1)
            t = time.perf_counter() - t0
            rec["vga"] = {"port_s": t, "ref_s": meta["ref_seconds"]["vga"]}
        if "stepdepth" in legs and "stepdepth_sel" in A and meta["ref_seconds"].get("stepdepth", 0) > 0:
            ps = A["stepdepth_sel"]                       # PixelRef ints -> x-major cell indices
            sel = (ps >> 16) * meta["rows"] + (ps & 0xFFFF)
            reps = max(1, int(0.5 / max(meta["ref_seconds"]["stepdepth"], 1e-4)))   # short runs: repeat
            t0 = time.perf_counter()
            for _ in range(reps):
                om.metric_stepdepth(sel)
            t = (time.perf_counter() - t0) / reps
            rec["stepdepth"] = {"port_s": t, "ref_s": meta["ref_seconds"]["stepdepth"], "repeats": reps}
        for v in rec.values():
            v["ref_over_port"] = v["ref_s"] / v["port_s"]
        out["cases"][name] = rec
        print(name, rec, flush=True)
    for leg in ("makegraph", "vga", "stepdepth"):
        r = [c[leg]["ref_over_port"] for c in out["cases"].values() if leg in c]
        out["ref_over_port_" + leg] = sum(r) / len(r)
    with open(os.path.join(REPO, "tests", "golden", "oracle_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
