"""Compact view of probe_big.py output lines (stdin)."""
import json
import sys

for line in sys.stdin:
    try:
        d = json.loads(line)
    except Exception:
        print(line.rstrip()[:300])
        continue
    if "config" not in d:
        print(d)
        continue
    ph = {k: round(v / 1e6, 2) for k, v in d["phase_cycles_per_src"].items()}
    print(d["config"], "same", d.get("same_as_first"), "est_s", round(d["est_full_vga_s"], 1), "td", round(d.get("topdown_cycles_per_src", 0) / 1e6, 2), ph,
          "Btiles", round(d.get("b_tiles_per_src", 0)), "Bcells", round(d.get("b_cells_per_src", 0)), "TT", round(d.get("tt_tiles_per_src", 0)), "TTprune", round(d.get("tt_pruned_per_src", 0)), "B1", round(d.get("b1_cycles_per_src", 0) / 1e6, 2), "Cbusy/wave", round(d.get("c_busy_per_src", 0) / 16e6, 2), "Cscan/wave", round(d.get("c_scan_per_src", 0) / 16e6, 2), "Cspec/wave", round(d.get("c_spec_per_src", 0) / 16e6, 2), "nspec", round(d.get("n_spec_per_src", 0), 1),
          "hard", round(d["hard_cells_per_src"]), "cert", round(d.get("hard_certain_per_src", 0)),
          "hardruns", round(d["hard_runs_per_src"]), "bu", round(d["levels_bu_per_src"], 3), "special", d.get("special_nodes"))
