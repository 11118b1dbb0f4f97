"""Generate the .graph regression fixtures under tests/golden/graphfiles/ from the REAL reference.

Runs oracle/_ref/ref_cli (our replay of depthmapXcli's runVisualPrep / runVga / runStepDepth on the
reference library built from /root/reference by oracle/Makefile) on the reference's own test inputs
(/root/reference/testdata, the files its RegressionTest cases use, regressionconfig.json) and stores:
  inputs/<file>.graph.xz     the reference's input files (data), xz-compressed
  cases.json                 per case: the command, sha256 + size of the reference's output .graph, the
                             analysis columns, and the sha256 of the output with those columns' values
                             and stats zeroed (graphfile_util.masked_digest)
  <case>_cols.npz            the analysis columns of the reference's output (float32 per attribute row)
The regression runner's check is a byte compare of the output files (RegressionTest/depthmaprunner.py:
72-75); the tests apply it, and where GPU floating-point columns may differ in the last bits they fall
back to the masked compare plus the north-star tolerance on the columns.

Run in this container only (it needs oracle/_ref/ref_cli):  python tests/golden/make_golden_graphfiles.py
"""
import hashlib
import json
import lzma
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, REPO)
import graphfile_util as gu  # noqa: E402

TESTDATA = "/root/reference/testdata"
REF_CLI = os.path.join(REPO, "oracle", "_ref", "ref_cli")
OUT = os.path.join(HERE, "graphfiles")

# Maps made by the reference itself with what depthmapXcli cannot do (the GUI's SEMIFILL fill mode and pencil
# tool, and a LINK run): name -> (source: testdata file or "@name" of an earlier one, ref_cli args).  Their
# reference outputs are stored as inputs/<name>.graph.xz, like the testdata inputs.
#   semi_gallery   gallery grid, one SEMIFILL seed: every cell CONTEXTFILLED (PointMap::makePoints(p, 1),
#                  pointdata.cpp:434-441)
#   mixed_gallery  semi_gallery with a block of cells redrawn by the pencil tool (PointMap::fillPoint remove
#                  then add, pointdata.cpp:375-394): FULL cells inside the context-filled map
#   mixed_link     mixed_gallery made (-pm), then two merge links by the LINK mode (runmethods.cpp:176-188):
#                  a context-filled odd cell to a full cell, and a context-filled even cell to an odd one
GALLERY_BL, GALLERY_S = (0.64, 4.8), 0.04


def _cell_pt(x, y):
    return "%.6f,%.6f" % (GALLERY_BL[0] + GALLERY_S * x, GALLERY_BL[1] + GALLERY_S * y)


PENCIL_BLOCK = [(x, y) for x in range(60, 76) for y in range(40, 53)]   # filtered to filled cells below
LINKS = [((21, 60), (65, 45)), ((100, 20), (25, 31))]
REF_INPUTS = [
    ("semi_gallery", "gallery_empty.graph", ["-m", "VISPREP", "-pg", "0.04", "-pps", "1.32,7.24"]),
    ("mixed_gallery", "@semi_gallery", None),   # pencil args computed from semi_gallery's states
    ("mixed_made", "@mixed_gallery", ["-m", "VISPREP", "-pm"]),
    ("mixed_link", "@mixed_made", ["-m", "LINK"] + sum([["-lnk", _cell_pt(*a) + "," + _cell_pt(*b)] for a, b in LINKS], [])),
]

INPUTS = ["gallery_empty.graph", "gallery_connected.graph", "turns_connected.graph", "rect1x1.graph",
          "barnsbury_drawing.graph", "polygons_drawing.graph"]

VGA_VIS = ["Visual Entropy", "Visual Integration [HH]", "Visual Integration [P-value]", "Visual Integration [Tekl]",
           "Visual Mean Depth", "Visual Node Count", "Visual Relativised Entropy"]
MK = ["Connectivity", "Point First Moment", "Point Second Moment"]

# name, input (testdata file or "@case" = an earlier case's output), mode + args, analysis columns,
# GPU needed, regression case it mirrors (RegressionTest/regressionconfig.json)
CASES = [
    ("dense_fill", "rect1x1.graph", ["-m", "VISPREP", "-pg", "0.02", "-pp", "0.5,0.5"], [], False,
     "dense_pointmap_create_fill_make"),
    ("gallery_grid", "gallery_empty.graph", ["-m", "VISPREP", "-pg", "0.04"], [], False,
     "pointmap_create_fill_make_unmake step 1"),
    ("gallery_fill", "@gallery_grid", ["-m", "VISPREP", "-pp", "1.32,7.24,4.88,5.24"], [], False,
     "pointmap_create_fill_make_unmake step 2"),
    ("gallery_make", "@gallery_fill", ["-m", "VISPREP", "-pm"], [], True, "pointmap_create_fill_make_unmake step 3"),
    ("gallery_unmake", "@gallery_make", ["-m", "VISPREP", "-pu"], [], False, "pointmap_create_fill_make_unmake step 4"),
    ("gallery_one_op", "gallery_empty.graph", ["-m", "VISPREP", "-pg", "0.04", "-pp", "1.32,7.24,4.88,5.24", "-pm"], [],
     True, "pointmap_create_fill_make_one_operation"),
    ("gallery_boundary", "gallery_empty.graph", ["-m", "VISPREP", "-pg", "0.04", "-pp", "1.32,7.24", "-pm", "-pb"], [],
     True, "(-pb boundary graph)"),
    ("gallery_maxdist", "gallery_empty.graph", ["-m", "VISPREP", "-pg", "0.04", "-pp", "1.32,7.24", "-pm", "-pr", "1.5"],
     [], True, "(-pr restricted visibility)"),
    ("barnsbury_make", "barnsbury_drawing.graph", ["-m", "VISPREP", "-pg", "2", "-pp", "531000,184000", "-pm"], [], True,
     "BASELINE configs[0] VISPREP"),
    ("barnsbury_vga", "@barnsbury_make", ["-m", "VGA", "-vm", "visibility", "-vg", "-vr", "n"], VGA_VIS, True,
     "BASELINE configs[0] VGA"),
    # the analyses on the gallery map made above (no merge links)
    ("vis_global_n", "@gallery_one_op", ["-m", "VGA", "-vm", "visibility", "-vg", "-vr", "n"], VGA_VIS, True,
     "visibility_global_n (on the made gallery map)"),
    ("vis_global_3", "@gallery_one_op", ["-m", "VGA", "-vm", "visibility", "-vg", "-vr", "3"],
     [c + " R3" for c in VGA_VIS], True, "visibility_global_3 (on the made gallery map)"),
    ("vis_global_simple", "@gallery_one_op", ["-s", "-m", "VGA", "-vm", "visibility", "-vg", "-vr", "n"],
     ["Visual Integration [HH]"], True, "(-s simple mode)"),
    ("sd_visual", "@gallery_one_op", ["-m", "STEPDEPTH", "-sdt", "visual", "-sdp", "3,5"], ["Visual Step Depth"],
     True, "vga_visual_step_depth (on the made gallery map)"),
    ("sd_metric", "@gallery_one_op", ["-m", "STEPDEPTH", "-sdt", "metric", "-sdp", "3,5"],
     ["Metric Step Shortest-Path Angle", "Metric Step Shortest-Path Length", "Metric Straight-Line Distance"], True,
     "vga_metric_step_depth (on the made gallery map)"),
    ("sd_angular", "@gallery_one_op", ["-m", "STEPDEPTH", "-sdt", "angular", "-sdp", "3,5"],
     ["Angular Step Depth"], True, "vga_angular_step_depth (on the made gallery map)"),
    # turns_connected without its merge links: VISPREP -pu -pl, then -pm
    ("turns_unlink", "turns_connected.graph", ["-m", "VISPREP", "-pu", "-pl"], [], False, "(-pu -pl unmake + unlink)"),
    ("turns_remake", "@turns_unlink", ["-m", "VISPREP", "-pm"], [], True, "(remake after unlink)"),
    ("vga_metric", "@turns_remake", ["-m", "VGA", "-vm", "metric", "-vr", "n"],
     ["Metric Mean Shortest-Path Angle", "Metric Mean Shortest-Path Distance", "Metric Mean Straight-Line Distance",
      "Metric Node Count"], True, "vga_metric (turns map without merge links)"),
    ("vga_angular", "@turns_remake", ["-m", "VGA", "-vm", "angular"],
     ["Angular Mean Depth", "Angular Total Depth", "Angular Node Count"], True, "vga_angular (turns map without merge "
                                                                              "links)"),
    # the regression inputs with merge links (LINK mode, PointMap::mergePixels): the reference's own
    # VGA / STEPDEPTH regression cases (RegressionTest/regressionconfig.json) run on these maps
    ("vis_local", "gallery_connected.graph", ["-m", "VGA", "-vm", "visibility", "-vl"],
     ["Visual Clustering Coefficient", "Visual Control", "Visual Controllability"], True, "visibility_local"),
    ("merge_vis_global_n", "gallery_connected.graph", ["-m", "VGA", "-vm", "visibility", "-vg", "-vr", "n"], VGA_VIS,
     True, "visibility_global_n"),
    ("merge_vis_global_3", "gallery_connected.graph", ["-m", "VGA", "-vm", "visibility", "-vg", "-vr", "3"],
     [c + " R3" for c in VGA_VIS], True, "visibility_global_3"),
    ("merge_sd_visual", "gallery_connected.graph", ["-m", "STEPDEPTH", "-sdt", "visual", "-sdp", "3,5"],
     ["Visual Step Depth"], True, "vga_visual_step_depth"),
    ("merge_sd_metric", "gallery_connected.graph", ["-m", "STEPDEPTH", "-sdt", "metric", "-sdp", "3,5"],
     ["Metric Step Shortest-Path Angle", "Metric Step Shortest-Path Length", "Metric Straight-Line Distance"], True,
     "vga_metric_step_depth"),
    ("merge_sd_angular", "gallery_connected.graph", ["-m", "STEPDEPTH", "-sdt", "angular", "-sdp", "3,5"],
     ["Angular Step Depth"], True, "vga_angular_step_depth"),
    ("merge_vga_metric", "turns_connected.graph", ["-m", "VGA", "-vm", "metric", "-vr", "n"],
     ["Metric Mean Shortest-Path Angle", "Metric Mean Shortest-Path Distance", "Metric Mean Straight-Line Distance",
      "Metric Node Count"], True, "vga_metric"),
    ("merge_vga_angular", "turns_connected.graph", ["-m", "VGA", "-vm", "angular"],
     ["Angular Mean Depth", "Angular Total Depth", "Angular Node Count"], True, "vga_angular"),
    ("merge_vga_metric_gallery", "gallery_connected.graph", ["-m", "VGA", "-vm", "metric", "-vr", "n"],
     ["Metric Mean Shortest-Path Angle", "Metric Mean Shortest-Path Distance", "Metric Mean Straight-Line Distance",
      "Metric Node Count"], True, "vga_metric_only_map (its VGA step)"),
    ("merge_vga_angular_gallery", "gallery_connected.graph", ["-m", "VGA", "-vm", "angular"],
     ["Angular Mean Depth", "Angular Total Depth", "Angular Node Count"], True, "vga_angular_only_map (its VGA step)"),
    # a map with merge links unmade without -pl keeps them; making its graph again writes them back
    ("merge_unmake", "gallery_connected.graph", ["-m", "VISPREP", "-pu"], [], False, "(-pu keeping merge links)"),
    ("merge_remake", "@merge_unmake", ["-m", "VISPREP", "-pm"], [], True, "(making a map with merge links)"),
    ("merge_remake_vga", "@merge_remake", ["-m", "VGA", "-vm", "visibility", "-vg", "-vr", "n"], VGA_VIS, True,
     "(VGA global on the re-made merge-linked map)"),
    # context-filled maps (SEMIFILL): odd cells are skipped as VGA sources and not expanded under a radius
    # or in visual step depth (vgavisualglobal.cpp:75,110, vgavisualglobaldepth.cpp:52, vgavisuallocal.cpp:43)
    ("semi_make", "semi_gallery.graph", ["-m", "VISPREP", "-pm"], [], True, "(makeGraph of a SEMIFILL map)"),
    ("semi_vis_global_n", "@semi_make", ["-m", "VGA", "-vm", "visibility", "-vg", "-vr", "n"], VGA_VIS, True,
     "(VGA global n, context-filled)"),
    ("semi_vis_global_3", "@semi_make", ["-m", "VGA", "-vm", "visibility", "-vg", "-vr", "3"],
     [c + " R3" for c in VGA_VIS], True, "(VGA global 3, context-filled)"),
    ("semi_sd_visual", "@semi_make", ["-m", "STEPDEPTH", "-sdt", "visual", "-sdp", "3,5"], ["Visual Step Depth"], True,
     "(visual step depth, context-filled)"),
    ("semi_vis_local", "@semi_make", ["-m", "VGA", "-vm", "visibility", "-vl"],
     ["Visual Clustering Coefficient", "Visual Control", "Visual Controllability"], True, "(VGA local, context-filled)"),
    ("mixed_make", "mixed_gallery.graph", ["-m", "VISPREP", "-pm"], [], True, "(makeGraph, context-filled + full)"),
    ("mixed_vis_global_n", "@mixed_make", ["-m", "VGA", "-vm", "visibility", "-vg", "-vr", "n"], VGA_VIS, True,
     "(VGA global n, context-filled + full)"),
    ("mixed_vis_global_3", "@mixed_make", ["-m", "VGA", "-vm", "visibility", "-vg", "-vr", "3"],
     [c + " R3" for c in VGA_VIS], True, "(VGA global 3, context-filled + full)"),
    ("mixed_vis_global_5_simple", "@mixed_make", ["-s", "-m", "VGA", "-vm", "visibility", "-vg", "-vr", "5"],
     ["Visual Integration [HH] R5"], True, "(VGA global 5 simple, context-filled + full)"),
    ("mixed_sd_visual", "@mixed_make", ["-m", "STEPDEPTH", "-sdt", "visual", "-sdp", "3,5"], ["Visual Step Depth"],
     True, "(visual step depth, context-filled + full)"),
    ("mixed_sd_visual_full_seed", "@mixed_make", ["-m", "STEPDEPTH", "-sdt", "visual", "-sdp", _cell_pt(65, 45)],
     ["Visual Step Depth"], True, "(visual step depth from a full cell)"),
    ("mixed_sd_metric", "@mixed_make", ["-m", "STEPDEPTH", "-sdt", "metric", "-sdp", "3,5"],
     ["Metric Step Shortest-Path Angle", "Metric Step Shortest-Path Length", "Metric Straight-Line Distance"], True,
     "(metric step depth, context-filled + full)"),
    ("mixed_sd_angular", "@mixed_make", ["-m", "STEPDEPTH", "-sdt", "angular", "-sdp", "3,5"], ["Angular Step Depth"],
     True, "(angular step depth, context-filled + full)"),
    ("mixed_vga_metric", "@mixed_make", ["-m", "VGA", "-vm", "metric", "-vr", "n"],
     ["Metric Mean Shortest-Path Angle", "Metric Mean Shortest-Path Distance", "Metric Mean Straight-Line Distance",
      "Metric Node Count"], True, "(VGA metric, context-filled + full)"),
    ("mixed_vga_angular", "@mixed_make", ["-m", "VGA", "-vm", "angular"],
     ["Angular Mean Depth", "Angular Total Depth", "Angular Node Count"], True, "(VGA angular, context-filled + full)"),
    ("mixed_vis_local", "@mixed_make", ["-m", "VGA", "-vm", "visibility", "-vl"],
     ["Visual Clustering Coefficient", "Visual Control", "Visual Controllability"], True,
     "(VGA local, context-filled + full)"),
    # merge links on context-filled cells: where every level is expanded (radius n, metric, angular) the
    # result does not depend on the pop order inside a level and the GPU path runs them
    ("link_vis_global_n", "mixed_link.graph", ["-m", "VGA", "-vm", "visibility", "-vg", "-vr", "n"], VGA_VIS, True,
     "(VGA global n, merge links on context-filled cells)"),
    ("link_sd_metric", "mixed_link.graph", ["-m", "STEPDEPTH", "-sdt", "metric", "-sdp", "3,5"],
     ["Metric Step Shortest-Path Angle", "Metric Step Shortest-Path Length", "Metric Straight-Line Distance"], True,
     "(metric step depth, merge links on context-filled cells)"),
    ("link_vga_metric", "mixed_link.graph", ["-m", "VGA", "-vm", "metric", "-vr", "n"],
     ["Metric Mean Shortest-Path Angle", "Metric Mean Shortest-Path Distance", "Metric Mean Straight-Line Distance",
      "Metric Node Count"], True, "(VGA metric, merge links on context-filled cells)"),
    ("link_vga_angular", "mixed_link.graph", ["-m", "VGA", "-vm", "angular"],
     ["Angular Mean Depth", "Angular Total Depth", "Angular Node Count"], True,
     "(VGA angular, merge links on context-filled cells)"),
    # ... and where a context-filled end is not expanded (radius 3, visual step depth), it does
    ("link_vis_global_3", "mixed_link.graph", ["-m", "VGA", "-vm", "visibility", "-vg", "-vr", "3"],
     [c + " R3" for c in VGA_VIS], True, "(VGA global 3, merge links on context-filled cells)"),
    ("link_sd_visual", "mixed_link.graph", ["-m", "STEPDEPTH", "-sdt", "visual", "-sdp", "3,5"], ["Visual Step Depth"],
     True, "(visual step depth, merge links on context-filled cells)"),
]


# Cases the engine refuses (DMX_ERR_UNSUPPORTED): a source of VGA global with a radius finds a context-filled
# odd cell (not expanded) and its linked cell at one level, and the reference counts the first or extracts it
# depending on which end it pops first inside the level (vgavisualglobal.cpp:99-122).  The reference's output
# is kept: tests/test_semifill.py shows with the oracle that it changes with that order.
REFUSED = {"link_vis_global_3": "merge links on context-filled cells"}


def _pencil_args(graph):
    """-unpen / -pen for every filled cell of PENCIL_BLOCK (the states come from the map's PointMap chunk)."""
    pm = gu.load_pointmap(graph)
    state, rows = pm["state"], pm["rows"]
    assert abs(pm["bottom_left"][0] - GALLERY_BL[0]) < 1e-9 and abs(pm["bottom_left"][1] - GALLERY_BL[1]) < 1e-9
    args = []
    for x, y in PENCIL_BLOCK:
        if state[x * rows + y] & 0x2:
            args += ["-unpen", _cell_pt(x, y), "-pen", _cell_pt(x, y)]
    assert args
    return ["-m", "VISPREP"] + args


def make_ref_inputs(tmp):
    made = {}
    for name, src, args in REF_INPUTS:
        srcp = made[src[1:]] if src.startswith("@") else os.path.join(TESTDATA, src)
        if args is None:
            args = _pencil_args(srcp)
        dst = os.path.join(tmp, name + ".graph")
        subprocess.check_call([REF_CLI, "-f", srcp, "-o", dst] + args, stdout=subprocess.DEVNULL)
        made[name] = dst
        with open(dst, "rb") as f, lzma.open(os.path.join(OUT, "inputs", name + ".graph.xz"), "wb", preset=9) as o:
            shutil.copyfileobj(f, o)
        print("input", name, os.path.getsize(dst))
    return made


def main():
    os.makedirs(os.path.join(OUT, "inputs"), exist_ok=True)
    for f in INPUTS:
        with open(os.path.join(TESTDATA, f), "rb") as src, lzma.open(os.path.join(OUT, "inputs", f + ".xz"), "wb",
                                                                     preset=9) as dst:
            shutil.copyfileobj(src, dst)
    meta = {}
    outputs = {}
    with tempfile.TemporaryDirectory() as tmp:
        ref_inputs = make_ref_inputs(tmp)
        for name, inp, args, cols, gpu, regression in CASES:
            if inp.startswith("@"):
                src = outputs[inp[1:]]
            elif inp[:-len(".graph")] in ref_inputs:
                src = ref_inputs[inp[:-len(".graph")]]
            else:
                src = os.path.join(TESTDATA, inp)
            dst = os.path.join(tmp, name + ".graph")
            subprocess.check_call([REF_CLI, "-f", src, "-o", dst] + args, stdout=subprocess.DEVNULL)
            outputs[name] = dst
            b = open(dst, "rb").read()
            m = {"input": inp, "args": args, "gpu": gpu, "regression": regression, "size": len(b),
                 "sha256": hashlib.sha256(b).hexdigest(), "columns": cols}
            if name in REFUSED:
                m["refused"] = REFUSED[name]
            if cols:
                m["masked_sha256"] = gu.masked_digest(b, cols)
                got = gu.columns(b, cols)
                assert sorted(got) == sorted(cols), (name, sorted(got))
                np.savez_compressed(os.path.join(OUT, name + "_cols.npz"), **got)
            meta[name] = m
            print(name, len(b), m["sha256"][:16])
    with open(os.path.join(OUT, "cases.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
