"""makeGraph's occluder-free spans (depthmapx_amd/csrc/kernels/span.hpp) against the sieve's per-cell rules.

The kernel processes a span of depths row by row: each row's visible depths per gap as one interval, and its
ratio-class boundaries from two evaluations of the per-cell bin decision.  tests/span/span_check.cpp compiles
span.hpp on the host (g++, -ffp-contract=off, as the kernel) and compares, for random gap lists (including
exact quarters and 1/k ends), depth windows and octants, every row's intervals with a cell-by-cell replay of
PointMap::sieve2 (salalib/pointdata.cpp:1512-1565: visit ranges with `firstind`, `centregap`) and every class
boundary with the per-cell bins (whichbin, pointdata.h:432-520).  The GPU side is pinned by the bit-exact
makeGraph tests (tests/test_gpu_parity.py, the whole-map digests in tests/test_gpu_scale.py).
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_span_rows_and_classes_equal_the_per_cell_sieve(tmp_path):
    exe = str(tmp_path / "span_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-include", "algorithm",
                           os.path.join(HERE, "span", "span_check.cpp"), "-o", exe])
    for seed in (11, 12):
        out = subprocess.run([exe, "400", str(seed)], capture_output=True, text=True)
        assert out.returncode == 0, out.stdout + out.stderr[-2000:]
        assert "mismatches 0" in out.stdout, out.stdout
