"""The product's host code (the .graph reader/writer, the PointMap chunk codec, the VISPREP host
model) under AddressSanitizer + UndefinedBehaviorSanitizer, on the reference's .graph inputs and
damaged copies of them (tests/san/san_host.cpp).  CPU only; the GPU code has no sanitizer here."""
import lzma
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
HOST = os.path.join(REPO, "depthmapx_amd", "csrc", "host")
INPUTS = os.path.join(HERE, "golden", "graphfiles", "inputs")


@pytest.fixture(scope="module")
def san_bin(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("san") / "san_host")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-static-libasan", "-o", out, os.path.join(HERE, "san", "san_host.cpp"),
           os.path.join(HOST, "graphfile.cpp"), os.path.join(HOST, "graphio.cpp"), os.path.join(HOST, "pointmap.cpp")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return out


def test_host_code_is_sanitizer_clean(san_bin, tmp_path):
    files = []
    for name in sorted(os.listdir(INPUTS)):
        dst = tmp_path / name[:-3]
        with lzma.open(os.path.join(INPUTS, name)) as f:
            dst.write_bytes(f.read())
        files.append(str(dst))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([san_bin, "150"] + files, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    assert "all ok" in r.stdout
