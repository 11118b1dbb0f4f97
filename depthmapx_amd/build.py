"""In-tree build of libdmx.so for gfx950 (hipcc).  Sources: csrc/dmx_api.hip (unity build with the
kernels) + csrc/host/*.cpp.  -ffp-contract=off keeps every FP64 expression in the reference's
rounding order (no FMA contraction) on host and device."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_lib", "libdmx.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DMX_OFFLOAD_ARCH", "gfx950")

SOURCES = ["dmx_api.hip", "host/pointmap.cpp", "host/graphio.cpp", "host/graphfile.cpp"]
FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-fno-fast-math", "-Wall", "-Wno-unused-variable", "-Wno-unused-function",
         "-Wno-bitwise-instead-of-logical"]


def _deps():
    out = []
    for root, _, files in os.walk(CSRC):
        for f in files:
            if f.endswith((".hip", ".cpp", ".hpp", ".h")):
                out.append(os.path.join(root, f))
    out.append(os.path.join(os.path.dirname(HERE), "include", "dmx.h"))
    return out


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(p) <= t for p in _deps())


CLI_SRC = os.path.join(CSRC, "cli", "dmxcli.cpp")
CLI_OUT = os.path.join(HERE, "_lib", "dmxcli")


def build_cli(verbose=True):
    """The depthmapXcli-compatible front-end (host C++ over libdmx.so)."""
    if os.path.exists(CLI_OUT) and os.path.getmtime(CLI_OUT) >= max(os.path.getmtime(CLI_SRC), os.path.getmtime(OUT)):
        return CLI_OUT
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-Wall", CLI_SRC, "-o", CLI_OUT,
           "-L" + os.path.dirname(OUT), "-ldmx", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return CLI_OUT


def build(force=False, verbose=True):
    if not force and up_to_date():
        build_cli(verbose)
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [HIPCC] + FLAGS + ["-o", OUT] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    build_cli(verbose)
    return OUT


if __name__ == "__main__":
    build(force=True)
