"""Stream discipline of the library (host code, no GPU needed).

Every device operation of libdmx runs on its context's stream, created hipStreamNonBlocking
(dmx_api.hip, dmx_ctx_create): such a stream is not ordered with the legacy null stream, so a plain
hipMemset / hipMemcpy (null stream, asynchronous for device memory) may still be running when the next
kernel on the context stream starts.  That race was the cause of the 4-rank one-GPU rehearsal's host
heap abort: prepare_symmetry zeroed its per-node counters with hipMemset, the
counting kernel on the context stream sometimes started from stale memory, and the host then indexed a
std::vector with an unwritten entry.  This scan fails on any such call in the library sources."""
import os
import re

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "depthmapx_amd", "csrc")
NULL_STREAM = re.compile(r"\b(hipMemset|hipMemcpy|hipMemsetD8|hipMemsetD32|hipMemcpy2D|hipMemcpyToSymbol)\s*\(")


def test_no_null_stream_copies_or_memsets():
    hits = []
    for root, _, files in os.walk(SRC):
        for f in files:
            if not f.endswith((".hip", ".cpp", ".hpp")):
                continue
            path = os.path.join(root, f)
            for i, line in enumerate(open(path), 1):
                code = line.split("//")[0]
                if NULL_STREAM.search(code):
                    hits.append("%s:%d: %s" % (os.path.relpath(path, SRC), i, line.strip()))
    assert not hits, "null-stream device operations (use the *Async form on the context stream):\n" + "\n".join(hits)
