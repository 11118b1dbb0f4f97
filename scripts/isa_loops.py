"""Loops of a kernel in an amdgcn .s file (backward branches), with their scratch traffic and waits.
usage: python scripts/isa_loops.py /tmp/mk_isa.s [kernel-substring]"""
import re, sys
path = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else "makegraph_kernel"
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % want, l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith("\t.section") or lines[i].strip().startswith(".Lfunc_end"))
body = lines[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", l)
    if m: labels[m.group(1)] = i
loops = []
for i, l in enumerate(body):
    m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        loops.append((labels[m.group(2)], i, m.group(2)))
def isins(l): return l.startswith("\t") and not l.strip().startswith((".", ";"))
for a, b, lab in sorted(loops, key=lambda t: t[1] - t[0]):
    seg = body[a:b + 1]
    n = sum(isins(l) for l in seg)
    sl = sum(bool(re.search(r"scratch_load|buffer_load\w* v\d+, off, s\[0:3\]", l)) for l in seg)
    ss = sum(bool(re.search(r"scratch_store|buffer_store\w* v\d+, off, s\[0:3\]", l)) for l in seg)
    wr = sum("v_writelane" in l for l in seg); rd = sum("v_readlane" in l for l in seg)
    w = sum("s_waitcnt" in l for l in seg)
    gl = sum(bool(re.search(r"global_load|flat_load", l)) for l in seg)
    ds = sum(bool(re.search(r"ds_", l)) for l in seg)
    print(f"{lab:12s} lines {a:5d}-{b:5d} ins {n:5d} scratch ld/st {sl:3d}/{ss:3d} wl/rl {wr:3d}/{rd:3d} waitcnt {w:4d} gload {gl:3d} ds {ds:3d}")
