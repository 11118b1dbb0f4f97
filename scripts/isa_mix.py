"""Instruction mix (scalar / vector / LDS / memory) of the largest loops of makegraph_kernel in an amdgcn .s file.
usage: python scripts/isa_mix.py /tmp/mk_isa.s [n]"""
import collections, re, sys
L = open(sys.argv[1]).read().split("\n")
n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
s = next(i for i, l in enumerate(L) if re.match(r"^_Z\S*makegraph_kernel\S*:", l))
e = next(i for i in range(s, len(L)) if L[i].strip().startswith(".Lfunc_end"))
B = L[s:e]
ext = {}
for i, l in enumerate(B):
    m = re.search(r"Header=(BB\w+) Depth=(\d+)", l)
    if m:
        k = m.group(1); ext.setdefault(k, [int(m.group(2)), i, i]); ext[k][2] = i
for k, (d, a, b) in sorted(ext.items(), key=lambda t: -(t[1][2] - t[1][1]))[:n]:
    c = collections.Counter()
    for l in B[a:b + 1]:
        t = l.strip().split()
        if not t or t[0].startswith((".", ";")): continue
        op = t[0]
        c["s" if op.startswith("s_") else "v" if op.startswith("v_") else "ds" if op.startswith("ds_") else
          "mem" if op.startswith(("global", "scratch", "buffer", "flat")) else "other"] += 1
    print(k, "depth", d, "lines", a, b, dict(c))
