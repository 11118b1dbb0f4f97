"""Loop nest of a kernel in an amdgcn .s file (from the compiler's 'Header=... Depth=...' annotations) with the
scratch spill traffic, waits and memory ops inside each loop.  usage: python scripts/isa_nest.py /tmp/mk_isa.s [maxdepth]"""
import re, sys
L = open(sys.argv[1]).read().split("\n")
maxd = int(sys.argv[2]) if len(sys.argv) > 2 else 4
kname = sys.argv[3] if len(sys.argv) > 3 else "makegraph_kernel"
s = next(i for i, l in enumerate(L) if re.match(r"^_Z\S*%s\S*:" % kname, l))
e = next(i for i in range(s, len(L)) if L[i].strip().startswith(".Lfunc_end"))
body = L[s:e]
ext = {}
for i, l in enumerate(body):
    for m in re.finditer(r"(?:Header|Parent Loop)=?\s*(BB\w+)(?: Depth=(\d+))?", l):
        pass
    m = re.search(r"Header=(BB\w+) Depth=(\d+)", l) or re.search(r"Parent Loop (BB\w+) Depth=(\d+)", l)
    if m:
        k = m.group(1); d = int(m.group(2))
        if re.search(r"Parent Loop", l):
            # '.LBBx: ; Parent Loop BBp Depth=d' starts loop x at depth d+1
            mm = re.match(r"^\.L(BB\w+):", l)
            if mm:
                ext.setdefault(mm.group(1), [d + 1, i, i])
            continue
        if k not in ext: ext[k] = [d, i, i]
        ext[k][1] = min(ext[k][1], i); ext[k][2] = max(ext[k][2], i)
def cnt(a, b, pat): return sum(bool(re.search(pat, body[i])) for i in range(a, b + 1))
for k, (d, a, b) in sorted(ext.items(), key=lambda t: t[1][1]):
    if d > maxd: continue
    ins = sum(1 for i in range(a, b + 1) if body[i].startswith("\t") and not body[i].strip().startswith((".", ";")))
    print(f"{'  ' * d}{k:10s} d{d} {a:5d}-{b:5d} ins {ins:5d} scr ld/st {cnt(a, b, 'scratch_load'):3d}/{cnt(a, b, 'scratch_store'):3d} "
          f"rl/wl {cnt(a, b, 'v_readlane_b32 s'):3d}/{cnt(a, b, 'v_writelane'):3d} vmwait {cnt(a, b, 'vmcnt'):3d} "
          f"gld {cnt(a, b, 'global_load'):3d} ds {cnt(a, b, 'ds_'):3d}")
