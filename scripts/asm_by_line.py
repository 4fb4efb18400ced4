"""Dev tool: static instruction mix of one kernel in a hipcc -S -gline-tables-only
listing, attributed to source-line ranges (Solver member functions).
usage: python scripts/asm_by_line.py <file.s> <kernel-substring> <source.hip>"""
import collections, re, sys
asm, kname, src = sys.argv[1], sys.argv[2], sys.argv[3]
lines = open(asm).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(kname) + r"\S*:", l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
# function ranges from the source: "__device__ ... name(" at line L, next such line ends it
srcl = open(src).read().split("\n")
marks = [(i + 1, re.search(r"(\w+)\(", l).group(1)) for i, l in enumerate(srcl)
         if re.match(r"\s*(__device__|template|__global__)", l) and re.search(r"(\w+)\(", l)]
def region(ln):
    name = "?"
    for L, n in marks:
        if L <= ln: name = n
        else: break
    return name
cur = 0
cnt = collections.defaultdict(collections.Counter)
for l in lines[start:end]:
    m = re.match(r"\s*\.loc\s+\d+\s+(\d+)", l)
    if m:
        cur = int(m.group(1)); continue
    t = l.strip()
    if not t or t.startswith((";", ".", "_")) or t.endswith(":"):
        continue
    op = t.split()[0]
    kind = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") and not op.startswith(("s_waitcnt", "s_load", "s_buffer")) else
            "smem" if op.startswith(("s_load", "s_buffer")) else "vmem" if op.startswith(("global_", "buffer_", "scratch_", "flat_")) else
            "lds" if op.startswith("ds_") else "wait" if op.startswith("s_waitcnt") else "other")
    cnt[region(cur) if cur else "?"][kind] += 1
tot = collections.Counter()
for r, c in sorted(cnt.items(), key=lambda x: -sum(x[1].values())):
    tot.update(c)
    print(f"{r:28s} " + " ".join(f"{k}={c[k]:5d}" for k in ("valu", "salu", "vmem", "lds", "smem", "wait")))
print("total", dict(tot))
