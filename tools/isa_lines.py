"""Static VALU / SALU / memory instruction counts of a disassembled code object per source line
range (llvm-objdump -d -l of a kernel compiled with -gline-tables-only, e.g. RT_JIT_OPTS=
-gline-tables-only RT_JIT_DUMP=x.co). Usage: python tools/isa_lines.py x.s [file:line ...]
Prints the per-line counts of each source file, largest first."""
import collections
import re
import sys

cur = None
cnt = collections.Counter()
kinds = collections.defaultdict(collections.Counter)
for line in open(sys.argv[1]):
    m = re.match(r"; (.*/)?([\w.]+):(\d+)", line)
    if m:
        cur = (m.group(2), int(m.group(3)))
        continue
    m = re.match(r"\s+([vsdgb]\w*?)_(\w+)", line)
    if m and cur:
        k = {"v": "valu", "s": "salu", "d": "lds", "g": "vmem", "b": "vmem"}[m.group(1)[0]]
        if line.strip().startswith(("s_waitcnt", "s_nop", "s_cbranch", "s_branch")):
            k = "ctl"
        cnt[(cur, k)] += 1
        kinds[cur][k] += 1
by_file = collections.defaultdict(int)
for (src, k), n in cnt.items():
    if k == "valu":
        by_file[src[0]] += n
print("VALU per file:", dict(by_file))
rows = sorted(kinds.items(), key=lambda kv: -kv[1]["valu"])
for (f, ln), c in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 60]:
    print(f"{f}:{ln:5d}  valu {c['valu']:4d}  salu {c['salu']:3d}  lds {c['lds']:3d}  vmem {c['vmem']:3d}")
