"""Diagnostic: per-loop instruction counts of a kernel in a hipcc -save-temps .s file (the
chain kernels' 16-step block loops).  python tools/isa_loops.py FILE.s KERNEL_SYMBOL"""
import re, sys
from collections import Counter
src = open(sys.argv[1]).read()
name = sys.argv[2]
a = src.index(name + ":"); b = src.index(".Lfunc_end", a)
lines = src[a:b].split("\n")
labels = {}
for i, l in enumerate(lines):
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        labels[m.group(1)] = i
loops = []
for i, l in enumerate(lines):
    m = re.match(r"^\s+s_cbranch_\w+\s+(\.LBB\d+_\d+)|^\s+s_branch\s+(\.LBB\d+_\d+)", l)
    if m:
        tgt = m.group(1) or m.group(2)
        if tgt in labels and labels[tgt] < i:
            loops.append((labels[tgt], i))
def cat(op):
    if op.startswith("v_"): return "valu"
    if op.startswith("s_waitcnt"): return "waitcnt"
    if op.startswith("s_nop"): return "nop"
    if op.startswith("s_barrier"): return "barrier"
    if op.startswith("s_"): return "salu"
    if op.startswith("ds_"): return "lds"
    if op.startswith(("global_", "buffer_", "flat_")): return "vmem"
    return "other"
for s0, s1 in sorted(loops, key=lambda x: x[1] - x[0], reverse=True)[:int(sys.argv[3]) if len(sys.argv) > 3 else 12]:
    ins = [l.strip().split()[0] for l in lines[s0:s1 + 1] if l.startswith("\t") and not l.strip().startswith((";", "."))]
    c = Counter(cat(o) for o in ins)
    ops = Counter(ins)
    dpp = sum(1 for l in lines[s0:s1 + 1] if "_dpp" in l or "row_bcast" in l or "quad_perm" in l or "row_" in l and l.strip().startswith("v_"))
    print(f"loop lines {s0}-{s1}: {len(ins)} instr  {dict(c)}  dpp={dpp}  top={ops.most_common(8)}")
