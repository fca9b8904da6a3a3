"""Static instruction mix of one kernel in a hipcc -S listing (device asm):
    python profiles/isa/isa_count.py <file.s> <kernel-name-substring>
Counts per class over the whole kernel and per basic block (largest blocks)."""
import re
import sys
from collections import Counter

path, name = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if name in l and not l.startswith((".", "\t", " ")) and ":" in l)
end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
body = lines[start:end]


def cls(op):
    if op.startswith("v_mfma"): return "mfma"
    if op.startswith(("v_exp", "v_rcp", "v_log", "v_sqrt", "v_rsq")): return "valu_trans"
    if op.startswith("v_pk_"): return "valu_pk"
    if op.startswith(("v_accvgpr",)): return "acc_move"
    if op.startswith("v_"): return "valu"
    if op.startswith(("global_load", "buffer_load", "flat_load")): return "vmem_load"
    if op.startswith(("global_store", "buffer_store", "flat_store")): return "vmem_store"
    if op.startswith(("scratch_",)): return "scratch"
    if op.startswith("ds_read") or op.startswith("ds_load"): return "lds_read"
    if op.startswith("ds_write") or op.startswith("ds_store"): return "lds_write"
    if op.startswith("ds_"): return "lds_other"
    if op.startswith("s_waitcnt"): return "waitcnt"
    if op.startswith(("s_load", "s_buffer_load")): return "smem"
    if op.startswith("s_nop"): return "nop"
    if op.startswith("s_"): return "salu"
    return "other"


tot = Counter()
blocks = []
cur, cname = Counter(), "entry"
for l in body:
    s = l.strip()
    if not s or s.startswith((";", ".", "//")):
        if re.match(r"^\.LBB\d+_\d+:", s):
            blocks.append((cname, cur)); cur, cname = Counter(), s
        continue
    if s.endswith(":"):
        blocks.append((cname, cur)); cur, cname = Counter(), s
        continue
    op = s.split()[0]
    c = cls(op)
    tot[c] += 1
    cur[c] += 1
blocks.append((cname, cur))
print("kernel total:", sum(tot.values()), dict(tot.most_common()))
for bn, c in sorted(blocks, key=lambda x: -sum(x[1].values()))[:int(sys.argv[3]) if len(sys.argv) > 3 else 12]:
    print(f"{bn:>16} {sum(c.values()):6d}", dict(c.most_common()))

# per innermost loop header (sum over its blocks: one iteration's static code)
loops = {}
for bn, c in blocks:
    m = re.search(r"Header=(BB\d+_\d+)", bn)
    key = m.group(1) if m else "(no loop)"
    loops.setdefault(key, Counter()).update(c)
for k, c in loops.items():
    print(f"loop {k:>12} {sum(c.values()):6d}", dict(c.most_common()))
