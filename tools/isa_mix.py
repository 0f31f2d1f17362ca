"""Instruction mix of a kernel's basic blocks in a hipcc .s file (finds loops by back edges).

    python tools/isa_mix.py file.s kernel_substring
"""
import re
import sys
from collections import Counter

path, name = sys.argv[1], sys.argv[2]
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith(name) or (l.endswith(":") and name in l and not l.startswith(".")))
end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
body = lines[start:end]
blocks, cur, label = [], [], "entry"
for l in body:
    s = l.strip()
    if re.match(r"^\.LBB\d+_\d+:", s) or re.match(r"^; %bb\.\d+:", s):
        blocks.append((label, cur))
        label, cur = s[:-1], []
        continue
    if not s or s.startswith(";") or s.startswith("."):
        continue
    cur.append(s.split()[0])
blocks.append((label, cur))


def cls(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_exp"):
        return "v_exp"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_")):
        return "vmem"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    return "other"


for label, ops in blocks:
    if len(ops) < 40:
        continue
    c = Counter(cls(o) for o in ops)
    valu_ops = Counter(o for o in ops if cls(o) == "valu")
    print(label, len(ops), dict(c))
    print("   top valu:", valu_ops.most_common(14))
