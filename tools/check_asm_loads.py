"""Audit inline-asm VGPR loads in a hipcc .s file (register safety of loads hipcc does not count).

For every `buffer_load_dword*` / `global_load_dword*` with a VGPR destination inside an
`;;#ASMSTART` block, scan forward (straight-line, same basic-block chain in emission order) to the
first `s_waitcnt` that names vmcnt, and report any instruction in between that reads or writes one
of the destination registers (a copy, a spill or a reuse while the load is in flight).

    python tools/check_asm_loads.py file.s [kernel_substring]
Exit status 1 when a kernel has a violation.
"""
import re
import sys


def regs(text):
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]", text):
        out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", text):
        out.add(int(m.group(1)))
    return out


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    lines = open(path).read().splitlines()
    kernel, in_asm, bad, checked = None, False, 0, 0
    pending = []  # (line index, dest regs)
    for i, raw in enumerate(lines):
        l = raw.split(";")[0].strip() if not raw.strip().startswith(";;#ASM") else raw.strip()
        if raw and not raw[0].isspace() and raw.rstrip().endswith(":") and not raw.startswith("."):
            kernel = raw.split(":")[0]
            pending = []
            continue
        if sub and (kernel is None or sub not in kernel):
            continue
        if l.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if l.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not l or l.startswith("."):
            continue
        op = l.split()[0]
        if op == "s_waitcnt" and "vmcnt" in l:
            pending = []
            continue
        if op.startswith("s_endpgm"):
            pending = []
            continue
        # a use of an in-flight destination by anything other than an empty keep-live statement
        args = l[len(op):]
        for (j, d) in pending:
            hit = regs(args) & d
            if hit:
                print(f"{kernel}: line {i + 1}: '{l}' touches v{sorted(hit)} loaded at line {j + 1} before its vmcnt wait")
                bad += 1
        if in_asm and re.match(r"(buffer|global)_load_dword", op) and " lds" not in l:
            dest = args.split(",")[0]
            pending.append((i, regs(dest)))
            checked += 1
    print(f"checked {checked} asm loads; {bad} violation(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
