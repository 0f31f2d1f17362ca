"""Audit the LDS-DMA issue sequences of the built library (gfx950 wait-state rules the compiler's
hazard recognizer does not apply inside inline asm).

For every `buffer_load_dword* ... lds` in the final code object, walk back over the instructions
before it (straight-line, in emission order) and check:
  * a VALU instruction that writes an SGPR the load reads (its descriptor, its soffset, M0) needs
    5 wait states before the load;
  * a SALU write of M0 needs 1 wait state before an LDS-DMA load.
Wait states: every instruction counts 1, `s_nop N` counts N + 1. The walk follows one path only,
so it stops at a branch target (an instruction some s_branch / s_cbranch jumps to: its other
predecessors are not walked) and counts that as a violation unless the 5 wait states are already
in place between the target and the load.

    python tools/check_dma_hazards.py [lib/libmha_hd64.so]
Exit status 1 on a violation. Needs objcopy, clang-offload-bundler and llvm-objdump (ROCm).
"""
import os
import re
import subprocess
import sys
import tempfile

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
LLVM = os.path.join(ROCM, "lib", "llvm", "bin")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd", "lib", "libmha_hd64.so")


def disassemble(lib):
    """The .hip_fatbin section holds one offload bundle per translation unit: unbundle each."""
    lines = []
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bundle")
        # (an explicit output file: objcopy with only an input rewrites it in place)
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", lib, os.path.join(d, "copy.so")],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts = [m.start() for m in re.finditer(re.escape(magic), data)]
        for n, (a, b) in enumerate(zip(starts, starts[1:] + [len(data)])):
            part, co = os.path.join(d, f"b{n}.bundle"), os.path.join(d, f"b{n}.co")
            open(part, "wb").write(data[a:b])
            r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                                f"--input={part}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                               capture_output=True)
            if r.returncode != 0 or not os.path.getsize(co):
                continue
            out = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co], check=True,
                                 capture_output=True, text=True).stdout
            lines += out.splitlines()
    return lines


def sgprs(text):
    out = set()
    for m in re.finditer(r"\bs\[(\d+):(\d+)\]", text):
        out.update(f"s{i}" for i in range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bs(\d+)\b", text):
        out.add(f"s{m.group(1)}")
    if re.search(r"\bm0\b", text):
        out.add("m0")
    return out


def parse(lines):
    """-> list of (function, [(op, dst_text, src_text)], {indices of branch targets})"""
    funcs, cur, addrs, tgts, name, start = [], [], [], [], None, 0

    def close():
        if name is not None:
            at = {a: k for k, a in enumerate(addrs)}
            funcs.append((name, cur, {at[t] for t in tgts if t in at}))

    for raw in lines:
        m = re.match(r"^([0-9a-f]+) <(.+)>:", raw)
        if m:
            close()
            name, start, cur, addrs, tgts = m.group(2), int(m.group(1), 16), [], [], []
            continue
        s = raw.strip()
        if not s or s.startswith(";") or s.endswith(">:") or ":" in s.split()[0]:
            continue
        code, _, comment = s.partition("//")
        a = re.match(r"\s*([0-9A-Fa-f]+):", comment)
        parts = code.strip().split(None, 1)
        op = parts[0]
        args = parts[1] if len(parts) > 1 else ""
        dst, _, src = args.partition(",")
        cur.append((op, dst.strip(), src))
        addrs.append(int(a.group(1), 16) if a else -1)
        t = re.search(r"<[^>+]+\+(0x[0-9a-f]+)>", comment)
        if op.startswith(("s_branch", "s_cbranch")) and t:
            tgts.append(start + int(t.group(1), 16))
    close()
    return funcs


def check(funcs):
    """funcs: (name, instructions[, branch-target indices]) -> (LDS-DMA loads checked, violations)"""
    bad = checked = 0
    for f in funcs:
        name, ins = f[0], f[1]
        targets = f[2] if len(f) > 2 else set()
        for i, (op, dst, src) in enumerate(ins):
            if not (op.startswith("buffer_load_dword") and " lds" in (dst + "," + src) + " "):
                if not (op.startswith("buffer_load_dword") and src.rstrip().endswith("lds")):
                    continue
            checked += 1
            reads = sgprs(src) | {"m0"}
            ws = 0  # wait states between instruction j and the load
            k = i  # the walk has covered ins[k .. i - 1]
            while k > 0 and ws < 5:
                if k in targets:  # other predecessors jump here: not walked
                    print(f"{name}: branch target {ws} wait states before '{op}' (predecessors not checked)")
                    bad += 1
                    break
                j = k - 1
                pop, pdst, _ = ins[j]
                written = sgprs(pdst) if not pop.startswith(("s_nop", "s_waitcnt", "s_barrier", "buffer_", "ds_", "s_cbranch", "s_branch")) else set()
                if pop.startswith("v_") and written & reads:
                    print(f"{name}: VALU '{pop} {pdst}' writes {sorted(written & reads)} {ws} wait states before '{op}'")
                    bad += 1
                if pop.startswith("s_") and "m0" in written and ws < 1:
                    print(f"{name}: SALU '{pop} {pdst}' writes m0 {ws} wait states before '{op}'")
                    bad += 1
                if pop == "s_nop":
                    m = re.match(r"(0x[0-9a-f]+|\d+)", pdst)
                    ws += (int(m.group(1), 0) if m else 0) + 1
                else:
                    ws += 1
                k = j
    return checked, bad


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_LIB
    checked, bad = check(parse(disassemble(lib)))
    print(f"checked {checked} LDS-DMA loads; {bad} wait-state violation(s)")
    return 1 if bad or checked == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
