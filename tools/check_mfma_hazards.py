"""Audit the built library for VALU reads of an MFMA result too soon after the MFMA (gfx950 wait
states the compiler's hazard recognizer does not count for instructions inside inline asm: an
`asm("v_... %0, %1" : : "v"(acc))` on an accumulator reads the register without the wait states
the recognizer would have put in front of a compiler-visible read).

For every VALU (v_*, not an MFMA) instruction of the final code object, walk back over the
instructions before it in emission order (stopping at a branch target, as tools/check_dma_hazards.py
does) and, for every MFMA whose destination registers overlap the VALU's operands, require the wait
states of the MFMA's pass count between them: XDL write -> VALU read / write, 2 passes 5, 4 passes
7, 8 passes 11, 16 passes 19 (CDNA3 ISA, "Required wait states for MFMA"; gfx950's 32x32x16 f16
form is 8 passes, 16x16x32 4 — the counts the compiler's own reads of them keep). Wait
states: every instruction counts 1, `s_nop N` counts N + 1, an MFMA counts its passes (the pipe
is busy).

    python tools/check_mfma_hazards.py [lib/libmha_hd64.so]
Exit status 1 on a violation (each printed with its kernel and the instructions between).
"""
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
from check_dma_hazards import disassemble  # noqa: E402

PASSES = {  # gfx950 MFMA forms used in this library: passes (4 cycles each)
    "v_mfma_f32_32x32x16_f16": 8, "v_mfma_f32_32x32x16_bf16": 8, "v_mfma_f32_16x16x32_f16": 4,
    "v_mfma_f32_16x16x32_bf16": 4, "v_mfma_f32_32x32x8_f16": 16, "v_mfma_f32_16x16x16_f16": 8,
    "v_mfma_f32_32x32x2_f32": 16, "v_mfma_f32_16x16x4_f32": 8,
}
NEED = {2: 5, 4: 7, 8: 11, 16: 19}
REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        kind = m.group(1)
        lo, hi = (int(m.group(2)), int(m.group(3))) if m.group(2) else (int(m.group(4)), int(m.group(4)))
        out.update((kind, r) for r in range(lo, hi + 1))
    return out


def parse(lines):
    """[(kernel, mnemonic, operands, address)] in emission order; branch targets as addresses."""
    insts, targets, kernel = [], set(), None
    for ln in lines:
        m = re.match(r"^[0-9a-f]+ <(.+)>:", ln)
        if m:
            kernel = m.group(1)
            continue
        if not ln.startswith("\t") or kernel is None:
            continue
        body, _, cmt = ln.partition("//")
        parts = body.strip().split(None, 1)
        if not parts:
            continue
        mn, ops = parts[0], (parts[1] if len(parts) > 1 else "")
        am = re.match(r"\s*([0-9A-F]+):", cmt)
        addr = int(am.group(1), 16) if am else None
        insts.append((kernel, mn, ops, addr))
        tm = re.search(r"<(.+)\+0x([0-9a-f]+)>", cmt)
        if mn.startswith("s_cbranch") or mn == "s_branch":
            tm2 = re.search(r"^\s*[0-9A-F]+:\s*[0-9A-F ]+<.*?\+0x([0-9a-f]+)>", cmt)
            if tm2:
                targets.add((kernel, int(tm2.group(1), 16)))
            elif tm:
                targets.add((kernel, int(tm.group(2), 16)))
    return insts, targets


def audit(insts, targets, window=40):
    bad = []
    kstart = {}
    for i, (k, mn, ops, addr) in enumerate(insts):
        kstart.setdefault(k, addr)
        if not mn.startswith("v_") or mn.startswith("v_mfma"):
            continue
        used = regs(ops)
        if not used:
            continue
        ws = 0
        j = i - 1
        while j >= 0 and i - j <= window and insts[j][0] == k:
            pk, pmn, pops, paddr = insts[j]
            if pmn.startswith("v_mfma"):
                p = PASSES.get(pmn.split("_e64")[0], 16)
                dst = pops.split(",")[0]
                if regs(dst) & used:
                    need = NEED[p]
                    if ws < need:
                        bad.append((k, i, j, ws, need))
                    break
                ws += p
            elif pmn == "s_nop":
                ws += int(pops.strip(), 0) + 1
            else:
                ws += 1
            if ws >= 20:
                break
            # a branch target: other predecessors are not walked
            if insts[j][3] is not None and kstart.get(k) is not None and (k, insts[j][3] - kstart[k]) in targets:
                break
            j -= 1
    return bad


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        REPO, "lightglue-with-flashattentionv2-tensorrt_amd", "lib", "libmha_hd64.so")
    text = disassemble(lib)
    lines = text.split("\n") if isinstance(text, str) else list(text)
    insts, targets = parse(lines)
    bad = audit(insts, targets)
    n_valu = sum(1 for _, mn, _, _ in insts if mn.startswith("v_") and not mn.startswith("v_mfma"))
    for k, i, j, ws, need in bad:
        print(f"{k}: {insts[j][1]} -> {insts[i][1]} {insts[i][2]} after {ws} wait states (needs {need})")
        for t in range(j, i + 1):
            print("    ", insts[t][1], insts[t][2])
    print(f"checked {n_valu} VALU instructions; {len(bad)} MFMA-result hazard(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
