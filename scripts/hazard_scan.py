#!/usr/bin/env python3
"""Scan gfx950 device assembly for a transcendental result read by the very next instruction.

On gfx950 a VALU transcendental (v_rcp / v_sqrt / v_rsq / v_exp / v_log / v_sin / v_cos) needs one wait state
before a dependent non-transcendental VALU reads its result.  The compiler's hazard recognizer inserts the
s_nop for its own instructions but cannot see into inline asm, so an inline-asm helper (max_abs, cvt_flr_i32,
f16_fma_lo, ...) scheduled right after the producer read a half-written register -- a lane-group pattern of
wrong values (round 6: k_eval_ref's paired-sample loop, max_abs of a v_sqrt result).  This scan flags every
(producer, next instruction) pair that reads the producer's result with no instruction in between.

usage: python scripts/hazard_scan.py file.s [...]     (hipcc --cuda-device-only -S output)
       python scripts/hazard_scan.py --so libacmmp.so    (the built library: its gfx950 code objects unbundled
                                                          and disassembled with the image's llvm-objdump)
exit 1 on a hit.
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

TRANS = re.compile(r"^\s*(v_(?:rcp|rcp_iflag|sqrt|rsq|exp|log|sin|cos)_f(?:32|16)(?:_e32|_e64)?)\s+(v\d+)")
INSTR = re.compile(r"^\s*([a-z_][a-z0-9_]*)\b(.*)$")


def regs(operands):
    out = set()
    for m in re.finditer(r"\bv(\d+)\b", operands):
        out.add(int(m.group(1)))
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]", operands):
        out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def disassemble_so(so):
    """The gfx950 code objects of a HIP shared library, disassembled -> list of (name, text)."""
    out = []
    with tempfile.TemporaryDirectory() as td:
        lib = os.path.join(td, "lib.so")
        shutil.copyfile(so, lib)
        subprocess.run([OBJDUMP, "--offloading", lib], check=True, capture_output=True, cwd=td)
        for f in sorted(os.listdir(td)):
            if "gfx950" in f:
                r = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", "--no-leading-addr", os.path.join(td, f)],
                                   check=True, capture_output=True, text=True)
                out.append((f, r.stdout))
    return out


def scan(path, text=None):
    hits = []
    lines = (open(path).read() if text is None else text).split("\n")
    fn = "?"
    for i, line in enumerate(lines):
        if re.match(r"^_Z\w+:", line) or re.match(r"^_Z\w+>:", line.lstrip("<")):
            fn = line.split(":")[0].strip("<>")
        m = TRANS.match(line)
        if not m:
            continue
        dst = int(m.group(2)[1:])
        in_asm = False
        for k in range(i + 1, min(i + 12, len(lines))):
            s = lines[k].strip()
            if s.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if not s or s.startswith(";") or s.startswith("."):
                continue
            s = s.split("//")[0].strip()
            im = INSTR.match(s)
            if not im:
                break
            op, rest = im.group(1), im.group(2)
            srcs = rest.split(",", 1)[1] if "," in rest else ""
            if dst in regs(srcs) and not op.startswith("s_nop"):
                hits.append((path, k + 1, fn, lines[i].strip(), s, in_asm))
            break
    return hits


def scan_so(so):
    hits = []
    for name, text in disassemble_so(so):
        hits += scan(name, text)
    return hits


if __name__ == "__main__":
    allhits = []
    if sys.argv[1:2] == ["--so"]:
        allhits = scan_so(sys.argv[2])
    else:
        for p in sys.argv[1:]:
            allhits += scan(p)
    for h in allhits:
        print(f"{h[0]}:{h[1]} {'(inline asm) ' if h[5] else ''}{h[3]}  ->  {h[4]}   [{h[2][:90]}]")
    print(f"{len(allhits)} trans -> immediate-use pairs")
    sys.exit(1 if allhits else 0)
