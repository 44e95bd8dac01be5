#!/usr/bin/env python3
"""Static VGPR-bank census of a kernel's VALU instructions (gfx950 code objects of a HIP .so or
executable; tools/codeobj.py extracts and disassembles them).

A VALU instruction reads its VGPR sources from the SIMD's register file, which is split into 4
banks by register number mod 4; tools/ubench/issue_ubench.hip measures what reading two or three
sources from one bank costs.  For every VALU instruction of the matching kernels
this counts how many of its VGPR source operands share a bank (a register read twice counts twice).

  python tools/bankstat.py LIB_OR_EXE KERNEL_SUBSTRING [--list N]
"""
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import codeobj  # noqa: E402

VREG = re.compile(r"^v(\d+)$|^v\[(\d+):(\d+)\]$")


def vgpr_base(op):
    m = VREG.match(op.strip().lstrip("-|").rstrip("|"))
    if not m:
        return None
    return int(m.group(1) if m.group(1) is not None else m.group(2))


def kernels(path, sub):
    out = {}
    for obj in codeobj.code_objects(codeobj.fatbin_section(path)):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(obj)
            f.flush()
            dis = subprocess.run([os.path.join(codeobj.LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", f.name],
                                 capture_output=True, text=True, check=True).stdout
        sym = None
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                sym = m.group(1) if sub in m.group(1) else None
                if sym:
                    out[sym] = []
                continue
            if sym and line.strip().startswith("v_"):
                out[sym].append(line.split("//")[0].strip())
    return out


def census(insts):
    c = Counter()
    worst = []
    for ins in insts:
        op, _, rest = ins.partition(" ")
        if op.startswith(("v_mfma", "v_readlane", "v_readfirstlane", "v_writelane", "v_accvgpr")):
            continue
        ops = [o.strip() for o in rest.split(",")]
        if len(ops) < 2:
            continue
        srcs = [vgpr_base(o) for o in ops[1:]]
        srcs = [s for s in srcs if s is not None]
        c["valu"] += 1
        if len(srcs) < 2:
            continue
        c["multi_src"] += 1
        banks = Counter(s % 4 for s in srcs)
        top = max(banks.values())
        if top >= 2:
            c["conflict%d" % top] += 1
            worst.append(ins)
    return c, worst


def main():
    path, sub = sys.argv[1], sys.argv[2]
    nlist = int(sys.argv[sys.argv.index("--list") + 1]) if "--list" in sys.argv else 0
    for sym, insts in kernels(path, sub).items():
        c, worst = census(insts)
        print("%s\n  VALU %d, >= 2 VGPR sources %d, two sources in one bank %d, three %d (%.1f %% of VALU)" % (
            sym[:110], c["valu"], c["multi_src"], c["conflict2"], c["conflict3"],
            100.0 * (c["conflict2"] + c["conflict3"]) / max(c["valu"], 1)))
        for w in worst[:nlist]:
            print("    " + w)


if __name__ == "__main__":
    main()
