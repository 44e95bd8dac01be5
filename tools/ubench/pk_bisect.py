#!/usr/bin/env python3
"""Diagnostic (never shipped): which packed-FP32 instructions of permlane_stress victim 9
(apply_update as the compiler emits it with packed FP32) carry the lane 48-63
disagreement seen beside an MFMA kernel?

The victim's device assembly (hipcc -S, packed FP32 allowed) is edited: every packed instruction
NOT in the kept set is replaced by its two 32-bit halves (v_mul/v_add/v_fma_f32 e64, v_mov_b32),
operand halves chosen by op_sel / op_sel_hi, so the edit changes the instruction forms and nothing
else.  Each edited copy is assembled and linked into a code object and run by pk_bisect_host
beside the MFMA aggressor.  A delta-debugging loop shrinks the kept set while the disagreement
stays.  Runs on the GPU box (gpurun); every run is time-limited.

  python tools/ubench/pk_bisect.py OUTDIR [ITERS]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LLVM = "/opt/rocm/lib/llvm/bin"
VICTIM = "_Z6victimILi9EEviPyS0_"


def sh(cmd, timeout=300):
    r = subprocess.run(cmd, shell=True, capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError("%s\n%s%s" % (cmd, r.stdout[-2000:], r.stderr[-2000:]))
    return r.stdout


def regpair(tok):
    """'v[10:11]' -> ('v', 10); 's[20:21]' -> ('s', 20); inline constants -> ('c', text)"""
    m = re.fullmatch(r"([vs])\[(\d+):(\d+)\]", tok)
    if m:
        assert int(m.group(3)) == int(m.group(2)) + 1, tok
        return (m.group(1), int(m.group(2)))
    return ("c", tok)


def half(op, sel):
    kind, v = op
    if kind == "c":
        assert sel == 0, "a constant's high half"
        return v
    return "%s%d" % (kind, v + sel)


def expand(line):
    """the two 32-bit instructions of one packed instruction (lo first, hi second), or None"""
    s = line.strip().split(";")[0].strip()
    m = re.match(r"(v_pk_(mul|add|fma)_f32|v_pk_mov_b32)\s+(.*)$", s)
    if not m:
        return None
    name, rest = m.group(1), m.group(3)
    mods = dict((k, [int(x) for x in v.split(",")]) for k, v in re.findall(r"(\w+):\[([\d,]+)\]", rest))
    ops = [t.strip() for t in re.sub(r"\w+:\[[\d,]+\]", "", rest).split(",")]
    assert not (set(mods) - {"op_sel", "op_sel_hi"}), line
    dst = regpair(ops[0])
    srcs = [regpair(t) for t in ops[1:]]
    n = len(srcs)
    sel_lo = mods.get("op_sel", [0] * n)
    sel_hi = mods.get("op_sel_hi", [1] * n)
    d_lo, d_hi = "v%d" % dst[1], "v%d" % (dst[1] + 1)
    if name == "v_pk_mov_b32":  # D.lo = src0[op_sel[0]], D.hi = src1[op_sel[1]]
        a = half(srcs[0], sel_lo[0])
        b = half(srcs[1], sel_lo[1] if len(sel_lo) > 1 else 0)
        lo = "v_mov_b32_e32 %s, %s" % (d_lo, a)
        hi = "v_mov_b32_e32 %s, %s" % (d_hi, b)
        lo_src, hi_src = [a], [b]
    else:
        op = {"v_pk_mul_f32": "v_mul_f32_e64", "v_pk_add_f32": "v_add_f32_e64", "v_pk_fma_f32": "v_fma_f32"}[name]
        lo_src = [half(x, sel_lo[i]) for i, x in enumerate(srcs)]
        hi_src = [half(x, sel_hi[i]) for i, x in enumerate(srcs)]
        lo = "%s %s, %s" % (op, d_lo, ", ".join(lo_src))
        hi = "%s %s, %s" % (op, d_hi, ", ".join(hi_src))
    # order so that neither half overwrites a register the other still reads
    if d_lo not in hi_src:
        return [lo, hi]
    if d_hi not in lo_src:
        return [hi, lo]
    # each half reads the other's destination (a half-swapped source, e.g. op_sel:[0,1] on the
    # destination pair): swap the pair's halves first, then both halves read their own register
    if name != "v_pk_mov_b32" and d_hi in lo_src and d_lo in hi_src:
        op = lo.split()[0]
        lo_s = [d_lo if x == d_hi else x for x in lo_src]
        hi_s = [d_hi if x == d_lo else x for x in hi_src]
        if d_hi in lo_s or d_lo in hi_s:
            return None
        return ["v_swap_b32 %s, %s" % (d_lo, d_hi), "%s %s, %s" % (op, d_lo, ", ".join(lo_s)),
                "%s %s, %s" % (op, d_hi, ", ".join(hi_s))]
    return None  # left packed


def packed_lines(asm):
    lines = asm.split("\n")
    i = next(k for k, l in enumerate(lines) if l.startswith(VICTIM + ":"))
    j = next(k for k in range(i, len(lines)) if lines[k].startswith(".Lfunc_end"))
    return lines, [k for k in range(i, j) if lines[k].strip().startswith("v_pk_")]


def variant(lines, idx, keep, path):
    out = list(lines)
    for n, k in enumerate(idx):
        if n in keep:
            continue
        e = expand(lines[k])
        if e is None:
            continue
        out[k] = "\n".join("\t" + x for x in e)
    with open(path, "w") as f:
        f.write("\n".join(out))


def run(outdir, lines, idx, keep, tag, iters, aggr=1):
    s = os.path.join(outdir, "v_%s.s" % tag)
    variant(lines, idx, keep, s)
    o = s[:-2] + ".o"
    co = s[:-2] + ".hsaco"
    sh("%s/clang -cc1as -triple amdgcn-amd-amdhsa -target-cpu gfx950 -filetype obj -mrelocation-model pic -o %s %s" % (LLVM, o, s))
    sh("%s/ld.lld -shared %s -o %s" % (LLVM, o, co))
    out = sh("timeout -k 5 90 %s/tools/ubench/pk_bisect_host %s %s %d %d" % (ROOT, co, VICTIM, aggr, iters), timeout=120)
    m = re.search(r"lanes0_47 (\d+) lanes48_63 (\d+) steps (\d+)", out)
    lo, hi, steps = int(m.group(1)), int(m.group(2)), int(m.group(3))
    os.remove(s)
    os.remove(o)
    os.remove(co)
    print("%-24s kept %2d packed  aggressor %d  mismatches lanes 0-47 %8d  48-63 %8d  of %d" %
          (tag, len(keep), aggr, lo, hi, steps), flush=True)
    return lo + hi


def main():
    outdir = sys.argv[1]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    os.makedirs(outdir, exist_ok=True)
    base = os.path.join(outdir, "base.s")
    sh("/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I%s/02-visualodometry_amd/csrc -I%s/include "
       "--cuda-device-only -S %s/tools/ubench/permlane_stress.hip -o %s" % (ROOT, ROOT, ROOT, base))
    lines, idx = packed_lines(open(base).read())
    os.remove(base)
    fixed = [n for n, k in enumerate(idx) if expand(lines[k]) is None]
    print("victim 9: %d packed instructions, %d not expandable (left packed in every run)" % (len(idx), len(fixed)))
    for n, k in enumerate(idx):
        print("  %2d %s%s" % (n, lines[k].strip(), "   [kept]" if n in fixed else ""))
    allset = set(range(len(idx)))
    full = run(outdir, lines, idx, allset, "all_packed", iters)
    run(outdir, lines, idx, allset, "all_packed_alone", iters, aggr=0)
    none = run(outdir, lines, idx, set(fixed), "none_packed", iters)
    if full == 0:
        print("no disagreement with every instruction packed: nothing to bisect")
        return
    if none > 0:
        print("the disagreement stays with every expandable instruction unpacked")
    # one packed instruction at a time, every other one unpacked (a single-instruction cause shows
    # here directly), and each instruction alone unpacked in the packed code
    singles = [n for n in range(len(idx)) if n not in fixed]
    hits = []
    for n in singles:
        if run(outdir, lines, idx, {n} | set(fixed), "only_%02d" % n, iters) > 0:
            hits.append(n)
    print("instructions that reproduce alone (every other one unpacked): %s" % hits)
    for n in hits:
        print("  %2d %s" % (n, lines[idx[n]].strip()))
        run(outdir, lines, idx, {n} | set(fixed), "only_%02d_alone" % n, iters, aggr=0)
        run(outdir, lines, idx, allset - {n}, "all_but_%02d" % n, iters)
    if hits:
        return
    # delta debugging over the kept set (ddmin, complements first)
    keep = sorted(allset - set(fixed))
    n_parts = 2
    step = 0
    while len(keep) >= 2 and step < 40:
        size = (len(keep) + n_parts - 1) // n_parts
        parts = [keep[i:i + size] for i in range(0, len(keep), size)]
        reduced = False
        for p in parts + [sorted(set(keep) - set(q)) for q in parts]:
            step += 1
            if run(outdir, lines, idx, set(p) | set(fixed), "step%02d_n%d" % (step, len(p)), iters) > 0:
                keep = p
                n_parts = max(n_parts - 1, 2) if p in parts else max(n_parts - 1, 2)
                reduced = True
                break
        if not reduced:
            if n_parts >= len(keep):
                break
            n_parts = min(len(keep), 2 * n_parts)
    print("minimal kept set (%d):" % len(keep))
    for n in keep:
        print("  %2d %s" % (n, lines[idx[n]].strip()))
    run(outdir, lines, idx, set(keep) | set(fixed), "minimal", iters)
    run(outdir, lines, idx, set(keep) | set(fixed), "minimal_alone", iters, aggr=0)


if __name__ == "__main__":
    main()
