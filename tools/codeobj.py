"""The gfx950 code objects inside a HIP shared library, and an ISA census of them.

A HIP .so keeps every translation unit's device code as a clang offload bundle in its
.hip_fatbin section (one bundle per TU, concatenated).  This reads the bundles, disassembles each
gfx950 code object with llvm-objdump and counts, per kernel symbol, the instruction classes the
build rules of DESIGN.md §4.9 forbid in shipped code:
  pk_f32 : packed-FP32 VALU (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32)
  calls  : s_swappc_b64 (a function call inside a kernel: nothing should be left un-inlined)
usage: python tools/codeobj.py LIB.so   -> one line per kernel with non-zero counts, then totals
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def fatbin_section(path):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "fat.bin")
        subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + out,
                               path, os.path.join(d, "copy")])
        return open(out, "rb").read()


def code_objects(blob, arch="gfx950"):
    """Every code object for `arch` in the concatenated bundles of a .hip_fatbin section."""
    objs = []
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + len(MAGIC))[0]
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.endswith(arch) and size:
                objs.append(blob[pos + off:pos + off + size])
        pos = blob.find(MAGIC, pos + len(MAGIC))
    return objs


PATTERNS = {"pk_f32": re.compile(r"^\s*v_pk_(fma|mul|add)_f32\b"), "calls": re.compile(r"^\s*s_swappc_b64\b")}


def census(path, arch="gfx950"):
    """{kernel symbol: {class: count}} over every code object of the library."""
    out = {}
    for i, obj in enumerate(code_objects(fatbin_section(path), arch)):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(obj)
            f.flush()
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", f.name],
                                 capture_output=True, text=True, check=True).stdout
        sym = None
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                sym = m.group(1)
                out.setdefault(sym, {k: 0 for k in PATTERNS})
                continue
            if sym is None:
                continue
            for k, rx in PATTERNS.items():
                if rx.match(line):
                    out[sym][k] += 1
    return out


if __name__ == "__main__":
    c = census(sys.argv[1])
    tot = {k: 0 for k in PATTERNS}
    for sym, cnt in sorted(c.items()):
        for k in tot:
            tot[k] += cnt[k]
        if any(cnt.values()):
            print("%-90s %s" % (sym[:90], " ".join("%s=%d" % kv for kv in cnt.items())))
    print("symbols %d  totals %s" % (len(c), " ".join("%s=%d" % kv for kv in tot.items())))
