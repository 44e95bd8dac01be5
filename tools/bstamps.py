#!/usr/bin/env python3
"""Phase breakdown of the block kernel (diagnostic stamp build, thread 0 of each block), rounds
11 and 12.  Stamps: 0 round start, 1 linearized, 2 wave partial in LDS, 3 after barrier 1,
4 totals converted (combine + partner exchange), 5 solve done, 6 after barrier 3; words 7/8 are
the block's HW_REG_XCC_ID / HW_REG_HW_ID.  With two blocks per CU (split 4) it also reports how
the two blocks' rounds are phased: 0 = in lockstep, 0.5 = alternating.
  python tools/bstamps.py --problems 250 --n 2000        (C5-like: one block per frame)
  PICP_BLOCK_SPLIT=4 python tools/bstamps.py --problems 128 --n 10000   (C4 per-rank shape at N=8)
PICP_STAMPS_LIB picks the stamp library (default lib/libpicp_amd_stamps.so)."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
os.environ["PICP_LIB"] = os.environ.get("PICP_STAMPS_LIB") or os.path.join(ROOT, "02-visualodometry_amd", "lib", "libpicp_amd_stamps.so")
NB = 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problems", type=int, default=250)
    ap.add_argument("--n", type=int, default=2000)
    args = ap.parse_args()
    import numpy as np
    import picp_amd
    from picp_amd import synth
    ps = [synth.make_problem(args.n, seed=42 + i, pixel_noise=0.5, shuffle=False) for i in range(args.problems)]
    b = picp_amd.Batch([args.n] * args.problems)
    info = b.info()
    assert info["mode"] == "block", info
    b.set_data(np.concatenate([p["xyz"] for p in ps]), np.concatenate([p["uv"] for p in ps]))
    b.set_poses(np.stack([p["T_init"] for p in ps]))
    for _ in range(3):
        b.solve(threshold=3000.0, max_rounds=50, conv_eps=-1.0)
    L = picp_amd.lib()
    L.picp_debug_bstamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros((2, NB, 10), np.uint64)
    assert L.picp_debug_bstamps(buf.ctypes.data, buf.size) == 0
    ran = np.nonzero(buf[0, :, 0] > 0)[0]
    names = ["linearize", "fold+reduce", "barrier1", "combine+exchange", "solve", "barrier3"]
    print("blocks stamped %d, info %s, residency %s" % (len(ran), info, b.residency()))
    for r in (0, 1):
        st = buf[r, ran].astype(np.int64)
        d = np.diff(st[:, :7], axis=1) * 10  # ns (100 MHz s_memrealtime)
        print("round %d: " % (11 + r) + "  ".join("%s %d" % (nm, np.median(d[:, k])) for k, nm in enumerate(names)))
    per = (buf[1, ran, 0].astype(np.int64) - buf[0, ran, 0].astype(np.int64)) * 10
    print("round period median %d ns (min %d max %d)" % (np.median(per), per.min(), per.max()))
    # co-resident blocks: the same (XCD, SE, SH, CU)
    xcc = buf[0, ran, 7].astype(np.int64) & 0xF
    hw = buf[0, ran, 8].astype(np.int64)
    key = xcc * 1024 + ((hw >> 13) & 0x7) * 64 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 0xF)
    groups = {}
    for i, k in zip(ran, key):
        groups.setdefault(int(k), []).append(int(i))
    sizes = np.bincount([len(g) for g in groups.values()])
    print("CUs used %d, blocks per CU histogram %s" % (len(groups), {i: int(c) for i, c in enumerate(sizes) if c}))
    phases, examples = [], []
    for k, g in groups.items():
        if len(g) != 2:
            continue
        a, c = g
        pa = (buf[1, a, 0] - buf[0, a, 0]) * 10
        off = ((int(buf[0, c, 0]) - int(buf[0, a, 0])) * 10) % max(int(pa), 1)
        phases.append(off / max(pa, 1))
        if len(examples) < 6:
            examples.append((a, c, round(off / max(pa, 1), 3)))
    if phases:
        ph = np.minimum(np.array(phases), 1 - np.array(phases))
        print("two-block CUs %d: phase offset (0 lockstep .. 0.5 alternating) median %.3f, p10 %.3f, p90 %.3f"
              % (len(ph), np.median(ph), np.percentile(ph, 10), np.percentile(ph, 90)))
        print("  examples (block a, block b, offset/period):", examples)


if __name__ == "__main__":
    main()
