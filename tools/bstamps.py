#!/usr/bin/env python3
"""Phase breakdown of the block kernel (diagnostic stamp build, thread 0 of each block), rounds
11 and 12.  Stamps: 0 round start, 1 linearized, 2 wave partial in LDS, 3 after barrier 1,
4 totals converted (after barrier 2), 5 solve done, 6 after barrier 3.
  python tools/bstamps.py --problems 250 --n 2000        (C5-like: one block per frame)
  PICP_BLOCK_SPLIT=2 python tools/bstamps.py --problems 128 --n 10000   (C4)"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
os.environ["PICP_LIB"] = os.environ.get("PICP_STAMPS_LIB") or os.path.join(ROOT, "02-visualodometry_amd", "lib", "libpicp_amd_stamps.so")


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
    nb = min(info["n_blocks"], 256)
    L = picp_amd.lib()
    L.picp_debug_bstamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros((2, 256, 8), np.uint64)
    assert L.picp_debug_bstamps(buf.ctypes.data, buf.size) == 0
    names = ["linearize", "fold+reduce", "barrier1", "combine+barrier2", "solve", "barrier3"]
    print("blocks %d, info %s" % (nb, info))
    for r in (0, 1):
        st = buf[r, :nb].astype(np.int64)
        ok = st[:, 0] > 0
        d = np.diff(st[ok, :7], axis=1) * 10  # ns (100 MHz s_memrealtime)
        print("round %d: " % (11 + r) + "  ".join("%s %d" % (nm, np.median(d[:, k])) for k, nm in enumerate(names)))
    per = (buf[1, :nb, 0].astype(np.int64) - buf[0, :nb, 0].astype(np.int64)) * 10
    print("round period median %d ns (min %d max %d)" % (np.median(per), per.min(), per.max()))


if __name__ == "__main__":
    main()
