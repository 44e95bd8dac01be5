#!/usr/bin/env python3
"""Phase breakdown of picp_round_kernel from the diagnostic stamp build (GPU).

Stamps (s_memrealtime, 10 ns ticks), thread 0 of each block, launches j=10 and j=11:
  0 kernel entry, 1 state read, 2 linearize loop done, 3 partial published + ticket taken,
  4 (last arriver only) all partials reduced, 5 (last arriver only) round finished.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
os.environ["PICP_LIB"] = os.path.join(ROOT, "02-visualodometry_amd", "lib", "libpicp_amd_stamps.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--problems", type=int, default=1)
    args = ap.parse_args()
    import numpy as np
    import picp_amd
    from picp_amd import synth
    if args.problems == 1:
        p = synth.make_problem(args.n, seed=42, pixel_noise=0.5, shuffle=False)
        xyz, uv, Ti, sizes = p["xyz"], p["uv"], p["T_init"][None], [args.n]
    else:
        bt = synth.make_batch(args.problems, args.n, pixel_noise=0.5)
        xyz, uv, Ti, sizes = bt["xyz"], bt["uv"], bt["T_init"], bt["sizes"]
    b = picp_amd.Batch(sizes)
    b.set_data(xyz, uv)
    b.set_poses(Ti)
    for _ in range(3):
        b.solve(threshold=3000.0, max_rounds=50, conv_eps=-1.0)
    nb = b.info()["n_blocks"]
    L = picp_amd.lib()
    L.picp_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    L.picp_debug_stamps.restype = ctypes.c_int
    buf = np.zeros((2, 4096, 8), np.uint64)
    assert L.picp_debug_stamps(buf.ctypes.data, buf.size) == 0
    for jj in (0, 1):
        st = buf[jj, :nb].astype(np.int64)
        t0 = st[:, 0].min()
        rel = (st - t0) * 10  # ns
        print("launch j=%d, %d blocks (ns from the first block's entry)" % (10 + jj, nb))
        for k, nm in enumerate(["entry", "state", "linearized", "published"]):
            print("  %-10s median %7d  max %7d" % (nm, np.median(rel[:, k]), rel[:, k].max()))
        last = np.nonzero(st[:, 4] > st[:, 3])[0]  # the last arriver stamped 4 and 5 this launch
        if len(last):
            i = last[np.argmax(st[last, 4])]
            print("  last arriver (block %d): reduced %d, finished %d  (reduce %d ns, solve %d ns)"
                  % (i, rel[i, 4], rel[i, 5], rel[i, 4] - rel[i, 3], rel[i, 5] - rel[i, 4]))
        d = np.diff(rel[:, :4], axis=1)
        print("  phase medians:", dict(zip(["state", "linearize", "publish"], np.median(d, 0).astype(int).tolist())))
    gap = (buf[1, :nb, 0].astype(np.int64).min() - buf[0, :nb, 5].astype(np.int64).max()) * 10
    print("gap round end (j=10) -> first block entry (j=11): %d ns" % gap)


if __name__ == "__main__":
    main()
