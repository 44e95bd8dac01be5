#!/usr/bin/env python3
"""Phase stamps of the pair-mode kernel (diagnostic stamp build of picp_pair.hip), rounds 11-12,
per frame of a block: 0 worker wave 0 has the pose, 1 it has published its sums, 2 the finishing
wave has every arrival, 3 its exchange is done, 4 the new pose is published.
  PICP_BLOCK_PAIR=1 python tools/pair_stamps.py --problems 128 --n 10000
PICP_STAMPS_LIB picks the stamp library (default lib/libpicp_amd_pairstamps.so)."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
os.environ["PICP_LIB"] = os.environ.get("PICP_STAMPS_LIB") or os.path.join(ROOT, "02-visualodometry_amd", "lib",
                                                                           "libpicp_amd_pairstamps.so")
os.environ.setdefault("PICP_BLOCK_PAIR", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problems", type=int, default=128)
    ap.add_argument("--n", type=int, default=10000)
    args = ap.parse_args()
    import numpy as np
    import picp_amd
    from picp_amd import synth
    bt = synth.make_batch(args.problems, args.n, base_seed=1000, pixel_noise=0.5)
    b = picp_amd.Batch(bt["sizes"])
    b.set_data(bt["xyz"], bt["uv"])
    b.set_poses(bt["T_init"])
    for _ in range(3):
        b.solve(threshold=3000.0, max_rounds=50, conv_eps=-1.0)
    L = picp_amd.lib()
    L.picp_debug_pair_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros((2, 256, 2, 8), np.uint64)
    assert L.picp_debug_pair_stamps(buf.ctypes.data, buf.size) == 0
    ran = np.nonzero(buf[0, :, 0, 0] > 0)[0]
    print("blocks stamped %d, info %s, residency %s" % (len(ran), b.info(), b.residency()))
    st = buf[:, ran].astype(np.int64) * 10  # ns
    for f in (0, 1):
        a = st[0, :, f]
        nxt = st[1, :, f]
        print("frame %d, round 11 (median ns from the worker's pose): lin %d | to all arrivals %d | exchange %d | "
              "finish+publish %d | next round's pose seen %d" % (
                  f, np.median(a[:, 1] - a[:, 0]), np.median(a[:, 2] - a[:, 0]), np.median(a[:, 3] - a[:, 2]),
                  np.median(a[:, 4] - a[:, 3]), np.median(nxt[:, 0] - a[:, 0])))
    print("frame 1 linearize starts after frame 0's by %d ns (median)" % np.median(st[0, :, 1, 0] - st[0, :, 0, 0]))


if __name__ == "__main__":
    main()
