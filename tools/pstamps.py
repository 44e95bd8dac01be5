#!/usr/bin/env python3
"""Phase breakdown of the persistent kernel (diagnostic stamp build), rounds 11 and 12.
Stamps: 0 round start, 1 partial published, 2 leader: sweep done / others: pose received,
3 leader: solve done; and the leader's sweep passes (issue, return) of thread 0."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
os.environ["PICP_LIB"] = os.environ.get("PICP_STAMPS_LIB") or os.path.join(ROOT, "02-visualodometry_amd", "lib", "libpicp_amd_stamps.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--outlier", type=float, default=0.0)
    args = ap.parse_args()
    import numpy as np
    import picp_amd
    from picp_amd import synth
    p = synth.make_problem(args.n, seed=42, outlier_frac=args.outlier, pixel_noise=0.5, shuffle=False)
    b = picp_amd.Batch([args.n])
    info = b.info()
    assert info["mode"] == "persistent", info
    b.set_data(p["xyz"], p["uv"])
    b.set_poses(p["T_init"][None])
    L = picp_amd.lib()
    L.picp_debug_sweepstamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    sw = np.zeros((2, 64), np.uint64)
    for _ in range(3):
        assert L.picp_debug_sweepstamps(sw.ctypes.data, sw.size) == 0  # read = clear
        b.solve(threshold=3000.0, max_rounds=50, conv_eps=-1.0)
    assert L.picp_debug_sweepstamps(sw.ctypes.data, sw.size) == 0
    nb = info["n_blocks"]
    L.picp_debug_pstamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros((2, 256, 8), np.uint64)
    assert L.picp_debug_pstamps(buf.ctypes.data, buf.size) == 0
    for r in (0, 1):
        st = buf[r, :nb].astype(np.int64)
        t0 = st[:, 0].min()
        rel = (st - t0) * 10
        print("round %d (%d blocks), ns from first round start" % (11 + r, nb))
        print("  leader: start %d published %d swept(all threads) %d combined %d solve_start %d solve_end %d" % (rel[0,0], rel[0,1], rel[0,2], rel[0,3], rel[0,4], rel[0,5]))
        # blocks 1..7 are the other solvers (picp_persistent.hip PICP_PSOLVERS), the rest followers
        ns = min(8, nb)
        if ns > 1:
            sol = rel[1:ns]
            print("  solvers 1-%d: published median %d, swept median %d (max %d), solve_end median %d (max %d)" % (
                ns - 1, np.median(sol[:, 1]), np.median(sol[:, 2]), sol[:, 2].max(), np.median(sol[:, 5]), sol[:, 5].max()))
        others = rel[ns:] if nb > ns else rel[1:]
        for k, nm in enumerate(["start", "published", "pose_received"]):
            print("  followers %-11s median %6d  min %6d  max %6d" % (nm, np.median(others[:, k]), others[:, k].min(), others[:, k].max()))
        last_pub = int(rel[:, 1].max())
        # the leader's sweep passes (thread 0): issue -> loads returned, ns from the round start
        p = sw[r].astype(np.int64)
        n = int(np.count_nonzero(p)) // 2
        passes = [((p[2 * i] - t0) * 10, (p[2 * i + 1] - t0) * 10) for i in range(n)]
        print("  leader sweep passes (issue..return ns): %s" % "  ".join("%d..%d" % x for x in passes))
        if passes:
            dur = [b - a for a, b in passes]
            after = [x for x in passes if x[0] >= last_pub]
            print("  pass duration median %d ns (min %d max %d); %d passes, %d issued after the last publish (%d)" %
                  (np.median(dur), min(dur), max(dur), n, len(after), last_pub))
    nxt = (buf[1, :nb, 0].astype(np.int64).min() - buf[0, :nb, 0].astype(np.int64).min()) * 10
    print("round period (first start r11 -> first start r12): %d ns" % nxt)


if __name__ == "__main__":
    main()
