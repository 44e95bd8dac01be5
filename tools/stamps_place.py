#!/usr/bin/env python3
"""Where the streaming round's arrival skew comes from (diagnostic stamp build, GPU): per-block
linearize duration of launches j=10/11 of picp_round_kernel, grouped by the XCD (HW_REG_XCC_ID)
and the CU (HW_REG_HW_ID) each block ran on, and whether a block's slowness repeats between the
two launches."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
os.environ["PICP_LIB"] = os.path.join(ROOT, "02-visualodometry_amd", "lib", "libpicp_amd_stamps.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16000000)
    args = ap.parse_args()
    import numpy as np
    import picp_amd
    from picp_amd import synth
    p = synth.make_problem(args.n, seed=42, pixel_noise=0.5, shuffle=False)
    b = picp_amd.Batch([args.n])
    b.set_data(p["xyz"], p["uv"])
    b.set_poses(p["T_init"][None])
    for _ in range(3):
        b.solve(threshold=3000.0, max_rounds=50, conv_eps=-1.0)
    nb = b.info()["n_blocks"]
    L = picp_amd.lib()
    L.picp_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros((2, 4096, 8), np.uint64)
    assert L.picp_debug_stamps(buf.ctypes.data, buf.size) == 0
    durs = []
    for jj in (0, 1):
        st = buf[jj, :nb].astype(np.int64)
        t0 = st[:, 0].min()
        start = (st[:, 0] - t0) * 10
        lin_end = (st[:, 2] - t0) * 10
        dur = lin_end - start
        durs.append(dur)
        xcc = st[:, 6] & 0xF
        hw = st[:, 7]
        cu = (hw >> 8) & 0xF
        sh = (hw >> 12) & 1
        se = (hw >> 13) & 0x7
        print("launch j=%d, %d blocks: entry spread %d ns; linearize end median %d max %d; duration median %d min %d max %d"
              % (10 + jj, nb, start.max(), np.median(lin_end), lin_end.max(), np.median(dur), dur.min(), dur.max()))
        for x in range(8):
            m = xcc == x
            if m.any():
                print("  xcc %d: %3d blocks, start med %6d, end med %6d max %6d, dur med %6d max %6d"
                      % (x, m.sum(), np.median(start[m]), np.median(lin_end[m]), lin_end[m].max(), np.median(dur[m]), dur[m].max()))
        key = xcc * 64 + se * 32 + sh * 16 + cu
        ks, cnt = np.unique(key, return_counts=True)
        print("  distinct CUs %d, blocks per CU: %s" % (len(ks), dict(zip(*np.unique(cnt, return_counts=True)))))
        # co-resident pairs: the later-starting block of a CU
        order = np.argsort(start)
        first_on_cu = {}
        late = np.zeros(nb, bool)
        for i in order:
            if key[i] in first_on_cu:
                late[i] = True
            else:
                first_on_cu[key[i]] = i
        print("  first-on-CU blocks: dur med %d max %d; second-on-CU: dur med %d max %d"
              % (np.median(dur[~late]), dur[~late].max(), np.median(dur[late]) if late.any() else 0, dur[late].max() if late.any() else 0))
        slow = np.argsort(lin_end)[-10:]
        print("  10 latest blocks:", [(int(i), int(xcc[i]), int(se[i]), int(cu[i]), int(start[i]), int(dur[i])) for i in slow])
    print("duration correlation j=10 vs j=11: %.3f" % np.corrcoef(durs[0], durs[1])[0, 1])


if __name__ == "__main__":
    main()
