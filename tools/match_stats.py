#!/usr/bin/env python3
"""Diagnostic (GPU, stamps build): candidate statistics of the MFMA matcher over a C5-shaped VO
run -- queries, candidates rescanned per query, full-scan fallbacks.

  make -C 02-visualodometry_amd stamps && python tools/match_stats.py --frames 2000
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
os.environ["PICP_LIB"] = os.path.join(ROOT, "02-visualodometry_amd", "lib", "libpicp_amd_stamps.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2000)
    ap.add_argument("--seg-len", type=int, default=40)
    args = ap.parse_args()
    import numpy as np
    import picp_amd
    from picp_amd.vo_synth import VOSequence, segments
    seq = VOSequence(args.frames, obs_per_frame=2000, seed=42)
    first, steps = segments(args.frames, args.seg_len)
    D = seq.frames(0, int(first[-1] + steps[-1]) + 1)
    rel = [np.linalg.inv(D["T_cw"][f].astype(np.float64)) for f in first]
    boot = np.stack([[np.eye(4), rel[k] @ D["T_cw"][f + 1]] for k, f in enumerate(first)]).astype(np.float32)
    vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], K=seq.K)
    vo.set_segments(first, steps, boot, threshold=3000.0)
    L = picp_amd.lib()
    L.picp_debug_match_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
    st = np.zeros(4, np.uint64)
    vo.run()
    assert L.picp_debug_match_stats(st.ctypes.data, 1) == 0  # reset after the warm run
    t = time.perf_counter()
    vo.run()
    el = time.perf_counter() - t
    assert L.picp_debug_match_stats(st.ctypes.data, 0) == 0
    q, c, fb, mx = int(st[2]), int(st[1]), int(st[0]), int(st[3])
    print("segments %d, run %.2f ms: queries %d, candidates/query %.3f, max %d, full-scan fallbacks %d (%.4f%%)"
          % (len(first), 1e3 * el, q, c / max(q, 1), mx, fb, 100.0 * fb / max(q, 1)))


if __name__ == "__main__":
    main()
