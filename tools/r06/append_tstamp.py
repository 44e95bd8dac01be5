#!/usr/bin/env python3
"""Diagnostic (GPU, -DVOA_TSTAMP build lib/libpicp_amd_voats.so): the VO append's phases at the
8e partition (8 x 1,250 steps) and the default 40-step segments: record + projections, pass 1
(flags and the ordered compaction), pass 2 (triangulate and append), the next problem and state;
mean us per append block.

  PICP_LIB=.../libpicp_amd_voats.so python tools/r06/append_tstamp.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))


def main():
    import numpy as np
    import picp_amd
    from picp_amd.vo_synth import VOSequence, segments
    L = picp_amd.lib()
    L.picp_debug_voa_tstamp.argtypes = [ctypes.c_void_p, ctypes.c_int]
    st = np.zeros(5, np.uint64)
    seq = VOSequence(10000, obs_per_frame=2000, seed=42)
    D = seq.frames(0, 10000)
    for L8 in (1250, 40):
        first, steps = segments(10000, L8)
        rel = [np.linalg.inv(D["T_cw"][f].astype(np.float64)) for f in first]
        boot = np.stack([[np.eye(4), rel[k] @ D["T_cw"][f + 1]] for k, f in enumerate(first)]).astype(np.float32)
        vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], K=seq.K)
        vo.set_segments(first, steps, boot, threshold=3000.0)
        vo.run()
        L.picp_debug_voa_tstamp(st.ctypes.data, 1)
        vo.run()
        L.picp_debug_voa_tstamp(st.ctypes.data, 0)
        n = max(int(st[4]), 1)
        rec = vo.step_records()
        nn = np.concatenate([r["n_new"][1:] for r in rec])
        print("segments of %d steps: %d append blocks, mean new points %.1f; us per block: record+proj %.2f, "
              "pass 1 %.2f, pass 2 %.2f, next problem %.2f" % (L8, n, nn.mean(), *(int(st[k]) / n / 100.0 for k in range(4))),
              flush=True)
        vo.close()


if __name__ == "__main__":
    main()
