#!/usr/bin/env python3
"""Dump (GPU box) segment 0 of the bench's 8e partition as the GPU ran it -- poses, step records,
the map -- so that its steps can be re-run on the oracle on the CPU (tools/r05/vo_step_cpu.py).

  python3 tools/r05/vo_dump.py OUT.npz [--seg 1250]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--seg", type=int, default=1250)
    a = ap.parse_args()
    import picp_amd
    from picp_amd.vo_synth import VOSequence
    S = a.seg
    seq = VOSequence(S + 2, obs_per_frame=2000, seed=42)
    D = seq.frames(0, S + 1)
    rel = np.linalg.inv(D["T_cw"][0].astype(np.float64))
    boot = np.stack([[np.eye(4), rel @ D["T_cw"][1]]]).astype(np.float32)
    vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], K=seq.K)
    vo.set_segments([0], [S], boot, threshold=3000.0)
    vo.run()
    P, R = vo.poses()[0], vo.step_records()[0]
    mx, md = vo.map(0)
    vo.close()
    np.savez_compressed(a.out, P=P, mx=mx, md=md, **{"R_" + k: np.asarray(v) for k, v in R.items()})
    print("wrote", a.out, P.shape, mx.shape)


if __name__ == "__main__":
    main()
