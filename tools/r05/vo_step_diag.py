#!/usr/bin/env python3
"""Diagnostic (GPU box): where does a late VO step's GPU pose part from the oracle's?

Runs segment 0 of the bench's 8e partition on the GPU (as tests/test_gpu_vo_long.py does), then
for chosen steps t re-runs the step's PICP from the GPU's own inputs (map prefix, correspondences,
the float32 prior) three ways, round by round:
  * the drop-in PICPSolver (picp_one_round on the device), pose after every round;
  * the oracle's one_round in float64 accumulation and in the reference's float32 arithmetic;
and prints, per round, the SE(3) distances between them, chi_in and n_in; plus, at the prior, the
GPU's H and b (picp_linearize, double) against the oracle's (float64 accumulation).

  python3 tools/r05/vo_step_diag.py [--steps 100,1249] [--rounds N]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", default="100,1249")
    ap.add_argument("--seg", type=int, default=1250)
    a = ap.parse_args()
    import oracle as O
    import picp_amd
    from picp_amd.synth import se3_log_norm
    from picp_amd.vo_synth import VOSequence
    from test_gpu_vo_long import _iso_inverse_f32
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
    K, off, uv, desc = seq.K, D["frame_off"], D["uv"], D["desc"]
    for t in [int(x) for x in a.steps.split(",")]:
        m = int(np.sum(R["n_new"][:t + 1]))
        nf = t + 1
        wm = O.match_points(desc[off[nf]:off[nf + 1]], md[:m])
        pairs = np.stack([np.nonzero(wm["accepted"])[0], wm["best_idx"][wm["accepted"]]], 1).astype(np.int32)
        img = uv[off[nf]:off[nf + 1]]
        T0 = _iso_inverse_f32(P[t])
        gr = int(R["rounds"][t + 1])
        print("=== step %d: map %d, n_corr %d, VO rounds %d, VO chi_in %.6g" % (t, m, len(pairs), gr,
                                                                            float(R["chi_in"][t + 1])))
        s = picp_amd.PICPSolver(K=K)
        s.init(T0, mx[:m], img)
        s.setKernelThreshold(3000.0)
        lin = s.linearize(pairs)
        ol = O.linearize(T0, K, 480, 640, mx[:m], img, pairs, 3000.0, mode=O.MODE_F64)
        Hg, bg = lin["H"], lin["b"]
        Ho, bo = np.asarray(ol["H"], np.float64).reshape(6, 6), np.asarray(ol["b"], np.float64)
        print("  at the prior: |H_gpu - H_f64|max / |H|max %.3g, |b_gpu - b_f64|max / |b|max %.3g, |b|max %.6g, "
              "n_in gpu %d f64 %d, chi_in gpu %.8g f64 %.8g" % (
                  np.abs(Hg - Ho).max() / np.abs(Ho).max(), np.abs(bg - bo).max() / np.abs(bo).max(), np.abs(bo).max(),
                  lin["n_in"], ol["n_in"], lin["chi_in"], ol["chi_in"]))
        Tg = T0.copy()
        Tf64 = T0.copy()
        Tfai = T0.copy()
        s.set_pose(T0)
        for r in range(gr):
            s.oneRound(pairs)
            Tg = s.pose()
            _, Tf64, st64 = O.one_round(Tf64, K, 480, 640, mx[:m], img, pairs, 3000.0, mode=O.MODE_F64)
            _, Tfai, stfa = O.one_round(Tfai, K, 480, 640, mx[:m], img, pairs, 3000.0, mode=O.MODE_FAITHFUL)
            print("  round %2d: gpu vs f64 %.3g, faithful vs f64 %.3g, |step| f64 %.3g; chi_in gpu %.8g f64 %.8g "
                  "faithful %.8g; n_in %d %d %d" % (
                      r + 1, se3_log_norm(Tg, Tf64), se3_log_norm(Tfai, Tf64),
                      se3_log_norm(Tf64, T0), s.chiInliers(), st64["chi_in"], stfa["chi_in"], s.numInliers(),
                      st64["n_in"], stfa["n_in"]))
        vo_pose = np.linalg.inv(P[t + 1].astype(np.float64))
        print("  VO pose vs drop-in after %d rounds: %.3g (bit-equal %s); VO vs f64 %.3g" % (
            gr, se3_log_norm(vo_pose, Tg.astype(np.float64)), np.array_equal(_iso_inverse_f32(P[t + 1]), Tg),
            se3_log_norm(vo_pose, Tf64.astype(np.float64))))
        s.close()


if __name__ == "__main__":
    main()
