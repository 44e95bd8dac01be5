#!/usr/bin/env python3
"""How sensitive is one VO step's PICP solve to float rounding, as the segment's map drifts?
(CPU only; the evidence behind the tolerance of tests/test_gpu_vo_long.py.)

Runs the oracle's VO loop (oracle.vo_segment, float64 accumulation) over frames 0 .. S of the
bench's C5 sequence (seed 42, 2,000 obs/frame, segment 0 of the 8e partition), then at each
checkpoint step t re-solves the step from the oracle's own inputs (its map prefix and pose of
frame t -- teacher forcing) three ways:
  * f64      : float32 per-point math, float64 sums and LDL^T (the mode the GPU tests compare to)
  * faithful : float32 sequential sums and float32 LDL^T (the reference's own arithmetic)
  * f64, prior nudged by one float32 ulp in each translation component
and prints the SE(3) log distance between the three results, the rounds run, chi_in and n_in.
If f64 and faithful (two correct restatements of the same algorithm) disagree by far more than
1e-4, the step is ill-conditioned and a 1e-4 pose bar cannot separate a correct GPU from a wrong
one there; the GPU is then held to the oracle's own mode spread instead.

  python3 tools/r05/step_sensitivity.py [--steps 400] [--check 100,200,300,400] [--out f.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--check", default="40,100,200,300,400")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import oracle as O
    from picp_amd.synth import se3_log_norm
    from picp_amd.vo_synth import VOSequence
    S = a.steps
    seq = VOSequence(S + 2, obs_per_frame=2000, seed=42)
    D = seq.frames(0, S + 1)
    rel = np.linalg.inv(D["T_cw"][0].astype(np.float64))
    T0 = np.eye(4, dtype=np.float32)
    T1 = (rel @ D["T_cw"][1]).astype(np.float32)
    t0 = time.time()
    r = O.vo_segment(seq.K, 480, 640, D["frame_off"], D["uv"], D["desc"], 0, S, T0, T1, mode=O.MODE_F64)
    run_s = time.time() - t0
    off, uv, desc, K = D["frame_off"], D["uv"], D["desc"], seq.K
    mx, md = r["map_xyz"], r["map_desc"]
    rows = []

    def cw(Twc):
        return np.linalg.inv(Twc.astype(np.float64))

    for t in [int(x) for x in a.check.split(",") if int(x) < S]:
        m = int(np.sum(r["n_new"][:t + 1]))
        nf = t + 1
        wm = O.match_points(desc[off[nf]:off[nf + 1]], md[:m])
        pairs = np.stack([np.nonzero(wm["accepted"])[0], wm["best_idx"][wm["accepted"]]], 1).astype(np.int32)
        Tp = np.linalg.inv(r["poses"][t].astype(np.float64)).astype(np.float32)  # world-in-camera prior
        img = uv[off[nf]:off[nf + 1]]
        Tf64, s64 = O.solve(Tp, K, 480, 640, mx[:m], img, pairs, 3000.0, mode=O.MODE_F64)
        Tfai, sfa = O.solve(Tp, K, 480, 640, mx[:m], img, pairs, 3000.0, mode=O.MODE_FAITHFUL)
        Tn = Tp.copy()
        Tn[:3, 3] = np.nextafter(Tn[:3, 3], np.float32(np.inf))
        Tnud, snu = O.solve(Tn, K, 480, 640, mx[:m], img, pairs, 3000.0, mode=O.MODE_F64)
        row = {"step": t, "map_points": m, "n_corr": int(len(pairs)),
               "f64_vs_faithful": float(se3_log_norm(cw(Tf64), cw(Tfai))),
               "f64_vs_nudged_prior": float(se3_log_norm(cw(Tf64), cw(Tnud))),
               "f64_vs_vo_run": float(se3_log_norm(cw(Tf64), r["poses"][t + 1].astype(np.float64))),
               "rounds": [int(s64["rounds"]), int(sfa["rounds"]), int(snu["rounds"])],
               "chi_in": [float(s64["chi_in"]), float(sfa["chi_in"])], "n_in": [int(s64["n_in"]), int(sfa["n_in"])],
               "drift_vs_gt": float(se3_log_norm(r["poses"][t].astype(np.float64), rel @ D["T_cw"][t].astype(np.float64)))}
        rows.append(row)
        print("step %4d map %6d n_corr %4d | f64 vs faithful %9.3g  f64 vs 1-ulp prior %9.3g | rounds %s  chi_in %s  "
              "n_in %s | drift %.3g" % (t, m, row["n_corr"], row["f64_vs_faithful"], row["f64_vs_nudged_prior"],
                                        row["rounds"], ["%.4g" % c for c in row["chi_in"]], row["n_in"],
                                        row["drift_vs_gt"]), flush=True)
    out = {"what": "per-step PICP sensitivity along the oracle's own VO run (segment 0 of the 8e partition)",
           "oracle_run_s": round(run_s, 1), "steps": S, "rows": rows}
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
