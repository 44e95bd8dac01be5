#!/usr/bin/env python3
"""CPU evidence for the C5 long-segment drift (VERDICT r04 "What's missing" 1).

Runs the ORACLE's VO loop (oracle.vo_segment: the restated exec/icp_test.cpp:36-136 with
add_new_world_points and DLT, no GPU anywhere) over the first segment of SURVEY §8e's 8-segment
partition of the bench's C5 sequence (picp_amd/vo_synth.py, seed 42, 2,000 observations per
frame; segment 0 = frames 0 .. steps), bootstrapped exactly as bench.py bootstraps it (segment
frame = its first camera, the ground-truth pose pair of frames 0/1), and prints the SE(3) log
drift of each estimated camera-in-world pose from the ground truth at checkpoints, plus the map
size and the per-step correspondence counts.

  python3 tools/r05/oracle_drift.py [--steps 1249] [--mode f64|faithful] [--out path.json]

The resulting log (profiles/r05/drift/) shows whether the 8e partition's large ATE is the
restated reference algorithm's own behaviour (the oracle drifts the same way) or a GPU artefact.
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
    ap.add_argument("--steps", type=int, default=1249)
    ap.add_argument("--f0", type=int, default=0)
    ap.add_argument("--mode", default="f64", choices=("f64", "faithful"))
    ap.add_argument("--obs", type=int, default=2000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import oracle as O
    from picp_amd.synth import se3_log_norm
    from picp_amd.vo_synth import VOSequence
    f0, S = a.f0, a.steps
    seq = VOSequence(f0 + S + 2, obs_per_frame=a.obs, seed=42)
    t0 = time.time()
    D = seq.frames(f0, f0 + S + 1)
    rel = np.linalg.inv(D["T_cw"][0].astype(np.float64))
    T0 = np.eye(4, dtype=np.float32)
    T1 = (rel @ D["T_cw"][1]).astype(np.float32)
    gen_s = time.time() - t0
    t0 = time.time()
    mode = O.MODE_F64 if a.mode == "f64" else O.MODE_FAITHFUL
    r = O.vo_segment(seq.K, 480, 640, D["frame_off"], D["uv"], D["desc"], 0, S, T0, T1, mode=mode)
    run_s = time.time() - t0
    drift = [float(se3_log_norm(r["poses"][t].astype(np.float64), rel @ D["T_cw"][t].astype(np.float64)))
             for t in range(S + 1)]
    pos = np.array([np.linalg.norm(r["poses"][t][:3, 3] - (rel @ D["T_cw"][t])[:3, 3]) for t in range(S + 1)])
    marks = sorted({t for t in (1, 10, 20, 40, 80, 100, 120, 160, 200, 300, 400, 600, 800, 1000, S) if t <= S})
    m = np.cumsum(r["n_new"])
    rows = [{"step": t, "se3_drift": drift[t], "position_err_m": float(pos[t]), "map_points": int(m[t]),
             "n_corr": int(r["n_corr"][t - 1]) if t >= 1 else None} for t in marks]
    out = {"what": "oracle VO loop (oracle.vo_segment, CPU), segment 0 of the 8e partition of the C5 sequence",
           "sequence": "picp_amd/vo_synth.py seed 42, %d obs/frame, frames %d..%d" % (a.obs, f0, f0 + S),
           "bootstrap": "segment frame = frame %d's camera; ground-truth pose pair of frames %d/%d" % (f0, f0, f0 + 1),
           "mode": a.mode, "steps": S, "generate_s": round(gen_s, 1), "oracle_s": round(run_s, 1),
           "checkpoints": rows, "n_corr_min": int(r["n_corr"].min()), "n_corr_max": int(r["n_corr"].max()),
           "final_map_points": int(m[-1]), "drift_all": drift}
    for row in rows:
        print("step %5d  se3 drift %10.4g  position error %9.4g m  map %7d  n_corr %s" % (
            row["step"], row["se3_drift"], row["position_err_m"], row["map_points"], row["n_corr"]))
    print("oracle %.1f s, generator %.1f s, n_corr %d..%d" % (run_s, gen_s, out["n_corr_min"], out["n_corr_max"]))
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
