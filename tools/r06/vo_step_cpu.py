#!/usr/bin/env python3
"""Re-run steps of a dumped GPU VO segment (tools/r05/vo_dump.py) on the oracle, on the CPU.

Calls tests/test_gpu_vo_long.py's teacher-forced step check with the dump in place of its GPU
fixture -- the rule of DESIGN.md §7: 1e-4 against the reference's float32 arithmetic, and
max(1e-4, 2 x the restatements' cloud) against every restatement in both pose bases, with cond(H)
-- then prints, per step, why the round-5 "world-in-camera" figure (1e-3 at step 1,249) was not
GPU error: it compared the oracle's raw world-in-camera solve with the GPU's Isometry3f inverse of
its camera-in-world pose, i.e. two different functions of the solve.  The oracle's OWN solve,
re-inverted the same way (inverse of its inverse), sits just as far from its raw form: that is the
float32 rotation's departure from orthonormality (|R^T R - I|, chained over the segment) times
the camera's distance from the segment origin.

  python3 tools/r06/vo_step_cpu.py DUMP.npz [--steps 0,100,400,800,1249]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/r06/..
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--steps", default="0,100,400,800,1249")
    a = ap.parse_args()
    import oracle as O
    from picp_amd.synth import se3_log_norm
    from picp_amd.vo_synth import VOSequence
    import test_gpu_vo_long as L
    z = np.load(a.dump)
    P, mx, md = z["P"], z["mx"], z["md"]
    R = {k[2:]: z[k] for k in z.files if k.startswith("R_")}
    S = len(P) - 1
    seq = VOSequence(S + 2, obs_per_frame=2000, seed=42)
    D = seq.frames(0, S + 1)
    g = dict(K=seq.K, D=D, S=S, P=P, R=R, mx=mx, md=md)
    K, off, uv, desc = seq.K, D["frame_off"], D["uv"], D["desc"]
    steps = [int(x) for x in a.steps.split(",")]
    for t in steps:
        L.test_vo_8e_segment_teacher_forced_late_steps(O, g, t)
    print("test checks passed at steps", steps)
    for t in steps:
        m = int(np.sum(R["n_new"][:t + 1]))
        nf = t + 1
        wm = O.match_points(desc[off[nf]:off[nf + 1]], md[:m])
        pairs = np.stack([np.nonzero(wm["accepted"])[0], wm["best_idx"][wm["accepted"]]], 1).astype(np.int32)
        T0 = L._iso_inverse_f32(P[t])
        gr = int(R["rounds"][t + 1])
        Ts, _ = O.solve(T0, K, 480, 640, mx[:m], uv[off[nf]:off[nf + 1]], pairs, 3000.0, max_rounds=gr,
                        conv_eps=-1.0)
        Rg = P[t + 1][:3, :3].astype(np.float64)
        ii = L._iso_inverse_f32(L._iso_inverse_f32(Ts))
        print("step %d: mixed comparison (round 5): raw f64 world-in-camera vs the GPU's inverse of its pose %.3g; "
              "the f64 solve vs its own inverse-of-inverse %.3g; like for like (both inverse-of-inverse) %.3g; "
              "|R^T R - I| %.3g, |t_cw| %.4g" % (
                  t, se3_log_norm(L._iso_inverse_f32(P[t + 1]), Ts), se3_log_norm(ii, Ts),
                  se3_log_norm(L._iso_inverse_f32(P[t + 1]), ii),
                  np.abs(Rg.T @ Rg - np.eye(3)).max(), np.linalg.norm(P[t + 1][:3, 3])))


if __name__ == "__main__":
    main()
