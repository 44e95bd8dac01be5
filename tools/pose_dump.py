#!/usr/bin/env python3
"""Bit-identity check of two library builds on the bench workloads' solves (GPU):
  python tools/pose_dump.py dump OUT.npz          (PICP_LIB selects the build)
  python tools/pose_dump.py cmp A.npz B.npz       -> per workload: identical or the max |diff|
Workloads: C2 (100k, persistent), C3 (1M 30 % outliers, persistent), a 128 x 10k block batch
(C4 shape), a 250 x 1500 block batch with convergence on, and a 401-frame VO sequence."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "02-visualodometry_amd"))


def dump(path):
    import picp_amd
    from picp_amd import synth
    from picp_amd.vo_synth import VOSequence, segments
    out = {}
    for name, n, frac in (("c2", 100000, 0.0), ("c3", 1000000, 0.3)):
        p = synth.make_problem(n, seed=42, outlier_frac=frac, pixel_noise=0.5, shuffle=False)
        b = picp_amd.Batch([n])
        b.set_data(p["xyz"], p["uv"])
        b.set_poses(p["T_init"][None])
        b.solve(threshold=3000.0, max_rounds=50, conv_eps=-1.0)
        out[name] = b.poses()
        out[name + "_mode"] = np.array([b.info()["mode"]])
    for name, P, n, eps in (("c4", 128, 10000, -1.0), ("blk", 250, 1500, 1e-5)):
        bt = synth.make_batch(P, n, base_seed=1000)
        b = picp_amd.Batch(np.full(P, n))
        b.set_data(bt["xyz"], bt["uv"])
        b.set_poses(bt["T_init"])
        b.solve(threshold=3000.0, max_rounds=50, conv_eps=eps)
        out[name] = b.poses()
        out[name + "_mode"] = np.array([b.info()["mode"]])
    seq = VOSequence(401, obs_per_frame=2000, seed=42)
    D = seq.frames(0, 401)
    first, steps = segments(401, 40)
    boot = np.stack([[D["T_cw"][f], D["T_cw"][f + 1]] for f in first]).astype(np.float32)
    vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], K=seq.K)
    vo.set_segments(first, steps, boot, threshold=3000.0)
    vo.run()
    out["vo"] = np.concatenate([np.asarray(x).reshape(-1) for x in vo.poses()])
    np.savez(path, **out)
    print("dumped", path, {k: (v.shape if v.dtype != object else v) for k, v in out.items() if not k.endswith("_mode")})


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    ok = True
    for k in A.files:
        if k.endswith("_mode"):
            print("%-4s mode %s / %s" % (k[:-5], A[k][0], B[k][0]))
            continue
        same = np.array_equal(A[k].view(np.uint32), B[k].view(np.uint32))
        ok &= same
        print("%-4s %s" % (k, "bit-identical" if same else "DIFFERS, max |d| %.3g" % np.abs(A[k] - B[k]).max()))
    return ok


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(0 if cmp(sys.argv[2], sys.argv[3]) else 1)
