#!/usr/bin/env python3
"""Tuning sweep (GPU): items-per-block partition for a workload, timed in ONE process with
interleaved rounds (rule: perf deltas from interleaved runs in one process).

  python tools/sweep.py --n 100000 --problems 1 --ipb 256,512,1024,2048
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--problems", type=int, default=1)
    ap.add_argument("--ipb", default="256,512,1024,2048,4096")
    ap.add_argument("--rounds", type=int, default=50)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--interleave", type=int, default=3)
    ap.add_argument("--outlier", type=float, default=0.0)
    ap.add_argument("--env", default="PICP_ITEMS_PER_BLOCK", help="env var the --ipb values are written to")
    args = ap.parse_args()
    import numpy as np
    import picp_amd
    from picp_amd import synth
    if args.problems == 1:
        p = synth.make_problem(args.n, seed=42, outlier_frac=args.outlier, pixel_noise=0.5, shuffle=False)
        xyz, uv, Ti, sizes = p["xyz"], p["uv"], p["T_init"][None], [args.n]
    else:
        bt = synth.make_batch(args.problems, args.n, outlier_frac=args.outlier, pixel_noise=0.5)
        xyz, uv, Ti, sizes = bt["xyz"], bt["uv"], bt["T_init"], bt["sizes"]
    batches = {}
    for ipb in args.ipb.split(","):
        os.environ[args.env] = str(ipb)
        b = picp_amd.Batch(sizes)
        b.set_data(xyz, uv)
        b.set_poses(Ti)
        b.solve(threshold=3000.0, max_rounds=args.rounds, conv_eps=-1.0)  # warm (graph build)
        batches[ipb] = b
    os.environ.pop(args.env, None)
    res = {k: [] for k in batches}
    kus = {}
    for _ in range(args.interleave):
        for ipb, b in batches.items():
            ms, lin = b.time(args.reps, threshold=3000.0, max_rounds=args.rounds, conv_eps=-1.0)
            res[ipb].append(ms / args.reps)
            kus[ipb] = (lin, b.time_single(threshold=3000.0, max_rounds=args.rounds, conv_eps=-1.0))
    corr = sum(sizes)
    for ipb, v in res.items():
        ms = float(np.median(v))
        it_s = len(sizes) * args.rounds / (ms * 1e-3)
        print(json.dumps({args.env: ipb, "blocks": batches[ipb].info()["n_blocks"], "mode": batches[ipb].info()["mode"], "ms_per_solve": round(ms, 4),
                          "us_per_round": round(1000 * ms / (args.rounds + 1), 3),
                          "iter_per_s": round(it_s, 1), "launch_us": round(kus[ipb][0], 3),
                          "pair_us": round(kus[ipb][1], 3),
                          "GBps_alg": round(20 * corr / (kus[ipb][0] * 1e-6) / 1e9, 1),
                          "pose_err": synth.se3_log_norm(batches[ipb].poses()[0], Ti[0] * 0 + (p["T_gt"] if args.problems == 1 else bt["T_gt"][0]))}))


if __name__ == "__main__":
    main()
