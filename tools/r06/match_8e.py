#!/usr/bin/env python3
"""Diagnostic (GPU): the 8e partition's world match in isolation.  Runs SURVEY §8e's partition
(8 segments x 1,250 steps, ground-truth bootstrap), takes segments 0-3's final maps and matches a
late frame of each against prefixes of its map, 4 problems per launch (one chain's world match),
in the accept-only form the VO runs.  Under rocprofv3 --kernel-trace the picp_match_mfma_kernel
dispatches come in the printed order; with the stamps library (PICP_LIB=..._stamps.so) the
candidate counters are printed per launch.

  python tools/r06/match_8e.py [--stamps]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--save", help="npz: keep the maps and queries (no matching)")
    ap.add_argument("--load", help="npz from --save: skip the VO run")
    ap.add_argument("--fracs", default="0.25,0.5,0.8,1.0", help="map prefixes matched")
    args = ap.parse_args()
    if args.stamps:
        os.environ["PICP_LIB"] = os.path.join(ROOT, "02-visualodometry_amd", "lib", "libpicp_amd_stamps.so")
    import numpy as np
    import picp_amd
    from picp_amd.vo_synth import VOSequence, segments
    L_ = picp_amd.lib()
    if args.stamps:
        L_.picp_debug_match_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
    st = np.zeros(4, np.uint64)
    if args.load:
        z = np.load(args.load)
        maps = [z["map%d" % s] for s in range(4)]
        qs = [z["q%d" % s] for s in range(4)]
    else:
        F, L = 10000, 1250
        seq = VOSequence(F, obs_per_frame=2000, seed=42)
        first, steps = segments(F, L)
        D = seq.frames(0, int(first[-1] + steps[-1]) + 1)
        rel = [np.linalg.inv(D["T_cw"][f].astype(np.float64)) for f in first]
        boot = np.stack([[np.eye(4), rel[k] @ D["T_cw"][f + 1]] for k, f in enumerate(first)]).astype(np.float32)
        vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], K=seq.K)
        vo.set_segments(first, steps, boot, threshold=3000.0)
        vo.run()
        maps = [vo.map(s)[1] for s in range(4)]
        # queries: the frame ~1,000 steps into each segment (its world match meets a map of that age)
        qs = [D["desc"][D["frame_off"][f + 1000]:D["frame_off"][f + 1001]] for f in first[:4]]
        if args.save:
            np.savez(args.save, **{"map%d" % s: maps[s] for s in range(4)}, **{"q%d" % s: qs[s] for s in range(4)})
            return
    print("final map sizes:", [len(m) for m in maps], flush=True)
    order = 0
    for frac in [float(x) for x in args.fracs.split(",")]:
        refs = [m[:int(frac * len(m))] for m in maps]
        for r in range(args.reps):
            if args.stamps:
                L_.picp_debug_match_stats(st.ctypes.data, 1)
            out = picp_amd.match_points_batch(qs, refs, 0.2, 0.8, form="accept_only")
            acc = sum(int(o["accepted"].sum()) for o in out)
            line = "launch %d: refs per problem %s, accepted %d" % (order, [len(x) for x in refs], acc)
            if args.stamps:
                L_.picp_debug_match_stats(st.ctypes.data, 0)
                q, c, fb, mx = int(st[2]), int(st[1]), int(st[0]), int(st[3])
                line += ", queries %d, candidates/query %.3f, max %d, full-scan fallbacks %d" % (
                    q, c / max(q, 1), mx, fb)
            print(line, flush=True)
            order += 1
    # duplicate descriptors in a final map (landmarks re-added when unmatched)
    for s, m in enumerate(maps):
        u = np.unique(m.view(np.dtype((np.void, m.dtype.itemsize * m.shape[1]))))
        print("segment %d: map %d points, %d distinct descriptors" % (s, len(m), len(u)), flush=True)


if __name__ == "__main__":
    main()
