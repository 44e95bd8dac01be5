"""Where the fused VO step (PICP_VO_FUSE=1, run twice) first differs from the separate kernels (0), per
segment: the first step whose pose or record differs, and the records there.
usage: python tools/vo_fuse_diff.py FRAMES OBS [SEED]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "02-visualodometry_amd"))
import picp_amd  # noqa: E402
from picp_amd.vo_synth import VOSequence, segments  # noqa: E402

n, obs = int(sys.argv[1]), int(sys.argv[2])
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 7
s = VOSequence(n, obs_per_frame=obs, seed=seed)
F = s.frames(0, n)
first, steps = segments(n, 40)
rel = [np.linalg.inv(F["T_cw"][f].astype(np.float64)) for f in first]
boot = np.stack([[np.eye(4), rel[k] @ F["T_cw"][f + 1]] for k, f in enumerate(first)]).astype(np.float32)
os.environ["PICP_VO_OVERLAP"] = "0"
os.environ["PICP_VO_CHAINS"] = "1"
res = {}
for fuse in ("0", "1", "1"):
    os.environ["PICP_VO_FUSE"] = fuse
    vo = picp_amd.VOSequence(F["frame_off"], F["uv"], F["desc"], device=0, K=s.K)
    vo.set_segments(first, steps, boot, threshold=3000.0)
    vo.run()
    out = (vo.poses(), vo.step_records(), vo.info())
    vo.close()
    if fuse not in res:
        res[fuse] = out
        print("fuse", fuse, "info", out[2])
    P0, R0, _ = res["0"]
    P, R, _ = out
    for k in range(len(first)):
        d = [t for t in range(len(P0[k])) if not np.array_equal(P0[k][t].view(np.uint32), P[k][t].view(np.uint32))]
        if d:
            t = d[0]
            rec = {f: (int(R0[k][f][t]), int(R[k][f][t])) for f in ("n_corr", "n_in", "rounds", "n_new")}
            print("fuse %s seg %d: %d poses differ, first step %d, records (ref, fused) %s" % (fuse, k, len(d), t, rec))
            break
    else:
        print("fuse %s: every pose equal" % fuse)
