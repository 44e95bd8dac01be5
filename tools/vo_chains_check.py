"""Determinism check of the VO step scheduling (PICP_VO_CHAINS / OVERLAP / GRAPH / PRIO): the
same synthetic sequence run under each setting, compared bit for bit with the first.
usage: python tools/vo_chains_check.py FRAMES[:OBS[:SEED]] "ENV=V,ENV=V" ...   (first = reference)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "02-visualodometry_amd"))
import picp_amd  # noqa: E402
from picp_amd.vo_synth import VOSequence, segments  # noqa: E402

spec = [int(x) for x in sys.argv[1].split(":")]
F, OBS, SEED = (spec + [2000, 42][len(spec) - 1:])[:3]
seq = VOSequence(F, obs_per_frame=OBS, seed=SEED)
first, steps = segments(F, 40)
D = seq.frames(0, F)
rel = [np.linalg.inv(D["T_cw"][f].astype(np.float64)) for f in first]
boot = np.stack([[np.eye(4), rel[k] @ D["T_cw"][f + 1]] for k, f in enumerate(first)]).astype(np.float32)
ref = None
for setting in sys.argv[2:]:
    keys = []
    for kv in filter(None, setting.split(",")):
        k, v = kv.split("=")
        os.environ[k] = v
        keys.append(k)
    vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], device=0, K=seq.K)
    vo.set_segments(first, steps, boot, threshold=3000.0)
    outs = []
    for rep in range(3):
        vo.run()
        PL = vo.poses()
        P = np.concatenate([np.asarray(p).reshape(-1) for p in PL])
        R = vo.step_records()
        n_new = np.concatenate([np.asarray(r["n_new"]) for r in R])
        M = [vo.map(k) for k in range(len(first))] if rep == 0 else None
        outs.append((P, n_new, PL, R, M))
    vo.close() if hasattr(vo, "close") else None
    if ref is None:
        ref = outs[0]
    bad = [int(not (np.array_equal(P.view(np.uint32), ref[0].view(np.uint32)) and np.array_equal(n, ref[1])))
           for P, n, _, _, _ in outs]
    dmax = max(float(np.abs(P - ref[0]).max()) for P, _, _, _, _ in outs)
    # the first differing (segment, step) of rep 0 and what differs in its step record
    segs = []
    for k in range(len(first)):
        a, b = np.asarray(outs[0][2][k]), np.asarray(ref[2][k])
        if not np.array_equal(a, b):
            t = int(np.nonzero([not np.array_equal(a[i], b[i]) for i in range(len(a))])[0][0])
            ra, rb = outs[0][3][k], ref[3][k]
            diff = {f: (float(ra[f][t]), float(rb[f][t])) for f in ra
                    if float(ra[f][t]) != float(rb[f][t])}
            tn = [i for i in range(len(ra["n_new"])) if int(ra["n_new"][i]) != int(rb["n_new"][i])]
            # the first differing map point and the step that appended it (slot 0 = bootstrap)
            ma, mb = outs[0][4][k], ref[4][k]
            nn = min(len(ma[0]), len(mb[0]))
            dm = np.nonzero(np.any(ma[0][:nn] != mb[0][:nn], axis=1))[0]
            cum = np.cumsum(np.asarray(rb["n_new"]))
            mstep = int(np.searchsorted(cum, dm[0], side="right")) - 1 if len(dm) else None
            segs.append((k, t, diff, tn[:3], "map pt %s (appended at step %s)" % (dm[0] if len(dm) else None, mstep)))
    if segs:
        print("  differing segments %d, first: %s" % (len(segs), segs[:6]), flush=True)
    print("setting %-40s reps differing from reference: %s  max |dpose| %.3g" % (setting or "(default)", bad, dmax),
          flush=True)
    for k in keys:
        del os.environ[k]
