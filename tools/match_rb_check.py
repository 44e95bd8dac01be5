"""Matcher form invariance on the VO frame pairs: accepted flags and the accepted best indices of
the exact scan vs the accept-only pre-filtered kernel at RB = 1 and RB = 2.
usage: python tools/match_rb_check.py FRAMES OBS SEED"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "02-visualodometry_amd"))
import picp_amd  # noqa: E402
from picp_amd.vo_synth import VOSequence  # noqa: E402

F, OBS, SEED = (int(x) for x in sys.argv[1:4])
D = VOSequence(F, obs_per_frame=OBS, seed=SEED).frames(0, F)
off, desc = D["frame_off"], D["desc"]
d1 = [desc[off[f]:off[f + 1]] for f in range(F - 1)]
d2 = [desc[off[f + 1]:off[f + 2]] for f in range(F - 1)]


def run(env):
    for k, v in env.items():
        os.environ[k] = v
    # the kernel form is an explicit argument (picp_match_batch_form); the two keys name it
    form = "exact" if env.get("PICP_MATCH_EXACT") == "1" else (
        "accept_only" if env.get("PICP_MATCH_ACCEPT_ONLY") == "1" else "full")
    r = picp_amd.match_points_batch(d1, d2, form=form)
    for k in env:
        del os.environ[k]
    acc = np.concatenate([x["accepted"] for x in r])
    bi = np.concatenate([x["best_idx"] for x in r])
    return acc, np.where(acc, bi, -1)


ref = run({"PICP_MATCH_EXACT": "1"})
print("exact: %d queries, %d accepted" % (len(ref[0]), int(ref[0].sum())))
for env in ({"PICP_MATCH_ACCEPT_ONLY": "1", "PICP_MATCH_RB": "1"}, {"PICP_MATCH_ACCEPT_ONLY": "1", "PICP_MATCH_RB": "2"},
            {"PICP_MATCH_RB": "1"}, {"PICP_MATCH_RB": "2"}):
    acc, bi = run(env)
    da = np.nonzero(acc != ref[0])[0]
    db = np.nonzero(bi != ref[1])[0]
    print("%-50s accepted differ: %d  best_idx differ: %d  first: %s" % (env, len(da), len(db), db[:5]), flush=True)
