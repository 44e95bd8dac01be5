"""Out-of-bounds store check of the VO path (PICP_VO_GUARD=1 pads around every buffer of the
handle): run the sequence serially and under the concurrent schedule, beside a second sequence,
then count changed pad bytes.  usage: python tools/vo_guard_check.py FRAMES OBS"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "02-visualodometry_amd"))
os.environ["PICP_VO_GUARD"] = "1"
import picp_amd  # noqa: E402
from picp_amd.vo_synth import VOSequence, segments  # noqa: E402

F, OBS = int(sys.argv[1]), int(sys.argv[2])


def make(seed):
    D = VOSequence(F, obs_per_frame=OBS, seed=seed).frames(0, F)
    first, steps = segments(F, 40)
    boot = np.stack([[D["T_cw"][f], D["T_cw"][f + 1]] for f in first])
    v = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], K=VOSequence(2, obs_per_frame=10).K)
    v.set_segments(first, steps, boot)
    return v


def guard(v):
    nb, bi = ctypes.c_int64(0), ctypes.c_int(0)
    picp_amd.lib().picp_vo_debug_guard(v._h, ctypes.byref(nb), ctypes.byref(bi))
    return nb.value, bi.value


for setting in ("", "PICP_VO_OVERLAP=1,PICP_VO_CHAINS=2"):
    for kv in filter(None, setting.split(",")):
        k, val = kv.split("=")
        os.environ[k] = val
    a, b = make(5), make(9)
    print("after create+set_segments:", guard(a), guard(b), flush=True)
    for r in range(4):
        picp_amd.lib().picp_vo_run_async(b._h)
        picp_amd.lib().picp_vo_run_async(a._h)
        picp_amd.lib().picp_vo_sync(a._h)
        picp_amd.lib().picp_vo_sync(b._h)
    print("setting %-40s after 4 concurrent runs: a %s  b %s" % (setting or "(serial)", guard(a), guard(b)), flush=True)
    a.close()
    b.close()
