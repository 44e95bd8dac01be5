"""Do the VO sequence's kernels disturb the cross-lane exchanges of a co-resident kernel?  The
permlane_stress victims (tools/ubench/permlane_stress.hip, library form libstress.so) run on their
own stream while the VO sequence (serial and PICP_VO_OVERLAP=1) or a block-kernel batch runs
beside them; every victim result is checked against its analytic value.
usage: python tools/vo_stress.py [reps]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
import picp_amd  # noqa: E402
from picp_amd import synth  # noqa: E402
from picp_amd.vo_synth import VOSequence, segments  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
L = picp_amd.lib()
S = ctypes.CDLL(os.path.join(ROOT, "tools", "ubench", "libstress.so"))
S.stress_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
hip = ctypes.CDLL("libamdhip64.so")
cnt = ctypes.c_void_p()
assert hip.hipMalloc(ctypes.byref(cnt), ctypes.c_size_t(16)) == 0
st = ctypes.c_void_p()
assert hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) == 0

F = 2001
seq = VOSequence(F, obs_per_frame=2000, seed=42)
first, steps = segments(F, 40)
D = seq.frames(0, F)
rel = [np.linalg.inv(D["T_cw"][f].astype(np.float64)) for f in first]
boot = np.stack([[np.eye(4), rel[k] @ D["T_cw"][f + 1]] for k, f in enumerate(first)]).astype(np.float32)
handles = {}
for name, env in (("serial", {}), ("overlap", {"PICP_VO_OVERLAP": "1"})):
    os.environ.update(env)
    v = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], device=0, K=seq.K)
    v.set_segments(first, steps, boot, threshold=3000.0)
    for k in env:
        del os.environ[k]
    handles[name] = v
os.environ["PICP_MODE"] = "block"
bt = synth.make_batch(250, 1500, base_seed=1000)
B = picp_amd.Batch(np.full(250, 1500))
B.set_data(bt["xyz"], bt["uv"])


def beside(victim, what, iters):
    h = np.zeros(2, np.uint64)
    assert hip.hipMemset(cnt, 0, ctypes.c_size_t(16)) == 0
    assert hip.hipDeviceSynchronize() == 0
    for _ in range(reps):
        assert S.stress_launch(victim, 256, iters, st, cnt) == 0
        if what == "batch":
            B.set_poses(bt["T_init"])
            B.solve_async(max_rounds=50, conv_eps=1e-5)
            B.sync()
        elif what != "none":
            L.picp_vo_run_async(handles[what]._h)
            L.picp_vo_sync(handles[what]._h)
        assert hip.hipStreamSynchronize(st) == 0
    assert hip.hipMemcpy(h.ctypes.data_as(ctypes.c_void_p), cnt, ctypes.c_size_t(16), 2) == 0
    if victim in (7, 8, 9, 10):
        print("victim %d beside %-8s: %d mismatches in lanes 0-47, %d in lanes 48-63, %d chain steps"
              % (victim, what, int(h[0]) & 0xFFFFFFFF, int(h[0]) >> 32, int(h[1])), flush=True)
    else:
        print("victim %d beside %-8s: %d mismatches in %d checks" % (victim, what, int(h[0]), int(h[1])), flush=True)


for victim, iters in ((9, 1000), (10, 100)):
    for what in ("none", "serial", "overlap", "batch"):
        beside(victim, what, iters)
