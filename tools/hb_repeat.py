"""H and b of one linearize (picp_linearize, 100k correspondences, 30 % outliers) repeated, alone
and while a second VO sequence runs beside it; prints how many repeats differ bit-wise from the
first lone one and saves that one to OUT.npz (to compare library builds with numpy afterwards).
usage: python tools/hb_repeat.py OUT"""
import os
import sys
import threading

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "02-visualodometry_amd"))
import picp_amd  # noqa: E402
from picp_amd import synth  # noqa: E402
from picp_amd.vo_synth import VOSequence, segments  # noqa: E402

p = synth.make_problem(100000, seed=7, outlier_frac=0.3)
s = picp_amd.PICPSolver(rows=480, cols=640, K=p["K"])
s.init(p["T_init"], p["world"], p["image"])
s.setKernelThreshold(3000.0)


def lin():
    r = s.linearize(p["pairs"])
    return np.concatenate([r["H"].ravel(), r["b"]])


ref = lin()
alone = sum(int(not np.array_equal(lin(), ref)) for _ in range(20))
F = 1201
D = VOSequence(F, obs_per_frame=1200, seed=9).frames(0, F)
first, steps = segments(F, 40)
boot = np.stack([[D["T_cw"][f], D["T_cw"][f + 1]] for f in first])
vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], K=VOSequence(2, obs_per_frame=10).K)
vo.set_segments(first, steps, boot)
stop = [False]


def vo_loop():
    while not stop[0]:
        vo.run()


th = threading.Thread(target=vo_loop)
th.start()
diffs = []
for _ in range(40):
    x = lin()
    if not np.array_equal(x, ref):
        diffs.append(float(np.max(np.abs(x - ref) / (np.abs(ref).max()))))
stop[0] = True
th.join()
print("alone: %d/20 differ; beside VO: %d/40 differ, max |d| / max|Hb| = %s" %
      (alone, len(diffs), max(diffs) if diffs else 0.0), flush=True)
np.savez(sys.argv[1], hb=ref)
