"""Which VO kernel perturbs a block-mode batch solving beside it?  The batch is run beside a VO
handle whose sequence leaves out one kernel kind (PICP_VO_DIAG_SKIP, read at the first run)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "02-visualodometry_amd"))
import picp_amd  # noqa: E402
from picp_amd import synth  # noqa: E402
from picp_amd.vo_synth import VOSequence, segments  # noqa: E402

os.environ["PICP_MODE"] = "block"
bt = synth.make_batch(250, 1500, base_seed=1000)
B = picp_amd.Batch(np.full(250, 1500))
B.set_data(bt["xyz"], bt["uv"])


def run_batch():
    B.set_poses(bt["T_init"])
    B.solve(max_rounds=50, conv_eps=1e-5)
    return B.poses()


ref = run_batch()
F = 1201
D = VOSequence(F, obs_per_frame=1200, seed=9).frames(0, F)
first, steps = segments(F, 40)
boot = np.stack([[D["T_cw"][f], D["T_cw"][f + 1]] for f in first])
vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], K=VOSequence(2, obs_per_frame=10).K)
vo.set_segments(first, steps, boot)
vo.run()
marks = []
for r in range(8):
    B.set_poses(bt["T_init"])
    picp_amd.lib().picp_vo_run_async(vo._h)
    B.solve_async(max_rounds=50, conv_eps=1e-5)
    B.sync()
    picp_amd.lib().picp_vo_sync(vo._h)
    marks.append("=" if np.array_equal(B.poses().view(np.uint32), ref.view(np.uint32)) else "X")
print("skip=%s batch beside VO: %s" % (os.environ.get("PICP_VO_DIAG_SKIP", "0"), " ".join(marks)), flush=True)
