"""Do kernel results depend on what else runs on the GPU?  The same PICP batch (block kernel) and
the same VO sequence (serial one-stream schedule) are run alone and while a torch stream keeps the
CUs busy with matmuls; every run must be bit-identical to the first lone run."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "02-visualodometry_amd"))
import picp_amd  # noqa: E402
from picp_amd import synth  # noqa: E402
from picp_amd.vo_synth import VOSequence, segments  # noqa: E402

dev = torch.device("cuda:0")
a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
b = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)


def load(n):  # n async matmuls on torch's stream (~0.1 ms each)
    for _ in range(n):
        torch.mm(a, b)


def check(name, run, reps=4, load_n=60):
    ref = run()
    res = []
    for r in range(reps):
        res.append(("alone", run()))
        load(load_n)
        res.append(("loaded", run()))
        torch.cuda.synchronize()
    out = []
    for tag, x in res:
        same = all(np.array_equal(np.asarray(u).view(np.uint32), np.asarray(v).view(np.uint32)) for u, v in zip(ref, x))
        out.append(tag[0] + ("=" if same else "X"))
    print("%-28s %s" % (name, " ".join(out)), flush=True)


os.environ["PICP_MODE"] = "block"
bt = synth.make_batch(250, 1500, base_seed=1000)
B = picp_amd.Batch(np.full(250, 1500))
B.set_data(bt["xyz"], bt["uv"])


def run_batch():
    B.set_poses(bt["T_init"])
    B.solve(max_rounds=50, conv_eps=1e-5)
    return [B.poses()]


check("block kernel (250 x 1500)", run_batch)

# the same kernel beside itself: a second batch (other data, its own stream) solving concurrently
bt2 = synth.make_batch(250, 1500, base_seed=5000)
B2 = picp_amd.Batch(np.full(250, 1500))
B2.set_data(bt2["xyz"], bt2["uv"])
ref = run_batch()
marks = []
for r in range(6):
    B2.set_poses(bt2["T_init"])
    B.set_poses(bt["T_init"])
    B2.solve_async(max_rounds=50, conv_eps=1e-5)
    B.solve_async(max_rounds=50, conv_eps=1e-5)
    B.sync()
    B2.sync()
    marks.append("=" if np.array_equal(B.poses().view(np.uint32), ref[0].view(np.uint32)) else "X")
print("%-28s %s" % ("block kernel beside itself", " ".join(marks)), flush=True)

os.environ.update({"PICP_VO_CHAINS": "1", "PICP_VO_OVERLAP": "0", "PICP_VO_PRIO": "0"})
F = 1201
D = VOSequence(F, obs_per_frame=1200, seed=5).frames(0, F)
first, steps = segments(F, 40)
boot = np.stack([[D["T_cw"][f], D["T_cw"][f + 1]] for f in first])
vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], K=VOSequence(2, obs_per_frame=10).K)
vo.set_segments(first, steps, boot)


def run_vo():
    vo.run()
    return vo.poses()


check("VO serial (30 segments)", run_vo)

# the VO kernels beside themselves: a second serial VO handle (other data) running concurrently
D2 = VOSequence(F, obs_per_frame=1200, seed=9).frames(0, F)
boot2 = np.stack([[D2["T_cw"][f], D2["T_cw"][f + 1]] for f in first])
vo2 = picp_amd.VOSequence(D2["frame_off"], D2["uv"], D2["desc"], K=VOSequence(2, obs_per_frame=10).K)
vo2.set_segments(first, steps, boot2)
ref = run_vo()
marks = []
for r in range(6):
    picp_amd.lib().picp_vo_run_async(vo2._h)
    picp_amd.lib().picp_vo_run_async(vo._h)
    picp_amd.lib().picp_vo_sync(vo._h)
    picp_amd.lib().picp_vo_sync(vo2._h)
    P = vo.poses()
    marks.append("=" if all(np.array_equal(x.view(np.uint32), y.view(np.uint32)) for x, y in zip(P, ref)) else "X")
print("%-28s %s" % ("VO serial beside itself", " ".join(marks)), flush=True)

# which outputs differ when the VO runs beside another VO: the match outputs (per observation) or
# only the poses?
import ctypes  # noqa: E402


def matches(v):
    n = int(D["frame_off"][-1])
    out = []
    for w in range(4):
        a = np.zeros(n, np.int32)
        picp_amd.lib().picp_vo_debug_matches(v._h, w, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        out.append(a)
    out[0] = np.where(out[1] != 0, out[0], -1)
    out[2] = np.where(out[3] != 0, out[2], -1)
    return out


vo.run()
ref_p, ref_m = vo.poses(), matches(vo)
for r in range(6):
    picp_amd.lib().picp_vo_run_async(vo2._h)
    picp_amd.lib().picp_vo_run_async(vo._h)
    picp_amd.lib().picp_vo_sync(vo._h)
    picp_amd.lib().picp_vo_sync(vo2._h)
    P, M = vo.poses(), matches(vo)
    dp = sum(int(not np.array_equal(x.view(np.uint32), y.view(np.uint32))) for x, y in zip(P, ref_p))
    dm = [int((a != b).sum()) for a, b in zip(M, ref_m)]
    first = [int(np.nonzero(a != b)[0][0]) if (a != b).any() else None for a, b in zip(M, ref_m)]
    print("beside: segments with pose diffs %d; match diffs pm_bi %d pm_acc %d wm_bi %d wm_acc %d; first obs %s"
          % (dp, *dm, first), flush=True)

# cross pairs: the batch (block kernel only) beside the VO, and the VO beside the batch
ref_b = run_batch()[0]
ref_v = run_vo()
mb, mv = [], []
for r in range(6):
    B.set_poses(bt["T_init"])
    picp_amd.lib().picp_vo_run_async(vo2._h)
    B.solve_async(max_rounds=50, conv_eps=1e-5)
    B.sync()
    picp_amd.lib().picp_vo_sync(vo2._h)
    mb.append("=" if np.array_equal(B.poses().view(np.uint32), ref_b.view(np.uint32)) else "X")
    B2.set_poses(bt2["T_init"])
    B2.solve_async(max_rounds=50, conv_eps=1e-5)
    picp_amd.lib().picp_vo_run_async(vo._h)
    picp_amd.lib().picp_vo_sync(vo._h)
    B2.sync()
    P = vo.poses()
    mv.append("=" if all(np.array_equal(x.view(np.uint32), y.view(np.uint32)) for x, y in zip(P, ref_v)) else "X")
print("%-28s %s" % ("batch beside VO", " ".join(mb)), flush=True)
print("batch residency after the VO pairs:", B.residency() if hasattr(B, "residency") else None, "info", B.info(), flush=True)
print("%-28s %s" % ("VO beside batch", " ".join(mv)), flush=True)

# the batch beside the matcher alone (a thread looping the batched matcher; ctypes drops the GIL)
import threading  # noqa: E402

Dm = VOSequence(400, obs_per_frame=2000, seed=3).frames(0, 400)
o = Dm["frame_off"]
m1 = [Dm["desc"][o[f]:o[f + 1]] for f in range(399)]
m2 = [Dm["desc"][o[f + 1]:o[f + 2]] for f in range(399)]
stop = [False]


def matcher_loop():
    while not stop[0]:
        picp_amd.match_points_batch(m1, m2)


print("batch residency before:", B.residency() if hasattr(B, "residency") else None, "info", B.info(), flush=True)
th = threading.Thread(target=matcher_loop)
th.start()
mm = []
for r in range(8):
    run_batch()
    mm.append("=" if np.array_equal(B.poses().view(np.uint32), ref_b.view(np.uint32)) else "X")
stop[0] = True
th.join()
print("%-28s %s" % ("batch beside matcher", " ".join(mm)), flush=True)
print("batch residency after:", B.residency() if hasattr(B, "residency") else None, flush=True)
