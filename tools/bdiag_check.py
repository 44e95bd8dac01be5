"""Where does a block-kernel batch first diverge when a VO sequence runs beside it?

Diagnostic build only (make -C 02-visualodometry_amd bdiag -> lib/libpicp_amd_bdiag.so, loaded through
PICP_LIB).  The batch of concurrency_check.py (250 x 1500, block mode, split 1) records, per
(problem, round): the pose each of its 8 waves linearized at, the 8 wave sums of every term, the
converted totals, the finishing wave's new pose, a lane-agreement count of the finishing wave, and
per wave the number of lanes whose permlane/DPP reduction differs from the ds_bpermute form of the
same sums.  Solo runs are compared with each other and runs beside a VO sequence with the solo
one; for every differing problem the first differing round and section are printed.
usage: python tools/bdiag_check.py [reps_beside]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
os.environ.setdefault("PICP_LIB", os.path.join(ROOT, "02-visualodometry_amd", "lib", "libpicp_amd_bdiag.so"))
os.environ["PICP_MODE"] = "block"
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
import picp_amd  # noqa: E402
from picp_amd import synth  # noqa: E402
from picp_amd.vo_synth import VOSequence, segments  # noqa: E402

NP, NC, R, REC = 250, 1500, 50, 416
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
L = picp_amd.lib()
L.picp_debug_bdiag_set.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.c_int,
                                    ctypes.c_int]
hip = ctypes.CDLL("libamdhip64.so")
dptr = ctypes.c_void_p()
nbytes = NP * R * REC * 4
assert hip.hipMalloc(ctypes.byref(dptr), ctypes.c_size_t(nbytes)) == 0
assert L.picp_debug_bdiag_set(dptr, NP, R, 0, 0, 0) == 0

bt = synth.make_batch(NP, NC, base_seed=1000)
B = picp_amd.Batch(np.full(NP, NC))
B.set_data(bt["xyz"], bt["uv"])

F = 1201
D = VOSequence(F, obs_per_frame=1200, seed=9).frames(0, F)
first, steps = segments(F, 40)
boot = np.stack([[D["T_cw"][f], D["T_cw"][f + 1]] for f in first])
vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], K=VOSequence(2, obs_per_frame=10).K)
vo.set_segments(first, steps, boot)


def grab():
    h = np.empty(NP * R * REC, np.float32)
    assert hip.hipDeviceSynchronize() == 0
    assert hip.hipMemcpy(h.ctypes.data_as(ctypes.c_void_p), dptr, ctypes.c_size_t(nbytes), 2) == 0
    return h.reshape(NP, R, REC)


def run(beside):
    assert hip.hipMemset(dptr, 0, ctypes.c_size_t(nbytes)) == 0
    assert hip.hipDeviceSynchronize() == 0
    B.set_poses(bt["T_init"])
    if beside:
        L.picp_vo_run_async(vo._h)
    B.solve_async(max_rounds=R, conv_eps=1e-5)
    B.sync()
    if beside:
        L.picp_vo_sync(vo._h)
    return B.poses().copy(), grab()


SECT = [("wave_pose", 0, 96), ("wave_sums", 96, 352), ("totals", 352, 384), ("pose_out", 384, 396),
        ("stats", 396, 400)]


def flags(rec, tag):
    lm = rec[:, :, 404]
    rb = rec[:, :, 405:413]
    if lm.any() or rb.any():
        print("  %s: lane disagreement in finish at %d (problem, round) records; reduction mismatches at %d"
              % (tag, int((lm != 0).sum()), int((rb != 0).sum())), flush=True)
        for p, r in list(zip(*np.nonzero(rb.any(axis=2))))[:8]:
            print("    reduction mismatch problem %d round %d per wave %s" % (p, r + 1, rb[p, r].astype(int).tolist()))


def compare(tag, ref, cur):
    (P0, R0), (P1, R1) = ref, cur
    same = np.array_equal(P0.view(np.uint32), P1.view(np.uint32))
    flags(R1, tag)
    if same and np.array_equal(R0.view(np.uint32), R1.view(np.uint32)):
        print("%-10s identical" % tag, flush=True)
        return
    bad = [p for p in range(NP) if not np.array_equal(R0[p].view(np.uint32), R1[p].view(np.uint32))]
    print("%-10s poses %s, %d problems with differing records" % (tag, "same" if same else "DIFFER", len(bad)),
          flush=True)
    for p in bad[:12]:
        d = R0[p].view(np.uint32) != R1[p].view(np.uint32)
        r = int(np.nonzero(d.any(axis=1))[0][0])
        where = []
        for name, a, b in SECT:
            idx = np.nonzero(d[r, a:b])[0]
            if len(idx):
                if name == "wave_pose":
                    where.append("%s waves %s" % (name, sorted(set((idx // 12).tolist()))))
                elif name == "wave_sums":
                    where.append("%s (term, wave) %s" % (name, [(int(i // 8), int(i % 8)) for i in idx[:6]]))
                else:
                    where.append("%s idx %s" % (name, idx[:6].tolist()))
        print("  problem %3d first round %2d: %s" % (p, r + 1, "; ".join(where)), flush=True)
        if any(s.startswith("wave_sums") for s in where) and not any(s.startswith("wave_pose") for s in where):
            idx = np.nonzero(d[r, 96:352])[0][:3]
            for i in idx:
                print("    term %d wave %d: %r vs %r" % (i // 8, i % 8, float(R0[p, r, 96 + i]), float(R1[p, r, 96 + i])))


ref = run(False)
flags(ref[1], "solo0")
for k in range(3):
    compare("solo%d" % (k + 1), ref, run(False))
for k in range(reps):
    compare("beside%d" % k, ref, run(True))
