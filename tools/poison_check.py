"""Stale-state probe for the VO determinism question.  Before each run
every CU's LDS and a full VGPR file are filled with a fixed pattern (tools/poison.hip), then the
same block-mode batch (the kernel that moves beside a co-running VO append) and the same serial VO
sequence run ALONE.  If a kernel reads LDS or registers it never wrote, its output follows the
pattern; if every pattern gives bit-identical output, stale on-chip state is ruled out."""
import ctypes
import os
import sys

import numpy as np
import torch  # noqa: F401  (device init through the library; torch only for parity with the other tools)

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "02-visualodometry_amd"))
import picp_amd  # noqa: E402
from picp_amd import synth  # noqa: E402
from picp_amd.vo_synth import VOSequence, segments  # noqa: E402

P = ctypes.CDLL(os.path.join(HERE, "_build", "libpoison.so"))
P.poison_fill.argtypes = [ctypes.c_uint, ctypes.c_int]
PATTERNS = [0x00000000, 0xFFFFFFFF, 0x7FC00001, 0x3F800000, 0x80000000, 0x00000000, 0x7F800000, 0x4B000000]


def same(a, b):
    return all(np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32)) for x, y in zip(a, b))


def probe(name, run):
    outs = []
    for pat in PATTERNS:
        rc = P.poison_fill(pat, 256 * 4)
        assert rc == 0, rc
        outs.append(run())
    marks = ["=" if same(outs[0], o) else "X" for o in outs]
    diffs = [max(float(np.abs(np.asarray(x, np.float64) - np.asarray(y, np.float64)).max()) for x, y in zip(outs[0], o))
             for o in outs]
    print("%-30s %s  max|d| %s" % (name, " ".join(marks), ["%.2g" % d for d in diffs]), flush=True)


for mode, F, n in (("block", 250, 1500), ("block", 128, 10000)):
    os.environ["PICP_MODE"] = mode
    bt = synth.make_batch(F, n, base_seed=1000)
    B = picp_amd.Batch(np.full(F, n))
    B.set_data(bt["xyz"], bt["uv"])

    def run_batch(B=B, bt=bt):
        B.set_poses(bt["T_init"])
        B.solve(max_rounds=50, conv_eps=1e-5)
        return [B.poses().copy()]

    probe("%s %d x %d (mode %s)" % (mode, F, n, B.info()["mode"]), run_batch)

os.environ.update({"PICP_VO_CHAINS": "1", "PICP_VO_OVERLAP": "0", "PICP_VO_PRIO": "0"})
F = 1201
D = VOSequence(F, obs_per_frame=1200, seed=5).frames(0, F)
first, steps = segments(F, 40)
boot = np.stack([[D["T_cw"][f], D["T_cw"][f + 1]] for f in first])
vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], K=VOSequence(2, obs_per_frame=10).K)
vo.set_segments(first, steps, boot)


def run_vo():
    vo.run()
    return [np.asarray(x).copy() for x in vo.poses()]


probe("VO serial (30 segments)", run_vo)
print("done", flush=True)
