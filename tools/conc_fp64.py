"""Is a block-mode batch perturbed by unrelated FP64 vector work running beside it (torch
elementwise float64 on its own stream), versus the same work in float32?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "02-visualodometry_amd"))
import picp_amd  # noqa: E402
from picp_amd import synth  # noqa: E402

os.environ["PICP_MODE"] = "block"
bt = synth.make_batch(250, 1500, base_seed=1000)
B = picp_amd.Batch(np.full(250, 1500))
B.set_data(bt["xyz"], bt["uv"])


def run_batch():
    B.set_poses(bt["T_init"])
    B.solve(max_rounds=50, conv_eps=1e-5)
    return B.poses()


ref = run_batch()
s = torch.cuda.Stream()
for dt in (torch.float32, torch.float64, torch.float32, torch.float64):
    x = torch.rand(1 << 22, device="cuda", dtype=dt)
    torch.cuda.synchronize()
    marks = []
    for r in range(8):
        with torch.cuda.stream(s):
            for _ in range(200):  # FMA-chain elementwise work, a few ms
                x = torch.addcmul(x, x, x, value=1e-7).sqrt_().mul_(1.0000001)
        B.set_poses(bt["T_init"])
        B.solve_async(max_rounds=50, conv_eps=1e-5)
        B.sync()
        torch.cuda.synchronize()
        marks.append("=" if np.array_equal(B.poses().view(np.uint32), ref.view(np.uint32)) else "X")
    print("batch beside torch %s elementwise: %s" % (dt, " ".join(marks)), flush=True)
