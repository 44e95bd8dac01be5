"""Per-problem pose error vs the F64 oracle of the ragged-batch problems, for the camera path this
process runs (PICP_FORCE_GENERAL_K=1 forces the general one).  Diagnostic."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "02-visualodometry_amd"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
import picp_amd  # noqa: E402
from picp_amd import synth  # noqa: E402

sizes = [1, 2, 3, 4, 6, 10, 30, 100, 1000, 5000, 20001]
for mode in ("graph", "block"):
    os.environ["PICP_MODE"] = mode
    probs = [synth.make_problem(n, seed=100 + i, outlier_frac=0.1, pixel_noise=0.5, shuffle=False)
             for i, n in enumerate(sizes)]
    b = picp_amd.Batch(sizes)
    b.set_data(np.concatenate([p["xyz"] for p in probs]), np.concatenate([p["uv"] for p in probs]))
    b.set_poses(np.stack([p["T_init"] for p in probs]))
    b.solve(threshold=3000.0, max_rounds=50, conv_eps=-1.0)
    P = b.poses()
    errs = []
    for i, (p, n) in enumerate(zip(probs, sizes)):
        T_ref, _ = oracle.solve_soa(p["T_init"], p["K"], 480, 640, p["x"], p["y"], p["z"], p["u"], p["v"], 3000.0,
                                    mode=oracle.MODE_F64, max_rounds=50, conv_eps=-1.0)
        T_f, _ = oracle.solve_soa(p["T_init"], p["K"], 480, 640, p["x"], p["y"], p["z"], p["u"], p["v"], 3000.0,
                                  mode=oracle.MODE_FAITHFUL, max_rounds=50, conv_eps=-1.0)
        errs.append("%d:%.1e(f/d %.1e)" % (n, synth.se3_log_norm(P[i], T_ref), synth.se3_log_norm(T_f, T_ref)))
    print(mode, "general" if os.environ.get("PICP_FORCE_GENERAL_K") else "pinhole", " ".join(errs))
