import os, sys, time
sys.path.insert(0, "/root/repo/02-visualodometry_amd")
import numpy as np
import picp_amd
rng = np.random.default_rng(0)
P, nq, nr = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
d2s = [rng.uniform(-1, 1, (nr, 10)).astype(np.float32) for _ in range(P)]
d1s = []
for d2 in d2s:
    d1 = rng.uniform(-1, 1, (nq, 10)).astype(np.float32)
    d1[: nq // 2] = d2[rng.choice(nr, nq // 2, replace=False)]
    d1s.append(d1)
for mode in ("0", "1", "0", "1"):
    os.environ["PICP_MATCH_ACCEPT_ONLY"] = mode
    picp_amd.match_points_batch(d1s, d2s)
    t = time.perf_counter()
    out = picp_amd.match_points_batch(d1s, d2s)
    print(mode, "%.2f ms" % (1e3 * (time.perf_counter() - t)), sum(int(o["accepted"].sum()) for o in out))
