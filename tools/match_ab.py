#!/usr/bin/env python3
"""A/B timing of the matcher forms on one synthetic batch (GPU; profile with rocprofv3
--kernel-trace to read the per-launch kernel times):
  python tools/match_ab.py P NQ NR [ENV=v,ENV=v;ENV=v ...]
Each ';'-separated variant sets its env vars before two timed match_points_batch calls."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "02-visualodometry_amd"))
import numpy as np  # noqa: E402

import picp_amd  # noqa: E402

rng = np.random.default_rng(0)
P, nq, nr = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
variants = (sys.argv[4] if len(sys.argv) > 4 else "PICP_MATCH_ACCEPT_ONLY=0;PICP_MATCH_ACCEPT_ONLY=1").split(";")
d2s = [rng.uniform(-1, 1, (nr, 10)).astype(np.float32) for _ in range(P)]
# MATCH_DUP=f: the last f*nr references re-use earlier rows (+1e-3 noise), as duplicated map
# landmarks do in the VO sequence (C5: ~2.2 candidates per query)
dup = float(os.environ.get("MATCH_DUP", "0"))
if dup > 0:
    k = int(dup * nr)
    for d2 in d2s:
        d2[nr - k:] = d2[:k] + rng.normal(0, 1e-3, (k, 10)).astype(np.float32)
d1s = []
for d2 in d2s:
    d1 = rng.uniform(-1, 1, (nq, 10)).astype(np.float32)
    d1[: nq // 2] = d2[rng.choice(nr, nq // 2, replace=False)]
    d1s.append(d1)
for rep in range(2):
    for v in variants:
        for kv in v.split(","):
            k, val = kv.split("=")
            os.environ[k] = val
        # PICP_MATCH_ACCEPT_ONLY / PICP_MATCH_EXACT name the explicit form argument
        form = "exact" if os.environ.get("PICP_MATCH_EXACT") == "1" else (
            "accept_only" if os.environ.get("PICP_MATCH_ACCEPT_ONLY") == "1" else "full")
        picp_amd.match_points_batch(d1s, d2s, form=form)
        t = time.perf_counter()
        out = picp_amd.match_points_batch(d1s, d2s, form=form)
        print(v, "%.2f ms (incl. copies)" % (1e3 * (time.perf_counter() - t)), sum(int(o["accepted"].sum()) for o in out))
        for kv in v.split(","):
            os.environ.pop(kv.split("=")[0], None)
