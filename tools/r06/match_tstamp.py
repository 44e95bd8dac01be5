#!/usr/bin/env python3
"""Diagnostic (GPU, -DMM_TSTAMP build lib/libpicp_amd_tstamp.so): where the folded matcher's tile
loop spends its cycles, per wave and tile: the fold vote + barrier, the next tile's fetch issue,
the compute (16 MFMA blocks at RB = 2), the fold check + stash.  Shapes: the 8e world match (4
problems against the saved maps, tools/r06/match_8e.py --save) and a default-C5-like launch (125
problems x 2,000 queries x 5,000 random references).

  PICP_LIB=.../libpicp_amd_tstamp.so python tools/r06/match_tstamp.py MAPS.npz
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))


def main():
    import numpy as np
    import picp_amd
    L = picp_amd.lib()
    L.picp_debug_match_tstamp.argtypes = [ctypes.c_void_p, ctypes.c_int]
    st = np.zeros(6, np.uint64)
    z = np.load(sys.argv[1])
    maps = [z["map%d" % s] for s in range(4)]
    qs = [z["q%d" % s] for s in range(4)]
    rng = np.random.default_rng(1)
    dq = [rng.uniform(-1, 1, (2000, 10)).astype(np.float32) for _ in range(125)]
    dr = [rng.uniform(-1, 1, (5000, 10)).astype(np.float32) for _ in range(125)]
    for name, a, b in (("8e world match (4 x ~2k x 180k)", qs, maps), ("default-like (125 x 2k x 5k)", dq, dr)):
        for _ in range(2):
            picp_amd.match_points_batch(a, b, 0.2, 0.8, form="accept_only")
        L.picp_debug_match_tstamp(st.ctypes.data, 1)
        picp_amd.match_points_batch(a, b, 0.2, 0.8, form="accept_only")
        L.picp_debug_match_tstamp(st.ctypes.data, 0)
        tiles = max(int(st[4]), 1)
        names = ("vote+barrier", "fetch issue", "compute", "check+stash")
        per = [int(st[k]) / tiles for k in range(4)]
        waves = tiles  # tiles counted per wave
        print("%s: wave-tiles %d, per wave-tile cycles: %s, sum %.0f; tile loop total %.3g wave-cycles" % (
            name, tiles, ", ".join("%s %.0f" % (n, v) for n, v in zip(names, per)), sum(per), float(st[5])), flush=True)


if __name__ == "__main__":
    main()
