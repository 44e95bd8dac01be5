#!/usr/bin/env python3
"""Diagnostic (GPU): what a descriptor-space bucketed world match would save, simulated with the
shipped matcher on host-built problems.  The 8e maps of segments 0-3 (tools/r06/match_8e.py
--save) are grouped by the sign of descriptor components 0..NB-1 (2^NB cells); a late frame's
queries are sorted by their 3-state code per component (below -m, within +-m, above +m with
m = 0.5 * 1.01: the radius sqrt(0.25) plus margin) and cut into groups of GQ consecutive queries;
each group is one problem against the cells its queries can reach (a reference in the other sign
cell of component k is at distance >= |q_k| > m from the query).  Results are mapped back to the
original indices and compared with the brute-force launch; the kernel trace gives the times.

  python tools/r06/match_bucket_sim.py MAPS.npz [NB] [GQ]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))


def main():
    import numpy as np
    import picp_amd
    z = np.load(sys.argv[1])
    NB = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    GQ = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    m = 0.5 * 1.01
    maps = [z["map%d" % s] for s in range(4)]
    qs = [z["q%d" % s] for s in range(4)]
    w = 1 << np.arange(NB)
    q_probs, r_probs, back = [], [], []
    pairs_bucket = 0
    for s in range(4):
        R, Q = maps[s], qs[s]
        rcell = ((R[:, :NB] >= 0) * w).sum(1)
        order_r = np.argsort(rcell, kind="stable")
        state = np.where(Q[:, :NB] < -m, 0, np.where(Q[:, :NB] > m, 2, 1))  # 0 neg only, 1 both, 2 pos only
        code = (state * (3 ** np.arange(NB))[::-1]).sum(1)
        order_q = np.argsort(code, kind="stable")
        for g0 in range(0, len(Q), GQ):
            qi = order_q[g0:g0 + GQ]
            need = np.zeros(1 << NB, bool)
            for st in state[qi]:
                ok = np.ones(1 << NB, bool)
                for k in range(NB):
                    bit = (np.arange(1 << NB) >> k) & 1
                    if st[k] == 0:
                        ok &= bit == 0
                    elif st[k] == 2:
                        ok &= bit == 1
                need |= ok
            ri = order_r[np.isin(rcell[order_r], np.nonzero(need)[0])]
            q_probs.append(Q[qi])
            r_probs.append(R[ri])
            back.append((s, qi, ri))
            pairs_bucket += len(qi) * len(ri)
    pairs_brute = sum(len(q) * len(r) for q, r in zip(qs, maps))
    print("NB %d GQ %d: %d problems, pairs %.3g vs brute force %.3g (%.3f)" % (
        NB, GQ, len(q_probs), pairs_bucket, pairs_brute, pairs_bucket / pairs_brute), flush=True)
    # brute force (reference), then the bucketed problems, 3 times each
    ref = picp_amd.match_points_batch(qs, maps, 0.2, 0.8, form="accept_only")
    for _ in range(3):
        picp_amd.match_points_batch(qs, maps, 0.2, 0.8, form="accept_only")
    for _ in range(3):
        out = picp_amd.match_points_batch(q_probs, r_probs, 0.2, 0.8, form="accept_only")
    acc = [np.zeros(len(q), bool) for q in qs]
    bi = [np.full(len(q), -1, np.int64) for q in qs]
    for (s, qi, ri), o in zip(back, out):
        acc[s][qi] = o["accepted"]
        bi[s][qi] = np.where(o["accepted"], ri[np.maximum(o["best_idx"], 0)], -1)
    bad = 0
    for s in range(4):
        a = ref[s]["accepted"]
        bad += int((a != acc[s]).sum()) + int((bi[s][a] != ref[s]["best_idx"][a]).sum())
    print("accepted %d, mismatches vs brute force %d" % (sum(int(r["accepted"].sum()) for r in ref), bad), flush=True)


if __name__ == "__main__":
    main()
