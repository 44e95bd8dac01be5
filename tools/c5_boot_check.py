#!/usr/bin/env python3
"""The reference's two-view bootstrap (exec/icp_test.cpp:44-58: match_points of frames 0 and 1,
Cam::computeEssentialAndRecoverPose, src/cam.cpp:37-91) on every C5 segment's first frame pair,
on the GPU (picp_match_points_batch + picp_essential_batch), against the ground-truth relative
pose: rotation angle error and translation-direction error per segment, and the time of both
batched launches.  usage: python tools/c5_boot_check.py [FRAMES [SEG_LEN]]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "02-visualodometry_amd"))
import picp_amd  # noqa: E402
from picp_amd.vo_synth import VOSequence, segments  # noqa: E402


def boot_pairs(D, f0_list):
    d1 = [D["desc"][D["frame_off"][f]:D["frame_off"][f + 1]] for f in f0_list]
    d2 = [D["desc"][D["frame_off"][f + 1]:D["frame_off"][f + 2]] for f in f0_list]
    m = picp_amd.match_points_batch(d1, d2)
    p1s, p2s = [], []
    for k, f in enumerate(f0_list):
        acc = np.nonzero(m[k]["accepted"])[0]
        uv1 = D["uv"][D["frame_off"][f]:D["frame_off"][f + 1]]
        uv2 = D["uv"][D["frame_off"][f + 1]:D["frame_off"][f + 2]]
        p1s.append(uv1[acc])
        p2s.append(uv2[m[k]["best_idx"][acc]])
    return p1s, p2s


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    seq = VOSequence(F, obs_per_frame=2000, seed=42)
    D = seq.frames(0, F)
    first, _ = segments(F, L)
    for rep in range(2):
        t0 = time.perf_counter()
        p1s, p2s = boot_pairs(D, first)
        t1 = time.perf_counter()
        res = picp_amd.essential_recover_pose_batch(p1s, p2s, K=seq.K)
        t2 = time.perf_counter()
    rot, tdir, bad = [], [], 0
    for k, f in enumerate(first):
        gt = np.linalg.inv(D["T_cw"][f].astype(np.float64)) @ D["T_cw"][f + 1].astype(np.float64)
        T = res[k]["T"].astype(np.float64)
        if not res[k]["good"]:
            bad += 1
        dR = T[:3, :3].T @ gt[:3, :3]
        rot.append(np.degrees(np.arccos(np.clip((np.trace(dR) - 1) / 2, -1, 1))))
        a, b = T[:3, 3], gt[:3, 3]
        tdir.append(np.degrees(np.arccos(np.clip(a @ b / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-30), -1, 1))))
    rot, tdir = np.array(rot), np.array(tdir)
    print("segments %d  pairs/segment median %d  not good %d" % (len(first), int(np.median([len(p) for p in p1s])), bad))
    print("rotation error deg: median %.3g  max %.3g" % (np.median(rot), rot.max()))
    print("translation direction error deg: median %.3g  max %.3g  (> 5 deg: %d)" % (np.median(tdir), tdir.max(),
                                                                                        int((tdir > 5).sum())))
    print("time: matching %.2f ms, essential + recoverPose %.2f ms (host-timed, second repetition)" %
          (1e3 * (t1 - t0), 1e3 * (t2 - t1)))


if __name__ == "__main__":
    main()
