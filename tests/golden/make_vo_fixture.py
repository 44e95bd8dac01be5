"""Generate tests/golden/vo_data.npz from the reference's own dataset (data/).

The reference's data/ directory IS its fixture: a noise-free simulated
world (world.dat: id x y z d0..d9), 121 frames (meas-NNNNN.dat: seq, gt_pose, odom_pose,
`point id_meas id_real u v d0..d9`) and the camera (camera.dat).  This script only
re-encodes those numbers (parsed exactly as src/my_utilities.cpp:35-182 does: whitespace
tokens, std::stof -> float32) into one compact .npz so the tests can run on the GPU box,
where /root/reference does not exist.

Run (in the build container only):  python tests/golden/make_vo_fixture.py [REF_ROOT]
"""
import os
import sys

import numpy as np

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vo_data.npz")


def f32(tok):
    return np.float32(tok)  # numpy parses decimal text directly to binary32


def main():
    data = os.path.join(REF, "data")
    wid, wxyz, wdesc = [], [], []
    with open(os.path.join(data, "world.dat")) as fh:
        for line in fh:
            t = line.split()
            if len(t) < 14:
                continue
            wid.append(int(t[0]))
            wxyz.append([f32(x) for x in t[1:4]])
            wdesc.append([f32(x) for x in t[4:14]])
    n_frames = 121  # exec/icp_test.cpp:21
    gt, odom = np.zeros((n_frames, 3), np.float32), np.zeros((n_frames, 3), np.float32)
    mf, mid, mreal, muv, mdesc = [], [], [], [], []
    for k in range(n_frames):
        with open(os.path.join(data, "meas-%05d.dat" % k)) as fh:
            for line in fh:
                t = line.split()
                if not t:
                    continue
                if t[0] == "gt_pose:":
                    gt[k] = [f32(x) for x in t[1:4]]
                elif t[0] == "odom_pose:":
                    odom[k] = [f32(x) for x in t[1:4]]
                elif t[0] == "point" and len(t) >= 15:
                    mf.append(k)
                    mid.append(int(t[1]))
                    mreal.append(int(t[2]))
                    muv.append([f32(t[3]), f32(t[4])])
                    mdesc.append([f32(x) for x in t[5:15]])
    # camera.dat (K and the robot->camera mount); values also hard-coded in src/cam.cpp:11-31
    K = np.array([[180, 0, 320], [0, 180, 240], [0, 0, 1]], np.float32)
    mount = np.array([[0, 0, 1, 0.2], [-1, 0, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1]], np.float32)
    # the reference's published run (output/errors.txt: frame, translational err, yaw err) -- a
    # loose end-to-end band only (UB-tainted, OpenCV-RANSAC bootstrap)
    errs = np.loadtxt(os.path.join(REF, "output", "errors.txt"), dtype=np.float64)
    # the reference's final map (output/estimated_world_points.txt, exec/icp_test.cpp:199-211):
    # for every id_real 0..999 the first map point carrying it -> the id column is the set of
    # distinct landmarks the run triangulated (490, README:7).  Only the ids are kept: the
    # coordinates depend on the RANSAC bootstrap and the umeyama scale.
    wp = np.loadtxt(os.path.join(REF, "output", "estimated_world_points.txt"), dtype=np.float64)
    # the reference's estimated trajectory (output/estimated_trajectory.txt, exec/icp_test.cpp:
    # 181-182: frame, x, y, heading of cameraToImage * pose): its row 1 is the bootstrap of
    # computeEssentialAndRecoverPose (src/cam.cpp:37-91) after frame 1's PICP
    traj = np.loadtxt(os.path.join(REF, "output", "estimated_trajectory.txt"), dtype=np.float64)
    np.savez_compressed(
        OUT, ref_errors=errs.astype(np.float32), ref_map_ids=wp[:, 0].astype(np.int32),
        ref_trajectory=traj,
        world_id=np.array(wid, np.int32), world_xyz=np.array(wxyz, np.float32),
        world_desc=np.array(wdesc, np.float32),
        gt_pose=gt, odom_pose=odom,
        meas_frame=np.array(mf, np.int32), meas_id=np.array(mid, np.int32),
        meas_real=np.array(mreal, np.int32), meas_uv=np.array(muv, np.float32),
        meas_desc=np.array(mdesc, np.float32),
        K=K, cam_mount=mount, rows=np.int32(480), cols=np.int32(640))
    print("wrote", OUT, os.path.getsize(OUT), "bytes;", len(wid), "world pts,", len(mf), "meas")


if __name__ == "__main__":
    main()
