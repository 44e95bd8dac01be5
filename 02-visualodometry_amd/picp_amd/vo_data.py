"""Reader for tests/golden/vo_data.npz, the re-encoded reference dataset (data/).

Frame k's ground-truth world-in-camera pose is (T_world_robot(gt_pose_k) * mount)^-1 with the
data/camera.dat mount; correspondences between a frame's measurements and world.dat are taken
by the simulator's ground-truth association id_real (the reference matches descriptors,
src/my_utilities.h:70-120; with the noise-free data both give the same pairs whenever the
descriptor match is correct).
"""
import os

import numpy as np

from .synth import MOUNT, planar, rigid_inverse

DEFAULT_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "tests", "golden", "vo_data.npz")


class VOData:
    def __init__(self, path=DEFAULT_PATH):
        d = np.load(path)  # plain arrays, no pickle
        self.world_id = d["world_id"]
        self.world_xyz = d["world_xyz"]
        self.world_desc = d["world_desc"]
        self.gt_pose = d["gt_pose"]
        self.odom_pose = d["odom_pose"]
        self.meas_frame = d["meas_frame"]
        self.meas_id = d["meas_id"]
        self.meas_real = d["meas_real"]
        self.meas_uv = d["meas_uv"]
        self.meas_desc = d["meas_desc"]
        self.K = d["K"]
        self.rows = int(d["rows"])
        self.ref_errors = d["ref_errors"] if "ref_errors" in d else None
        self.ref_map_ids = d["ref_map_ids"] if "ref_map_ids" in d else None
        self.ref_trajectory = d["ref_trajectory"] if "ref_trajectory" in d else None
        self.cols = int(d["cols"])
        self.n_frames = self.gt_pose.shape[0]
        self._id2row = {int(i): r for r, i in enumerate(self.world_id)}

    def write_reference_format(self, out_dir):
        """Re-emit data/meas-NNNNN.dat and data/world.dat in the reference's text format
        (parsed by src/my_utilities.cpp:35-182) for the C++ drop-in driver."""
        os.makedirs(out_dir, exist_ok=True)
        for k in range(self.n_frames):
            f = self.frame(k)
            with open(os.path.join(out_dir, "meas-%05d.dat" % k), "w") as fh:
                fh.write("seq: %d\n" % k)
                fh.write("gt_pose: %r %r %r\n" % tuple(float(x) for x in self.gt_pose[k]))
                fh.write("odom_pose: %r %r %r\n" % tuple(float(x) for x in self.odom_pose[k]))
                for i in range(len(f["uv"])):
                    fh.write("point %d %d %r %r %s\n" % (
                        int(f["id_meas"][i]), int(f["id_real"][i]), float(f["uv"][i][0]), float(f["uv"][i][1]),
                        " ".join(repr(float(x)) for x in f["desc"][i])))
        with open(os.path.join(out_dir, "world.dat"), "w") as fh:
            for r in range(len(self.world_id)):
                fh.write("%d %s %s\n" % (int(self.world_id[r]), " ".join(repr(float(x)) for x in self.world_xyz[r]),
                                         " ".join(repr(float(x)) for x in self.world_desc[r])))
        return out_dir

    def frame(self, k):
        sel = self.meas_frame == k
        return {"uv": self.meas_uv[sel], "id_meas": self.meas_id[sel],
                "id_real": self.meas_real[sel], "desc": self.meas_desc[sel]}

    def T_wc(self, k, pose=None):
        p = self.gt_pose[k] if pose is None else pose
        return rigid_inverse(planar(float(p[0]), float(p[1]), float(p[2])) @ MOUNT).astype(np.float32)

    def correspondences(self, k):
        """(image idx, world idx) pairs of frame k by id_real."""
        f = self.frame(k)
        pairs = [(i, self._id2row[int(r)]) for i, r in enumerate(f["id_real"]) if int(r) in self._id2row]
        return np.array(pairs, np.int32).reshape(-1, 2)

    def packed(self):
        """The 121 frames packed for the VO sequence APIs: (frame_off int64, uv, desc)."""
        order = np.lexsort((self.meas_id, self.meas_frame))
        off = np.zeros(self.n_frames + 1, np.int64)
        off[1:] = np.cumsum(np.bincount(self.meas_frame, minlength=self.n_frames))
        return off, np.ascontiguousarray(self.meas_uv[order]), np.ascontiguousarray(self.meas_desc[order])

    def trajectory_rows(self, poses):
        """The reference's output/estimated_trajectory.txt rows for camera-in-world poses
        (exec/icp_test.cpp:140-182): frame, x, y of cameraToImage * pose (src/cam.cpp:18-26)
        and the heading atan2(R10, R00) + pi/2."""
        c2i = np.zeros((4, 4))
        c2i[0, 2], c2i[1, 0], c2i[2, 1], c2i[3, 3] = 1.0, -1.0, -1.0, 1.0
        rows = []
        for k, T in enumerate(poses):
            P = c2i @ np.asarray(T, np.float64)
            rows.append((k, P[0, 3], P[1, 3], np.arctan2(P[1, 0], P[0, 0]) + np.pi / 2))
        return np.array(rows)

    def map_ids(self, map_desc):
        """id_real of map points by exact descriptor identity with world.dat (noise-free data)."""
        lut = {self.world_desc[r].tobytes(): int(self.world_id[r]) for r in range(len(self.world_id))}
        return np.array([lut.get(np.asarray(d, np.float32).tobytes(), -1) for d in map_desc], np.int64)
