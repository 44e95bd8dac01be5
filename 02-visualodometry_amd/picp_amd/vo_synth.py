"""Seeded synthetic VO sequence for C5 (a 10k-frame planar trajectory,
~2,000 observations per frame), mirroring the reference simulator that produced data/.

Robot: planar poses 0.2 m apart along a heading with a slow yaw (theta_k = yaw_amp *
sin(2 pi k / yaw_period)), camera = robot * data/camera.dat mount, K and 640x480 from
src/cam.cpp:11-31.  Landmarks are spawned per trajectory step in the band the robot sweeps
(longitudinal U[0, step), lateral U[-half_width, half_width], height U[-half_height,
half_height]) with 10-d descriptors U[-1, 1] like data/world.dat.  A frame observes every
landmark with depth in (z_near, z_far] whose float32 projection falls inside
[0, cols-1] x [0, rows-1] (the reference's bounds, src/camera.h:31-34); the observation carries
the landmark's descriptor exactly (data/ is noise-free) and, optionally, pixel noise.  Each
frame's observations are a seeded shuffle; id_meas = index in the frame, id_real = landmark id.

Every spawn step and every frame draws from its own seeded generator, so any frame range is
generated independently (multi-GPU ranks generate only their own segments).
"""
import numpy as np

from .synth import K_REF, MOUNT, ROWS, COLS, planar, rigid_inverse

STEP = 0.2
DIM = 10


class VOSequence:
    """A deterministic synthetic sequence; frames are generated on demand."""

    def __init__(self, n_frames, obs_per_frame=2000, seed=42, pixel_noise=0.0, half_width=8.0,
                 half_height=1.5, z_near=0.5, z_far=5.0, yaw_amp=0.3, yaw_period=400.0):
        self.n_frames = int(n_frames)
        self.seed = int(seed)
        self.pixel_noise = float(pixel_noise)
        self.hw, self.hh, self.z_near, self.z_far = half_width, half_height, z_near, z_far
        self.K = K_REF.astype(np.float32)
        self.rows, self.cols = ROWS, COLS
        # poses of steps -4 .. n_frames + 40 (landmarks are spawned ahead of the camera)
        self._k0 = -4
        ks = np.arange(self._k0, self.n_frames + 40)
        th = yaw_amp * np.sin(2 * np.pi * ks / yaw_period)
        dx, dy = STEP * np.cos(th), STEP * np.sin(th)
        x = np.concatenate([[0.0], np.cumsum(dx)[:-1]])
        y = np.concatenate([[0.0], np.cumsum(dy)[:-1]])
        i0 = -self._k0
        self._robot = np.stack([x - x[i0], y - y[i0], th], 1)  # frame 0 at the origin
        # landmark density from the expected frustum volume: obs ~= density * V_visible
        self.per_step = max(1, int(round(obs_per_frame / self._visible_steps_fraction())))

    # ------------------------------------------------------------------ geometry
    def robot_pose(self, k):
        return self._robot[np.asarray(k) - self._k0]

    def T_cw(self, k):
        """Camera-in-world pose of frame k (float64 4x4); the world-in-camera is its inverse."""
        x, y, th = self.robot_pose(k)
        return planar(x, y, th) @ MOUNT

    def _visible_steps_fraction(self):
        """Monte-Carlo estimate of how many landmarks of one spawn step a frame sees, summed
        over the spawn steps around it (so per_step = obs_per_frame / this)."""
        rng = np.random.default_rng(12345)
        n = 20000
        s = rng.uniform(0, STEP, n)
        lat = rng.uniform(-self.hw, self.hw, n)
        h = rng.uniform(-self.hh, self.hh, n)
        tot = 0.0
        T = np.linalg.inv(planar(0, 0, 0) @ MOUNT)
        for d in range(-4, 40):  # spawn step offset relative to the frame (straight line)
            pw = np.stack([d * STEP + s, lat, h], 0)
            pc = T[:3, :3] @ pw + T[:3, 3:4]
            ok, _ = self._project(pc)
            tot += ok.mean()
        return tot

    def _project(self, pc):
        z = pc[2]
        with np.errstate(divide="ignore", invalid="ignore"):
            u = (self.K[0, 0] * pc[0] + self.K[0, 2] * z) / z
            v = (self.K[1, 1] * pc[1] + self.K[1, 2] * z) / z
        uv = np.stack([u, v], 1).astype(np.float32)
        ok = (z > self.z_near) & (z <= self.z_far) & (uv[:, 0] >= 0) & (uv[:, 0] <= self.cols - 1) \
            & (uv[:, 1] >= 0) & (uv[:, 1] <= self.rows - 1)
        return ok, uv

    # ------------------------------------------------------------------ landmarks
    def landmarks(self, k):
        """Landmarks spawned at trajectory step k: (ids int64, xyz float64 (n,3), desc f32)."""
        rng = np.random.default_rng([self.seed, 1, k - self._k0])
        n = self.per_step
        s = rng.uniform(0, STEP, n)
        lat = rng.uniform(-self.hw, self.hw, n)
        h = rng.uniform(-self.hh, self.hh, n)
        x, y, th = self.robot_pose(k)
        c, sn = np.cos(th), np.sin(th)
        xyz = np.stack([x + s * c - lat * sn, y + s * sn + lat * c, h], 1)
        desc = rng.uniform(-1.0, 1.0, (n, DIM)).astype(np.float32)
        ids = (k - self._k0) * n + np.arange(n, dtype=np.int64)
        return ids, xyz, desc

    def frame(self, k, cache=None):
        """Observations of frame k: dict(uv f32 (m,2), desc f32 (m,10), id_real i64, id_meas i32).
        cache: optional dict step -> landmarks(step), shared by consecutive frames (each frame
        sees 33 spawn steps, so a range of frames reuses them; the values are the same)."""
        js = range(max(k - 3, self._k0), k + 30)
        if cache is None:
            parts = [self.landmarks(j) for j in js]
        else:
            for j in [j for j in cache if j < js[0]]:
                del cache[j]
            parts = []
            for j in js:
                if j not in cache:
                    cache[j] = self.landmarks(j)
                parts.append(cache[j])
        ids = np.concatenate([p[0] for p in parts])
        xyz = np.concatenate([p[1] for p in parts])
        desc = np.concatenate([p[2] for p in parts])
        T = rigid_inverse(self.T_cw(k))
        pc = T[:3, :3] @ xyz.T + T[:3, 3:4]
        ok, uv = self._project(pc)
        ids, uv, desc = ids[ok], uv[ok], desc[ok]
        rng = np.random.default_rng([self.seed, 2, k])
        perm = rng.permutation(len(ids))
        ids, uv, desc = ids[perm], uv[perm], desc[perm]
        if self.pixel_noise > 0:
            uv = (uv + rng.normal(0.0, self.pixel_noise, uv.shape)).astype(np.float32)
        return {"uv": np.ascontiguousarray(uv, np.float32), "desc": np.ascontiguousarray(desc),
                "id_real": ids, "id_meas": np.arange(len(ids), dtype=np.int32)}

    def frames(self, k0, k1):
        """Frames [k0, k1) packed: dict(frame_off int64 (n+1), uv, desc, id_real, T_cw (n,4,4) f32)."""
        cache = {}
        fs = [self.frame(k, cache) for k in range(k0, k1)]
        off = np.zeros(len(fs) + 1, np.int64)
        off[1:] = np.cumsum([len(f["uv"]) for f in fs])
        return {"frame_off": off,
                "uv": np.ascontiguousarray(np.concatenate([f["uv"] for f in fs])),
                "desc": np.ascontiguousarray(np.concatenate([f["desc"] for f in fs])),
                "id_real": np.concatenate([f["id_real"] for f in fs]),
                "T_cw": np.stack([self.T_cw(k) for k in range(k0, k1)]).astype(np.float32)}


def segments(n_frames, seg_len):
    """Contiguous segments with a one-frame overlap: segment s starts at frame s*seg_len and
    runs seg_len PICP steps (the last one may be shorter).  -> (first frame, steps) arrays."""
    first = np.arange(0, max(n_frames - 1, 0), seg_len, dtype=np.int64)
    steps = np.minimum(seg_len, (n_frames - 1) - first).astype(np.int32)
    return first, steps
