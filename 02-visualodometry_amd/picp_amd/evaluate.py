"""Trajectory evaluation of a VO run (host-side plumbing, never on the timed path).

The reference evaluates its trajectory with `alignTrajectories` (src/my_utilities.cpp:459-478):
Eigen::umeyama(P, Q, true) over the camera translations -- a similarity transform (scale,
rotation, translation) that maps the estimated positions onto the ground truth -- and then writes
per-frame translation errors after applying that scale (exec/icp_test.cpp:145-196).  `umeyama`
below restates Umeyama's closed form (IEEE PAMI 13(4), 1991), which is the algorithm Eigen's
`umeyama` implements; `ate` reports the absolute trajectory error after the full similarity
alignment (RMSE and max of the position residuals) and the rotation error after it.

`stitch_segments` turns the per-segment trajectories of a segmented C5 run (every
segment estimated in its own first camera's frame, consecutive segments overlapping by one frame)
into one whole-sequence trajectory: segment k's frame is placed at the estimated pose of its first
frame as the previous segment saw it (its last step), so the stitched sequence is a chain of
estimates anchored only at frame 0.
"""
import numpy as np


def umeyama(src, dst, with_scale=True):
    """Similarity (c, R, t) minimising sum |dst_i - (c R src_i + t)|^2.  src, dst: (n, 3).
    Returns the 4x4 matrix [[c R, t], [0, 1]] (float64), as Eigen::umeyama does."""
    src = np.asarray(src, np.float64)
    dst = np.asarray(dst, np.float64)
    n = src.shape[0]
    mu_s, mu_d = src.mean(0), dst.mean(0)
    xs, xd = src - mu_s, dst - mu_d
    var_s = (xs * xs).sum() / n
    sigma = xd.T @ xs / n
    U, D, Vt = np.linalg.svd(sigma)
    S = np.ones(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        S[2] = -1.0
    R = U @ np.diag(S) @ Vt
    c = (D * S).sum() / var_s if (with_scale and var_s > 0) else 1.0
    T = np.eye(4)
    T[:3, :3] = c * R
    T[:3, 3] = mu_d - c * R @ mu_s
    return T


def _rot_angle(R):
    return float(np.arccos(np.clip((np.trace(R) - 1.0) / 2.0, -1.0, 1.0)))


def ate(est, gt):
    """est, gt: (n, 4, 4) camera-in-world poses of the same frames.  Absolute trajectory error
    after the similarity alignment of the positions (umeyama with scale, as the reference):
    RMSE / max of the position residuals (m), the alignment's scale, and the largest rotation
    error (rad) of the aligned orientations."""
    est = np.asarray(est, np.float64)
    gt = np.asarray(gt, np.float64)
    S = umeyama(est[:, :3, 3], gt[:, :3, 3], True)
    c = np.linalg.norm(S[:3, 0])
    Ra = S[:3, :3] / c
    p = (S[:3, :3] @ est[:, :3, 3].T).T + S[:3, 3]
    res = np.linalg.norm(p - gt[:, :3, 3], axis=1)
    rot = max(_rot_angle(gt[i, :3, :3].T @ Ra @ est[i, :3, :3]) for i in range(len(est)))
    path = float(np.linalg.norm(np.diff(gt[:, :3, 3], axis=0), axis=1).sum()) if len(gt) > 1 else 0.0
    return {"frames": int(len(est)), "ate_rmse_m": float(np.sqrt((res ** 2).mean())), "ate_max_m": float(res.max()),
            "ate_rmse_over_path": float(np.sqrt((res ** 2).mean()) / path) if path > 0 else None,
            "path_length_m": path, "sim3_scale": float(c), "rot_err_max_rad": rot}


def stitch_segments(poses, first, steps, anchor):
    """poses: list over segments of (steps+1, 4, 4) camera-in-world poses in each segment's frame
    (pose 0 = identity, the segment's first camera); consecutive segments overlap by one frame
    (first[k+1] = first[k] + steps[k]).  anchor: the world pose of frame first[0].
    -> (frames int64, (n, 4, 4) float64 stitched camera-in-world poses) for frames
    first[0] .. first[-1] + steps[-1]."""
    first = np.asarray(first, np.int64)
    steps = np.asarray(steps, np.int64)
    W = np.asarray(anchor, np.float64)
    out = [W.copy()]
    for k in range(len(first)):
        if k > 0 and first[k] != first[k - 1] + steps[k - 1]:
            raise ValueError("segments must overlap by exactly one frame")
        P = np.asarray(poses[k], np.float64)
        for t in range(1, int(steps[k]) + 1):
            out.append(W @ P[t])
        W = W @ P[int(steps[k])]
    frames = np.arange(first[0], first[-1] + steps[-1] + 1, dtype=np.int64)
    return frames, np.stack(out)
