"""Seeded synthetic PICP problems, mirroring the reference simulator.

Camera: K = [180 0 320; 0 180 240; 0 0 1], 640x480 (src/cam.cpp:11-31), mounted on a planar
robot (x, y, theta) with the data/camera.dat mount (R = [[0,0,1],[-1,0,0],[0,-1,0]],
t = (0.2, 0, 0)).  Each correspondence: pixel (u, v) ~ U([0,639] x [0,479]), depth
z ~ U(0.6, 5.0) (data/ range 0.62-5.0, z_far = 5), back-projected to the camera and mapped
to the world with the ground-truth pose (float64, then stored as float32).  The initial
pose is gt perturbed by a left increment (translation N(0, 0.05 m), rotation N(0, 0.02 rad)
per axis).  Optional pixel noise and a fraction of outliers (image point replaced by a
uniform pixel).  Correspondences are a seeded shuffle, so the world-index gather of the
IntPairVector path is non-trivial.
"""
import numpy as np

K_REF = np.array([[180, 0, 320], [0, 180, 240], [0, 0, 1]], np.float64)
ROWS, COLS = 480, 640
MOUNT = np.array([[0, 0, 1, 0.2], [-1, 0, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1]], np.float64)


def planar(x, y, th):
    T = np.eye(4)
    c, s = np.cos(th), np.sin(th)
    T[:2, :2] = [[c, -s], [s, c]]
    T[0, 3], T[1, 3] = x, y
    return T


def rigid_inverse(T):
    Ti = np.eye(4, dtype=T.dtype)
    Ti[:3, :3] = T[:3, :3].T
    Ti[:3, 3] = -T[:3, :3].T @ T[:3, 3]
    return Ti


def euler_xyz(rx, ry, rz):
    """Rx*Ry*Rz (src/defs.h:100-136)."""
    cx, sx, cy, sy, cz, sz = np.cos(rx), np.sin(rx), np.cos(ry), np.sin(ry), np.cos(rz), np.sin(rz)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rx @ Ry @ Rz


def world_in_camera(robot_pose):
    """T_wc = (T_world_robot * T_robot_cam)^-1 for a planar robot pose (x, y, theta)."""
    return rigid_inverse(planar(*robot_pose) @ MOUNT)


def make_problem(n, seed=42, outlier_frac=0.0, pixel_noise=0.0, init_trans=0.05,
                 init_rot=0.02, robot_pose=None, shuffle=True):
    """One frame.  Returns dict with float32 world (n,3), image (n,2), int32 pairs (n,2)
    = (image idx, world idx), SoA arrays in pair order, T_gt / T_init (4x4 float32,
    world-in-camera) and the outlier mask (in pair order)."""
    rng = np.random.default_rng(seed)
    if robot_pose is None:
        robot_pose = (rng.uniform(-5, 5), rng.uniform(-5, 5), rng.uniform(-np.pi, np.pi))
    T_wc = world_in_camera(robot_pose)
    T_cw = rigid_inverse(T_wc)
    u = rng.uniform(0.0, COLS - 1, n)
    v = rng.uniform(0.0, ROWS - 1, n)
    z = rng.uniform(0.6, 5.0, n)
    Kinv = np.linalg.inv(K_REF)
    pc = (Kinv @ np.stack([u, v, np.ones(n)])) * z            # 3 x n camera points
    pw = (T_cw[:3, :3] @ pc + T_cw[:3, 3:4]).T                 # n x 3 world points
    uv = np.stack([u, v], 1)
    if pixel_noise > 0:
        uv = uv + rng.normal(0.0, pixel_noise, uv.shape)
    outl = np.zeros(n, bool)
    if outlier_frac > 0:
        k = int(round(outlier_frac * n))
        idx = rng.choice(n, k, replace=False)
        outl[idx] = True
        uv[idx] = np.stack([rng.uniform(0, COLS - 1, k), rng.uniform(0, ROWS - 1, k)], 1)
    # perturbed initial guess: T_init = D * T_gt
    D = np.eye(4)
    D[:3, :3] = euler_xyz(*rng.normal(0.0, init_rot, 3))
    D[:3, 3] = rng.normal(0.0, init_trans, 3)
    T_init = D @ T_wc
    # storage order: world and image arrays are independently permuted
    if shuffle:
        wperm = rng.permutation(n)   # world slot -> point
        iperm = rng.permutation(n)   # image slot -> point
    else:
        wperm = np.arange(n)
        iperm = np.arange(n)
    world = pw[wperm].astype(np.float32)
    image = uv[iperm].astype(np.float32)
    winv = np.empty(n, np.int64)
    winv[wperm] = np.arange(n)
    iinv = np.empty(n, np.int64)
    iinv[iperm] = np.arange(n)
    order = rng.permutation(n) if shuffle else np.arange(n)   # correspondence order
    pairs = np.stack([iinv[order], winv[order]], 1).astype(np.int32)
    xyz = world[pairs[:, 1]]
    uvp = image[pairs[:, 0]]
    return {
        "world": world, "image": image, "pairs": pairs,
        "x": np.ascontiguousarray(xyz[:, 0]), "y": np.ascontiguousarray(xyz[:, 1]),
        "z": np.ascontiguousarray(xyz[:, 2]), "u": np.ascontiguousarray(uvp[:, 0]),
        "v": np.ascontiguousarray(uvp[:, 1]), "xyz": np.ascontiguousarray(xyz),
        "uv": np.ascontiguousarray(uvp), "outlier": outl[order],
        "T_gt": T_wc.astype(np.float32), "T_init": T_init.astype(np.float32),
        "robot_pose": np.array(robot_pose, np.float64), "K": K_REF.astype(np.float32),
        "rows": ROWS, "cols": COLS,
    }


def make_batch(n_problems, n_corr, base_seed=1000, first=0, **kw):
    """C4: independent frames, problem i seeded with base_seed + (first + i).  Returns
    concatenated xyz (N,3), uv (N,2), per-problem sizes and T_gt/T_init stacks."""
    xyz, uv, Tg, Ti = [], [], [], []
    sizes = np.full(n_problems, n_corr, np.int64) if np.isscalar(n_corr) else np.asarray(n_corr)
    for i in range(n_problems):
        p = make_problem(int(sizes[i]), seed=base_seed + first + i, shuffle=False, **kw)
        xyz.append(p["xyz"])
        uv.append(p["uv"])
        Tg.append(p["T_gt"])
        Ti.append(p["T_init"])
    return {"xyz": np.concatenate(xyz) if xyz else np.zeros((0, 3), np.float32),
            "uv": np.concatenate(uv) if uv else np.zeros((0, 2), np.float32),
            "sizes": sizes, "T_gt": np.stack(Tg), "T_init": np.stack(Ti)}


def se3_log_norm(A, B):
    """||log(A^-1 B)|| (rotation angle and translation combined), float64.
    A^-1 is the full inverse, not R^T: a float32 pose chained over a long VO segment is not exactly
    orthonormal (|R^T R - I| ~5e-5 after 1,250 steps, as the reference's Isometry3f chain), and R^T
    would read that departure as pose error (~7e-5 at a 20 m translation)."""
    A = np.asarray(A, np.float64)
    B = np.asarray(B, np.float64)
    D = np.linalg.solve(A, B)
    R = D[:3, :3]
    w = 0.5 * np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    ang = np.arctan2(np.linalg.norm(w), (np.trace(R) - 1.0) / 2.0)  # well conditioned at 0
    return float(np.sqrt(ang ** 2 + np.sum(D[:3, 3] ** 2)))
