"""GPU parity tests: the HIP path (through the C-ABI) against the CPU oracle.

Tolerances (BASELINE.json north_star: poses within 1e-4 on SE(3) log):
  * pose after a solve      : se3_log_norm(gpu, oracle_f64) < 1e-4
  * inlier/outlier/skip gate: n_in and n_projected EXACT at the same pose (the gate is
                              evaluated with the oracle's exact float operation order)
  * H, b, chi               : relative 1e-5 of the largest entry (float32 per-thread partial
                              sums + double cross-block reduction vs the oracle's float64
                              sequential sum)
  * triangulation           : 1e-5 relative (double DLT on both sides, different SVD methods)
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4
THR = 3000.0  # exec/icp_test.cpp:86


def _pose_tol(n):
    """1-2 correspondences under-determine the 6-DoF pose (rank(J^T J) <= 4): 50 damped rounds
    amplify last-bit differences without bound in the unobservable directions -- the oracle's own
    float32 and float64 accumulations of the same problem end 1e-4..4e-4 apart, and a bit-exact
    Jacobian does not change that (tools/k_paths.py).  Those cases are held to 1e-2; every
    determined problem (n >= 3) to the north-star 1e-4."""
    return POSE_TOL if n >= 3 else 1e-2


def _synth():
    from picp_amd import synth
    return synth


def _chi_gate(T, K, xyz, uv, rows=480, cols=640):
    """float64 restatement of the gate of src/picp_solver.cpp:56-91 (projectPoint of
    src/camera.h:24-36, then chi = |e|^2): (projectable, chi) per correspondence at pose T."""
    T = np.asarray(T, np.float64)
    pc = xyz.astype(np.float64) @ T[:3, :3].T + T[:3, 3]
    z = pc[:, 2]
    with np.errstate(divide="ignore", invalid="ignore"):
        pi = pc @ np.asarray(K, np.float64).T
        u, v = pi[:, 0] / pi[:, 2], pi[:, 1] / pi[:, 2]
    ok = (z > 0) & (u >= 0) & (u <= cols - 1) & (v >= 0) & (v <= rows - 1)
    chi = np.where(ok, (u - uv[:, 0]) ** 2 + (v - uv[:, 1]) ** 2, np.inf)
    with np.errstate(invalid="ignore"):
        edge = np.minimum(np.minimum(np.abs(u), np.abs(u - (cols - 1))), np.minimum(np.abs(v), np.abs(v - (rows - 1))))
    return ok, chi, np.where(z > 0, edge, np.inf)


def _assert_n_in_explained(K, xyz, uv, T_gpu, T_ref, n_gpu, n_ref, thr=THR):
    """After a 50-round solve the GPU and oracle poses differ in the last bits, so a point whose
    chi lies within that difference of the threshold may be gated differently.  Instead of a
    fixed slack, the difference in n_in must be covered by the points that are ambiguous between
    the two poses: chi within 4x the largest per-point chi change between them (plus a 1e-6
    relative floor) of the threshold, or a projectability change.  The image-bound test
    (src/camera.h:31-34) runs on the float32 projection, so a point whose projection lies within
    1e-3 px (float32 rounding at 640 px, with margin) of a bound is ambiguous too."""
    if n_gpu == n_ref:
        return
    ok_g, chi_g, edge_g = _chi_gate(T_gpu, K, xyz, uv)
    ok_r, chi_r, edge_r = _chi_gate(T_ref, K, xyz, uv)
    both = ok_g & ok_r
    move = float(np.abs(chi_g[both] - chi_r[both]).max()) if both.any() else 0.0
    band = 4.0 * move + 1e-6 * thr
    at_edge = np.minimum(edge_g, edge_r) <= 1e-3
    ambiguous = int((both & ((np.abs(chi_r - thr) <= band) | at_edge)).sum() + (ok_g != ok_r).sum())
    assert abs(n_gpu - n_ref) <= ambiguous, (n_gpu, n_ref, ambiguous, move, float(np.min(np.minimum(edge_g, edge_r))))
    assert ambiguous <= max(2, len(xyz) // 1000), (ambiguous, move)  # the band stays narrow


def _lin_close(got, ref, rtol=1e-5):
    sH = np.abs(ref["H"]).max()
    np.testing.assert_allclose(got["H"], ref["H"], rtol=rtol, atol=rtol * sH)
    sb = max(np.abs(ref["b"]).max(), 1e-30)
    np.testing.assert_allclose(got["b"], ref["b"], rtol=rtol, atol=rtol * sb)
    np.testing.assert_allclose(got["chi_in"], ref["chi_in"], rtol=rtol, atol=1e-6)
    np.testing.assert_allclose(got["chi_out"], ref["chi_out"], rtol=rtol, atol=1e-6)


@pytest.mark.parametrize("n,seed,of,noise", [(1, 0, 0.0, 0.0), (17, 1, 0.0, 0.0), (1000, 0, 0.0, 0.0),
                                             (1000, 1, 0.3, 0.5), (20000, 2, 0.0, 0.5),
                                             (20000, 3, 0.3, 0.5), (100003, 4, 0.3, 0.5)])
@pytest.mark.parametrize("keep", [0, 1])
def test_linearize_matches_oracle(native, oracle, n, seed, of, noise, keep):
    synth = _synth()
    p = synth.make_problem(n, seed=seed, outlier_frac=of, pixel_noise=noise)
    s = native.PICPSolver(rows=480, cols=640, K=p["K"])
    s.init(p["T_init"], p["world"], p["image"])
    s.setKernelThreshold(THR)
    got = s.linearize(p["pairs"], keep_outliers=bool(keep))
    ref = oracle.linearize(p["T_init"], p["K"], 480, 640, p["world"], p["image"], p["pairs"], THR,
                           keep_outliers=keep, mode=oracle.MODE_F64)
    assert got["n_in"] == ref["n_in"]
    assert got["n_projected"] == ref["n_projected"]
    _lin_close(got, ref)


@pytest.mark.parametrize("n", [1000, 100003])
@pytest.mark.parametrize("keep", [0, 1])
def test_general_camera_path_matches_oracle(native, oracle, n, keep):
    """A K that is not [fx 0 cx; 0 fy cy; 0 0 1] (skew, and a non-unit K(2,2)) runs the general
    projection path (accumulate_one); the reference's pinhole K runs the specialised one.  Both
    are held to the same gate exactness and H/b tolerance."""
    synth = _synth()
    p = synth.make_problem(n, seed=5, outlier_frac=0.2, pixel_noise=0.5)
    K = np.array([[180, 3.5, 320], [0, 181, 240], [0, 0, 1.0000001]], np.float32)
    s = native.PICPSolver(rows=480, cols=640, K=K)
    s.init(p["T_init"], p["world"], p["image"])
    s.setKernelThreshold(THR)
    got = s.linearize(p["pairs"], keep_outliers=bool(keep))
    ref = oracle.linearize(p["T_init"], K, 480, 640, p["world"], p["image"], p["pairs"], THR,
                           keep_outliers=keep, mode=oracle.MODE_F64)
    assert got["n_in"] == ref["n_in"] and got["n_projected"] == ref["n_projected"]
    _lin_close(got, ref)
    st = s.solve(p["pairs"], max_rounds=20, conv_eps=-1.0, keep_outliers=bool(keep))
    T_ref, _ = oracle.solve(p["T_init"], K, 480, 640, p["world"], p["image"], p["pairs"], THR,
                            keep_outliers=bool(keep), max_rounds=20, conv_eps=-1.0)
    assert synth.se3_log_norm(s.pose(), T_ref) < POSE_TOL
    assert st["rounds"] == 20


def test_linearize_matches_golden_vectors(native):
    synth = _synth()
    g = np.load(os.path.join(GOLDEN, "picp_golden.npz"))
    for name in ("s0_n1k", "s1_n1k_out30"):
        s = native.PICPSolver()
        s.init(g[name + "/T_init"], g[name + "/world"], g[name + "/image"])
        s.setKernelThreshold(THR)
        for keep in (0, 1):
            got = s.linearize(g[name + "/pairs"], keep_outliers=bool(keep))
            tag = "%s/lin_keep%d" % (name, keep)
            sc = g[tag + "/scal"]
            ref = {"H": g[tag + "/H"], "b": g[tag + "/b"], "chi_in": sc[0], "chi_out": sc[1]}
            assert got["n_in"] == int(sc[2]) and got["n_projected"] == int(sc[3])
            _lin_close(got, ref)
        st = s.solve(g[name + "/pairs"], max_rounds=50, conv_eps=-1.0)
        assert synth.se3_log_norm(s.pose(), g[name + "/solve_f64/T"]) < POSE_TOL
        assert st["rounds"] == 50


def test_one_round_matches_oracle(native, oracle):
    synth = _synth()
    p = synth.make_problem(5000, seed=7, outlier_frac=0.2, pixel_noise=0.5)
    s = native.PICPSolver()
    s.init(p["T_init"], p["world"], p["image"])
    s.setKernelThreshold(THR)
    T = p["T_init"].copy()
    for r in range(5):
        ok = s.oneRound(p["pairs"], False)
        okr, T, st = oracle.one_round(T, p["K"], 480, 640, p["world"], p["image"], p["pairs"], THR,
                                      mode=oracle.MODE_F64)
        assert ok and okr
        assert s.numInliers() == st["n_in"]
        np.testing.assert_allclose(s.chiInliers(), st["chi_in"], rtol=1e-5)
        assert synth.se3_log_norm(s.pose(), T) < 1e-6
        T = s.pose()  # continue both from the GPU pose so rounds stay comparable


@pytest.mark.parametrize("n,seed,of,keep", [(10000, 10, 0.0, 0), (10000, 11, 0.3, 0),
                                            (10000, 12, 0.3, 1), (100000, 13, 0.0, 0)])
def test_solve_matches_oracle(native, oracle, n, seed, of, keep):
    synth = _synth()
    p = synth.make_problem(n, seed=seed, outlier_frac=of, pixel_noise=0.5)
    s = native.PICPSolver()
    s.init(p["T_init"], p["world"], p["image"])
    s.setKernelThreshold(THR)
    st = s.solve(p["pairs"], max_rounds=50, conv_eps=-1.0, keep_outliers=bool(keep))
    T_ref, st_ref = oracle.solve(p["T_init"], p["K"], 480, 640, p["world"], p["image"], p["pairs"],
                                 THR, keep_outliers=keep, mode=oracle.MODE_F64, max_rounds=50,
                                 conv_eps=-1.0)
    T_f, _ = oracle.solve(p["T_init"], p["K"], 480, 640, p["world"], p["image"], p["pairs"], THR,
                          keep_outliers=keep, mode=oracle.MODE_FAITHFUL, max_rounds=50, conv_eps=-1.0)
    assert st["rounds"] == 50 and st["ok"] == 1
    assert synth.se3_log_norm(s.pose(), T_ref) < POSE_TOL
    assert synth.se3_log_norm(s.pose(), T_f) < POSE_TOL
    _assert_n_in_explained(p["K"], p["xyz"], p["uv"], s.pose(), T_ref, st["n_in"], st_ref["n_in"])
    if not keep:  # keep_outliers=True: the saturated outliers still pull (biased, as in the reference)
        assert synth.se3_log_norm(s.pose(), p["T_gt"]) < 1e-2


def test_solve_convergence_rule_matches_oracle(native, oracle):
    """exec/icp_test.cpp:99-106 evaluated on the device."""
    synth = _synth()
    p = synth.make_problem(3000, seed=21, pixel_noise=1.0)
    s = native.PICPSolver()
    s.init(p["T_init"], p["world"], p["image"])
    s.setKernelThreshold(THR)
    st = s.solve(p["pairs"], max_rounds=50, conv_eps=1e-3)
    T_ref, st_ref = oracle.solve(p["T_init"], p["K"], 480, 640, p["world"], p["image"], p["pairs"],
                                 THR, mode=oracle.MODE_F64, max_rounds=50, conv_eps=1e-3)
    assert st["converged"] == 1 and st_ref["converged"]
    assert st["rounds"] == st_ref["rounds"]
    assert synth.se3_log_norm(s.pose(), T_ref) < POSE_TOL


def test_too_few_inliers_keeps_pose(native):
    synth = _synth()
    p = synth.make_problem(200, seed=3)
    s = native.PICPSolver()
    s.init(p["T_init"], p["world"], p["image"])
    s._min_inliers = 1000  # src/picp_solver.cpp:97-100
    assert s.oneRound(p["pairs"], False) is False
    np.testing.assert_array_equal(s.pose(), p["T_init"])
    st = s.solve(p["pairs"], max_rounds=50)
    assert st["ok"] == 0 and st["rounds"] == 1
    np.testing.assert_array_equal(s.pose(), p["T_init"])


def test_empty_and_out_of_range(native):
    synth = _synth()
    p = synth.make_problem(50, seed=3)
    s = native.PICPSolver()
    s.init(p["T_init"], p["world"], p["image"])
    st = s.solve(np.zeros((0, 2), np.int32), max_rounds=50)
    assert st["n_in"] == 0 and st["ok"] == 1
    np.testing.assert_array_equal(s.pose(), p["T_init"])  # H = I, b = 0 -> dx = 0
    with pytest.raises(native.PicpError) as ei:
        s.set_correspondences(np.array([[0, 50]], np.int32))
    assert ei.value.code == native.ERR_RANGE
    with pytest.raises(native.PicpError):
        s.set_correspondences(np.array([[-1, 0]], np.int32))


def test_points_behind_camera_and_outside_image_are_skipped(native, oracle):
    synth = _synth()
    p = synth.make_problem(2000, seed=8)
    world = p["world"].copy()
    # push a slice of points behind the camera and a slice far off-image
    T = p["T_gt"].astype(np.float64)
    cam = (T[:3, :3] @ world.T.astype(np.float64) + T[:3, 3:4]).T
    cam[:100, 2] *= -1
    cam[100:200, 0] += 50.0
    Tcw = synth.rigid_inverse(T)
    world = ((Tcw[:3, :3] @ cam.T) + Tcw[:3, 3:4]).T.astype(np.float32)
    pairs = np.stack([np.arange(2000), np.arange(2000)], 1).astype(np.int32)
    image = p["image"][p["pairs"][:, 0]]
    world_p = world[p["pairs"][:, 1]]
    s = native.PICPSolver()
    s.init(p["T_init"], world_p, image)
    s.setKernelThreshold(THR)
    got = s.linearize(pairs)
    ref = oracle.linearize(p["T_init"], p["K"], 480, 640, world_p, image, pairs, THR, mode=oracle.MODE_F64)
    assert got["n_projected"] == ref["n_projected"] <= 1800
    assert got["n_in"] == ref["n_in"]
    _lin_close(got, ref)


@pytest.mark.parametrize("mode", ["graph", "block"])
def test_batch_ragged_matches_single_and_oracle(native, oracle, mode):
    synth = _synth()
    sizes = [0, 1, 3, 1000, 5000, 20001, 1024, 4097]
    probs = [synth.make_problem(max(n, 1), seed=100 + i, outlier_frac=0.1, pixel_noise=0.5, shuffle=False)
             for i, n in enumerate(sizes)]
    xyz = np.concatenate([p["xyz"][:n] for p, n in zip(probs, sizes)])
    uv = np.concatenate([p["uv"][:n] for p, n in zip(probs, sizes)])
    b = _batch_mode(native, sizes, mode)
    assert b.info()["mode"] == mode
    b.set_data(xyz, uv)
    b.set_poses(np.stack([p["T_init"] for p in probs]))
    b.solve(threshold=THR, max_rounds=50, conv_eps=-1.0)
    poses, stats = b.poses(), b.stats()
    for i, (p, n) in enumerate(zip(probs, sizes)):
        T_ref, st_ref = oracle.solve_soa(p["T_init"], p["K"], 480, 640, p["x"][:n], p["y"][:n],
                                         p["z"][:n], p["u"][:n], p["v"][:n], THR,
                                         mode=oracle.MODE_F64, max_rounds=50, conv_eps=-1.0)
        assert synth.se3_log_norm(poses[i], T_ref) < _pose_tol(n), (i, n)
        assert stats[i]["rounds"] == 50
        _assert_n_in_explained(p["K"], p["xyz"][:n], p["uv"][:n], poses[i], T_ref, stats[i]["n_in"], st_ref["n_in"])
        if n >= 1000 and mode == "graph":
            import os
            pr = np.stack([np.arange(n), np.arange(n)], 1).astype(np.int32)
            os.environ["PICP_MODE"] = "graph"  # same mode as the batch
            try:
                s = native.PICPSolver()
                s.init(p["T_init"], p["xyz"][:n], p["uv"][:n])
                s.setKernelThreshold(THR)
                s.solve(pr, max_rounds=50, conv_eps=-1.0)
            finally:
                os.environ.pop("PICP_MODE", None)
            # same mode, partition and reduction order -> bit-identical to the batched solve
            np.testing.assert_array_equal(s.pose(), poses[i])
            s2 = native.PICPSolver()  # default (persistent) mode: same answer within tolerance
            s2.init(p["T_init"], p["xyz"][:n], p["uv"][:n])
            s2.setKernelThreshold(THR)
            s2.solve(pr, max_rounds=50, conv_eps=-1.0)
            assert synth.se3_log_norm(s2.pose(), poses[i]) < POSE_TOL


def test_solve_is_deterministic(native):
    synth = _synth()
    p = synth.make_problem(50000, seed=31, outlier_frac=0.3, pixel_noise=0.5)
    out = []
    for _ in range(2):
        s = native.PICPSolver()
        s.init(p["T_init"], p["world"], p["image"])
        s.setKernelThreshold(THR)
        st = s.solve(p["pairs"], max_rounds=50, conv_eps=-1.0)
        out.append((s.pose(), st["chi_in"], st["n_in"]))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1:] == out[1][1:]


def test_reference_data_kat_on_gpu(native, vo):
    """All 120 data/ frames (batched, one problem per frame) converge to ground truth."""
    synth = _synth()
    sizes, xyz, uv, Ti = [], [], [], []
    for k in range(1, vo.n_frames):
        pr = vo.correspondences(k)
        sizes.append(len(pr))
        xyz.append(vo.world_xyz[pr[:, 1]])
        uv.append(vo.frame(k)["uv"][pr[:, 0]])
        Ti.append(vo.T_wc(k - 1))
    b = native.Batch(sizes, K=vo.K)
    b.set_data(np.concatenate(xyz), np.concatenate(uv))
    b.set_poses(np.stack(Ti))
    b.solve(threshold=THR, max_rounds=50, conv_eps=1e-5)
    P = b.poses()
    worst = max(float(np.abs(P[k - 1] - vo.T_wc(k)).max()) for k in range(1, vo.n_frames))
    assert worst < 1e-3, worst
    for k, st in zip(range(1, vo.n_frames), b.stats()):
        assert len(vo.correspondences(k)) - 2 <= st["n_in"]


def test_drop_in_icp_loop_on_reference_data(native, oracle, vo):
    """exec/icp_test.cpp:78-117 driven through oneRound (host loop), frames 1..10."""
    synth = _synth()
    s = native.PICPSolver(K=vo.K)
    for k in range(1, 11):
        pr = vo.correspondences(k)
        s.init(vo.T_wc(k - 1), vo.world_xyz, vo.frame(k)["uv"])
        s.setKernelThreshold(3000.0)
        prev = np.finfo(np.float32).max
        for j in range(50):
            assert s.oneRound(pr, False)
            cur = s.chiInliers()
            rel = abs(prev - cur) / prev if prev > 1e-10 else 0.0
            if rel < 1e-5:
                break
            prev = cur
        T_ref, _ = oracle.solve(vo.T_wc(k - 1), vo.K, 480, 640, vo.world_xyz, vo.frame(k)["uv"], pr,
                                3000.0, mode=oracle.MODE_F64)
        assert synth.se3_log_norm(s.pose(), T_ref) < POSE_TOL
        assert synth.se3_log_norm(s.pose(), vo.T_wc(k)) < 2e-3


def test_triangulation_matches_oracle_and_world(native, oracle, vo):
    g = np.load(os.path.join(GOLDEN, "picp_golden.npz"))
    got = native.triangulate(g["tri/P1"], g["tri/P2"], g["tri/uv1"], g["tri/uv2"])
    np.testing.assert_allclose(got, g["tri/xyz"], rtol=1e-5, atol=1e-5)
    ref = vo.world_xyz[[int(np.where(vo.world_id == i)[0][0]) for i in g["tri/ids"]]]
    assert np.abs(got - ref).max() < 2e-3
    # random stress incl. near-degenerate rays, against the oracle
    rng = np.random.default_rng(9)
    uv1 = rng.uniform([0, 0], [639, 479], (5000, 2)).astype(np.float32)
    uv2 = (uv1 + rng.normal(0, 3, uv1.shape)).astype(np.float32)
    got = native.triangulate(g["tri/P1"], g["tri/P2"], uv1, uv2)
    ref = oracle.triangulate(g["tri/P1"], g["tri/P2"], uv1, uv2)
    rel = np.abs(got - ref) / np.maximum(np.abs(ref), 1.0)
    assert np.quantile(rel, 0.999) < 1e-4
    assert native.triangulate(g["tri/P1"], g["tri/P2"], uv1[:0], uv2[:0]).shape == (0, 3)


def test_projection_matrix_matches_oracle(native, oracle, vo):
    Tcw = _synth().rigid_inverse(vo.T_wc(3).astype(np.float64)).astype(np.float32)
    np.testing.assert_array_equal(native.projection_matrix(vo.K, Tcw), oracle.projection_matrix(vo.K, Tcw))


def test_full_size_c2_c3_properties(native, oracle):
    """BASELINE configs at full size: C2 (100k, 50 rounds) and C3 (1M, 30% outliers)."""
    synth = _synth()
    for n, of in ((100000, 0.0), (1000000, 0.3)):
        p = synth.make_problem(n, seed=42, outlier_frac=of, pixel_noise=0.5)
        b = native.Batch([n])
        b.set_data(p["xyz"], p["uv"])
        b.set_poses(p["T_init"][None])
        b.solve(threshold=THR, max_rounds=50, conv_eps=-1.0)
        T = b.poses()[0]
        st = b.stats()[0]
        assert synth.se3_log_norm(T, p["T_gt"]) < 2e-3
        # every true inlier is gated in; accidental outliers within sqrt(3000) px also pass
        assert st["n_in"] >= int(0.99 * (n - p["outlier"].sum()))
        T_ref, st_ref = oracle.solve_soa(p["T_init"], p["K"], 480, 640, p["x"], p["y"], p["z"],
                                         p["u"], p["v"], THR, mode=oracle.MODE_F64, max_rounds=50,
                                         conv_eps=-1.0)
        assert synth.se3_log_norm(T, T_ref) < POSE_TOL
        _assert_n_in_explained(p["K"], p["xyz"], p["uv"], T, T_ref, st["n_in"], st_ref["n_in"])


def _batch_mode(native, sizes, mode, **kw):
    import os
    old = os.environ.get("PICP_MODE")
    os.environ["PICP_MODE"] = mode
    try:
        return native.Batch(sizes, **kw)
    finally:
        if old is None:
            os.environ.pop("PICP_MODE", None)
        else:
            os.environ["PICP_MODE"] = old


@pytest.mark.parametrize("n,of,keep,conv", [(100000, 0.0, 0, -1.0), (100000, 0.3, 1, -1.0),
                                            (1000000, 0.3, 0, -1.0), (3000, 0.0, 0, 1e-4),
                                            (257, 0.0, 0, -1.0), (1, 0.0, 0, -1.0),
                                            (250000, 0.3, 0, -1.0), (500000, 0.0, 1, 1e-5)])
def test_persistent_and_graph_modes_agree_with_oracle(native, oracle, n, of, keep, conv):
    """Single-launch persistent solve vs one-launch-per-round graph solve vs the oracle.  The
    sizes cover every register-resident shape: 1 item per lane (100k), 2 (250k) and 4 (500k) --
    the one-slot accumulation -- and 8 (1M) -- the pair form (picp_device.h acc_pairs)."""
    synth = _synth()
    p = synth.make_problem(n, seed=77, outlier_frac=of, pixel_noise=0.5, shuffle=False)
    res = {}
    for mode in ("persistent", "graph"):
        b = _batch_mode(native, [n], mode)
        assert b.info()["mode"] == mode
        b.set_data(p["xyz"], p["uv"])
        b.set_poses(p["T_init"][None])
        b.solve(threshold=THR, max_rounds=50, conv_eps=conv, keep_outliers=keep)
        res[mode] = (b.poses()[0], b.stats()[0])
    T_ref, st_ref = oracle.solve_soa(p["T_init"], p["K"], 480, 640, p["x"], p["y"], p["z"], p["u"], p["v"],
                                     THR, keep_outliers=keep, mode=oracle.MODE_F64, max_rounds=50,
                                     conv_eps=conv)
    for mode, (T, st) in res.items():
        assert synth.se3_log_norm(T, T_ref) < _pose_tol(n), mode
        _assert_n_in_explained(p["K"], p["xyz"], p["uv"], T, T_ref, st["n_in"], st_ref["n_in"])
        if conv < 0:
            assert st["rounds"] == 50
    assert res["persistent"][1]["rounds"] == res["graph"][1]["rounds"]


@pytest.mark.parametrize("mode,P,n", [("persistent", 8, 5000), ("block", 8, 5000), ("block", 6, 20000),
                                      ("graph", 8, 5000)])
def test_uniform_multi_frame_batch_modes(native, oracle, mode, P, n):
    synth = _synth()
    bt = synth.make_batch(P, n, base_seed=500, pixel_noise=0.5, outlier_frac=0.1)
    b = _batch_mode(native, bt["sizes"], mode)
    assert b.info()["mode"] == mode
    b.set_data(bt["xyz"], bt["uv"])
    b.set_poses(bt["T_init"])
    b.solve(threshold=THR, max_rounds=50, conv_eps=1e-5)
    poses, stats = b.poses(), b.stats()
    for i in range(P):
        xyz = bt["xyz"][i * n:(i + 1) * n]
        uv = bt["uv"][i * n:(i + 1) * n]
        T_ref, st_ref = oracle.solve_soa(bt["T_init"][i], synth.K_REF.astype(np.float32), 480, 640,
                                         xyz[:, 0].copy(), xyz[:, 1].copy(), xyz[:, 2].copy(),
                                         uv[:, 0].copy(), uv[:, 1].copy(), THR, mode=oracle.MODE_F64,
                                         max_rounds=50, conv_eps=1e-5)
        assert synth.se3_log_norm(poses[i], T_ref) < POSE_TOL
        assert stats[i]["converged"] == int(st_ref["converged"])
    # repeated replays of the same graph give identical results (persistent / split block: the
    # granule tags continue from the tag bases the previous launch left, nothing is re-zeroed)
    b.solve(threshold=THR, max_rounds=50, conv_eps=1e-5)
    np.testing.assert_array_equal(b.poses(), poses)


@pytest.mark.parametrize("mode,P,n,split", [("persistent", 1, 100000, None), ("persistent", 4, 5000, None),
                                            ("block", 8, 8192, "2"), ("block", 8, 8192, "4")])
def test_tag_bases_across_launches(native, mode, P, n, split):
    """Persistent and split-block launches run without a memset between them: every solve's
    granule tags start past the previous launch's.  Interleave solves of 0, 1, 7 and 50 rounds
    and convergence-terminated ones (rounds differ per problem) on ONE batch, each compared
    bit for bit with the same solve on a fresh batch."""
    import os
    synth = _synth()
    bt = synth.make_batch(P, n, base_seed=900, pixel_noise=0.5, outlier_frac=0.1)
    old = os.environ.get("PICP_BLOCK_SPLIT")
    if split:
        os.environ["PICP_BLOCK_SPLIT"] = split
    try:
        def fresh():
            b = _batch_mode(native, bt["sizes"], mode)
            b.set_data(bt["xyz"], bt["uv"])
            b.set_poses(bt["T_init"])
            return b
        b = fresh()
        assert b.info()["mode"] == mode
        plan = [(50, -1.0), (0, -1.0), (7, -1.0), (1, -1.0), (50, 1e-5), (50, -1.0), (7, 1e-3), (50, 1e-5)]
        for R, eps in plan:
            b.solve(threshold=THR, max_rounds=R, conv_eps=eps)
            f = fresh()
            f.solve(threshold=THR, max_rounds=R, conv_eps=eps)
            np.testing.assert_array_equal(b.poses(), f.poses(), err_msg="R=%d eps=%g" % (R, eps))
            assert [s["rounds"] for s in b.stats()] == [s["rounds"] for s in f.stats()]
    finally:
        if old is None:
            os.environ.pop("PICP_BLOCK_SPLIT", None)
        else:
            os.environ["PICP_BLOCK_SPLIT"] = old


def test_fast_reciprocal_is_correctly_rounded(native):
    """The projection's 1/z (src/camera.h:30) feeds the bit-exact gate.  The kernels compute it
    as v_rcp + one FMA Newton step; over the 16 binades [2^-8, 2^8), both signs (268M floats),
    it must equal the IEEE division bit for bit -- which, by power-of-two scaling, proves it
    for every |z| in [2^-100, 2^100] (outside: the kernels use the division)."""
    assert native.selftest_rcp(-8, 8) == 0


@pytest.mark.parametrize("sizes", [[300003], [262147, 300001]])
def test_streaming_sweep_directions_ragged_tail(native, oracle, sizes):
    """Graph mode with float4 lanes (> 2^18 correspondences): odd rounds sweep each block's slice
    backwards (change 7).  Slices whose tail is not a multiple of 4 exercise the
    mirrored masking; both sweep orders must match the oracle, and each must replay bit-exactly."""
    import os
    synth = _synth()
    probs = [synth.make_problem(n, seed=900 + i, outlier_frac=0.2, pixel_noise=0.5, shuffle=False)
             for i, n in enumerate(sizes)]
    xyz = np.concatenate([p["xyz"] for p in probs])
    uv = np.concatenate([p["uv"] for p in probs])
    Ti = np.stack([p["T_init"] for p in probs])
    res = {}
    for fwd in ("0", "1"):
        os.environ["PICP_SWEEP_FORWARD"] = fwd
        try:
            b = _batch_mode(native, sizes, "graph")
            assert b.info()["mode"] == "graph"
            b.set_data(xyz, uv)
            b.set_poses(Ti)
            b.solve(threshold=THR, max_rounds=20, conv_eps=-1.0)
            poses, stats = b.poses(), b.stats()
            b.solve(threshold=THR, max_rounds=20, conv_eps=-1.0)
            np.testing.assert_array_equal(b.poses(), poses)
        finally:
            os.environ.pop("PICP_SWEEP_FORWARD", None)
        res[fwd] = (poses, stats)
    for i, p in enumerate(probs):
        T_ref, st_ref = oracle.solve_soa(p["T_init"], p["K"], 480, 640, p["x"], p["y"], p["z"], p["u"],
                                         p["v"], THR, mode=oracle.MODE_F64, max_rounds=20, conv_eps=-1.0)
        for fwd, (poses, stats) in res.items():
            assert synth.se3_log_norm(poses[i], T_ref) < POSE_TOL, (fwd, i)
            _assert_n_in_explained(p["K"], p["xyz"], p["uv"], poses[i], T_ref, stats[i]["n_in"], st_ref["n_in"])


def test_streaming_weighted_pair_split_matches_oracle(native, oracle):
    """A streaming single frame on two blocks per CU (>= 2^23 correspondences: 2 x CUs blocks)
    gives each CU-pair's older block the larger share of a contiguous range (PICP_STREAM_SHARE,
    DESIGN §4.1); equal shares (0.5) keep the uniform slices.  Both vs the oracle over a few
    rounds (the oracle at this size takes ~0.5 s a round), replays bit-identical."""
    import os
    synth = _synth()
    n = (1 << 23) + 4099  # ragged tail
    p = synth.make_problem(n, seed=901, outlier_frac=0.2, pixel_noise=0.5, shuffle=False)
    R = 3
    res = {}
    for share in ("0.5", "0.64"):
        os.environ["PICP_STREAM_SHARE"] = share
        try:
            b = _batch_mode(native, [n], "graph")
            info = b.info()
            assert info["mode"] == "graph" and info["n_blocks"] % 2 == 0
            b.set_data(p["xyz"], p["uv"])
            b.set_poses(p["T_init"][None])
            b.solve(threshold=THR, max_rounds=R, conv_eps=-1.0)
            T, st = b.poses()[0], b.stats()[0]
            b.solve(threshold=THR, max_rounds=R, conv_eps=-1.0)
            np.testing.assert_array_equal(b.poses()[0], T)
        finally:
            os.environ.pop("PICP_STREAM_SHARE", None)
        res[share] = (T, st)
    T_ref, st_ref = oracle.solve_soa(p["T_init"], p["K"], 480, 640, p["x"], p["y"], p["z"], p["u"], p["v"],
                                     THR, mode=oracle.MODE_F64, max_rounds=R, conv_eps=-1.0)
    for share, (T, st) in res.items():
        assert synth.se3_log_norm(T, T_ref) < POSE_TOL, share
        _assert_n_in_explained(p["K"], p["xyz"], p["uv"], T, T_ref, st["n_in"], st_ref["n_in"])


@pytest.mark.parametrize("sizes", [[5000, 1, 3, 4097, 12000, 7], [10000] * 32, [10000] * 128])
def test_block_split_matches_oracle(native, oracle, sizes):
    """Block mode with two or four blocks per problem (PICP_BLOCK_SPLIT=2: halves on 512-thread
    partner blocks; =4: quarters on 512-thread blocks, two per CU -- the C4 layout at 128 frames
    per GPU; partners exchange {round, hi|lo} granules every round) and with one block per
    problem: all vs the oracle, converged-round counts equal, replays bit-identical.  Problems of
    1-7 correspondences leave the later parts empty."""
    import os
    synth = _synth()
    probs = [synth.make_problem(n, seed=1300 + i, outlier_frac=0.1 if n >= 1000 else 0.0, pixel_noise=0.5,
                                shuffle=False) for i, n in enumerate(sizes)]
    xyz = np.concatenate([p["xyz"] for p in probs])
    uv = np.concatenate([p["uv"] for p in probs])
    Ti = np.stack([p["T_init"] for p in probs])
    res = {}
    for split in ("1", "2", "4"):
        os.environ["PICP_BLOCK_SPLIT"] = split
        try:
            b = _batch_mode(native, sizes, "block")
            assert b.info()["mode"] == "block"
            b.set_data(xyz, uv)
            b.set_poses(Ti)
            b.solve(threshold=THR, max_rounds=50, conv_eps=1e-5)
            poses, stats = b.poses(), b.stats()
            b.solve(threshold=THR, max_rounds=50, conv_eps=1e-5)
            np.testing.assert_array_equal(b.poses(), poses)
        finally:
            os.environ.pop("PICP_BLOCK_SPLIT", None)
        res[split] = (poses, stats)
    for i, p in enumerate(probs):
        if i >= 8 and i % 8:  # the uniform batch: every 8th problem against the oracle
            continue
        T_ref, st_ref = oracle.solve_soa(p["T_init"], p["K"], 480, 640, p["x"], p["y"], p["z"], p["u"],
                                         p["v"], THR, mode=oracle.MODE_F64, max_rounds=50, conv_eps=1e-5)
        n = sizes[i]
        for split, (poses, stats) in res.items():
            assert synth.se3_log_norm(poses[i], T_ref) < _pose_tol(n), (split, i)
            _assert_n_in_explained(p["K"], p["xyz"], p["uv"], poses[i], T_ref, stats[i]["n_in"], st_ref["n_in"])
            if n >= 1000:
                assert stats[i]["converged"] == int(st_ref["converged"]), (split, i)
