"""GPU parity of the essential-matrix bootstrap (src/cam.cpp:37-91: findEssentialMat + recoverPose,
SURVEY.md §8f rank 4) against the oracle (oracle/picp_essential.c), which is pinned by reproducing
the reference's published trajectory (tests/test_oracle.py::test_kat_bootstrap_reproduces_reference_run).

Both compute the same RANSAC subsets, five-point solutions and inlier counts in double (the
kernels with FP contraction off), so the chosen model, its inlier count and recoverPose's count
are equal and the poses agree to float rounding of the output.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _oracle_pose(oracle, p1, p2, K, **kw):
    E, cnt = oracle.find_essential(p1, p2, K, **kw)
    if E is None:
        return np.eye(4), 0, 0
    R, t, mask, good = oracle.recover_pose(E, p1, p2, K)
    T = np.eye(4)
    T[:3, :3], T[:3, 3] = R, t
    return np.linalg.inv(T), cnt, good


def _data_pairs(oracle, vo, ks):
    p1s, p2s = [], []
    for k in ks:
        fa, fb = vo.frame(k), vo.frame(k + 1)
        m = oracle.match_points(fa["desc"], fb["desc"])  # exec/icp_test.cpp:46
        acc = m["accepted"].astype(bool)
        p1s.append(fa["uv"][acc])
        p2s.append(fb["uv"][m["best_idx"][acc]])
    return p1s, p2s


def test_essential_matches_oracle_on_every_data_frame_pair(native, oracle, vo):
    """All 120 consecutive pairs of data/ in one batch (frames 0-1 is the reference's bootstrap;
    the others include near-pure-rotation pairs where recoverPose keeps few points)."""
    ks = list(range(vo.n_frames - 1))
    p1s, p2s = _data_pairs(oracle, vo, ks)
    K = vo.K.astype(np.float64)
    res = native.essential_recover_pose_batch(p1s, p2s, K=vo.K, want_mask=True)
    for k, r in zip(ks, res):
        T, inl, good = _oracle_pose(oracle, p1s[k], p2s[k], K)
        assert r["inliers"] == inl, k
        assert r["good"] == good, k
        assert r["mask"].sum() == good, k
        np.testing.assert_allclose(r["T"], T, atol=2e-6, err_msg="pair %d" % k)


def test_essential_bootstrap_frame0_is_reference_pose(native, oracle, vo):
    p1s, p2s = _data_pairs(oracle, vo, [0])
    r = native.essential_recover_pose_batch(p1s, p2s, K=vo.K)[0]
    assert r["inliers"] == 115 and r["good"] == 115
    # the reference's bootstrap after frame 1's PICP is output/estimated_trajectory.txt row 1
    row = vo.trajectory_rows([np.eye(4), r["T"]])[1]
    np.testing.assert_allclose(row[1:], vo.ref_trajectory[1, 1:], atol=5e-5)


def _two_view(rng, n, outlier_frac, noise_px):
    K = np.array([[180.0, 0, 320], [0, 180, 240], [0, 0, 1]])
    ang = rng.normal(0, 0.1, 3)
    th = np.linalg.norm(ang)
    kx = np.array([[0, -ang[2], ang[1]], [ang[2], 0, -ang[0]], [-ang[1], ang[0], 0]]) / th
    R = np.eye(3) + np.sin(th) * kx + (1 - np.cos(th)) * kx @ kx
    t = rng.normal(0, 1, 3)
    t[2] = abs(t[2])
    t /= np.linalg.norm(t)
    X = np.c_[rng.uniform(-3, 3, (n, 2)), rng.uniform(3, 10, n)]
    X2 = X @ R.T + t
    p1 = (X @ K.T)[:, :2] / X[:, 2:]
    p2 = (X2 @ K.T)[:, :2] / X2[:, 2:]
    p1 += rng.normal(0, noise_px, p1.shape)
    p2 += rng.normal(0, noise_px, p2.shape)
    bad = rng.random(n) < outlier_frac
    p2[bad] = rng.uniform([0, 0], [640, 480], (bad.sum(), 2))
    T = np.eye(4)
    T[:3, :3], T[:3, 3] = R, t
    return p1.astype(np.float32), p2.astype(np.float32), np.linalg.inv(T), K


def test_essential_synthetic_outliers_and_noise(native, oracle):
    rng = np.random.default_rng(7)
    cases = [_two_view(rng, n, of, nz) for n, of, nz in
             [(200, 0.0, 0.0), (200, 0.3, 0.3), (500, 0.5, 0.5), (60, 0.2, 0.2), (1000, 0.3, 0.5), (9, 0.0, 0.1)]]
    res = native.essential_recover_pose_batch([c[0] for c in cases], [c[1] for c in cases], K=cases[0][3])
    for i, (p1, p2, Tgt, K) in enumerate(cases):
        T, inl, good = _oracle_pose(oracle, p1, p2, K)
        assert res[i]["inliers"] == inl and res[i]["good"] == good, i
        np.testing.assert_allclose(res[i]["T"], T, atol=2e-6, err_msg="case %d" % i)
        # and the geometry is recovered (unit baseline)
        assert np.abs(res[i]["T"][:3, :3] - Tgt[:3, :3]).max() < 5e-2, i
        assert np.abs(res[i]["T"][:3, 3] - Tgt[:3, 3]).max() < 0.25, i  # 9 points, 0.1 px: 0.17


def test_essential_edge_cases(native, oracle):
    rng = np.random.default_rng(11)
    p1, p2, _, K = _two_view(rng, 40, 0.0, 0.0)
    res = native.essential_recover_pose_batch([p1[:3], np.zeros((0, 2)), p1[:5], p1], [p2[:3], np.zeros((0, 2)), p2[:5], p2],
                                              K=K)
    for r in res[:2]:  # fewer than five points: no model
        assert r["inliers"] == 0 and r["good"] == 0
        np.testing.assert_array_equal(r["T"], np.eye(4))
    T5, inl5, good5 = _oracle_pose(oracle, p1[:5], p2[:5], K)
    assert res[2]["inliers"] == inl5 == 5
    np.testing.assert_allclose(res[2]["T"], T5, atol=2e-6)
    assert res[3]["inliers"] == 40
    with pytest.raises(native.PicpError):
        native.essential_recover_pose_batch([p1], [p2], K=K, max_iters=0)
    with pytest.raises(native.PicpError):
        native.essential_recover_pose_batch([p1], [p2], K=K, prob=1.0)
