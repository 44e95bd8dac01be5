"""Trajectory evaluation of the C5 line (picp_amd/evaluate.py): the umeyama similarity of the
reference's alignTrajectories (src/my_utilities.cpp:459-478), the ATE after it, and the stitching of
segment trajectories at their one-frame overlaps.  CPU only."""
import numpy as np
import pytest

from picp_amd.evaluate import ate, stitch_segments, umeyama
from picp_amd.synth import planar
from picp_amd.vo_synth import VOSequence, segments


def _rot(a, b, c):
    ca, sa, cb, sb, cc, sc = np.cos(a), np.sin(a), np.cos(b), np.sin(b), np.cos(c), np.sin(c)
    Rx = np.array([[1, 0, 0], [0, ca, -sa], [0, sa, ca]])
    Ry = np.array([[cb, 0, sb], [0, 1, 0], [-sb, 0, cb]])
    Rz = np.array([[cc, -sc, 0], [sc, cc, 0], [0, 0, 1]])
    return Rx @ Ry @ Rz


def test_umeyama_recovers_a_similarity():
    rng = np.random.default_rng(3)
    src = rng.normal(size=(50, 3))
    R = _rot(0.3, -0.2, 1.1)
    c, t = 2.5, np.array([1.0, -4.0, 0.5])
    dst = c * src @ R.T + t
    S = umeyama(src, dst)
    np.testing.assert_allclose(S[:3, :3], c * R, atol=1e-10)
    np.testing.assert_allclose(S[:3, 3], t, atol=1e-10)
    # without scale: the rotation alone
    S1 = umeyama(src, src @ R.T + t, with_scale=False)
    np.testing.assert_allclose(S1[:3, :3], R, atol=1e-10)


def test_umeyama_handles_a_reflection_case():
    """A planar point set: Umeyama's sign correction keeps a proper rotation (det +1)."""
    rng = np.random.default_rng(4)
    src = np.c_[rng.normal(size=(30, 2)), np.zeros(30)]
    R = _rot(0.0, 0.0, 0.7)
    S = umeyama(src, src @ R.T)
    assert np.linalg.det(S[:3, :3]) > 0
    np.testing.assert_allclose(S[:3, :3], R, atol=1e-9)


def test_stitching_exact_segments_gives_the_ground_truth():
    seq = VOSequence(201, obs_per_frame=50, seed=1)
    first, steps = segments(201, 40)
    gt = np.stack([seq.T_cw(k) for k in range(201)])
    poses = [np.stack([np.linalg.inv(gt[f]) @ gt[f + t] for t in range(st + 1)]) for f, st in zip(first, steps)]
    frames, T = stitch_segments(poses, first, steps, gt[0])
    assert list(frames) == list(range(201))
    np.testing.assert_allclose(T, gt, atol=1e-9)
    r = ate(T, gt)
    assert r["ate_rmse_m"] < 1e-9 and r["rot_err_max_rad"] < 1e-6 and abs(r["sim3_scale"] - 1) < 1e-9
    assert r["path_length_m"] == pytest.approx(200 * 0.2, rel=1e-6)


def test_ate_is_invariant_to_a_similarity_of_the_estimate():
    """The reference aligns the estimate to the ground truth before measuring (umeyama with scale):
    a whole-trajectory rotation, translation and scale change nothing."""
    seq = VOSequence(60, obs_per_frame=50, seed=2)
    gt = np.stack([seq.T_cw(k) for k in range(60)])
    rng = np.random.default_rng(5)
    est = gt.copy()
    est[:, :3, 3] += rng.normal(scale=0.01, size=(60, 3))
    base = ate(est, gt)
    G = np.eye(4)
    G[:3, :3] = _rot(0.1, 0.2, -0.3)
    G[:3, 3] = [3, -1, 2]
    est2 = np.einsum("ij,njk->nik", G, est)
    est2[:, :3, 3] *= 0.5
    moved = ate(est2, gt)
    assert moved["ate_rmse_m"] == pytest.approx(base["ate_rmse_m"], rel=1e-6)
    assert moved["sim3_scale"] == pytest.approx(2.0 * base["sim3_scale"], rel=1e-6)


def test_stitching_rejects_segments_without_overlap():
    T = np.stack([np.eye(4)] * 3)
    with pytest.raises(ValueError):
        stitch_segments([T, T], [0, 3], [2, 2], planar(0, 0, 0))
