"""GPU parity of the device-resident VO sequence (picp_vo_*, exec/icp_test.cpp:36-136) against the
CPU oracle (oracle/picp_oracle.c or_vo_segment and its building blocks).

What is compared, and how strictly:
  * counts -- per step the map correspondences n_corr, the points appended n_new, the final map
    size and the map descriptors -- are EXACT: they follow from descriptor matching alone
    (bit-exact matcher) whatever the floating-point pose history;
  * the landmark set of the final data/ map equals the reference's own published run
    (output/estimated_world_points.txt, 490 ids; tests/golden/vo_data.npz ref_map_ids);
  * every STEP is checked under teacher forcing: the map is append-only, so the GPU's final map
    prefix plus its pose of frame k are exactly the inputs of the step that estimated frame k+1;
    the oracle re-runs that step (match, icp_test PICP loop in float64 accumulation,
    add_new_world_points, DLT) from those inputs:
      pose      : se3_log_norm(gpu, oracle) < 1e-4 (BASELINE.json north_star tolerance)
      new points: |gpu - oracle| <= 1e-4 * (1 + |oracle|) for 99% of points, all within 1e-2
                  relative (low-parallax points near the epipole are ill-conditioned; the two
                  sides use different SVD methods)
  * the free-running sequence is chaotic (a 1e-7 difference in one step grows through the
    triangulated map; the oracle's own float32-vs-float64 accumulation modes drift apart by
    2.4e-3 over data/), so whole-trajectory agreement is a loose band only (2e-2).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4
THR = 3000.0


def _se3(a, b):
    from picp_amd.synth import se3_log_norm, rigid_inverse
    return se3_log_norm(rigid_inverse(np.asarray(a, np.float64)), rigid_inverse(np.asarray(b, np.float64)))


def _teacher_forced(oracle, K, off, uv, desc, f0, poses, rec, map_xyz, map_desc):
    """Re-run every step of one GPU segment on the oracle from the GPU's own inputs."""
    steps = len(poses) - 1
    m = int(rec["n_new"][0])
    worst_pose, tri_err, tri_ref = 0.0, [], []
    for t in range(steps):
        cf, nf = f0 + t, f0 + t + 1
        dn = desc[off[nf]:off[nf + 1]]
        wm = oracle.match_points(dn, map_desc[:m])
        assert wm["accepted"].sum() == rec["n_corr"][t + 1]
        pairs = np.stack([np.nonzero(wm["accepted"])[0], wm["best_idx"][wm["accepted"]]], 1).astype(np.int32)
        T0 = np.linalg.inv(poses[t].astype(np.float64)).astype(np.float32)
        T, _ = oracle.solve(T0, K, 480, 640, map_xyz[:m], uv[off[nf]:off[nf + 1]], pairs, THR)
        worst_pose = max(worst_pose, _se3(np.linalg.inv(T.astype(np.float64)), poses[t + 1]))
        pm = oracle.match_points(desc[off[cf]:off[cf + 1]], dn)
        sel = pm["accepted"].copy()
        sel[sel] &= ~wm["accepted"][pm["best_idx"][sel]]
        ia = np.nonzero(sel)[0]
        ib = pm["best_idx"][ia]
        assert len(ia) == rec["n_new"][t + 1]
        np.testing.assert_array_equal(map_desc[m:m + len(ia)], desc[off[cf]:off[cf + 1]][ia])
        if len(ia):
            P1 = oracle.projection_matrix(K, poses[t])
            P2 = oracle.projection_matrix(K, poses[t + 1])
            X = oracle.triangulate(P1, P2, uv[off[cf]:off[cf + 1]][ia], uv[off[nf]:off[nf + 1]][ib])
            tri_err.append(np.abs(map_xyz[m:m + len(ia)] - X).max(1))
            tri_ref.append(1.0 + np.abs(X).max(1))
        m += len(ia)
    assert m == len(map_xyz)
    rel = np.concatenate(tri_err) / np.concatenate(tri_ref) if tri_err else np.zeros(1)
    return worst_pose, rel


def _check_segment(oracle, K, off, uv, desc, f0, T0, T1, poses, rec, mx, md):
    # bootstrap: exactly the oracle's bootstrap map
    pm = oracle.match_points(desc[off[f0]:off[f0 + 1]], desc[off[f0 + 1]:off[f0 + 2]])
    ia = np.nonzero(pm["accepted"])[0]
    assert rec["n_new"][0] == len(ia)
    X = oracle.triangulate(oracle.projection_matrix(K, T0), oracle.projection_matrix(K, T1),
                           uv[off[f0]:off[f0 + 1]][ia], uv[off[f0 + 1]:off[f0 + 2]][pm["best_idx"][ia]])
    np.testing.assert_allclose(mx[:len(ia)], X, rtol=1e-4, atol=1e-4)
    np.testing.assert_array_equal(poses[0], np.asarray(T0, np.float32))
    worst, rel = _teacher_forced(oracle, K, off, uv, desc, f0, poses, rec, mx, md)
    assert worst < POSE_TOL, worst
    assert np.quantile(rel, 0.99) < 1e-4 and rel.max() < 1e-2, (np.quantile(rel, 0.99), rel.max())


def test_vo_reference_data_sequence(native, oracle, vo):
    """data/ (C1): one segment over all 121 frames, bootstrap with the gt poses of frames 0/1."""
    from picp_amd.synth import MOUNT, planar
    off, uv, desc = vo.packed()
    Tc = [(planar(*vo.gt_pose[k]) @ MOUNT).astype(np.float32) for k in range(vo.n_frames)]
    seq = native.VOSequence(off, uv, desc, K=vo.K)
    seq.set_segments([0], [vo.n_frames - 1], [[Tc[0], Tc[1]]], threshold=THR)
    seq.run()
    poses, rec = seq.poses()[0], seq.step_records()[0]
    mx, md = seq.map(0)
    # the reference's published map: the same 490 landmarks
    ids = vo.map_ids(md)
    assert set(ids.tolist()) == set(vo.ref_map_ids.tolist()) and len(ids) == 490
    # counts equal the free-running oracle's (matching only)
    ref = oracle.vo_segment(vo.K, vo.rows, vo.cols, off, uv, desc, 0, vo.n_frames - 1, Tc[0], Tc[1])
    np.testing.assert_array_equal(rec["n_corr"][1:], ref["n_corr"])
    np.testing.assert_array_equal(rec["n_new"], ref["n_new"])
    np.testing.assert_array_equal(md, ref["map_desc"])
    _check_segment(oracle, vo.K, off, uv, desc, 0, Tc[0], Tc[1], poses, rec, mx, md)
    drift = max(_se3(poses[k], ref["poses"][k]) for k in range(vo.n_frames))
    assert drift < 2e-2, drift
    err = [np.linalg.norm(poses[k][:3, 3] - Tc[k][:3, 3]) for k in range(vo.n_frames)]
    assert max(err) < 0.1


@pytest.mark.parametrize("n_frames,obs,seg_len,noise", [(25, 600, 8, 0.0), (19, 1500, 6, 0.5)])
def test_vo_synthetic_segments(native, oracle, n_frames, obs, seg_len, noise):
    """C5 shape at test size: segments with a one-frame overlap (the last one shorter), all in one
    run; each segment checked step by step against the oracle."""
    from picp_amd.vo_synth import VOSequence, segments
    s = VOSequence(n_frames, obs_per_frame=obs, seed=11, pixel_noise=noise)
    F = s.frames(0, n_frames)
    first, steps = segments(n_frames, seg_len)
    boot = np.stack([[F["T_cw"][f], F["T_cw"][f + 1]] for f in first])
    seq = native.VOSequence(F["frame_off"], F["uv"], F["desc"], K=s.K)
    seq.set_segments(first, steps, boot, threshold=THR)
    seq.run()
    P, R = seq.poses(), seq.step_records()
    for k, (f0, st) in enumerate(zip(first, steps)):
        mx, md = seq.map(k)
        assert len(P[k]) == st + 1
        _check_segment(oracle, s.K, F["frame_off"], F["uv"], F["desc"], int(f0), boot[k][0], boot[k][1], P[k], R[k],
                       mx, md)
        ref = oracle.vo_segment(s.K, 480, 640, F["frame_off"], F["uv"], F["desc"], int(f0), int(st), boot[k][0],
                                boot[k][1])
        np.testing.assert_array_equal(R[k]["n_corr"][1:], ref["n_corr"])
        np.testing.assert_array_equal(R[k]["n_new"], ref["n_new"])
        gt = [_se3(P[k][t], F["T_cw"][f0 + t]) for t in range(st + 1)]
        assert max(gt) < (5e-3 if noise == 0 else 5e-2), max(gt)


def test_vo_replay_and_segment_independence(native, monkeypatch):
    """Replays are bit-identical, and a segment's result does not depend on which other segments
    run beside it (one block per segment, no cross-segment state).  Pinned to the serial order;
    test_vo_step_schedules_bit_identical covers the concurrent ones."""
    for k, v in {"PICP_VO_CHAINS": "1", "PICP_VO_OVERLAP": "0"}.items():
        monkeypatch.setenv(k, v)
    from picp_amd.vo_synth import VOSequence
    s = VOSequence(16, obs_per_frame=700, seed=2)
    F = s.frames(0, 16)
    seq = native.VOSequence(F["frame_off"], F["uv"], F["desc"], K=s.K)
    first, steps = np.array([0, 5, 9]), np.array([5, 4, 6])
    boot = np.stack([[F["T_cw"][f], F["T_cw"][f + 1]] for f in first])
    seq.set_segments(first, steps, boot)
    seq.run()
    a = seq.poses()
    m1 = seq.map(1)
    seq.run()
    seq.run()
    b = seq.poses()
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    seq.set_segments(first[1:2], steps[1:2], boot[1:2])
    seq.run()
    np.testing.assert_array_equal(seq.poses()[0], a[1])
    np.testing.assert_array_equal(seq.map(0)[0], m1[0])
    np.testing.assert_array_equal(seq.map(0)[1], m1[1])


def test_vo_graph_and_direct_enqueue_identical(native, monkeypatch):
    """The serial order replayed from its hipGraph and enqueued launch by launch (PICP_VO_GRAPH=0)
    give bit-identical poses, step records and maps, run after run."""
    from picp_amd.vo_synth import VOSequence, segments
    s = VOSequence(1201, obs_per_frame=1200, seed=5)
    F = s.frames(0, 1201)
    first, steps = segments(1201, 40)
    boot = np.stack([[F["T_cw"][f], F["T_cw"][f + 1]] for f in first])

    def run():
        seq = native.VOSequence(F["frame_off"], F["uv"], F["desc"], K=s.K)
        seq.set_segments(first, steps, boot)
        seq.run()
        seq.run()
        out = (seq.poses(), seq.step_records(), [seq.map(k) for k in (0, len(first) // 2, len(first) - 1)])
        seq.close()
        return out

    monkeypatch.setenv("PICP_VO_OVERLAP", "0")
    monkeypatch.setenv("PICP_VO_CHAINS", "1")
    base = run()
    monkeypatch.setenv("PICP_VO_GRAPH", "0")
    other = run()
    for x, y in zip(base[0], other[0]):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(base[1], other[1]):
        for f in ("n_corr", "n_in", "rounds", "n_new"):
            np.testing.assert_array_equal(x[f], y[f])
    for (xa, da), (xb, db) in zip(base[2], other[2]):
        np.testing.assert_array_equal(xa, xb)
        np.testing.assert_array_equal(da, db)


def test_vo_argument_errors(native):
    from picp_amd.vo_synth import VOSequence
    s = VOSequence(6, obs_per_frame=200, seed=1)
    F = s.frames(0, 6)
    seq = native.VOSequence(F["frame_off"], F["uv"], F["desc"], K=s.K)
    boot = np.stack([[F["T_cw"][0], F["T_cw"][1]]])
    with pytest.raises(native.PicpError):
        seq.set_segments([0], [6], boot)  # needs frames 0..6, only 0..5 exist
    with pytest.raises(native.PicpError):
        seq.set_segments([0], [0], boot)
    with pytest.raises(native.PicpError):
        seq.run()  # no segments
    seq.set_segments([0], [5], boot)
    seq.run()
    assert seq.step_records()[0]["n_corr"][1:].min() > 0


def _vo_outputs(native, F, K, first, steps, boot, runs=2):
    seq = native.VOSequence(F["frame_off"], F["uv"], F["desc"], K=K)
    seq.set_segments(first, steps, boot, threshold=THR)
    outs = []
    for _ in range(runs):
        seq.run()
        outs.append((seq.poses(), seq.step_records(), [seq.map(k) for k in range(len(first))]))
    seq.close()
    return outs


def _assert_same_bits(a, b, what):
    for x, y in zip(a[0], b[0]):
        np.testing.assert_array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32), err_msg=what)
    for x, y in zip(a[1], b[1]):
        for f in ("n_corr", "n_in", "rounds", "n_new", "chi_in"):
            np.testing.assert_array_equal(np.asarray(x[f]), np.asarray(y[f]), err_msg=what + " " + f)
    for (xa, da), (xb, db) in zip(a[2], b[2]):
        np.testing.assert_array_equal(xa.view(np.uint32), xb.view(np.uint32), err_msg=what + " map")
        np.testing.assert_array_equal(da, db, err_msg=what + " map descriptors")


def test_vo_step_schedules_bit_identical(native, monkeypatch):
    """The concurrent step schedules -- the frame->next match beside the step chain
    (PICP_VO_OVERLAP=1), two step chains (PICP_VO_CHAINS=2), both -- give the serial order's
    poses, step records and maps bit for bit, run after run; so does the library's default (the
    concurrent schedule, no variable set).  Before the device code was built without packed FP32
    (hipcc_nopk.sh), the matcher's MFMA waves beside the PICP block kernel changed its lanes 48-63
    and this differed in every run."""
    from picp_amd.vo_synth import VOSequence, segments
    s = VOSequence(2001, obs_per_frame=2000, seed=42)
    F = s.frames(0, 2001)
    first, steps = segments(2001, 40)
    rel = [np.linalg.inv(F["T_cw"][f].astype(np.float64)) for f in first]
    boot = np.stack([[np.eye(4), rel[k] @ F["T_cw"][f + 1]] for k, f in enumerate(first)]).astype(np.float32)
    schedules = [{"PICP_VO_OVERLAP": "0", "PICP_VO_CHAINS": "1"}, {"PICP_VO_OVERLAP": "1", "PICP_VO_CHAINS": "1"},
                 {"PICP_VO_OVERLAP": "0", "PICP_VO_CHAINS": "2"}, {"PICP_VO_OVERLAP": "1", "PICP_VO_CHAINS": "2"},
                 {"PICP_VO_OVERLAP": None, "PICP_VO_CHAINS": None}]
    ref = None
    for env in schedules:
        for k, v in env.items():
            if v is None:
                monkeypatch.delenv(k, raising=False)
            else:
                monkeypatch.setenv(k, v)
        outs = _vo_outputs(native, F, s.K, first, steps, boot)
        if ref is None:
            ref = outs[0]
        for o in outs:
            _assert_same_bits(ref, o, str(env))


def _set_env(monkeypatch, env):
    for k, v in env.items():
        if v is None:
            monkeypatch.delenv(k, raising=False)
        else:
            monkeypatch.setenv(k, v)


def test_vo_split_world_match_bit_identical(native, monkeypatch):
    """The world match split by map age (PICP_VO_SPLIT=1, an opt-in schedule; -1: the chains whose
    world match is range-split) -- the early part against the map two appends old on its own
    stream, the late part against the last append's points, merged on the chain -- gives the
    unsplit schedule's poses, step records and maps bit for bit, in the serial order and the
    concurrent schedule, run after run."""
    from picp_amd.vo_synth import VOSequence, segments
    n = 601
    s = VOSequence(n, obs_per_frame=2000, seed=3)
    F = s.frames(0, n)
    first, steps = segments(n, 200)
    rel = [np.linalg.inv(F["T_cw"][f].astype(np.float64)) for f in first]
    boot = np.stack([[np.eye(4), rel[k] @ F["T_cw"][f + 1]] for k, f in enumerate(first)]).astype(np.float32)
    ref = None
    for env in ({"PICP_VO_SPLIT": "0", "PICP_VO_OVERLAP": "0", "PICP_VO_CHAINS": "1"},
                {"PICP_VO_SPLIT": "1", "PICP_VO_OVERLAP": "0", "PICP_VO_CHAINS": "1"},
                {"PICP_VO_SPLIT": "0", "PICP_VO_OVERLAP": None, "PICP_VO_CHAINS": None},
                {"PICP_VO_SPLIT": "1", "PICP_VO_OVERLAP": None, "PICP_VO_CHAINS": None},
                {"PICP_VO_SPLIT": "-1", "PICP_VO_OVERLAP": None, "PICP_VO_CHAINS": None},
                {"PICP_VO_SPLIT": None, "PICP_VO_OVERLAP": None, "PICP_VO_CHAINS": None}):
        _set_env(monkeypatch, env)
        outs = _vo_outputs(native, F, s.K, first, steps, boot)
        if ref is None:
            ref = outs[0]
            assert min(int(r["n_corr"][1:].min()) for r in ref[1]) > 0
        for o in outs:
            _assert_same_bits(ref, o, str(env))


def test_vo_split_world_match_vs_oracle(native, oracle, monkeypatch):
    """The split world match forced on at test size: every step against the oracle (teacher
    forcing), counts exact, as test_vo_synthetic_segments checks the default schedule."""
    monkeypatch.setenv("PICP_VO_SPLIT", "1")
    test_vo_synthetic_segments(native, oracle, 25, 600, 8, 0.0)


@pytest.mark.parametrize("obs", [600, 2000, 2300])
def test_vo_fused_gather_bit_identical(native, monkeypatch, obs):
    """The step's gather inside the PICP block kernel (default; the items reach registers and the
    LDS stage without the SoA planes) gives the separate kernels' poses, step records and maps bit
    for bit, in the serial order and the concurrent schedule.  600 observations per frame:
    one register item per lane and most items in the LDS stage; 2300: four per lane, the rest in
    the stage."""
    from picp_amd.vo_synth import VOSequence, segments
    n = 401
    s = VOSequence(n, obs_per_frame=obs, seed=7)
    F = s.frames(0, n)
    first, steps = segments(n, 40)
    rel = [np.linalg.inv(F["T_cw"][f].astype(np.float64)) for f in first]
    boot = np.stack([[np.eye(4), rel[k] @ F["T_cw"][f + 1]] for k, f in enumerate(first)]).astype(np.float32)
    ref = None
    for env in ({"PICP_VO_FUSE": "0", "PICP_VO_OVERLAP": "0", "PICP_VO_CHAINS": "1"},
                {"PICP_VO_FUSE": "1", "PICP_VO_OVERLAP": "0", "PICP_VO_CHAINS": "1"},
                {"PICP_VO_FUSE": "0", "PICP_VO_OVERLAP": None, "PICP_VO_CHAINS": None},
                {"PICP_VO_FUSE": None, "PICP_VO_OVERLAP": None, "PICP_VO_CHAINS": None}):
        for k, v in env.items():
            if v is None:
                monkeypatch.delenv(k, raising=False)
            else:
                monkeypatch.setenv(k, v)
        outs = _vo_outputs(native, F, s.K, first, steps, boot)
        if ref is None:
            ref = outs[0]
            assert min(int(r["n_corr"][1:].min()) for r in ref[1]) > 0
        for o in outs:
            _assert_same_bits(ref, o, str(env))


def test_block_batch_beside_vo_bit_identical(native, monkeypatch):
    """A block-mode batch (the C4/C5 kernel) solved on its own stream while a VO sequence runs
    its matcher (MFMA) and step kernels beside it gives the bits of its solo run, every rep."""
    from picp_amd import synth
    from picp_amd.vo_synth import VOSequence, segments
    monkeypatch.setenv("PICP_MODE", "block")
    monkeypatch.setenv("PICP_VO_OVERLAP", "1")
    bt = synth.make_batch(250, 1500, base_seed=1000)
    B = native.Batch(np.full(250, 1500))
    B.set_data(bt["xyz"], bt["uv"])
    assert B.info()["mode"] == "block"
    B.set_poses(bt["T_init"])
    B.solve(max_rounds=50, conv_eps=1e-5)
    ref = B.poses().copy()
    s = VOSequence(1201, obs_per_frame=1200, seed=9)
    F = s.frames(0, 1201)
    first, steps = segments(1201, 40)
    boot = np.stack([[F["T_cw"][f], F["T_cw"][f + 1]] for f in first])
    vo = native.VOSequence(F["frame_off"], F["uv"], F["desc"], K=s.K)
    vo.set_segments(first, steps, boot, threshold=THR)
    L = native.lib()
    for _ in range(6):
        B.set_poses(bt["T_init"])
        assert L.picp_vo_run_async(vo._h) == 0
        B.solve_async(max_rounds=50, conv_eps=1e-5)
        B.sync()
        assert L.picp_vo_sync(vo._h) == 0
        np.testing.assert_array_equal(B.poses().view(np.uint32), ref.view(np.uint32))
    vo.close()
    B.close()


def test_vo_segments_querying_one_frame(native, monkeypatch):
    """Two segments that query one frame at the same step would write the same world-match rows
    in one launch: rejected.  Segments that query one frame at different steps run; with two step
    chains whose groups would share that frame the handle runs the serial order, so the result
    equals the serial handle's bit for bit."""
    from picp_amd.vo_synth import VOSequence
    s = VOSequence(14, obs_per_frame=600, seed=4)
    F = s.frames(0, 14)
    boot = lambda fs: np.stack([[F["T_cw"][f], F["T_cw"][f + 1]] for f in fs])  # noqa: E731
    seq = native.VOSequence(F["frame_off"], F["uv"], F["desc"], K=s.K)
    with pytest.raises(native.PicpError):
        seq.set_segments([0, 0], [5, 5], boot([0, 0]))
    # equal first frames that are not adjacent collide too (segment 0 and 2 query frame 2 at
    # step 0); a rejected call leaves the handle's previous segments in place
    seq.set_segments([0, 3], [5, 5], boot([0, 3]), threshold=THR)
    seq.run()
    before = (seq.poses(), seq.step_records(), [seq.map(k) for k in range(2)])
    with pytest.raises(native.PicpError):
        seq.set_segments([1, 0, 1], [4, 4, 4], boot([1, 0, 1]))
    with pytest.raises(native.PicpError):
        seq.set_segments([0, 13], [5, 5], boot([0, 12]))  # out of range
    seq.run()
    _assert_same_bits(before, (seq.poses(), seq.step_records(), [seq.map(k) for k in range(2)]),
                      "after rejected set_segments")
    seq.close()
    first, steps = np.array([0, 3]), np.array([8, 8])  # frames 4..9 queried by both, other steps
    monkeypatch.setenv("PICP_VO_OVERLAP", "0")
    monkeypatch.setenv("PICP_VO_CHAINS", "1")
    ref = _vo_outputs(native, F, s.K, first, steps, boot(first), runs=1)[0]
    monkeypatch.setenv("PICP_VO_CHAINS", "2")
    got = _vo_outputs(native, F, s.K, first, steps, boot(first), runs=1)[0]
    _assert_same_bits(ref, got, "chains=2, shared query frames")
