"""GPU parity of the VO path at large maps and long segments (VERDICT r04 "What's missing" 1).

The bench line's `c5.partition_8e` runs SURVEY §8e's partition: 8 segments of 1,250 PICP steps,
each map growing to ~1.9e5 landmarks.  test_gpu_vo.py / test_gpu_scale.py stop at 40-step
segments (a few thousand map rows); this file covers the long form at its full size:

* test_vo_8e_segment_teacher_forced_late_steps -- segment 0 of the 8e partition (frames
  0 .. 1,250 of the bench's C5 sequence, seed 42, 2,000 observations per frame) runs on the GPU
  exactly as the bench runs it; at steps 0, 100, 400, 800 and the last, the step is re-run on the
  oracle from the GPU's own inputs (the map is append-only, so the GPU's map prefix and its pose of
  frame t are exactly step t's inputs -- teacher forcing, as test_gpu_vo.py):
    - the world match of frame t+1 against the map prefix: n_corr EXACT (bit-exact matcher);
    - the PICP pose from the GPU's prior, at the GPU's round count, against four correct
      restatements at the same inputs (the oracle in float64 accumulation and in the reference's
      float32 arithmetic summing in three orders).  The rule:
        (1) SE(3) log < 1e-4 (north_star) against the reference's own arithmetic in its own order
            (FAITHFUL: sequential float sums, src/picp_solver.cpp:56-105), camera-in-world;
        (2) against EVERY restatement (the four above and two in the GPU's own arithmetic class:
            float64 sums, float32 H, a float32 or float64 solve), in both pose bases
            (camera-in-world, the trajectory's form;
            world-in-camera, the next step's prior), SE(3) log < max(1e-4, 2 x cloud), where the
            cloud is the largest distance between two restatements in that basis: what float
            rounding alone does to this step's pose.  Late in a long segment the f64-vs-float32
            spread alone exceeds 1e-4 at ill-conditioned steps (H's condition number is printed),
            so a fixed 1e-4 against the f64 restatement would judge the conditioning, not the GPU;
    - the points appended after the step: count and descriptors EXACT, positions vs the oracle's
      DLT within 1e-4 relative for 99 % (test_gpu_vo.py's bar).
  and the GPU matcher (picp_match_points, all three forms) is bit-exact against the oracle's
  match_points on the last step's 2,000 queries x the whole map prefix (~1.9e5 references).
* test_match_2000_x_262144_bit_exact -- the matcher at 2,000 queries x 262,144 references (>=
  2e5, the verdict's bar) with exact duplicates and near-ties, every output bit-exact, all forms.

Drift: the free-running 1,250-step segment leaves ground truth by design (the restated reference
has no loop closure, cheirality or reprojection check); the oracle's own run of the same segment
drifts the same way (tools/r05/oracle_drift.py, profiles/r05/drift/).  The GPU's drift is not
bounded here; each step is, against the oracle, from the GPU's own inputs.
"""
import numpy as np
import pytest

from picp_amd.synth import se3_log_norm

pytestmark = pytest.mark.gpu

THR = 3000.0
POSE_TOL = 1e-4


def _iso_inverse_f32(T):
    """Eigen::Isometry3f::inverse() of a camera-in-world pose in float32, in the order the GPU's
    append computes the next step's prior (picp_vo_device.h vo_iso_inverse, contraction off):
    R^T, and -(R^T t) summed k = 0, 1, 2 with every product and sum rounded to float32."""
    R = np.asarray(T, np.float32)[:3, :3]
    t = np.asarray(T, np.float32)[:3, 3]
    out = np.eye(4, dtype=np.float32)
    out[:3, :3] = R.T
    for i in range(3):
        s = np.float32(R[0, i] * t[0])
        s = np.float32(s + np.float32(R[1, i] * t[1]))
        s = np.float32(s + np.float32(R[2, i] * t[2]))
        out[i, 3] = -s
    return out


def _mixed_solve(oracle, T0, K, world, img, pairs, rounds, f32_solve):
    """The GPU's arithmetic class as a restatement: each round's H and b summed in float64 from the
    float32 per-correspondence terms (oracle MODE_F64 linearize, src/picp_solver.cpp:56-91), rounded
    to float32 with the damping added (:96), then solved in float32 by the Eigen-LDLT restatement
    (f32_solve) or in float64 from those float32 values, and T <- v2tEuler(dx) * T in float32
    (:102-103).  The oracle's two modes vary the summation only (FAITHFUL: float32 sums and solve,
    F64: float64 sums and solve); these two vary the solve's precision around float64 sums, which
    is what the GPU does (double partials, float32 LDL^T)."""
    T = np.asarray(T0, np.float32).copy()
    for _ in range(rounds):
        lin = oracle.linearize(T, K, 480, 640, world, img, pairs, THR, mode=oracle.MODE_F64)
        H = (np.asarray(lin["H"], np.float64) + np.eye(6)).astype(np.float32)
        b = np.asarray(lin["b"], np.float64).astype(np.float32)
        if f32_solve:
            dx = np.asarray(oracle.ldlt_solve6(H, -b, double=False), np.float32)
        else:
            dx = np.linalg.solve(H.astype(np.float64), -b.astype(np.float64)).astype(np.float32)
        T = (oracle.v2t_euler(dx).astype(np.float32) @ T).astype(np.float32)
    return T


def _cw_dist(T, P):
    """SE(3) distance of a solve's world-in-camera result T to the GPU's camera-in-world pose P, in
    the camera-in-world form the trajectory is kept in: T is inverted exactly as the GPU inverts
    its own result (_iso_inverse_f32), so both sides are the same function of their solve's output.
    (Inverting P back instead is not exact: a float32 rotation chained over 1,250 steps is ~5e-5
    from orthonormal, and R^T or a float64 inverse of P would read that as pose error.)"""
    from picp_amd.synth import se3_log_norm
    return se3_log_norm(_iso_inverse_f32(T), P)


@pytest.fixture(scope="module")
def segment_8e(native):
    """The GPU run of the 8e partition's segment 0, bootstrapped as bench.py does."""
    from picp_amd.vo_synth import VOSequence, segments
    first, steps = segments(10000, -(-(10000 - 1) // 8))
    S = int(steps[0])
    seq = VOSequence(S + 2, obs_per_frame=2000, seed=42)
    D = seq.frames(0, S + 1)
    rel = np.linalg.inv(D["T_cw"][0].astype(np.float64))
    boot = np.stack([[np.eye(4), rel @ D["T_cw"][1]]]).astype(np.float32)
    vo = native.VOSequence(D["frame_off"], D["uv"], D["desc"], K=seq.K)
    vo.set_segments([0], [S], boot, threshold=THR)
    vo.run()
    P, R = vo.poses()[0], vo.step_records()[0]
    mx, md = vo.map(0)
    vo.close()
    return dict(K=seq.K, D=D, rel=rel, S=S, P=P, R=R, mx=mx, md=md)


def test_8e_segment_is_the_bench_partition(segment_8e):
    # bench.py: c5.partition_8e = segments(10000, ceil(9999 / 8)) -> 8 segments of 1,250 steps
    from picp_amd.vo_synth import segments
    first, steps = segments(10000, -(-(10000 - 1) // 8))
    assert len(first) == 8 and int(steps[0]) == segment_8e["S"] == 1250
    R = segment_8e["R"]
    m = np.cumsum(R["n_new"])
    assert m[-1] == len(segment_8e["mx"]) > 150000  # the map the late steps match against
    assert R["n_corr"][1:].min() > 1000  # tracking is never lost


@pytest.mark.parametrize("t", [0, 100, 400, 800, 1249])
def test_vo_8e_segment_teacher_forced_late_steps(oracle, segment_8e, t):
    g = segment_8e
    K, D, P, R, mx, md = g["K"], g["D"], g["P"], g["R"], g["mx"], g["md"]
    off, uv, desc = D["frame_off"], D["uv"], D["desc"]
    m = int(np.sum(R["n_new"][:t + 1]))  # the map step t matched against (bootstrap + steps < t)
    cf, nf = t, t + 1
    dn = desc[off[nf]:off[nf + 1]]
    wm = oracle.match_points(dn, md[:m])
    assert int(wm["accepted"].sum()) == int(R["n_corr"][t + 1])
    pairs = np.stack([np.nonzero(wm["accepted"])[0], wm["best_idx"][wm["accepted"]]], 1).astype(np.int32)
    # the step's prior exactly as the GPU formed it: the float32 inverse of its pose of frame t
    # (exec/icp_test.cpp:77-78, Isometry3f::inverse: R^T).  Late in the segment P's rotation is
    # ~5e-5 from orthonormal, so a float64 inverse of P would differ from this prior by ~1e-3 in
    # translation and would not be this step's input.
    T0 = _iso_inverse_f32(P[t])
    img = uv[off[nf]:off[nf + 1]]
    gr = int(R["rounds"][t + 1])
    # The icp_test convergence test (relative chi change < 1e-5, exec/icp_test.cpp:99-106) fires at
    # the float noise floor, where the GPU's tree-ordered sums and the oracle's sequential ones
    # differ in the last bits: the two may stop a few rounds apart (as in the C4 converged test).
    # The round count is then teacher-forced too: the oracle runs exactly the GPU's rounds, in
    # float64 accumulation and in the reference's float32 arithmetic (FAITHFUL: sequential float
    # sums, float LDL^T) with the correspondences in their order, reversed and in a seeded random
    # order, and in the GPU's arithmetic class (float64 sums, float32 H, the solve in float32 or
    # float64: _mixed_solve).  Every one of them is a correct restatement; their spread (the
    # "cloud") is what float rounding alone does to this step's pose, printed beside the GPU's
    # distance to each.  (Measured on the round-6 dump: in world-in-camera form the summation-order
    # variants alone spread 1.8e-4 at step 1,249 while the solve-precision variants move the pose by
    # up to 5e-4 at step 800 -- the 28 m lever arm on a 1e-5 rotation -- so a cloud of summation
    # orders alone under-states float rounding there; profiles/r06/parity/.)
    variants = {}
    for name, mode, order in (("f64", oracle.MODE_F64, None), ("faithful", oracle.MODE_FAITHFUL, None),
                              ("faithful-rev", oracle.MODE_FAITHFUL, np.arange(len(pairs))[::-1]),
                              ("faithful-perm", oracle.MODE_FAITHFUL, np.random.default_rng(t).permutation(len(pairs)))):
        pp = pairs if order is None else np.ascontiguousarray(pairs[order])
        variants[name], _ = oracle.solve(T0, K, 480, 640, mx[:m], img, pp, THR, max_rounds=gr, conv_eps=-1.0,
                                         mode=mode)
    variants["f64sum-f32solve"] = _mixed_solve(oracle, T0, K, mx[:m], img, pairs, gr, True)
    variants["f64sum-f64solve"] = _mixed_solve(oracle, T0, K, mx[:m], img, pairs, gr, False)
    gpu_to = {k: _cw_dist(v, P[t + 1]) for k, v in variants.items()}
    names = list(variants)
    cloud = max(se3_log_norm(_iso_inverse_f32(variants[a]), _iso_inverse_f32(variants[b]))
                for i, a in enumerate(names) for b in names[i + 1:])
    # world-in-camera: the next step's prior, as each side would form it from its camera-in-world
    # pose (the GPU's append: Isometry3f::inverse of P[t+1]; a restatement: the same inverse of
    # its own camera-in-world pose), so both sides are again the same function of their solve's
    # output.  A 5e-5 departure from orthonormality times the camera's ~28 m distance from the
    # segment origin makes this basis ~10x more sensitive than camera-in-world late in the segment.
    wc = {k: _iso_inverse_f32(_iso_inverse_f32(v)) for k, v in variants.items()}
    gpu_wc = _iso_inverse_f32(P[t + 1])
    gpu_to_wc = {k: se3_log_norm(v, gpu_wc) for k, v in wc.items()}
    cloud_wc = max(se3_log_norm(wc[a], wc[b]) for i, a in enumerate(names) for b in names[i + 1:])
    # the conditioning of the step: H (src/picp_solver.cpp:56-91) at the f64 restatement's pose
    lin = oracle.linearize(variants["f64"], K, 480, 640, mx[:m], img, pairs, THR, mode=oracle.MODE_F64)
    cond = float(np.linalg.cond(np.asarray(lin["H"], np.float64) + np.eye(6)))  # + damping (:96)
    # the oracle run free (its own convergence test) lands within a few rounds of the GPU's
    Tfree, st = oracle.solve(T0, K, 480, 640, mx[:m], img, pairs, THR)
    err_free = _cw_dist(Tfree, P[t + 1])
    print("step %d: map %d, n_corr %d, GPU rounds %d (converged %d), oracle free rounds %d; cond(H) %.3g; at the "
          "GPU's rounds, camera-in-world: GPU vs %s, cloud %.3g; world-in-camera: GPU vs %s, cloud %.3g; free GPU vs "
          "f64 %.3g; chi_in GPU %.6g" % (
              t, m, len(pairs), gr, int(R["converged"][t + 1]), st["rounds"], cond,
              ", ".join("%s %.3g" % kv for kv in gpu_to.items()), cloud,
              ", ".join("%s %.3g" % kv for kv in gpu_to_wc.items()), cloud_wc, err_free, float(R["chi_in"][t + 1])))
    # (1) the reference's own float32 arithmetic, in its order, camera-in-world: north_star's 1e-4
    assert gpu_to["faithful"] < POSE_TOL, (t, gpu_to, cloud)
    # (2) every restatement, both bases, within the rounding cloud of that basis (at least 1e-4)
    for basis, d, c in (("camera-in-world", gpu_to, cloud), ("world-in-camera", gpu_to_wc, cloud_wc)):
        bar = max(POSE_TOL, 2.0 * c)
        assert max(d.values()) < bar, (t, basis, d, c, bar)
    assert abs(gr - st["rounds"]) <= 5 or err_free < POSE_TOL, (t, gr, st["rounds"], err_free)
    # the append after step t: add_new_world_points + DLT with (pose t, pose t+1)
    pm = oracle.match_points(desc[off[cf]:off[cf + 1]], dn)
    sel = pm["accepted"].copy()
    sel[sel] &= ~wm["accepted"][pm["best_idx"][sel]]
    ia = np.nonzero(sel)[0]
    ib = pm["best_idx"][ia]
    assert len(ia) == int(R["n_new"][t + 1])
    np.testing.assert_array_equal(md[m:m + len(ia)], desc[off[cf]:off[cf + 1]][ia])
    if not len(ia):  # step 0: every frame-1 point is already in the bootstrap map
        return
    X = oracle.triangulate(oracle.projection_matrix(K, P[t]), oracle.projection_matrix(K, P[t + 1]),
                           uv[off[cf]:off[cf + 1]][ia], uv[off[nf]:off[nf + 1]][ib])
    rel = np.abs(mx[m:m + len(ia)] - X).max(1) / (1.0 + np.abs(X).max(1))
    assert np.quantile(rel, 0.99) < 1e-4 and rel.max() < 1e-2, (t, np.quantile(rel, 0.99), rel.max())


@pytest.mark.parametrize("form", ["full", "exact", "accept_only"])
def test_vo_8e_last_step_world_match_bit_exact(native, oracle, segment_8e, form):
    """The GPU matcher on the last step's queries against the whole map prefix it matched."""
    g = segment_8e
    R, md, D = g["R"], g["md"], g["D"]
    t = g["S"] - 1
    m = int(np.sum(R["n_new"][:t + 1]))
    assert m > 150000
    off, desc = D["frame_off"], D["desc"]
    dn = desc[off[t + 1]:off[t + 2]]
    ref = oracle.match_points(dn, md[:m])
    _check_match(native, dn, md[:m], ref, form)


def _check_match(native, q, r, ref, form):
    got = native.match_points_batch([q], [r], form=form)[0]
    acc = ref["accepted"]
    np.testing.assert_array_equal(got["accepted"].astype(bool), acc)
    np.testing.assert_array_equal(got["best_idx"][acc], ref["best_idx"][acc])
    np.testing.assert_array_equal(got["best_dist"][acc].view(np.uint32), ref["best_dist"][acc].view(np.uint32))
    if form != "accept_only":  # every output exact for every query
        np.testing.assert_array_equal(got["best_idx"], ref["best_idx"])
        np.testing.assert_array_equal(got["best_dist"].view(np.uint32), ref["best_dist"].view(np.uint32))
        np.testing.assert_array_equal(got["second_dist"].view(np.uint32), ref["second_dist"].view(np.uint32))


@pytest.mark.parametrize("form", ["full", "exact", "accept_only"])
def test_match_2000_x_262144_bit_exact(native, oracle, form):
    """2,000 queries x 262,144 references (> 2e5), 10-d descriptors U[-1, 1] as the reference's
    data: half the queries are exact copies of a reference (distance 0), a quarter of those copied
    twice into the reference set (best = second = 0: the reference's ratio test gives NaN -> reject,
    and the first index wins), the rest near-copies at 1e-3..1e-2 (accepted or ratio-rejected), plus
    far queries (rejected by the 0.2 threshold)."""
    rng = np.random.default_rng(2026)
    n_r, n_q, dim = 262144, 2000, 10
    r = rng.uniform(-1, 1, (n_r, dim)).astype(np.float32)
    q = rng.uniform(-1, 1, (n_q, dim)).astype(np.float32)
    src = rng.choice(n_r, n_q, replace=False)
    q[:1000] = r[src[:1000]]
    r[src[1750:2000]] = r[src[1500:1750]]          # duplicates of the copied rows at other indices
    q[1500:1750] = r[src[1500:1750]]
    q[1000:1500] = r[src[1000:1500]] + rng.uniform(-1e-2, 1e-2, (500, dim)).astype(np.float32)
    ref = oracle.match_points(q, r)
    assert ref["accepted"].sum() > 500 and (~ref["accepted"]).sum() > 400
    _check_match(native, q, r, ref, form)
