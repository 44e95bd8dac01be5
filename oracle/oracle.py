"""ctypes binding of the CPU oracle (oracle/picp_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, and only as the checker / the timed CPU baseline.  The product path in
02-visualodometry_amd/ never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libpicp_oracle.so")

MODE_FAITHFUL = 0
MODE_F64 = 1

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


class Lin(ctypes.Structure):
    _fields_ = [("H", ctypes.c_double * 36), ("b", ctypes.c_double * 6),
                ("chi_in", ctypes.c_double), ("chi_out", ctypes.c_double),
                ("n_in", ctypes.c_int32), ("n_projected", ctypes.c_int32)]


class Stats(ctypes.Structure):
    _fields_ = [("chi_in", ctypes.c_float), ("chi_out", ctypes.c_float),
                ("n_in", ctypes.c_int32), ("ok", ctypes.c_int32)]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        i, i64, f = ctypes.c_int, ctypes.c_int64, ctypes.c_float
        L.or_project_point.argtypes = [_f32p, _f32p, i, i, _f32p, _f32p]
        L.or_project_point.restype = i
        L.or_error_and_jacobian.argtypes = [_f32p, _f32p, i, i, _f32p, _f32p, _f32p, _f32p]
        L.or_error_and_jacobian.restype = i
        L.or_linearize.argtypes = [_f32p, _f32p, i, i, _f32p, _f32p, _i32p, i64, f, i, i,
                                   ctypes.POINTER(Lin)]
        L.or_linearize_soa.argtypes = [_f32p, _f32p, i, i, _f32p, _f32p, _f32p, _f32p, _f32p,
                                       i64, f, i, i, ctypes.POINTER(Lin)]
        L.or_v2t_euler.argtypes = [_f32p, _f32p]
        L.or_ldlt_solve6_f.argtypes = [_f32p, _f32p, _f32p]
        L.or_ldlt_solve6_d.argtypes = [_f64p, _f64p, _f64p]
        L.or_one_round.argtypes = [_f32p, _f32p, i, i, _f32p, _f32p, _i32p, i64, f, f, i, i, i,
                                   ctypes.POINTER(Stats)]
        L.or_one_round.restype = i
        L.or_solve.argtypes = [_f32p, _f32p, i, i, _f32p, _f32p, _i32p, i64, f, f, i, i, i, i,
                               f, ctypes.POINTER(Stats), ctypes.POINTER(ctypes.c_int)]
        L.or_solve.restype = i
        L.or_solve_soa.argtypes = [_f32p, _f32p, i, i, _f32p, _f32p, _f32p, _f32p, _f32p, i64,
                                   f, f, i, i, i, i, f, ctypes.POINTER(Stats),
                                   ctypes.POINTER(ctypes.c_int)]
        L.or_solve_soa.restype = i
        L.or_solve_soa_mt.argtypes = [_f32p, _f32p, i, i, _f32p, _f32p, _f32p, _f32p, _f32p, i64,
                                      f, f, i, i, i, i, f, i, ctypes.POINTER(Stats),
                                      ctypes.POINTER(ctypes.c_int)]
        L.or_solve_soa_mt.restype = i
        _u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
        u64, d = ctypes.c_uint64, ctypes.c_double
        L.or_five_point.argtypes = [_f64p, _f64p, _f64p]
        L.or_five_point.restype = i
        L.or_essential_samples.argtypes = [i, i, _i32p]
        L.or_essential_samples.restype = i
        L.or_ransac_update_iters.argtypes = [d, d, i, i]
        L.or_ransac_update_iters.restype = i
        L.or_find_essential.argtypes = [_f32p, _f32p, i, _f64p, d, d, i, _f64p, _i32p, _f64p]
        L.or_find_essential.restype = i
        L.or_decompose_essential.argtypes = [_f64p, _f64p, _f64p, _f64p]
        L.or_recover_pose.argtypes = [_f64p, _f32p, _f32p, i, _f64p, d, _f64p, _f64p, _f64p, _u8p]
        L.or_recover_pose.restype = i
        L.or_triangulate.argtypes = [_f32p, _f32p, _f32p, _f32p, i64, _f32p]
        L.or_projection_matrix.argtypes = [_f32p, _f32p, _f32p]
        L.or_iso_inverse.argtypes = [_f32p, _f32p]
        L.or_match_points.argtypes = [_f32p, i64, _f32p, i64, i, f, f, _i32p, _f32p, _f32p, _i32p]
        L.or_match_points.restype = i64
        L.or_vo_segment.argtypes = [_f32p, i, i, np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS"),
                                    _f32p, _f32p, i, i64, i, _f32p, _f32p, f, i, i, f, _f32p, _i32p,
                                    _i32p, _i32p, _i32p, i64, _f32p, _f32p]
        L.or_vo_segment.restype = i64
        _lib = L
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _pose16(T):
    """4x4 numpy (row, col) -> column-major float[16] (Eigen Isometry3f memory)."""
    return _f32(np.asarray(T, dtype=np.float32).T.reshape(16))


def _pose44(p16):
    return np.asarray(p16, dtype=np.float32).reshape(4, 4).T.copy()


def _k9(K):
    return _f32(np.asarray(K, dtype=np.float32).T.reshape(9))


def project_point(T, K, rows, cols, p):
    out = np.zeros(2, np.float32)
    ok = lib().or_project_point(_pose16(T), _k9(K), rows, cols, _f32(p), out)
    return bool(ok), out


def error_and_jacobian(T, K, rows, cols, p, z):
    e = np.zeros(2, np.float32)
    J = np.zeros(12, np.float32)
    ok = lib().or_error_and_jacobian(_pose16(T), _k9(K), rows, cols, _f32(p), _f32(z), e, J)
    return bool(ok), e, J.reshape(6, 2).T.copy()


def _lin_dict(lin):
    return {"H": np.array(lin.H, np.float64).reshape(6, 6).T.copy(),
            "b": np.array(lin.b, np.float64), "chi_in": lin.chi_in, "chi_out": lin.chi_out,
            "n_in": lin.n_in, "n_projected": lin.n_projected}


def linearize(T, K, rows, cols, world, image, pairs, threshold, keep_outliers=False,
              mode=MODE_F64):
    lin = Lin()
    pairs = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 2)
    lib().or_linearize(_pose16(T), _k9(K), rows, cols, _f32(world).reshape(-1),
                       _f32(image).reshape(-1), pairs.reshape(-1), pairs.shape[0],
                       threshold, int(keep_outliers), mode, ctypes.byref(lin))
    return _lin_dict(lin)


def linearize_soa(T, K, rows, cols, x, y, z, u, v, threshold, keep_outliers=False,
                  mode=MODE_F64):
    lin = Lin()
    lib().or_linearize_soa(_pose16(T), _k9(K), rows, cols, _f32(x), _f32(y), _f32(z),
                           _f32(u), _f32(v), len(x), threshold, int(keep_outliers), mode,
                           ctypes.byref(lin))
    return _lin_dict(lin)


def v2t_euler(v):
    T = np.zeros(16, np.float32)
    lib().or_v2t_euler(_f32(v), T)
    return _pose44(T)


def one_round(T, K, rows, cols, world, image, pairs, threshold, damping=1.0, min_inliers=0,
              keep_outliers=False, mode=MODE_FAITHFUL):
    p = _pose16(T)
    st = Stats()
    pairs = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 2)
    ok = lib().or_one_round(p, _k9(K), rows, cols, _f32(world).reshape(-1),
                            _f32(image).reshape(-1), pairs.reshape(-1), pairs.shape[0],
                            threshold, damping, min_inliers, int(keep_outliers), mode,
                            ctypes.byref(st))
    return bool(ok), _pose44(p), {"chi_in": st.chi_in, "chi_out": st.chi_out, "n_in": st.n_in}


def solve(T, K, rows, cols, world, image, pairs, threshold, damping=1.0, min_inliers=0,
          keep_outliers=False, mode=MODE_F64, max_rounds=50, conv_eps=1e-5):
    p = _pose16(T)
    st = Stats()
    conv = ctypes.c_int(0)
    pairs = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 2)
    rounds = lib().or_solve(p, _k9(K), rows, cols, _f32(world).reshape(-1),
                            _f32(image).reshape(-1), pairs.reshape(-1), pairs.shape[0],
                            threshold, damping, min_inliers, int(keep_outliers), mode,
                            max_rounds, conv_eps, ctypes.byref(st), ctypes.byref(conv))
    return _pose44(p), {"chi_in": st.chi_in, "chi_out": st.chi_out, "n_in": st.n_in,
                        "ok": st.ok, "rounds": rounds, "converged": bool(conv.value)}


def solve_soa(T, K, rows, cols, x, y, z, u, v, threshold, damping=1.0, min_inliers=0,
              keep_outliers=False, mode=MODE_F64, max_rounds=50, conv_eps=1e-5):
    p = _pose16(T)
    st = Stats()
    conv = ctypes.c_int(0)
    rounds = lib().or_solve_soa(p, _k9(K), rows, cols, _f32(x), _f32(y), _f32(z), _f32(u),
                                _f32(v), len(x), threshold, damping, min_inliers,
                                int(keep_outliers), mode, max_rounds, conv_eps,
                                ctypes.byref(st), ctypes.byref(conv))
    return _pose44(p), {"chi_in": st.chi_in, "chi_out": st.chi_out, "n_in": st.n_in,
                        "ok": st.ok, "rounds": rounds, "converged": bool(conv.value)}


def solve_soa_mt(T, K, rows, cols, x, y, z, u, v, threshold, threads, damping=1.0, min_inliers=0,
                 keep_outliers=False, mode=MODE_FAITHFUL, max_rounds=50, conv_eps=1e-5):
    """solve_soa with the linearize as a chunked reduction over `threads` OpenMP threads.
    TIMING ONLY (the all-cores CPU baseline of SURVEY.md §8d): the summation order is not the
    reference's, so tests never use it as the parity oracle."""
    p = _pose16(T)
    st = Stats()
    conv = ctypes.c_int(0)
    rounds = lib().or_solve_soa_mt(p, _k9(K), rows, cols, _f32(x), _f32(y), _f32(z), _f32(u),
                                   _f32(v), len(x), threshold, damping, min_inliers,
                                   int(keep_outliers), mode, max_rounds, conv_eps, int(threads),
                                   ctypes.byref(st), ctypes.byref(conv))
    return _pose44(p), {"chi_in": st.chi_in, "chi_out": st.chi_out, "n_in": st.n_in,
                        "ok": st.ok, "rounds": rounds, "converged": bool(conv.value)}


def five_point(q1, q2):
    """Nister's five-point solver on 5 normalised correspondences -> list of 3x3 E (unit norm)."""
    Es = np.zeros(90, np.float64)
    n = lib().or_five_point(np.ascontiguousarray(q1, np.float64).reshape(-1),
                            np.ascontiguousarray(q2, np.float64).reshape(-1), Es)
    return [Es[9 * k:9 * k + 9].reshape(3, 3) for k in range(n)]


def essential_samples(n, max_iters=1000):
    """OpenCV RANSAC's subsets (its cv::RNG((uint64)-1) stream): (max_iters, 5) indices."""
    idx = np.zeros(5 * max_iters, np.int32)
    lib().or_essential_samples(int(n), int(max_iters), idx)
    return idx.reshape(-1, 5)


def find_essential(p1, p2, K, prob=0.999, threshold=1.0, max_iters=1000):
    """cv::findEssentialMat(p1, p2, K, RANSAC, prob, threshold, max_iters) restated (see
    picp_essential.c): -> (E 3x3 or None, inlier count)."""
    p1 = _f32(p1).reshape(-1, 2)
    p2 = _f32(p2).reshape(-1, 2)
    Kv = np.array([K[0][0], K[1][1], K[0][2], K[1][2]], np.float64)
    E = np.zeros(9, np.float64)
    scratch = np.zeros(4 * max(len(p1), 1), np.float64)
    idx = np.zeros(5 * max(max_iters, 1), np.int32)
    cnt = lib().or_find_essential(p1.reshape(-1), p2.reshape(-1), len(p1), Kv, float(prob), float(threshold),
                                  int(max_iters), scratch, idx, E)
    return (E.reshape(3, 3) if cnt > 0 else None), cnt


def recover_pose(E, p1, p2, K, dist=50.0):
    """cv::recoverPose(E, p1, p2, K, R, t, dist, mask) restated: -> (R 3x3, t (3,), mask bool, count)."""
    p1 = _f32(p1).reshape(-1, 2)
    p2 = _f32(p2).reshape(-1, 2)
    Kv = np.array([K[0][0], K[1][1], K[0][2], K[1][2]], np.float64)
    R = np.zeros(9, np.float64)
    t = np.zeros(3, np.float64)
    mask = np.zeros(max(len(p1), 1), np.uint8)
    scratch = np.zeros(4 * max(len(p1), 1), np.float64)
    cnt = lib().or_recover_pose(np.ascontiguousarray(E, np.float64).reshape(-1), p1.reshape(-1), p2.reshape(-1),
                                len(p1), Kv, float(dist), scratch, R, t, mask)
    return R.reshape(3, 3), t, mask[:len(p1)].astype(bool), cnt


def ldlt_solve6(A, rhs, double=True):
    x = np.zeros(6, np.float64 if double else np.float32)
    if double:
        lib().or_ldlt_solve6_d(np.ascontiguousarray(np.asarray(A, np.float64).T.reshape(36)),
                               np.ascontiguousarray(rhs, np.float64), x)
    else:
        lib().or_ldlt_solve6_f(_f32(np.asarray(A, np.float32).T.reshape(36)), _f32(rhs), x)
    return x


def projection_matrix(K, T_cw):
    P = np.zeros(12, np.float32)
    lib().or_projection_matrix(_k9(K), _pose16(T_cw), P)
    return P.reshape(3, 4)


def triangulate(P1, P2, uv1, uv2):
    uv1 = _f32(uv1).reshape(-1, 2)
    uv2 = _f32(uv2).reshape(-1, 2)
    out = np.zeros((uv1.shape[0], 3), np.float32)
    lib().or_triangulate(_f32(P1).reshape(12), _f32(P2).reshape(12), uv1.reshape(-1),
                         uv2.reshape(-1), uv1.shape[0], out.reshape(-1))
    return out


def match_points(d1, d2, dist_thr=0.2, ratio_thr=0.8):
    """src/my_utilities.h:70-120 -> dict(best_idx, best_dist, second_dist, accepted)."""
    d1 = _f32(d1)
    d2 = _f32(d2)
    n1 = d1.shape[0]
    dim = d1.shape[1] if d1.ndim == 2 else d2.shape[1]
    n2 = d2.shape[0] if d2.size else 0
    bi = np.zeros(n1, np.int32)
    bd = np.zeros(n1, np.float32)
    sd = np.zeros(n1, np.float32)
    acc = np.zeros(n1, np.int32)
    lib().or_match_points(d1.reshape(-1), n1, d2.reshape(-1) if d2.size else np.zeros(1, np.float32), n2,
                          dim, dist_thr, ratio_thr, bi, bd, sd, acc)
    return {"best_idx": bi, "best_dist": bd, "second_dist": sd, "accepted": acc.astype(bool)}


def vo_segment(K, rows, cols, frame_off, uv, desc, f0, steps, T0, T1, threshold=3000.0,
               mode=MODE_F64, max_rounds=50, conv_eps=1e-5, map_cap=None):
    """exec/icp_test.cpp:36-136 over frames [f0, f0+steps] (see picp_oracle.h or_vo_segment).
    T0/T1: camera-in-world bootstrap poses (4x4).  Returns dict(poses (steps+1,4,4) camera-in-world,
    n_corr, n_in, rounds, n_new, map_xyz, map_desc)."""
    frame_off = np.ascontiguousarray(frame_off, np.int64)
    desc = _f32(desc)
    dim = desc.shape[1]
    if map_cap is None:
        map_cap = int(frame_off[f0 + steps + 1] - frame_off[f0])
    poses = np.zeros((steps + 1) * 16, np.float32)
    n_corr = np.zeros(max(steps, 1), np.int32)
    n_in = np.zeros(max(steps, 1), np.int32)
    rounds = np.zeros(max(steps, 1), np.int32)
    n_new = np.zeros(steps + 1, np.int32)
    mx = np.zeros(max(map_cap, 1) * 3, np.float32)
    md = np.zeros(max(map_cap, 1) * dim, np.float32)
    n = lib().or_vo_segment(_k9(K), rows, cols, frame_off, _f32(uv).reshape(-1), desc.reshape(-1), dim,
                            int(f0), int(steps), _pose16(T0), _pose16(T1), threshold, mode, max_rounds,
                            conv_eps, poses, n_corr, n_in, rounds, n_new, map_cap, mx, md)
    if n < 0:
        raise RuntimeError("or_vo_segment: map capacity exceeded")
    return {"poses": np.stack([_pose44(poses[16 * k:16 * k + 16]) for k in range(steps + 1)]),
            "n_corr": n_corr[:steps], "n_in": n_in[:steps], "rounds": rounds[:steps], "n_new": n_new,
            "map_xyz": mx[:3 * n].reshape(-1, 3), "map_desc": md[:dim * n].reshape(-1, dim)}
