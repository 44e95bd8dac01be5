"""picp_amd -- Python binding of libpicp_amd.so (the MI355X PICP hot path, include/picp_c.h).

Thin ctypes layer used by the tests, bench.py and __graft_entry__; the product itself is the
C-ABI library and the C++ facade (include/pr/*.h).  There is deliberately no CPU fallback:
if the native library is missing or no HIP device is present, every compute call raises.

Mirrors the reference interface (llepa/02-VisualOdometry):
  * PICPSolver  -- pr::PICPSolver (src/picp_solver.h:21-82): init / oneRound /
                   setKernelThreshold / chiInliers / chiOutliers / numInliers / camera pose,
                   plus solve() = the exec/icp_test.cpp:88-107 loop fused on the device.
  * Batch       -- independent frames solved together on one device (the batch split).
  * triangulate -- Cam::triangulatePoints' DLT (src/cam.cpp:94-140).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
# PICP_LIB selects a diagnostic build (tools/stamps.py); the default is the shipped library
LIB_PATH = os.environ.get("PICP_LIB") or os.path.join(PKG_ROOT, "lib", "libpicp_amd.so")

OK = 0
ERR_ARG = -1
ERR_DEVICE = -2
ERR_RANGE = -3
ERR_STATE = -4
ERR_NOMEM = -5
TOO_FEW_INLIERS = 1

K_REF = np.array([[180, 0, 320], [0, 180, 240], [0, 0, 1]], np.float32)  # src/cam.cpp:11-16

# every symbol include/picp_c.h declares (tests check the library exports all of them)
EXPORTED = [
    "picp_params_default", "picp_abi_version", "picp_last_error", "picp_device_count",
    "picp_create", "picp_destroy", "picp_set_camera", "picp_clone", "picp_set_points",
    "picp_set_correspondences", "picp_set_pose", "picp_get_pose", "picp_one_round",
    "picp_solve", "picp_linearize", "picp_batch_create", "picp_batch_destroy",
    "picp_batch_set_data", "picp_batch_set_data_device", "picp_batch_set_poses",
    "picp_batch_get_poses", "picp_batch_get_stats", "picp_batch_solve",
    "picp_batch_solve_async", "picp_batch_sync", "picp_batch_time", "picp_batch_time_single",
    "picp_batch_info", "picp_batch_residency",
    "picp_triangulate", "picp_projection_matrix", "picp_match", "picp_match_batch", "picp_match_batch_form",
    "picp_vo_create", "picp_vo_destroy", "picp_vo_set_segments", "picp_vo_run", "picp_vo_run_async", "picp_vo_debug_matches", "picp_vo_debug_guard",
    "picp_vo_sync", "picp_vo_get_poses", "picp_vo_get_steps", "picp_vo_get_map", "picp_vo_time",
    "picp_vo_info", "picp_selftest_rcp", "picp_essential_params_default", "picp_essential_batch",
    "picp_shard_range", "picp_shard_pad", "picp_shard_unpack", "picp_comm_unique_id", "picp_comm_create", "picp_comm_destroy", "picp_comm_info",
    "picp_comm_allreduce_max", "picp_comm_barrier", "picp_batch_allgather", "picp_batch_allgather_host",
]
COMM_ID_BYTES = 128


class PicpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("picp error %d: %s" % (code, msg))
        self.code = code


class Stats(ctypes.Structure):
    _fields_ = [("chi_in", ctypes.c_float), ("chi_out", ctypes.c_float),
                ("n_in", ctypes.c_int32), ("ok", ctypes.c_int32), ("rounds", ctypes.c_int32),
                ("converged", ctypes.c_int32), ("n_projected", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved"}


class VOStep(ctypes.Structure):
    _fields_ = [("n_corr", ctypes.c_int32), ("n_in", ctypes.c_int32), ("rounds", ctypes.c_int32),
                ("n_new", ctypes.c_int32), ("chi_in", ctypes.c_float), ("chi_out", ctypes.c_float),
                ("converged", ctypes.c_int32), ("n_projected", ctypes.c_int32)]


class Params(ctypes.Structure):
    _fields_ = [("threshold", ctypes.c_float), ("damping", ctypes.c_float),
                ("min_inliers", ctypes.c_int32), ("keep_outliers", ctypes.c_int32),
                ("max_rounds", ctypes.c_int32), ("conv_eps", ctypes.c_float)]


_lib = None
# picp_exchange_fn (include/picp_c.h): int (*)(void* user, const void* send, void* recv, size_t bytes)
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-j8", "-C", PKG_ROOT])


def lib():
    """Load libpicp_amd.so (fails loudly if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PicpError(ERR_STATE, "native library %s missing: run `make -C %s`" % (LIB_PATH, PKG_ROOT))
    L = ctypes.CDLL(LIB_PATH)
    vp, i, i64, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
    fp = ctypes.POINTER(ctypes.c_float)
    dp = ctypes.POINTER(ctypes.c_double)
    sp = ctypes.POINTER(Stats)
    pp = ctypes.POINTER(Params)
    sig = {
        "picp_params_default": ([pp], None),
        "picp_abi_version": ([], i),
        "picp_last_error": ([], ctypes.c_char_p),
        "picp_device_count": ([ctypes.POINTER(i)], i),
        "picp_create": ([ctypes.POINTER(vp), i, i, i, fp], i),
        "picp_destroy": ([vp], i),
        "picp_set_camera": ([vp, i, i, fp], i),
        "picp_clone": ([vp, ctypes.POINTER(vp)], i),
        "picp_set_points": ([vp, fp, i64, fp, i64], i),
        "picp_set_correspondences": ([vp, ctypes.POINTER(ctypes.c_int32), i64], i),
        "picp_set_pose": ([vp, fp], i),
        "picp_get_pose": ([vp, fp], i),
        "picp_one_round": ([vp, f, f, i, i, sp], i),
        "picp_solve": ([vp, pp, sp], i),
        "picp_linearize": ([vp, f, i, dp, dp, sp], i),
        "picp_batch_create": ([ctypes.POINTER(vp), i, i, ctypes.POINTER(i64), i, i, fp], i),
        "picp_batch_destroy": ([vp], i),
        "picp_batch_set_data": ([vp, fp, fp], i),
        "picp_batch_set_data_device": ([vp, vp, vp, vp, vp, vp], i),
        "picp_batch_set_poses": ([vp, fp], i),
        "picp_batch_get_poses": ([vp, fp], i),
        "picp_batch_get_stats": ([vp, sp], i),
        "picp_batch_solve": ([vp, pp], i),
        "picp_batch_solve_async": ([vp, pp], i),
        "picp_batch_sync": ([vp], i),
        "picp_batch_time": ([vp, pp, i, fp, fp], i),
        "picp_batch_time_single": ([vp, pp, fp], i),
        "picp_batch_residency": ([vp, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(i)], i),
        "picp_batch_info": ([vp, ctypes.POINTER(i64), ctypes.POINTER(i), ctypes.POINTER(i)], i),
        "picp_triangulate": ([i, fp, fp, fp, fp, i64, fp], i),
        "picp_projection_matrix": ([fp, fp, fp], i),
        "picp_match": ([i, fp, i64, fp, i64, i, f, f, ctypes.POINTER(ctypes.c_int32), fp, fp,
                        ctypes.POINTER(ctypes.c_int32)], i),
        "picp_match_batch": ([i, i, ctypes.POINTER(i64), ctypes.POINTER(i64), fp, fp, i, f, f,
                              ctypes.POINTER(ctypes.c_int32), fp, fp, ctypes.POINTER(ctypes.c_int32)], i),
        "picp_match_batch_form": ([i, i, ctypes.POINTER(i64), ctypes.POINTER(i64), fp, fp, i, f, f,
                                   ctypes.POINTER(ctypes.c_int32), fp, fp, ctypes.POINTER(ctypes.c_int32), i], i),
        "picp_vo_create": ([ctypes.POINTER(vp), i, i, i, fp, i64, ctypes.POINTER(i64), fp, fp, i], i),
        "picp_vo_destroy": ([vp], i),
        "picp_vo_set_segments": ([vp, i, ctypes.POINTER(i64), ctypes.POINTER(ctypes.c_int32), fp, pp], i),
        "picp_vo_run": ([vp], i),
        "picp_vo_run_async": ([vp], i),
        "picp_vo_debug_matches": ([vp, i, ctypes.POINTER(ctypes.c_int32)], i),
        "picp_vo_debug_guard": ([vp, ctypes.POINTER(i64), ctypes.POINTER(i)], i),
        "picp_vo_sync": ([vp], i),
        "picp_vo_get_poses": ([vp, fp], i),
        "picp_vo_get_steps": ([vp, ctypes.POINTER(VOStep)], i),
        "picp_vo_get_map": ([vp, i, i64, fp, fp, ctypes.POINTER(i64)], i),
        "picp_vo_time": ([vp, i, fp], i),
        "picp_selftest_rcp": ([i, i, i, ctypes.POINTER(ctypes.c_uint64)], i),
        "picp_vo_info": ([vp, ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(i)], i),
        "picp_shard_range": ([i64, i, i, ctypes.POINTER(i64), ctypes.POINTER(i64)], i),
        "picp_shard_pad": ([i64, i], i64),
        "picp_shard_unpack": ([i64, i, i64, vp, vp], i),
        "picp_comm_unique_id": ([ctypes.POINTER(ctypes.c_uint8)], i),
        "picp_comm_create": ([ctypes.POINTER(vp), i, i, i, ctypes.POINTER(ctypes.c_uint8)], i),
        "picp_comm_destroy": ([vp], i),
        "picp_comm_info": ([vp, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(i)], i),
        "picp_comm_allreduce_max": ([vp, dp, i], i),
        "picp_comm_barrier": ([vp], i),
        "picp_batch_allgather": ([vp, vp, i64, fp, sp], i),
        "picp_batch_allgather_host": ([vp, i, i, EXCHANGE_FN, vp, i64, fp, sp], i),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def _check(rc, allow=()):
    if rc != OK and rc not in allow:
        raise PicpError(rc, lib().picp_last_error().decode(errors="replace"))
    return rc


def _fptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _f32(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a if shape is None else a.reshape(shape)


def pose_to_c(T):
    """4x4 (row, col) -> column-major float[16] (Eigen::Isometry3f memory)."""
    return np.ascontiguousarray(np.asarray(T, np.float32).T.reshape(16))


def pose_from_c(p16):
    return np.asarray(p16, np.float32).reshape(4, 4).T.copy()


def k_to_c(K):
    return np.ascontiguousarray(np.asarray(K, np.float32).T.reshape(9))


def device_count():
    n = ctypes.c_int(0)
    _check(lib().picp_device_count(ctypes.byref(n)))
    return n.value


def default_params(**kw):
    p = Params()
    lib().picp_params_default(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class PICPSolver:
    """pr::PICPSolver over the C-ABI (src/picp_solver.h:21-82).

    init(camera, world_points, image_points) copies the arrays to the device (the reference
    keeps raw pointers, src/picp_solver.cpp:21-22).  Correspondences are (image idx, world idx)
    pairs (src/picp_solver.cpp:65-66)."""

    def __init__(self, device=0, rows=480, cols=640, K=K_REF):
        self._h = ctypes.c_void_p()
        self.device = device
        _check(lib().picp_create(ctypes.byref(self._h), device, rows, cols, _fptr(k_to_c(K))))
        self._threshold = 1000.0  # src/picp_solver.cpp:14
        self._damping = 1.0       # src/picp_solver.cpp:11
        self._min_inliers = 0     # src/picp_solver.cpp:12
        self._stats = Stats()

    def close(self):
        if self._h:
            lib().picp_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- reference surface -------------------------------------------------------------
    def init(self, T_wc, world_points, image_points, rows=None, cols=None, K=None):
        if rows is not None:
            _check(lib().picp_set_camera(self._h, rows, cols, _fptr(k_to_c(K))))
        w = _f32(world_points, (-1,))
        im = _f32(image_points, (-1,))
        _check(lib().picp_set_points(self._h, _fptr(w), w.size // 3, _fptr(im), im.size // 2))
        self.set_pose(T_wc)

    def kernelThreshold(self):
        return self._threshold

    def setKernelThreshold(self, t):
        self._threshold = float(t)

    def chiInliers(self):
        return self._stats.chi_in

    def chiOutliers(self):
        return self._stats.chi_out

    def numInliers(self):
        return self._stats.n_in

    def set_pose(self, T_wc):
        _check(lib().picp_set_pose(self._h, _fptr(pose_to_c(T_wc))))

    def pose(self):
        out = np.zeros(16, np.float32)
        _check(lib().picp_get_pose(self._h, _fptr(out)))
        return pose_from_c(out)

    def set_correspondences(self, pairs):
        pr = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
        _check(lib().picp_set_correspondences(
            self._h, pr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), pr.shape[0]))

    def oneRound(self, correspondences, keep_outliers=False):
        """Returns the reference's bool (False when n_in < min_inliers)."""
        self.set_correspondences(correspondences)
        rc = _check(lib().picp_one_round(self._h, self._threshold, self._damping,
                                         self._min_inliers, int(keep_outliers),
                                         ctypes.byref(self._stats)), allow=(TOO_FEW_INLIERS,))
        return rc == OK

    # --- extensions ----------------------------------------------------------------------
    def solve(self, correspondences, max_rounds=50, conv_eps=1e-5, keep_outliers=False):
        """exec/icp_test.cpp:88-107 fused on the device.  Returns stats dict."""
        self.set_correspondences(correspondences)
        prm = default_params(threshold=self._threshold, damping=self._damping,
                             min_inliers=self._min_inliers, keep_outliers=int(keep_outliers),
                             max_rounds=max_rounds, conv_eps=conv_eps)
        _check(lib().picp_solve(self._h, ctypes.byref(prm), ctypes.byref(self._stats)))
        return self._stats.as_dict()

    def linearize(self, correspondences, keep_outliers=False):
        self.set_correspondences(correspondences)
        H = np.zeros(36, np.float64)
        b = np.zeros(6, np.float64)
        st = Stats()
        _check(lib().picp_linearize(self._h, self._threshold, int(keep_outliers),
                                    H.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                    b.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                    ctypes.byref(st)))
        return {"H": H.reshape(6, 6).T.copy(), "b": b, **st.as_dict()}


class Batch:
    """Independent PICP problems (frames) solved together on one device."""

    def __init__(self, sizes, device=0, rows=480, cols=640, K=K_REF):
        sizes = np.asarray(sizes, np.int64)
        offs = np.zeros(len(sizes) + 1, np.int64)
        offs[1:] = np.cumsum(sizes)
        self.offs = offs
        self.n = len(sizes)
        self.device = device
        self._b = ctypes.c_void_p()
        _check(lib().picp_batch_create(ctypes.byref(self._b), device, self.n,
                                       offs.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                       rows, cols, _fptr(k_to_c(K))))

    def close(self):
        if self._b:
            lib().picp_batch_destroy(self._b)
            self._b = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_data(self, xyz, uv):
        xyz = _f32(xyz, (-1,))
        uv = _f32(uv, (-1,))
        assert xyz.size == 3 * self.offs[-1] and uv.size == 2 * self.offs[-1]
        _check(lib().picp_batch_set_data(self._b, _fptr(xyz), _fptr(uv)))

    def set_poses(self, Ts):
        Ts = np.asarray(Ts, np.float32).reshape(self.n, 4, 4)
        flat = np.ascontiguousarray(np.transpose(Ts, (0, 2, 1)).reshape(-1))
        _check(lib().picp_batch_set_poses(self._b, _fptr(flat)))

    def poses(self):
        out = np.zeros(16 * self.n, np.float32)
        _check(lib().picp_batch_get_poses(self._b, _fptr(out)))
        return np.transpose(out.reshape(self.n, 4, 4), (0, 2, 1)).copy()

    def stats(self):
        st = (Stats * self.n)()
        _check(lib().picp_batch_get_stats(self._b, st))
        return [s.as_dict() for s in st]

    def solve(self, **params):
        prm = default_params(**params)
        _check(lib().picp_batch_solve(self._b, ctypes.byref(prm)))

    def solve_async(self, **params):
        prm = default_params(**params)
        _check(lib().picp_batch_solve_async(self._b, ctypes.byref(prm)))

    def sync(self):
        _check(lib().picp_batch_sync(self._b))

    def time(self, reps, **params):
        """reps back-to-back solves between two HIP events -> (total ms, mean launch period us)."""
        prm = default_params(**params)
        total = ctypes.c_float(0)
        lus = ctypes.c_float(0)
        _check(lib().picp_batch_time(self._b, ctypes.byref(prm), reps, ctypes.byref(total), ctypes.byref(lus)))
        return total.value, lus.value

    def time_single(self, **params):
        """Diagnostic: event pair around each launch of one solve (us; graph mode: per round)."""
        prm = default_params(**params)
        us = ctypes.c_float(0)
        _check(lib().picp_batch_time_single(self._b, ctypes.byref(prm), ctypes.byref(us)))
        return us.value

    def residency(self):
        g, r, f = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
        _check(lib().picp_batch_residency(self._b, ctypes.byref(g), ctypes.byref(r), ctypes.byref(f)))
        return {"handoff_grid": g.value, "resident_blocks": r.value, "fallbacks": f.value}

    def info(self):
        tot = ctypes.c_int64(0)
        nb = ctypes.c_int(0)
        mode = ctypes.c_int(0)
        _check(lib().picp_batch_info(self._b, ctypes.byref(tot), ctypes.byref(nb), ctypes.byref(mode)))
        return {"total_corr": tot.value, "n_blocks": nb.value,
                "mode": {0: "graph", 1: "persistent", 2: "block"}[mode.value]}


def shard_range(n_items, world, rank):
    """picp_shard_range: the contiguous [first, last) of n_items that rank owns."""
    a, e = ctypes.c_int64(0), ctypes.c_int64(0)
    _check(lib().picp_shard_range(n_items, world, rank, ctypes.byref(a), ctypes.byref(e)))
    return a.value, e.value


def shard_pad(n_items, world):
    """picp_shard_pad: rows per rank in the padded all-gather (ceil(n_items / world))."""
    r = lib().picp_shard_pad(n_items, world)
    if r < 0:
        raise PicpError(ERR_ARG, "picp_shard_pad: bad size")
    return int(r)


def shard_unpack(padded, n_items, world):
    """picp_shard_unpack: the (world * pad, ...) rank-ordered padded rows -> (n_items, ...) in
    problem order (host code: no device needed)."""
    padded = np.ascontiguousarray(padded)
    pad = shard_pad(n_items, world)
    assert padded.shape[0] == world * max(pad, 1) or (n_items == 0), "padded buffer has the wrong row count"
    row = padded.dtype.itemsize * int(np.prod(padded.shape[1:], dtype=np.int64))
    out = np.empty((n_items,) + padded.shape[1:], padded.dtype)
    _check(lib().picp_shard_unpack(n_items, world, row, padded.ctypes.data_as(ctypes.c_void_p),
                                   out.ctypes.data_as(ctypes.c_void_p)))
    return out


def comm_unique_id():
    """RCCL unique id (bytes) for Comm; rank 0 makes it, the launcher passes it to every rank."""
    buf = (ctypes.c_uint8 * COMM_ID_BYTES)()
    _check(lib().picp_comm_unique_id(buf))
    return bytes(buf)


class Comm:
    """picp_comm_t: this rank's RCCL communicator of the batch split, driven by the C++ library."""

    def __init__(self, device, world, rank, uid):
        assert len(uid) == COMM_ID_BYTES
        self._c = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        _check(lib().picp_comm_create(ctypes.byref(self._c), device, world, rank, buf))
        self.device, self.world, self.rank = device, world, rank

    def close(self):
        if self._c:
            lib().picp_comm_destroy(self._c)
            self._c = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def allreduce_max(self, values):
        v = np.ascontiguousarray(values, np.float64).reshape(-1).copy()
        _check(lib().picp_comm_allreduce_max(self._c, v.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), v.size))
        return v

    def barrier(self):
        _check(lib().picp_comm_barrier(self._c))

    def allgather_batch(self, batch, n_total):
        """Every rank's poses (n_total, 4, 4) and stats dicts, after this rank's batch solve."""
        T = np.zeros(16 * n_total, np.float32)
        st = (Stats * max(n_total, 1))()
        _check(lib().picp_batch_allgather(batch._b, self._c, n_total, _fptr(T), st))
        return np.transpose(T.reshape(n_total, 4, 4), (0, 2, 1)).copy(), [st[k].as_dict() for k in range(n_total)]


def allgather_batch_host(batch, world, rank, n_total, exchange):
    """picp_batch_allgather_host: the batch split's gather with the byte exchange done by the caller.
    exchange(send: bytes) -> bytes of world * len(send), rank order (e.g. a gloo all_gather).
    Returns every rank's poses (n_total, 4, 4) and stats dicts, like Comm.allgather_batch."""
    err = []

    def cb(user, send, recv, nbytes):
        try:
            out = exchange(ctypes.string_at(send, nbytes))
            if len(out) != world * nbytes:
                return 1
            ctypes.memmove(recv, out, len(out))
            return 0
        except Exception as e:  # reported through the library's status, never across the C frame
            err.append(e)
            return 2

    fn = EXCHANGE_FN(cb)
    T = np.zeros(16 * max(n_total, 1), np.float32)
    st = (Stats * max(n_total, 1))()
    rc = lib().picp_batch_allgather_host(batch._b, world, rank, fn, None, n_total, _fptr(T), st)
    if err:
        raise err[0]
    _check(rc)
    return (np.transpose(T[:16 * n_total].reshape(n_total, 4, 4), (0, 2, 1)).copy(),
            [st[k].as_dict() for k in range(n_total)])


def projection_matrix(K, T_cw):
    P = np.zeros(12, np.float32)
    _check(lib().picp_projection_matrix(_fptr(k_to_c(K)), _fptr(pose_to_c(T_cw)), _fptr(P)))
    return P.reshape(3, 4)


def triangulate(P1, P2, uv1, uv2, device=0):
    uv1 = _f32(uv1, (-1, 2))
    uv2 = _f32(uv2, (-1, 2))
    out = np.zeros((uv1.shape[0], 3), np.float32)
    _check(lib().picp_triangulate(device, _fptr(_f32(P1, (12,))), _fptr(_f32(P2, (12,))),
                                  _fptr(uv1), _fptr(uv2), uv1.shape[0], _fptr(out)))
    return out


def _i32ptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


# picp_match_batch_form kernel forms (include/picp_c.h PICP_MATCH_FORM_*)
MATCH_FORMS = {"full": 0, "accept_only": 1, "exact": 2}


def match_points(desc1, desc2, dist_thr=0.2, ratio_thr=0.8, device=0, form="full"):
    """match_points (src/my_utilities.h:70-120) on the GPU -> dict(best_idx, best_dist,
    second_dist, accepted); the reference's correspondences are the accepted (i, best_idx[i]).
    form: "full" (default), "accept_only" (only accepted and the best index of accepted queries
    are defined: the form the VO sequence runs) or "exact" (the exact scan; the same bits)."""
    d1 = np.asarray(desc1, np.float32)
    d2 = np.asarray(desc2, np.float32)
    dim = d1.shape[1] if d1.ndim == 2 and d1.shape[1] else (d2.shape[1] if d2.ndim == 2 else 10)
    return match_points_batch([d1.reshape(-1, dim)], [d2.reshape(-1, dim)], dist_thr, ratio_thr, device, form=form)[0]


def match_points_batch(desc1_list, desc2_list, dist_thr=0.2, ratio_thr=0.8, device=0, form="full"):
    """Many (set 1, set 2) pairs in one launch; returns a list of per-problem dicts."""
    o1 = np.zeros(len(desc1_list) + 1, np.int64)
    o2 = np.zeros(len(desc2_list) + 1, np.int64)
    o1[1:] = np.cumsum([len(d) for d in desc1_list])
    o2[1:] = np.cumsum([len(d) for d in desc2_list])
    dim = next((np.asarray(d).shape[1] for d in list(desc1_list) + list(desc2_list) if len(d)), 10)
    d1 = np.ascontiguousarray(np.concatenate([np.asarray(d, np.float32).reshape(-1, dim) for d in desc1_list]))
    d2 = np.ascontiguousarray(np.concatenate([np.asarray(d, np.float32).reshape(-1, dim) for d in desc2_list]))
    n1 = int(o1[-1])
    bi = np.zeros(n1, np.int32)
    bd = np.zeros(n1, np.float32)
    sd = np.zeros(n1, np.float32)
    acc = np.zeros(n1, np.int32)
    if n1 == 0:
        return [{"best_idx": bi, "best_dist": bd, "second_dist": sd, "accepted": acc.astype(bool)}
                for _ in desc1_list]
    _check(lib().picp_match_batch_form(device, len(desc1_list), o1.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                       o2.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), _fptr(d1),
                                       _fptr(d2) if d2.size else None, dim, dist_thr, ratio_thr,
                                       _i32ptr(bi), _fptr(bd), _fptr(sd), _i32ptr(acc), MATCH_FORMS[form]))
    return [{"best_idx": bi[o1[i]:o1[i + 1]], "best_dist": bd[o1[i]:o1[i + 1]],
             "second_dist": sd[o1[i]:o1[i + 1]], "accepted": acc[o1[i]:o1[i + 1]].astype(bool)}
            for i in range(len(desc1_list))]


class EssentialParams(ctypes.Structure):
    """picp_essential_params (include/picp_c.h): cv::findEssentialMat / cv::recoverPose knobs."""
    _fields_ = [("prob", ctypes.c_double), ("threshold", ctypes.c_double), ("max_iters", ctypes.c_int),
                ("reserved", ctypes.c_int), ("dist", ctypes.c_double)]


def essential_recover_pose_batch(p1_list, p2_list, K=None, prob=0.999, threshold=1.0, max_iters=1000,
                                 dist=50.0, device=0, want_mask=False):
    """Cam::computeEssentialAndRecoverPose (src/cam.cpp:37-91) on the GPU for many two-view
    problems: findEssentialMat(RANSAC) + recoverPose.  Returns per problem a dict with T (4x4
    camera-in-world of the second view, the first at the origin, unit baseline), inliers, good
    (and mask)."""
    K = K_REF if K is None else K
    offs = np.zeros(len(p1_list) + 1, np.int64)
    offs[1:] = np.cumsum([len(p) for p in p1_list])
    n = int(offs[-1])
    p1 = np.ascontiguousarray(np.concatenate([np.asarray(p, np.float32).reshape(-1, 2) for p in p1_list])
                              if n else np.zeros((0, 2), np.float32))
    p2 = np.ascontiguousarray(np.concatenate([np.asarray(p, np.float32).reshape(-1, 2) for p in p2_list])
                              if n else np.zeros((0, 2), np.float32))
    prm = EssentialParams(prob, threshold, max_iters, 0, dist)
    T = np.zeros(16 * len(p1_list), np.float32)
    inl = np.zeros(len(p1_list), np.int32)
    good = np.zeros(len(p1_list), np.int32)
    mask = np.zeros(max(n, 1), np.uint8) if want_mask else None
    _check(lib().picp_essential_batch(device, len(p1_list), offs.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                      _fptr(p1) if n else None, _fptr(p2) if n else None, _fptr(k_to_c(K)),
                                      ctypes.byref(prm), _fptr(T), _i32ptr(inl), _i32ptr(good),
                                      mask.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)) if want_mask else None))
    out = []
    for i in range(len(p1_list)):
        d = {"T": pose_from_c(T[16 * i:16 * i + 16]), "inliers": int(inl[i]), "good": int(good[i])}
        if want_mask:
            d["mask"] = mask[offs[i]:offs[i + 1]].astype(bool)
        out.append(d)
    return out


class VOSequence:
    """Device-resident VO over a packed observation sequence (C-ABI picp_vo_*): the reference's
    per-frame loop (exec/icp_test.cpp:61-136) run on the GPU for independent segments in
    lockstep.  Poses are camera-in-world 4x4 (numpy row/col)."""

    def __init__(self, frame_off, uv, desc, device=0, rows=480, cols=640, K=K_REF):
        self.frame_off = np.ascontiguousarray(frame_off, np.int64)
        uv = _f32(uv, (-1,))
        desc = np.ascontiguousarray(desc, np.float32)
        self.dim = desc.shape[1]
        self.n_frames = len(self.frame_off) - 1
        self._h = ctypes.c_void_p()
        _check(lib().picp_vo_create(ctypes.byref(self._h), device, rows, cols, _fptr(k_to_c(K)),
                                    self.n_frames, self.frame_off.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                    _fptr(uv), _fptr(desc.reshape(-1)), self.dim))
        self.first = self.steps = None

    def close(self):
        if self._h:
            lib().picp_vo_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_segments(self, first, steps, boot_poses, threshold=3000.0, **params):
        """boot_poses: (n_seg, 2, 4, 4) camera-in-world poses of frames first and first+1."""
        first = np.ascontiguousarray(first, np.int64)
        steps = np.ascontiguousarray(steps, np.int32)
        B = np.asarray(boot_poses, np.float32).reshape(len(first), 2, 4, 4)
        flat = np.ascontiguousarray(np.transpose(B, (0, 1, 3, 2)).reshape(-1))
        p = default_params(threshold=threshold, **params)
        _check(lib().picp_vo_set_segments(self._h, len(first), first.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                          steps.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                          _fptr(flat), ctypes.byref(p)))
        # a rejected call leaves the handle (and this view of it) unchanged
        self.first, self.steps = first, steps

    def run(self):
        _check(lib().picp_vo_run(self._h))

    def time(self, reps):
        ms = ctypes.c_float()
        _check(lib().picp_vo_time(self._h, reps, ctypes.byref(ms)))
        return ms.value

    def info(self):
        n_obs, n_slots, map_slots, npt = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int()
        _check(lib().picp_vo_info(self._h, ctypes.byref(n_obs), ctypes.byref(n_slots), ctypes.byref(map_slots),
                                  ctypes.byref(npt)))
        return {"n_obs": n_obs.value, "n_slots": n_slots.value, "map_slots": map_slots.value, "npt": npt.value}

    def _split(self, flat):
        out, o = [], 0
        for st in self.steps:
            out.append(flat[o:o + st + 1])
            o += st + 1
        return out

    def poses(self):
        """list over segments of (steps+1, 4, 4) camera-in-world poses ([0] = bootstrap pose)."""
        n = int((self.steps + 1).sum())
        out = np.zeros(16 * n, np.float32)
        _check(lib().picp_vo_get_poses(self._h, _fptr(out)))
        return self._split(np.transpose(out.reshape(n, 4, 4), (0, 2, 1)).copy())

    def step_records(self):
        """list over segments of dicts of arrays (steps+1 entries; entry 0 = bootstrap)."""
        n = int((self.steps + 1).sum())
        arr = (VOStep * n)()
        _check(lib().picp_vo_get_steps(self._h, arr))
        recs = {k: np.array([getattr(a, k) for a in arr]) for k, _ in VOStep._fields_}
        out, o = [], 0
        for st in self.steps:
            out.append({k: v[o:o + st + 1] for k, v in recs.items()})
            o += st + 1
        return out

    def map(self, seg):
        n = ctypes.c_int64()
        _check(lib().picp_vo_get_map(self._h, seg, 0, None, None, ctypes.byref(n)))
        xyz = np.zeros(max(n.value, 1) * 3, np.float32)
        desc = np.zeros(max(n.value, 1) * self.dim, np.float32)
        _check(lib().picp_vo_get_map(self._h, seg, n.value, _fptr(xyz), _fptr(desc), ctypes.byref(n)))
        return xyz[:3 * n.value].reshape(-1, 3), desc[:self.dim * n.value].reshape(-1, self.dim)


def selftest_rcp(e_lo=-8, e_hi=8, device=0):
    """Floats (both signs, exponents [e_lo, e_hi)) where the kernels' fast reciprocal differs
    from the IEEE division; 0 proves it for every |x| in [2^-100, 2^100] (picp_device.h)."""
    n = ctypes.c_uint64()
    _check(lib().picp_selftest_rcp(device, e_lo, e_hi, ctypes.byref(n)))
    return n.value
