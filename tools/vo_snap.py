"""Per-step snapshots of the VO sequence's PICP launches under each step schedule (serial vs
PICP_VO_OVERLAP / PICP_VO_CHAINS), compared with the serial run.  Diagnostic VO runtime only
(make -C 02-visualodometry_amd vodiag -> lib/libpicp_amd_vodiag.so, loaded through PICP_LIB; the
block kernel is the shipped one).  After every step's PICP block kernel the runtime copies, on
the launch's stream, the step's problems, initial states, SoA planes (its inputs) and final
states (its output).  For the first differing steps this prints whether the inputs differ or
only the output does, and saves the first output-only case (inputs + both outputs) to
gpurun_out/r03/vo_snap_case.npz for a solo replay.
usage: python tools/vo_snap.py [FRAMES[:OBS[:SEED]]] [SETTING ...]   (first setting = reference)"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
os.environ.setdefault("PICP_LIB", os.path.join(ROOT, "02-visualodometry_amd", "lib", "libpicp_amd_vodiag.so"))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
import picp_amd  # noqa: E402
from picp_amd.vo_synth import VOSequence, segments  # noqa: E402

spec = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2001").split(":")]
F, OBS, SEED = (spec + [2000, 42][len(spec) - 1:])[:3]
settings = sys.argv[2:] or ["PICP_VO_CHAINS=1,PICP_VO_OVERLAP=0", "PICP_VO_OVERLAP=1", "PICP_VO_CHAINS=2"]
seq = VOSequence(F, obs_per_frame=OBS, seed=SEED)
first, steps = segments(F, 40)
NS = len(first)
D = seq.frames(0, F)
cap = (int(np.diff(D["frame_off"]).max()) + 3) // 4 * 4
rel = [np.linalg.inv(D["T_cw"][f].astype(np.float64)) for f in first]
boot = np.stack([[np.eye(4), rel[k] @ D["T_cw"][f + 1]] for k, f in enumerate(first)]).astype(np.float32)

L = picp_amd.lib()
L.picp_vo_debug_snap_bytes.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int)]
L.picp_vo_debug_snap_set.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
hip = ctypes.CDLL("libamdhip64.so")
PROB = np.dtype([("offset", "<i8"), ("n", "<i4"), ("blk0", "<i4"), ("nblk", "<i4"), ("pad", "<i4")])
STATE = np.dtype([("R", "<f4", 9), ("t", "<f4", 3), ("chi_prev", "<f4"), ("chi_in", "<f4"), ("chi_out", "<f4"),
                  ("n_in", "<i4"), ("n_proj", "<i4"), ("rounds", "<i4"), ("done", "<i4"), ("ok", "<i4"),
                  ("converged", "<i4"), ("pad", "<i4", 11)])
assert PROB.itemsize == 24 and STATE.itemsize == 128


def run_setting(setting):
    keys = []
    for kv in filter(None, setting.split(",")):
        k, v = kv.split("=")
        os.environ[k] = v
        keys.append(k)
    vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], device=0, K=seq.K)
    vo.set_segments(first, steps, boot, threshold=3000.0)
    per, nst = ctypes.c_int64(), ctypes.c_int()
    assert L.picp_vo_debug_snap_bytes(vo._h, ctypes.byref(per), ctypes.byref(nst)) == 0
    total = per.value * nst.value
    buf = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(buf), ctypes.c_size_t(total)) == 0
    assert hip.hipMemset(buf, 0xFF, ctypes.c_size_t(total)) == 0
    assert L.picp_vo_debug_snap_set(vo._h, buf) == 0
    vo.run()
    assert hip.hipDeviceSynchronize() == 0
    h = np.empty(total, np.uint8)
    assert hip.hipMemcpy(h.ctypes.data_as(ctypes.c_void_p), buf, ctypes.c_size_t(total), 2) == 0
    assert L.picp_vo_debug_snap_set(vo._h, None) == 0
    hip.hipFree(buf)
    poses = np.concatenate([np.asarray(p).reshape(-1) for p in vo.poses()])
    vo.close() if hasattr(vo, "close") else None
    for k in keys:
        del os.environ[k]
    snaps = []
    for t in range(nst.value):
        b = h[t * per.value:(t + 1) * per.value]
        o = 0
        probs = b[o:o + NS * 24].view(PROB)
        o += NS * 24
        st_in = b[o:o + NS * 128].view(STATE)
        o += NS * 128
        st_out = b[o:o + NS * 128].view(STATE)
        o += NS * 128
        planes = b[o:o + 5 * NS * cap * 4].view(np.float32).reshape(5, NS, cap)
        snaps.append((probs, st_in, st_out, planes))
    return poses, snaps


def raw(a):
    return np.ascontiguousarray(a).view(np.uint8)


ref = None
saved = False
for setting in settings:
    for rep in range(2 if ref is not None else 1):
        poses, snaps = run_setting(setting)
        if ref is None:
            ref = (poses, snaps)
            print("reference %s: %d segments x %d steps, cap %d" % (setting, NS, len(snaps), cap), flush=True)
            continue
        same = np.array_equal(poses.view(np.uint32), ref[0].view(np.uint32))
        print("%s rep %d: poses %s" % (setting, rep, "same" if same else "DIFFER"), flush=True)
        shown = 0
        for t, ((p0, i0, o0, x0), (p1, i1, o1, x1)) in enumerate(zip(ref[1], snaps)):
            for s in range(NS):
                n = int(p0[s]["n"]) if p0[s]["n"] >= 0 else 0
                d_prob = not np.array_equal(raw(p0[s:s + 1]), raw(p1[s:s + 1]))
                d_in = not np.array_equal(raw(i0[s:s + 1])[:48], raw(i1[s:s + 1])[:48])  # R, t
                d_pl = not np.array_equal(raw(x0[:, s, :n]), raw(x1[:, s, :n]))
                d_out = not np.array_equal(raw(o0[s:s + 1]), raw(o1[s:s + 1]))
                if not (d_prob or d_in or d_pl or d_out):
                    continue
                if shown < 10:
                    what = [w for w, f in (("problem", d_prob), ("initial pose", d_in), ("planes", d_pl),
                                           ("OUTPUT", d_out)) if f]
                    extra = ""
                    if d_out and not (d_prob or d_in or d_pl):
                        a, b = o0[s], o1[s]
                        dp = float(np.abs(np.concatenate([a["R"], a["t"]]) - np.concatenate([b["R"], b["t"]])).max())
                        extra = " [same inputs] rounds %d/%d n_in %d/%d chi_in %r/%r max|dpose| %.3g" % (
                            a["rounds"], b["rounds"], a["n_in"], b["n_in"], float(a["chi_in"]), float(b["chi_in"]), dp)
                        if not saved:
                            np.savez(os.path.join(ROOT, "gpurun_out", "r03", "vo_snap_case.npz"),
                                     X=x0[:, s, :n], R0=i0[s]["R"], t0=i0[s]["t"], out_ref=raw(o0[s:s + 1]),
                                     out_cur=raw(o1[s:s + 1]), K=seq.K, step=t, seg=s, setting=setting)
                            saved = True
                    print("  step %2d seg %2d differs in %s%s" % (t, s, ", ".join(what), extra), flush=True)
                shown += 1
        print("  %d (step, segment) records differ" % shown, flush=True)
