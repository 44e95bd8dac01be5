"""Where does the VO sequence first diverge between step schedules (serial vs PICP_VO_OVERLAP /
PICP_VO_CHAINS)?  Diagnostic build only (make -C 02-visualodometry_amd bdiag, loaded through PICP_LIB):
every PICP block-kernel launch of the sequence records, per (segment, step, round), the pose each
wave linearized at, the 8 wave sums of every term, the converted totals, the new pose, the
finishing wave's lane agreement, the permlane-vs-bpermute reduction check and an XOR checksum of
the step's inputs (picp_block.hip, PICP_BDIAG).  For the first differing (segment, step) records
of each schedule it prints the first differing round and section.
usage: python tools/bdiag_vo.py [FRAMES[:OBS[:SEED]]] [SETTING ...]   (first setting = reference)"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
os.environ.setdefault("PICP_LIB", os.path.join(ROOT, "02-visualodometry_amd", "lib", "libpicp_amd_bdiag.so"))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
import picp_amd  # noqa: E402
from picp_amd.vo_synth import VOSequence, segments  # noqa: E402

spec = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2001").split(":")]
F, OBS, SEED = (spec + [2000, 42][len(spec) - 1:])[:3]
settings = sys.argv[2:] or ["PICP_VO_CHAINS=1,PICP_VO_OVERLAP=0", "PICP_VO_OVERLAP=1", "PICP_VO_CHAINS=2"]
R, REC = 50, 576
seq = VOSequence(F, obs_per_frame=OBS, seed=SEED)
first, steps = segments(F, 40)
NS, ST = len(first), int(steps.max())
D = seq.frames(0, F)
cap = (int(np.diff(D["frame_off"]).max()) + 3) // 4 * 4
rel = [np.linalg.inv(D["T_cw"][f].astype(np.float64)) for f in first]
boot = np.stack([[np.eye(4), rel[k] @ D["T_cw"][f + 1]] for k, f in enumerate(first)]).astype(np.float32)

L = picp_amd.lib()
DIAG = hasattr(L, "picp_debug_bdiag_set")  # False on the shipped library: poses only (the control)
if DIAG:
    L.picp_debug_bdiag_set.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.c_int,
                                       ctypes.c_int]
hip = ctypes.CDLL("libamdhip64.so")
nfl = NS * ST * R * REC
LANE = hasattr(L, "picp_debug_bdiag_lane")  # part 16 builds: per-lane folded partials of step 0
nlf = NS * R * 512 * 32
lptr = ctypes.c_void_p()
if LANE:
    L.picp_debug_bdiag_lane.argtypes = [ctypes.c_void_p]
    assert hip.hipMalloc(ctypes.byref(lptr), ctypes.c_size_t(nlf * 4)) == 0
dptr = ctypes.c_void_p()
assert hip.hipMalloc(ctypes.byref(dptr), ctypes.c_size_t(nfl * 4)) == 0

SECT = [("wave_pose", 0, 96), ("wave_sums", 96, 352), ("totals", 352, 384), ("pose_out", 384, 396),
        ("stats", 396, 400), ("laneagree", 404, 405), ("redcheck", 405, 413), ("inputs", 413, 415),
        ("posemask", 416, 432), ("finishmask", 432, 434), ("finish_inputs", 434, 440)]


def run(vo):
    assert hip.hipMemset(dptr, 0, ctypes.c_size_t(nfl * 4)) == 0
    if DIAG:
        assert L.picp_debug_bdiag_set(dptr, 0, R, cap, NS, ST) == 0
    if LANE:
        assert hip.hipMemset(lptr, 0, ctypes.c_size_t(nlf * 4)) == 0
        assert L.picp_debug_bdiag_lane(lptr) == 0
    assert hip.hipDeviceSynchronize() == 0
    vo.run()
    assert hip.hipDeviceSynchronize() == 0
    h = np.empty(nfl, np.float32)
    assert hip.hipMemcpy(h.ctypes.data_as(ctypes.c_void_p), dptr, ctypes.c_size_t(nfl * 4), 2) == 0
    P = np.concatenate([np.asarray(p).reshape(-1) for p in vo.poses()])
    lanes = None
    if LANE:
        lanes = np.empty(nlf, np.float32)
        assert hip.hipMemcpy(lanes.ctypes.data_as(ctypes.c_void_p), lptr, ctypes.c_size_t(nlf * 4), 2) == 0
        lanes = lanes.reshape(NS, R, 8, 64, 32)
    return P, h.reshape(NS, ST, R, REC), lanes


def masks(tag, Rx):
    """Lanes whose pose (or finish result) differed from lane 0's, wherever the kernel saw it."""
    pm = Rx[..., 416:432].view(np.uint32).reshape(Rx.shape[:-1] + (8, 2))
    fm = Rx[..., 432:434].view(np.uint32)
    hits = list(zip(*np.nonzero(pm.any(axis=-1))))
    fh = list(zip(*np.nonzero(fm.any(axis=-1))))
    if hits or fh:
        print("  %s: pose-lane disagreements %d, finish-lane disagreements %d" % (tag, len(hits), len(fh)), flush=True)
    for s_, t_, r_, w_ in hits[:10]:
        m = int(pm[s_, t_, r_, w_, 0]) | (int(pm[s_, t_, r_, w_, 1]) << 32)
        print("    seg %d step %d round %d wave %d lanes %s" % (s_, t_, r_ + 1, w_, [l for l in range(64) if m >> l & 1]))
    for s_, t_, r_ in fh[:10]:
        m = int(fm[s_, t_, r_, 0]) | (int(fm[s_, t_, r_, 1]) << 32)
        print("    finish seg %d step %d round %d lanes %s" % (s_, t_, r_ + 1, [l for l in range(64) if m >> l & 1]))
    im = Rx[..., 434:440].view(np.uint32).reshape(Rx.shape[:-1] + (3, 2))
    ih = list(zip(*np.nonzero(im.any(axis=(-1, -2)))))
    if ih:
        print("  %s: finish-input disagreements %d" % (tag, len(ih)), flush=True)
    for s_, t_, r_ in ih[:10]:
        desc = []
        for k, name in enumerate(("s_tot", "pose", "chi_prev")):
            m = int(im[s_, t_, r_, k, 0]) | (int(im[s_, t_, r_, k, 1]) << 32)
            if m:
                ls = [l for l in range(64) if m >> l & 1]
                desc.append("%s lanes %s" % (name, ls if len(ls) < 8 else "%d..%d (%d)" % (ls[0], ls[-1], len(ls))))
        print("    inputs seg %d step %d round %d: %s" % (s_, t_, r_ + 1, "; ".join(desc)))


def lanes48(tag, Rx):
    """Part 128: where lane 48's finish first departs from lane 0's (totals read, dx, pose)."""
    a, b = Rx[..., 448:498], Rx[..., 498:548]
    if not a.any():
        return
    d = a.view(np.uint32) != b.view(np.uint32)
    hits = list(zip(*np.nonzero(d.any(axis=-1))))
    print("  %s: lane-48 finish records differing from lane 0: %d" % (tag, len(hits)), flush=True)
    for s_, t_, r_ in hits[:8]:
        dd = d[s_, t_, r_]
        parts = []
        for name, lo, hi in (("totals", 0, 32), ("dx", 32, 38), ("pose", 38, 50)):
            idx = np.nonzero(dd[lo:hi])[0]
            if len(idx):
                parts.append("%s idx %s" % (name, idx[:8].tolist()))
        print("    seg %d step %d round %d: %s" % (s_, t_, r_ + 1, "; ".join(parts)), flush=True)
        if dd[0:32].any():
            i = int(np.nonzero(dd[0:32])[0][0])
            print("      total %d: lane0 %r lane48 %r" % (i, float(a[s_, t_, r_, i]), float(b[s_, t_, r_, i])))
        elif dd[32:38].any():
            print("      dx lane0 %s\n         lane48 %s" % (a[s_, t_, r_, 32:38].tolist(), b[s_, t_, r_, 32:38].tolist()))


def report(tag, ref, cur):
    (P0, R0, LA0), (P1, R1, LA1) = ref, cur
    masks(tag, R1)
    lanes48(tag, R1)
    if LA0 is not None:  # step 0: the first (segment, round, wave) whose per-lane partials differ
        dl = LA0.view(np.uint32) != LA1.view(np.uint32)
        segs = sorted(set(np.nonzero(dl.any(axis=(1, 2, 3, 4)))[0].tolist()))
        print("  step-0 per-lane partials differ in %d segments" % len(segs), flush=True)
        for s in segs[:6]:
            rr = int(np.nonzero(dl[s].any(axis=(1, 2, 3)))[0][0])
            ws = np.nonzero(dl[s, rr].any(axis=(1, 2)))[0].tolist()
            w = ws[0]
            ln = np.nonzero(dl[s, rr, w].any(axis=1))[0].tolist()
            tm = np.nonzero(dl[s, rr, w, ln[0]])[0].tolist()
            sums_same = np.array_equal(R0[s, 0, rr, 96:352].view(np.uint32), R1[s, 0, rr, 96:352].view(np.uint32))
            pose_same = np.array_equal(R0[s, 0, rr, 0:96].view(np.uint32), R1[s, 0, rr, 0:96].view(np.uint32))
            print("    seg %d round %d: waves %s; wave %d lanes %s; lane %d terms %s; wave poses %s; wave sums %s"
                  % (s, rr + 1, ws, w, ln[:16], ln[0], tm[:12], "same" if pose_same else "DIFFER",
                     "same" if sums_same else "DIFFER"), flush=True)
            print("      lane %d: %s\n   vs       %s" % (ln[0], LA0[s, rr, w, ln[0], tm[:6]].tolist(),
                                                      LA1[s, rr, w, ln[0], tm[:6]].tolist()), flush=True)
    lm, rb = R1[..., 404], R1[..., 405:413]
    print("%s: poses %s; lane disagreement records %d; reduction mismatch records %d" % (
        tag, "same" if np.array_equal(P0.view(np.uint32), P1.view(np.uint32)) else "DIFFER",
        int((lm != 0).sum()), int((rb != 0).any(axis=-1).sum())), flush=True)
    d = (R0.view(np.uint32) != R1.view(np.uint32))
    rec_bad = d.any(axis=(2, 3))  # (segment, step)
    if not rec_bad.any():
        print("  records identical", flush=True)
        return
    by_step = sorted(zip(*np.nonzero(rec_bad)), key=lambda x: (x[1], x[0]))
    print("  differing (segment, step) records: %d; first steps %s" % (len(by_step), [(int(a), int(b)) for a, b in by_step[:10]]))
    for s, t in by_step[:8]:
        rr = int(np.nonzero(d[s, t].any(axis=1))[0][0])
        where = []
        for name, a, b in SECT:
            idx = np.nonzero(d[s, t, rr, a:b])[0]
            if len(idx):
                if name == "wave_pose":
                    where.append("%s waves %s" % (name, sorted(set((idx // 12).tolist()))))
                elif name == "wave_sums":
                    where.append("%s (term, wave) %s" % (name, [(int(i // 8), int(i % 8)) for i in idx[:6]]))
                else:
                    where.append("%s idx %s" % (name, idx[:6].tolist()))
        inp = "same inputs" if np.array_equal(R0[s, t, 0, 413:415].view(np.uint32), R1[s, t, 0, 413:415].view(np.uint32)) \
            else "INPUTS DIFFER (n %g vs %g)" % (R0[s, t, 0, 414], R1[s, t, 0, 414])
        print("  seg %2d step %2d (%s): first round %2d: %s" % (s, t, inp, rr + 1, "; ".join(where)), flush=True)
        if any(w.startswith("wave_sums") for w in where) and not any(w.startswith("wave_pose") for w in where):
            for i in np.nonzero(d[s, t, rr, 96:352])[0][:4]:
                print("    term %d wave %d: %r vs %r" % (i // 8, i % 8, float(R0[s, t, rr, 96 + i]), float(R1[s, t, rr, 96 + i])))
        if any(w.startswith("pose_out") for w in where) and not any(w.startswith("totals") for w in where):
            print("    pose_out %s vs %s" % (R0[s, t, rr, 384:396].tolist(), R1[s, t, rr, 384:396].tolist()))


ref = None
for setting in settings:
    keys = []
    for kv in filter(None, setting.split(",")):
        k, v = kv.split("=")
        os.environ[k] = v
        keys.append(k)
    vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], device=0, K=seq.K)
    vo.set_segments(first, steps, boot, threshold=3000.0)
    for rep in range(2):
        cur = run(vo)
        if ref is None:
            ref = cur
            print("reference %s recorded (%d segments x %d steps)" % (setting, NS, ST), flush=True)
            masks("reference", cur[1])
            lanes48("reference", cur[1])
            continue
        report("%s rep %d" % (setting, rep), ref, cur)
    vo.close() if hasattr(vo, "close") else None
    for k in keys:
        del os.environ[k]
