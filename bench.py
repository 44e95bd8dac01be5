#!/usr/bin/env python3
"""PICP hot-path benchmark (BASELINE.json metric: PICP iterations/sec @ N correspondences).

Default workload (N=1): BASELINE configs[1] = C2, a single synthetic frame with 100,000
3D<->2D correspondences, 50 Gauss-Newton rounds (convergence test disabled for timing), on one
MI355X.  One "step" = one full 50-round solve of the frame (inputs resident in HBM, one hipGraph
replay: initial-state copy + 50 linearize launches + 1 finalize launch).  value = rounds
executed by all ranks / max-over-ranks wall time of the timed region.

Multi-GPU (torchrun, one process per GPU): every rank solves its own independent frame
(seed 42 + rank) -> weak scaling, no data-path collective; rank 0 gathers the final poses once
after timing (RCCL all_gather) to check them.

Printed JSON also carries:
  roofline     : the dominant kernel of the chosen execution mode (persistent: the whole 50-round
                 solve in one launch; graph: one launch per round); achieved = 20 algorithmic bytes
                 per correspondence-round (x,y,z,u,v float32 SoA) x correspondence-rounds per launch
                 / mean launch duration, the duration from HIP events around the timed replays on
                 the library's stream.
  cpu_baseline : the oracle's faithful float32 single-thread restatement (kind "port"), timed on
                 this host on a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
BYTES_PER_CORR = 20    # x,y,z,u,v float32 per correspondence-round

WORKLOADS = {
    "c2": dict(n=100000, problems=1, outlier=0.0, desc="C2 single-frame PICP, 100k synthetic correspondences, 50 GN rounds"),
    "c3": dict(n=1000000, problems=1, outlier=0.3, desc="C3 single-frame PICP, 1M synthetic correspondences, 30% outliers + chi2 rejection, 50 GN rounds"),
    "c4": dict(n=10000, problems=128, outlier=0.0, desc="C4 batch of independent frames x 10k correspondences (128 per GPU), 50 GN rounds each"),
    "c5": dict(frames=10000, obs=2000, desc="C5 full VO pipeline: 10k-frame synthetic sequence, per frame match -> PICP -> match -> triangulate on GPU, frame-parallel segments"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--rounds", type=int, default=50)
    ap.add_argument("--n", type=int, default=0, help="override correspondences per frame")
    ap.add_argument("--problems", type=int, default=0, help="override frames per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--skip-extras", action="store_true",
                    help="only the timed solves (profiling runs: no convergence-enabled re-solve)")
    ap.add_argument("--frames", type=int, default=0, help="c5: sequence length (default 10000)")
    ap.add_argument("--obs", type=int, default=0, help="c5: observations per frame (default 2000)")
    ap.add_argument("--seg-len", type=int, default=40, help="c5: PICP steps per segment")
    ap.add_argument("--stream-n", type=int, default=16000000,
                    help="c2: also measure one streaming single frame of this many correspondences "
                         "(roofline_streaming; 0 = skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch  # plumbing only: process group, barrier, device sync (loaded before the HIP lib)
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import picp_amd
    from picp_amd import synth

    wl = dict(WORKLOADS[args.workload])
    if args.workload == "c5":
        return bench_vo(args, wl, world, rank, local, dist, torch)
    n = args.n or wl["n"]
    nprob = args.problems or wl["problems"]
    R = args.rounds
    thr = 3000.0

    # ---- inputs (seeded, resident on the device before timing) ----
    if nprob == 1:
        p = synth.make_problem(n, seed=42 + rank, outlier_frac=wl["outlier"], pixel_noise=0.5, shuffle=False)
        xyz, uv, T_init, T_gt = p["xyz"], p["uv"], p["T_init"][None], p["T_gt"][None]
        sizes = [n]
    else:
        bt = synth.make_batch(nprob, n, base_seed=1000, first=rank * nprob,
                              outlier_frac=wl["outlier"], pixel_noise=0.5)
        xyz, uv, T_init, T_gt, sizes = bt["xyz"], bt["uv"], bt["T_init"], bt["T_gt"], bt["sizes"]
    b = picp_amd.Batch(sizes, device=local if world > 1 else 0)
    b.set_data(xyz, uv)
    b.set_poses(T_init)
    params = dict(threshold=thr, max_rounds=R, conv_eps=-1.0)

    def sync_all():
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        b.solve_async(**params)
    b.sync()
    sync_all()

    barrier()
    sync_all()
    t0 = time.perf_counter()
    # the K timed steps: K graph replays on the library's stream, bracketed by HIP events
    ev_ms, (launch_us, pair_us) = b.time(args.steps, **params)
    sync_all()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- correctness of what was timed (outside the timed region) ----
    poses = b.poses()
    err = max(synth.se3_log_norm(poses[i], T_gt[i]) for i in range(len(sizes)))
    if dist is not None:
        from picp_amd.dist import gather_rows
        # RCCL all-gather over xGMI: the only collective of the batch split (after timing)
        allp = gather_rows(poses.reshape(len(sizes), 16), world * len(sizes), dist, device="cuda")
        assert allp.shape == (world * len(sizes), 16)
        errs = torch.tensor([err], dtype=torch.float64, device="cuda")
        dist.all_reduce(errs, op=dist.ReduceOp.MAX)
        err = float(errs.item())

    # ---- roofline of the round kernel: algorithmic bytes per launch / mean launch duration,
    #      the duration from the HIP events around the timed region (launches back to back) ----
    info = b.info()
    # graph mode: one launch = one round over every correspondence; persistent/block mode: one
    # launch = the whole R-round solve
    corr_per_launch = int(info["total_corr"]) * (1 if info["mode"] == "graph" else R)
    achieved = BYTES_PER_CORR * corr_per_launch / (launch_us * 1e-6) / 1e9 if launch_us > 0 else 0.0

    # HBM traffic per launch from the committed PMC passes of the same default command
    # (tools/gpu_pmc.sh): C2 / C3 persistent kernel, C4 block kernel
    pmc_name = {("c2", "persistent"): "c2_persistent", ("c3", "persistent"): "c3_persistent",
                ("c4", "block"): "c4_block"}.get((args.workload, info["mode"]))
    default_cfg = (n == wl["n"] and len(sizes) == wl["problems"] and R == 50)
    traffic, tsrc = pmc_traffic(pmc_name) if (pmc_name and default_cfg) else (None, None)
    rounds_total = world * len(sizes) * R * args.steps
    value = rounds_total / elapsed
    out = {
        "metric": "PICP iterations/sec @ %d correspondences" % n,
        "value": round(value, 2),
        "unit": "iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded generator of SURVEY.md §8d; inputs resident in HBM)",
        "config": {
            "workload": wl["desc"],
            "n_corr": n,
            "frames_per_gpu": len(sizes),
            "rounds": R,
            "threshold": thr,
            "convergence_test": "disabled for timing",
            "parallelism": "independent frames, one process per GPU" if world > 1 else "single GPU",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic,
            "traffic_source": tsrc,
            "kernel": {"graph": "picp_round_kernel (one GN round per launch)",
                       "persistent": "picp_persistent_kernel (all GN rounds in one launch)",
                       "block": "picp_block_kernel (all GN rounds, one block per frame)"}[info["mode"]],
            "mode": info["mode"],
            "kernel_us": round(launch_us, 3),
            "kernel_us_event_pair": round(pair_us, 3),
            "timed_region_event_ms": round(ev_ms, 4),
            "bytes_per_launch": BYTES_PER_CORR * corr_per_launch,
            "blocks_per_launch": info["n_blocks"],
        },
        "pose_err_vs_gt_se3": err,
    }
    if args.workload in ("c2", "c3") and not args.skip_extras:
        # C2 is timed with exactly R rounds; also report the icp_test loop with its
        # convergence test on (exec/icp_test.cpp:99-106), measured after the timed region
        cparams = dict(params, conv_eps=1e-5)
        b.solve(**cparams)
        rounds_run = max(int(st["rounds"]) for st in b.stats())
        cms, _ = b.time(args.steps, **cparams)
        per_solve_ms = cms / args.steps
        out["with_convergence"] = {
            "conv_eps": 1e-5, "rounds_run": rounds_run, "ms_per_solve": round(per_solve_ms, 4),
            "iterations_per_s": round(len(sizes) * rounds_run / (per_solve_ms * 1e-3), 1),
            "pose_err_vs_gt_se3": max(synth.se3_log_norm(b.poses()[i], T_gt[i]) for i in range(len(sizes))),
        }
    if args.workload == "c3" and not args.skip_extras:
        # also with keep_outliers = true (outliers weighted by the robust
        # lambda = sqrt(threshold / chi), src/picp_solver.cpp:80-88), measured after the timed region
        kparams = dict(params, keep_outliers=1)
        b.set_poses(T_init)
        b.solve(**kparams)
        kerr = max(synth.se3_log_norm(b.poses()[i], T_gt[i]) for i in range(len(sizes)))
        kms, _ = b.time(args.steps, **kparams)
        out["keep_outliers_true"] = {
            "rounds": R, "ms_per_solve": round(kms / args.steps, 4),
            "iterations_per_s": round(len(sizes) * R / (kms / args.steps * 1e-3), 1),
            "pose_err_vs_gt_se3": kerr,
            "note": "outliers are weighted by the robust lambda, not rejected: the pose is biased by them "
                    "by design (the reference's keep_outliers mode); parity with the oracle is tested",
        }
    if args.workload == "c2" and args.stream_n > 0 and world == 1:
        out["roofline_streaming"] = streaming_roofline(args.stream_n, R, thr, local if world > 1 else 0)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(xyz[: sizes[0]], uv[: sizes[0]], T_init[0], R, thr, args.cpu_seconds)
        out["cpu_baseline_all_cores"] = cpu_baseline_mt(xyz[: sizes[0]], uv[: sizes[0]], T_init[0], R, thr,
                                                        max(2.0, args.cpu_seconds / 2))
    if rank == 0:
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


def pmc_traffic(name, fetch_scale=2.0):
    """HBM bytes per launch from the newest committed rocprofv3 PMC passes of the same command
    (profiles/rNN/<name>_pmc_{FETCH_SIZE,WRITE_SIZE}.json, written by tools/gpu_pmc*.sh from two
    separate --pmc passes).  FETCH_SIZE x fetch_scale (gfx950: x2 for wide coalesced streams,
    MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both in KiB.  (None, None) when absent: bench.py
    cannot collect PMC counters live."""
    import glob
    import json as _json
    dirs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9]*")))
    for d in reversed(dirs):
        f, w = (os.path.join(d, "%s_pmc_%s.json" % (name, c)) for c in ("FETCH_SIZE", "WRITE_SIZE"))
        if os.path.exists(f) and os.path.exists(w):
            fk = _json.load(open(f))["FETCH_SIZE"]["mean"]
            wk = _json.load(open(w))["WRITE_SIZE"]["mean"]
            src = "%s (FETCH_SIZE %.1f KiB x %g + WRITE_SIZE %.1f KiB per launch)" % (
                os.path.relpath(f, ROOT).replace("FETCH_SIZE", "{FETCH,WRITE}_SIZE"), fk, fetch_scale, wk)
            return round((fk * fetch_scale + wk) * 1024.0), src
    return None, None


def streaming_roofline(n, R, thr, device):
    """The same solve on one frame large enough to stream from HBM every round (SURVEY.md §8d:
    a > 256 MB working set, past the 256 MB Infinity Cache): 20 B x n per round-launch of
    picp_round_kernel.  Reported beside the C2 line, whose single 100k frame is latency-bound."""
    import picp_amd
    from picp_amd import synth
    p = synth.make_problem(n, seed=7, pixel_noise=0.5, shuffle=False)
    b = picp_amd.Batch([n], device=device)
    b.set_data(p["xyz"], p["uv"])
    b.set_poses(p["T_init"][None])
    params = dict(threshold=thr, max_rounds=R, conv_eps=-1.0)
    b.solve(**params)
    ev_ms, (launch_us, _) = b.time(5, **params)
    info = b.info()
    launches = 1 if info["mode"] == "graph" else 0
    per_launch = BYTES_PER_CORR * n * (1 if launches else R)
    achieved = per_launch / (launch_us * 1e-6) / 1e9
    err = synth.se3_log_norm(b.poses()[0], p["T_gt"])
    traffic, tsrc = pmc_traffic("stream16m") if (n == 16000000 and launches) else (None, None)
    return {"bound": "hbm", "n_corr": n, "working_set_MB": round(BYTES_PER_CORR * n / 1e6, 1),
            "kernel": "picp_round_kernel (one GN round per launch)" if launches else info["mode"],
            "mode": info["mode"], "blocks_per_launch": info["n_blocks"], "kernel_us": round(launch_us, 3),
            "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "traffic_source": tsrc,
            "bytes_per_launch": per_launch, "iterations_per_s": round(R * 5 / (ev_ms * 1e-3), 2),
            "pose_err_vs_gt_se3": err}


def bench_vo(args, wl, world, rank, local, dist, torch):
    """C5: the whole sequence is split into contiguous segments of --seg-len PICP steps (one-frame
    overlap); ranks take contiguous ranges of segments (strong scaling: the
    sequence is fixed).  One step = one replay of the captured run of this rank's segments
    (pair matching of all its frames, bootstrap, then per frame: world match, gather, PICP block
    kernel, triangulate/append).  value = frames estimated by all ranks / max-over-ranks time."""
    import numpy as np
    import picp_amd
    from picp_amd import synth
    from picp_amd.dist import shard_range
    from picp_amd.vo_synth import VOSequence, segments
    F = args.frames or wl["frames"]
    obs = args.obs or wl["obs"]
    L = args.seg_len
    seq = VOSequence(F, obs_per_frame=obs, seed=42)
    first, steps = segments(F, L)
    s0, s1 = shard_range(len(first), world, rank)
    fa, fb = int(first[s0]), int(first[s1 - 1] + steps[s1 - 1])
    D = seq.frames(fa, fb + 1)
    my_first, my_steps = first[s0:s1] - fa, steps[s0:s1]
    # each segment's world frame is its first camera, as the reference's is frame 0's
    # (exec/icp_test.cpp:36, bootstrap from Identity): float32 coordinates stay segment-sized
    rel = [np.linalg.inv(D["T_cw"][f].astype(np.float64)) for f in my_first]
    boot = np.stack([[np.eye(4), rel[k] @ D["T_cw"][f + 1]] for k, f in enumerate(my_first)]).astype(np.float32)
    vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], device=local if world > 1 else 0, K=seq.K)
    vo.set_segments(my_first, my_steps, boot, threshold=3000.0)

    def sync_all():
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    for _ in range(max(args.warmup, 1)):
        vo.run()
    sync_all()
    if dist is not None:
        dist.barrier()
    sync_all()
    t0 = time.perf_counter()
    ev_ms = vo.time(args.steps)
    sync_all()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # correctness of what was timed: drift vs gt, PICP work done
    P, Rr = vo.poses(), vo.step_records()
    err, rounds, corr = 0.0, 0, 0
    for k, f0 in enumerate(my_first):
        for t in range(1, len(P[k])):
            gt = rel[k] @ D["T_cw"][f0 + t].astype(np.float64)  # gt in the segment frame
            err = max(err, synth.se3_log_norm(P[k][t].astype(np.float64), gt))
        rounds += int(Rr[k]["rounds"][1:].sum())
        corr += int((Rr[k]["rounds"][1:].astype(np.int64) * Rr[k]["n_corr"][1:]).sum())
    stats = np.array([err, rounds, corr, int(my_steps.sum())], np.float64)
    if dist is not None:
        t = torch.tensor(stats, device="cuda")
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        e = t[:1].clone()
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        stats = t.cpu().numpy()
        stats[0] = float(e.item())
    frames_total = int(stats[3])
    info = vo.info()
    out = {
        "metric": "VO frames/sec (%d-frame synthetic sequence, ~%d obs/frame, per-frame match + PICP + triangulate)" % (F, obs),
        "value": round(frames_total * args.steps / elapsed, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic sequence (picp_amd/vo_synth.py, seed 42; observations resident in HBM)",
        "config": {"workload": wl["desc"], "frames": F, "obs_per_frame": obs, "segment_steps": L,
                   "segments": len(first), "segments_per_gpu": s1 - s0, "threshold": 3000.0,
                   "picp_loop": "icp_test: <= 50 rounds, relative chi convergence 1e-5",
                   "parallelism": "contiguous segment ranges, one process per GPU" if world > 1 else "single GPU",
                   "block_npt": info["npt"]},
        "picp_iterations_per_s": round(stats[1] * args.steps / elapsed, 1),
        "picp_corr_rounds_per_s": round(stats[2] * args.steps / elapsed, 1),
        "timed_region_event_ms": round(ev_ms * args.steps, 4),
        "pose_err_vs_gt_se3_max": stats[0],
        "pose_err_frame": "camera-in-world poses in each segment's frame (its first camera)",
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_vo(seq, L, args.cpu_seconds)
        out["cpu_baseline_all_cores"] = cpu_baseline_vo_mt(seq, L, max(2.0, args.cpu_seconds / 2))
    if rank == 0:
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline_vo(seq, L, budget_s):
    """Oracle VO loop (faithful float32, 1 thread) over whole segments of the same sequence
    until the budget is used: frames/s."""
    import numpy as np
    import oracle as O
    D = seq.frames(0, min(seq.n_frames, 4 * L + 1))
    frames, t0, f0 = 0, time.perf_counter(), 0
    while True:
        st = min(L, len(D["frame_off"]) - 2 - f0)
        if st < 1:
            f0 = 0
            continue
        T1 = (np.linalg.inv(D["T_cw"][f0].astype(np.float64)) @ D["T_cw"][f0 + 1]).astype(np.float32)
        O.vo_segment(seq.K, 480, 640, D["frame_off"], D["uv"], D["desc"], f0, st, np.eye(4, dtype=np.float32),
                     T1, mode=O.MODE_FAITHFUL)
        frames += st
        f0 += L
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": round(frames / el, 3), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": "%d frames in %d-step segments of the same sequence (oracle VO loop, faithful "
                      "float32, gcc -O3, 1 thread) in %.1f s" % (frames, L, el)}


def cpu_baseline_vo_mt(seq, L, budget_s):
    """SURVEY.md §8d all-cores variant of the C5 baseline: the oracle VO loop over independent
    segments in parallel, one segment per host thread (OMP_NUM_THREADS threads, 16 = the GPU box's
    CPU share).  ctypes releases the GIL around or_vo_segment, whose VO path keeps no static
    state, so the threads run concurrently.  Timing only, never a parity oracle."""
    import concurrent.futures as cf
    import numpy as np
    import oracle as O
    nt = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1, 64))
    D = seq.frames(0, min(seq.n_frames, nt * L + 1))
    nseg = max(1, (len(D["frame_off"]) - 2) // L)
    t0 = time.perf_counter()

    def worker(i):
        f0 = (i % nseg) * L
        st = min(L, len(D["frame_off"]) - 2 - f0)
        T1 = (np.linalg.inv(D["T_cw"][f0].astype(np.float64)) @ D["T_cw"][f0 + 1]).astype(np.float32)
        done = 0
        while time.perf_counter() - t0 < budget_s:
            O.vo_segment(seq.K, 480, 640, D["frame_off"], D["uv"], D["desc"], f0, st,
                         np.eye(4, dtype=np.float32), T1, mode=O.MODE_FAITHFUL)
            done += st
        return done

    with cf.ThreadPoolExecutor(max_workers=nt) as ex:
        frames = sum(ex.map(worker, range(nt)))
    el = time.perf_counter() - t0
    return {"value": round(frames / el, 3), "unit": "frames/s", "cores": nt, "kind": "port",
            "sample": "%d frames: %d threads, each re-running one %d-step segment of the same sequence "
                      "(oracle VO loop, faithful float32, gcc -O3) for %.1f s on %s" % (frames, nt, L, el, _cpu_model())}


def _cpu_model():
    import platform
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return model


def cpu_baseline_mt(xyz, uv, T_init, R, thr, budget_s):
    """SURVEY.md §8d's all-cores CPU baseline for C2/C3: the oracle's loop with the linearize as a
    chunked reduction over OMP_NUM_THREADS threads (the box's CPU share; os.cpu_count() shows the
    whole machine).  Timing only; its pose is checked against the sequential oracle's."""
    import numpy as np
    import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    x, y, z = (np.ascontiguousarray(xyz[:, i]) for i in range(3))
    u, v = np.ascontiguousarray(uv[:, 0]), np.ascontiguousarray(uv[:, 1])
    Kref = np.array([[180, 0, 320], [0, 180, 240], [0, 0, 1]], np.float32)
    solves, t0 = 0, time.perf_counter()
    while True:
        T_mt, _ = O.solve_soa_mt(T_init, Kref, 480, 640, x, y, z, u, v, thr, threads,
                                 mode=O.MODE_FAITHFUL, max_rounds=R, conv_eps=-1.0)
        solves += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": round(solves * R / el, 3), "unit": "iterations/s", "cores": threads, "kind": "port",
            "sample": "%d x %d-round solves of one %d-correspondence frame (faithful float32 oracle, "
                      "linearize as a chunked reduction over %d OpenMP threads, gcc -O3 "
                      "-march=x86-64-v3) in %.1f s on %s" % (solves, R, len(x), threads, el, _cpu_model())}


def cpu_baseline(xyz, uv, T_init, R, thr, budget_s):
    """Oracle (faithful float32, sequential) single thread on one frame of the workload:
    whole R-round solves until the time budget is used (at least one)."""
    import numpy as np
    import oracle as O
    x, y, z = (np.ascontiguousarray(xyz[:, i]) for i in range(3))
    u, v = np.ascontiguousarray(uv[:, 0]), np.ascontiguousarray(uv[:, 1])
    K = O._k9  # noqa: F841  (ensure module import)
    Kref = np.array([[180, 0, 320], [0, 180, 240], [0, 0, 1]], np.float32)
    solves, t0 = 0, time.perf_counter()
    while True:
        O.solve_soa(T_init, Kref, 480, 640, x, y, z, u, v, thr, mode=O.MODE_FAITHFUL,
                    max_rounds=R, conv_eps=-1.0)
        solves += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": round(solves * R / el, 3), "unit": "iterations/s", "cores": 1, "kind": "port",
            "sample": "%d x %d-round solves of one %d-correspondence frame (faithful float32 oracle, "
                      "gcc -O3 -march=x86-64-v3, 1 thread) in %.1f s on %s" % (solves, R, len(x), el,
                                                                              _cpu_model())}


if __name__ == "__main__":
    main()
