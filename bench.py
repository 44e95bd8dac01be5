#!/usr/bin/env python3
"""PICP hot-path benchmark (BASELINE.json metric: PICP iterations/sec @ N correspondences).

Headline (every N): BASELINE configs[1] = C2 on each GPU -- one synthetic frame of 100,000
3D<->2D correspondences per GPU, 50 Gauss-Newton rounds (convergence test disabled for timing).
One "step" = one full 50-round solve of the frame (inputs resident in HBM; one persistent
launch).  value = rounds executed by all ranks / max-over-ranks wall time of the timed region
(weak scaling: every rank solves its own independent frame, seed 42 + rank).

Multi-GPU: `python bench.py --gpus N` (no WORLD_SIZE in the environment) starts N child processes
itself (one per GPU, RANK/LOCAL_RANK/WORLD_SIZE set, never exec) and relays rank 0's line; under
torchrun the process is already one rank.  The ranks share a gloo group (CPU, only to hand the
RCCL unique id around); every collective of the measurement -- the barriers, the max over ranks
of the timed region, the all-gather of the C4 results -- is RCCL over xGMI driven by the C++
library (picp_comm_*, include/picp_c.h).

Sub-results on the same line (default run, bounded time):
  c4 : BASELINE configs[3]: 1024 independent frames x 10k correspondences, sharded across the N
       GPUs (strong scaling of the fixed batch: each rank solves picp_shard_range's frames; the
       timed region ends with one RCCL all-gather of all 1024 poses + stats).
  c3 : configs[2] (N = 1 only): one 1M-correspondence frame, 30 % outliers, chi2 gate.
  c5 : configs[4]: the 10k-frame synthetic VO sequence, contiguous segments split over ranks.
Each carries value, ms_per_step, the dominant kernel's launch time, its committed PMC traffic
(profiles/) and, at N = 1, the oracle's CPU baseline on a bounded sample.

The printed line is compact (< 2 KB: the driver keeps only the tail of stdout): the contract's
keys first, then each sub-result's value, step time, roofline fraction and projections
(compact_line).  The full result -- every sample, basis string and sub-result -- goes to the side
file named by "detail" (default gpurun_out/bench_detail_<workload>_n<N>.json).

The full result also carries:
  roofline     : the dominant kernel of the headline (picp_persistent_kernel: the whole 50-round
                 solve in one launch); achieved = 20 algorithmic bytes per correspondence-round
                 (x,y,z,u,v float32 SoA) x correspondence-rounds per launch / mean launch period,
                 the period from HIP events around the timed launches on the library's stream.
                 roofline.latency: the same kernel against its per-round latency floor (C2 is a
                 hand-off-latency-bound kernel).
                 Its floor is the price list's broadcast + fan-in row scaled to the launch's blocks.
  cpu_baseline : the oracle's faithful float32 single-thread restatement (kind "port"), timed on
                 this host on a bounded sample of the same workload; cpu_baseline_all_cores the
                 same over the box's CPU share (OMP_NUM_THREADS threads).  Every CPU figure is the
                 median of 5 samples, and every GPU value the median of --samples (5) timed
                 regions of K steps each, the per-sample values in "timing".
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
BYTES_PER_CORR = 20    # x,y,z,u,v float32 per correspondence-round
HANDOFF_US = 0.8       # MI355X_MICROARCH.md price list, handoff-1to1 (idle, 8-B granule)
FANIN_PAIR_US = 4.2    # price list, fanin: a 1->255 broadcast plus its 255->1 fan-in (idle, low end)
FANIN_ARRIVAL_US = 0.012  # price list, fanin: ~11-13 ns per arrival
FLOPS_PER_CORR = 160   # FP32 flops per correspondence-round (projection, J, J^T J, J^T e)
# FP32 vector ceiling: MI355X_MICROARCH.md -- 4 SIMD-32 units per CU, a wave64 v_fma_f32 issues in
# 2 cycles per SIMD (one wave alone sustains 4), so 256 CUs x 4 SIMDs x 32 lanes x 2 flops x 2.4 GHz
# = 157.3 TF/s with plain (unpacked) v_fma_f32, the form the device code is built with (DESIGN.md
# §4.9).  Calibrated on MI355X by tools/ubench/issue_ubench.hip (profiles/r05/issue/).
VALU_PEAK_TFS = 157.3
SIMDS = 1024           # 256 CUs x 4
VALU_ISSUE_CYCLES = 2  # SIMD cycles per wave64 VALU instruction at >= 2 waves per SIMD (SIMD-32)
CLOCK_GHZ = 2.4        # nominal shader clock (MI355X_MICROARCH.md; under load it can run lower)

WORKLOADS = {
    "c2": dict(n=100000, problems=1, outlier=0.0, desc="C2 single-frame PICP, 100k synthetic correspondences, 50 GN rounds"),
    "c3": dict(n=1000000, problems=1, outlier=0.3, desc="C3 single-frame PICP, 1M synthetic correspondences, 30% outliers + chi2 rejection, 50 GN rounds"),
    "c4": dict(n=10000, problems=1024, outlier=0.0, desc="C4 batch of 1024 independent frames x 10k correspondences, sharded across the GPUs, 50 GN rounds each"),
    "c5": dict(frames=10000, obs=2000, desc="C5 full VO pipeline: 10k-frame synthetic sequence, per frame match -> PICP -> match -> triangulate on GPU, frame-parallel segments"),
}
THRESHOLD = 3000.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`bench.py --gpus N` outside torchrun: N fresh child processes, one per GPU (subprocess,
    never exec; this parent never touches the GPU).  Rank 0's stdout is the bench line."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    try:
        # poll every rank (not in rank order): a rank that fails leaves the others blocked in a
        # collective, so the first failure anywhere terminates the rest
        while any(p.poll() is None for p in procs):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                rc = bad[0]
                for q in procs:
                    if q.poll() is None:
                        q.terminate()
                break
            time.sleep(0.1)
        for p in procs:
            p.wait()
            if rc == 0 and p.returncode != 0:
                rc = p.returncode
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    return rc if rc >= 0 else 1


class Ranks:
    """This process's place in the job: world/rank, the gloo group (CPU; the RCCL unique id and
    plan-only gathers) and the RCCL communicator of the C++ library (GPU runs)."""

    def __init__(self, plan_only):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        self.comm = None
        if self.world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist
        if not plan_only and self.world > 1:
            import picp_amd
            uid = [picp_amd.comm_unique_id() if self.rank == 0 else None]
            self.dist.broadcast_object_list(uid, src=0)
            self.comm = picp_amd.Comm(self.local, self.world, self.rank, uid[0])

    @property
    def device(self):
        return self.local if self.world > 1 else 0

    def barrier(self):
        if self.comm is not None:
            self.comm.barrier()

    def max(self, values):
        if self.comm is None:
            return list(values)
        return list(self.comm.allreduce_max(values))

    def gather_obj(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.comm is not None:
            self.comm.close()
        if self.dist is not None:
            self.dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--rounds", type=int, default=50)
    ap.add_argument("--n", type=int, default=0, help="override correspondences per frame")
    ap.add_argument("--problems", type=int, default=0, help="override frames (c4: total over ranks)")
    ap.add_argument("--samples", type=int, default=5,
                    help="timed regions of K steps each; value = the median (BASELINE.md: median of >= 5)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (headline)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--skip-extras", action="store_true",
                    help="only the timed solves (profiling runs: no sub-results, no side measurements)")
    ap.add_argument("--frames", type=int, default=0, help="c5: sequence length (default 10000)")
    ap.add_argument("--obs", type=int, default=0, help="c5: observations per frame (default 2000)")
    ap.add_argument("--seg-len", type=int, default=40, help="c5: PICP steps per segment")
    ap.add_argument("--c5-boot", default="gt", choices=("gt", "essential"),
                    help="c5: each segment's second pose from the ground-truth pair (gt) or from the "
                         "reference's two-view bootstrap on the GPU (essential: match_points + "
                         "findEssentialMat/recoverPose, unit baseline; drift then scale-aligned)")
    ap.add_argument("--stream-n", type=int, default=16000000,
                    help="c2: also measure one streaming single frame of this many correspondences "
                         "(roofline_streaming; 0 = skip)")
    ap.add_argument("--plan-only", action="store_true",
                    help="no GPU: start the ranks, shard every workload, gather the partition (CPU test)")
    ap.add_argument("--detail", default=None,
                    help="where rank 0 writes the full result (sample lists, bases, every sub-result); "
                         "default gpurun_out/bench_detail_<workload>_n<N>.json; '-' = nowhere")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    rk = Ranks(args.plan_only)
    try:
        if args.plan_only:
            return plan_only(args, rk)
        import torch  # plumbing only: device sync around the timed region
        if torch.cuda.is_available():
            torch.cuda.set_device(rk.device)
        if args.workload == "c5":
            out = bench_vo(args, rk, torch)
        elif args.workload == "c4":
            out = bench_c4(args, rk, torch)
        else:
            out = bench_frame(args, rk, torch)
        if rk.rank == 0:
            detail = write_detail(out, args, rk.world)
            print(json.dumps(compact_line(out, detail, args.workload in ("c4", "c5")), separators=(",", ":")),
                  flush=True)
    finally:
        rk.close()


def write_detail(out, args, world):
    """The full result (every sample, basis string and sub-result) goes to a side file; the printed
    line (compact_line) keeps the numbers, so the driver's record of the line holds all of them."""
    path = args.detail or os.path.join(ROOT, "gpurun_out", "bench_detail_%s_n%d.json" % (args.workload, world))
    if path == "-":
        return None
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as fh:
            json.dump(out, fh, indent=1)
        return os.path.relpath(path, ROOT)
    except OSError:
        return None


def _r(x, nd=4):
    """Round to nd significant digits (compact line)."""
    if x is None or isinstance(x, (bool, str)):
        return x
    if x == 0:
        return 0
    from math import floor, log10
    return round(x, max(0, nd - 1 - int(floor(log10(abs(x))))))


def _roof_short(roof):
    if not roof:
        return None
    o = {k: _r(roof[k]) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic") if k in roof}
    if "kernel_us" in roof:
        o["kernel_us"] = _r(roof["kernel_us"], 5)
    if "latency" in roof:
        o["latency_frac"] = _r(roof["latency"]["frac"])
        o["round_us"] = _r(roof["latency"]["per_round_us"])
    issue = roof.get("issue") or (roof.get("valu") or {}).get("issue")
    if issue:
        o["issue_frac"] = _r(issue["frac"])
    if "algorithmic_bytes_rate" in roof:
        o["hbm_frac"] = _r(roof["algorithmic_bytes_rate"]["frac"])
    return o


def _sub_short(d):
    """One sub-result (c3 / c4 / c5) in a few numbers."""
    if not d:
        return None
    o = {"value": _r(d.get("value"), 5)}
    if "chain_step_us" not in d:  # a VO figure carries its chain step instead
        o["ms_per_step"] = _r(d.get("ms_per_step"), 5)
    if d.get("roofline"):
        r = _roof_short(d["roofline"])
        o["roofline"] = {k: r[k] for k in ("bound", "frac", "kernel_us", "latency_frac", "issue_frac", "hbm_frac")
                         if k in r}
    for k in ("chain_step_us", "pose_err_vs_oracle_se3", "pose_err_vs_oracle_se3_frame0"):
        if k in d:
            o[k] = _r(d[k], 3)
    if "trajectory" in d:
        o["ate_m"] = _r(d["trajectory"].get("ate_rmse_m", d["trajectory"].get("ate_rmse")), 4)
    for k in ("cpu_baseline", "cpu_baseline_all_cores"):
        if k in d:
            o[k] = _r(d[k]["value"])
    if "projection" in d:
        o["proj_eff"] = {k: v["efficiency"] for k, v in d["projection"].items() if k.startswith("n")}
    if "per_rank" in d and "n8" in d["per_rank"]:
        o["per_rank_n8"] = _r(d["per_rank"]["n8"]["value"])
    if "projection_n8" in d:
        o["proj_eff_n8"] = d["projection_n8"]["efficiency"]
    if "per_rank_n8" in d:
        o["per_rank_n8"] = {"value": _r(d["per_rank_n8"]["value"]), "chain_step_us": d["per_rank_n8"].get("chain_step_us")}
    if "rounds_sync" in d:
        o["rounds_sync"] = d["rounds_sync"]["ratio"]
    if "essential_boot" in d:
        q = d["essential_boot"]
        o["essential_boot"] = {"value": _r(q["value"]), "ate_m": _r(q["trajectory"].get("ate_rmse_m"), 4),
                               "rot_err_deg_max": _r(q["bootstrap"].get("rot_err_deg_max"), 3)}
    if "gt_anchored_250" in d:
        q = d["gt_anchored_250"]
        o["gt_anchored_250"] = {"value": _r(q["value"]), "ate_m": _r(q["trajectory"].get("ate_rmse_m"), 4),
                                "proj_eff_n8": q.get("projection_n8", {}).get("efficiency"),
                                "per_rank_n8": _r(q["per_rank_n8"]["value"]) if "per_rank_n8" in q else None}
    return o


def compact_line(out, detail, sub_fields=False):
    """The printed JSON line: the driver contract's keys first, then every sub-result's numbers,
    in well under 2 KB (the driver keeps only the tail of stdout)."""
    line = {k: out[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                "higher_is_better", "scaling", "vs_baseline", "dtype") if k in out}
    line["data"] = "synthetic (seeded), resident in HBM"
    cfg = out.get("config", {})
    line["config"] = {k: cfg[k] for k in ("workload", "n_corr", "rounds", "frames", "segment_steps", "parallelism")
                      if k in cfg}
    if "workload" in line["config"]:
        line["config"]["workload"] = line["config"]["workload"].split(",")[0]
    line["roofline"] = _roof_short(out.get("roofline"))
    if "cpu_baseline" in out:
        c = out["cpu_baseline"]
        line["cpu_baseline"] = {"value": _r(c["value"]), "unit": c["unit"], "cores": c["cores"], "kind": c["kind"],
                                "sample": c["sample"].split(" of one")[0]}
    for k in ("pose_err_vs_oracle_se3", "pose_err_vs_oracle_se3_frame0"):
        if k in out:
            line[k] = _r(out[k], 3)
    if "cpu_baseline_all_cores" in out:
        line["cpu_all_cores"] = {"value": _r(out["cpu_baseline_all_cores"]["value"]),
                                 "cores": out["cpu_baseline_all_cores"]["cores"]}
    if "timing" in out:
        line["spread"] = out["timing"].get("spread")
    for k in ("c3", "c4", "c5"):
        if k in out:
            line[k] = _sub_short(out[k])
    if sub_fields:  # a c4 / c5 line of its own: its projections, trajectory, chain step
        for k, v in (_sub_short(out) or {}).items():
            line.setdefault(k, v)
    if "roofline_streaming" in out:
        q = out["roofline_streaming"]
        line["stream16m"] = {"frac": _r(q["frac"]), "kernel_us": _r(q["kernel_us"]), "traffic": q.get("traffic")}
    if "with_convergence" in out:
        line["with_conv_its"] = _r(out["with_convergence"]["iterations_per_s"])
    if "keep_outliers_true" in out:
        line["keep_outliers_its"] = _r(out["keep_outliers_true"]["iterations_per_s"])
    if "ranks" in out:
        line["world_size_observed"] = out["ranks"].get("world_size_observed")
    line["detail"] = detail
    return line


def _sync(torch):
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def pmc_traffic(name, fetch_scale=2.0):
    """HBM bytes per launch from the newest committed rocprofv3 PMC passes of the same command
    (profiles/rNN/<name>_pmc_{FETCH_SIZE,WRITE_SIZE}.json, written by tools/gpu_pmc*.sh from two
    separate --pmc passes).  FETCH_SIZE x fetch_scale (gfx950: x2 for wide coalesced streams,
    MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both in KiB.  (None, None) when absent: bench.py
    cannot collect PMC counters live."""
    import glob
    dirs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9]*")))
    for d in reversed(dirs):
        f, w = (os.path.join(d, "%s_pmc_%s.json" % (name, c)) for c in ("FETCH_SIZE", "WRITE_SIZE"))
        if os.path.exists(f) and os.path.exists(w):
            fk = json.load(open(f))["FETCH_SIZE"]["mean"]
            wk = json.load(open(w))["WRITE_SIZE"]["mean"]
            src = "%s (FETCH_SIZE %.1f KiB x %g + WRITE_SIZE %.1f KiB per launch)" % (
                os.path.relpath(f, ROOT).replace("FETCH_SIZE", "{FETCH,WRITE}_SIZE"), fk, fetch_scale, wk)
            return round((fk * fetch_scale + wk) * 1024.0), src
    return None, None


def _kernel_name(mode):
    return {"graph": "picp_round_kernel (one GN round per launch)",
            "persistent": "picp_persistent_kernel (all GN rounds in one launch)",
            "block": "picp_block_kernel (all GN rounds, one block per frame)"}[mode]


def _roofline(b, R, launch_us, pmc_name):
    """Roofline of the batch's dominant kernel from the mean launch period of the timed region."""
    info = b.info()
    corr_per_launch = int(info["total_corr"]) * (1 if info["mode"] == "graph" else R)
    per_launch = BYTES_PER_CORR * corr_per_launch
    achieved = per_launch / (launch_us * 1e-6) / 1e9 if launch_us > 0 else 0.0
    traffic, tsrc = pmc_traffic(pmc_name) if pmc_name else (None, None)
    out = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "traffic_source": tsrc,
           "kernel": _kernel_name(info["mode"]), "mode": info["mode"], "kernel_us": round(launch_us, 3),
           "bytes_per_launch": per_launch, "blocks_per_launch": info["n_blocks"]}
    # the FP32 vector view: 160 flops per correspondence-round over the same launch period, against
    # the FP32 vector peak (SIMD-32, plain v_fma_f32)
    tfs = FLOPS_PER_CORR * corr_per_launch / (launch_us * 1e-6) / 1e12 if launch_us > 0 else 0.0
    out["valu"] = {"achieved": round(tfs, 3), "peak": VALU_PEAK_TFS, "unit": "TFLOP/s",
                   "frac": round(tfs / VALU_PEAK_TFS, 5), "flops_per_launch": FLOPS_PER_CORR * corr_per_launch}
    issue = pmc_issue(pmc_name, launch_us) if pmc_name else None
    if issue:
        out["valu"]["issue"] = issue
    return out


def pmc_issue(name, launch_us):
    """VALU issue-bound fraction of a launch from the newest committed SQ pass of the same command
    (profiles/rNN/<name>_pmc_SQ.json: SQ_INSTS_VALU = wave-instructions per launch): the issue
    capacity of one launch is 1024 SIMDs x one wave64 VALU instruction per 2 cycles (SIMD-32,
    MI355X_MICROARCH.md; measured by tools/ubench/issue_ubench.hip) over the launch's busy cycles."""
    import glob
    for d in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9]*")))):
        f = os.path.join(d, "%s_pmc_SQ.json" % name)
        if os.path.exists(f):
            q = json.load(open(f))
            valu = q["SQ_INSTS_VALU"]["mean"]
            if "GRBM_GUI_ACTIVE" in q:
                # the profiled launch's own busy cycles (GRBM_GUI_ACTIVE summed over the 8 XCDs):
                # capacity = 1024 SIMDs x those cycles / 4, independent of the clock it ran at
                cyc = q["GRBM_GUI_ACTIVE"]["mean"] / 8.0
                cap = SIMDS * cyc / VALU_ISSUE_CYCLES
                basis = ("SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE/8 cycles / %d cycles per wave64 VALU), both "
                         "from the same profiled launches" % VALU_ISSUE_CYCLES)
            else:
                cap = SIMDS * launch_us * 1e-6 * CLOCK_GHZ * 1e9 / VALU_ISSUE_CYCLES
                basis = "SQ_INSTS_VALU / (1024 SIMDs x launch time x 2.4 GHz / %d cycles per wave64 VALU)" % (
                    VALU_ISSUE_CYCLES)
            out = {"valu_wave_instr_per_launch": valu, "issue_capacity_per_launch": round(cap),
                   "frac": round(valu / cap, 4), "source": os.path.relpath(f, ROOT), "basis": basis}
            if "SQ_WAVES" in q:
                out["valu_per_wave"] = round(valu / max(q["SQ_WAVES"]["mean"], 1.0), 1)
            return out
    return None


def _resident_bound(roof):
    """Sub-results whose frames stay in registers/LDS across rounds (counter traffic far below the
    algorithmic bytes) are bound by VALU issue, not HBM: report the FP32 vector roofline as the
    bound, the algorithmic-bytes rate beside it."""
    if roof.get("traffic") is not None and roof["traffic"] < 0.25 * roof["bytes_per_launch"]:
        v = roof.pop("valu")
        roof["algorithmic_bytes_rate"] = {k: roof.pop(k) for k in ("achieved", "peak", "unit", "frac")}
        roof.update({"bound": "valu", **v})
    return roof


def _timed(rk, torch, fn):
    """barrier + device sync on both sides of fn(); wall seconds, max over ranks (RCCL)."""
    rk.barrier()
    _sync(torch)
    t0 = time.perf_counter()
    res = fn()
    _sync(torch)
    rk.barrier()
    el = time.perf_counter() - t0
    return rk.max([el])[0], res


def _timed_samples(rk, torch, fn, samples):
    """BASELINE.md §"how measured": the timed region (barrier + sync on both sides, max over ranks)
    repeated `samples` times; returns (median elapsed, that sample's fn() result, every elapsed)."""
    runs = [_timed(rk, torch, fn) for _ in range(max(1, samples))]
    order = sorted(range(len(runs)), key=lambda i: runs[i][0])
    med = order[len(order) // 2]
    return runs[med][0], runs[med][1], [r[0] for r in runs]


def _sample_info(elapsed_all, steps, units_per_step, unit):
    rates = sorted(units_per_step * steps / e for e in elapsed_all)
    return {"samples": len(elapsed_all), "statistic": "median over %d timed regions of %d steps each" % (
        len(elapsed_all), steps), "values": [round(r, 2) for r in rates], "unit": unit,
        "spread": round((rates[-1] - rates[0]) / rates[len(rates) // 2], 4) if rates else None}


def bench_frame(args, rk, torch):
    """C2 (headline) / C3: one independent frame per rank, R rounds per step."""
    import picp_amd
    from picp_amd import synth
    wl = WORKLOADS[args.workload]
    n = args.n or wl["n"]
    R = args.rounds
    p = synth.make_problem(n, seed=42 + rk.rank, outlier_frac=wl["outlier"], pixel_noise=0.5, shuffle=False)
    xyz, uv, T_init, T_gt = p["xyz"], p["uv"], p["T_init"][None], p["T_gt"][None]
    b = picp_amd.Batch([n], device=rk.device)
    b.set_data(xyz, uv)
    b.set_poses(T_init)
    params = dict(threshold=THRESHOLD, max_rounds=R, conv_eps=-1.0)
    for _ in range(args.warmup):
        b.solve_async(**params)
    b.sync()
    # the K timed steps: K back-to-back fused solves on the library's stream, between HIP events;
    # the region is timed args.samples times and the median reported (median of >= 5)
    elapsed, (ev_ms, launch_us), el_all = _timed_samples(rk, torch, lambda: b.time(args.steps, **params),
                                                         args.samples)
    T_gpu = b.poses()[0]
    err = rk.max([synth.se3_log_norm(T_gpu, T_gt[0])])[0]

    info = b.info()
    default_cfg = (n == wl["n"] and R == 50)
    pmc_name = {("c2", "persistent"): "c2_persistent", ("c3", "persistent"): "c3_persistent"}.get(
        (args.workload, info["mode"])) if default_cfg else None
    roof = _roofline(b, R, launch_us, pmc_name)
    roof["timed_region_event_ms"] = round(ev_ms, 4)
    if info["mode"] == "persistent":
        roof["latency"] = _latency(launch_us, R, info["n_blocks"])
    value = rk.world * R * args.steps / elapsed
    out = {
        "metric": "PICP iterations/sec @ %d correspondences" % n,
        "value": round(value, 2),
        "unit": "iterations/s",
        "n_gpus": rk.world,
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
            "frames_per_gpu": 1,
            "rounds": R,
            "threshold": THRESHOLD,
            "convergence_test": "disabled for timing",
            "parallelism": ("independent frames (seed 42 + rank), one process per GPU, RCCL world %d" % rk.world)
                           if rk.world > 1 else "single GPU",
        },
        "timing": _sample_info(el_all, args.steps, rk.world * R, "iterations/s"),
        "roofline": roof,
        "pose_err_vs_gt_se3": err,
        "residency": b.residency(),
    }
    if rk.world > 1:
        out["ranks"] = {"world_size_observed": rk.comm.world, "partition": "rank r solves frame seed 42 + r",
                        "scaling_note": "the N > 1 headline is weak scaling: independent replicas, one "
                                        "frame per rank; the c4 sub-result is the strong-scaling curve "
                                        "(the fixed 1024-frame batch split over the ranks)"}
    if not args.skip_extras:
        # diagnostic after the timed region: one solve with an event pair around its launch
        out["roofline"]["kernel_us_event_pair"] = round(b.time_single(**params), 3)
    if args.workload in ("c2", "c3") and not args.skip_extras and rk.world == 1:
        # C2 is timed with exactly R rounds; also report the icp_test loop with its
        # convergence test on (exec/icp_test.cpp:99-106), measured after the timed region
        cparams = dict(params, conv_eps=1e-5)
        b.solve(**cparams)
        rounds_run = int(b.stats()[0]["rounds"])
        cms, _ = b.time(args.steps, **cparams)
        per_solve_ms = cms / args.steps
        out["with_convergence"] = {
            "conv_eps": 1e-5, "rounds_run": rounds_run, "ms_per_solve": round(per_solve_ms, 4),
            "iterations_per_s": round(rounds_run / (per_solve_ms * 1e-3), 1),
            "pose_err_vs_gt_se3": synth.se3_log_norm(b.poses()[0], T_gt[0]),
        }
    if args.workload == "c3" and not args.skip_extras and rk.world == 1:
        out["keep_outliers_true"] = _keep_outliers_leg(b, T_init, T_gt, params, args.steps)
    if rk.rank == 0 and rk.world == 1 and not args.no_cpu:
        out["cpu_baseline"], T_or = cpu_baseline(xyz, uv, T_init[0], R, args.cpu_seconds)
        # parity of the timed frame: the GPU's pose after the timed solves vs the faithful oracle's
        # solve of the same frame from the same prior (the cpu_baseline leg's last solve)
        out["pose_err_vs_oracle_se3"] = synth.se3_log_norm(T_gpu, T_or)
        out["pose_err_vs_oracle_note"] = ("SE(3) log norm, GPU %d-round solve vs the oracle's faithful float32 "
                                          "restatement of the reference (north_star tolerance 1e-4)" % R)
        out["cpu_baseline_all_cores"] = cpu_baseline_mt(xyz, uv, T_init[0], R, max(2.0, args.cpu_seconds / 2))
    del b
    if args.workload == "c2" and not args.skip_extras:
        if args.stream_n > 0 and rk.world == 1:
            out["roofline_streaming"] = streaming_roofline(args.stream_n, R, rk.device)
        # the other BASELINE configs, compact, on the same line (bounded time)
        sub = argparse.Namespace(**vars(args))
        sub.steps = max(5, min(args.steps, 10))
        sub.warmup = 2
        sub.cpu_seconds = 3.0
        sub.n = sub.problems = sub.frames = sub.obs = 0
        out["c4"] = _compact(bench_c4(sub, rk, torch))
        if rk.world == 1:
            out["c4"]["per_rank"], out["c4"]["projection"] = _c4_projection(sub, rk, torch, out["c4"]["value"])
        if rk.world == 1:
            sub.workload = "c3"
            sub.skip_extras = True
            sub.cpu_seconds = 5.0
            c3 = bench_frame(sub, rk, torch)
            c3["roofline"] = _resident_bound(c3["roofline"])
            out["c3"] = _compact(c3)
        # C5: SURVEY.md §8e's own partition leads -- 8 contiguous segments of
        # 1,250 steps (one per GPU of an 8-GPU node; here all 8 on this rank's GPU(s)), each
        # bootstrapped from its ground-truth pose pair; the same partition with the reference's
        # two-view bootstrap (match_points + findEssentialMat/recoverPose, exec/icp_test.cpp:44-58)
        # beside it; the 250 gt-anchored 40-step segments are a labelled side figure.
        F = args.frames or WORKLOADS["c5"]["frames"]
        L8 = -(-(F - 1) // 8)
        sub8 = argparse.Namespace(**vars(sub))
        sub8.steps, sub8.warmup, sub8.samples = 2, 1, 3
        c5_250 = bench_vo(sub, rk, torch)
        if rk.world <= 8:  # 8 segments: a world of more ranks would leave some with none
            c5 = _compact(bench_vo(sub8, rk, torch, seg_len=L8, tag="c5_8e"))
            ess = argparse.Namespace(**vars(sub8))
            ess.c5_boot = "essential"
            c5["essential_boot"] = _compact(bench_vo(ess, rk, torch, seg_len=L8, tag="c5_8e_ess"))
        else:
            c5 = {}
        g = _compact(c5_250)
        if rk.world == 1:
            # the per-rank shapes at N = 8 on this GPU alone: the 8e partition's one segment per
            # rank, and rank 0's 32 of the 250 segments
            total8 = c5["value"] * c5["ms_per_step"] * 1e-3  # frames per run
            n8 = bench_vo(sub8, rk, torch, seg_len=L8, shard=(8, 0), tag="c5_8e_n8")
            c5["per_rank_n8"] = _compact(n8)
            c5["projection_n8"] = {
                "projected_value": round(total8 / (n8["ms_per_step"] * 1e-3), 1),
                "efficiency": round(total8 / (n8["ms_per_step"] * 1e-3) / (8 * c5["value"]), 4),
                "basis": "the 8 segments' frames / the time of rank 0's share (1 of 8 segments, 1,250 dependent "
                         "steps) alone on one GPU"}
            n8 = bench_vo(sub, rk, torch, shard=(8, 0), tag="c5_n8")
            total = g["value"] * g["ms_per_step"] * 1e-3
            g["per_rank_n8"] = _compact(n8)
            g["projection_n8"] = {
                "projected_value": round(total / (n8["ms_per_step"] * 1e-3), 1),
                "efficiency": round(total / (n8["ms_per_step"] * 1e-3) / (8 * g["value"]), 4),
                "basis": "the whole sequence's frames / the time of rank 0's share (32 of 250 segments) alone on one "
                         "GPU: every rank still runs its segments' 40 dependent steps, so the time per run falls "
                         "with the width of each step, not with the step count"}
        for k in ("cpu_baseline", "cpu_baseline_all_cores"):  # measured on the 40-step segments
            if k in g:
                c5[k] = g[k]
        c5["gt_anchored_250"] = g
        out["c5"] = c5
    return out


def _compact(d):
    keep = ("metric", "value", "unit", "n_gpus", "steps", "ms_per_step", "scaling", "timing", "roofline",
            "cpu_baseline", "cpu_baseline_all_cores",
            "pose_err_vs_gt_se3", "pose_err_vs_gt_se3_max", "pose_err_vs_oracle_se3", "pose_err_vs_oracle_note",
            "pose_err_vs_oracle_se3_frame0", "trajectory", "chain_step_us", "per_rank", "projection",
            "kernel_us", "kernel", "traffic", "traffic_source",
            "picp_iterations_per_s", "ranks", "config", "bootstrap", "rounds_sync")
    out = {k: d[k] for k in keep if k in d}
    if "config" in out:
        out["config"] = {k: v for k, v in out["config"].items()
                         if k in ("workload", "frames_total", "frames", "parallelism", "partition", "segments",
                                  "segment_steps")}
    return out


def _latency(launch_us, R, n_blocks):
    """The persistent kernel against its per-round communication floor.  A round is one fan-in of
    every block's partial to the leader and one broadcast of the new pose back to every block.
    MI355X_MICROARCH.md's price list has that exact pair as a row ("fanin": a 1->255 broadcast plus
    its 255->1 fan-in, 4.2-4.6 us idle, the fan-in at ~11-13 ns per arrival); scaled to this
    launch's n_blocks at 12 ns per arrival below 255, from the row's low end.  The compute on the
    round's critical path (the linearize, the combine, the 6x6 solve) is not in the floor, so
    frac < 1 by that much even with perfect hand-offs; two idle handoff-1to1 hops (1.6 us) are
    the unreachable lower bound that ignores the arrival cost and is kept beside it."""
    per_round = launch_us / max(R, 1)
    floor = round(max(2 * HANDOFF_US, FANIN_PAIR_US - FANIN_ARRIVAL_US * max(0, 255 - n_blocks)), 3)
    return {"per_round_us": round(per_round, 3), "floor_us": floor, "frac": round(floor / per_round, 4),
            "floor_basis": "MI355X_MICROARCH.md fanin row: 1->255 broadcast + 255->1 fan-in 4.2 us idle, "
                           "minus %.3f us per arrival for the %d blocks of this launch; compute on the "
                           "critical path excluded" % (FANIN_ARRIVAL_US, n_blocks),
            "two_hop_bound_us": 2 * HANDOFF_US,
            "phases": "DESIGN.md §4.3 (stamp logs under profiles/)"}


def _keep_outliers_leg(b, T_init, T_gt, params, steps):
    """also with keep_outliers = true (outliers weighted by the robust
    lambda = sqrt(threshold / chi), src/picp_solver.cpp:80-88), measured after the timed region."""
    from picp_amd import synth
    kparams = dict(params, keep_outliers=1)
    b.set_poses(T_init)
    b.solve(**kparams)
    kerr = synth.se3_log_norm(b.poses()[0], T_gt[0])
    kms, _ = b.time(steps, **kparams)
    return {"rounds": params["max_rounds"], "ms_per_solve": round(kms / steps, 4),
            "iterations_per_s": round(params["max_rounds"] / (kms / steps * 1e-3), 1),
            "pose_err_vs_gt_se3": kerr,
            "note": "outliers are weighted by the robust lambda, not rejected: the pose is biased by them "
                    "by design (the reference's keep_outliers mode); parity with the oracle is tested"}


def bench_c4(args, rk, torch, shard=None):
    """C4: the fixed batch of 1024 frames x 10k split over the ranks (picp_shard_range); one step =
    one fused 50-round solve of this rank's frames; the timed region ends with the RCCL all-gather
    of every frame's pose + stats to every rank (C-ABI picp_batch_allgather).
    shard=(world, rank): that rank's frames solved on this GPU alone (the per-rank shape of an
    N-GPU run, no all-gather)."""
    import numpy as np
    import picp_amd
    from picp_amd import synth
    wl = WORKLOADS["c4"]
    n = args.n or wl["n"]
    total = args.problems or wl["problems"]
    R = args.rounds
    solo = shard is not None
    if solo:  # this GPU alone: no barriers, max or gather over the ranks
        rk = _Solo(rk.device)
    f0, f1 = picp_amd.shard_range(total, *(shard if solo else (rk.world, rk.rank)))
    bt = synth.make_batch(f1 - f0, n, base_seed=1000, first=f0, outlier_frac=0.0, pixel_noise=0.5)
    b = picp_amd.Batch(bt["sizes"], device=rk.device)
    b.set_data(bt["xyz"], bt["uv"])
    b.set_poses(bt["T_init"])
    params = dict(threshold=THRESHOLD, max_rounds=R, conv_eps=-1.0)
    for _ in range(max(args.warmup, 1)):
        b.solve_async(**params)
    b.sync()

    def job():
        r = b.time(args.steps, **params)
        if getattr(rk, "comm", None) is not None:
            return r, rk.comm.allgather_batch(b, total)[0]
        return r, b.poses()

    elapsed, ((ev_ms, launch_us), allT), el_all = _timed_samples(rk, torch, job, args.samples)
    err = max(synth.se3_log_norm(b.poses()[i], bt["T_gt"][i]) for i in range(f1 - f0))
    err = rk.max([err])[0]
    mine = np.array_equal(allT[f0:f1], b.poses())  # the gather put this rank's rows in place
    info = b.info()
    # PMC passes of the same kernel shape (tools/r04/gpu_prof_r04.sh): 1024 frames on one GPU, or
    # the 128-frame per-rank shape of an 8-GPU run
    shape = {1024: "c4x1024_block", 128: "c4x128"}.get(f1 - f0)
    pmc = shape if (info["mode"] == "block" and n == wl["n"] and R == 50 and (rk.world == 1 or solo)) else None
    roof = _resident_bound(_roofline(b, R, launch_us, pmc))
    if solo:  # this GPU solved f1 - f0 of the batch's frames
        out = {"frames": f1 - f0, "value": round((f1 - f0) * R * args.steps / elapsed, 2), "unit": "iterations/s",
               "ms_per_step": round(1000.0 * elapsed / args.steps, 4), "kernel_us": round(launch_us, 3),
               "mode": b.info()["mode"], "blocks": b.info()["n_blocks"], "handoff_grid": b.residency()["handoff_grid"],
               "timing": _sample_info(el_all, args.steps, (f1 - f0) * R, "iterations/s"), "pose_err_vs_gt_se3": err,
               "roofline": {k: roof[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                 "traffic_source", "issue") if k in roof}}
        del b
        return out
    out = {
        "metric": "PICP iterations/sec, batch of %d frames x %d correspondences" % (total, n),
        "value": round(total * R * args.steps / elapsed, 2),
        "unit": "iterations/s",
        "n_gpus": rk.world,
        "steps": args.steps,
        "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
        "scaling": "strong",
        "timing": _sample_info(el_all, args.steps, total * R, "iterations/s"),
        "roofline": roof,
        "pose_err_vs_gt_se3": err,
        "config": {"workload": wl["desc"], "frames_total": total, "frames_this_rank": f1 - f0,
                   "parallelism": "picp_shard_range over %d ranks, one RCCL all-gather of results per job" % rk.world
                   if rk.world > 1 else "single GPU"},
    }
    if rk.world > 1:
        out["ranks"] = {"world_size_observed": rk.comm.world,
                        "partition": [list(picp_amd.shard_range(total, rk.world, r)) for r in range(rk.world)],
                        "allgather_rows_match_local": bool(rk.max([0.0 if mine else 1.0])[0] == 0.0)}
    if rk.rank == 0 and rk.world == 1 and not args.no_cpu:
        sz = int(bt["sizes"][0])
        out["cpu_baseline"], T_or = cpu_baseline(bt["xyz"][:sz], bt["uv"][:sz], bt["T_init"][0], R, args.cpu_seconds)
        out["pose_err_vs_oracle_se3_frame0"] = synth.se3_log_norm(b.poses()[0], T_or)
        out["cpu_baseline_all_cores"] = cpu_baseline_batch_mt(bt, R, args.cpu_seconds)
    return out


def _c4_projection(args, rk, torch, v1):
    """The per-rank shapes of the N = 2, 4, 8 C4 runs (the fixed 1024-frame batch split over N
    GPUs: rank 0's 512, 256, 128 frames), each solved on this GPU alone.  projected_value = the
    whole batch's rounds / the per-rank time (ranks are independent and equal-sized; the job's one
    128-KB RCCL all-gather of the results is not included: it cannot be timed on one GPU, and it
    is one collective per K-step job); efficiency = projected / (N x the 1-GPU value)."""
    wl = WORKLOADS["c4"]
    total = args.problems or wl["problems"]
    per, proj = {}, {}
    for N in (2, 4, 8):
        r = bench_c4(args, rk, torch, shard=(N, 0))
        per["n%d" % N] = r
        pv = r["value"] * total / r["frames"]
        proj["n%d" % N] = {"projected_value": round(pv, 1), "efficiency": round(pv / (N * v1), 4) if v1 else None}
    proj["basis"] = ("per-rank time of rank 0's share measured on one GPU; excludes the all-gather of the results "
                     "(one per job); the driver's multi-GPU run measures the real curve")
    return per, proj


def streaming_roofline(n, R, device):
    """The same solve on one frame large enough to stream from HBM every round (SURVEY.md §8d:
    a > 256 MB working set, past the 256 MB Infinity Cache): 20 B x n per round-launch of
    picp_round_kernel.  Reported beside the C2 line, whose single 100k frame is latency-bound."""
    import picp_amd
    from picp_amd import synth
    p = synth.make_problem(n, seed=7, pixel_noise=0.5, shuffle=False)
    b = picp_amd.Batch([n], device=device)
    b.set_data(p["xyz"], p["uv"])
    b.set_poses(p["T_init"][None])
    params = dict(threshold=THRESHOLD, max_rounds=R, conv_eps=-1.0)
    b.solve(**params)
    ev_ms, launch_us = b.time(5, **params)
    info = b.info()
    graph = info["mode"] == "graph"
    per_launch = BYTES_PER_CORR * n * (1 if graph else R)
    achieved = per_launch / (launch_us * 1e-6) / 1e9
    err = synth.se3_log_norm(b.poses()[0], p["T_gt"])
    traffic, tsrc = pmc_traffic("stream16m") if (n == 16000000 and graph) else (None, None)
    return {"bound": "hbm", "n_corr": n, "working_set_MB": round(BYTES_PER_CORR * n / 1e6, 1),
            "kernel": _kernel_name(info["mode"]), "mode": info["mode"], "blocks_per_launch": info["n_blocks"],
            "kernel_us": round(launch_us, 3), "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "traffic_source": tsrc,
            "bytes_per_launch": per_launch, "iterations_per_s": round(R * 5 / (ev_ms * 1e-3), 2),
            "pose_err_vs_gt_se3": err}


_VO_CACHE = {}


def _vo_frames(F, obs, fa, fb):
    """The synthetic sequence (seed 42) and its packed frames fa .. fb (cached: the C5 lines share
    one sequence)."""
    from picp_amd.vo_synth import VOSequence
    key = (F, obs)
    if key not in _VO_CACHE:
        _VO_CACHE.clear()
        _VO_CACHE[key] = (VOSequence(F, obs_per_frame=obs, seed=42), {})
    seq, frames = _VO_CACHE[key]
    if (fa, fb) not in frames:
        frames.clear()
        frames[(fa, fb)] = seq.frames(fa, fb + 1)
    return seq, frames[(fa, fb)]


def bench_vo(args, rk, torch, seg_len=None, shard=None, tag="c5"):
    """C5: the whole sequence is split into contiguous segments of seg_len (--seg-len) PICP steps
    (one-frame overlap); ranks take contiguous ranges of segments (strong scaling:
    the sequence is fixed).  One step = one run of this rank's segments (pair matching of all its
    frames, bootstrap, then per frame: world match, PICP block kernel with the gather fused in,
    triangulate/append).  value = frames estimated by all ranks / max-over-ranks time.
    shard=(world, rank): run that rank's share of the partition on this GPU alone (the per-rank
    shape of an N-GPU run, measured on one GPU).
    The line also carries the whole-sequence trajectory: the segments stitched at their one-frame
    overlaps (picp_amd/evaluate.py) and its ATE after the reference's umeyama alignment
    (src/my_utilities.cpp:459-478)."""
    import numpy as np
    import picp_amd
    from picp_amd import synth
    from picp_amd.evaluate import ate, stitch_segments
    from picp_amd.vo_synth import segments
    wl = WORKLOADS["c5"]
    F = args.frames or wl["frames"]
    obs = args.obs or wl["obs"]
    L = seg_len or args.seg_len
    first, steps = segments(F, L)
    world, rank = shard if shard else (rk.world, rk.rank)
    s0, s1 = picp_amd.shard_range(len(first), world, rank)
    if s1 <= s0:
        raise ValueError("bench_vo: %d segments cannot give each of %d ranks one (--frames / --seg-len)" % (
            len(first), world))
    fa, fb = int(first[s0]), int(first[s1 - 1] + steps[s1 - 1])
    seq, D = _vo_frames(F, obs, fa, fb)
    my_first, my_steps = first[s0:s1] - fa, steps[s0:s1]
    # each segment's world frame is its first camera, as the reference's is frame 0's
    # (exec/icp_test.cpp:36, bootstrap from Identity): float32 coordinates stay segment-sized
    rel = [np.linalg.inv(D["T_cw"][f].astype(np.float64)) for f in my_first]
    scale = np.ones(len(my_first))
    boot_info = {"kind": "ground-truth pose pair of each segment's first two frames (SURVEY.md §8e stand-in)"}
    if args.c5_boot == "essential":
        # the reference's bootstrap (exec/icp_test.cpp:44-58, src/cam.cpp:37-91) per segment, on the
        # GPU, before the timed region (the reference bootstraps once per sequence)
        _sync(torch)
        t0 = time.perf_counter()
        d1 = [D["desc"][D["frame_off"][f]:D["frame_off"][f + 1]] for f in my_first]
        d2 = [D["desc"][D["frame_off"][f + 1]:D["frame_off"][f + 2]] for f in my_first]
        m = picp_amd.match_points_batch(d1, d2, device=rk.device)
        p1s, p2s = [], []
        for k, f in enumerate(my_first):
            acc = np.nonzero(m[k]["accepted"])[0]
            p1s.append(D["uv"][D["frame_off"][f]:D["frame_off"][f + 1]][acc])
            p2s.append(D["uv"][D["frame_off"][f + 1]:D["frame_off"][f + 2]][m[k]["best_idx"][acc]])
        ess = picp_amd.essential_recover_pose_batch(p1s, p2s, K=seq.K, device=rk.device)
        _sync(torch)
        boot_ms = 1e3 * (time.perf_counter() - t0)
        boot = np.stack([[np.eye(4), e["T"]] for e in ess]).astype(np.float32)
        # unit baseline: the drift below is measured after scaling each segment to the ground
        # truth's first baseline (the reference's evaluation aligns scale the same way, umeyama)
        rot_err, dir_err = [], []
        for k, f in enumerate(my_first):
            gt1 = rel[k] @ D["T_cw"][f + 1]
            scale[k] = np.linalg.norm(gt1[:3, 3]) / max(np.linalg.norm(boot[k][1][:3, 3]), 1e-30)
            # the bootstrap's own error vs the ground-truth relative pose: rotation angle and the
            # angle between the translation directions (the scale is not observable)
            Rd = boot[k][1][:3, :3].astype(np.float64).T @ gt1[:3, :3]
            rot_err.append(np.degrees(np.arccos(np.clip((np.trace(Rd) - 1.0) / 2.0, -1.0, 1.0))))
            a, b = boot[k][1][:3, 3].astype(np.float64), gt1[:3, 3]
            dir_err.append(np.degrees(np.arccos(np.clip(a @ b / max(np.linalg.norm(a) * np.linalg.norm(b), 1e-300),
                                                        -1.0, 1.0))))
        boot_info = {"kind": "essential: match_points + findEssentialMat(RANSAC) + recoverPose per segment on the "
                             "GPU (picp_match_points_batch, picp_essential_batch), unit baseline; before the timed "
                             "region", "ms": round(boot_ms, 3), "segments": len(my_first),
                     "not_good": int(sum(1 for e in ess if not e["good"])),
                     "rot_err_deg_max": float(np.max(rot_err)), "rot_err_deg_median": float(np.median(rot_err)),
                     "t_dir_err_deg_max": float(np.max(dir_err)), "t_dir_err_deg_median": float(np.median(dir_err))}
    else:
        boot = np.stack([[np.eye(4), rel[k] @ D["T_cw"][f + 1]] for k, f in enumerate(my_first)]).astype(np.float32)
    vo = picp_amd.VOSequence(D["frame_off"], D["uv"], D["desc"], device=rk.device, K=seq.K)
    vo.set_segments(my_first, my_steps, boot, threshold=THRESHOLD)
    for _ in range(max(args.warmup, 1)):
        vo.run()
    sync_ranks = shard is None  # a per-rank projection runs on this GPU alone
    trk = rk if sync_ranks else _Solo(rk.device)
    elapsed, ev_ms, el_all = _timed_samples(trk, torch, lambda: vo.time(args.steps), args.samples)
    # correctness of what was timed: drift vs gt, PICP work done
    P, Rr, vinfo = vo.poses(), vo.step_records(), vo.info()
    vo.close()
    err, rounds, corr = 0.0, 0, 0
    for k, f0 in enumerate(my_first):
        for t in range(1, len(P[k])):
            gt = rel[k] @ D["T_cw"][f0 + t].astype(np.float64)  # gt in the segment frame
            est = P[k][t].astype(np.float64)
            est[:3, 3] *= scale[k]
            err = max(err, synth.se3_log_norm(est, gt))
        rounds += int(Rr[k]["rounds"][1:].sum())
        corr += int((Rr[k]["rounds"][1:].astype(np.int64) * Rr[k]["n_corr"][1:]).sum())
    err = trk.max([err])[0]
    sync = _rounds_sync([Rr[k]["rounds"][1:] for k in range(len(my_first))])
    tot = trk.gather_obj([rounds, corr, int(my_steps.sum())])
    rounds, corr, frames_total = (sum(t[i] for t in tot) for i in range(3))
    # the whole trajectory: every rank's segments (gathered to all ranks, after timing), stitched
    # at the one-frame overlaps from the ground-truth pose of frame first[s0] (segments in metric
    # scale: gt-booted; essential-booted segments are scaled by their first baseline)
    mine = [_scaled(P[k], scale[k]) for k in range(len(my_first))]
    allP = trk.gather_obj((s0, mine))
    allP.sort(key=lambda x: x[0])
    segs = [p for _, ps in allP for p in ps]
    g0 = allP[0][0]
    gfirst, gsteps = first[g0:g0 + len(segs)], steps[g0:g0 + len(segs)]
    frames, Tst = stitch_segments(segs, gfirst, gsteps, seq.T_cw(int(gfirst[0])))
    traj = ate(Tst, np.stack([seq.T_cw(int(f)) for f in frames]))
    traj["stitching"] = ("%d segments stitched at their one-frame overlaps, anchored at the ground truth of frame %d "
                         "only; ATE after the similarity (umeyama, with scale) alignment of the positions, as "
                         "the reference's alignTrajectories" % (len(segs), int(gfirst[0])))
    out = {
        "metric": "VO frames/sec (%d-frame synthetic sequence, ~%d obs/frame, per-frame match + PICP + triangulate)" % (F, obs),
        "value": round(frames_total * args.steps / elapsed, 2),
        "unit": "frames/s",
        "n_gpus": rk.world if sync_ranks else 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic sequence (picp_amd/vo_synth.py, seed 42; observations resident in HBM)",
        "config": {"workload": wl["desc"], "frames": F, "obs_per_frame": obs, "segment_steps": L,
                   "segments": len(first), "segments_this_rank": s1 - s0,
                   "partition": "%d %s %d-frame segments (%d PICP steps each), each bootstrapped from %s; %d on this "
                                "GPU" % (len(first), "gt-anchored" if args.c5_boot == "gt" else "essential-bootstrapped",
                                         L + 1, L, "its ground-truth pose pair" if args.c5_boot == "gt"
                                         else "the two-view essential matrix", s1 - s0),
                   "threshold": THRESHOLD,
                   "picp_loop": "icp_test: <= 50 rounds, relative chi convergence 1e-5",
                   "parallelism": ("contiguous segment ranges (picp_shard_range), one process per GPU"
                                   if rk.world > 1 else "single GPU") if sync_ranks else
                   "rank %d of %d's share, alone on one GPU (per-rank shape of the %d-GPU run)" % (rank, world, world),
                   "block_npt": vinfo["npt"]},
        "timing": _sample_info(el_all, args.steps, frames_total, "frames/s"),
        "picp_iterations_per_s": round(rounds * args.steps / elapsed, 1),
        "picp_corr_rounds_per_s": round(corr * args.steps / elapsed, 1),
        "chain_step_us": round(1e6 * elapsed / args.steps / max(1, int(my_steps.max())), 2),
        "timed_region_event_ms": round(ev_ms * args.steps, 4),
        "pose_err_vs_gt_se3_max": err,
        "pose_err_frame": "camera-in-world poses in each segment's frame (its first camera)",
        "trajectory": traj,
        "bootstrap": boot_info,
        "rounds_sync": sync,
    }
    if rk.world > 1 and sync_ranks:
        out["ranks"] = {"world_size_observed": rk.comm.world,
                        "partition": [list(picp_amd.shard_range(len(first), rk.world, r)) for r in range(rk.world)]}
    if rk.rank == 0 and rk.world == 1 and not args.no_cpu and tag == "c5":
        out["cpu_baseline"] = cpu_baseline_vo(seq, L, args.cpu_seconds)
        out["cpu_baseline_all_cores"] = cpu_baseline_vo_mt(seq, L, max(2.0, args.cpu_seconds / 2))
    return out


def _rounds_sync(rounds, chains=2):
    """What the per-step synchronisation of a VO run costs in PICP rounds.
    Every step's PICP launch covers one chain's segments (the library's default: two contiguous
    groups, picp_vo_runtime.cpp) and lasts as long as its slowest segment's rounds, so a chain pays
    sum_t max_s rounds[s][t]; a segment alone would pay sum_t rounds[s][t].  ratio = the chains'
    largest sum_t max_s over the largest single-segment sum: 1.0 means desynchronising the segments
    cannot shorten the run (the slowest segment is slow at every step)."""
    import numpy as np
    n = len(rounds)
    C = max(1, min(chains, n))
    T = max(len(r) for r in rounds)
    M = np.zeros((n, T), np.int64)
    for k, r in enumerate(rounds):
        M[k, :len(r)] = r
    per_chain = [int(M[n * c // C:n * (c + 1) // C].max(0).sum()) for c in range(C)]
    solo = int(M.sum(1).max())
    return {"sum_t_max_s": max(per_chain), "max_s_sum_t": solo,
            "ratio": round(max(per_chain) / max(solo, 1), 4), "mean_rounds": round(float(M[M > 0].mean()), 2),
            "steps_at_50_any": int((M.max(0) >= 50).sum()), "steps": T, "chains": C}


def _scaled(P, s):
    """Poses with their translations scaled by s (a unit-baseline segment to metric)."""
    import numpy as np
    Q = np.array(P, np.float64)
    Q[:, :3, 3] *= s
    return Q


class _Solo:
    """Ranks-like stand-in for a measurement that runs on this process's GPU alone."""
    world, rank, comm = 1, 0, None

    def __init__(self, device=0):
        self.device = device

    def barrier(self):
        pass

    def max(self, values):
        return list(values)

    def gather_obj(self, obj):
        return [obj]


def plan_only(args, rk):
    """--plan-only (no GPU, gloo): every rank shards the workloads exactly as a GPU run would,
    builds its C4 inputs, and rank 0 gathers (rank, shard, input checksum) -- the CPU test of the
    multi-process launcher."""
    import numpy as np
    from picp_amd import synth
    from picp_amd.dist import shard_range
    total = args.problems or WORKLOADS["c4"]["problems"]
    n = args.n or 256
    if os.environ.get("PICP_PLAN_FAIL_RANK") == str(rk.rank):  # launcher test: one rank dies
        sys.exit(3)
    f0, f1 = shard_range(total, rk.world, rk.rank)
    bt = synth.make_batch(f1 - f0, n, base_seed=1000, first=f0)
    from picp_amd.vo_synth import segments
    first, _ = segments(args.frames or WORKLOADS["c5"]["frames"], args.seg_len)
    mine = {"rank": rk.rank, "pid": os.getpid(), "local_rank": rk.local, "c2_seed": 42 + rk.rank,
            "c4_frames": [f0, f1], "c4_checksum": float(np.float64(bt["xyz"]).sum() + np.float64(bt["uv"]).sum()),
            "c5_segments": list(shard_range(len(first), rk.world, rk.rank))}
    allm = rk.gather_obj(mine)
    # the C4 results gather in the layout picp_batch_allgather moves over RCCL (padded shards,
    # picp_shard_unpack): here each rank's initial poses stand in for its solved poses
    gather_ok = None
    if rk.dist is not None:
        from picp_amd.dist import gather_rows
        rows = bt["T_init"].reshape(f1 - f0, 16)
        allrows = gather_rows(rows, total, rk.dist)
        full = synth.make_batch(total, n, base_seed=1000)["T_init"].reshape(total, 16)
        gather_ok = bool(np.array_equal(allrows, full))
    if rk.rank == 0:
        print(json.dumps({"plan_only": True, "n_gpus": args.gpus, "world_size_observed": rk.world,
                          "backend": "gloo" if rk.dist is not None else "none", "ranks": allm,
                          "c4_gather_matches_single_process": gather_ok}), flush=True)


CPU_SAMPLES = 5  # every CPU figure is the median of >= 5 samples


def _median_rate(call, budget_s, samples=CPU_SAMPLES, warm=False):
    """call() -> units done; run it for budget_s / samples seconds (at least once) per sample;
    returns (median units/s, sorted per-sample rates, calls, seconds).  warm: one untimed call
    first (thread-pool start-up)."""
    if warm:
        call()
    rates, calls, t_all = [], 0, time.perf_counter()
    for _ in range(samples):
        units, t0 = 0, time.perf_counter()
        while True:
            units += call()
            calls += 1
            el = time.perf_counter() - t0
            if el >= budget_s / samples:
                break
        rates.append(units / el)
    rates.sort()
    return rates[len(rates) // 2], rates, calls, time.perf_counter() - t_all


def _cpu_result(rate, rates, unit, cores, sample):
    return {"value": round(rate, 3), "unit": unit, "cores": cores, "kind": "port",
            "statistic": "median of %d samples" % len(rates), "samples": [round(r, 3) for r in rates],
            "sample": sample}


def _host_threads():
    """The threads a CPU baseline may use: OMP_NUM_THREADS (16 on the GPU box = its CPU share;
    os.cpu_count() shows the whole machine there)."""
    return max(1, min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1), 64))


def cpu_baseline_vo(seq, L, budget_s):
    """Oracle VO loop (faithful float32, 1 thread) over whole segments of the same sequence:
    frames/s, median of CPU_SAMPLES samples."""
    import numpy as np
    import oracle as O
    D = seq.frames(0, min(seq.n_frames, 4 * L + 1))
    state = {"f0": 0}

    def one():
        f0 = state["f0"]
        st = min(L, len(D["frame_off"]) - 2 - f0)
        if st < 1:
            f0, st = 0, min(L, len(D["frame_off"]) - 2)
        T1 = (np.linalg.inv(D["T_cw"][f0].astype(np.float64)) @ D["T_cw"][f0 + 1]).astype(np.float32)
        O.vo_segment(seq.K, 480, 640, D["frame_off"], D["uv"], D["desc"], f0, st, np.eye(4, dtype=np.float32),
                     T1, mode=O.MODE_FAITHFUL)
        state["f0"] = f0 + L
        return st

    rate, rates, calls, el = _median_rate(one, budget_s)
    return _cpu_result(rate, rates, "frames/s", 1,
                       "%d segments of <= %d steps of the same sequence (oracle VO loop, faithful float32, "
                       "gcc -O3, 1 thread) in %.1f s" % (calls, L, el))


def cpu_baseline_vo_mt(seq, L, budget_s):
    """SURVEY.md §8d all-cores variant of the C5 baseline: the oracle VO loop over independent
    segments in parallel, one segment per host thread.  ctypes releases the GIL around
    or_vo_segment, whose VO path keeps no static state, so the threads run concurrently.  Timing
    only, never a parity oracle."""
    import concurrent.futures as cf
    import numpy as np
    import oracle as O
    nt = _host_threads()
    D = seq.frames(0, min(seq.n_frames, nt * L + 1))
    nseg = max(1, (len(D["frame_off"]) - 2) // L)

    def worker(i):
        f0 = (i % nseg) * L
        st = min(L, len(D["frame_off"]) - 2 - f0)
        T1 = (np.linalg.inv(D["T_cw"][f0].astype(np.float64)) @ D["T_cw"][f0 + 1]).astype(np.float32)
        O.vo_segment(seq.K, 480, 640, D["frame_off"], D["uv"], D["desc"], f0, st,
                     np.eye(4, dtype=np.float32), T1, mode=O.MODE_FAITHFUL)
        return st

    with cf.ThreadPoolExecutor(max_workers=nt) as ex:
        rate, rates, calls, el = _median_rate(lambda: sum(ex.map(worker, range(nt))), budget_s, warm=True)
    return _cpu_result(rate, rates, "frames/s", nt,
                       "%d rounds of %d threads, each running one <= %d-step segment of the same sequence "
                       "(oracle VO loop, faithful float32, gcc -O3) in %.1f s on %s" % (calls, nt, L, el, _cpu_model()))


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


KREF = [[180, 0, 320], [0, 180, 240], [0, 0, 1]]  # the synthetic generator's camera


def _soa(xyz, uv):
    import numpy as np
    return [np.ascontiguousarray(xyz[:, i]) for i in range(3)] + [np.ascontiguousarray(uv[:, i]) for i in range(2)]


def cpu_baseline_mt(xyz, uv, T_init, R, budget_s):
    """SURVEY.md §8d's all-cores CPU baseline for C2/C3: the oracle's loop with the linearize as a
    chunked reduction over the host threads.  Timing only (its summation order is not the
    reference's)."""
    import numpy as np
    import oracle as O
    threads = _host_threads()
    cols = _soa(xyz, uv)
    Kref = np.array(KREF, np.float32)

    def one():
        O.solve_soa_mt(T_init, Kref, 480, 640, *cols, THRESHOLD, threads, mode=O.MODE_FAITHFUL,
                       max_rounds=R, conv_eps=-1.0)
        return R

    rate, rates, calls, el = _median_rate(one, budget_s, warm=True)
    return _cpu_result(rate, rates, "iterations/s", threads,
                       "%d x %d-round solves of one %d-correspondence frame (faithful float32 oracle, linearize "
                       "as a chunked reduction over %d OpenMP threads, gcc -O3 -march=x86-64-v3) in %.1f s on %s"
                       % (calls, R, len(cols[0]), threads, el, _cpu_model()))


def cpu_baseline_batch_mt(bt, R, budget_s):
    """BASELINE.md's all-cores C4 baseline: "all-core OpenMP over problems" -- independent frames of
    the batch solved concurrently, one per host thread (the sequential oracle solve per frame;
    ctypes releases the GIL and or_solve_soa keeps no static state)."""
    import concurrent.futures as cf
    import numpy as np
    import oracle as O
    nt = _host_threads()
    Kref = np.array(KREF, np.float32)
    offs = np.concatenate([[0], np.cumsum(bt["sizes"])]).astype(np.int64)
    nf = len(bt["sizes"])
    frames = [_soa(bt["xyz"][offs[i]:offs[i + 1]], bt["uv"][offs[i]:offs[i + 1]]) for i in range(min(nf, nt))]

    def worker(i):
        O.solve_soa(bt["T_init"][i], Kref, 480, 640, *frames[i], THRESHOLD, mode=O.MODE_FAITHFUL,
                    max_rounds=R, conv_eps=-1.0)
        return R

    with cf.ThreadPoolExecutor(max_workers=nt) as ex:
        rate, rates, calls, el = _median_rate(lambda: sum(ex.map(worker, range(len(frames)))), budget_s, warm=True)
    return _cpu_result(rate, rates, "iterations/s", nt,
                       "%d rounds of %d frames of the batch (%d correspondences each) solved concurrently, one "
                       "%d-round sequential oracle solve per thread (faithful float32, gcc -O3 -march=x86-64-v3) "
                       "in %.1f s on %s" % (calls, len(frames), int(bt["sizes"][0]), R, el, _cpu_model()))


def cpu_baseline(xyz, uv, T_init, R, budget_s):
    """Oracle (faithful float32, sequential) single thread on one frame of the workload: whole
    R-round solves, median of CPU_SAMPLES samples (at least one solve each)."""
    import numpy as np
    import oracle as O
    cols = _soa(xyz, uv)
    Kref = np.array(KREF, np.float32)

    last = {}

    def one():
        last["T"], _ = O.solve_soa(T_init, Kref, 480, 640, *cols, THRESHOLD, mode=O.MODE_FAITHFUL, max_rounds=R,
                                   conv_eps=-1.0)
        return R

    rate, rates, calls, el = _median_rate(one, budget_s)
    out = _cpu_result(rate, rates, "iterations/s", 1,
                      "%d x %d-round solves of one %d-correspondence frame (faithful float32 oracle, gcc -O3 "
                      "-march=x86-64-v3, 1 thread) in %.1f s on %s" % (calls, R, len(cols[0]), el, _cpu_model()))
    return out, last["T"]


if __name__ == "__main__":
    main()
