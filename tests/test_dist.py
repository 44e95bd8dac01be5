"""Multi-process batch split on CPU (gloo, world_size 2): shard ranges and the final gather.

Each rank solves its shard of independent synthetic frames (with the CPU oracle standing in
for the device solve: this test covers the split/gather plumbing, the GPU tests cover the
solve), the poses are all-gathered in picp_batch_allgather's layout (shards padded to
picp_shard_pad rows, unpacked by the library's picp_shard_unpack), and rank 0 checks them
against a single-process run.
"""
import os
import socket

import numpy as np
import pytest


def test_shard_range_partitions():
    from picp_amd.dist import shard_range
    for n in (0, 1, 7, 128, 1024, 1025):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            sizes = [e - s for s, e in rs]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def test_shard_pad_unpack_ragged_matches_shard_order():
    """picp_shard_pad / picp_shard_unpack (the host half of picp_batch_allgather, no device):
    ragged shards padded to ceil(n / world) rows and concatenated in rank order come back in
    problem order, bit-exact; picp_shard_range agrees with the Python split."""
    import picp_amd
    from picp_amd.dist import shard_range
    for n, w in ((1025, 8), (9, 2), (5, 8), (0, 3), (7, 1), (128, 3)):
        pad = max(picp_amd.shard_pad(n, w), 1)
        full = np.arange(n * 32, dtype=np.int32).reshape(n, 32)  # a 128-byte PicpState per row
        padded = np.full((w * pad, 32), -1, np.int32)
        for r in range(w):
            a, e = shard_range(n, w, r)
            assert picp_amd.shard_range(n, w, r) == (a, e)
            padded[r * pad:r * pad + e - a] = full[a:e]
        np.testing.assert_array_equal(picp_amd.shard_unpack(padded, n, w), full)
    with pytest.raises(picp_amd.PicpError):
        picp_amd.shard_pad(4, 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _solve_frames(first, last, n_corr):
    import oracle as O
    from picp_amd import synth
    out = []
    for i in range(first, last):
        p = synth.make_problem(n_corr, seed=1000 + i, shuffle=False, pixel_noise=0.5)
        T, st = O.solve_soa(p["T_init"], p["K"], 480, 640, p["x"], p["y"], p["z"], p["u"], p["v"],
                            3000.0, max_rounds=20, conv_eps=-1.0)
        out.append(np.concatenate([T.T.reshape(-1), [st["chi_in"], st["n_in"]]]))
    return np.array(out, np.float32).reshape(-1, 18)


def _worker(rank, world, port, n_frames, n_corr, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "02-visualodometry_amd"), os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from picp_amd.dist import gather_rows, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s, e = shard_range(n_frames, world, rank)
    rows = _solve_frames(s, e, n_corr)
    allrows = gather_rows(rows, n_frames, dist)
    if rank == 0:
        q.put(allrows)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_split_and_gather_matches_single_process():
    import torch.multiprocessing as mp
    n_frames, n_corr = 5, 800  # odd count: ragged shards
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_frames, n_corr, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _solve_frames(0, n_frames, n_corr)
    np.testing.assert_array_equal(got, ref)


def test_bench_launcher_gpus2_plan_only_starts_shards_and_gathers():
    """`bench.py --gpus 2` (no WORLD_SIZE: the launcher starts the ranks itself, as the driver
    invokes it) in --plan-only mode (gloo, no device): two distinct rank processes start, shard
    C2 / C4 / C5 exactly as a GPU run would, and rank 0 gathers every rank's partition and the
    checksum of the C4 inputs it built."""
    import json
    import subprocess
    import sys
    from picp_amd import synth
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--plan-only",
                        "--problems", "9", "--n", "64", "--frames", "200"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["plan_only"] and out["n_gpus"] == 2 and out["world_size_observed"] == 2
    assert out["c4_gather_matches_single_process"] is True  # 9 frames over 2 ranks: padded 5 + 4
    ranks = out["ranks"]
    assert [x["rank"] for x in ranks] == [0, 1] and ranks[0]["pid"] != ranks[1]["pid"]
    assert [x["c4_frames"] for x in ranks] == [[0, 5], [5, 9]]
    assert [x["c2_seed"] for x in ranks] == [42, 43]
    # 200 frames in 40-step segments -> 5 segments: 3 + 2
    assert [x["c5_segments"] for x in ranks] == [[0, 3], [3, 5]]
    for x in ranks:
        f0, f1 = x["c4_frames"]
        bt = synth.make_batch(f1 - f0, 64, base_seed=1000, first=f0)
        assert x["c4_checksum"] == float(np.float64(bt["xyz"]).sum() + np.float64(bt["uv"]).sum())


def test_bench_launcher_one_failing_rank_ends_the_job():
    """A rank that dies (here rank 1, before the gather its peer blocks in) must end the whole
    launch with a failure, not leave rank 0 waiting in a collective forever (rank 0 may see the
    broken connection and fail first: either exit code is a failure)."""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PICP_PLAN_FAIL_RANK"] = "1"
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--plan-only",
                        "--problems", "9", "--n", "64", "--frames", "200"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode != 0, (r.returncode, r.stderr[-2000:])
    assert time.time() - t0 < 200


def _host_exchange_null_worker(rank, world, port, q):
    import ctypes
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "02-visualodometry_amd"))
    import torch
    import torch.distributed as dist
    import picp_amd
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def exchange(buf):
        calls.append(len(buf))
        t = torch.frombuffer(bytearray(buf), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return b"".join(o.numpy().tobytes() for o in out)

    class NoBatch:  # a rank with no batch: its local check fails
        _b = ctypes.c_void_p()

    try:
        picp_amd.allgather_batch_host(NoBatch(), world, rank, 5, exchange)
        q.put((rank, "no error", calls))
    except picp_amd.PicpError as e:
        q.put((rank, str(e), calls))
    dist.barrier()
    dist.destroy_process_group()


def test_host_exchange_gather_failure_needs_no_second_collective():
    """picp_batch_allgather_host (CPU, gloo world 2, no device): a rank whose local check fails
    (here: no batch at all) still takes part in the ONE exchange -- its status header travels in
    it -- and returns an error; no rank waits in a collective the other never enters.  The GPU
    suite runs the successful gather at world 2 and 3 (tests/test_gpu_dist.py)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_exchange_null_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=240) for _ in range(2)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, msg, calls in got:
        assert "null argument" in msg, (rank, msg)
        # one exchange of a 16-byte header + ceil(5 / 2) = 3 padded 128-byte states
        assert calls == [16 + 3 * 128], (rank, calls)
