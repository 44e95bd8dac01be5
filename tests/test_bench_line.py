"""The bench line's shape (CPU, no device): the driver keeps only the tail of stdout (about 2,000
characters), so the one JSON line must carry every sub-result's numbers in well under that, with
the contract's keys first; and the C5 rounds-sync figure's arithmetic."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, ROOT)
    import bench as B
    return B


def test_compact_line_fits_the_driver_tail(bench):
    detail = os.path.join(ROOT, "profiles", "r06", "final", "bench_detail_a.json")
    out = json.load(open(detail))
    line = json.dumps(bench.compact_line(out, "gpurun_out/bench_detail_c2_n1.json"), separators=(",", ":"))
    assert len(line) < 1950, len(line)
    d = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert list(d)[:2] == ["metric", "value"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in d["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in d["cpu_baseline"], k
    # every config's numbers: C3, C4 with its projections, C5 led by the 8e partition with its side figures
    assert {"c3", "c4", "c5", "stream16m"} <= set(d)
    assert {"n2", "n4", "n8"} <= set(d["c4"]["proj_eff"])
    assert {"essential_boot", "gt_anchored_250", "rounds_sync", "per_rank_n8", "proj_eff_n8"} <= set(d["c5"])


def test_rounds_sync(bench):
    # two chains of two segments; chain 0's per-step maxima: 5 + 9 = 14, chain 1's: 7 + 3 = 10; the
    # slowest segment alone: 2 + 9 = 11 (segment 1) -> ratio 14 / 11
    r = bench._rounds_sync([[5, 1], [2, 9], [7, 2], [3, 3]])
    assert r["sum_t_max_s"] == 14 and r["max_s_sum_t"] == 11 and r["chains"] == 2
    assert abs(r["ratio"] - round(14 / 11, 4)) < 1e-12
    r1 = bench._rounds_sync([[50, 50, 10]])  # one segment: no synchronisation cost
    assert r1["ratio"] == 1.0 and r1["steps_at_50_any"] == 2
