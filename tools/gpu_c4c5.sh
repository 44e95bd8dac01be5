#!/bin/bash
# GPU tests, then C4 (split block mode) and C5 (VO) bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python bench.py --workload c4 --no-cpu > gpurun_out/bench_c4.log 2>&1 || { echo c4 failed; tail gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log | cut -c1-200
timeout -k 10 300 python bench.py --workload c5 --no-cpu > gpurun_out/bench_c5.log 2>&1 || { echo c5 failed; tail gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log | cut -c1-200
