#!/bin/bash
# GPU session script: tests, bench, rocprof kernel stats (each step time-limited)
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"
tail -15 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench.log; exit 1; }
tail -3 gpurun_out/bench.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --no-cpu --steps 20 > gpurun_out/prof_c2.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_c2.log; exit 1; }
find gpurun_out/prof_c2 -name "*kernel_stats.csv" -exec cat {} \;
