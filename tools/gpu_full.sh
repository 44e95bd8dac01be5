#!/bin/bash
# full GPU pass: tests, smoke, bench, rocprof kernel stats (each step time-limited; stop on failure)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --no-cpu --skip-extras --steps 20 > gpurun_out/prof_c2.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_c2.log; exit 1; }
cat gpurun_out/prof_c2/run_kernel_stats.csv
tail -1 gpurun_out/prof_c2.log
