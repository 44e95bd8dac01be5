#!/bin/bash
# Round-2 health check on the GPU: the gpu test suite, one default bench line, a kernel-stats profile.
export TMPDIR=/tmp
mkdir -p gpurun_out/r02s5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02s5/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r02s5/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r02s5/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/r02s5/bench_c2.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r02s5/bench_c2.log; exit 1; }
tail -1 gpurun_out/r02s5/bench_c2.log
