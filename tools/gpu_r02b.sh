#!/bin/bash
# New GPU tests (comm, residency/fallback, full-size parity, matcher RB=2) then the whole suite,
# then the default bench line (headline + c4/c3/c5 sub-results).
export TMPDIR=/tmp
mkdir -p gpurun_out/r02b
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02b/pytest_new.log 2>&1 || { echo "new tests failed"; tail -40 gpurun_out/r02b/pytest_new.log; exit 1; }
tail -3 gpurun_out/r02b/pytest_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02b/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/r02b/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r02b/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/r02b/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r02b/bench.log; exit 1; }
tail -1 gpurun_out/r02b/bench.log
