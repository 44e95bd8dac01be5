#!/bin/bash
# Round-2 closing pass: the whole GPU suite at HEAD, then the concurrency check with the batch's
# residency/fallback counters printed after the batch-beside-VO pairs.  Each step time-limited;
# stop at the first failure.
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python -u tools/concurrency_check.py > $O/concurrency_check.log 2>&1 || { echo "concurrency check failed"; tail -20 $O/concurrency_check.log; exit 1; }
cat $O/concurrency_check.log
