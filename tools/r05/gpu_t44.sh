#!/bin/bash
# Round 5, call 44: the hand-off tests (residency fallback, timed-out waits) with the 300k frame
# whose persistent launch runs the staggered sweep.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t44}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest.log; exit $rc
