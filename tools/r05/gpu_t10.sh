#!/bin/bash
# Round 5, call 10: the whole GPU suite (long VO tests with the camera-in-world comparison) + smoke.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t10}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -o "step [0-9]*: map.*" $OUT/pytest_gpu.log; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; exit $rc
