#!/bin/bash
# Round 5, call 53: the whole GPU suite and smoke at HEAD (the fast FP64 triangulation as the default; the staggered solver sweep of
# two or more items per lane).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t53}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; exit $rc
