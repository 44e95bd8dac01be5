#!/bin/bash
# Round 5, call 58: the triangulation and VO tests (the long segment included) once more on the
# library built from the round's final HEAD.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t58}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vo.py tests/test_gpu_scale.py tests/test_gpu_vo_long.py -x -q -k "triangulation or vo or scale or long" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; exit $rc
