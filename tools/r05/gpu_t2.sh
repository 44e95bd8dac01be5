#!/bin/bash
# Round 5, call 2: the issue calibration (per-SIMD spans), the long-segment VO tests, and the C2/C3/C4
# A/B of the round-3 library (986d4e6, lib/libpicp_amd_r03.so) against HEAD, interleaved, one box.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t2}
mkdir -p $OUT
OUT=$OUT/issue bash tools/r05/gpu_issue.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_vo_long.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_long.log 2>&1
rc=$?; echo "pytest long rc=$rc"; grep -E "PASS|FAIL|Error|assert" $OUT/pytest_long.log | head -30; [ $rc -eq 0 ] || exit 1
OUT=$OUT/ab TESTS= WLS="c2 c3 c4" LIBS="libpicp_amd_r03 libpicp_amd" REPS=3 bash tools/gpu_ab.sh
