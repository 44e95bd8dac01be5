#!/bin/bash
# Round 5, call 42: the split exchange's polling wave at issue priority 0 (lib/libpicp_amd_pp0.so,
# -DPICP_XG_POLL_PRIO0; the tail's priority 3 restored after the wait) against polling at 3:
# split parity tests, then C4 at 128 frames, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t42}
mkdir -p $OUT
PICP_LIB=$PWD/02-visualodometry_amd/lib/libpicp_amd_pp0.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "split or tag_bases" --timeout 120 --timeout-method thread > $OUT/pytest_pp0.log 2>&1
rc=$?; echo "pytest pp0 rc=$rc"; tail -2 $OUT/pytest_pp0.log; [ $rc -eq 0 ] || exit 1
OUT=$OUT/ab128 TESTS= WLS="c4" ARGS="--problems 128" LIBS="libpicp_amd libpicp_amd_pp0" REPS=3 bash tools/gpu_ab.sh || exit 1
