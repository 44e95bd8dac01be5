#!/bin/bash
# Round 5, call 39: persistent-kernel poll settings around the new default: the solvers' second
# sweep pass 16 x 64 clocks behind the first (lib/libpicp_amd_sw16.so) instead of 8, and three
# staggered pose polls per follower (lib/libpicp_amd_np3.so) instead of two; C2 and C3, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t39}
mkdir -p $OUT
PICP_LIB=$PWD/02-visualodometry_amd/lib/libpicp_amd_np3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "persistent or c3 or c2" --timeout 120 --timeout-method thread > $OUT/pytest_np3.log 2>&1
rc=$?; echo "pytest np3 rc=$rc"; tail -2 $OUT/pytest_np3.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit 1
OUT=$OUT/ab TESTS= WLS="c2 c3" LIBS="libpicp_amd libpicp_amd_sw16 libpicp_amd_np3" REPS=3 bash tools/gpu_ab.sh || exit 1
