#!/bin/bash
# Round 5, call 48: C2's persistent launch as 256-thread blocks with two items per lane
# (-DPICP_PNARROW=1, lib/libpicp_amd_pn.so: one wave per SIMD instead of two) against 512 x 1:
# parity tests on it, then C2, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t48}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
PICP_LIB=$L/libpicp_amd_pn.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_pn.log 2>&1
rc=$?; echo "pytest pn rc=$rc"; tail -2 $OUT/pytest_pn.log; [ $rc -eq 0 ] || exit 1
OUT=$OUT/ab TESTS= WLS="c2" LIBS="libpicp_amd libpicp_amd_pn" REPS=3 bash tools/gpu_ab.sh || exit 1
