#!/bin/bash
# Round 5, call 36: the solvers' sweep with two passes in flight (-DPICP_SWEEP_STAGGER=4 / 8:
# lib/libpicp_amd_sw4.so, _sw8.so) against one (lib/libpicp_amd.so): parity tests on sw4, then
# C2 and C3 interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t36}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
PICP_LIB=$L/libpicp_amd_sw4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_sw4.log 2>&1
rc=$?; echo "pytest sw4 rc=$rc"; tail -2 $OUT/pytest_sw4.log; [ $rc -eq 0 ] || exit 1
OUT=$OUT/ab TESTS= WLS="c2 c3" LIBS="libpicp_amd libpicp_amd_sw4 libpicp_amd_sw8" REPS=3 bash tools/gpu_ab.sh || exit 1
