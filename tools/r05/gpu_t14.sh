#!/bin/bash
# Round 5, call 14: eight solver blocks per persistent problem, each publishing the pose into its
# XCD's L2 (PICP_PSOLVERS=8) against one leader (-DPICP_PSOLVERS=1, lib/libpicp_amd_ps1.so): the
# whole GPU suite on the candidate, then C2 and C3 interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t14}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
OUT=$OUT/ab TESTS= WLS="c2 c3" LIBS="libpicp_amd_ps1 libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
