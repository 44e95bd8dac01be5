#!/bin/bash
# Round-2 session d: register-carried finish (lower-triangle LDL^T, merged sincos branch):
# microbenchmark, GPU parity suites, A/B vs base, phase stamps.
export TMPDIR=/tmp
O=gpurun_out/r02d
mkdir -p $O
timeout -k 5 60 tools/ubench/parts_ubench > $O/ubench.log 2>&1 || { echo "ubench failed"; cat $O/ubench.log; exit 1; }
cat $O/ubench.log
OUT=$O/ab TESTS="tests/test_gpu_parity.py tests/test_gpu_vo.py tests/test_gpu_scale.py tests/test_gpu_dist.py tests/test_driver.py tests/test_dropin.py" REPS=3 bash tools/gpu_ab.sh || exit 1
OUT=$O/pst PICP_STAMPS_LIB=$PWD/02-visualodometry_amd/lib/libpicp_amd_stamps_new.so bash tools/gpu_pstamps.sh > /dev/null 2>&1 || { echo "pstamps failed"; exit 1; }
tail -6 $O/pst/pstamps_c2.log; tail -6 $O/pst/pstamps_c3.log
OUT=$O/bst VARS="new" bash tools/gpu_bstamps_ab.sh
