#!/bin/bash
# probe-first partial sweep (persistent kernel): parity, A/B vs the previous build, phase stamps
export TMPDIR=/tmp
O=gpurun_out/r02g
mkdir -p $O
OUT=$O/ab WLS="c2 c3" LIBS="libpicp_amd_f libpicp_amd" REPS=4 TESTS="tests/test_gpu_parity.py tests/test_gpu_dist.py" bash tools/gpu_ab.sh || exit 1
OUT=$O/pst PICP_STAMPS_LIB=$PWD/02-visualodometry_amd/lib/libpicp_amd_stamps_new.so bash tools/gpu_pstamps.sh > /dev/null 2>&1 || { echo "pstamps failed"; exit 1; }
tail -6 $O/pst/pstamps_c2.log; tail -6 $O/pst/pstamps_c3.log
