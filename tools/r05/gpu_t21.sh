#!/bin/bash
# Round 5, call 21: the round's pose in SGPRs (v_readfirstlane of the LDS copy, PICP_POSE_SGPR)
# against VGPRs (-DPICP_POSE_SGPR=0, lib/libpicp_amd_nosg.so): parity tests on the candidate, then
# C2, C3, C4 and C4 at 128 frames interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t21}
mkdir -p $OUT
OUT=$OUT/ab TESTS="tests/test_gpu_parity.py tests/test_gpu_vo.py" WLS="c2 c3 c4" LIBS="libpicp_amd_nosg libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
OUT=$OUT/ab128 TESTS= WLS="c4" ARGS="--problems 128" LIBS="libpicp_amd_nosg libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
