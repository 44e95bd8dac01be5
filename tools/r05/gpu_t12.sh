#!/bin/bash
# Round 5, call 12: C5 A/B of HEAD (lib/libpicp_amd_head.so), the matcher's block-mask entries alone
# (libpicp_amd_m.so) and with the append's round trips cut (libpicp_amd.so), interleaved, 3 reps;
# the 8e partition HEAD vs candidate; the VO and block-split tests on the candidate first.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t12}
mkdir -p $OUT
OUT=$OUT/ab TESTS="tests/test_gpu_vo.py tests/test_gpu_match.py tests/test_gpu_parity.py" WLS="c5" LIBS="libpicp_amd_head libpicp_amd_m libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
OUT=$OUT/ab8e TESTS= WLS="c5" ARGS="--seg-len 1250 --steps 2 --warmup 1 --samples 1" LIBS="libpicp_amd_head libpicp_amd" REPS=2 bash tools/gpu_ab.sh || exit 1
