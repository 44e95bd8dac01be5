#!/bin/bash
# Round 5, call 29: spin-wait bounds read lazily (PollBound: the clock on every 16th check, no
# round-start read) against HEAD (lib/libpicp_amd_head.so): parity + VO tests on the candidate,
# then C2 / C3 / C4 and C4 at 128 frames interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t29}
mkdir -p $OUT
OUT=$OUT/ab TESTS="tests/test_gpu_parity.py tests/test_gpu_vo.py tests/test_gpu_scale.py" WLS="c2 c3 c4" LIBS="libpicp_amd_head libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
OUT=$OUT/ab128 TESTS= WLS="c4" ARGS="--problems 128" LIBS="libpicp_amd_head libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
