#!/bin/bash
# Round 5, call 15: the followers' pose-poll stagger now that they poll an L2 line: two polls in
# flight PICP_POSE_STAGGER x 64 clocks apart (default 8) against 0 (one poll), 2 and 4; C2 and C3
# interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t15}
mkdir -p $OUT
OUT=$OUT/ab TESTS= WLS="c2 c3" LIBS="libpicp_amd libpicp_amd_st0 libpicp_amd_st2 libpicp_amd_st4" REPS=3 bash tools/gpu_ab.sh || exit 1
