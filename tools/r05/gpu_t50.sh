#!/bin/bash
# Round 5, call 50: the followers' pose-poll stagger with the staggered sweep in place: 4 and 16 x
# 64 clocks (lib/libpicp_amd_ps4 / _ps16.so) against 8; C3 and C2, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t50}
mkdir -p $OUT
OUT=$OUT/ab TESTS= WLS="c3 c2" LIBS="libpicp_amd libpicp_amd_ps4 libpicp_amd_ps16" REPS=3 bash tools/gpu_ab.sh || exit 1
