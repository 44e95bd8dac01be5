#!/bin/bash
# Round 5, call 3: the issue calibration with occupancy pinned by LDS (exactly W blocks per CU),
# then the C2/C3/C4 A/B of the round-3 library (986d4e6, lib/libpicp_amd_r03.so) against HEAD,
# interleaved, three repetitions on one box.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t3}
mkdir -p $OUT
OUT=$OUT/issue bash tools/r05/gpu_issue.sh || exit 1
OUT=$OUT/ab TESTS= WLS="c2 c3 c4" LIBS="libpicp_amd_r03 libpicp_amd" REPS=3 bash tools/gpu_ab.sh
