#!/bin/bash
# Round 5, call 38: the split block kernel's partner exchange with two polls in flight
# (PICP_XG_STAGGER 8, lib/libpicp_amd.so) against one (lib/libpicp_amd_xg0.so): parity tests,
# then C4 at 128 frames (split 4: the exchange every round), C4 and C5 (no exchange), 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t38}
mkdir -p $OUT
OUT=$OUT/ab128 TESTS="tests/test_gpu_parity.py" WLS="c4" ARGS="--problems 128" LIBS="libpicp_amd_xg0 libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
OUT=$OUT/ab TESTS= WLS="c4 c5" LIBS="libpicp_amd_xg0 libpicp_amd" REPS=2 bash tools/gpu_ab.sh || exit 1
