#!/bin/bash
# Round 5, call 17: the split exchange through the XCD's L2 with round-1 placement detection (one
# set polled per partner) against the agent-scope exchange (-DPICP_XG_L2=0, lib/libpicp_amd_xg0.so):
# the block-split parity tests on the candidate, then C4 at 128 frames interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t17}
mkdir -p $OUT
OUT=$OUT/ab TESTS="tests/test_gpu_parity.py" WLS="c4" ARGS="--problems 128" LIBS="libpicp_amd_xg0 libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
