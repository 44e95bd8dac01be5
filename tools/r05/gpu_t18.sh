#!/bin/bash
# Round 5, call 18: C4 at 128 frames, the exchange granules at sync + 16 B (lib/libpicp_amd_head.so,
# the committed layout) against sync + 128 B (lib/libpicp_amd_xg0.so: 128-B aligned sets, the
# agent-scope exchange) and the L2 exchange (lib/libpicp_amd.so); interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t18}
mkdir -p $OUT
OUT=$OUT/ab TESTS= WLS="c4" ARGS="--problems 128" LIBS="libpicp_amd_head libpicp_amd_xg0 libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
