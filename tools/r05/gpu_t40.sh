#!/bin/bash
# Round 5, call 40: the staggered sweep for one item per lane (C2) after an initial delay of the
# solvers' first pass (lib/libpicp_amd_d8 / d16 / d32.so: 8, 16, 32 x 64 clocks), against C2's
# unstaggered sweep (lib/libpicp_amd.so); C2, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t40}
mkdir -p $OUT
OUT=$OUT/ab TESTS= WLS="c2" LIBS="libpicp_amd libpicp_amd_d8 libpicp_amd_d16 libpicp_amd_d32" REPS=3 bash tools/gpu_ab.sh || exit 1
