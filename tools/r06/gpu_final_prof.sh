#!/bin/bash
# Round 6 end pass, part 2: the kernel traces of every workload with the FETCH/WRITE/SQ PMC passes
# the bench line reads (tools/r04/gpu_prof_r04.sh: C2, C3, C4, C4 at 128 frames, the 16M frame)
# and the C5 shapes by kernel and stream (tools/r05/gpu_prof_c5.sh: 250 segments, 8e, N = 8 share).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/final}
mkdir -p $OUT
WLS="c2 c3 c4 c4x128 c2n16m" OUT=$OUT bash tools/r04/gpu_prof_r04.sh || exit 1
OUT=$OUT bash tools/r05/gpu_prof_c5.sh
