#!/bin/bash
# Round 5, call 4: bisect of the C2/C3 drop since round 3: the round-3
# library, HEAD, and HEAD with the dpp() move in round 3's mov_dpp form, with bound_ctrl on, with
# the pose update's contraction left to the compiler, and both; C2 and C3 interleaved, 3 reps.
# Then the C5 shapes' kernel breakdown (tools/r05/gpu_prof_c5.sh).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t4}
mkdir -p $OUT
OUT=$OUT/ab TESTS= WLS="c2 c3" LIBS="libpicp_amd_r03 libpicp_amd libpicp_amd_dppmov libpicp_amd_dppbc libpicp_amd_ctr libpicp_amd_both" REPS=3 bash tools/gpu_ab.sh || exit 1
OUT=$OUT/prof_c5 bash tools/r05/gpu_prof_c5.sh
