#!/bin/bash
# Round 6, calls 3+4 in one (the pool had no box for them separately): tools/r06/gpu_t4.sh (the
# merge kernel's batched loads, the matcher and long-VO tests; the persistent kernel's error-word
# check on C2/C3), then tools/r06/gpu_t3.sh (the CU-masked side stream and the world match's
# knobs at the C5 shapes).
export TMPDIR=/tmp
OUT=gpurun_out/r06/t4 bash tools/r06/gpu_t4.sh || exit 1
OUT=gpurun_out/r06/t3 bash tools/r06/gpu_t3.sh
