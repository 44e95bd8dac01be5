#!/bin/bash
# Round 6: tools/r06/gpu_verify.sh (suite, smoke, one line at the final HEAD), then
# tools/r06/gpu_pmc_c2.sh (C2's FETCH_SIZE reproducibility).
export TMPDIR=/tmp
OUT=gpurun_out/r06/verify bash tools/r06/gpu_verify.sh || exit 1
OUT=gpurun_out/r06/pmc_c2 bash tools/r06/gpu_pmc_c2.sh
