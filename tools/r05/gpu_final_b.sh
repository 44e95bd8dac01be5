#!/bin/bash
# Round 5 end, part B: the HBM traffic counters (FETCH_SIZE, WRITE_SIZE) and the SQ pass, each in its
# own --pmc run (MI355X_MICROARCH.md), for the kernels bench.py prices (tools/r04/gpu_prof_r04.sh's
# PMC loop).  OUT=${OUT:-gpurun_out/r05/pmc}
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/pmc}
mkdir -p $OUT
WLS=" " OUT=$OUT bash tools/r04/gpu_prof_r04.sh
