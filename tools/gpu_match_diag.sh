#!/bin/bash
# Where the matcher's time goes: kernel traces of the accept-only 1024 x 2000 x 2000 batch (and
# MATCH_DUP=0.5, C5-like candidate density) for lib/libpicp_amd_v{VARIANTS}.so -- the shipped
# build and diagnostic builds that drop one piece each (MM_DIAG_*: wrong results, timing only).
export TMPDIR=/tmp
mkdir -p gpurun_out/md
L=$PWD/02-visualodometry_amd/lib
for dup in 0 0.5; do
  for v in ${VARIANTS:-v2 nocand novote norescan}; do
    PICP_LIB=$L/libpicp_amd_$v.so MATCH_DUP=$dup timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/md/t_${v}_$dup -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > gpurun_out/md/t_${v}_$dup.log 2>&1 || { echo "trace $v failed"; tail -5 gpurun_out/md/t_${v}_$dup.log; exit 1; }
    python3 -c "
import csv
t=[int(x['End_Timestamp'])-int(x['Start_Timestamp']) for x in csv.DictReader(open('gpurun_out/md/t_${v}_$dup/run_kernel_trace.csv')) if 'mfma' in x['Kernel_Name']]
print('$v dup=$dup', t)" | tee -a gpurun_out/md/summary.log
  done
done
