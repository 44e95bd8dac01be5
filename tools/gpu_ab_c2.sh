#!/bin/bash
# C2 A/B of lib/libpicp_amd_v0.so vs _v1.so: 4 interleaved reps of 100 timed solves each
mkdir -p gpurun_out
L=$PWD/02-visualodometry_amd/lib
: > gpurun_out/ab_c2.log
for rep in 1 2 3 4; do for v in 0 1; do
PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 200 python bench.py --workload c2 --no-cpu --skip-extras --stream-n 0 --steps 100 > gpurun_out/abc2.log 2>&1 || { echo bench failed; tail gpurun_out/abc2.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/abc2.log').read().strip().splitlines()[-1]); print('v$v c2', d['value'], d['roofline']['kernel_us'])" | tee -a gpurun_out/ab_c2.log
done; done
