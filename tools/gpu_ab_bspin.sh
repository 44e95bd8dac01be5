#!/bin/bash
# C4 A/B of the block kernel partner polls: lib/libpicp_amd_v0.so (s_sleep 1) vs _v1.so (-DPICP_BPOLL_SPIN)
# 4 interleaved reps; every run time-limited, stop at the first failure.
mkdir -p gpurun_out
L=$PWD/02-visualodometry_amd/lib
: > gpurun_out/ab_bspin.log
for rep in 1 2 3 4; do for w in c4; do for v in 0 1; do
PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 200 python bench.py --workload $w --no-cpu --skip-extras --stream-n 0 --steps 100 > gpurun_out/abbspin.log 2>&1 || { echo bench failed; tail gpurun_out/abbspin.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/abbspin.log').read().strip().splitlines()[-1]); print('v$v $w', d['value'], d['roofline']['kernel_us'])" | tee -a gpurun_out/ab_bspin.log
done; done; done
