#!/bin/bash
# C2 and C3 A/B of lib/libpicp_amd_v0.so (s_sleep 1 between hand-off polls) vs _v1.so
# (-DPICP_POLL_SPIN): 4 interleaved reps each; every run time-limited, stop at the first failure.
mkdir -p gpurun_out
L=$PWD/02-visualodometry_amd/lib
: > gpurun_out/ab_spin.log
for rep in 1 2 3 4; do for w in c2 c3; do for v in 0 1; do
PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 200 python bench.py --workload $w --no-cpu --skip-extras --stream-n 0 --steps 100 > gpurun_out/abspin.log 2>&1 || { echo bench failed; tail gpurun_out/abspin.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/abspin.log').read().strip().splitlines()[-1]); print('v$v $w', d['value'], d['roofline']['kernel_us'])" | tee -a gpurun_out/ab_spin.log
done; done; done
