#!/bin/bash
# C4 (split block) A/B of lib v0 / v1: parity tests on v1, then 3 interleaved reps of C4 + C5
mkdir -p gpurun_out
L=$PWD/02-visualodometry_amd/lib
PICP_LIB=$L/libpicp_amd_v1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_c4.log 2>&1
rc=$?; echo "pytest(v1) rc=$rc"; tail -2 gpurun_out/pt_c4.log; [ $rc -eq 0 ] || exit 1
: > gpurun_out/ab_c4.log
for rep in 1 2 3; do for v in 0 1; do
PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 200 python bench.py --workload c4 --no-cpu --skip-extras --steps 50 > gpurun_out/abc4.log 2>&1 || { echo bench failed; tail gpurun_out/abc4.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/abc4.log').read().strip().splitlines()[-1]); print('v$v c4', d['value'], d['roofline']['kernel_us'])" | tee -a gpurun_out/ab_c4.log
done; done
