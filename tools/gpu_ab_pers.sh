#!/bin/bash
# persistent-kernel A/B (lib v0 / v1): parity tests on v1, then C2 and C3 interleaved, 100 solves each
mkdir -p gpurun_out
L=$PWD/02-visualodometry_amd/lib
PICP_LIB=$L/libpicp_amd_v1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_pers.log 2>&1
rc=$?; echo "pytest(v1) rc=$rc"; tail -2 gpurun_out/pt_pers.log; [ $rc -eq 0 ] || exit 1
: > gpurun_out/ab_pers.log
for rep in 1 2 3; do for w in c2 c3; do for v in 0 1; do
PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 200 python bench.py --workload $w --no-cpu --skip-extras --stream-n 0 --steps 100 > gpurun_out/abp.log 2>&1 || { echo bench failed; tail gpurun_out/abp.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/abp.log').read().strip().splitlines()[-1]); print('v$v $w', d['value'], d['roofline']['kernel_us'])" | tee -a gpurun_out/ab_pers.log
done; done; done
