#!/bin/bash
# A/B of two library builds (lib/libpicp_amd_v0.so, _v1.so) on C2/C3/C4/C5, interleaved; the GPU
# suite on the shipped build first
mkdir -p gpurun_out
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
: > gpurun_out/ab2.log
for rep in 1 2; do for w in ${WLS:-c2 c3 c4 c5}; do for v in 0 1; do
PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 200 python bench.py --workload $w --no-cpu --skip-extras --stream-n 0 > gpurun_out/ab2_$w.log 2>&1 || { echo bench failed; tail gpurun_out/ab2_$w.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/ab2_$w.log').read().strip().splitlines()[-1]); print('v$v $w', d['value'], d['ms_per_step'])" | tee -a gpurun_out/ab2.log
done; done; done
