#!/bin/bash
# C2 loop: PICP parity tests, persistent phase stamps, C2 bench (no CPU leg)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/pstamps.py > gpurun_out/pstamps.log 2>&1 || { echo pstamps failed; tail gpurun_out/pstamps.log; exit 1; }
cat gpurun_out/pstamps.log
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu --skip-extras --stream-n 0 > gpurun_out/bench_c2_$i.log 2>&1 || { echo bench failed; tail gpurun_out/bench_c2_$i.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/bench_c2_$i.log').read().strip().splitlines()[-1]); print('C2', d['value'], d['roofline']['kernel_us'])"
done
