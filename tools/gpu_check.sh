#!/bin/bash
# full GPU test suite, block-kernel stamps, C4 and C5 benches (no CPU leg)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_bstamps.sh || exit 1
for w in c4 c5 c4 c5; do
timeout -k 10 200 python bench.py --workload $w --no-cpu --skip-extras --stream-n 0 > gpurun_out/bench_$w.log 2>&1 || { echo bench failed; tail gpurun_out/bench_$w.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$w.log').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'])"
done
