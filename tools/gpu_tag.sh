#!/bin/bash
# persistent-mode check: every GPU test, then C2 and C3 benches (no CPU leg)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu --skip-extras --stream-n 0 > gpurun_out/bench_c2_$i.log 2>&1 || { echo bench failed; tail gpurun_out/bench_c2_$i.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/bench_c2_$i.log').read().strip().splitlines()[-1]); print('C2', d['value'], d['roofline']['kernel_us'], d['roofline']['kernel_us_event_pair'])"
done
timeout -k 10 200 python bench.py --workload c3 --no-cpu --skip-extras > gpurun_out/bench_c3.log 2>&1 || { echo bench failed; tail gpurun_out/bench_c3.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/bench_c3.log').read().strip().splitlines()[-1]); print('C3', d['value'], d['roofline']['kernel_us'])"
