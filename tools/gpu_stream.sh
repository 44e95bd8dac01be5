#!/bin/bash
# streaming configurations: C3 (1M, 30% outliers) and single frames past the MALL
mkdir -p gpurun_out
for args in "--workload c3" "--workload c2 --n 4000000" "--workload c2 --n 16000000"; do
  timeout -k 10 300 python bench.py $args --steps 10 --warmup 3 --no-cpu >> gpurun_out/stream.log 2>&1 || { echo "bench $args failed"; tail -20 gpurun_out/stream.log; exit 1; }
  tail -1 gpurun_out/stream.log | cut -c1-200
done
for m in graph persistent; do
  PICP_MODE=$m timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu >> gpurun_out/stream.log 2>&1 || { echo "c3 $m failed"; exit 1; }
done
python - <<'PY'
import json
for l in open('gpurun_out/stream.log'):
    if l.startswith('{'):
        d = json.loads(l); r = d['roofline']
        print(d['config']['n_corr'], r['mode'], d['value'], r['achieved'], r['frac'], r['kernel_us'], r['blocks_per_launch'])
PY
