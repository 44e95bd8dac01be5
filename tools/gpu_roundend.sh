#!/bin/bash
# Round-end measurement pass: every BASELINE config's bench line plus a rocprofv3 kernel-stats
# profile of the same command (each step time-limited; stop at the first failure).
export TMPDIR=/tmp
mkdir -p gpurun_out/re
for w in c2 c3 c4 c5; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/re/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -5 gpurun_out/re/bench_$w.log; exit 1; }
  tail -1 gpurun_out/re/bench_$w.log > gpurun_out/re/bench_$w.json
  python -c "import json; d=json.load(open('gpurun_out/re/bench_$w.json')); print('$w', d['value'], d['unit'], d['ms_per_step'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/re/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --no-cpu --skip-extras --steps 10 --warmup 2 > gpurun_out/re/prof_$w.log 2>&1 || { echo "rocprof $w failed"; tail -5 gpurun_out/re/prof_$w.log; exit 1; }
  cp gpurun_out/re/prof_$w/run_kernel_stats.csv gpurun_out/re/kernel_stats_$w.csv
done
