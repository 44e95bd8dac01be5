#!/bin/bash
# C5 (device-resident VO sequence): segment-length sweep + rocprof kernel stats of the default
mkdir -p gpurun_out
for L in ${C5_SEGS:-10 20 40 80}; do
  timeout -k 10 300 python bench.py --workload c5 --seg-len $L --steps ${C5_STEPS:-5} --warmup 1 --no-cpu >> gpurun_out/c5_sweep.log 2>&1 || { echo "c5 L=$L failed"; tail -20 gpurun_out/c5_sweep.log; exit 1; }
  tail -1 gpurun_out/c5_sweep.log
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_c5.log 2>&1 || { echo "rocprof c5 failed"; tail -20 gpurun_out/prof_c5.log; exit 1; }
cat gpurun_out/prof_c5/run_kernel_stats.csv
