#!/bin/bash
# Round 5, call 45: a C5 kernel trace kept whole (run_kernel_trace.csv, gzipped) to locate the step
# chains' gaps (tools/vo_timeline.py reports only their sum).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t45}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/c5_trace -o run --output-format csv -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --skip-extras --samples 1 --detail - > $OUT/c5_trace.log 2>&1 || { echo "trace failed"; tail $OUT/c5_trace.log; exit 1; }
gzip -c $OUT/c5_trace/run_kernel_trace.csv > $OUT/c5_kernel_trace.csv.gz && rm -f $OUT/c5_trace/run_kernel_trace.csv
ls -la $OUT
