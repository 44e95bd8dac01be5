#!/bin/bash
# Kernel trace of C5 (one warmup run + one timed run) and the per-stream timeline of the last run
# (tools/vo_timeline.py): which kernels each VO chain waits on and how long its gaps are.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/vtl}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --workload c5 --no-cpu --skip-extras --steps 1 --warmup 1 --samples 1 > $OUT/tr.log 2>&1 || { echo "trace failed"; tail $OUT/tr.log; exit 1; }
python3 tools/vo_timeline.py $OUT/tr/run_kernel_trace.csv ${LAST_MS:-15.5} | tee $OUT/timeline.log
