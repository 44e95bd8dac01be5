#!/bin/bash
# PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes) of the C3 persistent kernel and the C4
# block kernel at the bench's default configs, then the C3 bench line (keep_outliers leg)
set -o pipefail
mkdir -p gpurun_out/pmc_c3c4
WL=c3 KERNEL=picp_persistent_kernel bash tools/gpu_pmc.sh > gpurun_out/pmc_c3.log 2>&1 || { echo pmc c3 failed; tail -20 gpurun_out/pmc_c3.log; exit 1; }
cp gpurun_out/pmc/c3_FETCH_SIZE.json gpurun_out/pmc_c3c4/c3_persistent_pmc_FETCH_SIZE.json
cp gpurun_out/pmc/c3_WRITE_SIZE.json gpurun_out/pmc_c3c4/c3_persistent_pmc_WRITE_SIZE.json
cp gpurun_out/pmc/c3_trace/run_kernel_stats.csv gpurun_out/pmc_c3c4/c3_pmc_trace_kernel_stats.csv
WL=c4 KERNEL=picp_block_kernel bash tools/gpu_pmc.sh > gpurun_out/pmc_c4.log 2>&1 || { echo pmc c4 failed; tail -20 gpurun_out/pmc_c4.log; exit 1; }
cp gpurun_out/pmc/c4_FETCH_SIZE.json gpurun_out/pmc_c3c4/c4_block_pmc_FETCH_SIZE.json
cp gpurun_out/pmc/c4_WRITE_SIZE.json gpurun_out/pmc_c3c4/c4_block_pmc_WRITE_SIZE.json
cp gpurun_out/pmc/c4_trace/run_kernel_stats.csv gpurun_out/pmc_c3c4/c4_pmc_trace_kernel_stats.csv
grep -h '"mean"' gpurun_out/pmc_c3c4/*.json
timeout -k 10 300 python bench.py --workload c3 --no-cpu > gpurun_out/bench_c3k.log 2>&1 || { echo bench failed; tail gpurun_out/bench_c3k.log; exit 1; }
tail -1 gpurun_out/bench_c3k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['keep_outliers_true'], d['with_convergence'])"
