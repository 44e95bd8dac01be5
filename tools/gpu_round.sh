#!/bin/bash
# Round-end measurement pass: tests + smoke + default bench + C2 kernel trace (gpu_full.sh),
# streaming lines (gpu_stream.sh), 16M PMC (gpu_pmc_stream.sh), then C4 and C5 bench lines.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_full.sh || exit 1
bash tools/gpu_stream.sh || exit 1
bash tools/gpu_pmc_stream.sh || exit 1
timeout -k 10 300 python bench.py --workload c4 --no-cpu > gpurun_out/bench_c4.log 2>&1 || { echo c4 failed; tail gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log | cut -c1-300
timeout -k 10 300 python bench.py --workload c5 --no-cpu > gpurun_out/bench_c5.log 2>&1 || { echo c5 failed; tail gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log | cut -c1-300
timeout -k 10 300 python bench.py --workload c5 --seg-len 10 --no-cpu > gpurun_out/bench_c5_l10.log 2>&1 || { echo c5 l10 failed; exit 1; }
tail -1 gpurun_out/bench_c5_l10.log | cut -c1-300
