#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --cpu-seconds 10 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
WL=c2 bash tools/gpu_pmc.sh || exit 1
WL=c4 bash tools/gpu_pmc.sh || exit 1
