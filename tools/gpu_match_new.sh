#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/match_stats.py --frames 2000 > gpurun_out/match_stats.log 2>&1 && cat gpurun_out/match_stats.log
FRAMES=10000 VARIANTS="0 1" bash tools/gpu_match_ab.sh
