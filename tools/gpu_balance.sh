#!/bin/bash
# Block-count balance sweep of the streaming round kernel (16M, 4M, 2M): old ipb vs CU-multiple.
set -e
mkdir -p gpurun_out
L=gpurun_out/sweep_balance.log
: > $L
timeout -k 10 200 python tools/sweep.py --n 16000000 --ipb 32768,31252,15628 --reps 10 --interleave 2 >> $L 2>&1
timeout -k 10 200 python tools/sweep.py --n 4000000 --ipb 8192,7816,3908 --reps 20 --interleave 2 >> $L 2>&1
timeout -k 10 200 python tools/sweep.py --n 2000000 --ipb 8192,7816,3908 --reps 20 --interleave 2 >> $L 2>&1
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
