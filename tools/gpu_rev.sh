#!/bin/bash
# A/B of the alternating sweep direction (Infinity-Cache reuse) at 16M / 8M / 4M, then GPU tests.
set -e
mkdir -p gpurun_out
L=gpurun_out/sweep_rev.log
: > $L
for n in 16000000 12000000 8000000 4000000; do
  timeout -k 10 200 python tools/sweep.py --n $n --env PICP_SWEEP_FORWARD --ipb 1,0 --reps 10 --interleave 3 >> $L 2>&1
done
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
