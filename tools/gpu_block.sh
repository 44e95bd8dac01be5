#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/sweep.py --n 10000 --problems 256 --env PICP_BLOCK_NPT --ipb 1,2,4,8 --reps 5 > gpurun_out/sweep_c4b.log 2>&1 || { echo sweep failed; tail -20 gpurun_out/sweep_c4b.log; exit 1; }
cat gpurun_out/sweep_c4b.log
timeout -k 10 300 python tools/sweep.py --n 10000 --problems 128 --env PICP_MODE --ipb block,graph --reps 5 > gpurun_out/sweep_c4m.log 2>&1 || { echo sweep failed; tail -20 gpurun_out/sweep_c4m.log; exit 1; }
cat gpurun_out/sweep_c4m.log
timeout -k 10 400 python tools/sweep.py --n 10000 --problems 2048 --env PICP_MODE --ipb block,graph --reps 2 --interleave 2 > gpurun_out/sweep_c4big.log 2>&1 || { echo sweep failed; tail -20 gpurun_out/sweep_c4big.log; exit 1; }
cat gpurun_out/sweep_c4big.log
