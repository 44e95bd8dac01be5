#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/sweep.py --n 10000 --problems 256 --ipb 1024,2048,4096,8192 --reps 5 > gpurun_out/sweep_c4.log 2>&1 || { echo sweep4 failed; tail -20 gpurun_out/sweep_c4.log; exit 1; }
cat gpurun_out/sweep_c4.log
timeout -k 10 300 python tools/sweep.py --n 1000000 --outlier 0.3 --env PICP_MODE --ipb graph --reps 5 > gpurun_out/sweep_c3.log 2>&1; cat gpurun_out/sweep_c3.log
timeout -k 10 400 python tools/sweep.py --n 10000 --problems 2048 --ipb 2048,4096,8192 --reps 3 --interleave 2 > gpurun_out/sweep_c4big.log 2>&1 || { echo sweep4big failed; tail -20 gpurun_out/sweep_c4big.log; exit 1; }
cat gpurun_out/sweep_c4big.log
