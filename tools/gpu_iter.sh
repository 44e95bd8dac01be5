#!/bin/bash
# quick GPU iteration: gpu tests + sweeps + stamps (each step time-limited, stop on failure)
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/sweep.py --n 100000 --ipb ${C2_IPB:-256,512,1024} > gpurun_out/sweep_c2.log 2>&1 || { echo sweep failed; tail -20 gpurun_out/sweep_c2.log; exit 1; }
cat gpurun_out/sweep_c2.log
timeout -k 10 300 python tools/sweep.py --n 1000000 --outlier 0.3 --ipb ${C3_IPB:-2048,4096,8192} --reps 5 > gpurun_out/sweep_c3.log 2>&1 || { echo sweep3 failed; tail -20 gpurun_out/sweep_c3.log; exit 1; }
cat gpurun_out/sweep_c3.log
timeout -k 10 300 python tools/sweep.py --n 10000 --problems 256 --ipb ${C4_IPB:-2048,4096,10240} --reps 5 > gpurun_out/sweep_c4.log 2>&1 || { echo sweep4 failed; tail -20 gpurun_out/sweep_c4.log; exit 1; }
cat gpurun_out/sweep_c4.log
timeout -k 10 200 python tools/stamps.py --n 100000 > gpurun_out/stamps_c2.log 2>&1 || { echo stamps failed; tail gpurun_out/stamps_c2.log; exit 1; }
cat gpurun_out/stamps_c2.log
