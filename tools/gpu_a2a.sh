#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
PICP_PERSIST_A2A=1 timeout -k 10 400 python -m pytest tests -m gpu -q -x -k "persistent or solve or smoke or kat" > gpurun_out/pytest_gpu_a2a.log 2>&1
rc=$?; echo "pytest a2a rc=$rc"; tail -3 gpurun_out/pytest_gpu_a2a.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/sweep.py --n 100000 --env PICP_PERSIST_A2A --ipb 0,1 > gpurun_out/sweep_a2a.log 2>&1 || { echo sweep failed; tail -20 gpurun_out/sweep_a2a.log; exit 1; }
cat gpurun_out/sweep_a2a.log
PICP_PERSIST_A2A=1 timeout -k 10 120 python tools/pstamps.py > gpurun_out/pstamps_a2a.log 2>&1; cat gpurun_out/pstamps_a2a.log
