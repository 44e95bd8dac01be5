#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/sweep.py --n 100000 --env PICP_MODE --ipb persistent,graph > gpurun_out/sweep_c2.log 2>&1 || { echo sweep failed; tail -20 gpurun_out/sweep_c2.log; exit 1; }
cat gpurun_out/sweep_c2.log
timeout -k 10 120 python tools/pstamps.py > gpurun_out/pstamps.log 2>&1 || { echo pstamps failed; tail gpurun_out/pstamps.log; exit 1; }
cat gpurun_out/pstamps.log
