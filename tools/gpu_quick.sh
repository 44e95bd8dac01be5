#!/bin/bash
# fast loop: gpu tests + C2 sweep + C2 stamps
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/sweep.py --n 100000 --ipb ${C2_IPB:-256,512,1024} > gpurun_out/sweep_c2.log 2>&1 || { echo sweep failed; tail -20 gpurun_out/sweep_c2.log; exit 1; }
cat gpurun_out/sweep_c2.log
PICP_ITEMS_PER_BLOCK=${STAMP_IPB:-512} timeout -k 10 200 python tools/stamps.py --n 100000 > gpurun_out/stamps_c2.log 2>&1 || { echo stamps failed; tail gpurun_out/stamps_c2.log; exit 1; }
cat gpurun_out/stamps_c2.log
