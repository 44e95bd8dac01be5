#!/bin/bash
# Split block mode (C4: two blocks per frame): parity tests, then C4 with and without the split.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
: > gpurun_out/c4_split.log
for s in 1 2 1 2; do
  PICP_BLOCK_SPLIT=$s timeout -k 10 200 python bench.py --workload c4 --no-cpu >> gpurun_out/c4_split.log 2>&1 || { echo c4 split=$s failed; tail gpurun_out/c4_split.log; exit 1; }
  echo "split=$s $(tail -1 gpurun_out/c4_split.log | cut -c1-160)"
done
