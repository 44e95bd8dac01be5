#!/bin/bash
# C4 block-mode split A/B: parity tests for the block paths, then the C4 bench at split 2 and 4
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "block or batch or uniform" --timeout 300 --timeout-method thread > gpurun_out/pt_block.log 2>&1
rc=$?; tail -3 gpurun_out/pt_block.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
for sp in 2 4; do
  PICP_BLOCK_SPLIT=$sp timeout -k 10 300 python bench.py --workload c4 --no-cpu --steps 10 --warmup 3 > gpurun_out/c4_s$sp.log 2>&1 || { tail gpurun_out/c4_s$sp.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/c4_s$sp.log').read().strip().splitlines()[-1]); print('split=$sp', d['value'], d['ms_per_step'], d['roofline'].get('kernel_us'))"
done
done
