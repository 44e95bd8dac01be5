#!/bin/bash
# Round 5, call 33: C2's persistent grid with eight solvers: 196 blocks (one item per lane,
# default) against 98 (PICP_PERSIST_BLOCKS=128: two items per lane), 3 interleaved reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t33}
mkdir -p $OUT
: > $OUT/ab.log
for rep in 1 2 3; do for pb in 256 128; do
  PICP_PERSIST_BLOCKS=$pb timeout -k 10 200 python bench.py --workload c2 --no-cpu --skip-extras --steps 20 > $OUT/run.log 2>&1 || { echo "bench $pb failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('c2 blocks_cap=$pb', d['value'], r.get('kernel_us'), d.get('pose_err_vs_gt_se3'))" | tee -a $OUT/ab.log
done; done
