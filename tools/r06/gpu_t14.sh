#!/bin/bash
# Round 6, call 14: is the split world match slow because its early streams share hardware queues
# with the step chains?  Split off / on with 4 (default) and 8 hardware queues at the 8e and N = 8
# per-rank shapes.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t14}
mkdir -p $OUT
: > $OUT/ab.log
for A in "--seg-len 1250 --steps 2 --warmup 1 --samples 3" "--frames 1281"; do for q in 4 8; do for v in 0 1; do
  GPU_MAX_HW_QUEUES=$q PICP_VO_SPLIT=$v timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 [$A]', 'queues $q split $v', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done; done
