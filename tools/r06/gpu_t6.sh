#!/bin/bash
# Round 6, call 6: more VO step chains with more hardware queues.  Round 6's t2 found 4 and 8 chains
# far slower with HIP's default 4 hardware queues per process (two chains on one queue serialise);
# GPU_MAX_HW_QUEUES=16 gives each chain stream its own queue.  8e partition and the N = 8 per-rank
# shape, chains 2 / 4 / 8, queues 4 / 16.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t6}
mkdir -p $OUT
: > $OUT/ab.log
for A in "--seg-len 1250 --steps 2 --warmup 1 --samples 1" "--frames 1281"; do for q in 4 16; do for ch in 2 4 8; do
  GPU_MAX_HW_QUEUES=$q PICP_VO_CHAINS=$ch timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench q$q ch$ch failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 $A', 'queues $q chains $ch', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done; done
