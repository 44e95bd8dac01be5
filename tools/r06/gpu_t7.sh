#!/bin/bash
# Round 6, call 7: is the multi-chain VO schedule host-bound?  Eight chains enqueue 4 launches per
# segment group and step from one host thread (~40k launches per 8e run).  The same schedules
# captured once into a hipGraph and replayed (PICP_VO_GRAPH=1), chains 2 / 4 / 8, with 16 hardware
# queues; the enqueued form beside them.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t7}
mkdir -p $OUT
: > $OUT/ab.log
for A in "--seg-len 1250 --steps 2 --warmup 1 --samples 1" "--frames 1281"; do for g in 0 1; do for ch in 2 4 8; do
  GPU_MAX_HW_QUEUES=16 PICP_VO_GRAPH=$g PICP_VO_CHAINS=$ch timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench g$g ch$ch failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 $A', 'graph $g chains $ch', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done; done
