#!/bin/bash
# Round 6, call 26: the 8e world match's range split at one generation of four blocks per CU
# (PICP_MATCH_KSPLIT=28: 4 x 9 x 28 = 1,008 blocks at RB = 2; isolated -17 %, profiles/r06/t12) in
# the VO, against the default rule (16), interleaved, 3 samples each; 24 and 32 beside them.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t26}
mkdir -p $OUT
: > $OUT/ab.log
for rep in 1 2; do for k in 0 28 24 32; do
  PICP_MATCH_KSPLIT=$k timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - --seg-len 1250 --steps 2 --warmup 1 --samples 3 > $OUT/run.log 2>&1 || { echo "bench failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 8e ksplit $k', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done
