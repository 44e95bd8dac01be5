#!/bin/bash
# Round 6, call 28: the N = 8 per-rank shape's world match (16 problems, default 4 ranges at RB = 1)
# with 6 / 7 ranges at RB = 2 (864 / 1,008 blocks: one generation) and 5 at RB = 1, interleaved.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t28}
mkdir -p $OUT
: > $OUT/ab.log
for rep in 1 2; do for v in "PICP_MATCH_KSPLIT=0" "PICP_MATCH_KSPLIT=7 PICP_MATCH_RB=2" "PICP_MATCH_KSPLIT=6 PICP_MATCH_RB=2" "PICP_MATCH_KSPLIT=5 PICP_MATCH_RB=1"; do
  env $v timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - --frames 1281 > $OUT/run.log 2>&1 || { echo "bench failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 n8 [$v]', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done
