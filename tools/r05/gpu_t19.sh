#!/bin/bash
# Round 5, call 19: C2's block count with the eight-solver kernel -- 196 blocks of one item per lane
# (default) against 98 blocks of two (PICP_PERSIST_BLOCKS=98) -- interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t19}
mkdir -p $OUT
: > $OUT/ab.log
for rep in 1 2 3; do for B in 0 98; do
  if [ $B = 0 ]; then E=""; else E="PICP_PERSIST_BLOCKS=$B"; fi
  env $E timeout -k 10 200 python bench.py --workload c2 --no-cpu --skip-extras --steps 20 > $OUT/run.log 2>&1 || { echo "bench failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('c2 blocks=$B', d['value'], r.get('kernel_us'))" | tee -a $OUT/ab.log
done; done
