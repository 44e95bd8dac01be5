#!/bin/bash
# Round 5, call 56: a second sample of the default bench line at the round's final HEAD, on
# another box (box-to-box spread beside profiles/r05/final/bench_default.json).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t56}
mkdir -p $OUT
timeout -k 10 500 python -u bench.py > $OUT/bench_default_b.json 2> $OUT/bench_default_b.err || { echo "bench failed"; tail -20 $OUT/bench_default_b.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_default_b.json').read().strip().splitlines()[-1]); print('c2', d['value'], 'c3', d['c3']['value'], 'c4', d['c4']['value'], d['c4']['per_rank_n8'], 'c5', d['c5']['value'], d['c5']['per_rank_n8']['value'], d['c5']['partition_8e']['value'])"
