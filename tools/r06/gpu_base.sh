#!/bin/bash
# Round 6, first call: the default bench line at the round's starting HEAD, and a dump of the
# 8e partition's segment 0 as the GPU runs it (tools/r05/vo_dump.py) for the CPU-side parity study.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/base}
mkdir -p $OUT
timeout -k 10 500 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['ms_per_step'], 'c3', d['c3']['value'], d['c3']['ms_per_step'], 'c4', d['c4']['value'], d['c4']['ms_per_step'], 'c5', d['c5']['value'])"
timeout -k 10 300 python -u tools/r05/vo_dump.py $OUT/seg0_8e.npz
