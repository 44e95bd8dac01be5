#!/bin/bash
# Round 4 end: the default bench line and the rocprofv3 kernel traces of its workloads on ONE box,
# so that each dominant kernel's traced average can be set beside the untraced line's ms_per_step
# (boxes differ by several per cent).  OUT=${OUT:-gpurun_out/r04/same_box}
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04/same_box}
mkdir -p $OUT
timeout -k 10 500 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['ms_per_step'], 'c3', d['c3']['value'], d['c3']['ms_per_step'], 'c4', d['c4']['value'], d['c4']['ms_per_step'], 'c5', d['c5']['value'])"
WLS="c2 c3 c4 c4x128 c5 c2n16m" PMCS=" " OUT=$OUT bash tools/r04/gpu_prof_r04.sh
