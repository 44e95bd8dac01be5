#!/bin/bash
# Round 5 end, part A: the default bench line, then on the same box the rocprofv3 kernel traces of
# its workloads (tools/r04/gpu_prof_r04.sh: C2, C3, C4, C4 at the 128-frame per-rank shape, the 16M
# streaming frame, each with trace_summary_<w>.json) and the C5 shapes with their per-stream
# timelines (tools/r05/gpu_prof_c5.sh: the default partition, the 8e partition, the N = 8 per-rank
# shape).  OUT=${OUT:-gpurun_out/r05/final}
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/final}
mkdir -p $OUT
timeout -k 10 500 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['ms_per_step'], 'c3', d['c3']['value'], d['c3']['ms_per_step'], 'c4', d['c4']['value'], d['c4']['ms_per_step'], 'c5', d['c5']['value'])"
WLS="c2 c3 c4 c4x128 c2n16m" PMCS=" " OUT=$OUT bash tools/r04/gpu_prof_r04.sh || exit 1
OUT=$OUT bash tools/r05/gpu_prof_c5.sh
