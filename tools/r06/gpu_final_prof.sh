#!/bin/bash
# Round 6 end pass, part 2: the one-segment 8e share (the N = 8 per-rank shape of the 8e partition)
# with the row-block rule fixed for one problem (lib/libpicp_amd_m16.so = the previous rule), the
# default line once more, then the kernel traces of every workload with the FETCH/WRITE/SQ PMC passes
# the bench line reads (tools/r04/gpu_prof_r04.sh: C2, C3, C4, C4 at 128 frames, the 16M frame) and
# the C5 shapes by kernel and stream (tools/r05/gpu_prof_c5.sh: 250 segments, 8e, N = 8 share).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/final}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
: > $OUT/ab_seg1.log
for rep in 1 2; do for v in libpicp_amd_m16 libpicp_amd; do
  PICP_LIB=$L/$v.so timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - --frames 1252 --seg-len 1250 --steps 2 --warmup 1 --samples 1 > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 one 8e segment', '$v', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab_seg1.log
done; done
timeout -k 10 600 python -u bench.py --detail $OUT/bench_detail_c.json > $OUT/bench_default_c.json 2> $OUT/bench_default_c.err || { echo "bench failed"; tail -20 $OUT/bench_default_c.err; exit 1; }
tail -c 2100 $OUT/bench_default_c.json
WLS="c2 c3 c4 c4x128 c2n16m" OUT=$OUT bash tools/r04/gpu_prof_r04.sh || exit 1
OUT=$OUT bash tools/r05/gpu_prof_c5.sh
