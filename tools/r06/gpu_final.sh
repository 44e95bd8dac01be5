#!/bin/bash
# Round 6 end pass: the whole GPU suite and smoke at HEAD, the default bench line twice, the C5
# A/B of the merge kernel's chunk and the row-block rule for split launches (lib/libpicp_amd_m16.so
# = 16-range chunks always, RB = 2 only for large grids).  The traces and PMC passes are the next call
# (tools/r06/gpu_final_prof.sh).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/final}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
for s in a b; do
  timeout -k 10 600 python -u bench.py --detail $OUT/bench_detail_$s.json > $OUT/bench_default_$s.json 2> $OUT/bench_default_$s.err || { echo "bench failed"; tail -20 $OUT/bench_default_$s.err; exit 1; }
  tail -c 2100 $OUT/bench_default_$s.json
done
: > $OUT/ab_match.log
for A in "--seg-len 1250 --steps 2 --warmup 1 --samples 1" "--frames 1281" ""; do for rep in 1 2 3; do for v in libpicp_amd_m16 libpicp_amd; do
  PICP_LIB=$L/$v.so timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 $A', '$v', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab_match.log
done; done; done
