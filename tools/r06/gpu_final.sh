#!/bin/bash
# Round 6 end pass: the whole GPU suite and smoke at HEAD, the default bench line twice, the C2/C3
# A/B of the persistent kernel's error-word check (lib/libpicp_amd_perr0.so = round 5's kernel),
# then the kernel traces of every workload with the FETCH/WRITE/SQ PMC passes the bench line reads
# (tools/r04/gpu_prof_r04.sh) and the C5 shapes by kernel and stream (tools/r05/gpu_prof_c5.sh).
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
: > $OUT/ab_perr.log
for W in c2 c3; do for rep in 1 2 3; do for v in libpicp_amd_perr0 libpicp_amd; do
  PICP_LIB=$L/$v.so timeout -k 10 300 python bench.py --workload $W --no-cpu --skip-extras --detail - > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('$W', '$v', d['value'], d['ms_per_step'])" | tee -a $OUT/ab_perr.log
done; done; done
WLS="c2 c3 c4 c4x128 c2n16m" OUT=$OUT bash tools/r04/gpu_prof_r04.sh || exit 1
OUT=$OUT bash tools/r05/gpu_prof_c5.sh
