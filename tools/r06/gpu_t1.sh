#!/bin/bash
# Round 6, call 1: the whole GPU suite (new: the long-segment parity rule, the world-2/3 host-exchange
# split, the >2^24-reference matcher, the inverse-iteration triangulation), smoke, the default bench
# line, a dump of the 8e segment 0 (tools/r05/vo_dump.py), then the triangulation A/B on the C5 shapes
# (lib/libpicp_amd_trijac.so = -DPICP_TRI_JACOBI_ONLY, the round-5 Jacobi for every point).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t1}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
grep -E "^step |cond" $OUT/pytest_gpu.log | head -20
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
timeout -k 10 300 python -u tools/r05/vo_dump.py $OUT/seg0_8e.npz || exit 1
timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
tail -c 2000 $OUT/bench_default.json
: > $OUT/ab_tri.log
for args in "" "--frames 1281" "--seg-len 1250 --steps 2 --warmup 1 --samples 1"; do for v in libpicp_amd_trijac libpicp_amd; do
  PICP_LIB=$L/$v.so timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras $args --detail - > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 $args', '$v', d['value'], d.get('chain_step_us'), d.get('ate_m'))" | tee -a $OUT/ab_tri.log
done; done
