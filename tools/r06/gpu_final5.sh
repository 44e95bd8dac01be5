#!/bin/bash
# Round 6 fifth end pass (after the arrival-counter A/B: the persistent launch carries the counter
# space): the whole GPU suite and smoke, the default bench line once.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/final5}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
for s in a; do
  timeout -k 10 600 python -u bench.py --detail $OUT/bench_detail_$s.json > $OUT/bench_default_$s.json 2> $OUT/bench_default_$s.err || { echo "bench failed"; tail -20 $OUT/bench_default_$s.err; exit 1; }
  tail -c 2100 $OUT/bench_default_$s.json
done
