#!/bin/bash
# Round 6: the whole GPU suite and smoke at the final HEAD (after the end pass's row-block rule fix
# and the RB = 2 range-split test), then one default bench line.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/verify}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 600 python -u bench.py --detail $OUT/bench_detail.json > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
tail -c 2100 $OUT/bench_default.json
