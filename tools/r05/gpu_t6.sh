#!/bin/bash
# Round 5, call 6: the long-segment VO and large matcher tests, then the default bench line.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t6}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_vo_long.py -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_long.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" $OUT/pytest_long.log | tail -8; grep -o "step [0-9]*: map.*" $OUT/pytest_long.log; [ $rc -le 1 ] || exit 1
timeout -k 10 900 python3 bench.py --detail $OUT/bench_detail_default.json > $OUT/bench_default.log 2>&1 || { echo "bench failed"; tail $OUT/bench_default.log; exit 1; }
tail -1 $OUT/bench_default.log > $OUT/bench_default.json; wc -c $OUT/bench_default.json; cat $OUT/bench_default.json
