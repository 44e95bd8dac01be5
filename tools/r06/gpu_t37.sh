#!/bin/bash
# Round 6, call 37: splits of 17-32 ranges merged in one 32-range chunk (one round trip; the 8e
# world match's 28) against two 16-range chunks (lib/libpicp_amd_m16.so): matcher and long-VO tests,
# the 8e partition interleaved.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t37}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo_long.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" $OUT/pytest.log | tail -30; exit 1; }
tail -1 $OUT/pytest.log
: > $OUT/ab.log
for rep in 1 2 3; do for v in m16 base; do
  L=02-visualodometry_amd/lib/libpicp_amd.so; [ $v != base ] && L=02-visualodometry_amd/lib/libpicp_amd_$v.so
  PICP_LIB=$L timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - --seg-len 1250 --steps 2 --warmup 1 --samples 3 > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 8e', '$v', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done
