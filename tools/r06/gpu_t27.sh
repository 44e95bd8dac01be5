#!/bin/bash
# Round 6, call 27: the split rule for the folded form at two row blocks per wave (one generation of
# four blocks per CU, up to 32 ranges): the matcher and VO suites, then the 8e partition against the
# previous count forced (PICP_MATCH_KSPLIT=16), and the other C5 shapes (rule off there).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t27}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo.py tests/test_gpu_vo_long.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" $OUT/pytest.log | tail -30; exit 1; }
tail -1 $OUT/pytest.log
: > $OUT/ab.log
for rep in 1 2 3; do for k in 16 0; do
  PICP_MATCH_KSPLIT=$k timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - --seg-len 1250 --steps 2 --warmup 1 --samples 3 > $OUT/run.log 2>&1 || { echo "bench failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 8e ksplit $k', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done
for A in "--frames 1281" ""; do
  timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 [$A]', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done
