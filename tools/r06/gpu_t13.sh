#!/bin/bash
# Round 6, call 13: the world match split by map age (PICP_VO_SPLIT).  The VO and matcher GPU tests
# (the split's bit-identity and oracle tests among them), then the C5 shapes with the split off /
# on / auto, interleaved.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t13}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_vo.py tests/test_gpu_match.py tests/test_gpu_vo_long.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error" $OUT/pytest.log | tail -30; exit 1; }
tail -3 $OUT/pytest.log
: > $OUT/ab.log
for rep in 1 2; do for A in "--seg-len 1250 --steps 2 --warmup 1 --samples 3" "--frames 1281" ""; do for v in 0 1 auto; do
  if [ $v = auto ]; then unset PICP_VO_SPLIT; else export PICP_VO_SPLIT=$v; fi
  timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 [$A]', 'split $v', d['value'], d.get('chain_step_us'), d.get('pose_err_vs_gt', d.get('ate_m')))" | tee -a $OUT/ab.log
done; done; done
unset PICP_VO_SPLIT
