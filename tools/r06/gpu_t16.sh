#!/bin/bash
# Round 6, call 16: the split world match with the early part started after the step's merge
# (beside its own PICP kernel), its range split (PICP_VO_EKS) and CU-masked early queues
# (PICP_VO_ECU_SKIP), against the unsplit schedule at the 8e and N = 8 per-rank shapes.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t16}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_vo.py -x -v -m gpu -k "split" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error" $OUT/pytest.log | tail -30; exit 1; }
tail -2 $OUT/pytest.log
: > $OUT/ab.log
for rep in 1 2; do for A in "--seg-len 1250 --steps 2 --warmup 1 --samples 3" "--frames 1281"; do
 for v in "PICP_VO_SPLIT=0" "PICP_VO_SPLIT=1" "PICP_VO_SPLIT=1 PICP_VO_EKS=1" "PICP_VO_SPLIT=1 PICP_VO_EKS=4" "PICP_VO_SPLIT=1 PICP_VO_ECU_SKIP=2" "PICP_VO_SPLIT=1 PICP_VO_ECU_SKIP=4"; do
  env $v timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 [$A]', '$v', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done; done
