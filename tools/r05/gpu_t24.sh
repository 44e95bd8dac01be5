#!/bin/bash
# Round 5, call 24: C5 with the append's loads issued before its FP64 triangulation (candidate)
# against HEAD (lib/libpicp_amd_head.so), and the candidate with three step chains
# (PICP_VO_CHAINS=3); VO tests on the candidate first; interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t24}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_vo.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
: > $OUT/ab.log
for rep in 1 2 3; do for v in head cand chains3; do
  case $v in head) E="PICP_LIB=$L/libpicp_amd_head.so" ;; cand) E="PICP_LIB=$L/libpicp_amd.so" ;; chains3) E="PICP_LIB=$L/libpicp_amd.so PICP_VO_CHAINS=3" ;; esac
  env $E timeout -k 10 200 python bench.py --workload c5 --no-cpu --skip-extras --steps 20 > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 $v', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done
