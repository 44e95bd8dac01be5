#!/bin/bash
# Round 5, call 7: the long-segment VO tests with the GPU's exact float32 prior; the block split
# parity test with split 8 (four 256-thread parts per CU); C4 at the 128-frame per-rank shape and
# at 256 frames, split 4 vs split 8, interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t7}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_vo_long.py -m gpu -v -s --timeout 300 --timeout-method thread -k teacher > $OUT/pytest_long.log 2>&1
rc=$?; echo "pytest long rc=$rc"; grep -o "step [0-9]*: map.*" $OUT/pytest_long.log; [ $rc -le 1 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "block_split or tag_bases" > $OUT/pytest_split.log 2>&1
rc=$?; echo "pytest split rc=$rc"; grep -E "PASS|FAIL" $OUT/pytest_split.log | tail -8; [ $rc -eq 0 ] || exit 1
: > $OUT/ab_split.log
for rep in 1 2 3; do for P in 128 256; do for S in 4 8; do
  PICP_BLOCK_SPLIT=$S timeout -k 10 200 python bench.py --workload c4 --problems $P --no-cpu --skip-extras --steps 20 --detail - > $OUT/run.log 2>&1 || { echo "bench failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); r=d['roofline']; print('c4x$P split$S', d['value'], r.get('kernel_us'), d.get('pose_err_vs_gt_se3'))" | tee -a $OUT/ab_split.log
done; done; done
