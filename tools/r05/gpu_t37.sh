#!/bin/bash
# Round 5, call 37: the staggered solver sweep from two items per lane on (lib/libpicp_amd.so:
# PICP_SWEEP_STAGGER 8, PICP_SWEEP_MIN_NPT 2) against none (lib/libpicp_amd_sw0.so): parity
# tests, then C2 (one item per lane: the same code), C3 at 250k / 500k / 1M correspondences (two,
# four, eight items per lane), interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t37}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
: > $OUT/ab.log
for rep in 1 2 3; do for cfg in "c2" "c3 --n 250000" "c3 --n 500000" "c3"; do for v in libpicp_amd_sw0 libpicp_amd; do
  set -- $cfg
  PICP_LIB=$L/$v.so timeout -k 10 200 python bench.py --workload $cfg --no-cpu --skip-extras --steps 20 > $OUT/run.log 2>&1 || { echo "bench $v $cfg failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$cfg', '$v', d['value'], r.get('kernel_us'), d.get('pose_err_vs_gt_se3'))" | tee -a $OUT/ab.log
done; done; done
