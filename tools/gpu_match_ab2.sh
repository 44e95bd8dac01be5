#!/bin/bash
# matcher A/B: the matcher GPU tests on the candidate build, then a kernel trace of one
# 1024 x 2000 x 2000 accept-only batch per build and REPS interleaved C5 bench runs
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/mab}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
for v in ${LIBS:-libpicp_amd_c1 libpicp_amd}; do
  PICP_LIB=$L/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/tr_$v -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > $OUT/tr_$v.log 2>&1 || { echo "trace $v failed"; tail $OUT/tr_$v.log; exit 1; }
  echo "$v $(grep mfma $OUT/tr_$v/run_kernel_stats.csv | cut -d, -f1-4)"
done
for rep in $(seq ${REPS:-2}); do for v in ${LIBS:-libpicp_amd_c1 libpicp_amd}; do
  PICP_LIB=$L/$v.so timeout -k 10 200 python bench.py --workload c5 --no-cpu --skip-extras --steps 10 > $OUT/c5.log 2>&1 || { echo "c5 $v failed"; tail $OUT/c5.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c5.log').read().strip().splitlines()[-1]); print('c5', '$v', d['value'], d['pose_err_vs_gt_se3_max'])"
done; done
