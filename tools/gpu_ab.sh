#!/bin/bash
# A/B of library builds: the GPU parity suite on the candidate (lib/libpicp_amd.so), then REPS
# interleaved bench runs of each workload for every build in LIBS (names under lib/, without .so).
# OUT=gpurun_out/ab  WLS="c2 c3 c4 c5"  LIBS="libpicp_amd_base libpicp_amd"  REPS=3  TESTS="..."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
if [ -n "${TESTS-tests/test_gpu_parity.py tests/test_gpu_vo.py}" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS-tests/test_gpu_parity.py tests/test_gpu_vo.py} -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
fi
: > $OUT/ab.log
for rep in $(seq ${REPS:-3}); do for W in ${WLS:-c2 c3 c4 c5}; do for v in ${LIBS:-libpicp_amd_base libpicp_amd}; do
  PICP_LIB=$L/$v.so timeout -k 10 200 python bench.py --workload $W --no-cpu --skip-extras --steps ${STEPS:-20} ${ARGS} > $OUT/run.log 2>&1 || { echo "bench $v $W failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$W', '$v', d['value'], r.get('kernel_us'), d.get('pose_err_vs_gt_se3', d.get('pose_err_vs_gt_se3_max')))" | tee -a $OUT/ab.log
done; done; done
