#!/bin/bash
# matcher candidate extraction: lane-private LDS lists (default build) vs the register buffer
# (libpicp_amd_prev): GPU matcher/VO tests, kernel traces of one accept-only 1024 x 2000 x 2000
# batch with duplicated references, interleaved C5 runs
export TMPDIR=/tmp
OUT=gpurun_out/mlane
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo.py tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in libpicp_amd_prev libpicp_amd; do
  MATCH_DUP=0.5 PICP_LIB=$L/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/tr_$v -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > $OUT/tr_$v.log 2>&1 || { echo "trace $v failed"; tail $OUT/tr_$v.log; exit 1; }
  echo "$v $(grep mfma $OUT/tr_$v/run_kernel_stats.csv | cut -d, -f2-4)"
done
OUT=$OUT/ab WLS="c5" LIBS="libpicp_amd_prev libpicp_amd" REPS=3 TESTS="" bash tools/gpu_ab.sh
