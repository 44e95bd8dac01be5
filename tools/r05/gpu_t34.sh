#!/bin/bash
# Round 5, call 34: the folded matcher at four row blocks per wave (RB = 4, 128 queries per wave,
# PICP_MATCH_RB=4, an A/B form): matcher tests with it forced, 1,024 x 2,000 x 2,000 accept-only at
# RB = 2 / 4 (rocprofv3 kernel stats), then C5 at HEAD, RB = 2 (candidate library) and RB = 4.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t34}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
PICP_MATCH_RB=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_rb4.log 2>&1
rc=$?; echo "pytest rb4 rc=$rc"; tail -2 $OUT/pytest_rb4.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
for rb in 2 4; do
  PICP_MATCH_RB=$rb timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/mab_$rb -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > $OUT/mab_$rb.log 2>&1 || { echo "mab $rb failed"; tail $OUT/mab_$rb.log; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open("$OUT/mab_$rb/run_kernel_stats.csv")):
    if "mfma" in r["Name"]: print("rb=$rb", r["Name"][:52], r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
done
: > $OUT/ab.log
for rep in 1 2; do for v in head rb2 rb4; do
  lib=$L/libpicp_amd.so; env=""
  [ $v = head ] && lib=$L/libpicp_amd_head.so
  [ $v = rb4 ] && env="PICP_MATCH_RB=4"
  env $env PICP_LIB=$lib timeout -k 10 200 python bench.py --workload c5 --no-cpu --skip-extras --steps 20 > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5', '$v', d['value'], d.get('pose_err_vs_gt_se3', d.get('pose_err_vs_gt_se3_max')))" | tee -a $OUT/ab.log
done; done
