#!/bin/bash
# Round 5, call 52: the append's FP64 Jacobi triangulation with hardware reciprocal / rsqrt
# estimates refined by two Newton steps (-DPICP_TRI_FAST), rotation threshold as shipped
# (lib/libpicp_amd_tf34.so) or 1e-12 instead of 1e-17 relative (_tf24.so): triangulation and VO
# tests on both, the append per launch (rocprofv3, C5 and 8e), then C5 / 8e / per-rank A/B.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t52}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
for v in libpicp_amd_tf34 libpicp_amd_tf24; do
  PICP_LIB=$L/$v.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vo.py tests/test_gpu_scale.py tests/test_gpu_vo_long.py -x -q -k "triangulation or vo or scale or long" --timeout 300 --timeout-method thread > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -2 $OUT/pytest_$v.log; [ $rc -eq 0 ] || exit 1
done
for v in libpicp_amd libpicp_amd_tf34 libpicp_amd_tf24; do
  PICP_LIB=$L/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${v}_c5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 3 --warmup 2 --no-cpu --skip-extras --samples 1 --detail - > $OUT/${v}_c5.log 2>&1 || { echo "trace $v failed"; tail $OUT/${v}_c5.log; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open("$OUT/${v}_c5/run_kernel_stats.csv")):
    if "append" in r["Name"]: print("$v c5", r["Name"][:26], r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
  rm -f $OUT/${v}_c5/run_kernel_trace.csv
done
: > $OUT/ab.log
for args in "" "--frames 1281" "--seg-len 1250 --steps 2 --warmup 1 --samples 1"; do for rep in 1 2; do for v in libpicp_amd libpicp_amd_tf34 libpicp_amd_tf24; do
  PICP_LIB=$L/$v.so timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras $args > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 $args', '$v', d['value'], d.get('ms_per_step'), d.get('pose_err_vs_gt_se3_max'), d.get('ate_m', (d.get('c5') or {}).get('ate_m')))" | tee -a $OUT/ab.log
done; done; done
