#!/bin/bash
# VO GPU tests, then a kernel trace of C5 under the default schedule.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/vo_tr}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_vo.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/tr -o run --output-format csv -- python3 bench.py --workload c5 --no-cpu --skip-extras --steps 3 > $OUT/tr.log 2>&1 || { echo "trace failed"; tail $OUT/tr.log; exit 1; }
cut -d, -f1-5 $OUT/tr/run_kernel_stats.csv | cut -c1-150
