#!/bin/bash
# C5 loop: VO + triangulation + driver parity tests, then the C5 bench and its kernel stats
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_vo.py tests/test_driver.py tests/test_gpu_parity.py -x -q -k "vo or tri or driver or icp or reference" --timeout 300 --timeout-method thread > gpurun_out/pt_c5.log 2>&1
rc=$?; tail -2 gpurun_out/pt_c5.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --workload c5 --no-cpu > gpurun_out/b_c5.log 2>&1 || exit 1
python -c "import json; d=json.loads(open('gpurun_out/b_c5.log').read().strip().splitlines()[-1]); print('c5', d['value'], d['ms_per_step'], d['pose_err_vs_gt_se3_max'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5q -o run --output-format csv -- python3 bench.py --workload c5 --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_c5q.log 2>&1 || exit 1
python3 -c "
import csv
for x in list(csv.DictReader(open('gpurun_out/prof_c5q/run_kernel_stats.csv')))[:5]: print(x['Name'][:40], x['Calls'], x['AverageNs'], x['Percentage'], x['MinNs'], x['MaxNs'])
"
