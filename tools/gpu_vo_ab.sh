#!/bin/bash
# A/B of VO builds lib/libpicp_amd_v{0,1,2}.so on C5: the VO tests on each build, then C5
# interleaved with a kernel trace of one short run per build
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/02-visualodometry_amd/lib
for v in 0 1 2 3; do
  PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_vo.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_vo_$v.log 2>&1
  rc=$?; echo "v$v $(tail -1 gpurun_out/pt_vo_$v.log)"; [ $rc -eq 0 ] || exit 1
done
: > gpurun_out/vo_ab.log
for rep in 1 2; do
  for v in 0 1 2 3; do
    PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 200 python bench.py --workload c5 --no-cpu --steps 10 --warmup 2 > gpurun_out/ab_$v.log 2>&1 || { echo "v$v failed"; tail gpurun_out/ab_$v.log; exit 1; }
    echo "v$v $(tail -1 gpurun_out/ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/vo_ab.log
  done
done
for v in 0 1 2 3; do
  PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/vo_$v -o run --output-format csv -- python3 bench.py --workload c5 --no-cpu --skip-extras --steps 2 --warmup 1 > gpurun_out/vo_prof_$v.log 2>&1 || { echo "prof v$v failed"; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/vo_$v/run_kernel_stats.csv')):
    if 'vo_' in r['Name'] or 'block' in r['Name'] or 'mfma' in r['Name']: print('v$v', r['Name'][:40], r['Calls'], r['AverageNs'], r['Percentage'])"
done
