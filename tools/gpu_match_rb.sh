#!/bin/bash
# matcher A/B of lib v0 / v1: matcher + VO tests on v1, kernel traces of two shapes, C5 interleaved
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/02-visualodometry_amd/lib
PICP_LIB=$L/libpicp_amd_v1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_match.log 2>&1
rc=$?; tail -1 gpurun_out/pt_match.log; [ $rc -eq 0 ] || exit 1
for v in 0 1; do
  for shape in "64 2000 8000" "1024 2000 2000"; do
    tag=$(echo $shape | tr ' ' x)
    PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/rb_${v}_$tag -o run --output-format csv -- python3 tools/match_ab.py $shape "PICP_MATCH_ACCEPT_ONLY=1" > gpurun_out/rb_${v}_$tag.log 2>&1 || { echo "trace v$v failed"; tail -3 gpurun_out/rb_${v}_$tag.log; exit 1; }
    python3 -c "
import csv
t=[int(x['End_Timestamp'])-int(x['Start_Timestamp']) for x in csv.DictReader(open('gpurun_out/rb_${v}_$tag/run_kernel_trace.csv')) if 'mfma' in x['Kernel_Name']]
print('v$v $tag', t)"
  done
done
for rep in 1 2; do for v in 0 1; do
  PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 200 python bench.py --workload c5 --no-cpu --steps 10 --warmup 2 > gpurun_out/rb_c5.log 2>&1 || { echo "c5 v$v failed"; exit 1; }
  echo "v$v c5 $(tail -1 gpurun_out/rb_c5.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
