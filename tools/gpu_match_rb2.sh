#!/bin/bash
# adaptive matcher RB: matcher + VO tests with RB forced 1 and 2 and adaptive, traces, C5 x2
export TMPDIR=/tmp
mkdir -p gpurun_out
for rb in 1 2 auto; do
  if [ $rb = auto ]; then unset PICP_MATCH_RB; else export PICP_MATCH_RB=$rb; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_rb_$rb.log 2>&1
  rc=$?; echo "rb=$rb $(tail -1 gpurun_out/pt_rb_$rb.log)"; [ $rc -eq 0 ] || exit 1
done
unset PICP_MATCH_RB
for shape in "64 2000 8000" "1024 2000 2000"; do
  tag=$(echo $shape | tr ' ' x)
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/rba_$tag -o run --output-format csv -- python3 tools/match_ab.py $shape "PICP_MATCH_ACCEPT_ONLY=1" > gpurun_out/rba_$tag.log 2>&1 || { echo "trace failed"; exit 1; }
  python3 -c "
import csv
t=[int(x['End_Timestamp'])-int(x['Start_Timestamp']) for x in csv.DictReader(open('gpurun_out/rba_$tag/run_kernel_trace.csv')) if 'mfma' in x['Kernel_Name']]
print('auto $tag', t)"
done
for rep in 1 2; do
  timeout -k 10 200 python bench.py --workload c5 --no-cpu --steps 10 --warmup 2 > gpurun_out/rba_c5.log 2>&1 || { echo "c5 failed"; exit 1; }
  echo "auto c5 $(tail -1 gpurun_out/rba_c5.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
